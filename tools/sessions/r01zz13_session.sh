#!/bin/bash
# Plan kernel: candidate loop rolled (DECDS_PLAN_UNROLL=0: one copy of the step, instruction cache
# stays hot) against fully unrolled (16 copies of a ~400-instruction step, fetched once per CU).
set -o pipefail
out=${1:-gpurun_out/r01zz13}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_pr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread > $out/parity_pr.log 2>&1 || { echo "PARITY FAILED"; tail -20 $out/parity_pr.log; exit 1; }
tail -1 $out/parity_pr.log
L="build/ab/lib_cur.so build/ab/lib_pr.so"
for n in 103 1639; do
  r=10; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], 'enc', d['encode_ms'], 'plan', d['plan_ms'], 'dec', d['decode_ms'])"
echo session-ok
