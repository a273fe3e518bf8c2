#!/bin/bash
# Load cache policies with plain stores (now the decode default): decode loads nt / sc0, encode
# loads nt / sc0. Parity of the new default, then kernel A/B.
set -o pipefail
out=${1:-gpurun_out/r01zi}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_cur.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/dl2_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/dl2_tests.log; exit 1; }
tail -1 $out/dl2_tests.log
L="build/ab/lib_cur.so build/ab/lib_dl2s0.so build/ab/lib_dl1s0.so build/ab/lib_el2.so build/ab/lib_el1.so"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=5
  timeout -k 10 500 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
