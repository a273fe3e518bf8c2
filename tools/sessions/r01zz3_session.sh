#!/bin/bash
# Per-tile workgroup barrier on the branch-free loop (SYNC 1: at each tile's start; 2: before its
# stores), encode and decode: parity of the barrier builds, then kernel A/B.
set -o pipefail
out=${1:-gpurun_out/r01zz3}
mkdir -p $out
export TMPDIR=/tmp
for v in es1 ds1 es2; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
L="build/ab/lib_cur.so build/ab/lib_es1.so build/ab/lib_es2.so build/ab/lib_ds1.so build/ab/lib_ds2.so"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
