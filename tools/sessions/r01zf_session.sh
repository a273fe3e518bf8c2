#!/bin/bash
# Encode walks after the do-while fix (no spills, vmcnt(25) everywhere): non-persistent (cur) vs the
# committed build (old), persistent round-robin units of 8 (rr8), persistent per-XCD work queues of
# 8 / 16-tile units (q8, q16); dph = decode with the column phase. Parity first, then a kernel A/B.
set -o pipefail
out=${1:-gpurun_out/r01zf}
mkdir -p $out
export TMPDIR=/tmp
for v in cur dph rr8 q8 q16; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
L="build/ab/lib_old.so build/ab/lib_cur.so build/ab/lib_rr8.so build/ab/lib_q8.so build/ab/lib_q16.so"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=5
  timeout -k 10 500 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
