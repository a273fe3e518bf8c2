#!/bin/bash
# Encode unit size above 512 chunksets: units of 8 (current) against units of 4 / 2 at every batch
# size (DECDS_ENC_SMALL_N=100000, DECDS_ENC_MAP_SMALL=-4 / -2). Parity of both variants first.
set -o pipefail
out=${1:-gpurun_out/r01zz9}
mkdir -p $out
export TMPDIR=/tmp
for v in u4 u2; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $out/parity_$v.log; exit 1; }
  tail -1 $out/parity_$v.log
done
L="build/ab/lib_cur.so build/ab/lib_u4.so build/ab/lib_u2.so"
for n in 600 1024 1639; do
  timeout -k 10 400 python tools/abbench.py --n $n --rounds 6 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 600 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['encode_GBps'], d['decode_ms'])"
echo session-ok
