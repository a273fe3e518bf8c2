#!/bin/bash
# Encode-only XCD remaps: contiguous eighths vs runs of 8 / 32 / 128 workgroups dealt to the XCDs in
# turn; parity, then a kernel A/B over four batch sizes.
set -o pipefail
out=${1:-gpurun_out/r01zc}
mkdir -p $out
export TMPDIR=/tmp
for v in xc8 xc32 xc128; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
L="build/ab/lib_cur.so build/ab/lib_xr.so build/ab/lib_xc8.so build/ab/lib_xc32.so build/ab/lib_xc128.so"
for n in 103 256 1024 1639; do
  r=10; [ $n -ge 1024 ] && r=5
  timeout -k 10 500 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'])"
echo session-ok
