#!/bin/bash
# Branch-free per-chunkset encode segments: parity through the C-ABI for each variant, then kernel A/B.
set -o pipefail
out=${1:-gpurun_out/r01y}
mkdir -p $out
export TMPDIR=/tmp
for v in ebf ebfnt ebfc ebfnp8; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
L="build/ab/lib_np.so build/ab/lib_ebf.so build/ab/lib_ebfnt.so build/ab/lib_ebfc.so build/ab/lib_ebfnp8.so"
for n in 103 256 1639; do
  r=12; [ $n -ge 1024 ] && r=5
  timeout -k 10 500 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
grep -h tag $out/ab*.jsonl | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'])"
echo session-ok
