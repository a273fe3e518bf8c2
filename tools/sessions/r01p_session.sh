#!/bin/bash
# Warp-specialised streaming kernels: parity through the C-ABI, then kernel A/B against the default.
set -o pipefail
out=${1:-gpurun_out/r01p}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_ws.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/ws_tests.log 2>&1 || { echo "WS TESTS FAILED"; tail -30 $out/ws_tests.log; exit 1; }
tail -1 $out/ws_tests.log
L="build/ab/lib_base.so build/ab/lib_ws.so build/ab/lib_ws_c.so"
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 16 $L > $out/ab103.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab103.jsonl; exit 1; }
timeout -k 10 400 python tools/abbench.py --n 1639 --rounds 6 $L > $out/ab1639.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab1639.jsonl; exit 1; }
grep tag $out/ab103.jsonl $out/ab1639.jsonl
echo session-ok
