#!/bin/bash
# Non-persistent walk (workgroups of T tiles, dispatcher refill): parity + kernel A/B.
set -o pipefail
out=${1:-gpurun_out/r01t}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_d_np8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/np8_tests.log 2>&1 || { echo "NP8 TESTS FAILED"; tail -30 $out/np8_tests.log; exit 1; }
tail -1 $out/np8_tests.log
L="build/ab/lib_base.so build/ab/lib_d_np6.so build/ab/lib_d_np8.so build/ab/lib_d_np12.so build/ab/lib_d_np8_s0.so"
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 16 $L > $out/ab103.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab103.jsonl; exit 1; }
timeout -k 10 400 python tools/abbench.py --n 1639 --rounds 6 $L > $out/ab1639.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab1639.jsonl; exit 1; }
grep tag $out/ab103.jsonl $out/ab1639.jsonl
echo session-ok
