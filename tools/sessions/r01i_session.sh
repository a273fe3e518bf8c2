#!/bin/bash
# Wave-sync study: per-tile workgroup barrier in the kernels (A/B) and in the pattern bench; parity
# of the s1 build.
set -o pipefail
out=${1:-gpurun_out/r01i}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_s1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/s1_tests.log 2>&1 || { echo "S1 TESTS FAILED"; tail -30 $out/s1_tests.log; exit 1; }
tail -1 $out/s1_tests.log
L="build/ab/lib_base.so build/ab/lib_s1.so build/ab/lib_s2.so build/ab/lib_band_s1.so"
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 16 $L > $out/ab103.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab103.jsonl; exit 1; }
timeout -k 10 400 python tools/abbench.py --n 1639 --rounds 6 $L > $out/ab1639.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab1639.jsonl; exit 1; }
grep tag $out/ab103.jsonl $out/ab1639.jsonl
timeout -k 10 120 build/patbench 103 8 > $out/pat103.jsonl 2>&1 || { echo "PATBENCH FAILED"; exit 1; }
timeout -k 10 300 build/patbench 1639 4 > $out/pat1639.jsonl 2>&1 || { echo "PATBENCH FAILED"; exit 1; }
echo session-ok
