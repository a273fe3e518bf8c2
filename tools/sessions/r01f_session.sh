#!/bin/bash
# Work-map study: parity of the band build, pattern ceilings per map/throttle, kernel A/B.
set -o pipefail
out=${1:-gpurun_out/r01f}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_band.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/band_tests.log 2>&1 || { echo "BAND TESTS FAILED"; tail -30 $out/band_tests.log; exit 1; }
tail -1 $out/band_tests.log
timeout -k 10 300 build/patbench 1639 6 > $out/pat1639.jsonl 2>&1 || { echo "PATBENCH FAILED"; cat $out/pat1639.jsonl; exit 1; }
timeout -k 10 120 build/patbench 103 10 > $out/pat103.jsonl 2>&1 || { echo "PATBENCH FAILED"; exit 1; }
cat $out/pat1639.jsonl $out/pat103.jsonl
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 16 build/ab/lib_base.so build/ab/lib_band.so build/ab/lib_e8.so > $out/ab103.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab103.jsonl; exit 1; }
timeout -k 10 400 python tools/abbench.py --n 1639 --rounds 8 build/ab/lib_base.so build/ab/lib_band.so build/ab/lib_e8.so > $out/ab1639.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab1639.jsonl; exit 1; }
grep tag $out/ab103.jsonl $out/ab1639.jsonl
echo session-ok
