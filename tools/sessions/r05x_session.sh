#!/bin/bash
# decode lookups reading 12 of a table row's 16 bytes (ds_read_b96: outputs 0-11; a quarter less LDS
# data, accumulators and XORs): parity on the narrow build, then A/B against full rows, and the narrow
# rows at 4 waves/SIMD with groups of 1 byte (123 VGPRs) / 3 waves with groups of 4 bytes (168)
set -o pipefail
out=gpurun_out/r05x; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_nar.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blob.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $out/parity_nar.log 2>&1 || { echo PARITY FAILED; tail -30 $out/parity_nar.log; exit 1; }
tail -1 $out/parity_nar.log
for n in 1639 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --check --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_nar.so build/ab/lib_nar4h1.so build/ab/lib_nar3h4.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
timeout -k 10 300 python -u tools/abbench.py --check --n 103 --rounds 12 build/ab/lib_base.so build/ab/lib_nar.so build/ab/lib_nar4h1.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
cat $out/ab.jsonl
