#!/bin/bash
# decode as a persistent tile sweep (DECDS_DEC_SWEEP, one global counter) against the one-tile
# workgroups; row offsets in the buffer instructions' SGPR offset (soff0 = VGPR sums, as shipped)
set -o pipefail
out=gpurun_out/r05p; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_dsw3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_blob.py -x -q --timeout 200 --timeout-method thread > $out/parity_dsw3.log 2>&1 || { echo PARITY FAILED; tail -30 $out/parity_dsw3.log; exit 1; }
tail -1 $out/parity_dsw3.log
timeout -k 10 300 python -u tools/abbench.py --check --n 1639 --rounds 12 build/ab/lib_base.so build/ab/lib_soff0.so build/ab/lib_dsw3.so build/ab/lib_dsw4h1.so build/ab/lib_dsw4.so > $out/ab1639.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
for n in 103 256; do
timeout -k 10 300 python -u tools/abbench.py --check --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_dsw3.so build/ab/lib_dsw4h1.so >> $out/ab_small.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/ab1639.jsonl $out/ab_small.jsonl
