#!/bin/bash
# decode sweep with tiles dealt to XCDs in runs of XR (per-XCD counters) against one global counter
# and the one-tile workgroups
set -o pipefail
out=gpurun_out/r05q; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_dsw3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_blob.py -x -q --timeout 200 --timeout-method thread > $out/parity_dsw3.log 2>&1 || { echo PARITY FAILED; tail -30 $out/parity_dsw3.log; exit 1; }
tail -1 $out/parity_dsw3.log
timeout -k 10 300 python -u tools/abbench.py --check --n 1639 --rounds 12 build/ab/lib_base.so build/ab/lib_dsw3.so build/ab/lib_dsw3x1.so build/ab/lib_dsw3x4.so build/ab/lib_dsw3x16.so > $out/ab1639.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
for n in 103 256; do
timeout -k 10 300 python -u tools/abbench.py --check --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_dsw3.so build/ab/lib_dsw3x1.so >> $out/ab_small.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/ab1639.jsonl $out/ab_small.jsonl
