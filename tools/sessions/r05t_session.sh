#!/bin/bash
# input-major plan inverse (one dword coefficient load per lane in the decode sweep): GPU suite on the
# shipped build, then the decode sweep at 4 waves/SIMD with lookup groups of 1 byte (128 VGPRs, no
# spills now) against 3 waves with groups of 2
set -o pipefail
out=gpurun_out/r05t; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for n in 1639 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --check --check-reps 2 --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_s4h1.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/ab.jsonl
