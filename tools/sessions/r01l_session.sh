#!/bin/bash
# Older/younger-half work share study: kernel A/B of the share variants + timeline of one.
set -o pipefail
out=${1:-gpurun_out/r01l}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_d0_530.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/share_tests.log 2>&1 || { echo "SHARE TESTS FAILED"; tail -30 $out/share_tests.log; exit 1; }
tail -1 $out/share_tests.log
L="build/ab/lib_base.so build/ab/lib_e520.so build/ab/lib_e540.so build/ab/lib_d0.so build/ab/lib_d0_530.so build/ab/lib_d0_560.so"
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 16 $L > $out/ab103.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab103.jsonl; exit 1; }
timeout -k 10 400 python tools/abbench.py --n 1639 --rounds 6 $L > $out/ab1639.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab1639.jsonl; exit 1; }
grep tag $out/ab103.jsonl $out/ab1639.jsonl
timeout -k 10 200 python tools/tracebench.py build/ab/lib_trace_w.so --n 103 --reps 3 --dump $out/tw103.npz > $out/trace.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/tracebench.py build/ab/lib_trace_w.so --n 1639 --reps 3 --dump $out/tw1639.npz >> $out/trace.jsonl 2>&1 || exit 1
echo session-ok
