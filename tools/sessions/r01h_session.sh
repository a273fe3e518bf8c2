#!/bin/bash
# Rebuild-cost study: kernel A/B of the default and band maps with and without table rebuilds
# (DECDS_TIMING_NOREBUILD builds are timing-only: wrong output by construction).
set -o pipefail
out=${1:-gpurun_out/r01h}
mkdir -p $out
export TMPDIR=/tmp
L="build/ab/lib_base.so build/ab/lib_band.so build/ab/lib_nr_base.so build/ab/lib_nr_band.so"
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 16 $L > $out/ab103.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab103.jsonl; exit 1; }
timeout -k 10 400 python tools/abbench.py --n 1639 --rounds 6 $L > $out/ab1639.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab1639.jsonl; exit 1; }
grep tag $out/ab103.jsonl $out/ab1639.jsonl
echo session-ok
