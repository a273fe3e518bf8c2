#!/bin/bash
# decode sweep correctness at XR=8 (r05q: 7 bad chunksets in one check at 1639): repeated output
# checks, positions of the bad bytes, a re-decode of the same coded rows
set -o pipefail
out=gpurun_out/r05r; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/abbench.py --check --check-reps 6 --n 1639 --rounds 2 --warmup-s 1 build/ab/lib_base.so build/ab/lib_dsw3.so build/ab/lib_dsw3x1.so build/ab/lib_dsw3x4.so > $out/check1639.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
cat $out/check1639.jsonl
