#!/bin/bash
# decode form by batch size: one-tile workgroups against the persistent sweep at 256-1639 chunksets
# (output-checked), then the full session on the shipped build (threshold 512)
set -o pipefail
out=gpurun_out/r05s; mkdir -p $out
export TMPDIR=/tmp
for n in 512 1024 256 1639; do
timeout -k 10 300 python -u tools/abbench.py --check --check-reps 2 --n $n --rounds 12 build/ab/lib_tiles.so build/ab/lib_sweep.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/ab.jsonl
bash tools/gpu_session.sh $out 20 cfg3
