#!/bin/bash
# decode sweep without per-tile address recomputation (165 VGPRs at 3 waves, no spills; remat cost the
# encode 5.6 %, r05u) and the register-pressure trackers for all kernels, on a second box
set -o pipefail
out=gpurun_out/r05v; mkdir -p $out
export TMPDIR=/tmp
for n in 1639 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --check --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_trk.so build/ab/lib_dnr.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/ab.jsonl
for n in 103 256 1024; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 10 build/ab/lib_base.so build/ab/lib_trk.so >> $out/fuse.jsonl 2>$out/fuse.err || { echo FUSE FAILED; tail -20 $out/fuse.err; exit 1; }
done
cat $out/fuse.jsonl
