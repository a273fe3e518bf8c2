#!/bin/bash
# encode sweep at 3 waves/SIMD with lookup groups of 2 bytes: fits without spills once the table-build
# addresses are recomputed per tile (DECDS_ENC_REMAT) and the backend's register-pressure trackers
# schedule it (-amdgpu-use-amdgpu-trackers); the trackers alone (all kernels) and remat alone at 2 waves
set -o pipefail
out=gpurun_out/r05u; mkdir -p $out
export TMPDIR=/tmp
for n in 1639 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --check --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_trk.so build/ab/lib_e3trk.so build/ab/lib_e2remat.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/ab.jsonl
for n in 103 256; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 10 build/ab/lib_base.so build/ab/lib_trk.so >> $out/fuse.jsonl 2>$out/fuse.err || { echo FUSE FAILED; tail -20 $out/fuse.err; exit 1; }
done
cat $out/fuse.jsonl
