#!/bin/bash
# fused ChunkSet::new with a step's BLAKE3 compressions interleaved (G function by G function) with the
# next step's encode lookups (DECDS_FH_PIPE): groups of 1 byte at 3 waves (144 VGPRs) / groups of 2
# at 2 waves (177) against the shipped sequential form, and the sequential form with groups of 1
set -o pipefail
out=gpurun_out/r05y; mkdir -p $out
export TMPDIR=/tmp
for l in p1 p2w2; do
DECDS_LIB=build/ab/lib_$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_hostpath.py -x -q --timeout 200 --timeout-method thread > $out/parity_$l.log 2>&1 || { echo PARITY $l FAILED; tail -30 $out/parity_$l.log; exit 1; }
tail -1 $out/parity_$l.log
done
for n in 103 256 1024; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 10 build/ab/lib_base.so build/ab/lib_p1.so build/ab/lib_p2w2.so build/ab/lib_b1.so >> $out/fuse.jsonl 2>>$out/fuse.err || { echo FUSE FAILED; tail -20 $out/fuse.err; exit 1; }
done
cat $out/fuse.jsonl
