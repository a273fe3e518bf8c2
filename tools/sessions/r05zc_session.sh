#!/bin/bash
# fused ChunkSet::new with 2 / 4 of its 10 inputs looked up in byte tables (one read per byte, pairs
# combined per v_bitop3; 4 KiB of tables each, 3 workgroups per CU still fit) against nibble tables only
set -o pipefail
out=gpurun_out/r05zc; mkdir -p $out
export TMPDIR=/tmp
for l in fh2 fh4; do
DECDS_LIB=build/ab/lib_$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_hostpath.py -x -q --timeout 200 --timeout-method thread > $out/parity_$l.log 2>&1 || { echo PARITY $l FAILED; tail -30 $out/parity_$l.log; exit 1; }
tail -1 $out/parity_$l.log
done
for n in 103 256 1024; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 10 build/ab/lib_fh0.so build/ab/lib_fh2.so build/ab/lib_fh4.so >> $out/fuse.jsonl 2>>$out/fuse.err || { echo FUSE FAILED; tail -20 $out/fuse.err; exit 1; }
done
cat $out/fuse.jsonl
