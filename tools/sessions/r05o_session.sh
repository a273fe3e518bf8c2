#!/bin/bash
# fused ChunkSet::new with byte tables (one lookup per input byte, pairs of inputs per v_bitop3; 40 KiB
# of tables: 2 workgroups per CU) against the nibble-table form
set -o pipefail
out=gpurun_out/r05o; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_fhb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_hostpath.py -x -q --timeout 200 --timeout-method thread > $out/parity_fhb.log 2>&1 || { echo PARITY FAILED; tail -30 $out/parity_fhb.log; exit 1; }
tail -1 $out/parity_fhb.log
for n in 103 256 1024; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 10 build/ab/lib_base.so build/ab/lib_fhb.so >> $out/fuse.jsonl 2>$out/fuse.err || { echo FUSE FAILED; tail -20 $out/fuse.err; exit 1; }
done
cat $out/fuse.jsonl
