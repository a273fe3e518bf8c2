#!/bin/bash
# fused ChunkSet::new with the cross-wave fold (16-chunk subtrees) and the shallow fold kernel
set -o pipefail
out=gpurun_out/r03h; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_validate.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u tools/fusebench.py --n 103 --rounds 8 build/ab/lib_fold16.so build/ab/lib_nt.so > $out/fuse_103.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_103.jsonl; exit 1; }
cat $out/fuse_103.jsonl
cmd="python3 tools/fusebench.py --n 103 --rounds 4 --warmup-s 0.5 build/ab/lib_fold16.so"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o fuse -- $cmd > $out/trace.log 2>&1 || { echo TRACE FAILED; tail -5 $out/trace.log; exit 1; }
echo ok
