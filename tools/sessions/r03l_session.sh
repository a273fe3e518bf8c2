#!/bin/bash
# fused ChunkSet::new at 4 waves/SIMD (128 VGPRs, 164 B/lane of spills) against 3; full-size test incl. the fused path
set -o pipefail
out=gpurun_out/r03l; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fusebench.py --n 103 --rounds 8 build/ab/lib_cur.so build/ab/lib_fh4w.so > $out/fuse_103.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_103.jsonl; exit 1; }
cat $out/fuse_103.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
