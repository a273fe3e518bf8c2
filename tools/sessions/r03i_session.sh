#!/bin/bash
# LDS-staged chunk digest kernel: parity (commit / validate / files / fullsize tests), A/B of the
# separate commitment against the lane-per-chunk digest (lib_nt), kernel trace
set -o pipefail
out=gpurun_out/r03i; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_validate.py tests/test_gpu_files.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u tools/fusebench.py --n 103 --rounds 8 build/ab/lib_dglds.so build/ab/lib_nt.so > $out/fuse_103.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_103.jsonl; exit 1; }
cat $out/fuse_103.jsonl
cmd="python3 tools/fusebench.py --n 103 --rounds 4 --warmup-s 0.5 build/ab/lib_dglds.so"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o fuse -- $cmd > $out/trace.log 2>&1 || { echo TRACE FAILED; tail -5 $out/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc2 -o fuse -- $cmd > $out/pmc2.log 2>&1 || { echo PMC2 FAILED; tail -5 $out/pmc2.log; exit 1; }
echo ok
