#!/bin/bash
# current tree: GPU suite, then the RepairingBlob under chunkset-major and share-major arrival with
# device budgets (spill) and over 2 contexts, 1 GiB blob
set -o pipefail
out=gpurun_out/r05l; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -u tools/blob_bench.py --gib 1 --budgets-mb 0,512 > $out/blob_chunkset_major.json 2> $out/blob.err || { echo BLOB BENCH FAILED; tail -20 $out/blob.err; exit 1; }
timeout -k 10 300 python -u tools/blob_bench.py --gib 1 --share-major --budgets-mb 0,512 > $out/blob_share_major.json 2>> $out/blob.err || { echo BLOB BENCH 2 FAILED; tail -20 $out/blob.err; exit 1; }
timeout -k 10 300 python -u tools/blob_bench.py --gib 1 --share-major --contexts 2 > $out/blob_share_major_2ctx.json 2>> $out/blob.err || { echo BLOB BENCH 3 FAILED; tail -20 $out/blob.err; exit 1; }
cat $out/blob_*.json
