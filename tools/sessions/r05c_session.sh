#!/bin/bash
# round-3 tree: full GPU suite (sharded RepairingBlob, coalesced ChunkSet::new, cfg5 last shard,
# aligned-layout spot checks), then the per-chunkset mirror with and without coalescing
set -o pipefail
out=gpurun_out/r05c; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -u tools/mirror_bench.py --threads 1,4,8,16 --seconds 2 --no-blob > $out/mirror_coalesced.jsonl 2> $out/mirror.err || { echo MIRROR FAILED; tail -20 $out/mirror.err; exit 1; }
DECDS_CHUNKSET_COALESCE=0 timeout -k 10 300 python -u tools/mirror_bench.py --threads 1,4,8,16 --seconds 2 --no-blob > $out/mirror_lanes.jsonl 2>> $out/mirror.err || { echo MIRROR LANES FAILED; tail -20 $out/mirror.err; exit 1; }
cat $out/mirror_coalesced.jsonl $out/mirror_lanes.jsonl
