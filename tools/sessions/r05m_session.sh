#!/bin/bash
# RepairingBlob spill add path after the copy-during-hash change; the N = 2 bench path at the cfg3
# default rehearsed with 2 gloo ranks sharing the one GPU (each rank its 16 GiB shard of a 32 GiB blob)
set -o pipefail
out=gpurun_out/r05m; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/blob_bench.py --gib 1 --share-major --budgets-mb 0,512 > $out/blob_share_major.json 2> $out/blob.err || { echo BLOB BENCH FAILED; tail -20 $out/blob.err; exit 1; }
cat $out/blob_share_major.json
DECDS_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --settle-s 0.2 --no-commit > $out/gloo2.json 2> $out/gloo2.err || { echo GLOO REHEARSAL FAILED; tail -30 $out/gloo2.err; exit 1; }
cat $out/gloo2.json
