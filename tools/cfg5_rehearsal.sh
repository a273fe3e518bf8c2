#!/bin/bash
# cfg5 (BASELINE.json: 128 GiB blob encode + repair sharded by chunkset index across 8 MI355X) on a
# one-GPU box: each of the 8 ranks' shards (16 GiB = 1639 chunksets; the last 1635, its final
# chunkset 2 MiB of data) runs in turn as its own process through bench.py --rehearse-shard, every
# repaired chunkset compared with its source on the device. Output: one JSON line per shard.
out=${1:-gpurun_out/cfg5_rehearsal.jsonl}; steps=${2:-10}
mkdir -p "$(dirname "$out")"
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 300 python bench.py --config cfg3 --rehearse-shard $r/8 --steps $steps --warmup 3 --no-cpu-baseline --no-sweep >> "$out" || exit 1
done
