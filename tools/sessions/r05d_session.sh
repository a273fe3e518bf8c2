#!/bin/bash
# per-chunkset mirror: coalesced ChunkSet::new (rows repacked on the device) against the lane path
# with 16 / 8 / 4 lanes at 1-16 caller threads
set -o pipefail
out=gpurun_out/r05d; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_hostpath.py -x -q --timeout 120 --timeout-method thread > $out/hostpath.log 2>&1 || { echo TESTS FAILED; tail -30 $out/hostpath.log; exit 1; }
tail -1 $out/hostpath.log
timeout -k 10 300 python -u tools/mirror_bench.py --threads 1,4,8,16 --seconds 2 --no-blob > $out/mirror_coalesced.jsonl 2> $out/mirror.err || { echo MIRROR FAILED; tail -20 $out/mirror.err; exit 1; }
for L in 16 8 4; do
DECDS_CHUNKSET_COALESCE=0 DECDS_MAX_LANES=$L timeout -k 10 300 python -u tools/mirror_bench.py --threads 1,4,8,16 --seconds 2 --no-blob > $out/mirror_lanes$L.jsonl 2>> $out/mirror.err || { echo MIRROR LANES FAILED; tail -20 $out/mirror.err; exit 1; }
done
for f in $out/mirror_*.jsonl; do echo "== $f"; grep chunkset_new $f | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['threads'], d['GiBps'])"; done
