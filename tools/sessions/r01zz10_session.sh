#!/bin/bash
# Encode units of 8 (current) vs 4 above 512 chunksets, inside bench.py's own buffer placement
# (cfg3 step + the cfg2 run's batch sweep), builds alternated: abbench's buffers never reached the
# fast DRAM mode that bench.py's reach at 1639 chunksets on some boxes.
set -o pipefail
out=${1:-gpurun_out/r01zz10}
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur u4; do
    DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python bench.py --config cfg3 --steps 10 --warmup 3 --no-sweep --no-cpu-baseline --no-commit > $out/cfg3_${v}_$r.json 2>/dev/null || { echo "BENCH FAILED"; exit 1; }
    DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-commit > $out/cfg2_${v}_$r.json 2>/dev/null || { echo "BENCH FAILED"; exit 1; }
  done
done
for f in $out/*.json; do python -c "
import json,sys
d=json.load(open('$f')); b=d['breakdown']
print('$f'.split('/')[-1], d['value'], b['encode_ms'], b['encode_GBps'], [(s['chunksets'], s['encode_GBps']) for s in (d['encode_batch_sweep'] or [])][3:])"; done
echo session-ok
