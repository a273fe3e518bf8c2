#!/bin/bash
# rocprofv3 kernel trace + HBM traffic passes of the bench at cfg3 (1639 chunksets per launch: the
# north-star batch >= 256), beside the cfg2 session profiles
set -o pipefail
out=${1:-gpurun_out/r04v}; export TMPDIR=/tmp; mkdir -p $out
cmd="python3 bench.py --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline --no-sweep --no-commit"
timeout -k 10 300 $cmd > $out/bench.json 2> $out/bench.err || { echo BENCH FAILED; tail -5 $out/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench -- $cmd > $out/trace.log 2>&1 || { echo TRACE FAILED; tail -5 $out/trace.log; exit 1; }
i=0
for pmc in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o bench -- $cmd > $out/pmc$i.log 2>&1 || { echo PMC $i FAILED; tail -5 $out/pmc$i.log; exit 1; }
done
echo session-ok
