#!/bin/bash
# GPU-box session: full GPU test suite, smoke, default bench, and the encode memory-pattern
# ceilings (tools/membench.hip) at cfg2 / cfg3 sizes. Outputs under $1.
set -o pipefail
out=${1:-gpurun_out/r01e}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "BENCH FAILED"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 120 build/membench 103 8 > $out/membench103.jsonl 2>&1 || { echo "MEMBENCH FAILED"; exit 1; }
timeout -k 10 300 build/membench 1639 6 > $out/membench1639.jsonl 2>&1 || { echo "MEMBENCH FAILED"; exit 1; }
cat $out/membench103.jsonl $out/membench1639.jsonl
echo session-ok
