#!/bin/bash
# GPU suite on the shipped build with the nothing-ready decode test
set -o pipefail
out=gpurun_out/r05z; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
grep nothing_ready $out/gpu_tests.log
