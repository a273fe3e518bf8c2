set -o pipefail
mkdir -p gpurun_out/r01n
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01n/tests.log 2>&1 || { tail -30 gpurun_out/r01n/tests.log; exit 1; }
tail -1 gpurun_out/r01n/tests.log
timeout -k 10 120 python tools/kbench.py --n 103 --reps 20 --check > gpurun_out/r01n/k103.json && timeout -k 10 120 python tools/kbench.py --n 1639 --reps 5 --check > gpurun_out/r01n/k1639.json && cat gpurun_out/r01n/k103.json gpurun_out/r01n/k1639.json
