#!/bin/bash
# full session on the shipped build (fused kernel with SDWA lookup addresses)
set -o pipefail
bash tools/gpu_session.sh gpurun_out/r05zb 20 cfg3
