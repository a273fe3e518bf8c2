#!/bin/bash
# full session on the shipped build (decode sweep, input-major plan inverse, trackers schedules)
set -o pipefail
bash tools/gpu_session.sh gpurun_out/r05w 20 cfg3
