#!/bin/bash
# Exploration batch for one gpurun call. Outputs under gpurun_out/explore/.
set -o pipefail
o=gpurun_out/explore; mkdir -p $o
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $o/gput.log 2>&1 || { tail -30 $o/gput.log; exit 1; }
tail -1 $o/gput.log
timeout -k 10 300 python tools/abbench.py --n 103 --rounds 12 build/variants/lib_s0.so build/variants/lib_s8.so build/variants/lib_d4.so build/variants/lib_d32.so build/variants/lib_e8d8.so > $o/ab103.log 2>&1 || exit 1
timeout -k 10 300 python tools/abbench.py --n 1639 --rounds 6 build/variants/lib_s0.so build/variants/lib_s8.so build/variants/lib_d32.so > $o/ab1639.log 2>&1 || exit 1
timeout -k 10 300 python tools/e2e_files.py --gib 1 > $o/e2e_files.log 2>&1 || exit 1
timeout -k 10 120 python tools/pipebench.py --n 103 --parts 4 > $o/pipe.log 2>&1 || exit 1
DECDS_WGS_PER_CU=1 timeout -k 10 120 python tools/pipebench.py --n 103 --parts 4 >> $o/pipe.log 2>&1 || exit 1
echo explore-ok
