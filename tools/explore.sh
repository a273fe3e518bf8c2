#!/bin/bash
set -o pipefail
o=gpurun_out/explore; mkdir -p $o
V=build/variants
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 12 $V/lib_s0.so $V/lib_e1.so $V/lib_e1skip.so $V/lib_e8.so $V/lib_e8skip.so > $o/ab103.log 2>&1 || exit 1
echo explore-ok
