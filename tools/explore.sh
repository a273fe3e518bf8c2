#!/bin/bash
set -o pipefail
o=gpurun_out/explore; mkdir -p $o
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $o/gput.log 2>&1 || { tail -30 $o/gput.log; exit 1; }
tail -1 $o/gput.log
V=build/variants
timeout -k 10 400 python tools/abbench.py --n 103 --rounds 12 $V/lib_s0.so $V/lib_d8.so $V/lib_d8fullsync.so $V/lib_e1d1.so $V/lib_e2d2.so $V/lib_e4d4.so $V/lib_e8d8.so > $o/ab103.log 2>&1 || exit 1
timeout -k 10 400 python tools/abbench.py --n 1639 --rounds 6 $V/lib_s0.so $V/lib_d8.so $V/lib_e1d1.so $V/lib_e2d2.so $V/lib_e4d4.so > $o/ab1639.log 2>&1 || exit 1
echo explore-ok
