#!/bin/bash
# Encode range rotation: parity + kernel A/B across batch sizes (ranges aligned to chunksets at 256/1024).
set -o pipefail
out=${1:-gpurun_out/r01u}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_rot.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/rot_tests.log 2>&1 || { echo "ROT TESTS FAILED"; tail -30 $out/rot_tests.log; exit 1; }
tail -1 $out/rot_tests.log
L="build/ab/lib_base.so build/ab/lib_rot.so build/ab/lib_e_np8.so build/ab/lib_e8.so"
for n in 103 256 1024 1639; do
  r=8; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
grep -h tag $out/ab*.jsonl
echo session-ok
