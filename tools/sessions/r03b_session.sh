#!/bin/bash
# wave-step fused ChunkSet::new: parity of the commit tests, then A/B against the unit-hash form
set -o pipefail
out=gpurun_out/r03b; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for n in 103 256; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 8 build/ab/lib_wave3.so build/ab/lib_unit.so build/ab/lib_wave2.so > $out/fuse_$n.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_$n.jsonl; exit 1; }
cat $out/fuse_$n.jsonl
done
