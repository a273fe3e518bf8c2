#!/bin/bash
# line-aligned decode (rlnc_decode_lines_kernel): full GPU suite, then in-process A/B against the plain decode
set -o pipefail
out=gpurun_out/r03n; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for n in 103 256 1639; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 10 --warmup-s 2 build/ab/lib_declines.so:1048704+118 build/ab/lib_dec0.so:1048704+118 >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
timeout -k 10 300 python -u tools/abbench.py --n 103 --rounds 10 --warmup-s 2 build/ab/lib_declines.so build/ab/lib_dec0.so >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
cat $out/ab.jsonl
