#!/bin/bash
# Tiny batches: units of 1 / 2 (/ 4 for decode) tiles for n <= 2 / 8 (/ 32) against the fixed units.
# Parity of the new default (its small-n tests run the tiny maps), then kernel A/B at 1..32 chunksets.
set -o pipefail
out=${1:-gpurun_out/r01zm}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_tiny.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tiny_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tiny_tests.log; exit 1; }
tail -1 $out/tiny_tests.log
L="build/ab/lib_notiny.so build/ab/lib_tiny.so"
for n in 1 2 4 8 16 32; do
  timeout -k 10 300 python tools/abbench.py --n $n --rounds 20 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 1 2 4 8 16 32; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['plan_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
