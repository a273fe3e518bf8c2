#!/bin/bash
# Edge columns done by the whole workgroup (one pass instead of five on wave 0), with and without the
# tiny-batch unit sizes, against the committed build: parity, then kernel A/B at 1..103 chunksets.
set -o pipefail
out=${1:-gpurun_out/r01zn}
mkdir -p $out
export TMPDIR=/tmp
for v in edge edgetiny; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
L="build/ab/lib_old.so build/ab/lib_edge.so build/ab/lib_edgetiny.so"
for n in 1 2 4 8 16 32 103; do
  timeout -k 10 300 python tools/abbench.py --n $n --rounds 15 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 1 2 4 8 16 32 103; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['plan_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
