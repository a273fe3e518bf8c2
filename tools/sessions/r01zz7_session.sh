#!/bin/bash
# Plan kernel with 6 dependent table reads per candidate instead of 9: full GPU suite on the new
# build (verdicts against the oracle decoder, repairs), then plan time A/B at 1 / 103 / 1639.
set -o pipefail
out=${1:-gpurun_out/r01zz7}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_pfast.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pfast_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/pfast_tests.log; exit 1; }
tail -1 $out/pfast_tests.log
for n in 1 103 1639; do
  r=10; [ $n -ge 1024 ] && r=3
  timeout -k 10 300 python tools/abbench.py --n $n --rounds $r build/ab/lib_old.so build/ab/lib_pfast.so > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 1 103 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['plan_ms'], d['encode_ms'], d['decode_ms'])"
echo session-ok
