#!/bin/bash
# stream_range with the column helper (encode 220 VGPRs, no spills, against 256 + 24 B of spills in
# the committed build): parity, then kernel A/B from 1 to 1639 chunksets.
set -o pipefail
out=${1:-gpurun_out/r01zu}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_col.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/col_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/col_tests.log; exit 1; }
tail -1 $out/col_tests.log
L="build/ab/lib_old.so build/ab/lib_col.so"
for n in 1 4 16 103 1639; do
  r=15; [ $n -ge 1024 ] && r=5
  timeout -k 10 300 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 1 4 16 103 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['plan_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
