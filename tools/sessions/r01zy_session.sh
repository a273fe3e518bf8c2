#!/bin/bash
# Unit sizes again after the conflict-free table builds (cheaper rebuilds): encode 2 / 8 tiles for
# n <= 512, encode 4 tiles above 512, decode 4 tiles. Kernel A/B (no parity: same code paths as
# the tested unit sizes).
set -o pipefail
out=${1:-gpurun_out/r01zy}
mkdir -p $out
export TMPDIR=/tmp
L="build/ab/lib_cur.so build/ab/lib_s2.so build/ab/lib_s8.so build/ab/lib_l4.so build/ab/lib_d4.so"
for n in 103 256 1024 1639; do
  r=10; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
