#!/bin/bash
# sc1 (and sc0|sc1) cache policy on the streaming loads, encode and decode (cache-policy bits only:
# no parity change). Kernel A/B.
set -o pipefail
out=${1:-gpurun_out/r01zz8}
mkdir -p $out
export TMPDIR=/tmp
L="build/ab/lib_cur.so build/ab/lib_el16.so build/ab/lib_dl16.so build/ab/lib_el17.so"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
