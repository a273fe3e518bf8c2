#!/bin/bash
# Encode rate landscape over batch sizes on one box (current build): which sizes run fast?
set -o pipefail
out=${1:-gpurun_out/r01zz6}
mkdir -p $out
export TMPDIR=/tmp
for n in 96 100 103 104 110 120 128 150 200 256 300 400 512 513 600 800 1024 1200 1639; do
  r=4; [ $n -ge 1024 ] && r=2
  timeout -k 10 300 python tools/abbench.py --n $n --rounds $r --warmup-s 1 build/ab/lib_cur.so > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 96 100 103 104 110 120 128 150 200 256 300 400 512 513 600 800 1024 1200 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['n'], d['encode_ms'], d['encode_GBps'], d['decode_GBps'])"
echo session-ok
