#!/bin/bash
# Encode XCD remap on / off with the current kernels (units of 4 tiles up to 512 chunksets, 8 above).
set -o pipefail
out=${1:-gpurun_out/r01zz4}
mkdir -p $out
export TMPDIR=/tmp
L="build/ab/lib_cur.so build/ab/lib_nox.so"
for n in 64 103 256 1024 1639; do
  r=10; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 64 103 256 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['encode_GBps'])"
echo session-ok
