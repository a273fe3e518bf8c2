#!/bin/bash
# Encode / decode rate over a fine batch-size sweep (which sizes reach 5.4 TB/s encode?).
# One build, 600 .. 1800 chunksets.
set -o pipefail
out=${1:-gpurun_out/r01zr}
mkdir -p $out
export TMPDIR=/tmp
for n in 600 700 800 900 950 1000 1100 1200 1300 1400 1500 1600 1700 1800; do
  timeout -k 10 300 python tools/abbench.py --n $n --rounds 3 build/ab/lib_cur.so > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 600 700 800 900 950 1000 1100 1200 1300 1400 1500 1600 1700 1800; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'])"
echo session-ok
