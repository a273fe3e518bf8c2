#!/bin/bash
# Encode XCD eighths: forward (cur), odd XCDs backwards (m1), odd XCDs from mid-range (m2); parity of m1 / m2 is by construction (a permutation of the same units), checked in the GPU suite when adopted.
set -o pipefail
out=${1:-gpurun_out/r01zz5}
mkdir -p $out
export TMPDIR=/tmp
L="build/ab/lib_cur.so build/ab/lib_m1.so build/ab/lib_m2.so"
for n in 64 103 256 1024 1639; do
  r=10; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 64 103 256 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['encode_GBps'])"
echo session-ok
