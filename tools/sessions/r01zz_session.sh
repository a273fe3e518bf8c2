#!/bin/bash
# Plan kernel: full kernel against its setup alone (loads + log/exp tables, no candidate loop;
# timing-only build with wrong output) at 1 / 103 / 1639 chunksets.
set -o pipefail
out=${1:-gpurun_out/r01zz}
mkdir -p $out
export TMPDIR=/tmp
for n in 1 103 1639; do
  r=10; [ $n -ge 1024 ] && r=3
  timeout -k 10 300 python tools/abbench.py --n $n --rounds $r build/ab/lib_cur.so build/ab/lib_psetup.so > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 1 103 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['plan_ms'])"
echo session-ok
