#!/bin/bash
# Encode / decode rate against batch size around powers of two (is 1024 slow because its XCD eighths
# are 128 chunksets apart?): one build, sizes 768 / 1000 / 1024 / 1030 / 1536 / 1639 / 2048.
set -o pipefail
out=${1:-gpurun_out/r01zq}
mkdir -p $out
export TMPDIR=/tmp
for n in 768 1000 1024 1030 1536 1639 2048; do
  timeout -k 10 300 python tools/abbench.py --n $n --rounds 4 build/ab/lib_cur.so > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 768 1000 1024 1030 1536 1639 2048; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'])"
echo session-ok
