#!/bin/bash
# Does the allocation size decide the encode rate? The same batch run in exactly-sized buffers and
# inside buffers sized for 1800 chunksets (at the start and in the middle).
set -o pipefail
out=${1:-gpurun_out/r01zs}
mkdir -p $out
export TMPDIR=/tmp
i=0
for spec in "103 0 0" "103 1800 0" "103 1800 800" "1000 0 0" "1000 1800 0" "1000 1800 700" "1639 0 0" "103 0 0"; do
  set -- $spec; i=$((i+1))
  timeout -k 10 300 python tools/abbench.py --n $1 --alloc-n $2 --at $3 --rounds 6 build/ab/lib_cur.so > $out/ab$i.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$i.jsonl; exit 1; }
done
cat $out/ab*.jsonl | grep tag | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['n'], d['alloc_n'], d['at'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'])"
echo session-ok
