#!/bin/bash
# Allocation-size probe on a box that shows the fast large-batch encode: first 1639 chunksets in
# exact buffers; only if that runs above 5 TB/s, 103 / 1000 chunksets inside buffers sized for 1800.
set -o pipefail
out=${1:-gpurun_out/r01zt}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python tools/abbench.py --n 1639 --rounds 3 build/ab/lib_cur.so > $out/probe.jsonl 2>&1 || { echo "AB FAILED"; tail $out/probe.jsonl; exit 1; }
fast=$(grep tag $out/probe.jsonl | python -c "import sys,json; print(int(json.loads(sys.stdin.read())['encode_GBps'] > 5000))")
grep tag $out/probe.jsonl
if [ "$fast" != "1" ]; then echo "slow box: skipped"; echo session-ok; exit 0; fi
i=0
for spec in "103 0 0" "103 1800 0" "103 1800 900" "1000 0 0" "1000 1800 0" "1639 1800 0" "1200 0 0" "1639 0 0"; do
  set -- $spec; i=$((i+1))
  timeout -k 10 300 python tools/abbench.py --n $1 --alloc-n $2 --at $3 --rounds 5 build/ab/lib_cur.so > $out/ab$i.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$i.jsonl; exit 1; }
done
cat $out/ab*.jsonl | grep tag | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['n'], d['alloc_n'], d['at'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'])"
echo session-ok
