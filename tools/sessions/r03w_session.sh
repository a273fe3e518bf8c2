#!/bin/bash
# sweep encode: 8-column blocks at 3 waves/SIMD against 16-column at 2 (in-process A/B)
set -o pipefail
out=gpurun_out/r03w; mkdir -p $out
export TMPDIR=/tmp
for n in 103 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 10 --warmup-s 2 build/ab/lib_cur.so:1048704+118 build/ab/lib_enc8c3w.so:1048704+118 >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'])
"
