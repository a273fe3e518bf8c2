#!/bin/bash
# line-aligned vs plain decode once more: in-process A/B at 103 (20 rounds, two orders)
set -o pipefail
out=gpurun_out/r03s; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/abbench.py --n 103 --rounds 20 --warmup-s 3 build/ab/lib_cur.so:1048704+118 build/ab/lib_dec0.so:1048704+118 > $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
timeout -k 10 300 python -u tools/abbench.py --n 103 --rounds 20 --warmup-s 3 build/ab/lib_dec0.so:1048704+118 build/ab/lib_cur.so:1048704+118 >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
timeout -k 10 300 python -u tools/abbench.py --n 256 --rounds 12 --warmup-s 2 build/ab/lib_cur.so:1048704+118 build/ab/lib_dec0.so:1048704+118 >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['decode_ms'], d['decode_min_ms'])
"
