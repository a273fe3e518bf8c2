#!/bin/bash
# decode occupancy: 3 workgroups per CU (5 KiB LDS) vs 2 (56 KiB LDS caps it) vs 3 (40 KiB), in-process A/B
set -o pipefail
out=gpurun_out/r03z; mkdir -p $out
export TMPDIR=/tmp
for n in 103 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 12 --warmup-s 2 build/ab/lib_cur.so:1048704+118 build/ab/lib_dec2wg.so:1048704+118 build/ab/lib_dec3wg40.so:1048704+118 >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['decode_ms'], d['decode_min_ms'])
"
