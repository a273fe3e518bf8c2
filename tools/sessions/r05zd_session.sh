#!/bin/bash
# decode sweep's piece stores with cache-policy bits nt / sc1 / sc0 against plain
set -o pipefail
out=gpurun_out/r05zd; mkdir -p $out
export TMPDIR=/tmp
for n in 1639 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --check --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_nt.so build/ab/lib_sc1.so build/ab/lib_sc0.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'): d=json.loads(l); print(d['tag'], d['n'], d['decode_ms'], d['check']['bad'])"
