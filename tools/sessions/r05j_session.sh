#!/bin/bash
# decode with 8-column lane blocks (8-byte stores) at 5 / 6 / 8 waves/SIMD against the shipped
# 16-column blocks at 4 waves
set -o pipefail
out=gpurun_out/r05j; mkdir -p $out
export TMPDIR=/tmp
for v in dw2w5 dw2w6 dw2h1w8 dw2h1w6 cwd; do
DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo PARITY $v FAILED; tail -20 $out/parity_$v.log; exit 1; }
tail -1 $out/parity_$v.log
done
L="build/ab/lib_base.so:1048704+118 build/ab/lib_dw2w5.so:1048704+118 build/ab/lib_dw2w6.so:1048704+118 build/ab/lib_dw2h1w8.so:1048704+118 build/ab/lib_dw2h1w6.so:1048704+118 build/ab/lib_cwd.so:1048704+118"
for n in 103 256 1024 1639; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 12 --warmup-s 2 $L >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['decode_ms'], d['decode_GBps'])
"
