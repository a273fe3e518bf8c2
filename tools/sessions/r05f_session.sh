#!/bin/bash
# decode at 4 waves/SIMD: lookup groups of 2 / 1 bytes, units of 2 tiles, XCD runs of 4 / 16 tiles
set -o pipefail
out=gpurun_out/r05f; mkdir -p $out
export TMPDIR=/tmp
for v in dec4h1 dec4u2 dec4r4 dec4r16; do
DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo PARITY $v FAILED; tail -20 $out/parity_$v.log; exit 1; }
tail -1 $out/parity_$v.log
done
L="build/ab/lib_base.so:1048704+118 build/ab/lib_dec4.so:1048704+118 build/ab/lib_dec4h1.so:1048704+118 build/ab/lib_dec4u2.so:1048704+118 build/ab/lib_dec4r4.so:1048704+118 build/ab/lib_dec4r16.so:1048704+118"
for n in 103 256 1024 1639; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 12 --warmup-s 2 $L >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['decode_ms'], d['decode_GBps'])
"
