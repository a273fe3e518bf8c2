#!/bin/bash
# encode with smaller lookup groups: 3 waves/SIMD (groups of 1 byte, 167 VGPRs) and the same group
# sizes at 2 waves; decode XCD runs of 16 at 4 waves/SIMD
set -o pipefail
out=gpurun_out/r05g; mkdir -p $out
export TMPDIR=/tmp
for v in enc3h1 enc2h1; do
DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo PARITY $v FAILED; tail -20 $out/parity_$v.log; exit 1; }
tail -1 $out/parity_$v.log
done
L="build/ab/lib_base.so:1048704+118 build/ab/lib_enc3h1.so:1048704+118 build/ab/lib_enc2h2.so:1048704+118 build/ab/lib_enc2h1.so:1048704+118 build/ab/lib_dec4.so:1048704+118"
for n in 103 256 1024 1639; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 12 --warmup-s 2 $L >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'])
"
