#!/bin/bash
# sweep encode with fewer resident workgroups than fit (87.5 / 75 / 62.5 % of 2 per CU): fewer
# concurrent DRAM streams against less latency hiding
set -o pipefail
out=gpurun_out/r05n; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_g75.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/parity_g75.log 2>&1 || { echo PARITY FAILED; tail -20 $out/parity_g75.log; exit 1; }
tail -1 $out/parity_g75.log
L="build/ab/lib_base.so:1048704+118 build/ab/lib_g875.so:1048704+118 build/ab/lib_g75.so:1048704+118 build/ab/lib_g625.so:1048704+118"
for n in 256 1024 1639; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 12 --warmup-s 2 $L >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'])
"
