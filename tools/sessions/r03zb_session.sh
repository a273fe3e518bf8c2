#!/bin/bash
# small-batch encode: edge pass spread over the first tiles (lib_edge) against one workgroup per chunkset (lib_cur)
set -o pipefail
out=gpurun_out/r03zb; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for n in 1 2 4 16; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 30 --warmup-s 1 build/ab/lib_cur.so:1048704+118 build/ab/lib_edge.so:1048704+118 >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['encode_GBps'])
"
