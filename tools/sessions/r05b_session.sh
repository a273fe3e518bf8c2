#!/bin/bash
# encode table-build variants: conflict-free (XOR-staggered) build, double-buffered tables with one
# barrier per tile, both; parity of each on the GPU suite's encode/repair tests, then in-process A/B
set -o pipefail
out=gpurun_out/r05b; mkdir -p $out
export TMPDIR=/tmp
for v in xor dbuf xordbuf; do
DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo PARITY $v FAILED; tail -20 $out/parity_$v.log; exit 1; }
tail -1 $out/parity_$v.log
done
for n in 256 1639 103; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 12 --warmup-s 2 build/ab/lib_base.so:1048704+118 build/ab/lib_xor.so:1048704+118 build/ab/lib_dbuf.so:1048704+118 build/ab/lib_xordbuf.so:1048704+118 >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'])
"
# the sharded / memory-bounded RepairingBlob and HostBuffer lifetime (product build)
timeout -k 10 300 python -u -m pytest tests/test_gpu_blob.py tests/test_gpu_hostpath.py -x -v --timeout 200 --timeout-method thread > $out/blob_tests.log 2>&1 || { echo BLOB TESTS FAILED; tail -40 $out/blob_tests.log; exit 1; }
tail -3 $out/blob_tests.log
