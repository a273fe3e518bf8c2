#!/bin/bash
# fused ChunkSet::new at 4 waves/SIMD (lookup groups of 2 bytes: 117 VGPRs) and decode at 3 / 4 waves
# per SIMD (same trick): parity of each variant, then in-process A/B
set -o pipefail
out=gpurun_out/r05e; mkdir -p $out
export TMPDIR=/tmp
for v in fh4 fh3h2; do
DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py -x -q --timeout 200 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo PARITY $v FAILED; tail -20 $out/parity_$v.log; exit 1; }
tail -1 $out/parity_$v.log
done
for v in dec4 dec3; do
DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo PARITY $v FAILED; tail -20 $out/parity_$v.log; exit 1; }
tail -1 $out/parity_$v.log
done
for n in 103 256; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 10 build/ab/lib_base.so build/ab/lib_fh4.so build/ab/lib_fh3h2.so >> $out/fuse.jsonl 2>$out/fuse.err || { echo FUSE FAILED; tail -20 $out/fuse.err; exit 1; }
done
for n in 103 256 1639; do
timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 12 --warmup-s 2 build/ab/lib_base.so:1048704+118 build/ab/lib_dec4.so:1048704+118 build/ab/lib_dec3.so:1048704+118 >> $out/ab.jsonl 2>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/fuse.jsonl
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['decode_ms'], d['decode_GBps'])
"
timeout -k 10 300 python -u -m pytest tests/test_gpu_hostpath.py -x -q --timeout 200 --timeout-method thread > $out/hostpath.log 2>&1 || { echo HOSTPATH FAILED; tail -30 $out/hostpath.log; exit 1; }
tail -1 $out/hostpath.log
