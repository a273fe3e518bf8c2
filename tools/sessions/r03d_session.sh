#!/bin/bash
# wave-step fused ChunkSet::new: 8-column (128-B steps, 3 waves/SIMD) vs 16-column (256-B steps, 2 waves/SIMD)
set -o pipefail
out=gpurun_out/r03d; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fusebench.py --n 103 --rounds 8 build/ab/lib_dw2.so build/ab/lib_dw4.so > $out/fuse_103.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_103.jsonl; exit 1; }
cat $out/fuse_103.jsonl
timeout -k 10 300 python -u tools/fusebench.py --no-check --n 103 --rounds 8 build/ab/lib_dw4nohash.so build/ab/lib_nohash.so > $out/fuse_nohash.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_nohash.jsonl; exit 1; }
cat $out/fuse_nohash.jsonl
timeout -k 10 300 python -u tools/fusebench.py --n 256 --rounds 8 build/ab/lib_dw2.so build/ab/lib_dw4.so > $out/fuse_256.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_256.jsonl; exit 1; }
cat $out/fuse_256.jsonl
cmd="python3 tools/fusebench.py --n 103 --rounds 4 --warmup-s 0.5 build/ab/lib_dw4.so"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc2 -o fuse -- $cmd > $out/pmc2.log 2>&1 || { echo PMC2 FAILED; tail -5 $out/pmc2.log; exit 1; }
echo ok
