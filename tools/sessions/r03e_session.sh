#!/bin/bash
# wave-step fused ChunkSet::new: cache policy of the coded-row stores (plain / nt / sc1 / nt sc1)
set -o pipefail
out=gpurun_out/r03e; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fusebench.py --n 103 --rounds 8 build/ab/lib_dw2.so build/ab/lib_nt.so build/ab/lib_sc1.so build/ab/lib_ntsc1.so > $out/fuse_103.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_103.jsonl; exit 1; }
cat $out/fuse_103.jsonl
timeout -k 10 300 python -u tools/fusebench.py --no-check --n 103 --rounds 8 build/ab/lib_ntnohash.so build/ab/lib_nohash.so > $out/fuse_nohash.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_nohash.jsonl; exit 1; }
cat $out/fuse_nohash.jsonl
cmd="python3 tools/fusebench.py --n 103 --rounds 4 --warmup-s 0.5 build/ab/lib_nt.so"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc2 -o fuse -- $cmd > $out/pmc2.log 2>&1 || { echo PMC2 FAILED; tail -5 $out/pmc2.log; exit 1; }
echo ok
