#!/bin/bash
# lookup addresses by one SDWA op each (inline asm; hipcc emitted shift + and pairs for most):
# parity on the asm build, then encode / decode / fused A/B against hipcc's address code
set -o pipefail
out=gpurun_out/r05za; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_asm.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/parity_asm.log 2>&1 || { echo PARITY FAILED; tail -30 $out/parity_asm.log; exit 1; }
tail -1 $out/parity_asm.log
for n in 1639 256 1024; do
timeout -k 10 300 python -u tools/abbench.py --check --n $n --rounds 12 build/ab/lib_base.so build/ab/lib_asm.so >> $out/ab.jsonl 2>>$out/ab.err || { echo AB FAILED; tail -20 $out/ab.err; exit 1; }
done
cat $out/ab.jsonl
for n in 103 256 1024; do
timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 10 build/ab/lib_base.so build/ab/lib_asm.so >> $out/fuse.jsonl 2>>$out/fuse.err || { echo FUSE FAILED; tail -20 $out/fuse.err; exit 1; }
done
cat $out/fuse.jsonl
