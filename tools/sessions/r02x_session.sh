#!/bin/bash
# r02x: where the fused ChunkSet::new's time goes: full fused kernel (fuse), its hash phase's loads
# without compressions (fnh), its hashing without the encode stream (fns), 16-column blocks (f4)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02x; mkdir -p $out
export TMPDIR=/tmp
for n in 103 256; do
  timeout -k 10 300 python -u tools/fusebench.py --no-check --n $n --rounds 8 build/ab/lib_fuse.so build/ab/lib_fnh.so build/ab/lib_fns.so build/ab/lib_f4.so > $out/fuse$n.jsonl 2>&1 || { echo "FUSE FAILED"; tail $out/fuse$n.jsonl; exit 1; }
  grep tag $out/fuse$n.jsonl
done
echo session-ok
