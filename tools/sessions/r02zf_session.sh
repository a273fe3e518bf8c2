#!/bin/bash
# r02zf: ChunkSet::new as encode / commitment kernels overlapped on two streams in sub-batches
# (tools/pipecommit.py) against the fused kernel, cfg2 and 256 chunksets, normal and high priority
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02zf; mkdir -p $out
export TMPDIR=/tmp
for n in 103 256; do
  timeout -k 10 200 python -u tools/pipecommit.py --n $n > $out/pipe$n.jsonl 2>&1 || { echo "PIPE FAILED"; tail $out/pipe$n.jsonl; exit 1; }
  cat $out/pipe$n.jsonl
done
timeout -k 10 200 python -u tools/pipecommit.py --n 103 --priority > $out/pipe103p.jsonl 2>&1 || { echo "PIPE FAILED"; tail $out/pipe103p.jsonl; exit 1; }
cat $out/pipe103p.jsonl
echo session-ok
