#!/bin/bash
# r02za: host-memory end-to-end rates of the blob host paths on the registry build (tools/e2e_bench.py:
# 4 GiB blob, batches 16 / 32; first rep staged through the bounce rings, then registered buffers)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02za; mkdir -p $out
export TMPDIR=/tmp
for b in 16 32; do
  timeout -k 10 300 python -u tools/e2e_bench.py --gib 4 --batch $b > $out/e2e_b$b.json 2> $out/e2e_b$b.err || { echo "E2E FAILED"; tail $out/e2e_b$b.err; exit 1; }
  cat $out/e2e_b$b.json
done
echo session-ok
