#!/bin/bash
# r02zi(b): decode store patterns (tools/layoutbench --only dec): + pieces 1 MiB + 16 apart (aligned, L-like spacing)
# aligned ones, 4-byte-aligned ones, and per-lane split stores (12-B middle + byte/short edges)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02zi; mkdir -p $out
timeout -k 10 240 ./tools/bin/layoutbench --only dec --reps 20 > $out/layout_dec_b.jsonl 2>&1 || { echo "LAYOUT FAILED"; tail $out/layout_dec_b.jsonl; exit 1; }
cat $out/layout_dec_b.jsonl
echo session-ok
