#!/bin/bash
# r02b: HBM ceiling study v2 — flat (dispatcher-ordered) streams and the codec access patterns with
# different units / workgroup orders / occupancy, warmed clocks (tools/hbmbench.hip)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 tools/bin/hbmbench --gib 4 --only flat,codec > gpurun_out/r02b_hbm.jsonl 2> gpurun_out/r02b_hbm.err || { echo hbmbench failed; tail gpurun_out/r02b_hbm.err; exit 5; }
echo done
