#!/bin/bash
# rocprofv3 passes over tools/kbench.py (run on the GPU box from the repo root).
# usage: bash tools/profile.sh <outdir> <n_chunksets> [extra counter passes...]
set -o pipefail
out=${1:-gpurun_out/prof}; n=${2:-1639}; shift 2
export TMPDIR=/tmp
mkdir -p $out
cmd="python3 tools/kbench.py --n $n --reps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- $cmd > $out/trace.log 2>&1 || { echo "trace failed"; tail -5 $out/trace.log; exit 1; }
i=0
for pmc in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o run -- $cmd > $out/pmc$i.log 2>&1 || { echo "pmc pass $i ($pmc) failed"; tail -5 $out/pmc$i.log; exit 1; }
done
echo profile-ok
