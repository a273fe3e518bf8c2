#!/bin/bash
# Digest kernel: blocks loaded in pairs (whole 128-byte lines of the lane's chunk, next pair
# prefetched; DECDS_DG_PAIR=1) against one block at a time. Commit parity tests of the variant first.
set -o pipefail
out=${1:-gpurun_out/r01zz14}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_dgp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread > $out/parity_dgp.log 2>&1 || { echo "PARITY FAILED"; tail -20 $out/parity_dgp.log; exit 1; }
tail -1 $out/parity_dgp.log
for r in 1 2; do
  for v in cur dgp; do
    for n in 103 1639; do
      DECDS_LIB=build/ab/lib_$v.so timeout -k 10 200 python tools/kbench.py --n $n --reps 10 --commit --check --tag ${v}_$r >> $out/kb.jsonl 2>/dev/null || { echo "KBENCH FAILED"; exit 1; }
    done
  done
done
python -c "
import json
for l in open('$out/kb.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('tag'), d.get('n'), d.get('commit_ms'), d.get('commit_GBps'), d.get('check', d.get('ok')))"
echo session-ok
