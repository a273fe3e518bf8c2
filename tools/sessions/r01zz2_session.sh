#!/bin/bash
# Row digests split over 1 / 2 / 4 workgroups (CPT = 4 / 2 / 1 chunks per thread) + finish kernel:
# commitment and validation parity for the default, then the commitment time per build at 103 and
# 1639 chunksets (kbench --commit, alternating builds).
set -o pipefail
out=${1:-gpurun_out/r01zz2}
mkdir -p $out
export TMPDIR=/tmp
for v in cpt1 cpt2; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
for n in 103 1639; do
  for r in 1 2; do
    for v in old cpt4 cpt2 cpt1; do
      DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python tools/kbench.py --n $n --reps 10 --commit --tag $v >> $out/kb$n.jsonl 2>&1 || { echo "KB FAILED"; tail $out/kb$n.jsonl; exit 1; }
    done
  done
done
cat $out/kb*.jsonl | grep '"tag"' | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d.get('tag'), d.get('n'), {k: v for k, v in d.items() if 'commit' in k})"
echo session-ok
