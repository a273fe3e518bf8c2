#!/bin/bash
# Per-wave timeline of the non-persistent encode / decode at 103 and 413 chunksets (trace build).
set -o pipefail
out=${1:-gpurun_out/r01ze}
mkdir -p $out
export TMPDIR=/tmp
for n in 103 413; do
  timeout -k 10 300 python tools/tracebench.py build/ab/lib_trace.so --n $n --reps 4 --dump $out/trace$n.npz > $out/trace$n.json 2>&1 || { echo "TRACE FAILED"; tail $out/trace$n.json; exit 1; }
done
python -c "
import json
for n in (103, 413):
    d = json.load(open('$out/trace%d.json' % n))
    for k in ('encode', 'decode'):
        print(n, k, json.dumps(d['runs'][-1][k]))"
echo session-ok
