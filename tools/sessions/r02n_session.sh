#!/bin/bash
# r02n: encode access-pattern orders at the codec kernels' occupancy (2 workgroups per CU): units of
# 4 tiles with XCD eighths (shipped), dispatcher order, strided units; units of 2 / 1 (tools/layoutbench --only occ)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02n; mkdir -p $out
timeout -k 10 300 tools/bin/layoutbench --only occ > $out/layout_occ.jsonl 2> $out/layout.err || { echo layoutbench failed; tail $out/layout.err; exit 1; }
python -c "
import json
for l in open('$out/layout_occ.jsonl'):
    d=json.loads(l); print('%-22s n=%5d med %7.1f best %7.1f' % (d['variant'], d['chunksets'], d['GBps_med'], d['GBps_best']))"
echo session-ok
