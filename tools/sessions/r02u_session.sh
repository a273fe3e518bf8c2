#!/bin/bash
# r02u: decode access pattern with byte-misaligned piece outputs (i*L, the real layout) against 16-byte
# aligned ones (tools/layoutbench --only dec); parity of the sweep build that skips the tile counter
# for batches of at most one tile per workgroup, and its small-batch encode times
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02u; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_commit.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 tools/bin/layoutbench --only dec > $out/layout_dec.jsonl 2> $out/layout.err || { echo layoutbench failed; tail $out/layout.err; exit 1; }
python -c "
import json
for l in open('$out/layout_dec.jsonl'):
    d=json.loads(l); print('%-22s n=%5d med %7.1f best %7.1f' % (d['variant'], d['chunksets'], d['GBps_med'], d['GBps_best']))"
for n in 1 2 16; do
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 20 --warmup-s 1 build/ab/lib_q.so:1048704+118 build/ab/lib_u4all.so:1048704+118 > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 1 2 16; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s) dec %.4f' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms']))"
echo session-ok
