#!/bin/bash
# r02y: self-resetting tile counter (last workgroup out zeroes it; no hipMemsetAsync launch per encode):
# parity (codec, commit, blob), A/B against the memset build (q), then the bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02y; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_commit.py tests/test_gpu_blob.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
L="build/ab/lib_q.so:1048704+118 build/ab/lib_qr.so:1048704+118"
for n in 103 256 1024; do
  r=10; [ $n -ge 1024 ] && r=6
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s = %.3f) dec %.4f' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['encode_GBps']/8000, d['decode_ms']))"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail $out/bench.err; exit 4; }
python -c "
import json; d=json.load(open('$out/bench.json')); print(d['value'], d['breakdown']); print([(x['chunksets'], x['frac']) for x in d['encode_batch_sweep']])"
echo session-ok
