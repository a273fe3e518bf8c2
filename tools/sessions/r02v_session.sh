#!/bin/bash
# r02v: decode with realigned piece stores (LDS-staged outputs, 16-byte-aligned stores: da1) against unaligned stores (da0): parity, then in-process A/B
# stores) against the unaligned stores: parity (codec, commit, blob, host paths), then in-process A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02v; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blob.py tests/test_gpu_hostpath.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
L="build/ab/lib_da0.so:1048704+118 build/ab/lib_da1.so:1048704+118"
for n in 103 256 1024; do
  r=8; [ $n -ge 1024 ] && r=5
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s = %.3f) dec %.4f (%.0f GB/s = %.3f)' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['encode_GBps']/8000, d['decode_ms'], d['decode_GBps'], d['decode_GBps']/8000))"
echo session-ok
