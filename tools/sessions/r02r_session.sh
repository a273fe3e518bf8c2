#!/bin/bash
# r02r: queue-fed sweep encode (tile counter, one atomic per workgroup and tile) against the fixed-stride
# sweep and units of 4 per XCD eighth, at every batch size (sweeps forced for all n: qall / sall)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02r; mkdir -p $out
export TMPDIR=/tmp
for v in; do DECDS_LIB=build/ab/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_commit.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }; tail -1 $out/${v}_tests.log; done
L="build/ab/lib_u4all.so:1048704+118 build/ab/lib_sall.so:1048704+118 build/ab/lib_qall.so:1048704+118"
for n in 103 256 512 1024 1639; do
  r=8; [ $n -ge 1024 ] && r=5
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 512 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s = %.3f) dec %.4f (%.0f GB/s)' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['encode_GBps']/8000, d['decode_ms'], d['decode_GBps']))"
echo session-ok
