#!/bin/bash
# r02z: tile-counter sweep encode with 8-column lane blocks at 3 waves per SIMD (sd2: 143 VGPRs, 768
# resident workgroups) against 16-column blocks at 2 (qr): parity of sd2, then in-process A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02z; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_sd2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
L="build/ab/lib_qr.so:1048704+118 build/ab/lib_sd2.so:1048704+118"
for n in 103 256 1024; do
  r=10; [ $n -ge 1024 ] && r=6
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s = %.3f) dec %.4f' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['encode_GBps']/8000, d['decode_ms']))"
echo session-ok
