#!/bin/bash
# r02e: 256-byte-aligned coded-row payloads (pitch 1048832, rows start 246 B into the buffer; r02d's
# pattern study: aligned row stores +15 %) and 128-byte alignment, with decode units 1 / 2 / 8,
# compact tables + first-tile prefetch; parity of the new variants first
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02e; mkdir -p $out
export TMPDIR=/tmp
for v in d1p d2p e2d1p; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  echo "$v $(tail -1 $out/${v}_tests.log)"
done
A=1048832+246
L="build/ab/lib_cur.so build/ab/lib_ctp.so build/ab/lib_ctp.so:$A build/ab/lib_ctp.so:1048704+118 build/ab/lib_d1p.so:$A build/ab/lib_d2p.so:$A build/ab/lib_e2d1p.so:$A build/ab/lib_ct1p.so:$A build/ab/lib_ct2p.so:$A"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=6
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-24s n=%5d enc %.4f (%.0f GB/s) dec %.4f (%.0f GB/s) step %.4f' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'], d['encode_ms']+d['plan_ms']+d['decode_ms']))"
echo session-ok
