#!/bin/bash
# r02g: encode with 8-column lane blocks (half the registers: 168 VGPRs, 3 workgroups per CU) at
# units 1 / 2 / 4 against the 16-column default, all on the aligned coded layout; parity first
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02g; mkdir -p $out
export TMPDIR=/tmp
for v in w3u1 w3u2 w3u4x; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  echo "$v $(tail -1 $out/${v}_tests.log)"
done
A=1048704+118
L="build/ab/lib_base.so:$A build/ab/lib_w3u1.so:$A build/ab/lib_w3u2.so:$A build/ab/lib_w3u4x.so:$A build/ab/lib_w2u1.so:$A"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=6
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-24s n=%5d enc %.4f (%.0f GB/s) dec %.4f (%.0f GB/s) step %.4f' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'], d['encode_ms']+d['plan_ms']+d['decode_ms']))"
echo session-ok
