#!/bin/bash
# r02c: encode/decode work units + workgroup order + first-tile prefetch (r02b: the unit-1,
# dispatcher-ordered access pattern streams 19 % faster than unit 4 with XCD eighths). Parity of the
# two leading variants first, then in-process A/B at 103 / 256 / 1639 chunksets, rlnc and aligned pitch.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02c; mkdir -p $out
export TMPDIR=/tmp
for v in e1p e2p; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
L="build/ab/lib_cur.so build/ab/lib_p.so build/ab/lib_e1.so build/ab/lib_e1p.so build/ab/lib_e2p.so build/ab/lib_e1xp.so build/ab/lib_e1p.so:1048592 build/ab/lib_cur.so:1048592"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=6
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-16s n=%5d enc %.4f (%.0f GB/s) dec %.4f (%.0f GB/s)' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps']))"
echo session-ok
