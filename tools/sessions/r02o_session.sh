#!/bin/bash
# r02o: persistent sweep encode (rlnc_encode_sweep_kernel: resident workgroups grid-stride over
# tiles, tables rebuilt per tile from coefficient bytes loaded a tile ahead) against units of 4 tiles
# per XCD eighth: parity of the sweep build (codec + commit suites), then in-process A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02o; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_sw.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_commit.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/sw_tests.log 2>&1 || { echo "sw TESTS FAILED"; tail -30 $out/sw_tests.log; exit 1; }
tail -1 $out/sw_tests.log
L="build/ab/lib_msg.so:1048704+118 build/ab/lib_sw.so:1048704+118 build/ab/lib_msg.so:1048704+16 build/ab/lib_sw.so:1048704+16"
for n in 103 256 1024 1639; do
  r=8; [ $n -ge 1024 ] && r=5
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s = %.3f) dec %.4f (%.0f GB/s)' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['encode_GBps']/8000, d['decode_ms'], d['decode_GBps']))"
echo session-ok
