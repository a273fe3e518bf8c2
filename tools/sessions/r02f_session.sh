#!/bin/bash
# r02f: the new defaults (compact tables, first-tile prefetch, decode units of 1, aligned coded layout
# in bench.py): full -m gpu suite, smoke, bench; then decode occupancy 2 / 3 / 4 waves per SIMD A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02f; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail $out/smoke.log; exit 3; }
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo bench failed; tail $out/bench.err; exit 4; }
python -c "
import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['breakdown'])); print([ (s['chunksets'], s['frac']) for s in d['encode_batch_sweep']]); print(d['roofline']['frac'], d['roofline']['decode']['frac'])"
A=1048704+118
L="build/ab/lib_new.so:$A build/ab/lib_dw3.so:$A build/ab/lib_dw4.so:$A build/ab/lib_cur.so"
for n in 103 1639; do
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 8 --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-24s n=%5d enc %.4f (%.0f GB/s) dec %.4f (%.0f GB/s) step %.4f' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps'], d['encode_ms']+d['plan_ms']+d['decode_ms']))"
timeout -k 10 300 python -u tools/mirror_bench.py > $out/mirror.jsonl 2> $out/mirror.err || { echo mirror_bench failed; tail $out/mirror.err; exit 6; }
cat $out/mirror.jsonl
timeout -k 10 300 tools/bin/hbmbench --gib 4 --only codec > $out/hbm.jsonl 2> $out/hbm.err || { echo hbmbench failed; exit 5; }
echo session-ok
