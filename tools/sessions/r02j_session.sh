#!/bin/bash
# r02j: full -m gpu suite after the gather-decode address fix (readfirstlane sign extension), then an
# in-process A/B of the coded-row pitch (all 128-B-aligned payloads: +128 B ... 1.25 MiB + 128 B past
# 1 MiB) and of encode units of 1 (dispatcher order) / 2 against the shipped units of 4
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02j; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 240 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
L=""
for p in 1048704 1048960 1049728 1050752 1052800 1056896 1114240 1310848; do L="$L build/ab/lib_cur.so:$p+118"; done
L="$L build/ab/lib_eu1.so:1048704+118 build/ab/lib_eu2.so:1048704+118"
for n in 256 1024; do
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 8 --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 256 1024; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s) dec %.4f (%.0f GB/s)' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps']))"
echo session-ok
