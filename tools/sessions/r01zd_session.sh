#!/bin/bash
# Column phase for 16-byte-aligned pitches: parity (all GPU tests), then kernel A/B of the aligned
# pitches against the rlnc pitch, phase on / off.
set -o pipefail
out=${1:-gpurun_out/r01zd}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_ph.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/ph_tests.log 2>&1 || { echo "PH TESTS FAILED"; tail -30 $out/ph_tests.log; exit 1; }
tail -1 $out/ph_tests.log
L="build/ab/lib_noph.so build/ab/lib_ph.so build/ab/lib_ph.so:1048592 build/ab/lib_ph.so:1048704 build/ab/lib_noph.so:1048592"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=5
  timeout -k 10 500 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
echo session-ok
