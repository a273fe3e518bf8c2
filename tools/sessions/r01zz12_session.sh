#!/bin/bash
# Encode XCD-remap family re-checked with units of 4 tiles: runs of 64 (one chunkset) / 16
# workgroups dealt to the XCDs in turn, odd XCDs sweeping backwards / from the middle.
set -o pipefail
out=${1:-gpurun_out/r01zz12}
mkdir -p $out
export TMPDIR=/tmp
for v in ck64 ck16 md1 md2; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $out/parity_$v.log; exit 1; }
  tail -1 $out/parity_$v.log
done
L="build/ab/lib_cur.so build/ab/lib_ck64.so build/ab/lib_ck16.so build/ab/lib_md1.so build/ab/lib_md2.so"
for n in 103 256 1024 1639; do
  r=8; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], 'enc', d['encode_ms'], d['encode_GBps'], 'dec', d['decode_ms'], d['decode_min_ms'], d['decode_GBps'])"
echo session-ok
