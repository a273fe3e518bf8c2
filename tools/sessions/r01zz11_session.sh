#!/bin/bash
# Re-check on the current build (encode units of 4, conflict-free tables): decode units of 4 / 16
# tiles and the XCD-eighth remap for decode; encode without the remap. Parity of each variant first.
set -o pipefail
out=${1:-gpurun_out/r01zz11}
mkdir -p $out
export TMPDIR=/tmp
for v in dt4 dt16 drm erm0; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $out/parity_$v.log; exit 1; }
  tail -1 $out/parity_$v.log
done
L="build/ab/lib_cur.so build/ab/lib_dt4.so build/ab/lib_dt16.so build/ab/lib_drm.so build/ab/lib_erm0.so"
for n in 103 256 1639; do
  r=8; [ $n -ge 1024 ] && r=4
  timeout -k 10 400 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], 'enc', d['encode_ms'], d['encode_GBps'], 'dec', d['decode_ms'], d['decode_min_ms'], d['decode_GBps'])"
echo session-ok
