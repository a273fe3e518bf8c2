#!/bin/bash
# XCD-contiguous remap of the non-persistent walk: parity, kernel A/B, and HBM traffic per variant.
set -o pipefail
out=${1:-gpurun_out/r01za}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/cur_tests.log 2>&1 || { echo "CUR TESTS FAILED"; tail -30 $out/cur_tests.log; exit 1; }
tail -1 $out/cur_tests.log
for v in xr xr16; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  tail -1 $out/${v}_tests.log
done
L="build/ab/lib_cur.so build/ab/lib_xr.so build/ab/lib_xr16.so"
for n in 103 256 1639; do
  r=12; [ $n -ge 1024 ] && r=5
  timeout -k 10 500 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
grep -h tag $out/ab*.jsonl | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
bcmd="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sweep"
for v in cur xr; do
  for pmc in FETCH_SIZE WRITE_SIZE; do
    DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc_${v}_$pmc -o bench -- $bcmd > $out/pmc_${v}_$pmc.log 2>&1 || { echo "PMC $v $pmc FAILED"; tail -5 $out/pmc_${v}_$pmc.log; exit 1; }
  done
done
echo session-ok
