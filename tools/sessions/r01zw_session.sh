#!/bin/bash
# Table build with the first copy of each row in replica (2i + h) mod 16 (conflict-free first writes)
# on top of the flat replica copies: parity, kernel A/B, LDS bank-conflict counters.
set -o pipefail
out=${1:-gpurun_out/r01zw}
mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_flat2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/flat2_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/flat2_tests.log; exit 1; }
tail -1 $out/flat2_tests.log
L="build/ab/lib_old.so build/ab/lib_flat.so build/ab/lib_flat2.so"
for n in 1 4 16 103 256 1639; do
  r=12; [ $n -ge 1024 ] && r=5
  timeout -k 10 300 python tools/abbench.py --n $n --rounds $r $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 1 4 16 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['n'], d['encode_ms'], d['encode_min_ms'], d['decode_ms'], d['decode_min_ms'])"
bcmd="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-commit"
for v in flat flat2; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $out/pmc_$v -o bench -- $bcmd > $out/pmc_$v.log 2>&1 || { echo "PMC $v FAILED"; tail -5 $out/pmc_$v.log; exit 1; }
done
echo session-ok
