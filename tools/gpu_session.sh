#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 trace + PMC passes of the bench
# command (separate --pmc passes: MI355X_MICROARCH.md §rocprofv3). Outputs under $1 (gpurun_out/...).
# usage: bash tools/gpu_session.sh <outdir> [steps] [config]   (config: bench.py --config, default cfg3)
set -o pipefail
out=${1:-gpurun_out/session}; steps=${2:-20}; cfg=${3:-cfg3}
export TMPDIR=/tmp
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python bench.py --config $cfg --steps $steps --warmup 5 > $out/bench.json 2> $out/bench.err || { echo "BENCH FAILED"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
bcmd="python3 bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline --no-sweep --no-extras"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench -- $bcmd > $out/trace.log 2>&1 || { echo "TRACE FAILED"; tail -5 $out/trace.log; exit 1; }
i=0
for pmc in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o bench -- $bcmd > $out/pmc$i.log 2>&1 || { echo "PMC $i FAILED"; tail -5 $out/pmc$i.log; exit 1; }
done
echo session-ok
