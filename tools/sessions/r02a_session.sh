#!/bin/bash
# r02a: first GPU run of round 2 — full -m gpu suite (device-status check after every test), smoke,
# bench (cfg2), HBM ceiling study (tools/hbmbench, warmed clocks)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r02a
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/${T}_gpu_tests.log
# 0 = green, 1 = test failures: keep going; anything else (abort, segfault, timeout) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/${T}_smoke.log | tail; exit 3; }
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 4; }
cat gpurun_out/${T}_bench.json | cut -c1-600
timeout -k 10 240 tools/bin/hbmbench > gpurun_out/${T}_hbm.jsonl 2> gpurun_out/${T}_hbm.err || { echo hbmbench failed; exit 5; }
echo done
