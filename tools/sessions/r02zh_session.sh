#!/bin/bash
# r02zh: host-path coefficient upload, bench roofline fix: full -m gpu suite, smoke, bench, rocprofv3 trace + PMC
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02zh; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 180 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $out/gpu_tests.log
# 0 = green, 1 = test failures: keep going; anything else (abort, segfault, timeout) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail $out/smoke.log; exit 3; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo bench failed; tail $out/bench.err; exit 4; }
cut -c1-900 $out/bench.json
bcmd="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench -- $bcmd > $out/trace.log 2>&1 || { echo "TRACE FAILED"; tail -5 $out/trace.log; exit 5; }
i=0
for pmc in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o bench -- $bcmd > $out/pmc$i.log 2>&1 || { echo "PMC $i FAILED"; tail -5 $out/pmc$i.log; exit 6; }
done
echo session-ok
