# round-6 session zg: the driver's round-end sequence on the final tree — GPU suite, smoke, default bench
set -o pipefail
out=gpurun_out/r09zg; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
start=$(date +%s)
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
echo "default bench wall: $(( $(date +%s) - start )) s"
echo session-ok
