# round-6 session q: the plan's Gauss-Jordan fast path — plan / repair GPU tests, then kernel-trace durations
# of the plan kernel and the fused plan + decode against the incremental-only build (DECDS_PLAN_FAST=0)
set -o pipefail
out=gpurun_out/r09q; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "plan or repair or fused" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for lib in default tools/bin/lib_plan_incr.so; do for nn in 1 2 16; do
  tag=$(basename $lib .so)_$nn
  if [ $lib = default ]; then envs=""; else envs="DECDS_LIB=$PWD/$lib"; fi
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$tag -o kb -- python3 tools/kbench.py --n $nn --reps 40 --repair --check > $out/kbench_$tag.json 2>$out/kbench_$tag.err || { tail $out/kbench_$tag.err; exit 1; }
done; done
echo session-ok
