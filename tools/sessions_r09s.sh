# round-6 session s: plan fast path with unreduced log sums (three-period exp table): plan / repair GPU tests,
# kernel-trace A/B against the incremental-only build, phase timeline
set -o pipefail
out=gpurun_out/r09s; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "plan or repair or fused" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for lib in default tools/bin/lib_plan_incr.so; do for nn in 1 2 16; do
  tag=$(basename $lib .so)_$nn
  if [ $lib = default ]; then envs=""; else envs="DECDS_LIB=$PWD/$lib"; fi
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$tag -o kb -- python3 tools/kbench.py --n $nn --reps 40 --repair --check > $out/kbench_$tag.json 2>$out/kbench_$tag.err || { tail $out/kbench_$tag.err; exit 1; }
done; done
DECDS_LIB=$PWD/tools/bin/lib_ptrace.so timeout -k 10 120 python tools/repair_phases.py --sizes 1,2 > $out/phases.jsonl 2> $out/phases.err || { tail $out/phases.err; exit 1; }
echo session-ok
