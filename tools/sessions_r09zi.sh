# round-6 session zi: the 4-column one-chunkset forms in the product — GPU suite (every encode / decode form),
# the fused repair's kernel trace at 1 / 2 chunksets, and a bench line (sweep incl. 1 chunkset)
set -o pipefail
out=gpurun_out/r09zi; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for nn in 1 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_default_$nn -o kb -- python3 tools/kbench.py --n $nn --reps 40 --repair --check > $out/kbench_$nn.json 2>$out/kbench_$nn.err || { tail $out/kbench_$nn.err; exit 1; }
done
timeout -k 10 600 python bench.py --steps 10 --no-api-shapes --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
echo session-ok
