# round-6 session u: 8-column one-tile decode (and fused plan + decode) for small batches: the parity file
# (every decode form), then kernel-trace durations with DECDS_DEC_NARROW_MAX_N = 0 (16-column) / 64 (8-column)
set -o pipefail
out=gpurun_out/r09u; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for nar in 0 64; do for nn in 1 2 4 8 16 32; do
  tag=nar${nar}_$nn
  DECDS_DEC_NARROW_MAX_N=$nar DECDS_PLAN_DECODE_MAX_N=64 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$tag -o kb -- python3 tools/kbench.py --n $nn --reps 30 --repair --check > $out/kbench_$tag.json 2>$out/kbench_$tag.err || { tail $out/kbench_$tag.err; exit 1; }
done; done
echo session-ok
