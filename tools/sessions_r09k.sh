# round-6 session k: plan kernel variants (broadcast reads vs v_readlane), kernel-trace durations at 1 / 16 / 1639 chunksets; D2H piece sizes
set -o pipefail
out=gpurun_out/r09k; mkdir -p $out; export TMPDIR=/tmp
for lib in default tools/bin/lib_plan_readlane.so; do for nn in 1 16 1639; do
  tag=$(basename $lib .so)_$nn
  if [ $lib = default ]; then envs=""; else envs="DECDS_LIB=$PWD/$lib"; fi
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$tag -o kb -- python3 tools/kbench.py --n $nn --reps 30 --repair --check > $out/kbench_$tag.json 2>$out/kbench_$tag.err || { tail $out/kbench_$tag.err; exit 1; }
done; done
for rep in 1 2 3; do for mb in 16 64; do for g in 1 2; do
  DECDS_D2H_PIECE_MB=$mb timeout -k 10 120 python tools/e2e_bench.py --gib $g --batch 16 --reps 5 --memory alloc > $out/tmp.json || exit 1
  sed "s/^{/{\"piece_mb\": $mb, /" $out/tmp.json >> $out/d2h_piece.jsonl
done; done; done
echo session-ok
