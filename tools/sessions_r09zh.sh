# round-6 session zh: 4-column lane blocks (DW=1) for the small-batch encode and the narrow one-tile decode —
# in-process A/B at 1 / 2 chunksets (outputs checked), kernel trace of the fused repair
set -o pipefail
out=gpurun_out/r09zh; mkdir -p $out; export TMPDIR=/tmp
for nn in 1 2; do
  timeout -k 10 300 python tools/abbench.py --n $nn --rounds 30 --check default:1048704+118 tools/bin/lib_dw1.so:1048704+118 > $out/ab_$nn.jsonl 2> $out/ab_$nn.err || { tail $out/ab_$nn.err; exit 1; }
done
for lib in default tools/bin/lib_dw1.so; do for nn in 1 2; do
  tag=$(basename $lib .so)_$nn
  if [ $lib = default ]; then envs=""; else envs="DECDS_LIB=$PWD/$lib"; fi
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$tag -o kb -- python3 tools/kbench.py --n $nn --reps 40 --repair --check > $out/kbench_$tag.json 2>$out/kbench_$tag.err || { tail $out/kbench_$tag.err; exit 1; }
done; done
echo session-ok
