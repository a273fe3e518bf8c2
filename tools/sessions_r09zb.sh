# round-6 session zb: the small-batch encode form (8-column blocks, 4 waves/SIMD) against the 16-column sweep
# at 4 .. 64 chunksets on the aligned layout (in-process, knob-forced)
set -o pipefail
out=gpurun_out/r09zb; mkdir -p $out; export TMPDIR=/tmp
for nn in 4 8 16 32 64; do
  timeout -k 10 300 python tools/abbench.py --n $nn --rounds 20 default:1048704+118 default:1048704+118@DECDS_ENC_SMALL_MAX_N=1024 > $out/ab_$nn.jsonl 2> $out/ab_$nn.err || { tail $out/ab_$nn.err; exit 1; }
done
echo session-ok
