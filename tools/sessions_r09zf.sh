# round-6 session zf: the encode's first-tile coefficient bytes by scalar loads (DECDS_ENC_FIRST_COEF) —
# in-process A/B on the aligned layout at 1 .. 1639 chunksets (outputs checked), then its phase timeline
set -o pipefail
out=gpurun_out/r09zf; mkdir -p $out; export TMPDIR=/tmp
for nn in 1 2 16 64 256 1639; do
  timeout -k 10 300 python tools/abbench.py --n $nn --rounds 20 --check default:1048704+118 tools/bin/lib_firstcoef.so:1048704+118 > $out/ab_$nn.jsonl 2> $out/ab_$nn.err || { tail $out/ab_$nn.err; exit 1; }
done
DECDS_LIB=$PWD/tools/bin/lib_firstcoef_ptrace.so timeout -k 10 120 python tools/phasetrace.py --sizes 1,16,64 --runs 3 > $out/phases.jsonl 2> $out/phases.err || { tail $out/phases.err; exit 1; }
echo session-ok
