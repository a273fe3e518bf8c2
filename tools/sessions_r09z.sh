# round-6 session v: encode phase timeline with placement at 16 / 64 chunksets on the current kernels (DECDS_PHASE_TRACE build)
set -o pipefail
out=gpurun_out/r09z; mkdir -p $out; export TMPDIR=/tmp
DECDS_LIB=$PWD/tools/bin/lib_ptrace.so timeout -k 10 120 python tools/phasetrace.py --sizes 16,64 --runs 3 > $out/phases.jsonl 2> $out/phases.err || { tail $out/phases.err; exit 1; }
echo session-ok
