# round-6 session ze: the encode's first tile at 1 / 16 / 64 chunksets: when the coefficient bytes arrive,
# when their tables are built, when they are ready for all waves (DECDS_PHASE_TRACE build)
set -o pipefail
out=gpurun_out/r09ze; mkdir -p $out; export TMPDIR=/tmp
DECDS_LIB=$PWD/tools/bin/lib_ptrace.so timeout -k 10 120 python tools/phasetrace.py --sizes 1,16,64 --runs 3 > $out/phases.jsonl 2> $out/phases.err || { tail $out/phases.err; exit 1; }
echo session-ok
