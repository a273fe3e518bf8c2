set -o pipefail
out=gpurun_out/r09r; mkdir -p $out; export TMPDIR=/tmp
DECDS_LIB=$PWD/tools/bin/lib_ptrace.so timeout -k 10 120 python tools/repair_phases.py --sizes 1,2 > $out/phases.jsonl 2> $out/phases.err || { tail $out/phases.err; exit 1; }
cat $out/phases.jsonl
