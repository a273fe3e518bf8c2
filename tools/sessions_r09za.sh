# round-6 session za: wave priority by closeness to the sweep's end (DECDS_ENC_TAIL_PRIO) — in-process A/B
# against the shipped build at 16 / 64 / 256 / 1639 chunksets, and its phase timeline with placement
set -o pipefail
out=gpurun_out/r09za; mkdir -p $out; export TMPDIR=/tmp
for nn in 16 64 256 1639; do
  timeout -k 10 300 python tools/abbench.py --n $nn --rounds 16 --check default tools/bin/lib_tailprio.so > $out/ab_$nn.jsonl 2> $out/ab_$nn.err || { tail $out/ab_$nn.err; exit 1; }
done
DECDS_LIB=$PWD/tools/bin/lib_tailprio_ptrace.so timeout -k 10 120 python tools/phasetrace.py --sizes 16,64 --runs 3 > $out/phases.jsonl 2> $out/phases.err || { tail $out/phases.err; exit 1; }
echo session-ok
