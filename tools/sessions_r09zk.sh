# round-6 session zk: the 8-column small-batch forms against the 16-column ones at 1 / 2 chunksets, timed as
# bench.py's sweep times them (tools/tiny_ab.py: DECDS_ENC_SMALL_MAX_N, DECDS_DEC_NARROW_MAX_N)
set -o pipefail
out=gpurun_out/r09zk; mkdir -p $out; export TMPDIR=/tmp
for nn in 1 2; do
  timeout -k 10 300 python tools/tiny_ab.py --n $nn --rounds 8 > $out/forms_ab_$nn.jsonl 2> $out/forms_ab.err || { tail $out/forms_ab.err; exit 1; }
done
echo session-ok
