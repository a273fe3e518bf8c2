# round-6 session i: repair host path knobs (D2H piece size, host threads, ramp), default bench wall time
set -o pipefail
out=gpurun_out/r09i; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do for cfg in "base" "DECDS_D2H_PIECE_MB=64" "DECDS_D2H_PIECE_MB=4" "DECDS_HOST_THREADS=4" "DECDS_HOST_RAMP=0" "DECDS_HOST_THREADS=12"; do
  if [ $cfg = base ]; then timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch 16 --reps 5 --memory alloc > $out/tmp.json || exit 1
  else env $cfg timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch 16 --reps 5 --memory alloc > $out/tmp.json || exit 1; fi
  sed "s/^{/{\"knob\": \"$cfg\", /" $out/tmp.json >> $out/repair_knobs.jsonl
done; done
timeout -k 10 120 python tools/e2e_bench.py --gib 2 --batch 16 --reps 3 --memory alloc > $out/e2e_2gib.json || exit 1
( time timeout -k 10 900 python bench.py > $out/bench_default.json ) 2> $out/bench_default.err || { tail $out/bench_default.err; exit 1; }
tail -4 $out/bench_default.err
echo session-ok
