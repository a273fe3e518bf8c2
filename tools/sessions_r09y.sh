# round-6 session y: the host pool's spin-before-sleep (DECDS_HOST_SPIN_US 200 vs 0) on the reference's
# bench shapes through the blob API and on the host blob paths, alternating
set -o pipefail
out=gpurun_out/r09y; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do for sp in 200 0; do
  DECDS_HOST_SPIN_US=$sp timeout -k 10 300 python tools/api_shape_ab.py --gib 1 --tag spin$sp >> $out/api.jsonl 2>> $out/api.err || { tail $out/api.err; exit 1; }
  DECDS_HOST_SPIN_US=$sp timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch 16 --reps 5 --memory alloc > $out/tmp.json 2>> $out/e2e.err || { tail $out/e2e.err; exit 1; }
  sed "s/^{/{\"spin_us\": $sp, /" $out/tmp.json >> $out/e2e.jsonl
done; done
echo session-ok
