# round-6 session zl: host pool size (DECDS_HOST_THREADS) against the host blob paths at 1 GiB, two rounds
set -o pipefail
out=gpurun_out/r09zl; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do for t in 4 6 8 12 16; do
  DECDS_HOST_THREADS=$t timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch 16 --reps 5 --memory alloc > $out/tmp.json 2>> $out/e2e.err || { tail $out/e2e.err; exit 1; }
  sed "s/^{/{\"host_threads\": $t, /" $out/tmp.json >> $out/threads.jsonl
done; done
echo session-ok
