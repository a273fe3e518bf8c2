# round-6 session j: D2H piece size for the host paths (encode is D2H-bound), 1 and 2 GiB
set -o pipefail
out=gpurun_out/r09j; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2 3; do for mb in 16 32 64 128; do for g in 1 2; do
  DECDS_D2H_PIECE_MB=$mb timeout -k 10 120 python tools/e2e_bench.py --gib $g --batch 16 --reps 5 --memory alloc > $out/tmp.json || exit 1
  sed "s/^{/{\"piece_mb\": $mb, /" $out/tmp.json >> $out/d2h_piece.jsonl
done; done; done
echo session-ok
