# round-6 session f: parity + host-path tests, fused repair latency, repair A/B + copy timeline, full cfg3 bench
set -o pipefail
out=gpurun_out/r09f; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hostpath.py tests/test_gpu_blob.py tests/test_gpu_validate.py tests/test_gpu_files.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for nn in 1 16; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt$nn -o kb -- python3 tools/kbench.py --n $nn --reps 50 --repair --check > $out/kbench$nn.json 2>$out/kbench$nn.err || { tail $out/kbench$nn.err; exit 1; }
done
for rep in 1 2; do for cfg in "1 3 16" "1 4 16" "1 3 8" "0 3 16"; do set -- $cfg
  DECDS_REPAIR_GATHER=$1 DECDS_REPAIR_SLOTS=$2 timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch $3 --reps 5 --memory alloc > $out/tmp.json || exit 1
  sed "s/^{/{\"gather\": $1, \"slots\": $2, /" $out/tmp.json >> $out/repair_ab.jsonl
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/mt -o e2e -- python3 tools/e2e_bench.py --gib 1 --batch 16 --reps 3 --memory alloc > $out/e2e_traced.json 2>$out/e2e_traced.err || { tail $out/e2e_traced.err; exit 1; }
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cut -c1-400 $out/bench.json
echo session-ok
