# round-6 session e: fused repair parity + latency, host-path A/Bs, Blob::new breakdown, bench extras
set -o pipefail
out=gpurun_out/r09e; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hostpath.py tests/test_gpu_files.py tests/test_gpu_blob.py tests/test_gpu_validate.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for nn in 1 2 16; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt$nn -o kb -- python3 tools/kbench.py --n $nn --reps 50 --repair --check > $out/kbench$nn.json 2>$out/kbench$nn.err || { tail $out/kbench$nn.err; exit 1; }
done
for rep in 1 2; do for sl in 3 4 5; do for b in 8 16; do
  DECDS_REPAIR_SLOTS=$sl timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch $b --reps 5 --memory alloc > $out/tmp.json || exit 1
  sed "s/^{/{\"slots\": $sl, /" $out/tmp.json >> $out/repair_slots.jsonl
done; done; done
for rep in 1 2; do for m in default h2d; do
  if [ $m = default ]; then timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch 16 --reps 5 --memory alloc > $out/tmp.json || exit 1
  else DECDS_PIPE_STREAMS=h2d timeout -k 10 120 python tools/e2e_bench.py --gib 1 --batch 16 --reps 5 --memory alloc > $out/tmp.json || exit 1; fi
  sed "s/^{/{\"pipe\": \"$m\", /" $out/tmp.json >> $out/pipe_streams.jsonl
done; done
timeout -k 10 200 python tools/blob_breakdown.py --gib 1 --only encode_host_pinned,encode_host_pageable,blob_new_pinned,blob_new_pageable > $out/breakdown.json || exit 1
( time timeout -k 10 500 python bench.py --config cfg2 --steps 2 --warmup 1 --no-cpu-baseline --no-sweep --no-commit > $out/bench_api.json ) 2> $out/bench_api.err || { tail $out/bench_api.err; exit 1; }
tail -3 $out/bench_api.err
echo session-ok
