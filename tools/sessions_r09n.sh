# round-6 session n: persistent per-context host pipe vs streams + events per call
set -o pipefail
out=gpurun_out/r09n; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hostpath.py tests/test_gpu_blob.py tests/test_gpu_files.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3; do for lib in default tools/bin/lib_pipe_percall.so; do for g in 1 0.05; do
  if [ $lib = default ]; then envs=""; tag=persistent; else envs="DECDS_LIB=$PWD/$lib"; tag=percall; fi
  env $envs timeout -k 10 120 python tools/e2e_bench.py --gib $g --batch 16 --reps 7 --memory alloc > $out/tmp.json || exit 1
  sed "s/^{/{\"pipe\": \"$tag\", /" $out/tmp.json >> $out/pipe_ab.jsonl
done; done; done
timeout -k 10 200 python tools/blob_breakdown.py --gib 1 --only encode_host_pinned,blob_new_pinned,blob_new_pageable > $out/breakdown.json || exit 1
echo session-ok
