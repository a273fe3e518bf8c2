# round-6 session x: Blob::new's whole-blob digest from device group values (blob_group_kernel): the GPU
# suite, then tools/blob_breakdown.py with the device digest and with DECDS_BLOB_DIGEST=host, alternating
set -o pipefail
out=gpurun_out/r09x; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2; do
  timeout -k 10 300 python tools/blob_breakdown.py --gib 1 --repeats 7 --only encode_host_pinned,blob_new_pinned,blob_new_pageable > $out/tmp.json || exit 1
  sed "s/^{/{\"digest\": \"device\", /" $out/tmp.json >> $out/breakdown.jsonl
  DECDS_BLOB_DIGEST=host timeout -k 10 300 python tools/blob_breakdown.py --gib 1 --repeats 7 --only encode_host_pinned,blob_new_pinned,blob_new_pageable > $out/tmp.json || exit 1
  sed "s/^{/{\"digest\": \"host\", /" $out/tmp.json >> $out/breakdown.jsonl
done
echo session-ok
