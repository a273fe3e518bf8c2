#!/bin/bash
# r02ze: blob encode with the whole range's coding vectors uploaded once (no per-batch staged
# copy): host-path parity, then the blob host paths by memory kind for huge-page registered
# library buffers (default) and hipHostMalloc ones (hm), twice each, and the e2e bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02ze; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hostpath.py tests/test_gpu_blob.py tests/test_gpu_validate.py tests/test_gpu_files.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
for v in default hm; do
  lib=decds_amd/libdecds_rlnc.so; [ $v = hm ] && lib=build/ab/lib_hm.so
  DECDS_LIB=$lib timeout -k 10 300 python -u tools/mirror_bench.py --blob-only --reps 5 > $out/blob_${v}_$i.jsonl 2> $out/blob_${v}_$i.err || { echo "blob $v failed"; tail $out/blob_${v}_$i.err; exit 2; }
  echo "== $v $i"; cat $out/blob_${v}_$i.jsonl
done
done
timeout -k 10 300 python -u tools/e2e_bench.py --gib 4 --batch 16 > $out/e2e.json 2> $out/e2e.err || { echo "e2e failed"; tail $out/e2e.err; exit 3; }
cat $out/e2e.json
echo session-ok
