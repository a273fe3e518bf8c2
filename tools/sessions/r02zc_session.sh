#!/bin/bash
# r02zc: huge-page anonymous memory + hipHostRegister for the library's large page-locked buffers
# (rings, lane staging, decds_host_alloc) against non-coherent hipHostMalloc memory (hm): host-path parity,
# then the per-chunkset mirror and blob host paths (tools/mirror_bench.py) and tools/e2e_bench.py for both
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02zc; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hostpath.py tests/test_gpu_blob.py tests/test_gpu_validate.py tests/test_gpu_files.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in default hm; do
  lib=decds_amd/libdecds_rlnc.so; [ $v = hm ] && lib=build/ab/lib_hm.so
  DECDS_LIB=$lib timeout -k 10 400 python -u tools/mirror_bench.py --threads 1,4,16 --seconds 2 > $out/mirror_$v.jsonl 2> $out/mirror_$v.err || { echo "mirror $v failed"; tail $out/mirror_$v.err; exit 2; }
  DECDS_LIB=$lib timeout -k 10 300 python -u tools/e2e_bench.py --gib 4 --batch 16 > $out/e2e_$v.json 2> $out/e2e_$v.err || { echo "e2e $v failed"; tail $out/e2e_$v.err; exit 3; }
  echo "== $v"; cat $out/mirror_$v.jsonl $out/e2e_$v.json
done
echo session-ok
