#!/bin/bash
# r02zd: blob host paths by memory kind (pageable / decds_host_alloc / registered caller memory),
# huge-page registered library buffers (default) against hipHostMalloc ones (hm), alternating
# processes twice so box drift shows; then the e2e bench once per build
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02zd; mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do
for v in default hm; do
  lib=decds_amd/libdecds_rlnc.so; [ $v = hm ] && lib=build/ab/lib_hm.so
  DECDS_LIB=$lib timeout -k 10 300 python -u tools/mirror_bench.py --blob-only --reps 5 > $out/blob_${v}_$i.jsonl 2> $out/blob_${v}_$i.err || { echo "blob $v failed"; tail $out/blob_${v}_$i.err; exit 2; }
  echo "== $v $i"; cat $out/blob_${v}_$i.jsonl
done
done
for v in default hm; do
  lib=decds_amd/libdecds_rlnc.so; [ $v = hm ] && lib=build/ab/lib_hm.so
  DECDS_LIB=$lib timeout -k 10 300 python -u tools/mirror_bench.py --threads 1,4,16 --seconds 2 --modes pageable > $out/mirror_$v.jsonl 2> $out/mirror_$v.err || { echo "mirror $v failed"; tail $out/mirror_$v.err; exit 3; }
  echo "== mirror $v"; cat $out/mirror_$v.jsonl
done
echo session-ok
