#!/bin/bash
# r02m: fused ChunkSet::new with 8-column blocks at 3 waves per SIMD (fd2) against 16-column blocks
# at 2 (msg): parity of fd2's commitment, tools/fusebench (fused vs separate kernels, cfg2 and 256 cs);
# plain encode on the old layout (rows at +118) against the message layout (+16); layout study and
# the per-chunkset mirror under concurrent host threads
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02m; mkdir -p $out
export TMPDIR=/tmp
DECDS_LIB=build/ab/lib_fd2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/fd2_tests.log 2>&1 || { echo "fd2 TESTS FAILED"; tail -30 $out/fd2_tests.log; exit 1; }
tail -1 $out/fd2_tests.log
for n in 103 256; do
  timeout -k 10 300 python -u tools/fusebench.py --n $n --rounds 8 build/ab/lib_msg.so build/ab/lib_fd2.so > $out/fuse$n.jsonl 2>&1 || { echo "FUSE FAILED"; tail $out/fuse$n.jsonl; exit 1; }
  cat $out/fuse$n.jsonl
done
L="build/ab/lib_msg.so:1048704+118 build/ab/lib_msg.so:1048704+16"
for n in 103 256 1024; do
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds 8 --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1024; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-28s n=%5d enc %.4f (%.0f GB/s) dec %.4f (%.0f GB/s)' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps']))"
timeout -k 10 240 tools/bin/layoutbench > $out/layout.jsonl 2> $out/layout.err || { echo layoutbench failed; tail $out/layout.err; exit 1; }
timeout -k 10 400 python -u tools/mirror_bench.py --threads 1,4,16 --seconds 2 > $out/mirror.jsonl 2> $out/mirror.err || { echo mirror failed; tail $out/mirror.err; exit 2; }
echo session-ok
