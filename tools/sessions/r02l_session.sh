#!/bin/bash
# r02l: message tiling (16-byte-aligned rows: tiles = 4 BLAKE3 chunks) and the fused ChunkSet::new
# (rlnc_encode_kernel<COMMIT> + commit_fold_kernel): parity first (commit + codec suites), then the
# bench line (commitment.chunkset_new: fused vs separate), then the plain encode on the old layout
# (payload 128-B aligned, rows at +118) against the message layout (rows at +16), in-process A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02l; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_parity.py tests/test_gpu_files.py -m gpu -v -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail $out/bench.err; exit 4; }
python -c "
import json; d=json.load(open('$out/bench.json')); print(d['value'], d['breakdown']); print(d['commitment']); print([ (x['chunksets'], x['frac']) for x in d['encode_batch_sweep']])"
L="build/ab/lib_msg.so:1048704+118 build/ab/lib_msg.so:1048704+16 build/ab/lib_cur.so:1048704+118 build/ab/lib_cur.so:1048704+16"
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
