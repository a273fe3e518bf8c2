#!/bin/bash
# r02k: coded-row layout study (tools/layoutbench: the encode/decode access pattern with rows vs
# tile-major coded rows, against the flat copy), and the per-chunkset drop-in path under 1-16
# concurrent host threads next to the blob host paths (tools/mirror_bench.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02k; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py -m gpu -q --timeout 120 --timeout-method thread > $out/files_tests.log 2>&1 || { echo "FILES TESTS FAILED"; tail -30 $out/files_tests.log; exit 3; }
tail -1 $out/files_tests.log
timeout -k 10 240 tools/bin/layoutbench > $out/layout.jsonl 2> $out/layout.err || { echo layoutbench failed; tail $out/layout.err; exit 1; }
cat $out/layout.jsonl
timeout -k 10 400 python -u tools/mirror_bench.py --threads 1,4,16 --seconds 2 > $out/mirror.jsonl 2> $out/mirror.err || { echo mirror failed; tail $out/mirror.err; exit 2; }
cat $out/mirror.jsonl
echo session-ok
