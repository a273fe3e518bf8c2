#!/bin/bash
# r02zg: chunk digest kernel with one compression copy per alignment variant (dgc, 40 KB of code)
# against the unrolled form (dgu, 167 KB): commitment parity, then decds_commit_batch A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02zg; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_validate.py -m gpu -q -x --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python -u tools/digestbench.py --n 103 build/ab/lib_dgc.so build/ab/lib_dgu.so > $out/digest.jsonl 2>&1 || { echo "DIGEST FAILED"; tail $out/digest.jsonl; exit 2; }
cat $out/digest.jsonl
echo session-ok
