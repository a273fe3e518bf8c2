# round-6 session zj: one-chunkset forms, 4-column vs 8-column, timed as bench.py's sweep times them
set -o pipefail
out=gpurun_out/r09zj; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python tools/tiny_ab.py --n 1 --rounds 8 > $out/tiny_ab_1.jsonl 2> $out/tiny_ab.err || { tail $out/tiny_ab.err; exit 1; }
timeout -k 10 300 python tools/tiny_ab.py --n 1 --rounds 8 --n-alloc 1639 > $out/tiny_ab_1_big.jsonl 2>> $out/tiny_ab.err || { tail $out/tiny_ab.err; exit 1; }
echo session-ok
