#!/bin/bash
# r02d: compact (unreplicated) LDS tables — parity of the variants, LDS bank conflicts vs the
# replicated build, in-process A/B of units / order / prefetch at 103 / 256 / 1639 chunksets, and the
# codec access pattern with each side aligned (tools/hbmbench)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r02d; mkdir -p $out
export TMPDIR=/tmp
for v in ct ct1p ct2p ct1xp; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $out/${v}_tests.log; exit 1; }
  echo "$v $(tail -1 $out/${v}_tests.log)"
done
for v in cur ct; do
  DECDS_LIB=build/ab/lib_$v.so timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $out/pmc_$v -o run -- python3 tools/kbench.py --n 103 --reps 5 > $out/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $out/pmc_$v.log; exit 1; }
done
L="build/ab/lib_cur.so build/ab/lib_p.so build/ab/lib_ct.so build/ab/lib_ctp.so build/ab/lib_ct1.so build/ab/lib_ct1p.so build/ab/lib_ct2p.so build/ab/lib_ct1xp.so build/ab/lib_ct1p.so:1048592 build/ab/lib_ctp.so:1048592"
for n in 103 256 1639; do
  r=10; [ $n -ge 1024 ] && r=6
  timeout -k 10 300 python -u tools/abbench.py --n $n --rounds $r --warmup-s 2 $L > $out/ab$n.jsonl 2>&1 || { echo "AB FAILED"; tail $out/ab$n.jsonl; exit 1; }
done
for n in 103 256 1639; do grep -h tag $out/ab$n.jsonl; done | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-16s n=%5d enc %.4f (%.0f GB/s) dec %.4f (%.0f GB/s)' % (d['tag'], d['n'], d['encode_ms'], d['encode_GBps'], d['decode_ms'], d['decode_GBps']))"
timeout -k 10 300 tools/bin/hbmbench --gib 4 --only codec > $out/hbm.jsonl 2> $out/hbm.err || { echo hbmbench failed; exit 5; }
echo session-ok
