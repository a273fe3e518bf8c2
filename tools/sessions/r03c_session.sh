#!/bin/bash
# wave-step fused ChunkSet::new: A/B of priority / no-hash study builds, kernel trace, PMC pass
set -o pipefail
out=gpurun_out/r03c; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fusebench.py --no-check --n 103 --rounds 8 build/ab/lib_wave3.so build/ab/lib_prio.so build/ab/lib_nohash.so > $out/fuse_103.jsonl 2>&1 || { echo FUSE FAILED; tail -20 $out/fuse_103.jsonl; exit 1; }
cat $out/fuse_103.jsonl
cmd="python3 tools/fusebench.py --n 103 --rounds 4 --warmup-s 0.5 build/ab/lib_wave3.so"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o fuse -- $cmd > $out/trace.log 2>&1 || { echo TRACE FAILED; tail -5 $out/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $out/pmc1 -o fuse -- $cmd > $out/pmc1.log 2>&1 || { echo PMC FAILED; tail -5 $out/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc2 -o fuse -- $cmd > $out/pmc2.log 2>&1 || { echo PMC2 FAILED; tail -5 $out/pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $out/pmc3 -o fuse -- $cmd > $out/pmc3.log 2>&1 || { echo PMC3 FAILED; tail -5 $out/pmc3.log; exit 1; }
echo ok
