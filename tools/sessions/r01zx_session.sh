#!/bin/bash
# Memory-side counters of the codec kernels (one rocprofv3 --pmc pass per group, each within the
# per-block limits): L2-to-DRAM request sizes and credit stalls, L2 hit rate, TA/TCP stalls.
set -o pipefail
out=${1:-gpurun_out/r01zx}
mkdir -p $out
export TMPDIR=/tmp
bcmd="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-commit"
i=0
for pmc in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_TAG_STALL_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o bench -- $bcmd > $out/pmc$i.log 2>&1 || { echo "PMC $i FAILED"; tail -5 $out/pmc$i.log; exit 1; }
done
echo session-ok
