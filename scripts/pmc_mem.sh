#!/bin/bash
# Memory-path PMC passes for the update kernels (regex $1, default wgrad + head kernels): L2->fabric
# read queue level (Little's law latency), DRAM credit stalls, TA busy / stalls.  One pass per
# counter group (<= 4 TCC, <= 2 TA counters each).  Output: gpurun_out/pmc_mem/p<i>/
set -u
REGEX=${1:-'wgrad_kernel|mlp_head'}
OUT=${OUT:-gpurun_out}/pmc_mem
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for P in "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE" \
         "TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum TCC_BUSY_sum GRBM_GUI_ACTIVE" \
         "TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$REGEX" -d "$OUT/p$i" -o run \
      --output-format csv -- python3 bench.py --steps 1 --warmup 1 --variants "" ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
