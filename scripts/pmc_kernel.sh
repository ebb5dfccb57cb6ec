#!/bin/bash
# PMC passes for one kernel (regex $1) over a short bench run; one pass per counter group.
# Output: gpurun_out/pmc_<tag>/p<i>/...   usage: bash scripts/pmc_kernel.sh 'wgrad_kernel' wgrad
set -u
REGEX=$1; TAG=${2:-k}
OUT=${OUT:-gpurun_out}/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
         "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$REGEX" -d "$OUT/p$i" -o run \
      --output-format csv -- python3 bench.py --steps 1 --warmup 1 --variants "" ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
