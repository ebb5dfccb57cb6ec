#!/bin/bash
# PMC passes for the fused update kernel at both row tiles (DPPO_MLP_ROWS=32 / 64).
set -u
OUT=${OUT:-gpurun_out}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for R in 64 32; do
  i=0
  for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
    i=$((i+1))
    mkdir -p "$OUT/pmc_rows/r$R"
    DPPO_MLP_ROWS=$R timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex 'mlp_train|mlp_value' \
        -d "$OUT/pmc_rows/r$R/p$i" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 \
        > "$OUT/pmc_rows/r$R/p$i.log" 2>&1
    rc=$?
    echo "rows=$R pass $i rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_rows/r$R/p$i.log"; exit $rc; }
  done
done
