#!/bin/bash
# PMC counter passes over a short bench run (counters only with --kernel-trace; never with
# sys/runtime traces).  Output: gpurun_out/pmc/<pass>/...
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT/pmc"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rocprofv3 -L > "$OUT/pmc/counters_list.txt" 2>&1 || true
REGEX=${REGEX:-'mlp_head|mlp_train|wgrad_kernel|rollout_kernel|mlp_value|gather_adam|phead'}
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
         "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" \
         "FETCH_SIZE" \
         "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $P"
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$REGEX" -d "$OUT/pmc/p$i" -o run \
      --output-format csv -- python3 bench.py --steps 1 --warmup 1 --variants "" ${BENCH_ARGS:-} > "$OUT/pmc/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$OUT/pmc/p$i.log"; [ $rc -ge 124 ] && exit $rc; }
done
exit 0
