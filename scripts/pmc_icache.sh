#!/bin/bash
# Instruction-fetch counters of the fused update / rollout kernels (one PMC pass).
set -u
OUT=${OUT:-gpurun_out}/pmc_icache
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES \
    --kernel-include-regex "${1:-mlp_train|rollout_kernel|wgrad_kernel}" -d "$OUT" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > "$OUT/log" 2>&1
