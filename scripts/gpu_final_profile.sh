#!/bin/bash
# One GPU call that refreshes the committed profiles of the current tree:
#   bench (3 x 20 steps), rocprofv3 kernel trace + stats, PMC passes of the four hot kernels,
#   phase timeline of the fused update and the rollout.
# Outputs under gpurun_out/final/; scripts/kernel_stats_md.py and scripts/pmc_print.py turn them
# into the profiles/*.md summaries.  Each GPU step has its own time limit and the script stops at
# the first failure.
set -u
OUT=${OUT:-gpurun_out/final}
rm -rf "$OUT"; mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit $?
  tail -1 "$OUT/bench_$i.json"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > "$OUT/prof.log" 2>&1 || exit $?
OUT="$OUT" bash scripts/pmc_kernel.sh "mlp_train|wgrad_kernel|rollout_kernel|mlp_value" hot > "$OUT/pmc.log" 2>&1 || exit $?
timeout -k 10 200 python scripts/phase_timeline.py bf16 > "$OUT/timeline.json" 2> "$OUT/timeline.err" || exit $?
echo done
