#!/bin/bash
# Round 3: the BASELINE.json configs end to end through train.py on one MI355X, plus 300-iteration
# learning curves at the headline geometry (Humanoid dims, 4096 envs x 16 steps) from one seed at
# fp32-accurate split-bf16, exact fp32 MFMA and fp8 (e4m3 forward GEMMs + e4m3 wgrad operands).
# Each step has its own time limit; the script stops at the first failure.
set -u
OUT=${OUT:-gpurun_out/e2e3}
rm -rf "$OUT"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; return $rc; }
run cfg2_halfcheetah_bf16 300 python train.py --preset dppo --device gpu --env-name HalfCheetah-v2 --num-envs 1024 \
    --exploration-size 16384 --batch-size 16384 --dtype bf16 --max-iters 60 --num-processes 1 \
    --log-jsonl "$OUT/cfg2.jsonl" || exit $?
DPPO_DIST_BACKEND=gloo run cfg3_walker_4ranks 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29677 train.py --preset dppo --device gpu --env-name Walker2d-v2 \
    --num-envs 256 --exploration-size 4096 --batch-size 4096 --dtype bf16x3 --max-iters 10 \
    --verify-sync-every 5 --log-jsonl "$OUT/cfg3.jsonl" || exit $?
for dt in bf16x3 fp8 fp32; do
  run humanoid_${dt}_300 400 python train.py --preset dppo --device gpu --env-name Humanoid-v2 --num-envs 4096 \
      --exploration-size 65536 --batch-size 65536 --dtype $dt --max-iters 300 --num-processes 1 --seed 5 \
      --log-jsonl "$OUT/humanoid_${dt}.jsonl" || exit $?
done
echo "== done"
