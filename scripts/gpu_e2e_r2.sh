#!/bin/bash
# BASELINE.json configs end to end on one MI355X through train.py (the product entry point),
# at the fp32-accurate default dtype unless the config names one:
#   cfg2  HalfCheetah-v2, 1 worker, 1024 vectorised envs, bf16 (as BASELINE names it) -- learning curve
#   cfg3  Walker2d-v2, 4 DPPO workers: 4 torchrun ranks sharing this one GPU over gloo
#         (DPPO_DIST_BACKEND=gloo: RCCL refuses two ranks on one device; the 4-GPU run is RCCL)
#   cfg4  Humanoid-v2, 65k-step HBM-resident buffer: one worker of the 8 (bench.py covers the node)
#   cfg5  Humanoid-v2 with the fp8 forward GEMMs
# Each step has its own time limit; the script stops at the first failure.
set -u
OUT=${OUT:-gpurun_out/e2e2}
rm -rf "$OUT"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "rc=$rc"; tail -n 3 "$OUT/$name.log"; return $rc; }
run cfg2_halfcheetah_bf16 300 python train.py --preset dppo --device gpu --env-name HalfCheetah-v2 --num-envs 1024 \
    --exploration-size 16384 --batch-size 16384 --dtype bf16 --max-iters 60 --num-processes 1 \
    --log-jsonl "$OUT/cfg2.jsonl" --log-csv "$OUT/cfg2.csv" || exit $?
run cfg2_halfcheetah_bf16x3 300 python train.py --preset dppo --device gpu --env-name HalfCheetah-v2 --num-envs 1024 \
    --exploration-size 16384 --batch-size 16384 --dtype bf16x3 --max-iters 60 --num-processes 1 \
    --log-jsonl "$OUT/cfg2_s3.jsonl" --log-csv "$OUT/cfg2_s3.csv" || exit $?
DPPO_DIST_BACKEND=gloo run cfg3_walker_4ranks 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29677 train.py --preset dppo --device gpu --env-name Walker2d-v2 \
    --num-envs 256 --exploration-size 4096 --batch-size 4096 --dtype bf16x3 --max-iters 10 \
    --verify-sync-every 5 --log-jsonl "$OUT/cfg3.jsonl" || exit $?
run cfg4_humanoid_65k 300 python train.py --preset dppo --device gpu --env-name Humanoid-v2 --num-envs 4096 \
    --exploration-size 65536 --batch-size 65536 --dtype bf16x3 --max-iters 20 --num-processes 1 \
    --log-jsonl "$OUT/cfg4.jsonl" || exit $?
run cfg5_humanoid_fp8 300 python train.py --preset dppo --device gpu --env-name Humanoid-v2 --num-envs 4096 \
    --exploration-size 65536 --batch-size 65536 --dtype fp8 --max-iters 20 --num-processes 1 \
    --log-jsonl "$OUT/cfg5.jsonl" || exit $?
echo "== done"
