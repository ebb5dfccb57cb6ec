#!/bin/bash
# End-to-end on one MI355X: train.py (DPPO preset, GPU engine) with checkpoints + the evaluator
# process, resume from the checkpoint, the single-process PPO preset, and a reference-format
# model.pt load.  Each step has its own time limit; stops at the first failure.
set -u
OUT=${OUT:-gpurun_out/e2e}
rm -rf "$OUT"; mkdir -p "$OUT"
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "rc=$rc"; tail -3 "$OUT/$name.log"; return $rc; }
run dppo_train 240 python train.py --preset dppo --device gpu --env-name Humanoid-v2 --num-envs 256 \
    --exploration-size 4096 --batch-size 4096 --dtype bf16 --max-iters 4 --num-processes 1 \
    --checkpoint-dir "$OUT/ckpt" --checkpoint-every 2 --eval-every 2 --log-jsonl "$OUT/train.jsonl" \
    --log-csv "$OUT/curve.csv" || exit $?
run dppo_resume 240 python train.py --preset dppo --device gpu --env-name Humanoid-v2 --num-envs 256 \
    --exploration-size 4096 --batch-size 4096 --dtype bf16 --max-iters 6 --num-processes 1 \
    --resume "$OUT/ckpt" --log-jsonl "$OUT/resume.jsonl" || exit $?
run ppo_train 240 python ppo.py --device gpu --env-name HalfCheetah-v2 --num-envs 64 --num-steps 2048 \
    --exploration-size 2048 --max-iters 3 --dtype bf16 || exit $?
run load_ref 120 python -c "
import torch, glob, sys
sys.path.insert(0, '.')
from pytorch_dppo_amd.models.actor_critic import ActorCritic
p = sorted(glob.glob('$OUT/ckpt/**/model.pt', recursive=True))[0]
sd = torch.load(p, weights_only=True)
m = ActorCritic(376, 17); m.load_state_dict(sd, strict=True)
print('model.pt', p, 'keys', list(sd)[:3], 'ok')
" || exit $?
echo "== jsonl tail"; tail -2 "$OUT/resume.jsonl"
