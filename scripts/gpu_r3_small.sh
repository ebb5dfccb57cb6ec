# per-head vs tile update by batch size (which path small configs should take)
set -u
OUT=gpurun_out/small; mkdir -p $OUT
for cfg in "HalfCheetah-v2 1024 bf16" "Humanoid-v2 1024 bf16x3" "Humanoid-v2 256 bf16x3" "InvertedPendulum-v1 256 bf16"; do
  set -- $cfg
  for heads in 1 0; do
    tag=${1}_${2}_${3}_h$heads
    DPPO_HEADS=$heads timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --variants "" --dtype $3 --env-name $1 --num-envs $2 --rollout-len 16 > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
    tail -1 $OUT/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step'],3), 'ms')"
  done
done
