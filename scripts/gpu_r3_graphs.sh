# hipGraph replay at a small, launch-bound config (InvertedPendulum dims, 64 envs x 16 steps): on/off, both update paths
set -u
OUT=gpurun_out/graphs; mkdir -p $OUT
for i in 1 2; do
  for heads in 1 0; do
    for g in "" "--graphs"; do
      tag=h${heads}${g:+_graphs}_$i
      DPPO_HEADS=$heads timeout -k 10 200 python3 bench.py --steps 50 --warmup 5 --variants "" --dtype bf16 --env-name InvertedPendulum-v1 --num-envs 64 --rollout-len 16 $g > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
      tail -1 $OUT/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step'],3), 'ms')"
    done
  done
done
