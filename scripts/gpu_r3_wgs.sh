#!/bin/bash
# wgrad task count (DPPO_WGRAD_WGS: split-K chunks per launch; 0 = one per CU) vs iteration time,
# fp8 and split-bf16, one bench invocation per setting on one box
set -u
OUT=gpurun_out/wgs; mkdir -p $OUT
for dt in fp8 bf16x3; do
  for n in 0 128 384 512; do
    DPPO_WGRAD_WGS=$n timeout -k 10 300 python bench.py --steps 10 --warmup 2 --dtype $dt --variants "" > $OUT/${dt}_$n.log 2>&1 || { tail -5 $OUT/${dt}_$n.log; exit 1; }
    echo "$dt wgs=$n $(tail -1 $OUT/${dt}_$n.log | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
