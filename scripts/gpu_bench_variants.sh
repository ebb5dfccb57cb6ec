#!/bin/bash
# bench variants on one box: dtype x overlap x collectives; each run time-limited, stop on fault
set -u
OUT=${OUT:-gpurun_out}
STEPS=${STEPS:-20}
mkdir -p "$OUT"
for v in "bf16" "bf16 --overlap-rollout" "bf16 --force-collectives" "bf16 --force-collectives --grad-buckets on" \
         "bf16 --graphs" "fp8" "fp32"; do
  set -- $v
  name="bench_$(echo $v | tr ' -' '__')"
  timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 --dtype $v > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-260
  [ $rc -eq 0 ] || exit $rc
done
