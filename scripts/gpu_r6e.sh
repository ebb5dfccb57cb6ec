set -u
OUT=gpurun_out/r6e; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for dt in bf16x3 bf16; do
  timeout -k 10 240 python -u scripts/ab_vhead.py $dt A,late,hot,nostore,spread,h16 3 > $OUT/ab_vhead_$dt.log 2>&1 || { tail -20 $OUT/ab_vhead_$dt.log; exit 1; }
  tail -1 $OUT/ab_vhead_$dt.log
done
for arm in off on; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --variants "" --force-collectives --overlap-value $arm > $OUT/forced_$arm.log 2>&1 || { tail -20 $OUT/forced_$arm.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"overlap_value_step": "[a-z_]*"\|"overlapped_value_steps_per_iter": [0-9.]*' $OUT/forced_$arm.log | tr '\n' ' '; echo " $arm"
done
for arm in off on; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --variants "" --force-collectives --overlap-value $arm > $OUT/forced2_$arm.log 2>&1 || { tail -20 $OUT/forced2_$arm.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $OUT/forced2_$arm.log | tr '\n' ' '; echo " $arm"
done
echo OK
