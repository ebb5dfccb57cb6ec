set -u
OUT=gpurun_out/r6i; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for dt in bf16x3 bf16; do
  timeout -k 10 400 python -u scripts/ab_heads.py $dt 3 10 p32,fc1,narrow > $OUT/ab_heads_$dt.log 2>&1 || { tail -20 $OUT/ab_heads_$dt.log; exit 1; }
  tail -1 $OUT/ab_heads_$dt.log
done
timeout -k 10 400 python -u scripts/ab_iter.py bf16x3 A,sb24,sb32 3 10 > $OUT/ab_iter_sb.log 2>&1 || { tail -20 $OUT/ab_iter_sb.log; exit 1; }
tail -1 $OUT/ab_iter_sb.log
echo OK
