set -u
OUT=gpurun_out/r6c; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for dt in bf16x3 bf16; do
  timeout -k 10 200 python -u scripts/ab_vhead.py $dt A,h16,nostore,nodma,v3 3 > $OUT/ab_vhead_$dt.log 2>&1 || { tail -20 $OUT/ab_vhead_$dt.log; exit 1; }
  tail -1 $OUT/ab_vhead_$dt.log
  timeout -k 10 200 python -u scripts/head_timeline.py $dt --vhead > $OUT/tl_$dt.json 2>&1 || { tail -20 $OUT/tl_$dt.json; exit 1; }
  grep -A 12 '"value"' $OUT/tl_$dt.json
done
echo OK
