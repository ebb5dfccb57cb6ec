set -u
OUT=gpurun_out/r6d; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "vhead or value_forward or wgrad_row_major or phead_gate or head_kernels_match" > $OUT/t_vhead.log 2>&1 || { tail -40 $OUT/t_vhead.log; exit 1; }
tail -3 $OUT/t_vhead.log
for dt in bf16x3 bf16; do
  timeout -k 10 200 python -u scripts/ab_vhead.py $dt A,kb,h16,nostore 3 > $OUT/ab_vhead_$dt.log 2>&1 || { tail -20 $OUT/ab_vhead_$dt.log; exit 1; }
  tail -1 $OUT/ab_vhead_$dt.log
  timeout -k 10 200 python -u scripts/head_timeline.py $dt --vhead > $OUT/tl_$dt.json 2>&1 || { tail -20 $OUT/tl_$dt.json; exit 1; }
  grep -A 12 '"value"' $OUT/tl_$dt.json | tail -9
done
timeout -k 10 300 python -u scripts/ab_heads.py bf16x3 3 10 p32,pv32 > $OUT/ab_s3.log 2>&1 || { tail -20 $OUT/ab_s3.log; exit 1; }
tail -1 $OUT/ab_s3.log
timeout -k 10 300 python -u scripts/ab_heads.py bf16 3 10 p32,pv32 > $OUT/ab_bf16.log 2>&1 || { tail -20 $OUT/ab_bf16.log; exit 1; }
tail -1 $OUT/ab_bf16.log
timeout -k 10 300 python -u scripts/probe_side_kernel.py bf16x3 8,16,32,64 25 > $OUT/probe_side.log 2>&1 || { tail -20 $OUT/probe_side.log; exit 1; }
cat $OUT/probe_side.log | grep kernel
echo OK
