set -u
OUT=gpurun_out/r6b; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "vhead or value_forward or wgrad_row_major or phead_gate" > $OUT/t_vhead.log 2>&1 || { tail -30 $OUT/t_vhead.log; exit 1; }
tail -3 $OUT/t_vhead.log
timeout -k 10 300 python -u scripts/ab_heads.py bf16x3 3 10 p32,pv32 > $OUT/ab_s3.log 2>&1 || { tail -20 $OUT/ab_s3.log; exit 1; }
tail -4 $OUT/ab_s3.log
timeout -k 10 300 python -u scripts/ab_heads.py bf16 3 10 p32,pv32 > $OUT/ab_bf16.log 2>&1 || { tail -20 $OUT/ab_bf16.log; exit 1; }
tail -4 $OUT/ab_bf16.log
timeout -k 10 200 python -u scripts/head_timeline.py bf16x3 --vhead > $OUT/tl_s3.json 2>&1 || { tail -20 $OUT/tl_s3.json; exit 1; }
timeout -k 10 200 python -u scripts/head_timeline.py bf16 --vhead > $OUT/tl_bf16.json 2>&1 || { tail -20 $OUT/tl_bf16.json; exit 1; }
cat $OUT/tl_s3.json | tail -30
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_pv32 -o run --output-format csv -- python3 scripts/ab_heads.py bf16x3 1 5 pv32 > $OUT/stats_pv32.log 2>&1 || { tail -20 $OUT/stats_pv32.log; exit 1; }
echo OK
