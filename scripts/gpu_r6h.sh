set -u
OUT=gpurun_out/r6h; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for dt in bf16x3 bf16; do
  timeout -k 10 400 python -u scripts/ab_heads.py $dt 3 10 p32,narrow > $OUT/ab_heads_$dt.log 2>&1 || { tail -20 $OUT/ab_heads_$dt.log; exit 1; }
  tail -1 $OUT/ab_heads_$dt.log
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s_bf16x3 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --variants "" > $OUT/stats_bf16x3.log 2>&1 || { tail -20 $OUT/stats_bf16x3.log; exit 1; }
echo OK
