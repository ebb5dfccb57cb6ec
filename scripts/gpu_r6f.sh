set -u
OUT=gpurun_out/r6f; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for dt in bf16x3 bf16; do
  timeout -k 10 400 python -u scripts/ab_iter.py $dt A,phrm,ipb8 3 10 > $OUT/ab_iter_$dt.log 2>&1 || { tail -20 $OUT/ab_iter_$dt.log; exit 1; }
  tail -1 $OUT/ab_iter_$dt.log
done
echo OK
