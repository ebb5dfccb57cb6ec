#!/bin/bash
# register-staged wgrad: gradient tests, then same-box A/B against the DMA-ring build (variant b)
# at every update precision
set -u
OUT=gpurun_out/rs; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "grad or wgrad or head or geometry or e4m3 or fp8_update or resume" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for dt in bf16x3 bf16 fp8; do
  timeout -k 10 300 python3 scripts/ab_iter.py $dt A,B 4 10 > $OUT/ab_$dt.json 2> $OUT/ab_$dt.err || { tail -5 $OUT/ab_$dt.err; exit 1; }
  tail -1 $OUT/ab_$dt.json
done
