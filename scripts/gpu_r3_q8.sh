#!/bin/bash
# fp8 mode's e4m3 wgrad operands: GPU tests, bench (headline + variants), kernel stats of fp8
set -u
OUT=gpurun_out/q8
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  -s ${TESTK:+-k "$TESTK"} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
grep -E "rel diff|per-layer|learning curves" $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --dtype fp8 --variants bf16 > $OUT/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/rocprof.log; exit 1; }
echo done
