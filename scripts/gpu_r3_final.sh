#!/bin/bash
# end-of-round evidence on one box: full GPU suite, smoke, 10-step bench, kernel stats of the
# three precisions, PMC passes of the fp8 kernels.  Stops at the first failing GPU step.
set -u
OUT=gpurun_out/final; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread -s \
  > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for dt in bf16x3 bf16 fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s_$dt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --variants "" --dtype $dt > $OUT/s_$dt.log 2>&1 || { echo "rocprof $dt failed"; tail -20 $OUT/s_$dt.log; exit 1; }
done
OUT=$OUT REGEX='mlp_head|wgrad_kernel|gather_adam' BENCH_ARGS="--dtype fp8" bash scripts/pmc.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
echo done
