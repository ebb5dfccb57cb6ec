# A/B: per-head kernels (joint world-1 path) vs the one-kernel update, same box
set -u
OUT=gpurun_out/abh; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  -k "head_kernels_match or head_chains or fused_gather_adam" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for h in 1 0 1 0; do
  DPPO_HEADS=$h timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --variants "" > $OUT/bench_h$h.log 2>&1 || { tail -5 $OUT/bench_h$h.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_h$h.log').read().strip().splitlines()[-1]); print('heads=$h', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms')"
done
