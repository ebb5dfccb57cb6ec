# per-head kernels: numerics tests, then bench + kernel stats
set -u
OUT=gpurun_out/r3h; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  -k "head_kernels_match or head_chains or fused_loss_backward_matches or past_2gib or fused_gather_adam" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
OUT=$OUT/pq bash scripts/gpu_prof_quick.sh
