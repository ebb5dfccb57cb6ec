# per-step obs-norm mode: its tests, then its cost vs rollout mode at the bench geometry
set -u
OUT=gpurun_out/obsstep; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "obs_observe or step_obs_norm or obs_reduce" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/probe_obs_norm_step.py 10 > $OUT/probe.log 2>&1 || { tail -8 $OUT/probe.log; exit 1; }
tail -4 $OUT/probe.log
