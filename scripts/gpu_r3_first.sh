# round-3 first GPU pass: new tests, baseline bench, kernel stats
set -u
OUT=gpurun_out/r3a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_bench_contract.py tests/test_gym_backend.py \
  "tests/test_gpu_kernels.py::test_gae_kernel_matches_oracle" \
  "tests/test_gpu_kernels.py::test_update_reads_rows_past_2gib_of_the_observation_buffer" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
OUT=$OUT/pq bash scripts/gpu_prof_quick.sh
