set -u
OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_update_reads_rows_past_2gib_of_the_observation_buffer" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
OUT=$OUT/pq bash scripts/gpu_prof_quick.sh
