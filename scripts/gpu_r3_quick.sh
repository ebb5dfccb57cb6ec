# quick GPU check: selected tests (K=pytest -k expr) then a 20-step bench (BENCH_ARGS extra)
set -u
OUT=gpurun_out/quick; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "${K}" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --variants "" ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms')"
