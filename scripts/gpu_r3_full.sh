# round-3 full GPU check: every gpu test, smoke(), the headline bench (3 runs, with variants)
set -u
OUT=gpurun_out/full; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { tail -5 $OUT/bench_$i.log; exit 1; }
  tail -1 $OUT/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms', {k:round(v['ms_per_step'],3) for k,v in d['variants'].items()})"
done
