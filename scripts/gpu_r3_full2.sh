# full GPU suite, then same-box A/B of the working tree vs variant b (bf16x3, bf16) and the gather probe
set -u
OUT=gpurun_out/full2; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for dt in bf16x3 bf16; do
  timeout -k 10 400 python3 scripts/ab_iter.py $dt A,B 4 10 > $OUT/ab_$dt.json 2> $OUT/ab_$dt.err || { tail -5 $OUT/ab_$dt.err; exit 1; }
  tail -1 $OUT/ab_$dt.json
done
timeout -k 10 200 python3 scripts/probe_gather.py bf16x3 2>&1 | tail -1
