# fp8 F8 value head: kernel stats bf16 vs fp8, the fp8 error printout, head-stream A/B
set -u
OUT=gpurun_out/f8; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "fp8_update_per_layer" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
grep "fp8 value forward" $OUT/pytest.log
for dt in bf16 fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s_$dt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --variants "" --dtype $dt > $OUT/s_$dt.log 2>&1 || { tail -20 $OUT/s_$dt.log; exit 1; }
  python scripts/kernel_stats_md.py $(find $OUT/s_$dt -name run_kernel_stats.csv | head -1) "$dt" > $OUT/stats_$dt.md && sed -n 7,14p $OUT/stats_$dt.md
done
timeout -k 10 400 python3 scripts/ab_iter.py bf16x3 hs0,hs1 4 10 > $OUT/ab_hs.json 2> $OUT/ab_hs.err || { tail -5 $OUT/ab_hs.err; exit 1; }
tail -1 $OUT/ab_hs.json
