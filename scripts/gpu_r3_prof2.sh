# kernel stats of the headline and the bf16 variant + per-head phase timelines
set -u
OUT=gpurun_out/prof2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for dt in bf16x3 bf16 fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s_$dt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --variants "" --dtype $dt > $OUT/s_$dt.log 2>&1 || { tail -20 $OUT/s_$dt.log; exit 1; }
  python scripts/kernel_stats_md.py $(find $OUT/s_$dt -name run_kernel_stats.csv | head -1) "$dt, bench geometry, 5 steps" > $OUT/stats_$dt.md && sed -n 5,16p $OUT/stats_$dt.md
done
for dt in bf16x3 bf16; do
  timeout -k 10 200 python3 scripts/head_timeline.py $dt > $OUT/timeline_$dt.json 2> $OUT/timeline_$dt.err || { tail -5 $OUT/timeline_$dt.err; exit 1; }
done
