# kernel-trace stats of a short bench run (OUT=dir; extra env passes through)
set -u
OUT=${OUT:-gpurun_out/pq}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
python scripts/kernel_stats_md.py $(find $OUT -name run_kernel_stats.csv | head -1) quick > $OUT/stats.md && head -16 $OUT/stats.md
