# per-kernel time vs update row count (MALL residency of the wgrad operands) + HBM bytes PMC
set -u
OUT=gpurun_out/mall; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for bs in 0 32768 16384; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s$bs -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --variants "" --batch-size $bs > $OUT/s$bs.log 2>&1 || { tail -20 $OUT/s$bs.log; exit 1; }
  python scripts/kernel_stats_md.py $(find $OUT/s$bs -name run_kernel_stats.csv | head -1) "batch $bs" > $OUT/stats_$bs.md && head -14 $OUT/stats_$bs.md
done
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "mlp_head|wgrad|gather" -d $OUT/p$P -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --variants "" > $OUT/p$P.log 2>&1 || { tail -5 $OUT/p$P.log; exit 1; }
done
ls -R $OUT | head -50
