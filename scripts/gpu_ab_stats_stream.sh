# GPU tests, then an interleaved A/B of the side-stream obs-stats merge (DPPO_STATS_STREAM=1 vs 0)
set -u
OUT=${OUT:-gpurun_out/ss}; mkdir -p $OUT; BARGS=${BARGS:-}
[ "${TESTS:-1}" = 1 ] && { timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }; }
tail -3 $OUT/pytest.log
for r in 1 2 3; do
for f in auto 0; do
DPPO_STATS_STREAM=$f timeout -k 10 300 python bench.py --steps 20 --warmup 3 $BARGS > $OUT/b_${f}_${r}.json 2>$OUT/b.err || exit 1
echo "stream=$f $(grep '^{"metric' $OUT/b_${f}_${r}.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), round(d['ms_per_step'],4))")"
done; done
