# RCCL paths: tests, then forced-collective (world size 1) vs plain benches alternating on one box
# (native in-stream communicator, and the process-group chains with DPPO_NATIVE_COMM=0), then a
# kernel trace of the forced native run for the overlap report
set -u
OUT=gpurun_out/rccl; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "rccl or two_ranks" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for arm in plain forced pg; do
    f=""; env=""
    [ $arm = forced ] && f="--force-collectives"
    [ $arm = pg ] && f="--force-collectives" && env="DPPO_NATIVE_COMM=0"
    env $env timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --variants "" $f > $OUT/b_${arm}_$i.log 2>&1 || { tail -5 $OUT/b_${arm}_$i.log; exit 1; }
    tail -1 $OUT/b_${arm}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', round(d['ms_per_step'],3), 'ms')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --variants "" --force-collectives > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
python3 scripts/overlap_report.py $(find $OUT/tr -name run_kernel_trace.csv | head -1) > $OUT/overlap.md && head -8 $OUT/overlap.md
