#!/bin/bash
# The one GPU job script (replaces the per-experiment gpu_*.sh wrappers of rounds 1-3).
#
#   STEPS="tests smoke bench" bash scripts/gpu_round.sh            # default
#   STEPS="bench stats pmc" DTYPES="bf16x3 fp8" bash scripts/gpu_round.sh
#
# Steps (run in the order given; every GPU step has its own time limit and the script stops at
# the first failing one — a failed step may be a GPU fault, so nothing else runs on the GPU after):
#   tests      pytest -m gpu (TESTS_K: a -k filter)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py --steps $BSTEPS --warmup 3 (BENCH_ARGS: extra flags)
#   ab         bench.py arms alternated $AB_REPS times: AB_ARMS="name=flags;name=flags"
#   stats      rocprofv3 --kernel-trace --stats of bench.py per dtype in $DTYPES -> $OUT/s_<dtype>
#   pmc        PMC passes of the hot kernels (scripts/pmc.sh; REGEX, BENCH_ARGS)
#   multirank  bench.py as 2 ranks on the one GPU (gloo: the in-stream production branch)
#   e2e        the BASELINE configs through train.py + 300-iteration learning curves
set -u
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
BSTEPS=${BSTEPS:-20}
DTYPES=${DTYPES:-"bf16x3 bf16 fp8"}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 3 "$OUT/$name.log" | cut -c1-400
  return $rc
}
prof_env() { cd /tmp && export TMPDIR=/tmp && cd - >/dev/null; }
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests) run pytest_gpu 1500 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 240 \
             --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 600 python bench.py --steps "$BSTEPS" --warmup 3 ${BENCH_ARGS:-} || exit $? ;;
    ab)    IFS=';' read -ra ARMS <<< "${AB_ARMS:?AB_ARMS=name=flags;...}"
           for i in $(seq 1 "${AB_REPS:-2}"); do
             for arm in "${ARMS[@]}"; do
               n=${arm%%=*}; f=${arm#*=}
               run "ab_${n}_$i" 300 python bench.py --steps "$BSTEPS" --warmup 3 --variants "" $f || exit $?
             done
           done ;;
    stats) prof_env
           for dt in $DTYPES; do
             run "s_$dt" 300 rocprofv3 --kernel-trace --stats -d "$OUT/s_$dt" -o run --output-format csv -- \
                 python3 bench.py --steps 5 --warmup 2 --variants "" --dtype "$dt" ${BENCH_ARGS:-} || exit $?
           done ;;
    pmc)   OUT=$OUT run pmc 1200 bash scripts/pmc.sh || exit $? ;;
    multirank)
           run multirank 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
               --master-port 29677 bench.py --gpus 2 --steps 5 --warmup 2 --verify-sync --dist-backend gloo \
               ${BENCH_ARGS:-} || exit $? ;;
    e2e)   run cfg2_halfcheetah_bf16 300 python train.py --preset dppo --device gpu --env-name HalfCheetah-v2 \
               --num-envs 1024 --exploration-size 16384 --batch-size 16384 --dtype bf16 --max-iters 60 \
               --num-processes 1 --log-jsonl "$OUT/cfg2.jsonl" || exit $?
           run cfg3_walker_4ranks 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
               --master-addr 127.0.0.1 --master-port 29678 train.py --preset dppo --device gpu --env-name Walker2d-v2 \
               --num-envs 256 --exploration-size 4096 --batch-size 4096 --dtype bf16x3 --max-iters 10 \
               --dist-backend gloo --verify-sync-every 5 --log-jsonl "$OUT/cfg3.jsonl" || exit $?
           for dt in $DTYPES; do
             run "humanoid_${dt}_300" 400 python train.py --preset dppo --device gpu --env-name Humanoid-v2 \
                 --num-envs 4096 --exploration-size 65536 --batch-size 65536 --dtype "$dt" --max-iters 300 \
                 --num-processes 1 --seed 5 --log-jsonl "$OUT/humanoid_${dt}.jsonl" || exit $?
           done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
