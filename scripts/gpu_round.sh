#!/bin/bash
# One GPU session: GPU tests -> smoke -> short bench -> kernel profile.  Each GPU step has its
# own time limit; the script stops at the first failing step (a failed test may be a GPU fault:
# nothing else runs on the GPU after it).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  return $rc
}
STEPS=${STEPS:-"tests smoke bench"}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 600 python bench.py --steps ${BSTEPS:-5} --warmup 2 --verbose || exit $? ;;
    prof)  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
           run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 || exit $? ;;
  esac
done
exit 0
