#!/bin/bash
# same-box whole-iteration A/B/C of the working tree (A) against variant builds b and c
# (ops/_build.py --variant b|c), at ${DT:-bf16x3}
set -u
OUT=gpurun_out/abc; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python3 scripts/ab_iter.py ${DT:-bf16x3} ${ARMS:-A,B,C} ${ROUNDS:-4} 10 > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
tail -1 $OUT/ab.json
