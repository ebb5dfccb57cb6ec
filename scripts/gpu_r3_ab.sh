# same-box A/B of the working tree (A) against the variant build B (ops/_build.py --variant b),
# then the per-head phase timeline and the gather probe
set -u
OUT=gpurun_out/ab2; mkdir -p $OUT
timeout -k 10 400 python3 scripts/ab_iter.py ${DT:-bf16x3} A,B 4 10 > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
tail -1 $OUT/ab.json
timeout -k 10 200 python3 scripts/head_timeline.py ${DT:-bf16x3} > $OUT/timeline.json 2> $OUT/timeline.err || { tail -5 $OUT/timeline.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/timeline.json')); print({k:(v['total_cycles_median'], v['phases_median_cycles(max over waves)']) for k,v in d.items()})"
timeout -k 10 200 python3 scripts/probe_gather.py ${DT:-bf16x3} 2>&1 | tail -1
