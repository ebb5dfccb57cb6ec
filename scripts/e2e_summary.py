#!/usr/bin/env python3
"""Learning-curve table of the train.py JSONL logs the `e2e` step of scripts/gpu_round.sh writes
(docs/ARCHITECTURE.md: "learning at scale"): mean episode return averaged over 25-iteration windows,
the last-25 mean, and the median env steps/s of each run.

    python scripts/e2e_summary.py gpurun_out/e2e/humanoid_fp32.jsonl gpurun_out/e2e/humanoid_bf16x3.jsonl ...
"""
import json
import os
import statistics
import sys


def load(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip().startswith("{")]


def main():
    runs = [(os.path.basename(p).rsplit(".", 1)[0].split("_", 1)[-1], load(p)) for p in sys.argv[1:]]
    n = min(len(r) for _, r in runs)
    wins = [(a, min(a + 25, n)) for a in range(0, n, 50) if a + 25 <= n]
    print("| dtype | " + " | ".join(f"it {a + 1}-{b}" for a, b in wins) + " | last 25 | env steps/s |")
    print("|---" * (len(wins) + 3) + "|")
    for name, r in runs:
        ret = [x["mean_ep_return"] for x in r[:n]]
        cells = [f"{statistics.fmean(ret[a:b]):.1f}" for a, b in wins]
        sps = statistics.median(x["steps_per_s"] for x in r[:n])
        print(f"| {name} | " + " | ".join(cells) + f" | {statistics.fmean(ret[-25:]):.1f} | {sps:.3g} |")


if __name__ == "__main__":
    main()
