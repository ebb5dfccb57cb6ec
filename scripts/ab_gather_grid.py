#!/usr/bin/env python3
"""Same-box A/B of the fused gather + Adam launch's grid: the engine's sizing (one slab element per
thread) vs an override (e.g. the round-4 formula, A + 8 reduce blocks + one per 256 parameters),
interleaved rounds of K deferred iterations in one process.  Diagnostics.

    python scripts/ab_gather_grid.py OVERRIDE_BLOCKS [rounds] [iters]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.parallel.dist import init_single_rank_collective  # noqa: E402
from pytorch_dppo_amd.runtime.launcher import free_port  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402


def main():
    override = int(sys.argv[1])
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = init_single_rank_collective(dev, port=free_port())
    ws = {}
    for arm in ("engine", "override"):
        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536,
                        batch_size=65536, dtype="bf16x3", seed=1, phase_timing=0)
        w = DPPOWorker(p, ctx)
        if arm == "override":
            assert override <= w.engine.norm_part.numel()
            w.engine.norm_n_whole = override
        for _ in range(2):
            w.iteration_step()
        ws[arm] = w
    print(json.dumps({"grid": {a: w.engine.norm_n_whole for a, w in ws.items()}}), flush=True)
    res = {a: [] for a in ws}
    for r in range(rounds):
        for a, w in ws.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                w.iteration_step(defer=True)
            w.finish_metrics()
            torch.cuda.synchronize()
            res[a].append((time.perf_counter() - t0) / iters * 1e3)
        print(json.dumps({"round": r, **{a: round(v[-1], 4) for a, v in res.items()}}), flush=True)
    print(json.dumps({"ms_per_iter_min": {a: round(min(v), 4) for a, v in res.items()},
                      "ms_per_iter_median": {a: round(sorted(v)[len(v) // 2], 4) for a, v in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
