#!/usr/bin/env python3
"""Whole-iteration A/B of the update's head kernels on the bench configuration: the 16x16 head
kernels (csrc/mlp_head.hip) vs the 32x32 transposed-chain policy head (csrc/phead.hip) beside the
16x16 value head, and the wgrad's wide tiles vs one quadrant per wave ("narrow").  One worker per arm in ONE process, interleaved
rounds of K deferred iterations each (the bench's production loop); ms per iteration per round.

    python scripts/ab_heads.py [dtype] [rounds] [iters] [arms: h16,p32,narrow]
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

# arm -> Params overrides: the 16x16 policy head, the default, the wgrad with one quadrant per wave
ARMS = {"h16": {"phead_kernel": False}, "p32": {}, "narrow": {"wgrad_wide": False},
        "p2on": {"phead_fused_dw2": "on"}, "p2off": {"phead_fused_dw2": "off"}}


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    arms = sys.argv[4].split(",") if len(sys.argv) > 4 else list(ARMS)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = init_single_rank_collective(dev, port=free_port())
    workers = {}
    for a in arms:
        # "<arm>:w<N>": the same arm with Params.wgrad_wgs = N (wgrad tasks per launch)
        base, _, wg = a.partition(":w")

        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536,
                        batch_size=65536, dtype=dtype, seed=1, phase_timing=0)
        for k, v in ARMS[base].items():
            setattr(p, k, v)
        if wg:
            p.wgrad_wgs = int(wg)
        w = DPPOWorker(p, ctx)
        assert w.engine.phead == (p.phead_kernel and dtype != "fp8"), a   # (fp8: the 16x16 policy head)
        for _ in range(2):
            w.iteration_step()
        workers[a] = w
    torch.cuda.synchronize()
    res = {a: [] for a in arms}
    for r in range(rounds):
        for a in arms:
            w = workers[a]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                w.iteration_step(defer=True)
            w.finish_metrics()
            torch.cuda.synchronize()
            res[a].append((time.perf_counter() - t0) / iters * 1e3)
        print(json.dumps({"round": r, **{a: round(res[a][-1], 4) for a in arms}}), flush=True)
    print(json.dumps({"dtype": dtype, "ms_per_iter_min": {a: round(min(v), 4) for a, v in res.items()},
                      "ms_per_iter_median": {a: round(sorted(v)[len(v) // 2], 4) for a, v in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
