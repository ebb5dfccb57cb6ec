#!/usr/bin/env python3
"""Does the next rollout's COMPUTE overlap the last epoch's update on one MI355X?

VERDICT r1 #5 asked for rollout i+1 (1-update policy lag) on a side stream, concurrent with the
final epoch's fused update + wgrad + Adam.  This measures the ceiling of that schedule before
any engine refactor (the rollout would need a second [T, E] buffer set, since the last epoch
still reads the current one): two independent workers at the bench geometry (Humanoid dims,
E = 4096, T = 16), worker B's rollout and worker A's full-batch epoch (mlp_train -> wgrad ->
gather + Adam), timed
  alone:       each on its own
  serial:      rollout then epoch, one stream
  concurrent:  rollout on a side stream, epoch on the main stream, joined
If `concurrent` is not clearly below `serial`, the hardware cannot co-schedule them (each kernel
fills a CU's LDS or VGPR file, so their workgroups never co-reside and the two streams only
time-slice the CUs) and the refactor buys nothing.

    python scripts/ab_overlap.py [--dtype bf16x3] [--reps 20] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.parallel.dist import DistContext  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16x3")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    E, T = args.num_envs, 16
    ws = []
    for seed in (1, 2):
        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T,
                        batch_size=E * T, num_epoch=2, dtype=args.dtype, seed=seed)
        w = DPPOWorker(p, DistContext(device=dev))
        w.iteration_step()                      # warm: code objects, LDS attributes, buffers
        ws.append(w)
    A, B = ws
    assert A.engine.can_fuse_apply()
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)

    def epoch():
        A.engine.grad(None, apply=True)

    def rollout():
        B.engine.rollout()

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps * 1e6

    def serial():
        rollout()
        epoch()

    def concurrent():
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            rollout()
        epoch()
        main_s.wait_stream(side)

    res = {}
    for rnd in range(2):                        # interleaved arms, two rounds
        for name, fn in (("rollout", rollout), ("epoch", epoch), ("serial", serial), ("concurrent", concurrent)):
            res.setdefault(name, []).append(timed(fn))
    out = {k: min(v) for k, v in res.items()}
    out["sum_alone"] = out["rollout"] + out["epoch"]
    out["saved_us"] = out["serial"] - out["concurrent"]
    out["dtype"] = args.dtype
    out["all"] = res
    print(json.dumps(out))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
