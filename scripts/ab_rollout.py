#!/usr/bin/env python3
"""Same-box A/B of the rollout kernel: the current extension vs a variant build of another
source tree (ops/_build.py --variant NAME --src DIR), interleaved in one process at the bench
geometry (Humanoid dims, 4096 envs x 16 steps).  Diagnostics.

    python scripts/ab_rollout.py VARIANT [dtype] [reps]

Before timing, one rollout from the same env state through each build: every buffer it writes
(observation rows, x^T operand, actions, log-probs, rewards, dones, moments, episode stats, env
state) must be bitwise identical ("bitwise_equal" in the output) for a layout-only change.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.ops import native  # noqa: E402
from pytorch_dppo_amd.parallel.dist import DistContext  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402


def main():
    var = sys.argv[1]
    dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536,
                    batch_size=65536, num_epoch=1, dtype=dtype, seed=1)
    w = DPPOWorker(p, DistContext(device=dev))
    w.iteration_step()
    eng = w.engine
    exts = {"cur": eng.ext, var: native.load_variant(var)}
    sd = eng.env.state_dict()
    outs = {}
    for k, e in exts.items():
        eng.ext = e
        eng.env.load_state_dict(sd)
        eng.rollout()
        torch.cuda.synchronize()
        outs[k] = [t.clone() for t in (eng.x_buf, eng.xT, eng.actions, eng.logp, eng.rewards, eng.dones, eng.mom,
                                       eng.epstat, eng.env.state, eng.env.ep_len, eng.env.ep_ret)]
    same = all(torch.equal(a, b) for a, b in zip(outs["cur"], outs[var]))
    res = {k: [] for k in exts}
    for _ in range(3):
        for k, e in exts.items():
            eng.ext = e
            eng.rollout()
            torch.cuda.synchronize()
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                eng.rollout()
            t.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(t) / reps * 1e3)
    eng.ext = exts["cur"]
    print(json.dumps({"dtype": dtype, "bitwise_equal": same, **{k: min(v) for k, v in res.items()}, "all": res}))


if __name__ == "__main__":
    main()
