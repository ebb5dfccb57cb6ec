#!/usr/bin/env python3
"""Per-step phase split of the one-launch per-step observation filter (obs_norm_update='step',
csrc/rollout.hip SN path) at the bench geometry: s_memtime cycles per step (median over workgroups of
the max over waves) for the filter's moments / reduce (first hand-off) / gather (second hand-off) /
barrier, and the rest of the step; plus the rollout time without stamps, and the cross-workgroup
spread of step 8's hand-offs (absolute 100 MHz stamps: min / median / max over workgroups).

    python scripts/probe_filter_phases.py [reps] [step|rollout]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.parallel.dist import init_single_rank_collective  # noqa: E402
from pytorch_dppo_amd.runtime.launcher import free_port  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402

NAMES = ["observe", "fc1", "fc2", "fc3", "sample", "logp/reward", "env", "sn moments", "sn reduce (hand-off 1)",
         "sn gather (hand-off 2)", "sn barrier"]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    mode = sys.argv[2] if len(sys.argv) > 2 else "step"   # obs_norm_update: step | rollout
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = init_single_rank_collective(dev, port=free_port())
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536, batch_size=65536,
                    dtype="bf16x3", seed=1, obs_norm_update=mode)
    w = DPPOWorker(p, ctx)
    eng = w.engine
    for _ in range(2):
        w.iteration_step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        eng.rollout()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    nblk = (eng.E + 15) // 16
    buf = torch.zeros(nblk * 8 * 16, dtype=torch.int64, device=dev)
    eng.ext.set_rollout_tstamp(buf)
    eng.rollout()
    torch.cuda.synchronize()
    eng.ext.set_rollout_tstamp(torch.empty(0, dtype=torch.int64, device=dev))
    t = buf.view(nblk, 8, 16)[:, :, :11].double() / eng.T
    per = {n: float(t[:, :, i].max(dim=1).values.median()) for i, n in enumerate(NAMES)}
    if mode != "step":
        print(json.dumps({"rollout_ms": round(ms, 4), "cycles_per_step(median blk, max wave)": per}, indent=1),
              flush=True)
        return
    # step 8's absolute 100 MHz stamps (slots 11-14): per workgroup the latest wave; relative to
    # the earliest filter entry, in microseconds
    ab = buf.view(nblk, 8, 16)[:, :, 11:15].double()
    t0 = ab[:, :, 0][ab[:, :, 0] > 0].min()
    us = (ab - t0) / 100.0
    wg = us.amax(dim=1)                    # [nblk, 4]: entry, moments published, reduce done, gather done
    nred = min(nblk, (eng.O + 3) // 4)     # workgroups whose wave 0 reduces a 4-feature unit
    red = us[:nred, 0, 2]
    q = lambda v: [round(float(v.min()), 2), round(float(v.median()), 2), round(float(v.max()), 2)]
    skew = {"entry": q(wg[:, 0]), "moments published": q(wg[:, 1]), "reducers done (wave 0)": q(red),
            "gather done": q(wg[:, 3])}
    npl = buf.view(nblk, 8, 16)[:, :, 15]
    skew["reduce polls (reducers, wave 0)"] = q((npl[:nred, 0] & 0xFFFFFFFF).double())
    skew["gather polls (wave 7)"] = q((npl[:, 7] >> 32).double())
    print(json.dumps({"rollout_ms": round(ms, 4), "cycles_per_step(median blk, max wave)": per,
                      "sum": sum(per.values()), "step8_us_min_median_max": skew}, indent=1), flush=True)


if __name__ == "__main__":
    main()
