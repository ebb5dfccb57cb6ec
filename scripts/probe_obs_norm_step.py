#!/usr/bin/env python3
"""Cost of the per-step obs-norm mode (obs_norm_update='step', the reference's per-observation
filter update, model.py:68) at the bench geometry (Humanoid dims, 4096 envs x 16 steps, bf16x3):
rollout() and a whole iteration in 'rollout' mode (one fused T-step launch) vs 'step' mode as ONE
cooperative launch (round 4: in-kernel granule hand-offs, csrc/rollout.hip sn_step), 'step_launches'
(round 3: T x [obs_observe + one-step rollout] + one reduce), and 'step_torch_observe' (round 2:
the observe by torch ops) for comparison.  Diagnostics.

    python scripts/probe_obs_norm_step.py [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.parallel.dist import DistContext  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    for mode in ("rollout", "step", "step_launches", "step_torch_observe"):
        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536,
                        batch_size=65536, dtype="bf16x3", seed=1,
                        obs_norm_update="rollout" if mode == "rollout" else "step")
        w = DPPOWorker(p, DistContext(device=dev))
        eng = w.engine
        if mode != "step":
            eng._sn_cap = 0          # the per-step launch sequence
        if mode == "step_torch_observe":
            eng._observe_step = lambda norm, obs, shift: norm.observes(obs.to(eng.device, torch.float32))
        w.iteration_step()
        out[mode] = {"rollout_ms": round(timed(eng.rollout, reps), 3),
                     "iteration_ms": round(timed(w.iteration_step, max(2, reps // 3)), 3)}
        print(json.dumps({mode: out[mode]}), flush=True)
        del w, eng
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
