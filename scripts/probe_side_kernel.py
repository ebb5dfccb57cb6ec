#!/usr/bin/env python3
"""Does a collective launched on a side stream get CUs while the update's head kernels hold them?
(the per-epoch value all-reduce would run beside the next epoch's policy kernel.)
RCCL launches no kernel at world size 1, so a stand-in with an all-reduce kernel's footprint runs
instead (csrc/optim.hip probe_spin_kernel: NB workgroups of 256 threads, each spinning US µs once it
has a CU).  Bench geometry (Humanoid dims, 65,536 rows), one engine, CUDA events.

    python scripts/probe_side_kernel.py [dtype] [nblk,...] [us]

Prints, per stand-in size: the head kernel alone, the stand-in alone, and both (the stand-in
forked to a side stream right BEFORE the head kernel — its all-reduce is ready at the end of the
previous epoch's gather — or right AFTER it): the head kernel's time on the main stream and when
the stand-in finished, both from the common start."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.envs import get_spec, make_vec_env  # noqa: E402
from pytorch_dppo_amd.models.actor_critic import ActorCritic  # noqa: E402
from pytorch_dppo_amd.runtime.engine_hip import HipEngine  # noqa: E402
from pytorch_dppo_amd.utils.obs_stats import RunningObsStats  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [8, 16, 32, 64]
    us = float(sys.argv[3]) if len(sys.argv) > 3 else 25.0
    torch.cuda.set_device(DEV)
    E, T = 4096, 16
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T, batch_size=E * T,
                    dtype=dt, update_kernels="heads")
    spec = get_spec(p.env_name)
    torch.manual_seed(0)
    model = ActorCritic(spec.obs_dim, spec.act_dim, p.hidden).to(DEV)
    env = make_vec_env(spec, p.num_envs, seed=p.seed, device=DEV)
    eng = HipEngine(p, model, env, RunningObsStats(spec.obs_dim, DEV), DEV, 0)
    eng.begin_update()
    mbt = eng._minibatch(None)
    ext = eng.ext
    sink = torch.zeros(4096, dtype=torch.int32, device=DEV)
    main_s = torch.cuda.current_stream(DEV)
    side = torch.cuda.Stream(device=DEV)

    def head(h):
        eng._head_kernel(h, mbt[0], False, mbt[2], eng.part_joint, eng.part_dw_joint[h])

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def run(h, nb, mode, reps=8):
        """mode: head | spin | before | after -> medians (main us, side-finish us) from the start"""
        out_m, out_s = [], []
        for _ in range(reps + 2):
            torch.cuda.synchronize()
            t0, tm, ts = ev(), ev(), ev()
            t0.record(main_s)
            if mode in ("spin", "before"):
                side.wait_event(t0)
                with torch.cuda.stream(side):
                    ext.probe_spin(nb, 256, 4096, us, sink)
                    ts.record(side)
            if mode != "spin":
                head(h)
            if mode == "after":
                t1 = ev()
                t1.record(main_s)   # (fork right after the head kernel's launch: same start point)
                side.wait_event(t0)
                with torch.cuda.stream(side):
                    ext.probe_spin(nb, 256, 4096, us, sink)
                    ts.record(side)
            tm.record(main_s)
            torch.cuda.synchronize()
            out_m.append(t0.elapsed_time(tm) * 1e3)
            out_s.append(t0.elapsed_time(ts) * 1e3 if mode != "head" else 0.0)
        return round(statistics.median(out_m[2:]), 1), round(statistics.median(out_s[2:]), 1)

    for h, name in ((0, "policy"), (1, "value")):
        base = run(h, 1, "head")[0]
        for nb in sizes:
            res = {"kernel": name, "dtype": dt, "standin_blocks": nb, "standin_us": us, "head_alone_us": base,
                   "standin_alone_us": run(h, nb, "spin")[1]}
            for mode in ("before", "after"):
                m, s_ = run(h, nb, mode)
                res[f"{mode}: head_us"] = m
                res[f"{mode}: standin_done_us"] = s_
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
