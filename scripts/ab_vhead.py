#!/usr/bin/env python3
"""Value-head kernel A/B (diagnostics): the update kernel alone (one full-batch 65,536-row call of
the value head, csrc/vhead.hip or the 16x16 csrc/mlp_head.hip) and V(x) (values(), 69,632 rows), per
extension build, interleaved in ONE process on one box.

    python scripts/ab_vhead.py dtype arm[,arm...] [rounds]

arm: "A" = the default build with the 32x32 value head, "h16" = the default build with the 16x16
value head, any other name = the variant module _dppo_hip_<name> (ops/_build.py --variant <name>
--define ...) with the 32x32 value head.  Prints µs per call (median over rounds)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.envs import get_spec, make_vec_env  # noqa: E402
from pytorch_dppo_amd.models.actor_critic import ActorCritic  # noqa: E402
from pytorch_dppo_amd.ops import native  # noqa: E402
from pytorch_dppo_amd.runtime.engine_hip import HipEngine  # noqa: E402
from pytorch_dppo_amd.utils.obs_stats import RunningObsStats  # noqa: E402

DEV = torch.device("cuda", 0)


def engine(dt, vhead):
    E, T = 4096, 16
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T, batch_size=E * T,
                    dtype=dt, update_kernels="heads")
    p.vhead_kernel = vhead
    spec = get_spec(p.env_name)
    torch.manual_seed(0)
    model = ActorCritic(spec.obs_dim, spec.act_dim, p.hidden).to(DEV)
    env = make_vec_env(spec, p.num_envs, seed=p.seed, device=DEV)
    eng = HipEngine(p, model, env, RunningObsStats(spec.obs_dim, DEV), DEV, 0)
    O, M = model.num_inputs, (T + 1) * E
    xb = torch.zeros(M, eng.d0, device=DEV)
    xb[:, :O] = torch.randn(M, O, device=DEV).clamp(-5, 5)
    xb[:, O] = 1.0
    eng.x_buf.copy_(eng.encode(xb))
    eng.adv.normal_()
    eng.ret.normal_()
    eng.begin_update()
    assert eng.vhead == vhead
    return eng


def timed(fn, n=20):
    for _ in range(3):
        fn()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(n):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / n * 1e3


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    arms = sys.argv[2].split(",") if len(sys.argv) > 2 else ["A", "h16"]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    torch.cuda.set_device(DEV)
    engs = {True: engine(dt, True), False: engine(dt, False)}
    base = engs[True].ext
    res = {a: {"update_us": [], "vx_us": []} for a in arms}
    for _ in range(rounds):
        for a in arms:
            eng = engs[a != "h16"]
            eng.ext = base if a in ("A", "h16") else native.load_variant(a)
            eng.ext.set_vhead(0 if a == "h16" else 1)
            mbt = eng._minibatch(None)

            def upd():
                eng._head_kernel(1, mbt[0], False, mbt[2], eng.part_h[1], eng.part_dw[1])
            res[a]["update_us"].append(timed(upd))
            res[a]["vx_us"].append(timed(eng.values))
            eng.ext.set_vhead(1)
            eng.ext = base
    out = {"dtype": dt, **{a: {k: round(statistics.median(v), 1) for k, v in r.items()} for a, r in res.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
