#!/usr/bin/env python3
"""The transposed-chain 32x32 value head (csrc/vhead.hip) against the 16x16 head kernel
(csrc/mlp_head.hip FWD) and the fp32 torch model: values() at the bench geometry (Humanoid dims,
4096 envs x 16 steps + the bootstrap rows), max error and time per call of each path.

    python scripts/probe_vhead.py [dtype ...]     (default: bf16x3 bf16)
"""
import json
import os
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
    dtypes = sys.argv[1:] or ["bf16x3", "bf16"]
    E, T = 4096, 16
    for dt in dtypes:
        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T,
                        batch_size=E * T, dtype=dt)
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
        with torch.no_grad():
            _, _, v = model(eng.decode(eng.x_buf)[:, :O])
        v = v.reshape(-1)
        scale = v.abs().max().item()
        res = {"dtype": dt}
        outs = {}
        for name, on in (("vhead32", 1), ("head16", 0)):
            eng.ext.set_vhead(on)
            eng.values_buf.fill_(float("nan"))
            eng.values()
            torch.cuda.synchronize()
            outs[name] = eng.values_buf.clone()
            res[f"{name}_max_rel_err"] = (outs[name] - v).abs().max().item() / scale
            res[f"{name}_finite"] = bool(torch.isfinite(outs[name]).all())
            for _ in range(3):
                eng.values()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(20):
                eng.values()
            t1.record()
            torch.cuda.synchronize()
            res[f"{name}_us"] = t0.elapsed_time(t1) / 20 * 1e3
        eng.ext.set_vhead(1)
        res["vhead32_vs_head16_max_rel"] = (outs["vhead32"] - outs["head16"]).abs().max().item() / scale
        bad = (outs["vhead32"] - v).abs() > 1e-3 * scale
        res["vhead32_bad_rows"] = int(bad.sum())
        if bad.any():
            idx = torch.nonzero(bad).flatten()[:8].tolist()
            res["first_bad"] = [(i, outs["vhead32"][i].item(), v[i].item()) for i in idx]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
