"""In-process A/B timing of kernel variants on the bench configuration (diagnostics).

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24):
  adam:  fused no-clip Adam (1 launch) vs sumsq + Adam (2 launches)
  wgrad: LDS-DMA staged vs register-streamed (inside eng.grad)
  rows:  64-row / 8-wave vs 32-row / 4-wave tiles of the fused update and value kernels
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


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536, batch_size=65536,
                    dtype=dtype, use_graphs=False)
    spec = get_spec(p.env_name)
    torch.manual_seed(0)
    model = ActorCritic(spec.obs_dim, spec.act_dim).to(dev)
    env = make_vec_env(spec, p.num_envs, device=dev)
    stats = RunningObsStats(spec.obs_dim, dev)
    eng = HipEngine(p, model, env, stats, dev, 0)
    stats.observes(env.observe())
    eng.rollout()
    eng.values()
    eng.gae()
    eng.begin_update()
    ext = eng.ext
    eng.grad(None)

    def rows(n):
        ext.set_mlp_rows(n)
        eng.sync_tile()

    waves0 = eng.wgrad_waves

    def plan(waves=None, aligned=False):
        eng.wgrad_waves = waves or waves0
        eng.wgrad_aligned = aligned
        eng._build_wgrad_plan(model)

    def knobs(adam=1, wgrad=0, r=0):   # every arm sets every knob (no state leaks between arms)
        return lambda: (ext.set_adam_fused(adam), ext.set_wgrad_impl(wgrad), rows(r), ext.set_wgrad_stages(4),
                        plan(8 if wgrad == 1 else None))

    arms = {
        "adam_fused": (knobs(adam=1), eng.apply),
        "adam_sumsq_pair": (knobs(adam=0), eng.apply),
        "grad_wgrad_lds_dma": (knobs(wgrad=0), lambda: eng.grad(None)),
        "grad_wgrad_register": (knobs(wgrad=1), lambda: eng.grad(None)),
        "rollout_8waves": (lambda: (knobs()(), ext.set_rollout_waves(8)), eng.rollout),
        "rollout_4waves": (lambda: (knobs()(), ext.set_rollout_waves(4)), eng.rollout),
        "values_rows64": (knobs(r=64), eng.values),
        "values_rows32": (knobs(r=32), eng.values),
        "grad_rows64": (knobs(r=64), lambda: eng.grad(None)),
        "grad_rows32": (knobs(r=32), lambda: eng.grad(None)),
    }
    for t in (1024, 512, 256, 100):
        arms[f"grad_wgrad_wgs{t}"] = ((lambda t=t: (knobs()(), eng._build_wgrad_plan(model, t))),
                                      lambda: eng.grad(None))
    arms["grad_wgrad_prop"] = (lambda: (knobs()(), plan()), lambda: eng.grad(None))
    arms["grad_wgrad_aligned"] = (lambda: (knobs()(), plan(aligned=True)), lambda: eng.grad(None))
    arms["grad_wgrad_w8"] = (lambda: (knobs()(), plan(8)), lambda: eng.grad(None))
    arms["grad_wgrad_w16"] = (lambda: (knobs()(), plan(16)), lambda: eng.grad(None))
    # wgrad DMA ring depth x batch chunks (tasks = chunks x tiles per chunk)
    for st in (3, 4, 6):   # ring depth of the 8-wave kernel
        for ch in (16, 24, 32, 40):
            arms[f"grad_wgrad_s{st}_c{ch}"] = (
                (lambda st=st, ch=ch: (knobs()(), ext.set_wgrad_stages(st), setattr(eng, "wgrad_waves", 8),
                                       eng._build_wgrad_plan(model, chunks_override=ch))),
                lambda: eng.grad(None))
    if os.environ.get("AB_ARMS"):   # regex filter on arm names
        import re
        arms = {k: v for k, v in arms.items() if re.search(os.environ["AB_ARMS"], k)}
    res = {k: [] for k in arms}
    for _ in range(5):
        for k, (setup, fn) in arms.items():
            setup()
            res[k].append(timed(fn))
    ext.set_adam_fused(1)
    ext.set_wgrad_impl(0)
    rows(0)
    ext.set_rollout_waves(8)
    ext.set_wgrad_stages(4)
    plan()
    print(json.dumps({k: {"median_us": sorted(v)[len(v) // 2], "min_us": min(v)} for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
