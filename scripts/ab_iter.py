"""Whole-iteration A/B of runtime knobs on the bench configuration (diagnostics).

Arms run interleaved in ONE process on ONE worker (same box, same clocks): each round runs K
deferred iterations per arm (the bench's production loop) and reports ms per iteration.

    python scripts/ab_iter.py bf16x3 A,b,c [rounds] [iters]

Arm names: "A" = the default build; a name of the table below = a runtime knob; any other name =
the variant module _dppo_hip_<name> (ops/_build.py --variant <name> --define ...).  The engine
state (parameters, Adam moments and step) is restored before every timed block, so an ablation
variant (wrong numerics by design) cannot leave the next arm different weights.
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
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    want = sys.argv[2].split(",") if len(sys.argv) > 2 else ["x_cached", "x_stream"]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = init_single_rank_collective(dev, port=free_port())
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536, batch_size=65536,
                    dtype=dtype, seed=1, phase_timing=0)
    w = DPPOWorker(p, ctx)
    ext = w.engine.ext
    from pytorch_dppo_amd.ops import native
    variants = {}

    def use_ext(name):
        # "A": the default build; any other name: the variant module _dppo_hip_<name> (same
        # bindings, another kernel source tree: ops/_build.py --variant)
        if name == "A":
            w.engine.ext = ext
        else:
            if name not in variants:
                variants[name] = native.load_variant(name)
            w.engine.ext = variants[name]

    arms = {
        "A": lambda: use_ext("A"), "B": lambda: use_ext("b"), "C": lambda: use_ext("c"),
        "x_cached": lambda: ext.set_x_stream(0), "x_stream": lambda: ext.set_x_stream(1),
        "s3w8": lambda: ext.set_s3_train_waves(8), "s3w4": lambda: ext.set_s3_train_waves(4),
        "pv": lambda: setattr(w.engine, "head_order", (0, 1)), "vp": lambda: setattr(w.engine, "head_order", (1, 0)),
    }
    for _ in range(2):
        w.iteration_step()
    eng = w.engine
    snap = (w.model.flat.data.clone(), eng.adam_m.clone(), eng.adam_v.clone(), eng.adam_step,
            w.stats.mean.clone(), w.stats.mean_diff.clone(), w.stats.n)

    def restore():
        w.model.flat.data.copy_(snap[0])
        eng.adam_m.copy_(snap[1])
        eng.adam_v.copy_(snap[2])
        eng.adam_step = snap[3]
        w.stats.mean.copy_(snap[4])
        w.stats.mean_diff.copy_(snap[5])
        w.stats.n = snap[6]
        w.stats._refresh()
        eng.params_changed()
    res = {k: [] for k in want}
    for _ in range(rounds):
        for k in want:
            (arms[k] if k in arms else (lambda k=k: use_ext(k)))()
            restore()
            w.iteration_step()                     # settle on the arm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                w.iteration_step(defer=True)
            torch.cuda.synchronize()
            w.finish_metrics()
            res[k].append((time.perf_counter() - t0) / iters * 1e3)
    out = {k: {"median_ms": sorted(v)[len(v) // 2], "all_ms": [round(x, 3) for x in v]} for k, v in res.items()}
    print(json.dumps({"dtype": dtype, "arms": out}))
    ctx.destroy()


if __name__ == "__main__":
    main()
