#!/usr/bin/env python3
"""Where do the ~20 us of gather_adam go?  (diagnostics, bench geometry, one process)

Arms, interleaved, each timed over `reps` back-to-back launches with HIP events:
  fused        gather_adam as the bench runs it (slab gather + Adam + both weight images)
  no_images    the same launch with every w_map entry -1 (no weight-image stores)
  gather       grad_gather alone (slab gather + partials, writes grad_flat)
  adam         the no-clip Adam alone (reads grad_flat; images written)
  adam_noimg   the no-clip Adam alone without image stores

    python scripts/ab_gather.py [dtype] [reps] [variant]

With a variant name (an extension built from another source tree, ops/_build.py --variant) the
fused and gather arms are also timed through that build, interleaved: a same-box A/B.
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
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536,
                    batch_size=65536, num_epoch=2, dtype=dtype, seed=1)
    w = DPPOWorker(p, DistContext(device=dev))
    w.iteration_step()
    eng = w.engine
    ext = eng.ext
    b = eng.buckets[0]
    b1, b2 = p.adam_betas
    neg = torch.full_like(eng.w_map, -1)

    def fused(wm):
        def f():
            ext.gather_adam(b["slab"], eng.src_off, eng.src_meta, eng.part, eng.ntrain_blk, eng.npart, eng.A,
                            1.0 / eng.mb, eng.loss_sums, eng.grad_flat, eng.model.flat.data, eng.adam_m, eng.adam_v,
                            float(p.lr), float(b1), float(b2), float(p.adam_eps), 5, eng.adam_state,
                            eng.norm_part, eng.wimg, wm, eng.wt_map, eng.dt, eng.no_q)
        return f

    def gather():
        ext.grad_gather(b["slab"], eng.src_off, eng.src_meta, eng.part, eng.ntrain_blk, eng.npart, eng.A,
                        1.0 / eng.mb, eng.grad_flat, eng.loss_sums, b["lo"], b["hi"], b["partials"])

    def adam(wm):
        def f():
            ext.adam(eng.model.flat.data, eng.grad_flat, eng.adam_m, eng.adam_v, float(p.lr), float(b1), float(b2),
                     float(p.adam_eps), 0.0, eng.adam_state, eng.norm_part, eng.wimg, wm, eng.wt_map, eng.dt,
                     eng.no_q, 5)
        return f

    arms = {"fused": fused(eng.w_map), "no_images": fused(neg), "gather": gather, "adam": adam(eng.w_map),
            "adam_noimg": adam(neg)}
    if len(sys.argv) > 3:
        from pytorch_dppo_amd.ops import native

        def with_ext(e, fn):     # the arms' closures read `ext` at call time
            def f():
                nonlocal ext
                old, ext = ext, e
                try:
                    fn()
                finally:
                    ext = old
            return f
        v = native.load_variant(sys.argv[3])
        arms[f"fused_{sys.argv[3]}"] = with_ext(v, fused(eng.w_map))
        arms[f"gather_{sys.argv[3]}"] = with_ext(v, gather)
    res = {k: [] for k in arms}
    for _ in range(3):
        for k, fn in arms.items():
            res[k].append(timed(fn, reps))
    out = {k: min(v) for k, v in res.items()}
    out["dtype"] = dtype
    out["all"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
