#!/usr/bin/env python3
"""Bit-identity of a kernel variant build against the tree (diagnostics for A/B variants that
must not change numerics, e.g. a different DMA issue point): for each precision, two fresh
engines from the same seed, one on the default extension and one on _dppo_hip_<variant>, one
rollout + values + GAE + two update steps each; parameters and the last gradient must be equal.

    python scripts/variant_check.py g [dtypes]
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


def run(dtype, ext):
    dev = torch.device("cuda", 0)
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=2048, exploration_size=2048 * 16,
                    batch_size=2048 * 16, num_epoch=2, dtype=dtype, seed=7, update_kernels="heads")
    w = DPPOWorker(p, DistContext(device=dev))
    if ext is not None:
        w.engine.ext = ext
    w.iteration_step()
    w.iteration_step()
    torch.cuda.synchronize()
    return w.model.flat.data.clone(), w.engine.grad_flat.clone()


def main():
    var = sys.argv[1]
    dtypes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["bf16x3", "bf16", "fp8"]
    ext = native.load_variant(var)
    out = {}
    for dt in dtypes:
        a, ga = run(dt, None)
        b, gb = run(dt, ext)
        out[dt] = {"params_equal": bool(torch.equal(a, b)), "grad_equal": bool(torch.equal(ga, gb)),
                   "max_param_diff": float((a - b).abs().max())}
    print(json.dumps({"variant": var, **out}))
    if not all(v["params_equal"] and v["grad_equal"] for v in out.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
