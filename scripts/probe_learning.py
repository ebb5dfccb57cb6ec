"""Learning-signal probe (diagnostics): mean per-step reward over DPPO iterations for a few
(env, dtype) pairs, to size the GPU learning test.   python scripts/probe_learning.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.parallel.dist import DistContext  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    iters = int(os.environ.get("ITERS", 30))
    pairs = [x.split(":") for x in os.environ.get("PAIRS", "Humanoid-v2:fp32,Humanoid-v2:bf16x3").split(",")]
    for env, dt in pairs:
        t0 = time.time()
        p = dppo_preset(device="gpu", env_name=env, num_envs=1024, exploration_size=1024 * 16,
                        batch_size=1024 * 16, num_epoch=10, dtype=dt, seed=11)
        w = DPPOWorker(p, DistContext(device=dev))
        r = []
        for _ in range(iters):
            w.iteration_step()
            r.append(round(w.engine.rewards.mean().item(), 4))
        print(json.dumps({"env": env, "dtype": dt, "s": round(time.time() - t0, 1), "curve": r}), flush=True)


if __name__ == "__main__":
    main()
