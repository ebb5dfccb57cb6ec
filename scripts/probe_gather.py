"""Where the fused gather + Adam time goes (diagnostics): the joint world-1 launch at the bench
geometry, timed back to back as is, without the slab elements (reduce items only), and without
the reduce items (slab elements only).   python scripts/probe_gather.py [bf16x3|bf16]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.parallel.dist import DistContext  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    dev = torch.device("cuda", 0)
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536, batch_size=65536,
                    dtype=dt, seed=1)
    w = DPPOWorker(p, DistContext(device=dev))
    w.iteration_step()
    eng = w.engine
    ext = eng.ext
    b = eng.joint_bucket
    src_off, src_meta = eng.joint_src
    rc, rd = eng.items["joint"]
    b1, b2 = p.adam_betas
    n = eng.model.num_params
    empty_i = torch.empty(0, dtype=torch.int32, device=dev)

    def run(items, runs):
        c, d = (rc, rd) if items else (empty_i, empty_i)
        ext.gather_adam(b["slab"], src_off, src_meta, eng.part_joint, eng.nhead_blk, eng.part_joint.shape[1], c, d,
                        runs, 1.0 / eng.mb, eng.loss_sums, eng.grad_flat, eng.model.flat.data, eng.adam_m,
                        eng.adam_v, 0.0, float(b1), float(b2), float(p.adam_eps), 1, eng.adam_state,
                        eng.norm_part[:eng.norm_n_whole], eng.wimg, eng.w_map, eng.wt_map, eng.dt, eng.no_q,
                        *eng._f8())
    arms = {"full": (True, b["runs"]), "items_only": (True, [n, n]), "slab_only": (False, b["runs"])}
    res = {}
    for name, (items, runs) in arms.items():
        for _ in range(3):
            run(items, runs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run(items, runs)
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1e3 / 50, 2)
    res["nitems"] = int(rc.numel())
    res["grid"] = int(eng.norm_n_whole)
    print(json.dumps({"dtype": dt, "us": res}))


if __name__ == "__main__":
    main()
