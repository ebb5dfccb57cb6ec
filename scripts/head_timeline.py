"""Per-phase cycle timeline of the per-head update kernels (csrc/mlp_head.hip HD_STAMP).

Lane 0 of every wave of every EVERY-th workgroup stamps s_memtime (shader clock) at the phase
boundaries; this prints the median cycles per phase (max over the 4 waves) for the policy and
the value kernel at the bench geometry (Humanoid dims, 65,536-row full batch).

    python scripts/head_timeline.py [bf16x3|bf16]
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

# stamp i -> i+1 phases (HD_STAMP 0..7), plus fc1 sub-spans from stamps 8 / 9
PHASES = ["fc1", "fc2", "fc3 wait", "fc3 + loss", "dgrad fc3", "dgrad fc2", "partials"]
EVERY = 8


def main():
    dev = torch.device("cuda", 0)
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536, batch_size=65536,
                    dtype=args[0] if args else "bf16x3", update_kernels="heads")
    p.phead_kernel = False     # (the 32x32 policy head, csrc/phead.hip, takes no stamps)
    spec = get_spec(p.env_name)
    torch.manual_seed(0)
    model = ActorCritic(spec.obs_dim, spec.act_dim).to(dev)
    env = make_vec_env(spec, p.num_envs, device=dev)
    stats = RunningObsStats(spec.obs_dim, dev)
    eng = HipEngine(p, model, env, stats, dev, 0)
    assert eng.heads
    stats.observes(env.observe())
    eng.rollout()
    eng.values()
    eng.gae()
    eng.begin_update()
    ext = eng.ext
    nblk = eng.nhead_blk
    out = {}
    mbt = eng._minibatch(None)
    for h in (0, 1):
        nw = int(ext.head_waves(h))
        buf = torch.zeros(((nblk + EVERY - 1) // EVERY) * nw * 16, dtype=torch.int64, device=dev)
        for _ in range(3):
            eng._head_chain(h, *mbt)
        torch.cuda.synchronize()
        ext.set_train_tstamp(buf, EVERY)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        eng._head_chain(h, *mbt)
        ev[1].record()
        torch.cuda.synchronize()
        ext.set_train_tstamp(torch.empty(0, dtype=torch.int64, device=dev), 1)
        t = buf.view(-1, nw, 16).cpu().double()
        d = t[:, :, 1:8] - t[:, :, 0:7]
        tot = t[:, :, 7] - t[:, :, 0]
        res = {"kernel": "mlp_head_kernel",
               "sampled_blocks": t.shape[0], "total_cycles_median": float(tot.max(dim=1).values.median()),
               "chain_ms": ev[0].elapsed_time(ev[1]),
               "phases_median_cycles(max over waves)": {ph: float(d[:, :, i].max(dim=1).values.median())
                                                        for i, ph in enumerate(PHASES)},
               }
        res["fc1_first_span"] = float((t[:, :, 8] - t[:, :, 0]).max(dim=1).values.median())
        res["fc1_mid_span(4 k-steps value / 3 stages policy)"] = float((t[:, :, 9] - t[:, :, 8]).max(dim=1).values.median())
        # sub-spans (max over waves): fc3 MFMAs (3 -> 12) vs the loss (12 -> 4); the partials phase as
        # the fused narrow-layer dW MFMAs (6 -> 10), the wave's store / DMA drain (10 -> 11) and the
        # workgroup reduction + partial-row stores (11 -> 7)
        res["sub_spans_median_cycles"] = {
            name: float((t[:, :, b] - t[:, :, a_]).max(dim=1).values.median())
            for name, a_, b in (("fc3", 3, 12), ("loss", 12, 4), ("narrow dW", 6, 10), ("drain", 10, 11),
                                ("reduce + store", 11, 7))}
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        blk = torch.arange(t.shape[0]) * EVERY
        rnd = blk // ncu
        res["total_by_round"] = {int(r): float(tot[rnd == r].max(dim=1).values.median()) for r in sorted(set(rnd.tolist()))}
        out["policy" if h == 0 else "value"] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
