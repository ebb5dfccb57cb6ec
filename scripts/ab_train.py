"""In-process A/B timing of the fused update kernel (mlp_train) and the wgrad/gather chain on
the bench configuration (Humanoid dims, 65,536-row full batch), interleaved rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24).  Diagnostics only.

    python scripts/ab_train.py bf16x3 [arm,arm,...]
arms: s3w4 / s3w8 (split-bf16 32-row tile at 4 / 8 waves), grad (mlp_train + wgrad + gather),
      train (mlp_train alone), wgrad (wgrad alone), values, rollout
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


def build(dtype):
    dev = torch.device("cuda", 0)
    E = int(os.environ.get("AB_ENVS", 4096))   # rows = 16 * E
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=16 * E, batch_size=16 * E,
                    dtype=dtype)
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
    eng.grad(None)
    return p, eng


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    want = sys.argv[2].split(",") if len(sys.argv) > 2 else ["s3w4", "s3w8"]
    p, eng = build(dtype)
    ext = eng.ext
    state = ext.s3_stream_state()
    wg_dense = ext.wgrad_dense()
    M = eng.mb

    def train():
        train_with(ext)

    def train_with(mod):
        opts = [0 if p.loss == "ppo" else 1, 0 if p.value_loss == "mse" else 1,
                1 if p.std_convention == "var" else 0, 0, eng.npart]
        mod.mlp_train(eng.dt, eng.x_buf, eng.empty, 0, M, eng.wimg, eng.layout, eng.scales, eng.model.flat.data,
                      eng.log_std_old, eng.A, eng.actions, eng.logp, eng.adv, eng.ret, eng.values_buf, eng.mu_prev,
                      eng.v_prev, opts, [float(p.clip), float(p.ent_coeff)], eng.tbufs, eng.ldT, eng.part, False,
                      eng._xT_valid)

    def wgrad():
        b = eng.buckets[0]
        ext.wgrad(eng.dt, eng.wg_g, eng.wg_x, eng.g_rows, eng.x_rows, eng.ldT, b["tasks"], b["tasks_host"], b["slab"],
                  eng.wgrad_waves)

    from pytorch_dppo_amd.ops import native
    ext_a = ext
    variants = {}

    def use_ext(name):   # "A" default build, else the variant module _dppo_hip_<name>
        if name == "A":
            mod = ext_a
        else:
            mod = variants.setdefault(name, native.load_variant(name))
        eng.ext = mod
        return mod

    def plan_mode(aligned):   # wgrad task plan: proportional chunks per tile vs one aligned row grid
        if getattr(eng, "wgrad_aligned", None) != aligned:
            eng.wgrad_aligned = aligned
            eng._build_wgrad_plan(eng.model)

    def plan_wgs(n):   # wgrad task count of the plan (engine_hip WGRAD_TARGET_WGS)
        if getattr(eng, "_ab_wgs", None) != n:
            eng._ab_wgs = n
            eng._build_wgrad_plan(eng.model, target_wgs=n)

    def waves(n):
        return lambda: (ext.set_s3_train_waves(n), eng.sync_tile())

    arms = {
        "s3w4": (waves(4), train), "s3w8": (waves(8), train),
        "wg_prop": (lambda: plan_mode(False), wgrad), "wg_aligned": (lambda: plan_mode(True), wgrad),
        "rs2": (lambda: (ext.set_s3_stream(True, 2, 0), eng.sync_tile()), train),
        "rs3": (lambda: (ext.set_s3_stream(True, 3, 0), eng.sync_tile()), train),
        "rs3d": (lambda: (ext.set_s3_stream(True, 3, 1), eng.sync_tile()), train),
        "rs2d": (lambda: (ext.set_s3_stream(True, 2, 1), eng.sync_tile()), train),
        "wg_sparse": (lambda: ext.set_wgrad_dense(False), wgrad),
        "wg_dense": (lambda: ext.set_wgrad_dense(True), wgrad),
        "tile32": (lambda: (ext.set_s3_stream(False, 3), eng.sync_tile()), train),
        "trainA": (lambda: use_ext("A"), lambda: train_with(ext_a)),
        "trainB": (lambda: use_ext("b"), lambda: train_with(variants["b"])),
        "valA": (lambda: use_ext("A"), eng.values), "valB": (lambda: use_ext("b"), eng.values),
        "rollA": (lambda: use_ext("A"), eng.rollout), "rollB": (lambda: use_ext("b"), eng.rollout),
        "train": (waves(8), train), "wgrad": (waves(8), wgrad),
        "grad": (waves(8), lambda: eng.grad(None)), "values": (waves(8), eng.values),
        "rollout": (waves(8), eng.rollout),
        "abl0": (lambda: ext.set_train_ablation(0), train), "abl1": (lambda: ext.set_train_ablation(1), train),
        "abl2": (lambda: ext.set_train_ablation(2), train), "abl4": (lambda: ext.set_train_ablation(4), train), "abl3": (lambda: ext.set_train_ablation(3), train),
        "abl8": (lambda: ext.set_train_ablation(8), train), "abl16": (lambda: ext.set_train_ablation(16), train),
        "abl7": (lambda: ext.set_train_ablation(7), train),
        "val4": (lambda: ext.set_s3_value_waves(4), eng.values),
        "val8": (lambda: ext.set_s3_value_waves(8), eng.values),
        "refresh": (lambda: None, eng.refresh_fwd_image),
        "roll4": (lambda: ext.set_rollout_waves(4), eng.rollout),
        "roll8": (lambda: ext.set_rollout_waves(8), eng.rollout),
    }
    for n in (192, 224, 240, 256, 272, 288, 320, 384, 448, 512):
        arms[f"wgs{n}"] = ((lambda n=n: plan_wgs(n)), wgrad)
    res = {k: [] for k in want}
    for _ in range(5):
        for k in want:
            setup, fn = arms[k]
            setup()
            res[k].append(timed(fn))
    use_ext("A")
    ext.set_s3_stream(state > 0, (state % 10) or 3, state // 10 if state else -1)
    eng.sync_tile()
    ext.set_wgrad_dense(wg_dense)
    plan_mode(False)
    plan_wgs(0)
    ext.set_s3_train_waves(8)
    ext.set_train_ablation(0)
    out = {k: {"median_us": sorted(v)[len(v) // 2], "all_us": [round(x, 1) for x in v]} for k, v in res.items()}
    print(json.dumps({"dtype": dtype, "arms": out}, indent=1))


if __name__ == "__main__":
    main()
