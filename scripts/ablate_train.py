"""Phase ablation of mlp_train_kernel (diagnostics; cdna_hip_programming.md §7 step 2).

Times the fused update kernel with phases switched off, interleaved rounds in ONE process
(§5.4 rule 24), on the bench configuration (Humanoid dims, 65,536-row full batch, bf16).
Ablated calls do not produce gradients; nothing here feeds training.
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

# name -> (mlp_train ablation mask, wgrad impl)
VARIANTS = {"full": (0, 0), "wgrad_register_path": (0, 1), "no_transposed_stores": (1, 0), "no_v_fc1": (2, 0),
            "no_dgrad": (4, 0), "no_loss": (8, 0), "fwd_only_no_stores": (1 | 4 | 8, 0)}


def main():
    dev = torch.device("cuda", 0)
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536, batch_size=65536,
                    dtype=dtype)
    spec = get_spec(p.env_name)
    torch.manual_seed(0)
    model = ActorCritic(spec.obs_dim, spec.act_dim).to(dev)
    env = make_vec_env(spec, p.num_envs, device=dev)
    stats = RunningObsStats(spec.obs_dim, dev)
    p.use_graphs = False   # the ablation mask is read at launch time
    eng = HipEngine(p, model, env, stats, dev, 0)
    stats.observes(env.observe())
    eng.rollout()
    eng.values()
    eng.gae()
    eng.begin_update()
    ext = eng.ext
    rows_list = [int(r) for r in os.environ.get("ABLATE_ROWS", "64,32").split(",")]
    waves0 = eng.wgrad_waves
    res = {f"{k}@{r}": [] for r in rows_list for k in VARIANTS}
    for rnd in range(6):
        for key in res:
            name, rows = key.split("@")
            mask, impl = VARIANTS[name]
            ext.set_mlp_rows(int(rows))
            eng.sync_tile()
            ext.set_train_ablation(mask)
            ext.set_wgrad_impl(impl)
            eng.wgrad_waves = 8 if impl == 1 else waves0   # the register kernel takes 8-wave tiles
            eng._build_wgrad_plan(model)
            for _ in range(2):
                eng.grad(None)   # warm
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                eng.grad(None)
            e.record()
            torch.cuda.synchronize()
            res[key].append(s.elapsed_time(e) / 5 * 1e3)
    ext.set_train_ablation(0)
    ext.set_mlp_rows(0)
    ext.set_wgrad_impl(0)
    out = {k: {"median_us": sorted(v)[len(v) // 2], "min_us": min(v)} for k, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
