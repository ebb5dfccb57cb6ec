"""Per-phase cycle timeline of the fused update kernel (diagnostics).

Lane 0 of every wave of every EVERY-th workgroup stamps s_memtime (shader clock) at the phase
boundaries of mlp_train_kernel (csrc/mlp.hip STAMP(i)); this prints the median cycles per
phase over the sampled workgroups, for each row tile.  Bench configuration (Humanoid dims,
65,536-row full batch).
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

PHASES_RS = ["fc1 (X ring + 39 tiles)", "fc2 (chained)", "h2 epilogue + fc3", "loss + dY stores", "dgrad fc3",
             "dgrad fc2 policy", "dgrad fc2 value"]
PHASES = ["load_x+preset", "fc1 (p,v) own", "fc1 barrier wait", "preset", "fc2 own", "fc2 barrier wait",
          "fc3 + sync", "loss + sync", "partials+dY^T stores", "dgrad fc3 own", "dgrad fc3 barrier",
          "dgrad fc2 own"]
EVERY = 16


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
    out = {}
    for rows in [int(r) for r in os.environ.get("TIMELINE_ROWS", "64,32").split(",")]:
        ext.set_mlp_rows(rows)      # 0: split-bf16 -> the streaming kernel (mlp_stream.hip)
        rs = rows == 0
        if rs:
            ext.set_s3_stream(True, int(os.environ.get("TIMELINE_RS_STAGES", "3")))
        eng.sync_tile()
        rows = eng.train_rows
        phases = PHASES_RS if rs else PHASES
        nph = len(phases)
        nw = int(ext.train_waves(eng.dt, eng.layout, eng.A))
        nblk = eng.ldT // rows
        buf = torch.zeros(((nblk + EVERY - 1) // EVERY) * nw * 16, dtype=torch.int64, device=dev)
        for _ in range(3):
            eng.grad(None)
        ext.set_train_tstamp(buf, EVERY)
        ext.set_train_ablation(int(os.environ.get("TIMELINE_ABLATE", "0")))   # diagnostics
        eng.grad(None)
        torch.cuda.synchronize()
        ext.set_train_ablation(0)
        ext.set_train_tstamp(torch.empty(0, dtype=torch.int64, device=dev), 1)
        t = buf.view(-1, nw, 16).cpu().double()
        d = t[:, :, 1:nph + 1] - t[:, :, 0:nph]        # [blk][wave][phase]
        tot = (t[:, :, nph] - t[:, :, 0])
        res = {"rows": rows, "kernel": "streaming" if rs else "tile", "sampled_blocks": t.shape[0],
               "total_cycles_median": float(tot.median()),
               "phases_median_cycles(max over waves)": {ph: float(d[:, :, i].max(dim=1).values.median())
                                                        for i, ph in enumerate(phases)},
               "phases_median_cycles(mean over waves)": {ph: float(d[:, :, i].mean(dim=1).median())
                                                         for i, ph in enumerate(phases)}}
        # per dispatch round (blocks b .. b + #CUs - 1 start together): is the x load slower in
        # the first, lockstep round than in later ones?  (s_memtime is per XCD: compare within
        # XCD = block % 8, relative to that XCD's first stamp.)
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        blk = torch.arange(t.shape[0]) * EVERY
        rnd = blk // ncu
        by_round = {}
        for r_ in sorted(set(rnd.tolist())):
            m = rnd == r_
            by_round[int(r_)] = {"blocks": int(m.sum()),
                                 "load_x": float(d[m, :, 0].max(dim=1).values.median()),
                                 "fc1": float(d[m, :, 1].max(dim=1).values.median()),
                                 "total": float(tot[m].median())}
        res["by_round"] = by_round
        start = t[:, 0, 0]
        xcd = blk % 8
        rel = torch.zeros_like(start)
        for x_ in range(8):
            m = xcd == x_
            if m.any():
                rel[m] = start[m] - start[m].min()
        res["start_rel_cycles_by_round"] = {int(r_): [float(v) for v in rel[rnd == r_].quantile(
            torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64))] for r_ in sorted(set(rnd.tolist()))}
        out[("rs" if rs else "rows") + str(rows)] = res
        if rs:
            ext.set_s3_stream(False, 3)
    ext.set_mlp_rows(0)
    # rollout: per-wave cycles per phase summed over the T steps, median over workgroups
    nblk = (eng.E + 15) // 16
    rb = torch.zeros(nblk * 8 * 8, dtype=torch.int64, device=dev)
    eng.rollout()
    ext.set_rollout_tstamp(rb)
    eng.rollout()
    torch.cuda.synchronize()
    ext.set_rollout_tstamp(torch.empty(0, dtype=torch.int64, device=dev))
    r = rb.view(nblk, 8, 8).cpu().double()
    names = ["observe+norm (a)", "fc1", "fc2", "fc3", "sample (c)", "logp/reward (d)", "env step (e)"]
    out["rollout_per_step_cycles"] = {n: float(r[:, :, i].max(dim=1).values.median()) / eng.T
                                      for i, n in enumerate(names)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
