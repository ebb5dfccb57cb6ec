#!/usr/bin/env python3
"""Debug aid: the 32x32 policy head's row-major operand and partials vs torch (fp32) on one
update call: g1 per row/feature, the per-workgroup dW_mu and dW_p2 blocks, and the whole gradient.

    python scripts/debug_phead.py [dtype] [mb|full]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

from pytorch_dppo_amd.config import ppo_preset  # noqa: E402
from test_gpu_kernels import DEV, _engine, _fill_buffer, _torch_grad  # noqa: E402


def report(name, k, r, tol):
    err = (k - r).abs()
    bad = (err > tol * (r.abs().max() + 1e-12)) | ~torch.isfinite(k)
    rows, feats = torch.nonzero(bad, as_tuple=True)
    print(f"{name}: bad {int(bad.sum())}/{bad.numel()}  max err {err[torch.isfinite(err)].max().item():.3e}  "
          f"ref max {r.abs().max().item():.3e}", flush=True)
    if bad.any():
        print("   rows%32", torch.bincount(rows % 32, minlength=32).tolist())
        print("   rows//32 (first 16)", torch.bincount(rows // 32, minlength=16)[:16].tolist())
        print("   feats", torch.bincount(feats, minlength=k.shape[1]).tolist()[:128])
        print("   ex", [(int(a), int(b), float(k[a, b]), float(r[a, b])) for a, b in zip(rows[:6], feats[:6])])


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
    mode = sys.argv[2] if len(sys.argv) > 2 else "full"
    N = 128 * 16
    mb = N if mode == "full" else int(mode)
    p = ppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=128, exploration_size=N, batch_size=mb, dtype=dt,
                   ent_coeff=0.01, update_kernels="heads")
    p.phead_kernel = True
    eng, model, _, _ = _engine(p)
    print("phead", eng.phead, "ldT", eng.ldT, flush=True)
    xq = _fill_buffer(eng, model)
    idx = None if mode == "full" else torch.randperm(eng.N, generator=torch.Generator().manual_seed(5))[:mb]
    for nm in ("g1pT", "xT"):
        getattr(eng, nm).zero_()
    eng.begin_update()
    eng.grad(idx)
    torch.cuda.synchronize()
    print("x_mode", eng._x_mode, flush=True)
    ii = torch.arange(eng.N, device=DEV) if idx is None else idx.to(DEV)
    M = ii.numel()
    x = xq[ii].clone()
    W1, b1 = model.view("p_fc1.weight").data, model.view("p_fc1.bias").data
    W2, b2 = model.view("p_fc2.weight").data, model.view("p_fc2.bias").data
    W3 = model.view("mu.weight").data
    h1 = torch.tanh(x @ W1.t() + b1)
    h2 = torch.tanh(h1 @ W2.t() + b2)
    h2r = h2.detach().requires_grad_(True)
    mu = h2r @ W3.t() + model.view("mu.bias").data
    mu_l = mu.detach().requires_grad_(True)
    g_ref, out = _torch_grad(model, p, xq, eng, ii)
    # dL/dmu per row (unnormalised: the kernel's partials are sums, the gather scales by 1/M)
    from pytorch_dppo_amd.ops import oracle   # noqa: E402
    with torch.no_grad():
        _, ls, v = model(x)
    out2 = oracle.ppo_loss(mu_l, ls.detach(), v.detach(), eng.actions[ii], eng.logp[ii], eng.adv[ii], eng.ret[ii],
                           eng.values_buf[:eng.N][ii], clip=p.clip, ent_coeff=p.ent_coeff,
                           value_loss=p.value_loss, convention=p.std_convention)
    dmu = torch.autograd.grad(out2["loss"], mu_l)[0] * M
    g2 = (dmu @ W3) * (1 - h2 * h2)
    g1 = (g2 @ W2) * (1 - h1 * h1)
    dec = lambda t: eng.decode(t.view(-1)).view(eng.ldT, -1)[:M]
    # (h1 and g2 stay on chip: p_fc2's weight gradient is summed in the kernel, checked below)
    report("g1", dec(eng.g1pT)[:, :100], g1, 2e-3)
    if mode != "full":
        report("x", dec(eng.xT)[:, :model.num_inputs], x, 1e-3)
    # the per-workgroup dW_mu blocks [32][128] (bias column 100) vs torch's sum over each block's rows
    # (the joint world-1 path's partial rows, or the per-head path's)
    joint = bool(eng.part_joint.abs().sum() > 0)
    part = eng.part_joint if joint else eng.part_h[0]
    c0 = eng.part_dw_joint[0] if joint else eng.part_dw[0]
    blk = part[: (M + 127) // 128, c0:c0 + 32 * 128].view(-1, 32, 128)
    A = model.num_outputs
    h2b = torch.cat([h2, torch.ones(M, 1, device=DEV)], 1)
    ref = torch.zeros(blk.shape[0], 32, 128, device=DEV)
    for b_ in range(blk.shape[0]):
        rr = slice(128 * b_, min(128 * (b_ + 1), M))
        ref[b_, :A, :101] = dmu[rr].t() @ h2b[rr]
    print("dW_mu block: kernel absmax", blk.abs().max().item(), "ref absmax", ref.abs().max().item(),
          "max err", (blk - ref).abs().max().item(), flush=True)
    nz = torch.nonzero(blk[0].abs() > 0)
    print("   block0 nonzero entries", nz.shape[0], nz[:8].tolist(), flush=True)
    # the per-workgroup dW_p2 blocks [128 out][128 in] (bias column 100; only out < 100, in <= 100
    # are written) vs torch's sum over each block's rows
    if eng.phead_p2:   # (bf16: h1p / g2p go to the wgrad instead)
        b2 = part[: (M + 127) // 128, c0 + 32 * 128:c0 + 32 * 128 + 128 * 128].view(-1, 128, 128)[:, :100, :101]
        h1b = torch.cat([h1, torch.ones(M, 1, device=DEV)], 1)
        ref2 = torch.stack([g2[128 * b_:128 * (b_ + 1)].t() @ h1b[128 * b_:128 * (b_ + 1)]
                            for b_ in range(b2.shape[0])])
        print("dW_p2 blocks: max err", (b2 - ref2).abs().max().item(), "ref absmax", ref2.abs().max().item(),
              flush=True)
    g = eng.grad_flat
    for k_ in ("log_std", "p_fc1.weight", "p_fc1.bias", "p_fc2.weight", "p_fc2.bias", "mu.weight", "mu.bias",
               "v_fc1.weight", "v_fc2.weight", "v.weight"):
        o, n = model.offsets[k_]
        rel = (g[o:o + n] - g_ref[o:o + n]).norm().item() / (g_ref[o:o + n].norm().item() + 1e-12)
        print(f"grad {k_:14s} rel {rel:.3e}", flush=True)


if __name__ == "__main__":
    main()
