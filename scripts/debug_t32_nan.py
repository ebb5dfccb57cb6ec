#!/usr/bin/env python3
"""Debug aid: the transposed-chain head update on one minibatch — which gradient ranges / operand
buffers / partial columns hold non-finite values (python scripts/debug_t32_nan.py [dtype])."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

from pytorch_dppo_amd.config import ppo_preset  # noqa: E402
from test_gpu_kernels import _engine, _fill_buffer  # noqa: E402


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    mb = 1024
    p = ppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=128, exploration_size=128 * 16, batch_size=mb,
                   dtype=dt, ent_coeff=0.01, loss="ppo", value_loss="mse", update_kernels="heads")
    eng, model, _, _ = _engine(p)
    print("phead", getattr(eng, "phead", None), flush=True)
    _fill_buffer(eng, model)
    idx = torch.randperm(eng.N, generator=torch.Generator().manual_seed(5))[:mb]
    for name in ("h1vT", "g1vT", "g2vT", "h1pT", "g1pT", "g2pT", "xT"):
        getattr(eng, name).fill_(0)
    for rep in range(3):
        eng.g1vT.fill_(0)
        eng.begin_update()
        eng.grad(idx)
        torch.cuda.synchronize()
        b = eng.decode(eng.g1vT.view(-1)).view(eng.ldT, -1)
        print("rep", rep, "g1vT nonfinite at", torch.nonzero(~torch.isfinite(b))[:8].tolist(),
              "huge", int((b.abs() > 1e3).sum()), flush=True)
        for nm in ("g1vT", "g2vT", "h1vT"):
            bb = eng.decode(getattr(eng, nm).view(-1)).view(eng.ldT, -1)
            bad = (~torch.isfinite(bb)) | (bb.abs() > 1e3)
            rows = torch.nonzero(bad.any(1)).flatten()
            print("  ", nm, "bad rows", rows[:24].tolist(), "per-row counts", bad.sum(1)[rows][:24].tolist(), flush=True)
    # reference g1 from the kernel's own g2 / h1 operands: (W2^T g2) * (1 - h1^2)
    W2 = model.view("v_fc2.weight").data
    if W2 is not None:
        g2 = eng.decode(eng.g2vT.view(-1)).view(eng.ldT, -1)[:, :W2.shape[0]]
        h1 = eng.decode(eng.h1vT.view(-1)).view(eng.ldT, -1)[:, :W2.shape[1]]
        g1r = (g2 @ W2) * (1 - h1 * h1)
        g1k = eng.decode(eng.g1vT.view(-1)).view(eng.ldT, -1)[:, :W2.shape[1]]
        err = (g1k - g1r).abs()
        bad = (err > 1e-2 * g1r.abs().max()) | ~torch.isfinite(g1k)
        print("g1 vs ref: bad", int(bad.sum()), "of", bad.numel())
        rr, ff = torch.nonzero(bad, as_tuple=True)
        print(" rows mod 32 hist", torch.bincount(rr % 32, minlength=32).tolist())
        print(" feat mod 32 hist", torch.bincount(ff % 32, minlength=32).tolist())
        print(" feat // 32 hist", torch.bincount(ff // 32, minlength=16).tolist())
        print(" row // 128 hist", torch.bincount(rr // 128, minlength=8).tolist())
        h1f = eng.decode(eng.h1vT.view(-1)).view(eng.ldT, -1)
        gar = g2 @ W2
        bad2 = ((g1k - gar).abs() > 1e-2 * gar.abs().max()) | ~torch.isfinite(g1k)
        r2, f2 = torch.nonzero(bad2, as_tuple=True)
        print(" DBG2: ga bad", int(bad2.sum()), "rows%32", torch.bincount(r2 % 32, minlength=32).tolist(),
              "feat%32", torch.bincount(f2 % 32, minlength=32).tolist())
        print(" DBG2 ex", [(int(a), int(b), float(g1k[a, b]), float(gar[a, b])) for a, b in zip(r2[:8], f2[:8])])
        print(" DBG1: g1vT == h1vT ?", bool(torch.equal(g1k, h1f[:, :g1k.shape[1]])),
              "mismatch", int((g1k != h1f[:, :g1k.shape[1]]).sum()))
        mm = torch.nonzero(g1k != h1f[:, :g1k.shape[1]])[:6].tolist()
        print(" DBG1 mismatches", [(a, b, float(g1k[a, b]), float(h1f[a, b])) for a, b in mm])
        print(" examples", [(int(a), int(b), float(g1k[a, b]), float(g1r[a, b])) for a, b in zip(rr[:6], ff[:6])])
    g = eng.grad_flat
    for k, (off, n) in model.offsets.items():
        seg = g[off:off + n]
        bad = (~torch.isfinite(seg)).sum().item()
        print(f"{k:16s} n={n:7d} nonfinite={bad} absmax={seg[torch.isfinite(seg)].abs().max().item() if n - bad else 0:.3e}")
    for name in ("h1vT", "g1vT", "g2vT", "h1pT", "g1pT", "g2pT", "xT"):
        b = eng.decode(getattr(eng, name).view(-1)) if hasattr(eng, "decode") else getattr(eng, name)
        bad = (~torch.isfinite(b)).sum().item()
        print(f"{name}: nonfinite {bad} of {b.numel()} absmax {b[torch.isfinite(b)].abs().max().item():.3e}")
        if bad:
            nz = torch.nonzero(~torch.isfinite(b.view(eng.ldT, -1)))[:6].tolist()
            print("   first", nz)
    for name, b in (("part_joint", eng.part_joint), ("part_h0", eng.part_h[0]), ("part_h1", eng.part_h[1])):
        bad = ~torch.isfinite(b)
        print(name, "nonfinite", int(bad.sum()), "cols", torch.nonzero(bad.any(0)).flatten()[:20].tolist(),
              "rows", torch.nonzero(bad.any(1)).flatten()[:20].tolist())


if __name__ == "__main__":
    main()
