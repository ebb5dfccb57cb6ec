#!/usr/bin/env python3
"""Probe: what would the library GEMM (hipBLASLt via torch.mm) take for the split-bf16 wgrad?

The hand-written wgrad (csrc/wgrad.hip) computes all six dW = dY^T X at the bench geometry
(65,536 rows) as 3 bf16 MFMA products per element pair (hi.hi + hi.lo + lo.hi) in one grouped
split-K launch: ~155 us.  This times the same 18 GEMMs (3 per layer) as plain library calls on
row-major [rows][features] bf16 operands (the layout the library wants; ours are fragment-major),
with fp32 output where torch offers it.  Diagnostics for the design of the next wgrad, not a
product path.

    python scripts/probe_wgrad_blas.py [rows] [--bf16-out]
"""
import json
import sys

import torch

LAYERS = [("p_fc1", 100, 377), ("p_fc2", 100, 101), ("mu", 17, 101),
          ("v_fc1", 500, 377), ("v_fc2", 100, 501), ("v", 1, 101)]


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 65536
    dev = torch.device("cuda", 0)
    ops = []
    for name, n, k in LAYERS:
        dy = [torch.randn(M, n, device=dev, dtype=torch.bfloat16) for _ in range(2)]   # hi, lo
        x = [torch.randn(M, k, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        ops.append((name, n, k, dy, x))
    out = {}
    have_f32 = "--bf16-out" not in sys.argv
    if have_f32:
        try:
            torch.mm(ops[0][3][0].t(), ops[0][4][0], out_dtype=torch.float32)
        except Exception:  # noqa: BLE001
            have_f32 = False
    out["fp32_out"] = have_f32

    def run_all():
        for _, n, k, dy, x in ops:
            if have_f32:
                acc = torch.mm(dy[0].t(), x[0], out_dtype=torch.float32)
                acc += torch.mm(dy[0].t(), x[1], out_dtype=torch.float32)
                acc += torch.mm(dy[1].t(), x[0], out_dtype=torch.float32)
            else:
                acc = torch.mm(dy[0].t(), x[0]).float()
                acc += torch.mm(dy[0].t(), x[1]).float()
                acc += torch.mm(dy[1].t(), x[0]).float()

    def run_cat():
        # one GEMM per layer with the split terms concatenated along the reduction axis:
        # [dy_hi | dy_hi | dy_lo]^T [x_hi ; x_lo ; x_hi] = hi.hi + hi.lo + lo.hi
        for _, n, k, dy, x in ops:
            a = torch.cat([dy[0], dy[0], dy[1]], 0)
            b = torch.cat([x[0], x[1], x[0]], 0)
            if have_f32:
                torch.mm(a.t(), b, out_dtype=torch.float32)
            else:
                torch.mm(a.t(), b)

    cat_ops = []
    for _, n, k, dy, x in ops:
        cat_ops.append((torch.cat([dy[0], dy[0], dy[1]], 0), torch.cat([x[0], x[1], x[0]], 0)))

    def run_cat_pre():
        for a, b in cat_ops:
            if have_f32:
                torch.mm(a.t(), b, out_dtype=torch.float32)
            else:
                torch.mm(a.t(), b)

    per_layer = {}
    for name, n, k, dy, x in ops:
        def one(dy=dy, x=x):
            if have_f32:
                torch.mm(dy[0].t(), x[0], out_dtype=torch.float32)
            else:
                torch.mm(dy[0].t(), x[0])
        per_layer[name] = timed(one)
    out["one_gemm_per_layer_us"] = per_layer
    out["three_gemms_all_layers_us"] = timed(run_all)
    out["cat_k_one_gemm_per_layer_incl_cat_us"] = timed(run_cat)
    out["cat_k_one_gemm_per_layer_us"] = timed(run_cat_pre)
    out["rows"] = M
    print(json.dumps(out))


if __name__ == "__main__":
    main()
