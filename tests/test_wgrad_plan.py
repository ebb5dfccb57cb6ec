"""Host-side plan of the grouped wgrad launch (pytorch_dppo_amd/runtime/engine_hip.py
wgrad_tiles): every layer's [fan_out][fan_in + 1] gradient is covered exactly once by tiles the
kernel accepts (csrc/wgrad.hip wgrad_task_ok: nq*kq <= 8 waves and nq + kq <= 6 fragment slots, or
wide: two quadrants per wave, nq even, nq + kq <= 10; tiles inside the 128-row padded operand
buffers).  CPU only — the kernel itself is checked against autograd in
tests/test_gpu_kernels.py."""

import pytest
import torch

from pytorch_dppo_amd.runtime.engine_hip import WT, wgrad_tile_ok, wgrad_tiles

# (fan_out, fan_in) of the six layers for the reference envs' obs / act dims
LAYERS = {
    "Humanoid-v2": [(100, 376), (100, 100), (17, 100), (500, 376), (100, 500), (1, 100)],
    "HalfCheetah-v2": [(100, 17), (100, 100), (6, 100), (500, 17), (100, 500), (1, 100)],
    "InvertedPendulum-v1": [(100, 4), (100, 100), (1, 100), (500, 4), (100, 500), (1, 100)],
}


def _r(x, m):
    return -(-x // m) * m


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("env", sorted(LAYERS))
def test_tiles_cover_each_gradient_once(env, wide):
    for li, (n, fan_in) in enumerate(LAYERS[env]):
        k = fan_in + 1
        cover = torch.zeros(_r(n, 64), _r(k, 64), dtype=torch.int32)
        for (tl, n0, k0, nq, kq) in wgrad_tiles(li, n, k, wide):
            assert tl == li
            assert wgrad_tile_ok(nq, kq, wide)
            if nq * kq > 8:
                assert wide and nq * kq <= 16 and nq % 2 == 0 and nq + kq <= 10
            else:
                assert nq + kq <= 6
            assert n0 % 64 == 0 and k0 % 64 == 0
            # operand buffers hold _r(rows, WT) rows (engine_hip: g_rows / x_rows)
            assert n0 + 64 * nq <= _r(n, WT) and k0 + 64 * kq <= _r(k, WT)
            cover[n0:n0 + 64 * nq, k0:k0 + 64 * kq] += 1
        assert bool((cover == 1).all()), (env, li)


def test_humanoid_value_fc1_streams_fewer_rows_than_square_tiles():
    tiles = wgrad_tiles(3, 500, 377)
    rows_per_step = sum(64 * (nq + kq) for (_, _, _, nq, kq) in tiles)
    square = (_r(500, 128) // 128) * (_r(377, 128) // 128) * 256   # 128x128 tiles
    assert rows_per_step == 2304 and rows_per_step < square
    # two quadrants per wave: 4x3 tiles (two waves per 128 x 64 output rows)
    wide = wgrad_tiles(3, 500, 377, True)
    assert sorted((nq, kq) for (_, _, _, nq, kq) in wide) == [(4, 3)] * 4
    assert sum(64 * (nq + kq) for (_, _, _, nq, kq) in wide) == 1792


@pytest.mark.parametrize("heads,q8,wide", [(False, False, False), (True, False, False), (True, True, False),
                                           (True, False, True)])
@pytest.mark.parametrize("env", ["Humanoid-v2", "HalfCheetah-v2"])
def test_plan_tasks_cover_tiles_and_batch_once(env, heads, q8, wide):
    """The full task list (HipEngine._build_wgrad_plan run on a CPU stand-in): each output tile's
    tasks cover the batch rows [0, ldT) exactly once with 64-row-aligned chunks, every task owns
    a disjoint slab region, the task count is ~one per CU, and every parameter's gather entry
    (offset, chunk count, stride) matches its tile.  q8 (fp8 mode's e4m3 wgrad): 128-row chunks
    (the kernel's 16x16x128 MFMA consumes four 32-row k-steps at a time)."""
    from types import SimpleNamespace
    from pytorch_dppo_amd.envs import get_spec
    from pytorch_dppo_amd.models.actor_critic import ActorCritic
    from pytorch_dppo_amd.runtime.engine_hip import HipEngine

    spec = get_spec(env)
    model = ActorCritic(spec.obs_dim, spec.act_dim)
    stub = SimpleNamespace(L=model.packed_layout(), ldT=65536, A=spec.act_dim, device=torch.device("cpu"),
                           heads=heads, q8=q8, wgrad_wide=wide, head_range=[model.head_ranges["policy"], model.head_ranges["value"]],
                           _slab_index=HipEngine._slab_index, _slab_runs=HipEngine._slab_runs)
    HipEngine._build_wgrad_plan(stub, model, target_wgs=256)
    total = 0
    for b in stub.buckets:
        t = b["tasks_host"].view(-1, 8).tolist()
        total += len(t)
        assert len(t) <= 256 + 16
        used = torch.zeros(b["slab"].numel(), dtype=torch.int32)
        rows = {}
        for (li, n0, k0, m0, m1, off, nq, kq) in t:
            assert wgrad_tile_ok(nq, kq, wide)
            al = 128 if q8 else 64
            assert m0 % al == 0 and (m1 - m0) % al == 0 and 0 <= m0 < m1 <= stub.ldT
            used[off:off + 64 * nq * 64 * kq] += 1
            rows.setdefault((li, n0, k0), []).append((m0, m1))
        assert bool((used == 1).all())
        for key, rs in rows.items():
            rs.sort()
            assert rs[0][0] == 0 and rs[-1][1] == stub.ldT and all(a[1] == b_[0] for a, b_ in zip(rs, rs[1:]))
    lo = min(b["lo"] for b in stub.buckets)
    slab_fed = torch.ones(model.num_params, dtype=torch.bool)
    slab_fed[:lo] = False
    if heads:   # mu and v are the head kernels' reduce items (fused dW partials): no tile, meta 0
        for name in ("mu.weight", "mu.bias", "v.weight", "v.bias"):
            o, n = model.offsets[name]
            slab_fed[o:o + n] = False
    meta = stub.src_meta
    assert bool(((meta[slab_fed] >> 5) >= 1).all()) and bool(((meta[slab_fed] & 31) >= 1).all())
    assert bool((meta[~slab_fed] == 0).all())
    # the gathers' slab runs cover exactly the slab-fed elements of each bucket's range
    for b in stub.buckets:
        r = b["runs"]
        covered = torch.zeros(model.num_params, dtype=torch.bool)
        for k in range(0, len(r), 2):
            assert b["lo"] <= r[k] < r[k + 1] <= b["hi"]
            covered[r[k]:r[k + 1]] = True
        want = torch.zeros(model.num_params, dtype=torch.bool)
        want[b["lo"]:b["hi"]] = slab_fed[b["lo"]:b["hi"]]
        assert torch.equal(covered, want)
    if heads:   # per-head buckets: policy [A, v_fc1.weight), value [v_fc1.weight, n)
        (b0, b1) = stub.buckets
        assert (b0["lo"], b0["hi"]) == (spec.act_dim, model.head_ranges["policy"][1]) and b0["partials"]
        assert (b1["lo"], b1["hi"]) == model.head_ranges["value"] and not b1["partials"]
    assert total >= 200


def test_tile_rule_matches_the_kernel():
    """The host plan's tile rule (wgrad_tile_ok) is the kernel's (csrc/wgrad.hip wgrad_task_ok, which
    the launch binding enforces) for every dtype: fp32 / e4m3 one quadrant per wave only, split-bf16 /
    bf16 also the two-quadrant tiles.  Needs the built extension (it loads on the CPU too)."""
    from pytorch_dppo_amd.ops import native
    try:
        ext = native.load()
    except Exception as e:  # noqa: BLE001 — not built in this checkout
        pytest.skip(f"HIP extension not built: {e}")
    for dt in (native.DT_CODE[d] for d in ("fp32", "bf16x3", "bf16", "fp8")):
        wide = dt in (native.DT_CODE["bf16x3"], native.DT_CODE["bf16"])
        for nq in range(0, 18):
            for kq in range(0, 18):
                assert bool(ext.wgrad_task_ok(dt, nq, kq)) == wgrad_tile_ok(nq, kq, wide), (dt, nq, kq)
