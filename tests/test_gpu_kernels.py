"""HIP kernel numerics vs the plain-PyTorch fp32 oracle (SURVEY §4 'Unit: HIP kernels').

fp32 operands run the exact-f32 MFMA path (v_mfma_f32_16x16x4_f32) and bf16x3 (split-bf16 hi/lo
operands on three bf16 MFMAs, the fp32-accurate fast mode) -> the same tight tolerances;
bf16 operands -> loose, relative budgets.  Shapes cover Pendulum (3/1), HalfCheetah (17/6)
and Humanoid (376/17) dims with odd E and padded tails.
"""
import json
import math

import pytest
import torch

from pytorch_dppo_amd.config import Params, dppo_preset, ppo_preset
from pytorch_dppo_amd.envs import get_spec, make_vec_env
from pytorch_dppo_amd.models.actor_critic import ActorCritic
from pytorch_dppo_amd.ops import oracle, storage
from pytorch_dppo_amd.utils.obs_stats import RunningObsStats

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0) if torch.cuda.is_available() else None


def _ext():
    from pytorch_dppo_amd.ops import native
    return native.load()


def _model(O, A, hidden=(100, 100), seed=0):
    torch.manual_seed(seed)
    m = ActorCritic(O, A, hidden).to(DEV)
    with torch.no_grad():
        m.flat.data[:A] = torch.linspace(-0.5, 0.3, A, device=DEV)  # non-trivial log_std
    return m


def _engine(params, seed=0):
    from pytorch_dppo_amd.runtime.engine_hip import HipEngine
    spec = get_spec(params.env_name)
    torch.manual_seed(seed)
    model = ActorCritic(spec.obs_dim, spec.act_dim, params.hidden).to(DEV)
    env = make_vec_env(spec, params.num_envs, seed=params.seed, device=DEV)
    stats = RunningObsStats(spec.obs_dim, DEV)
    return HipEngine(params, model, env, stats, DEV, 0), model, env, stats


def test_extension_loads_for_gfx950():
    ext = _ext()
    assert ext.arch == "gfx950"
    assert ext.__file__.endswith(".so")


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "bf16x3"])
def test_pack_matches_reference_layout(dtype):
    p = dppo_preset(device="gpu", env_name="HalfCheetah-v2", num_envs=64, exploration_size=256,
                    batch_size=256, dtype=dtype)
    eng, model, _, _ = _engine(p)
    ref = storage.encode(model.packed_layout().pack(model.flat.data), eng.dt)
    assert torch.equal(eng.wimg, ref)       # bit-exact, incl. the device hi/lo split (RNE both)
    if dtype == "bf16x3":
        err = (eng.decode(eng.wimg) - model.packed_layout().pack(model.flat.data)).abs().max().item()
        assert err <= 2 ** -16 * model.flat.data.abs().max().item()


@pytest.mark.parametrize("env_name,dtype,tol", [("Pendulum-v0", "fp32", 2e-5), ("HalfCheetah-v2", "fp32", 2e-5),
                                                ("Humanoid-v2", "fp32", 5e-5), ("Pendulum-v0", "bf16x3", 2e-5),
                                                ("HalfCheetah-v2", "bf16x3", 2e-5), ("Humanoid-v2", "bf16x3", 5e-5),
                                                ("Humanoid-v2", "bf16", 3e-2),
                                                ("Humanoid-v2", "fp8", 1.5e-1), ("HalfCheetah-v2", "fp8", 1.5e-1)])
def test_value_forward(env_name, dtype, tol):
    p = dppo_preset(device="gpu", env_name=env_name, num_envs=37, exploration_size=37 * 5,
                    batch_size=37 * 5, dtype=dtype)
    eng, model, _, _ = _engine(p)
    O = model.num_inputs
    M = (eng.T + 1) * eng.E
    x = torch.randn(M, O, device=DEV).clamp(-5, 5)
    xb = torch.zeros(M, eng.d0, device=DEV)
    xb[:, :O] = x
    xb[:, O] = 1.0
    eng.x_buf.copy_(eng.encode(xb))
    eng.values()
    with torch.no_grad():
        _, _, v = model(eng.decode(eng.x_buf)[:, :O])
    err = (eng.values_buf - v.reshape(-1)).abs().max().item()
    scale = v.abs().max().item() + 1e-3
    assert err / scale < tol, (err, scale)


@pytest.mark.parametrize("dtype,tol", [("bf16x3", 2e-5), ("bf16", 3e-2)])
@pytest.mark.parametrize("E,T", [(3001, 15), (2048, 16)])
def test_value_forward_on_head_kernel_matches_tile_kernel(dtype, tol, E, T):
    """values() on the value head's streaming kernel in forward mode (csrc/mlp_head.hip FWD, 128
    rows per workgroup; taken from one full round of workgroups up) vs mlp.hip's value kernel and
    the fp32 torch model: 3001 x 16 rows (not a multiple of 128, tail > a quarter round: all on the
    head kernel) and 2048 x 17 rows on 256 CUs (one past a whole round, whose tail rows the 32-row
    kernel takes)"""
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T,
                    batch_size=E * T, dtype=dtype)
    eng, model, _, _ = _engine(p)
    O = model.num_inputs
    M = (eng.T + 1) * eng.E
    assert M % 128 != 0 or M > 128 * torch.cuda.get_device_properties(DEV).multi_processor_count
    xb = torch.zeros(M, eng.d0, device=DEV)
    xb[:, :O] = torch.randn(M, O, device=DEV).clamp(-5, 5)
    xb[:, O] = 1.0
    eng.x_buf.copy_(eng.encode(xb))
    out = {}
    try:
        for on in (True, False):
            eng.ext.set_head_kernels(on)
            eng.values_buf.fill_(float("nan"))
            eng.values()
            out[on] = eng.values_buf.clone()
    finally:
        eng.ext.set_head_kernels(True)
    with torch.no_grad():
        _, _, v = model(eng.decode(eng.x_buf)[:, :O])
    scale = v.abs().max().item()
    assert torch.isfinite(out[True]).all()
    assert (out[True] - v.reshape(-1)).abs().max().item() < tol * scale
    assert (out[True] - out[False]).abs().max().item() < tol * scale


@pytest.mark.parametrize("dtype", ["bf16x3", "bf16"])
@pytest.mark.parametrize("loss,mb", [("ppo", None), ("ppo", 1024), ("ppo", 1000), ("dppo_ref", 768)])
def test_phead_update_matches_16x16_head_update(dtype, loss, mb):
    """The policy head's update on the 32x32 transposed-chain kernel (csrc/phead.hip: row-major
    h1p / g1p / g2p, the observation operand of both fc1 layers row-major — x_buf itself for a
    full batch (mb None), the kernel's gathered rows for a minibatch; dW_mu by MFMA over the
    LDS-staged h2 / dL/dmu; at bf16x3 dW_p2 too) vs the 16x16 head kernels: the whole gradient, the loss sums and the
    reference loss's mu_prev; vs autograd for the ppo loss.  Ragged minibatches (1000, 768) leave
    rows past M in the last workgroup (zero gradient)."""
    N = 128 * 16
    kw = dict(device="gpu", env_name="Humanoid-v2", num_envs=128, exploration_size=N, batch_size=mb or N,
              dtype=dtype, ent_coeff=0.01, loss=loss, update_kernels="heads")
    bf = dtype == "bf16"
    res = {}
    for ph in (True, False):
        p = ppo_preset(**kw) if loss == "ppo" else dppo_preset(**kw)
        p.phead_kernel = ph
        eng, model, _, _ = _engine(p)
        assert eng.phead == ph
        # (bf16x3: p_fc2's weight gradient summed in the kernel; bf16: h1p / g2p row-major for the wgrad)
        assert eng.phead_p2 == (ph and not bf)
        xq = _fill_buffer(eng, model)
        idx = None if mb is None else torch.randperm(eng.N, generator=torch.Generator().manual_seed(5))[:mb]
        eng.begin_update()
        eng.grad(idx)
        torch.cuda.synchronize()
        res[ph] = (eng.grad_flat.clone(), eng.last_losses(), eng.mu_prev.clone())
        if ph:   # (no rollout wrote x^T: a full batch reads x_buf's rows)
            assert eng._x_mode == ("buf" if mb is None else "mb")
        if ph and loss == "ppo":
            ii = torch.arange(eng.N, device=DEV) if idx is None else idx.to(DEV)
            g_ref, _ = _torch_grad(model, p, xq, eng, ii)
            assert (eng.grad_flat - g_ref).norm().item() / g_ref.norm().item() < (6e-2 if bf else 2e-4)
            for name in ("p_fc1", "p_fc2", "mu"):
                for part in ("weight", "bias"):
                    o, n = model.offsets[f"{name}.{part}"]
                    gr, gk = g_ref[o:o + n], eng.grad_flat[o:o + n]
                    assert (gk - gr).norm().item() <= (1e-1 if bf else 6e-4) * (gr.norm().item() + 1e-8), (name, part)
            o, n = model.offsets["log_std"]
            assert (eng.grad_flat[o:o + n] - g_ref[o:o + n]).norm().item() <= (
                (1e-1 if bf else 6e-4) * (g_ref[o:o + n].norm().item() + 1e-8))
    (g1, l1, mp1), (g0, l0, mp0) = res[True], res[False]
    assert torch.isfinite(g1).all()
    rel = (g1 - g0).norm().item() / g0.norm().item()
    assert rel < (2e-2 if bf else 2e-5), rel
    for k in ("loss_value", "loss_clip", "loss_ent"):
        assert abs(l1[k] - l0[k]) < (1e-2 if bf else 1e-5) * (1 + abs(l0[k])), (k, l1[k], l0[k])
    if loss == "dppo_ref":
        assert (mp1 - mp0).abs().max().item() <= (2e-2 if bf else 2e-5) * (1 + mp0.abs().max().item())


@pytest.mark.parametrize("env_name", ["Synthetic-64x8", "Ant-v2"])
def test_phead_gate_on_observation_width(env_name):
    """the 32x32 policy kernel's wgrad reads the observation operand as rows of
    the operand width (d0 rounded up to the 128-row wgrad tile), so x_buf's rows serve only when d0
    is a multiple of 128.  d0 = 96 (Synthetic-64x8) must fall back to the 16x16 policy head (it
    used to raise at construction), d0 = 128 (Ant-v2) takes the 32x32 kernel; both full-batch
    gradients match autograd at fp32 tolerance."""
    N = 256 * 16
    p = ppo_preset(device="gpu", env_name=env_name, num_envs=256, exploration_size=N, batch_size=N,
                   dtype="bf16x3", ent_coeff=0.01, update_kernels="heads")
    eng, model, _, _ = _engine(p)
    assert eng.heads and eng.phead == (eng.d0 % 128 == 0), (eng.d0, eng.phead)
    xq = _fill_buffer(eng, model)
    eng.begin_update()
    eng.grad(None)
    torch.cuda.synchronize()
    g_ref, _ = _torch_grad(model, p, xq, eng, torch.arange(eng.N, device=DEV))
    assert (eng.grad_flat - g_ref).norm().item() / g_ref.norm().item() < 2e-4


@pytest.mark.parametrize("dtype", ["bf16x3", "bf16"])
def test_wgrad_row_major_operands_match_fragment_major(dtype):
    """The wgrad reading the 32x32 policy head's row-major operands ([ldT][features]: g1p, and at bf16
    g2p / h1p; per-lane DMA into XOR-swizzled 128-byte-row images, ds_read_b64_tr_b16) gives the same
    slabs as the fragment-major copies of the same values (rm flag 0).  (p_fc1's observation operand
    stays x_buf's rows in both.)"""
    from pytorch_dppo_amd.models.actor_critic import fm_index
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=256, exploration_size=256 * 16,
                    batch_size=256 * 16, dtype=dtype, update_kernels="heads")
    eng, model, _, _ = _engine(p)
    assert eng.phead
    _fill_buffer(eng, model)
    eng.begin_update()
    eng.grad(None)
    torch.cuda.synchronize()
    assert eng._x_mode == "buf"
    b = eng.buckets[0]   # the policy layers' bucket (p_fc1 [, p_fc2])
    wg_x = list(eng.wg_x_full)
    eng.ext.wgrad(eng._wgrad_dt(), eng.wg_g, wg_x, eng.g_rows, eng.x_rows, eng.ldT, b["tasks"],
                  b["tasks_host"], b["slab"], *eng._q8_args(), eng.rm)
    slab_rm = b["slab"].clone()
    ops = [("g1pT", 0, "g")] + ([] if eng.phead_p2 else [("g2pT", 1, "g"), ("h1pT", 1, "x")])
    wg_g, rm = list(eng.wg_g), list(eng.rm)
    for name, li, side in ops:
        assert rm[li if side == "g" else 6 + li] == 1
        buf = getattr(eng, name)
        width = (eng.g_rows if side == "g" else eng.x_rows)[li]
        rows = eng.decode(buf).view(eng.ldT, width)             # [ldT][features]
        f = torch.arange(width, device=DEV).repeat_interleave(eng.ldT)
        c = torch.arange(eng.ldT, device=DEV).repeat(width)
        flat = torch.zeros(width * eng.ldT, device=DEV)
        flat[fm_index(f, c, eng.ldT)] = rows.t().reshape(-1)
        (wg_g if side == "g" else wg_x)[li] = eng.encode(flat).view_as(buf)
        rm[li if side == "g" else 6 + li] = 0
    b["slab"].zero_()
    eng.ext.wgrad(eng._wgrad_dt(), wg_g, wg_x, eng.g_rows, eng.x_rows, eng.ldT, b["tasks"],
                  b["tasks_host"], b["slab"], *eng._q8_args(), rm)
    slab_fm = b["slab"]
    # (the fragment-major copies are re-encoded from the decoded fp32 rows: a split-bf16 value can
    # re-split with its lo part one rounding step off, so the slabs agree to that rounding)
    if dtype == "bf16":
        assert torch.equal(slab_rm, slab_fm)
    else:
        assert (slab_rm - slab_fm).abs().max().item() <= 2e-5 * slab_fm.abs().max().item() + 1e-6


def _torch_rollout(params, model, seed_state_from):
    from pytorch_dppo_amd.runtime.engine_torch import TorchEngine
    spec = get_spec(params.env_name)
    env = make_vec_env(spec, params.num_envs, seed=params.seed, device=DEV)
    stats = RunningObsStats(spec.obs_dim, DEV)
    stats.copy_from(seed_state_from)
    eng = TorchEngine(params, model, env, stats, DEV, 0)
    return eng


@pytest.mark.parametrize("env_name,dtype", [("Pendulum-v0", "fp32"), ("HalfCheetah-v2", "fp32"), ("Humanoid-v2", "fp32"),
                                            ("Pendulum-v0", "bf16x3"), ("HalfCheetah-v2", "bf16x3"),
                                            ("Humanoid-v2", "bf16x3")])
def test_rollout_matches_torch_engine(env_name, dtype):
    p = dppo_preset(device="gpu", env_name=env_name, num_envs=45, exploration_size=45 * 8,
                    batch_size=45 * 8, dtype=dtype)
    eng, model, env, stats = _engine(p)
    stats.observes(env.observe())
    with torch.no_grad():
        model.flat.data[:model.num_outputs] = -0.3
    eng.params_changed()
    p_cpu = Params.from_dict({**p.to_dict(), "device": "cpu"})
    ref = _torch_rollout(p_cpu, model, stats)
    ro_h = eng.rollout()
    ro_t = ref.rollout()
    T, E = eng.T, eng.E
    O = model.num_inputs
    assert torch.allclose(eng.actions.view(T, E, -1), ref.actions, atol=2e-4, rtol=1e-4)
    assert torch.allclose(eng.logp.view(T, E), ref.logp, atol=1e-4, rtol=1e-5)
    assert torch.allclose(eng.rewards.view(T, E), ref.rewards, atol=2e-4, rtol=1e-4)
    assert torch.equal(eng.dones.view(T, E), ref.dones)
    xk = eng.decode(eng.x_buf).view(T + 1, E, -1)[..., :O]
    assert torch.allclose(xk, ref.x, atol=2e-4, rtol=1e-4)
    assert torch.allclose(env.state, ref.env.state, atol=2e-4, rtol=1e-4)
    assert torch.allclose(ro_h["s1"], ro_t["s1"], rtol=1e-4, atol=1e-2)
    # sum of squares of the moment partials too (a bug there only shows via the variance)
    s2_scale = ro_t["s2"].abs().max().item() + 1.0
    assert torch.allclose(ro_h["s2"], ro_t["s2"], rtol=1e-4, atol=1e-4 * s2_scale)
    assert abs(ro_h["ep_count"] - ro_t["ep_count"]) < 0.5


@pytest.mark.parametrize("env_name,dtype", [("HalfCheetah-v2", "fp32"), ("Humanoid-v2", "bf16x3")])
def test_rollout_step_obs_norm_matches_torch_engine(env_name, dtype):
    """obs_norm_update='step' (model.py:68: the running stats absorb every observation before
    it is normalised): T single-step kernel launches against a per-rollout copy of the stats,
    vs the torch engine's per-step loop (no GPU test)."""
    p = dppo_preset(device="gpu", env_name=env_name, num_envs=45, exploration_size=45 * 8,
                    batch_size=45 * 8, dtype=dtype, obs_norm_update="step")
    eng, model, env, stats = _engine(p)
    stats.observes(env.observe())
    eng.params_changed()
    p_cpu = Params.from_dict({**p.to_dict(), "device": "cpu"})
    ref = _torch_rollout(p_cpu, model, stats)
    ro_h = eng.rollout()
    ro_t = ref.rollout()
    T, E, O = eng.T, eng.E, model.num_inputs
    assert torch.allclose(eng.actions.view(T, E, -1), ref.actions, atol=2e-4, rtol=1e-4)
    assert torch.allclose(eng.logp.view(T, E), ref.logp, atol=1e-4, rtol=1e-5)
    assert torch.equal(eng.dones.view(T, E), ref.dones)
    xk = eng.decode(eng.x_buf).view(T + 1, E, -1)[..., :O]
    assert torch.allclose(xk, ref.x, atol=2e-4, rtol=1e-4)
    # the per-rollout stats copy absorbed all T*E observations, like the torch engine's
    assert eng.local_stats.n == pytest.approx(ref.local_stats.n)
    assert torch.allclose(eng.local_stats.mean, ref.local_stats.mean, rtol=1e-6, atol=1e-6)
    assert torch.allclose(ro_h["s1"], ro_t["s1"], rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("E", [45, 4096])
def test_stepnorm_single_launch_matches_per_step_launches(E):
    """obs_norm_update='step' as ONE cooperative rollout launch (csrc/rollout.hip sn_step: each
    step's moments and merged stats exchanged between the workgroups as tagged granules) == the
    per-step launch sequence (observe + one-step rollout per step), up to the fp32 partial-sum
    order; at the bench geometry (4,096 envs, 256 workgroups) it is also timed (VERDICT r3 #6:
    <= 0.45 ms vs 1.21 ms)."""
    import time
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * 16,
                    batch_size=E * 16, dtype="bf16x3", obs_norm_update="step")
    res = {}
    for coop in (True, False):
        eng, model, env, stats = _engine(p)
        stats.observes(env.observe())
        eng.params_changed()
        if not coop:
            eng._sn_cap = 0
        assert eng._stepnorm_fits() == coop
        ro = eng.rollout()
        torch.cuda.synchronize()
        out = (eng.decode(eng.x_buf).clone(), eng.actions.clone(), eng.logp.clone(), eng.local_stats.mean.clone(),
               eng.local_stats.mean_diff.clone(), eng.local_stats.inv_std_f32.clone(), ro["s1"].clone(),
               ro["ep_count"].item(), eng.local_stats.n)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.rollout()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        res[coop] = (out, sorted(ts)[2])
        if coop:
            assert int(eng._sn_bufs[2].item()) == 0          # no hand-off timed out
    (a, ta), (b, tb) = res[True], res[False]
    print(f"step-norm rollout E={E}: one launch {ta:.3f} ms, per-step launches {tb:.3f} ms")
    assert a[8] == b[8]
    assert torch.allclose(a[3], b[3], rtol=1e-7, atol=1e-7)     # running mean (fp64)
    assert torch.allclose(a[4], b[4], rtol=1e-5)                # M2
    assert torch.allclose(a[5], b[5], rtol=1e-5)
    assert torch.allclose(a[0], b[0], atol=2e-4, rtol=1e-4)      # normalised rows
    assert torch.allclose(a[1], b[1], atol=2e-4, rtol=1e-4)      # actions
    assert torch.allclose(a[2], b[2], atol=1e-3, rtol=1e-4)
    assert torch.allclose(a[6], b[6], rtol=1e-4, atol=1e-2)
    assert a[7] == b[7]


@pytest.mark.parametrize("O,nblk,alias", [(37, 19, False), (376, 259, True)])
def test_obs_reduce_and_merge_kernels_match_torch_welford(O, nblk, alias):
    """O=37/19 blocks: two column groups, one ragged, tail loop only.  O=376/259 blocks:
    the 4-rows-in-flight loop of obs_reduce plus an uneven remainder and the episode-stat block's
    strided loop past 64 blocks; and obs_merge with shift ALIASING mean_f32, as the engine calls it
    (the kernel must read shift[d] before it writes mean_f32[d])."""
    ext = _ext()
    g = torch.Generator(device="cpu").manual_seed(4)
    ref = RunningObsStats(O, DEV)
    dev_st = RunningObsStats(O, DEV)
    for it in range(3):
        x = (torch.randn(nblk * 8, O, generator=g) * 3 + 10 * it).to(DEV)
        shift = ref.shift().clone()
        c, s1, s2 = RunningObsStats.moments(x, shift)
        ref.merge_moments(c, s1, s2, shift)
        # partials per block as the rollout kernel leaves them
        d = (x - dev_st.shift()).view(nblk, 8, O)
        part = torch.stack([d.sum(1), (d * d).sum(1)], 1).float().contiguous()
        s12 = torch.zeros(2, O, dtype=torch.float64, device=DEV)
        epstat = torch.rand(nblk, 2, generator=g).to(DEV)
        ep = torch.zeros(2, dtype=torch.float64, device=DEV)
        ext.obs_reduce(part, nblk, O, s12, epstat, ep)
        assert torch.allclose(s12[0], s1, rtol=1e-5, atol=1e-3)
        assert torch.allclose(s12[1], s2, rtol=1e-5, atol=1e-2)
        assert torch.allclose(ep, epstat.double().sum(0), rtol=1e-12)
        sh = dev_st.shift() if alias else dev_st.shift().clone()
        if alias:
            assert sh.data_ptr() == dev_st.mean_f32.data_ptr()
        ext.obs_merge(s12, float(nblk * 8), float(dev_st.n), sh, dev_st.mean, dev_st.mean_diff,
                      dev_st.mean_f32, dev_st.inv_std_f32, 1e-2)
        dev_st.n += nblk * 8
    assert torch.allclose(dev_st.mean, ref.mean, rtol=1e-5, atol=1e-4)
    assert torch.allclose(dev_st.mean_diff, ref.mean_diff, rtol=1e-4)
    assert torch.allclose(dev_st.inv_std_f32, ref.inv_std_f32, rtol=1e-4)


@pytest.mark.parametrize("E,O", [(4096, 376), (1031, 37), (45, 17)])
def test_obs_observe_matches_running_stats(E, O):
    """obs_observe (the per-step obs-norm mode's observe: moments -> reduce -> merge, three
    launches) over several steps' batches with drifting means, vs RunningObsStats.observes (fp64
    torch); E = 4096 / 1031: many 64-row moment blocks, one ragged."""
    ext = _ext()
    g = torch.Generator(device="cpu").manual_seed(E + O)
    ref = RunningObsStats(O, DEV)
    st = RunningObsStats(O, DEV)
    shift = st.shift().clone()          # the iteration's snapshot, fixed across the steps
    nb = int(ext.obs_moments_nblk(E))
    assert nb == -(-E // 64)
    part = torch.zeros(nb, 2, O, device=DEV)
    s12 = torch.zeros(2, O, dtype=torch.float64, device=DEV)
    for t in range(4):
        x = (torch.randn(E, O, generator=g) * (1 + t) + 3 * t).to(DEV)
        ref.observes(x)
        ext.obs_observe(x, shift, st.mean, st.mean_diff, st.mean_f32, st.inv_std_f32, float(st.n), part, s12, 1e-2)
        st.n += E
    assert torch.allclose(st.mean, ref.mean, rtol=1e-5, atol=1e-4)
    assert torch.allclose(st.mean_diff, ref.mean_diff, rtol=1e-4)
    assert torch.allclose(st.inv_std_f32, ref.inv_std_f32, rtol=1e-4)
    with pytest.raises(RuntimeError):   # the shift must not alias the stats being merged into
        ext.obs_observe(x, st.mean_f32, st.mean, st.mean_diff, st.mean_f32, st.inv_std_f32, float(st.n), part, s12,
                        1e-2)


@pytest.mark.parametrize("T,E,mode,seg", [(33, 1031, 0, 0), (33, 1031, 1, 0), (2048, 1, 0, 0), (2048, 3, 2, 0),
                                          (1000, 5, 2, 0), (7, 2, 2, 0), (33, 1031, 1, 5), (1000, 5, 2, 64),
                                          (2048, 3, 2, 100), (40, 257, 1, 7)])
def test_gae_kernel_matches_oracle(T, E, mode, seg):
    """mode 1 = per-env lanes, 2 = parallel-in-time scan (auto picks it for 2048 x 1), ragged chunks included."""
    ext = _ext()
    g = torch.Generator(device="cpu").manual_seed(T * 7 + E)
    r = torch.randn(T, E, generator=g).to(DEV)
    v = torch.randn(T + 1, E, generator=g).to(DEV)
    d = (torch.rand(T, E, generator=g) < 0.05).float().to(DEV)
    adv = torch.empty(T, E, device=DEV)
    ret = torch.empty(T, E, device=DEV)
    ext.gae(r, v, d, adv, ret, 0.99, 0.95, mode, seg)
    a_ref, r_ref = oracle.gae(r.double(), v.double(), d.double(), 0.99, 0.95, segment=seg)
    assert torch.allclose(adv.double(), a_ref, atol=2e-5, rtol=2e-5)
    assert torch.allclose(ret.double(), r_ref, atol=2e-5, rtol=2e-5)


def _fill_buffer(eng, model, gen_seed=3):
    g = torch.Generator(device="cpu").manual_seed(gen_seed)
    N, O, A = eng.N, model.num_inputs, model.num_outputs
    x = torch.randn(N + eng.E, O, generator=g).clamp(-5, 5).to(DEV)
    xb = torch.zeros(N + eng.E, eng.d0, device=DEV)
    xb[:, :O] = x
    xb[:, O] = 1.0
    eng.x_buf.copy_(eng.encode(xb))
    xq = eng.decode(eng.x_buf)[:N, :O]
    with torch.no_grad():
        mu, ls, v = model(xq)
    a = (mu + 0.6 * torch.randn(N, A, generator=g).to(DEV))
    eng.actions.copy_(a)
    sig = torch.exp(ls if eng.p.std_convention == "std" else 0.5 * ls)
    logp_old = oracle.gaussian_logp(a, mu + 0.05 * torch.randn(N, A, generator=g).to(DEV), ls, eng.p.std_convention)
    eng.logp.copy_(logp_old.reshape(-1))
    eng.adv.copy_(torch.randn(N, generator=g).to(DEV))
    eng.ret.copy_((v.reshape(-1) + 0.5 * torch.randn(N, generator=g).to(DEV)))
    eng.values_buf[:N].copy_(v.reshape(-1) + 0.3 * torch.randn(N, generator=g).to(DEV))
    return xq


def _torch_grad(model, p, xq, eng, idx):
    x = xq[idx]
    model.flat.grad = None
    mu, ls, v = model(x)
    out = oracle.ppo_loss(mu, ls, v, eng.actions[idx], eng.logp[idx], eng.adv[idx], eng.ret[idx],
                          eng.values_buf[:eng.N][idx], clip=p.clip, ent_coeff=p.ent_coeff,
                          value_loss=p.value_loss, convention=p.std_convention)
    out["loss"].backward()
    return model.flat.grad.detach().clone(), out


@pytest.mark.parametrize("env_name,dtype,value_loss,conv,mb,tol", [
    ("HalfCheetah-v2", "fp32", "mse", "std", 256, 1e-4),
    ("HalfCheetah-v2", "fp32", "clipped_half", "var", 200, 1e-4),
    ("Humanoid-v2", "fp32", "clipped_half", "std", 512, 2e-4),
    ("Humanoid-v2", "bf16", "mse", "std", 512, 6e-2),
    ("Pendulum-v0", "fp32", "mse", "std", 64, 1e-4),
    ("HalfCheetah-v2", "bf16x3", "mse", "std", 256, 1e-4),
    ("HalfCheetah-v2", "bf16x3", "clipped_half", "var", 200, 1e-4),
    ("Humanoid-v2", "bf16x3", "clipped_half", "std", 512, 2e-4),
    ("Pendulum-v0", "bf16x3", "mse", "std", 64, 1e-4),
])
def test_fused_loss_backward_matches_autograd(env_name, dtype, value_loss, conv, mb, tol):
    p = ppo_preset(device="gpu", env_name=env_name, num_envs=64, exploration_size=64 * 8,
                   batch_size=mb, dtype=dtype, value_loss=value_loss, std_convention=conv, ent_coeff=0.01)
    eng, model, _, _ = _engine(p)
    with torch.no_grad():
        model.flat.data[:model.num_outputs] = torch.linspace(-0.4, 0.2, model.num_outputs, device=DEV)
    eng.params_changed()
    xq = _fill_buffer(eng, model)
    idx = torch.randperm(eng.N, generator=torch.Generator().manual_seed(5))[:mb]
    eng.begin_update()
    eng.grad(idx)
    g_ref, out = _torch_grad(model, p, xq, eng, idx.to(DEV))
    g = eng.grad_flat
    rel = (g - g_ref).norm().item() / (g_ref.norm().item() + 1e-12)
    assert rel < tol, rel
    ll = eng.last_losses()
    assert abs(ll["loss_clip"] - out["loss_clip"].item()) < max(5e-3, 50 * tol) * (1 + abs(out["loss_clip"].item()))
    assert abs(ll["loss_value"] - out["loss_value"].item()) < max(5e-3, 50 * tol) * (1 + abs(out["loss_value"].item()))


@pytest.mark.parametrize("rows", [32, 64])
@pytest.mark.parametrize("env_name,mb", [("Humanoid-v2", 200), ("HalfCheetah-v2", 320)])
def test_fused_loss_backward_row_tiles(rows, env_name, mb, monkeypatch):
    """bf16 one-kernel tile update (csrc/mlp.hip; update_kernels=tile) at both row tiles (64 rows / 8
    waves and 32 rows / 4 waves), with a ragged last tile, vs autograd; and the value kernel at
    both tiles."""
    ext = _ext()
    p = ppo_preset(device="gpu", env_name=env_name, num_envs=64, exploration_size=64 * 8,
                   batch_size=mb, dtype="bf16", ent_coeff=0.01, update_kernels="tile")
    ext.set_mlp_rows(rows)
    try:
        eng, model, _, _ = _engine(p)
        assert eng.train_rows == rows
        xq = _fill_buffer(eng, model)
        idx = torch.randperm(eng.N, generator=torch.Generator().manual_seed(7))[:mb]
        eng.begin_update()
        eng.grad(idx)
        g_ref, _ = _torch_grad(model, p, xq, eng, idx.to(DEV))
        rel = (eng.grad_flat - g_ref).norm().item() / (g_ref.norm().item() + 1e-12)
        assert rel < 6e-2, rel
        eng.values()
        with torch.no_grad():
            _, _, v = model(eng.decode(eng.x_buf)[:, :model.num_inputs])
        err = (eng.values_buf - v.reshape(-1)).abs().max().item()
        assert err / (v.abs().max().item() + 1e-3) < 3e-2, err
    finally:
        ext.set_mlp_rows(0)


def test_s3_other_hidden_sizes_fall_back_to_tile_kernel():
    """the per-head kernels are specialised for the reference network's tile counts; any other
    hidden sizes run the 32-row tile kernel, still at fp32 accuracy"""
    p = ppo_preset(device="gpu", env_name="HalfCheetah-v2", num_envs=64, exploration_size=64 * 8,
                   batch_size=256, dtype="bf16x3", ent_coeff=0.01, hidden=(64, 48))
    eng, model, _, _ = _engine(p)
    assert eng.train_rows == 32
    xq = _fill_buffer(eng, model)
    idx = torch.randperm(eng.N, generator=torch.Generator().manual_seed(3))[:256]
    eng.begin_update()
    eng.grad(idx)
    g_ref, _ = _torch_grad(model, p, xq, eng, idx.to(DEV))
    assert (eng.grad_flat - g_ref).norm().item() / g_ref.norm().item() < 1e-4


@pytest.mark.parametrize("dtype", ["bf16", "bf16x3"])
def test_rollout_written_xT_equals_kernel_written_xT(dtype):
    """full-batch: the x^T operand the rollout emits == the one mlp_train would transpose."""
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=64, exploration_size=64 * 4,
                    batch_size=64 * 4, dtype=dtype)
    eng, model, env, stats = _engine(p)
    stats.observes(env.observe())
    assert eng.xT_from_rollout
    eng.rollout()
    eng.values()
    eng.gae()
    eng.begin_update()
    assert eng._xT_valid
    xT_roll = eng.xT.clone()
    eng.grad(None)
    g_roll = eng.grad_flat.clone()
    eng._xT_valid = False            # force the fused kernel to write x^T itself
    eng.xT.zero_()
    eng.grad(None)
    # split-bf16: equal VALUES (hi + lo); the (hi, lo) bits may differ where a lo of -0.0 / a
    # flushed denormal was re-split from the sum (the streaming kernel re-splits hi + lo)
    assert torch.equal(eng.decode(eng.xT), eng.decode(xT_roll))
    if dtype == "bf16":
        assert torch.equal(eng.grad_flat, g_roll)
    else:
        assert (eng.grad_flat - g_roll).norm().item() <= 1e-6 * g_roll.norm().item()


@pytest.mark.parametrize("dtype", ["fp32", "bf16x3"])
def test_dppo_ref_loss_two_steps_matches_autograd(dtype):
    p = dppo_preset(device="gpu", env_name="HalfCheetah-v2", num_envs=32, exploration_size=256,
                    batch_size=256, dtype=dtype, loss="dppo_ref", ent_coeff=0.01)
    eng, model, _, _ = _engine(p)
    xq = _fill_buffer(eng, model)
    eng.begin_update()
    old_flat = model.flat.data.clone()
    eng.grad(None)
    # step 1: old == current
    x = xq
    model.flat.grad = None
    mu, ls, v = model(x)
    out = oracle.dppo_ref_loss(mu, ls, v, mu.detach(), ls.detach(), v.detach(), eng.actions, eng.adv, eng.ret,
                               clip=p.clip, ent_coeff=p.ent_coeff)
    out["loss"].backward()
    rel = (eng.grad_flat - model.flat.grad).norm() / model.flat.grad.norm()
    assert rel < 1e-4
    eng.apply()
    # step 2: old = params of step 1
    eng.grad(None)
    model.flat.grad = None
    mu, ls, v = model(x)
    from pytorch_dppo_amd.runtime.engine_torch import _forward_with
    with torch.no_grad():
        mu_o, ls_o, v_o = _forward_with(model, old_flat, x)
    out = oracle.dppo_ref_loss(mu, ls, v, mu_o, ls_o, v_o, eng.actions, eng.adv, eng.ret,
                               clip=p.clip, ent_coeff=p.ent_coeff)
    out["loss"].backward()
    rel = (eng.grad_flat - model.flat.grad).norm() / model.flat.grad.norm()
    assert rel < 2e-4


@pytest.mark.parametrize("max_norm", [0.0, 0.5])
def test_adam_kernel_matches_oracle(max_norm):
    p = ppo_preset(device="gpu", env_name="HalfCheetah-v2", num_envs=16, exploration_size=128,
                   batch_size=128, dtype="fp32", max_grad_norm=max_norm or None)
    eng, model, _, _ = _engine(p)
    n = model.num_params
    p_ref = model.flat.data.clone()
    m_ref = torch.zeros(n, device=DEV)
    v_ref = torch.zeros(n, device=DEV)
    for step in range(1, 4):
        g = torch.randn(n, device=DEV) * 0.3
        eng.grad_flat.copy_(g)
        eng.apply()
        # step counter committed by the last block; the clip path also reports the pre-clip norm
        assert float(eng.adam_state[0]) == step and float(eng.adam_state[3]) == 0.0
        if max_norm:
            assert abs(float(eng.adam_state[2]) - g.norm().item()) <= 1e-4 * g.norm().item()
        gr = g.clone()
        if max_norm:
            oracle.clip_grad_norm_(gr, max_norm)
        oracle.adam_step_(p_ref, gr, m_ref, v_ref, step, p.lr, p.adam_betas, p.adam_eps)
    assert torch.allclose(model.flat.data, p_ref, atol=1e-6, rtol=1e-5)
    ref_img = storage.encode(model.packed_layout().pack(model.flat.data), eng.dt)
    assert torch.equal(eng.wimg, ref_img)


def test_engine_iteration_matches_torch_engine_fp32():
    """Full iteration (rollout -> values -> GAE -> 2 full-batch steps) HIP vs torch oracle."""
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    common = dict(env_name="HalfCheetah-v2", num_envs=48, exploration_size=48 * 6, batch_size=48 * 6,
                  num_epoch=2, dtype="fp32", max_iters=1)
    pg = dppo_preset(device="gpu", **common)
    pc = dppo_preset(device="cpu", **common)
    wg = DPPOWorker(pg, DistContext(device=DEV))
    wc = DPPOWorker(pc, DistContext(device=torch.device("cpu")))
    assert torch.equal(wg.model.flat.data.cpu(), wc.model.flat.data)
    mg = wg.iteration_step()
    mc = wc.iteration_step()
    d = (wg.model.flat.data.cpu() - wc.model.flat.data).abs()
    # Adam moves every element by ~lr per step whatever the gradient magnitude, so elements
    # whose true gradient is ~0 may legitimately differ by up to 2*lr*steps; the bulk must agree.
    assert d.max().item() <= 2 * pg.lr * pg.num_epoch + 1e-6
    assert (d > 1e-5).float().mean().item() < 0.01
    assert abs(mg["loss_value"] - mc["loss_value"]) < 1e-3 * (1 + abs(mc["loss_value"]))


def test_fp8_rollout_tracks_fp32_and_engine_trains():
    """fp8 e4m3 forward GEMMs (rollout policy + value): actions close to the fp32 path for the same
    noise; a full fp8 iteration (bf16 update) stays finite and the fp8 scales follow amax."""
    common = dict(device="gpu", env_name="Humanoid-v2", num_envs=64, exploration_size=64 * 4, batch_size=64 * 4,
                  num_epoch=2)
    e32, m32, env32, st32 = _engine(dppo_preset(dtype="fp32", **common))
    e8, m8, env8, st8 = _engine(dppo_preset(dtype="fp8", **common))
    assert torch.equal(m32.flat.data, m8.flat.data)
    for st, env in ((st32, env32), (st8, env8)):
        st.observes(env.observe())
    e32.rollout()
    e8.rollout()
    mu_err = (e8.actions - e32.actions).abs()
    assert mu_err.mean().item() < 0.05, mu_err.mean().item()
    amax = torch.stack([m8.view(f"{n}.weight").abs().amax() for n in ("p_fc1", "p_fc2", "mu", "v_fc1", "v_fc2", "v")])
    assert torch.all(e8.qscale * 416.0 >= amax * (1 - 1e-6))
    e8.values()
    e8.gae()
    e8.begin_update()
    e8.grad(None)
    e8.apply()
    assert torch.isfinite(m8.flat.data).all() and torch.isfinite(e8.values_buf).all()


def test_rccl_world1_allreduce_and_training_step():
    """The real RCCL collective path at world size 1 (the 1-GPU box): grads, obs moments."""
    from pytorch_dppo_amd.parallel.dist import init_single_rank_collective
    from pytorch_dppo_amd.runtime.launcher import free_port
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    ctx = init_single_rank_collective(DEV, port=free_port())
    ctx.force_collectives = True      # the identity sum still goes through RCCL
    try:
        g = torch.arange(1000, device=DEV, dtype=torch.float32)
        ctx.allreduce_grads(g)
        assert torch.equal(g, torch.arange(1000, device=DEV, dtype=torch.float32))
        p = dppo_preset(device="gpu", env_name="Walker2d-v2", num_envs=64, exploration_size=64 * 4,
                        batch_size=128, num_epoch=2, dtype="bf16", verify_sync_every=1)
        w = DPPOWorker(p, ctx)
        m = w.iteration_step()
        assert m["replicas_in_sync"] is True
        assert math.isfinite(m["loss"]) and m["updates"] == 4
        # the episode [return sum, count] rode on the moments' RCCL all-reduce (identity at
        # world 1): the packed metrics hold exactly the rollout's sums
        m = w.iteration_step()
        ep = w.engine.ep_sum.tolist()
        assert torch.equal(w.engine.metrics_buf[:2], w.engine.ep_sum)
        assert m["ep_count"] == ep[1]
        if ep[1] > 0:
            assert m["mean_ep_return"] == pytest.approx(ep[0] / ep[1])
        assert ctx.native is not None          # the worker made the in-stream communicator
    finally:
        ctx.destroy()


def test_native_comm_failure_falls_back_to_process_group(monkeypatch):
    """A rank whose native RCCL communicator cannot be created (here: comm_init raises) makes
    every rank fall back to the process group's collectives (one MIN all-reduce of the outcome):
    the worker trains through ProcessGroupNCCL instead of failing or hanging a 2-path world."""
    from pytorch_dppo_amd.parallel.dist import init_single_rank_collective
    from pytorch_dppo_amd.runtime.launcher import free_port
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    ext = _ext()

    class Broken:
        def __getattr__(self, k):
            if k == "comm_init":
                def fail(*a):
                    raise RuntimeError("RCCL ncclCommInitRank failed: test")
                return fail
            return getattr(ext, k)
    ctx = init_single_rank_collective(DEV, port=free_port())
    ctx.force_collectives = True
    try:
        assert ctx.init_native_comm(Broken()) is False and ctx.native is None
        p = dppo_preset(device="gpu", env_name="Walker2d-v2", num_envs=64, exploration_size=64 * 4,
                        batch_size=128, num_epoch=2, dtype="bf16")
        ctx.grad_comm = "process_group"     # (the worker's own attempt would succeed)
        w = DPPOWorker(p, ctx)
        assert ctx.native is None
        m = w.iteration_step()
        assert math.isfinite(m["loss"]) and m["updates"] == 4
    finally:
        ctx.destroy()


@pytest.mark.parametrize("overlap", [False, True, "every"])
@pytest.mark.parametrize("native", [False, True])
def test_head_chains_through_rccl_bit_identical_to_fused(overlap, native, monkeypatch):
    """The collective paths through the real RCCL call at world size 1.  Process-group RCCL
    (grad_comm=process_group): per-head chains (policy all-reduce issued before the value kernel,
    value all-reduce + Adam left pending into the next step — and with --overlap-rollout past the
    next rollout) == the same chains without collectives (fused_apply=False), bit-identical after
    2 iterations, and == the joint world-size-1 path (one wgrad + one gather/Adam) to fp32
    summation-order tolerance.  Native in-stream RCCL (csrc/comm.cpp): the joint kernels, the
    gather, the all-reduce and the whole-vector Adam == the joint world-size-1 path, bit for bit;
    with --overlap-rollout the last step's value all-reduce + Adam on the side stream (second
    communicator) beside the next rollout, still bit for bit; with overlap_value_epochs ("every")
    every epoch's value all-reduce + Adam on the side stream, joined before the next value kernel
    (the policy Adam and the next policy kernel run beside it), bit for bit."""
    from pytorch_dppo_amd.parallel.dist import DistContext, init_single_rank_collective
    from pytorch_dppo_amd.runtime.launcher import free_port
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    if overlap == "every" and not native:
        pytest.skip("the process-group chains overlap every value step already")
    gc = "native" if native else "process_group"
    kw = dict(device="gpu", env_name="Humanoid-v2", num_envs=64, exploration_size=64 * 8, batch_size=64 * 8,
              num_epoch=3, dtype="bf16x3", seed=3, overlap_rollout=overlap is True,
              overlap_value_epochs=overlap == "every", update_kernels="heads", grad_comm=gc)
    wj = DPPOWorker(dppo_preset(**kw), DistContext(device=DEV))     # joint world-1 path
    for _ in range(2):
        wj.iteration_step()
    ref = wj
    if not native:
        w1 = DPPOWorker(dppo_preset(**kw, fused_apply=False), DistContext(device=DEV))
        assert w1.engine.heads and len(w1.engine.buckets) == 2 and not w1.engine.can_fuse_apply()
        for _ in range(2):
            w1.iteration_step()
        w1.flush_pending()
        torch.cuda.synchronize()
        rel = (w1.model.flat.data - wj.model.flat.data).norm() / wj.model.flat.data.norm()
        assert rel.item() < 1e-5, rel.item()
        ref = w1
    ctx = init_single_rank_collective(DEV, port=free_port(), grad_comm=gc)
    ctx.force_collectives = True
    try:
        w2 = DPPOWorker(dppo_preset(**kw), ctx)
        assert (ctx.native is not None) == native
        assert (ctx.native_side is not None) == (native and bool(overlap))
        for _ in range(2):
            m = w2.iteration_step()
        if overlap == "every":
            assert w2.engine.side_steps == 6    # every step of the 2 iterations x 3 epochs
        elif overlap:
            # the last value step waits for the rollout: on the side stream (native) or as the
            # process group's pending work
            assert w2.engine._pending_value is not None
            assert w2.engine._pending_value[0] == ("side" if native else "work")
            w2.flush_pending()
        assert w2.engine._pending_value is None
        torch.cuda.synchronize()
        assert torch.equal(ref.model.flat.data, w2.model.flat.data)
        assert torch.equal(ref.engine.adam_v, w2.engine.adam_v)
        assert math.isfinite(m["loss"]) and m["updates"] == 6
    finally:
        ctx.destroy()


@pytest.mark.parametrize("env_name,mb,dtype", [("Humanoid-v2", 512, "bf16x3"), ("Humanoid-v2", 200, "bf16x3"),
                                               ("HalfCheetah-v2", 256, "bf16x3"), ("Pendulum-v0", 64, "bf16x3"),
                                               ("Humanoid-v2", 512, "bf16"), ("HalfCheetah-v2", 200, "bf16")])
@pytest.mark.parametrize("loss", ["ppo", "dppo_ref"])
def test_head_kernels_match_one_kernel_update(env_name, mb, dtype, loss, monkeypatch):
    """split-bf16: the per-head streaming kernels (csrc/mlp_head.hip, 128 rows per workgroup,
    policy and value chains separately) vs the one-kernel 32-row tile update (csrc/mlp.hip,
    update_kernels=tile) on the
    same minibatch — gradient, loss sums and the wgrad operands both write (idx gather, ragged last
    tile, the in-kernel X^T path) — and vs autograd.  bf16: both kernels round the same fp32 values
    to bf16 operands, but their fp32 sums run in different orders, so a value next to a rounding
    boundary can round differently: relative budgets instead of the split-bf16 ones."""
    from pytorch_dppo_amd.models.actor_critic import fm_index
    kw = dict(device="gpu", env_name=env_name, num_envs=64, exploration_size=64 * 8, batch_size=mb,
              dtype=dtype, ent_coeff=0.01, loss=loss)
    bf = dtype == "bf16"
    p = ppo_preset(**kw) if loss == "ppo" else dppo_preset(**kw)
    res = {}
    for heads in ("1", "0"):
        p.update_kernels = "heads" if heads == "1" else "tile"
        eng, model, _, _ = _engine(p)
        assert eng.heads == (heads == "1")
        xq = _fill_buffer(eng, model)
        idx = torch.randperm(eng.N, generator=torch.Generator().manual_seed(11))[:mb]
        eng.begin_update()
        eng.grad(idx)
        n1p, n1v = model.layer("p_fc1").fan_out, model.layer("v_fc1").fan_out

        def rowmajor(buf, nfeat, rm=False):   # FM [features][ldT] -> [features][mb]
            if rm:   # [ldT][width] rows (the 32x32 policy head's X rows)
                return eng.decode(buf).view(eng.ldT, -1)[:mb, :nfeat].t()
            r = torch.arange(nfeat, device=DEV).repeat_interleave(mb)
            c = torch.arange(mb, device=DEV).repeat(nfeat)
            return eng.decode(buf).reshape(-1)[fm_index(r, c, eng.ldT)].view(nfeat, mb)

        # (the 32x32 policy head: X rows row-major, h1p row-major or not stored — p_fc2's weight
        # gradient summed in the kernel — so both arms compare h1v instead)
        ph = bool(getattr(eng, "phead", False))
        if heads == "1":
            use_h1v = ph
        h1 = (rowmajor(eng.h1vT, model.layer("v_fc2").fan_in) if use_h1v
              else rowmajor(eng.h1pT, n1p))
        res[heads] = (eng.grad_flat.clone(), eng.last_losses(), h1,
                      rowmajor(eng.g1vT, n1v),
                      rowmajor(eng.xT, model.num_inputs, ph), eng.mu_prev.clone(), eng.v_prev.clone())
        if heads == "1" and loss == "ppo":
            g_ref, _ = _torch_grad(model, p, xq, eng, idx.to(DEV))
            assert (eng.grad_flat - g_ref).norm().item() / g_ref.norm().item() < (6e-2 if bf else 2e-4)
    g_h, l_h, h1_h, g1_h, x_h, mp_h, vp_h = res["1"]
    g_o, l_o, h1_o, g1_o, x_o, mp_o, vp_o = res["0"]
    rel = (g_h - g_o).norm().item() / (g_o.norm().item() + 1e-12)
    assert rel < (2e-2 if bf else 2e-5), rel
    for k in ("loss_clip", "loss_value", "loss_ent", "approx_kl", "clipfrac"):
        assert abs(l_h[k] - l_o[k]) < (1e-2 if bf else 1e-5) * (1 + abs(l_o[k])), (k, l_h[k], l_o[k])
    for a_, b_ in ((h1_h, h1_o), (g1_h, g1_o)):
        assert (a_ - b_).norm().item() <= (1e-2 if bf else 1e-5) * b_.norm().item()
    assert torch.equal(x_h, x_o)            # x^T is a copy of the observation rows
    if loss == "dppo_ref":                  # train.py:164 model_old <- model, per row (fp32 summation order differs)
        t = 2e-2 if bf else 2e-5
        assert (mp_h - mp_o).abs().max().item() <= t * (1 + mp_o.abs().max().item())
        assert (vp_h - vp_o).abs().max().item() <= t * (1 + vp_o.abs().max().item())
        assert bool((mp_h != 0).any()) and bool((vp_h != 0).any())


def test_deferred_metrics_match_synchronous():
    """iteration_step(defer=True) returns iteration i's metrics during iteration i+1; the values
    must equal the synchronous path's (same seed, same work)."""
    import math
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    common = dict(device="gpu", env_name="Hopper-v2", num_envs=64, exploration_size=512, batch_size=512,
                  num_epoch=2, dtype="bf16", seed=5)
    ws = DPPOWorker(dppo_preset(**common), DistContext(device=DEV))
    wd = DPPOWorker(dppo_preset(**common), DistContext(device=DEV))
    sync = [ws.iteration_step() for _ in range(3)]
    dfr = [wd.iteration_step(defer=True) for _ in range(3)] + [wd.finish_metrics()]
    assert dfr[0] == {}
    for a, b in zip(sync, dfr[1:]):
        assert a["iteration"] == b["iteration"] and a["env_steps"] == b["env_steps"]
        for k in ("loss", "loss_value", "grad_norm", "approx_kl", "ep_count"):
            assert a[k] == b[k], (k, a[k], b[k])
        assert (math.isnan(a["mean_ep_return"]) and math.isnan(b["mean_ep_return"])) or \
            a["mean_ep_return"] == b["mean_ep_return"]
        assert b["ms_update"] > 0 and b["steps_per_s"] > 0
    assert torch.equal(ws.model.flat.data, wd.model.flat.data)


@pytest.mark.parametrize("max_norm", [None, 0.5])
def test_packed_metrics_match_torch(max_norm):
    """One-launch metric staging (Adam's per-block sums of squares + loss sums + episode stats)
    == the torch reductions of the same device state."""
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    p = dppo_preset(device="gpu", env_name="Walker2d-v2", num_envs=64, exploration_size=64 * 4,
                    batch_size=64 * 4, num_epoch=2, dtype="bf16", max_grad_norm=max_norm)
    w = DPPOWorker(p, DistContext(device=DEV))
    m = w.iteration_step()
    eng = w.engine
    gn = torch.linalg.vector_norm(eng.grad_flat.double()).item()
    assert abs(m["grad_norm"] - gn) <= 1e-5 * max(gn, 1.0), (m["grad_norm"], gn)
    ls = eng.loss_sums.double()
    assert abs(m["loss_clip"] - (ls[0] / max(ls[5], 1)).item()) < 1e-9
    assert torch.equal(eng.metrics_buf[:2], eng.ep_sum)


@pytest.mark.parametrize("extra", [[], ["--overlap-rollout", "off"], ["--grad-comm", "process_group"],
                                   ["--overlap-value", "on"]])
def test_two_ranks_on_one_gpu_stay_in_sync(extra):
    """bench.py as 2 ranks sharing the box's GPU (RCCL refuses two ranks on one device, so
    --dist-backend gloo): by default the gloo adapter runs the PRODUCTION multi-rank branch (the
    in-stream one an N-GPU RCCL run takes: joint kernels → gather → all-reduce → whole-vector
    Adam, and — the world > 1 default, --overlap-rollout auto — the last epoch's value step on
    the side stream beside the next rollout; --overlap-value: every epoch's); the ranks must end
    with bit-identical parameters (--verify-sync).  2,048 envs x 16 steps = 32,768 rows per rank:
    the per-head path the bench geometry takes (>= 128 rows x the CUs), so the side-stream counts
    the JSON reports (from the engine, not the flags) are the head path's."""
    import os
    import subprocess
    import sys
    from pytorch_dppo_amd.runtime.launcher import free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--num-envs", "2048", "--verify-sync", "--variants", "bf16,fp8",
           "--dist-backend", "gloo"] + extra
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    for dt in ("bf16x3", "bf16", "fp8"):
        assert f"{dt} replicas_in_sync True" in r.stderr, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 2
    pg = "process_group" in extra
    assert d["config"]["grad_allreduce"] == ("process_group" if pg else "gloo_in_stream")
    assert ("grad_allreduce process_group" if pg else "grad_allreduce in_stream") in r.stderr
    assert d["config"]["per_head_kernels"] is True
    off = "off" in extra
    assert d["config"]["overlap_rollout"] is (not off)
    # value steps per iteration the engine overlapped: the last epoch's (overlap-rollout), every
    # epoch's (overlap-value, 10), the per-head process-group chains' pending ones (10), none
    n = d["config"]["overlapped_value_steps_per_iter"]
    if off:
        assert d["config"]["overlap_value_step"] == "none" and n == 0
    elif pg:
        assert d["config"]["overlap_value_step"] == "pending_work" and n == 10
    else:
        assert d["config"]["overlap_value_step"] == "side_stream"
        assert n == (10 if "--overlap-value" in extra else 1), n


def _two_rank_child(rank, world, port, out_dir):
    """one of 2 ranks sharing cuda:0 over gloo: (a) 2 iterations per (dtype, gradient comm,
    overlap) from the same seed → final parameters; (b) grad_reduce=mean on the tile and the
    per-head update → the local and the reduced gradient (the in-stream mean must not
    be scaled again)"""
    import os
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    from pytorch_dppo_amd.parallel.dist import DistContext, init_distributed
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    base = init_distributed("gpu", rank=rank, world_size=world, backend="gloo", timeout_s=120)
    out = {}

    def ctx_for(gc):
        return DistContext(rank=rank, world_size=world, local_rank=0, backend="gloo", device=base.device,
                           timeout_s=120, grad_comm=gc)
    common = dict(device="gpu", env_name="Humanoid-v2", num_envs=256, exploration_size=256 * 8,
                  batch_size=256 * 8, num_epoch=3, seed=3, num_processes=world, dist_backend="gloo",
                  verify_sync_every=1, update_kernels="heads")
    for dtype in ("bf16x3", "bf16", "fp8"):
        for gc, ov in (("auto", False), ("auto", True), ("auto", "every"), ("process_group", False)):
            ctx = ctx_for(gc)
            w = DPPOWorker(dppo_preset(**common, dtype=dtype, overlap_rollout=ov is True,
                                       overlap_value_epochs=ov == "every", grad_comm=gc), ctx)
            for _ in range(2):
                m = w.iteration_step()
            w.flush_pending()
            torch.cuda.synchronize()
            out[f"{dtype}/{gc}/{ov}"] = (w.model.flat.data.cpu(), bool(m["replicas_in_sync"]),
                                         ctx.native is not None, ctx.native_side is not None)
    for dtype, uk in (("fp32", "tile"), ("bf16x3", "heads")):
        for gc in ("auto", "process_group"):
            ctx = ctx_for(gc)
            w = DPPOWorker(dppo_preset(**{**common, "update_kernels": uk}, dtype=dtype, grad_comm=gc,
                                       grad_reduce="mean"), ctx)
            eng = w.engine
            assert eng.heads == (uk == "heads")
            w.init_stats()
            ro = eng.rollout()
            w._merge_stats(ro["count"], ro["s1"], ro["s2"], ro["shift"])
            eng.values()
            eng.gae()
            eng.begin_update()
            eng.grad(None)
            local = eng.grad_flat.clone()
            eng.begin_update()
            eng.step(None, allreduce=ctx.grad_allreduce_fn(True), mean=True)
            eng.finish_steps()
            torch.cuda.synchronize()
            out[f"mean/{dtype}/{gc}"] = (local.cpu(), eng.grad_flat.cpu())
    torch.save(out, os.path.join(out_dir, f"two{rank}.pt"))
    base.destroy()


def test_two_rank_engine_paths_bit_identical_and_mean_scaled_once(tmp_path):
    """2 ranks on the one GPU (gloo): the in-stream production branch (GlooStreamComm) and the
    process-group per-head chains give bit-identical parameters (the wgrad splits every tile the
    same way on both, parallel/dist.py), with and without the side-stream value step of
    --overlap-rollout, at bf16x3 / bf16 / fp8; replicas stay identical; and grad_reduce=mean
    gives (g0 + g1) / 2 on the tile and per-head updates over both communicators (once, not
    divided by N again: ADVICE r3 medium)."""
    import torch.multiprocessing as mp
    from pytorch_dppo_amd.runtime.launcher import free_port
    port = free_port()
    ctxm = mp.get_context("spawn")
    procs = [ctxm.Process(target=_two_rank_child, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p_ in procs:
        p_.start()
    for p_ in procs:
        p_.join(115)
    codes = [p_.exitcode for p_ in procs]
    for p_ in procs:
        if p_.is_alive():
            p_.kill()
    assert codes == [0, 0], codes
    r0 = torch.load(tmp_path / "two0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "two1.pt", weights_only=True)
    for dtype in ("bf16x3", "bf16", "fp8"):
        ref = r0[f"{dtype}/process_group/False"][0]
        for key in (f"{dtype}/auto/False", f"{dtype}/auto/True", f"{dtype}/auto/every",
                    f"{dtype}/process_group/False"):
            (f0, s0, n0, side0), (f1, s1, _, _) = r0[key], r1[key]
            assert s0 and s1, key
            assert torch.equal(f0, f1), key                      # replicas bit-identical
            assert n0 == ("auto" in key), key                    # the adapter ran the in-stream branch
            assert side0 == (key.endswith("auto/True") or key.endswith("auto/every")), key
            assert torch.equal(f0, ref), (key, (f0 - ref).abs().max().item())
    for dtype in ("fp32", "bf16x3"):
        for gc in ("auto", "process_group"):
            (l0, g0), (l1, g1) = r0[f"mean/{dtype}/{gc}"], r1[f"mean/{dtype}/{gc}"]
            assert not torch.equal(l0, l1)
            want = (l0 + l1) * 0.5
            assert torch.equal(g0, g1)
            assert torch.allclose(g0, want, rtol=1e-6, atol=1e-9), (dtype, gc, (g0 - want).abs().max().item())


def _fault_child(rank, world, port, out_dir):
    """rank 1 dies at iteration 1, epoch 2 (DPPO_DEBUG_FAULT); rank 0 must leave with an error"""
    import os
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DPPO_DEBUG_FAULT"] = "1:1:2"
    torch.set_num_threads(2)
    import time
    from pytorch_dppo_amd.parallel.dist import init_distributed
    from pytorch_dppo_amd.runtime.launcher import run_worker
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=256, exploration_size=256 * 8,
                    batch_size=256 * 8, num_epoch=4, seed=3, num_processes=world, dist_backend="gloo",
                    dtype="bf16x3", max_iters=5, dist_timeout_s=30, heartbeat_s=0.5, heartbeat_timeout_s=10)
    ctx = init_distributed("gpu", rank=rank, world_size=world, backend="gloo", timeout_s=30)
    t0 = time.time()
    try:
        run_worker(p, ctx, evaluator=False, quiet=True)
    finally:
        with open(os.path.join(out_dir, f"fault{rank}.txt"), "w") as f:
            f.write(f"{time.time() - t0:.1f}")


def test_dead_rank_on_the_production_path_fails_the_survivor_fast(tmp_path):
    """Fault injection on the default multi-rank GPU path (reference Q21: a dead worker
    deadlocks the chief forever, chief.py:13): rank 1 exits before epoch 3 of iteration 1; the
    survivor must exit non-zero by itself, well inside the timeout."""
    import time
    import torch.multiprocessing as mp
    from pytorch_dppo_amd.runtime.launcher import free_port
    port = free_port()
    ctxm = mp.get_context("spawn")
    procs = [ctxm.Process(target=_fault_child, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    t0 = time.time()
    for p_ in procs:
        p_.start()
    for p_ in procs:
        p_.join(100)
    codes = [p_.exitcode for p_ in procs]
    for p_ in procs:
        if p_.is_alive():
            p_.kill()
    assert codes[1] == 13, codes
    assert codes[0] not in (0, None), codes                      # the survivor failed, on its own
    assert time.time() - t0 < 100


def test_debug_sync_mode_runs_an_iteration_bit_identical():
    """DPPO_DEBUG_SYNC mode (every op synchronises + checks after its launch) changes no result."""
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    common = dict(device="gpu", env_name="Humanoid-v2", num_envs=64, exploration_size=64 * 4,
                  batch_size=64 * 4, num_epoch=1, dtype="bf16")
    ext = _ext()
    out = []
    for on in (False, True):
        ext.set_debug_sync(on)
        try:
            w = DPPOWorker(dppo_preset(**common), DistContext(device=DEV))
            w.iteration_step()
            torch.cuda.synchronize()
            out.append(w.model.flat.data.clone())
        finally:
            ext.set_debug_sync(False)
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("dtype,loss", [("bf16", "ppo"), ("fp32", "ppo"), ("bf16", "dppo_ref"), ("bf16x3", "ppo")])
def test_fused_gather_adam_bit_identical_to_gather_then_adam(dtype, loss, monkeypatch):
    """World size 1 runs grad_gather + no-clip Adam as ONE launch (gather_adam): parameters, Adam
    moments and weight images after a full iteration equal the two-launch path's bit for bit."""
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    common = dict(device="gpu", env_name="Humanoid-v2", num_envs=64, exploration_size=64 * 4,
                  batch_size=64 * 4, num_epoch=3, dtype=dtype, loss=loss)
    out = []
    for fused in ("1", "0"):
        w = DPPOWorker(dppo_preset(**common, fused_apply=fused == "1"), DistContext(device=DEV))
        assert w.engine.fused_apply == (fused == "1")
        assert w.engine.can_fuse_apply() == (fused == "1")
        m = w.iteration_step()
        torch.cuda.synchronize()
        e = w.engine
        out.append((w.model.flat.data.clone(), e.adam_m.clone(), e.adam_v.clone(), e.wimg.clone(),
                    e.grad_flat.clone(), m))
    (p0, m0, v0, i0, g0, mt0), (p1, m1, v1, i1, g1, mt1) = out
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    assert torch.equal(i0.view(torch.uint8), i1.view(torch.uint8))
    assert torch.equal(g0, g1)
    assert abs(mt0["grad_norm"] - mt1["grad_norm"]) <= 1e-5 * (1 + mt1["grad_norm"])
    assert mt0["loss"] == mt1["loss"]


def test_side_stream_obs_stats_bit_identical(monkeypatch):
    """The rollout-mode obs-stat reduce + merge on a side stream (overlapping values/GAE/update)
    leaves parameters, normaliser state and metrics exactly as the inline path does."""
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    common = dict(device="gpu", env_name="Humanoid-v2", num_envs=64, exploration_size=64 * 4,
                  batch_size=64 * 4, num_epoch=2, dtype="bf16")
    out = []
    for on in ("1", "0"):
        w = DPPOWorker(dppo_preset(**common, stats_stream="on" if on == "1" else "off"), DistContext(device=DEV))
        assert (w._stats_stream is not None) == (on == "1")
        ms = [w.iteration_step(), w.iteration_step(defer=True), w.iteration_step(defer=True)]
        ms.append(w.finish_metrics())
        torch.cuda.synchronize()
        out.append((w.model.flat.data.clone(), w.stats.mean.clone(), w.stats.mean_diff.clone(), w.stats.n,
                    repr([(m["mean_ep_return"], m["ep_count"], m["loss"]) for m in ms if m])))
    a, b = out
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    assert a[3] == b[3] and a[4] == b[4]


@pytest.mark.parametrize("dtype,tol", [("bf16x3", 2e-4), ("bf16", 6e-2)])
def test_bench_geometry_full_batch_gradient_matches_autograd(dtype, tol):
    """The benchmarked geometry exactly (bench.py defaults): Humanoid-v2, E=4096, T=16, one
    full-batch step of 65,536 rows, x^T written by the rollout kernel (xT_ready), the 256-task
    wgrad plan with up to 1,024 batch chunks — vs fp32 autograd on the same decoded buffer."""
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=4096 * 16,
                    batch_size=4096 * 16, dtype=dtype, num_epoch=1)
    eng, model, env, stats = _engine(p)
    stats.observes(env.observe())
    # (the 32x32 policy head reads the observation rows from x_buf: the rollout writes no x^T)
    assert (eng.xT_from_rollout or eng.phead) and eng.N == 65536
    assert sum(b["tasks_host"].numel() // 8 for b in eng.buckets) >= 200
    eng.rollout()
    eng.values()
    eng.gae()
    eng.begin_update()
    assert eng._xT_valid or eng.phead
    eng.grad(None)
    assert not eng.phead or eng._x_mode == "buf"
    xq = eng.decode(eng.x_buf)[:eng.N, :model.num_inputs]
    model.flat.grad = None
    mu, ls, v = model(xq)
    out = oracle.ppo_loss(mu, ls, v, eng.actions, eng.logp, eng.adv, eng.ret, eng.values_buf[:eng.N],
                          clip=p.clip, ent_coeff=p.ent_coeff, value_loss=p.value_loss, convention=p.std_convention)
    out["loss"].backward()
    g_ref = model.flat.grad.detach()
    rel = (eng.grad_flat - g_ref).norm().item() / (g_ref.norm().item() + 1e-12)
    assert rel < tol, rel
    # per-layer too: no layer may hide behind the others' norm
    for name in ("p_fc1", "p_fc2", "mu", "v_fc1", "v_fc2", "v"):
        o, n = model.offsets[f"{name}.weight"]
        gr, gk = g_ref[o:o + n], eng.grad_flat[o:o + n]
        assert (gk - gr).norm().item() <= 3 * tol * (gr.norm().item() + 1e-8), name


@pytest.mark.parametrize("dtype,tol", [("bf16x3", 2e-4), ("fp32", 1e-4)])
def test_bench_geometry_gradient_vs_autograd_on_fp32_observations(dtype, tol):
    """The benchmarked geometry (65,536-row full batch, Humanoid dims, the 256-task wgrad plan)
    against fp32 autograd on the fp32 observation rows themselves, not on the decoded storage:
    the storage rounding of X (split-bf16: ~2^-17 relative) and of every stored wgrad operand
    counts against the budget."""
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=4096 * 16,
                    batch_size=4096 * 16, dtype=dtype, num_epoch=1)
    eng, model, _, _ = _engine(p)
    assert eng.N == 65536
    _fill_buffer(eng, model, gen_seed=5)
    # the same first draw as _fill_buffer: the un-quantised rows
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(eng.N + eng.E, model.num_inputs, generator=g).clamp(-5, 5).to(DEV)[:eng.N]
    if dtype == "bf16x3":
        xq = eng.decode(eng.x_buf)[:eng.N, :model.num_inputs]
        assert 0 < (xq - x).abs().max().item() <= 2 ** -16 * 5
    eng.begin_update()
    eng.grad(None)
    model.flat.grad = None
    mu, ls, v = model(x)
    out = oracle.ppo_loss(mu, ls, v, eng.actions, eng.logp, eng.adv, eng.ret, eng.values_buf[:eng.N],
                          clip=p.clip, ent_coeff=p.ent_coeff, value_loss=p.value_loss, convention=p.std_convention)
    out["loss"].backward()
    g_ref = model.flat.grad.detach()
    rel = (eng.grad_flat - g_ref).norm().item() / (g_ref.norm().item() + 1e-12)
    assert rel < tol, rel
    for name in ("p_fc1", "p_fc2", "mu", "v_fc1", "v_fc2", "v"):
        o, n = model.offsets[f"{name}.weight"]
        gr, gk = g_ref[o:o + n], eng.grad_flat[o:o + n]
        assert (gk - gr).norm().item() <= 3 * tol * (gr.norm().item() + 1e-8), name


@pytest.mark.parametrize("dtype", ["bf16x3", "bf16"])
def test_wgrad_wide_tiles_match_one_quadrant_per_wave(dtype):
    """The wgrad's wide plan (csrc/wgrad.hip: up to 16 quadrants per task, two per wave, a 40-slot
    ring; Humanoid v_fc1 as four 4x3 tiles, p_fc1 one 2x6 tile over row-major operands) vs one
    quadrant per wave (Params.wgrad_wide False) on the same full-batch buffer: the same products,
    summed over different batch chunks — equal to fp32 rounding of the chunk sums."""
    res = {}
    for wide in (True, False):
        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=1024, exploration_size=1024 * 16,
                        batch_size=1024 * 16, dtype=dtype, update_kernels="heads")
        p.wgrad_wide = wide
        eng, model, _, _ = _engine(p)
        assert eng.wgrad_wide == wide
        qs = [t[6] * t[7] for t in eng.joint_bucket["tasks_host"].view(-1, 8).tolist()]
        assert (max(qs) > 8) == wide
        _fill_buffer(eng, model, gen_seed=7)
        eng.begin_update()
        eng.grad(None)
        torch.cuda.synchronize()
        res[wide] = eng.grad_flat.clone()
    assert torch.isfinite(res[True]).all()
    for name in ("p_fc1", "p_fc2", "v_fc1", "v_fc2"):
        for part in ("weight", "bias"):
            o, n = model.offsets[f"{name}.{part}"]
            a_, b_ = res[True][o:o + n], res[False][o:o + n]
            assert (a_ - b_).norm().item() <= 1e-5 * (b_.norm().item() + 1e-8), (name, part)


@pytest.mark.parametrize("env_name", ["Humanoid-v2"])
def test_rollout_bf16_eight_wave_kernel_tracks_torch_engine(env_name):
    """The benchmarked bf16 rollout variant (rollout_kernel<bf16, 16 envs, 8 waves>) vs the torch
    engine with the same noise: log-probs depend only on the noise (tight), actions/obs carry the
    bf16 policy error (loose), done flags are action-independent (exact)."""
    p = dppo_preset(device="gpu", env_name=env_name, num_envs=64, exploration_size=64 * 8,
                    batch_size=64 * 8, dtype="bf16")
    eng, model, env, stats = _engine(p)
    stats.observes(env.observe())
    eng.params_changed()
    p_cpu = Params.from_dict({**p.to_dict(), "device": "cpu"})
    ref = _torch_rollout(p_cpu, model, stats)
    eng.rollout()
    ref.rollout()
    T, E = eng.T, eng.E
    assert torch.allclose(eng.logp.view(T, E), ref.logp, atol=1e-4, rtol=1e-5)
    assert torch.equal(eng.dones.view(T, E), ref.dones)
    da = (eng.actions.view(T, E, -1) - ref.actions).abs()
    assert da.max().item() < 5e-2 and da.mean().item() < 5e-3, (da.max().item(), da.mean().item())
    xk = eng.decode(eng.x_buf).view(T + 1, E, -1)[..., :model.num_inputs]
    dx = (xk - ref.x).abs()
    assert dx.max().item() < 5e-2 and dx.mean().item() < 5e-3, (dx.max().item(), dx.mean().item())


def test_learning_tracks_exact_fp32():
    """GPU learning check: 80 DPPO iterations of synthetic Humanoid from one
    seed at every precision, against the EXACT fp32 path (v_mfma_f32_16x16x4_f32 tile kernels).
    Each run must learn by a wide margin (measured on MI355X: mean step reward 0.460 -> 0.542,
    +0.083, at every precision); the fp32-accurate split-bf16 curve must stay on the fp32 one at
    every iteration, and the bf16 / fp8 curves must end within a band of it."""
    import statistics
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    curves = {}
    for dt in ("fp32", "bf16x3", "bf16", "fp8"):
        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=1024, exploration_size=1024 * 16,
                        batch_size=1024 * 16, num_epoch=10, dtype=dt, seed=11)
        w = DPPOWorker(p, DistContext(device=DEV))
        r = []
        for _ in range(80):
            w.iteration_step()
            # mean per-step (clipped) reward of the iteration's rollout: episode returns would
            # also grow with episode length alone
            r.append(w.engine.rewards.mean().item())
        curves[dt] = r
    late = {k: statistics.fmean(v[-10:]) for k, v in curves.items()}
    early = {k: statistics.fmean(v[:5]) for k, v in curves.items()}
    print("learning curves (mean step reward)", {k: [round(x, 4) for x in v[::8]] for k, v in curves.items()})
    gain = late["fp32"] - early["fp32"]
    assert gain > 0.05, (early["fp32"], late["fp32"])
    for k in curves:
        assert late[k] > early[k] + 0.05, (k, early[k], late[k])
    drift = max(abs(a - b) for a, b in zip(curves["bf16x3"], curves["fp32"]))
    assert drift <= 0.004 and abs(late["bf16x3"] - late["fp32"]) <= 0.05 * gain, (drift, late)
    for k in ("bf16", "fp8"):
        assert abs(late[k] - late["fp32"]) <= 0.2 * gain, (k, late)


@pytest.mark.parametrize("dtype", ["fp32", "bf16x3"])
def test_compat_bootstrap_uses_raw_state_on_gpu(dtype):
    """--compat Q8 on the HIP engine: the bootstrap row of values_buf is
    V(raw s_T) (train.py:109-112), the other rows V(normalised s_t); matches the torch engine."""
    p = dppo_preset(device="gpu", env_name="HalfCheetah-v2", num_envs=48, exploration_size=48 * 4,
                    batch_size=48 * 4, dtype=dtype, compat=True)
    eng, model, env, stats = _engine(p)
    stats.observes(env.observe())
    eng.rollout()
    eng.values()
    raw = env.observe()
    with torch.no_grad():
        _, _, v_raw = model(raw)
        _, _, v_norm = model(eng.decode(eng.x_buf)[eng.N:, :model.num_inputs])
    vb = eng.values_buf[eng.N:]
    assert torch.allclose(vb, v_raw.reshape(-1), atol=5e-5, rtol=5e-5)
    assert not torch.allclose(vb, v_norm.reshape(-1), atol=1e-3)


@pytest.mark.parametrize("dtype,envs", [("bf16x3", 64), ("fp8", 64), ("fp8", 2048)])
def test_gpu_resume_continues_bit_identically(dtype, envs, tmp_path):
    """SURVEY §5.4 on the HIP engine: 3 iterations straight == 2 iterations,
    checkpoint, resume (load + broadcast + params_changed), 1 more — parameters, Adam moments,
    Adam step and the packed weight images (fp8: the e4m3 forward image and its scales) agree
    bit for bit."""
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.launcher import run_worker
    # (2048 envs x 16 steps: the per-head path, fp8 with the e4m3 wgrad operands and their
    # delayed-scale ring in the checkpoint)
    T = 4 if envs == 64 else 16
    base = dict(device="gpu", env_name="Humanoid-v2", num_processes=1, num_envs=envs, exploration_size=envs * T,
                batch_size=envs * T, num_epoch=2, dtype=dtype, seed=4)
    ctx = DistContext(device=DEV)
    w_full, _ = run_worker(dppo_preset(max_iters=3, **base), ctx, evaluator=False, quiet=True)
    ck = str(tmp_path / "ck")
    run_worker(dppo_preset(max_iters=2, checkpoint_dir=ck, **base), ctx, evaluator=False, quiet=True)
    w_res, _ = run_worker(dppo_preset(max_iters=3, resume=ck, **base), ctx, evaluator=False, quiet=True)
    torch.cuda.synchronize()
    assert w_res.iteration == 3 and w_res.engine.adam_step == w_full.engine.adam_step
    a, b = w_full.engine, w_res.engine
    assert torch.equal(w_full.model.flat.data, w_res.model.flat.data)
    assert torch.equal(a.adam_m, b.adam_m) and torch.equal(a.adam_v, b.adam_v)
    assert torch.equal(a.wimg, b.wimg) and torch.equal(a.wimg_fwd, b.wimg_fwd) and torch.equal(a.qscale, b.qscale)
    assert torch.equal(w_full.stats.mean, w_res.stats.mean)
    assert a.q8 == (envs == 2048 and dtype == "fp8") and torch.equal(a.q8_amax, b.q8_amax)


def test_launch_error_raises_instead_of_stale_result():
    """A refused launch raises a Python exception naming the op (launch errors
    were only printed).  debug_invalid_launch asks the runtime for a 2048-thread workgroup (the
    limit is 1024): the runtime refuses it before anything reaches the GPU, the launcher records
    the error, and the binding raises; the channel is clean again afterwards."""
    ext = _ext()
    with pytest.raises(RuntimeError, match="debug_invalid_launch: HIP launch failed"):
        ext.debug_invalid_launch()
    g = torch.zeros(4, 4, device=DEV)
    ext.gae(g, torch.zeros(5, 4, device=DEV), g, torch.empty_like(g), torch.empty_like(g), 0.99, 0.95, 0, 0)
    torch.cuda.synchronize()


def test_fp8_device_refresh_matches_torch_quantisation():
    """fp8 forward image refresh on the device (fp8_scale + pack_fp8 kernels): per-layer scales ==
    amax / 416 over each layer's weight and bias, and the e4m3 image == torch's float8_e4m3fn
    rounding of p / scale (both round to nearest even; no value reaches the 448 saturation)."""
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=64, exploration_size=64 * 4, batch_size=64 * 4,
                    dtype="fp8")
    eng, model, _, _ = _engine(p)
    with torch.no_grad():
        model.flat.data.mul_(torch.linspace(0.5, 3.0, model.num_params, device=DEV))   # distinct layer amax
    eng.refresh_fwd_image()
    L = model.packed_layout()
    names = [l.name for l in L.layers]
    amax = torch.stack([torch.maximum(model.view(f"{n}.weight").abs().amax(), model.view(f"{n}.bias").abs().amax())
                        for n in names])
    # (torch divides by a python scalar as a multiply by its reciprocal: allow that 1-ulp gap;
    # the kernel divides exactly, as the tensor-by-tensor division below does)
    assert torch.allclose(eng.qscale, torch.clamp(amax.detach() / 416.0, min=1e-12), rtol=2e-7, atol=0)
    lid = eng.layer_id.long()
    sel = lid >= 0
    q = (model.flat.data[sel] / eng.qscale[lid[sel]]).to(torch.float8_e4m3fn).view(torch.uint8)
    w_map = L.flat_to_w.to(DEV).long()[sel]
    wt_map = L.flat_to_wt.to(DEV).long()[sel]
    has_t = wt_map >= 0            # (the first layer of each head has no transposed image)
    same = (eng.wimg_fwd[w_map] == q).float().mean().item()
    assert same > 0.9999 and torch.equal(eng.wimg_fwd[w_map][has_t], eng.wimg_fwd[wt_map[has_t]]), same


@pytest.mark.parametrize("policy_gemms", [False, True])
def test_fp8_update_per_layer_error_and_shadow_image(policy_gemms, monkeypatch):
    """fp8 mode (BASELINE config 5) on the per-head path: forward GEMMs on the e4m3 MFMA
    (csrc/mlp_head.hip F8: e4m3 weight image x e4m3-rounded observations / activations — the value
    fc1 on the 16x16x32 form; with fp8_policy_gemms the policy's fc1 and fc2 on the block-scaled
    16x16x128 form, else bf16), in the
    update and in values().  Per-layer relative error of the gradient vs fp32 autograd on the fp32 rows, the
    value forward vs the fp32 model, and the shadow e4m3 image the Adam step refreshes (== torch's
    float8_e4m3fn rounding of p / qscale for the new parameters)."""
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=2048, exploration_size=2048 * 16,
                    batch_size=2048 * 16, dtype="fp8", ent_coeff=0.01, update_kernels="heads",
                    fp8_policy_gemms=policy_gemms)
    eng, model, _, _ = _engine(p)
    assert eng.fp8 and eng.heads
    eng.refresh_fwd_image()
    _fill_buffer(eng, model, gen_seed=7)
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(eng.N + eng.E, model.num_inputs, generator=g).clamp(-5, 5).to(DEV)
    # value forward (fp8 fc1) vs the fp32 model on the fp32 rows
    eng.values()
    with torch.no_grad():
        _, _, v32 = model(x)
    verr = (eng.values_buf - v32.reshape(-1)).abs().max().item() / v32.abs().max().item()
    # gradient vs fp32 autograd on the fp32 rows
    eng.begin_update()
    eng.grad(None)
    model.flat.grad = None
    mu, ls, v = model(x[:eng.N])
    out = oracle.ppo_loss(mu, ls, v, eng.actions, eng.logp, eng.adv, eng.ret, eng.values_buf[:eng.N],
                          clip=p.clip, ent_coeff=p.ent_coeff, value_loss=p.value_loss, convention=p.std_convention)
    out["loss"].backward()
    g_ref = model.flat.grad.detach().clone()
    errs = {}
    for name in ("p_fc1", "p_fc2", "mu", "v_fc1", "v_fc2", "v"):
        o, n = model.offsets[f"{name}.weight"]
        errs[name] = (eng.grad_flat[o:o + n] - g_ref[o:o + n]).norm().item() / (g_ref[o:o + n].norm().item() + 1e-12)
    print("fp8 value forward max rel err", verr, "per-layer gradient rel err", errs)
    assert verr < 0.05, verr
    # (measured on MI355X with the policy's two e4m3 GEMMs: p_fc1 14.3 %, p_fc2 15.7 %, mu 15.9 %, with
    # bf16 policy GEMMs ~5 %; the value's e4m3 fc1: v_fc1 8.6 %, v_fc2 9.7 %, v 8.0 %
    # (profiles/r4/fp8_heads.md).  e4m3's 3-bit mantissa on both operands of each GEMM, ~3.6 % RMS per
    # rounding, compounds through the chain into a gradient that is mostly noise)
    pol = 0.22 if policy_gemms else 0.06
    for name, e in errs.items():
        assert e < (pol if name.startswith(("p_", "mu")) else 0.12), (name, e)
    # the Adam step refreshes the e4m3 shadow image with the iteration's scales
    eng.apply()
    L = model.packed_layout()
    lid = eng.layer_id.long()
    sel = lid >= 0
    q = (model.flat.data[sel] / eng.qscale[lid[sel]]).to(torch.float8_e4m3fn).view(torch.uint8)
    w_map = L.flat_to_w.to(DEV).long()[sel]
    wt_map = L.flat_to_wt.to(DEV).long()[sel]
    has_t = wt_map >= 0            # (the first layer of each head has no transposed image)
    same = (eng.wimg_fwd[w_map] == q).float().mean().item()
    assert same > 0.9999 and torch.equal(eng.wimg_fwd[w_map][has_t], eng.wimg_fwd[wt_map[has_t]]), same


def _e4m3(t: torch.Tensor) -> torch.Tensor:
    return t.view(torch.float8_e4m3fn).float()


def test_fp8_e4m3_wgrad_operands_match_bf16_operands(monkeypatch):
    """fp8 mode's e4m3 wgrad operands (csrc/common.h Q8): the same full-batch step with e4m3 and
    with bf16 operands (fp8_wgrad_operands=False).  The e4m3 activations decode (/ their fixed scale) to the bf16
    ones within e4m3 rounding; the gradient maxima the head kernels record in the amax ring are
    the bf16 gradient operands' maxima; the step-1 gradient operands use the power-of-two scale
    that puts the step-0 maximum in [64, 128); the per-layer gradients agree within 5 % (measured
    on MI355X: 3.6-3.9 % for all four layers — e4m3's 3-bit mantissa on both operands of every
    product, ~4 % RMS, does not average out of a gradient that is mostly noise, as with these
    random advantages)."""
    p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=2048, exploration_size=2048 * 16,
                    batch_size=2048 * 16, dtype="fp8", ent_coeff=0.01, update_kernels="heads")
    eq, model, _, _ = _engine(p)
    p.fp8_wgrad_operands = False
    eb, model_b, _, _ = _engine(p)
    assert eq.q8 and not eb.q8 and eq.heads and eb.heads
    assert torch.equal(model.flat.data, model_b.flat.data)
    for e in (eq, eb):
        e.refresh_fwd_image()
        _fill_buffer(e, model if e is eq else model_b, gen_seed=5)
        e.begin_update()
        e.grad(None)
    torch.cuda.synchronize()
    ld = eq.ldT
    # activations: e4m3(h * 256) vs bf16(h); x^T: e4m3(x * 64) vs bf16(x)
    for name, sc in (("h1vT", 256.0), ("h1pT", 256.0), ("xT", 64.0)):
        a = _e4m3(getattr(eq, name)) / sc
        b = eb.decode(getattr(eb, name)).float()
        err = (a - b).abs()
        assert bool((err <= 2 ** -4 * b.abs() + 2 ** -9 / sc + 2 ** -8 * b.abs()).all()), (name, err.max().item())
    # the amax ring: step 0 accumulated into slot 0 (the calibration pass into slot 2)
    amax = eq.q8_maxima()
    for k, name in enumerate(("g1pT", "g2pT", "g1vT", "g2vT")):
        ref = eb.decode(getattr(eb, name)).float().abs().max().item()
        assert abs(amax[0, k].item() - ref) <= 2 ** -7 * ref, (name, amax[0, k].item(), ref)
        assert abs(amax[2, k].item() - ref) <= 2 ** -7 * ref, (name, "calibration", amax[2, k].item(), ref)
    errs = {}
    for name in ("p_fc1", "p_fc2", "v_fc1", "v_fc2"):
        o, n = model.offsets[f"{name}.weight"]
        g_b = eb.grad_flat[o:o + n]
        errs[name] = (eq.grad_flat[o:o + n] - g_b).norm().item() / (g_b.norm().item() + 1e-12)
    print("e4m3 vs bf16 wgrad operands, per-layer gradient rel diff", errs)
    for name, e in errs.items():
        assert e < 0.05, (name, e)
    # step 1 stores g with 2^e, e = 6 - floor(log2(step-0 amax)): the stored maximum in [64, 128)
    eq.grad(None)
    torch.cuda.synchronize()
    amax = eq.q8_maxima()
    for k, name in enumerate(("g1pT", "g1vT")):
        kk = (0, 2)[k]
        e = 6 - int(math.floor(math.log2(amax[0, kk].item())))
        stored = _e4m3(getattr(eq, name)).abs().max().item()
        assert 32 <= stored <= 448 and abs(stored / 2 ** e - amax[1, kk].item()) <= 2 ** -3 * amax[1, kk].item(), \
            (name, stored, e, amax[1, kk].item())


@pytest.mark.parametrize("case", ["ppo_minibatch_clip", "dppo_ref"])
def test_fp8_e4m3_operands_on_other_update_paths(case, monkeypatch):
    """The e4m3 wgrad operands on the other per-head update paths: an index-gathered minibatch of
    half the buffer with global-norm clipping (ppo preset: the policy kernel writes x^T of the
    gathered rows every step), and the reference DPPO loss (mu_prev / v_prev writes, also in the
    calibration pass).  Per-layer gradients within 5 % of the bf16-operand path, two full steps
    finite and the replicated parameters moving."""
    E, T = 2048, 32
    if case == "ppo_minibatch_clip":
        p = ppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T,
                       batch_size=E * T // 2, dtype="fp8")
    else:
        p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T // 2,
                        batch_size=E * T // 2, dtype="fp8", loss="dppo_ref", std_convention="var")
    p.update_kernels = "heads"
    engs = {}
    for q8 in ("1", "0"):
        p.fp8_wgrad_operands = q8 == "1"
        e, m, _, _ = _engine(p)
        assert e.heads and e.q8 == (q8 == "1")
        e.refresh_fwd_image()
        _fill_buffer(e, m, gen_seed=9)
        engs[q8] = (e, m)
    g = torch.Generator(device="cpu").manual_seed(4)
    idx = None if case == "dppo_ref" else torch.randperm(engs["1"][0].N, generator=g)[:engs["1"][0].mb].to(DEV)
    for q8, (e, m) in engs.items():
        e.begin_update()
        e.grad(idx)
    torch.cuda.synchronize()
    (eq, mq), (eb, _) = engs["1"], engs["0"]
    for name in ("p_fc1", "p_fc2", "v_fc1", "v_fc2"):
        o, n = mq.offsets[f"{name}.weight"]
        gb = eb.grad_flat[o:o + n]
        err = (eq.grad_flat[o:o + n] - gb).norm().item() / (gb.norm().item() + 1e-12)
        assert err < 0.05, (case, name, err)
    p0 = mq.flat.data.clone()
    for _ in range(2):
        eq.step(idx)
    eq.finish_steps()
    torch.cuda.synchronize()
    assert bool(torch.isfinite(mq.flat.data).all()) and not torch.equal(p0, mq.flat.data)
    assert float(eq.q8_maxima().max()) > 0


@pytest.mark.parametrize("heads", ["1", "0"])
@pytest.mark.parametrize("dtype", ["bf16x3", "bf16"])
def test_update_reads_rows_past_2gib_of_the_observation_buffer(dtype, heads, monkeypatch):
    """A Humanoid buffer of 65,536 envs x 22 (44 at bf16) steps (x_buf 2.3 GB): a minibatch whose
    rows all lie past the 2 GiB mark gets the gradient of autograd on exactly those rows — the
    per-head kernels' observation gather (64-bit per-lane LDS-DMA addresses) and the tile kernel's
    both address the buffer with 64-bit offsets."""
    E, mb = 65536, 512
    T = 22 if dtype == "bf16x3" else 44      # 4 / 2 bytes per element: > 2.2 GB either way
    p = ppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=E, exploration_size=E * T, batch_size=mb,
                   dtype=dtype, ent_coeff=0.01, update_kernels="heads" if heads == "1" else "tile")
    eng, model, _, _ = _engine(p)
    assert eng.heads == (heads == "1")
    row_bytes = eng.x_buf.element_size() * eng.d0
    first = (1 << 31) // row_bytes + 1
    assert eng.x_buf.numel() * eng.x_buf.element_size() > 2.2e9 and first + mb < eng.N
    g = torch.Generator(device="cpu").manual_seed(17)
    idx = (first + torch.randperm(eng.N - first, generator=g)[:mb]).to(DEV)
    O, A = model.num_inputs, model.num_outputs
    xb = torch.zeros(mb, eng.d0, device=DEV)
    xb[:, :O] = torch.randn(mb, O, generator=g).clamp(-5, 5).to(DEV)
    xb[:, O] = 1.0
    eng.x_buf[idx] = eng.encode(xb)
    xq = torch.zeros(eng.N, O, device=DEV)
    xq[idx] = eng.decode(eng.x_buf[idx])[:, :O]
    with torch.no_grad():
        mu, ls, v = model(xq[idx])
    a = mu + 0.6 * torch.randn(mb, A, generator=g).to(DEV)
    eng.actions[idx] = a
    eng.logp[idx] = oracle.gaussian_logp(a, mu + 0.05 * torch.randn(mb, A, generator=g).to(DEV), ls,
                                         p.std_convention).reshape(-1)
    eng.adv[idx] = torch.randn(mb, generator=g).to(DEV)
    eng.ret[idx] = v.reshape(-1) + 0.5 * torch.randn(mb, generator=g).to(DEV)
    eng.values_buf[idx] = v.reshape(-1) + 0.3 * torch.randn(mb, generator=g).to(DEV)
    eng.begin_update()
    eng.grad(idx.cpu())
    g_ref, _ = _torch_grad(model, p, xq, eng, idx)
    rel = (eng.grad_flat - g_ref).norm().item() / g_ref.norm().item()
    assert rel < (2e-4 if dtype == "bf16x3" else 6e-2), rel
