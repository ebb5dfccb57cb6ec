"""Oracle math vs literal re-statements of the reference semantics (SURVEY §4 'Unit: oracle math')."""
import math

import pytest
import torch

from pytorch_dppo_amd.ops import oracle


def _gae_reference_loop(rewards, values, gamma, lam):
    """One segment, reference style (train.py:109-122): python reverse loop, scalar floats.

    values has len(rewards)+1 entries; the last is the bootstrap R (0 if the segment ended in
    a terminal state)."""
    A = 0.0
    adv, ret = [], []
    for i in reversed(range(len(rewards))):
        td = rewards[i] + gamma * values[i + 1] - values[i]
        A = td + gamma * lam * A
        adv.insert(0, A)
        ret.insert(0, A + values[i])
    return adv, ret


def test_gae_matches_reference_loop_with_segment_breaks():
    g = torch.Generator().manual_seed(0)
    T, E = 40, 3
    r = torch.randn(T, E, generator=g, dtype=torch.float64)
    v = torch.randn(T + 1, E, generator=g, dtype=torch.float64)
    d = torch.zeros(T, E, dtype=torch.float64)
    d[7, 0] = d[22, 0] = d[39, 1] = d[0, 2] = 1.0
    adv, ret = oracle.gae(r, v, d, 0.99, 0.95)
    for e in range(E):
        start = 0
        for t in range(T):
            if d[t, e] > 0 or t == T - 1:
                end = t + 1
                seg_r = r[start:end, e].tolist()
                seg_v = v[start:end, e].tolist()
                boot = 0.0 if d[t, e] > 0 else float(v[end, e])
                a_ref, r_ref = _gae_reference_loop(seg_r, seg_v + [boot], 0.99, 0.95)
                assert torch.allclose(adv[start:end, e], torch.tensor(a_ref, dtype=torch.float64))
                assert torch.allclose(ret[start:end, e], torch.tensor(r_ref, dtype=torch.float64))
                start = end


@pytest.mark.parametrize("seg", [5, 8, 13])
def test_gae_segment_length_matches_reference_num_steps_segments(seg):
    """num_steps (train.py:82 / ppo.py:87): a segment ends at done OR after num_steps steps; a
    not-done segment end bootstraps R = V(s_end) (train.py:109-112) and the GAE loop restarts."""
    g = torch.Generator().manual_seed(seg)
    T, E = 40, 3
    r = torch.randn(T, E, generator=g, dtype=torch.float64)
    v = torch.randn(T + 1, E, generator=g, dtype=torch.float64)
    d = torch.zeros(T, E, dtype=torch.float64)
    d[7, 0] = d[22, 0] = d[39, 1] = d[0, 2] = d[11, 2] = 1.0
    adv, ret = oracle.gae(r, v, d, 0.99, 0.95, segment=seg)
    for e in range(E):
        # the reference's segment loop literally (train.py:69-106): `for step in range(num_steps)`
        # with a `break` at done, then the next segment starts fresh
        start = 0
        while start < T:
            t = start
            for step in range(seg):
                t = start + step
                if t == T - 1 or d[t, e] > 0:
                    break
            end = t + 1
            boot = 0.0 if d[t, e] > 0 else float(v[end, e])
            a_ref, r_ref = _gae_reference_loop(r[start:end, e].tolist(), v[start:end, e].tolist() + [boot],
                                               0.99, 0.95)
            assert torch.allclose(adv[start:end, e], torch.tensor(a_ref, dtype=torch.float64))
            assert torch.allclose(ret[start:end, e], torch.tensor(r_ref, dtype=torch.float64))
            start = end


def test_inert_reference_knobs_warn():
    """update_treshold != N-1 cannot be honoured by synchronous collectives: it warns instead of
    being a silent no-op."""
    from pytorch_dppo_amd.config import dppo_preset
    with pytest.warns(UserWarning, match="update_treshold"):
        dppo_preset(num_processes=4, update_treshold=1)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        p = dppo_preset(num_processes=4)
        assert p.update_treshold == 3 and p.gae_segment() == 0
    assert dppo_preset(num_envs=4, exploration_size=400, num_steps=30).gae_segment() == 30


@pytest.mark.parametrize("conv", ["std", "var"])
def test_gaussian_logp_and_entropy_match_torch_distributions(conv):
    g = torch.Generator().manual_seed(1)
    mu = torch.randn(50, 6, generator=g)
    ls = torch.randn(1, 6, generator=g) * 0.3
    a = mu + torch.randn(50, 6, generator=g)
    sigma = torch.exp(ls) if conv == "std" else torch.exp(0.5 * ls)
    dist = torch.distributions.Normal(mu, sigma.expand_as(mu))
    ref = dist.log_prob(a).sum(-1, keepdim=True)
    assert torch.allclose(oracle.gaussian_logp(a, mu, ls, conv), ref, atol=1e-5)
    assert torch.allclose(oracle.gaussian_entropy(ls, conv), dist.entropy()[0].sum(), atol=1e-5)


def test_normal_pdf_var_is_reference_density():
    x, mu, var = torch.tensor([0.3]), torch.tensor([0.1]), torch.tensor([0.5])
    # train.py:41-44: a = exp(-(x-mu)^2/(2 std)); b = 1/sqrt(2 std pi) with std == variance
    expect = math.exp(-(0.2 ** 2) / (2 * 0.5)) / math.sqrt(2 * 0.5 * math.pi)
    assert abs(oracle.normal_pdf_var(x, mu, var).item() - expect) < 1e-7


def test_ppo_loss_terms_by_hand():
    mu = torch.tensor([[0.0], [1.0]], requires_grad=True)
    ls = torch.zeros(1, 1, requires_grad=True)
    v = torch.tensor([[0.5], [0.0]], requires_grad=True)
    a = torch.tensor([[0.1], [0.9]])
    logp_old = oracle.gaussian_logp(a, torch.tensor([[0.0], [1.0]]), ls.detach())
    adv = torch.tensor([1.0, -2.0])
    ret = torch.tensor([1.0, 1.0])
    out = oracle.ppo_loss(mu, ls, v, a, logp_old, adv, ret, None, clip=0.2, ent_coeff=0.01, value_loss="mse")
    # ratio == 1 -> surrogate = -mean(adv) = 0.5; value = mean((v-R)^2) = (0.25 + 1)/2
    assert abs(out["loss_clip"].item() - 0.5) < 1e-6
    assert abs(out["loss_value"].item() - 0.625) < 1e-6
    ent = 0.5 + 0.5 * math.log(2 * math.pi)
    assert abs(out["loss_ent"].item() + 0.01 * ent) < 1e-6


def test_ppo_clip_gradient_zero_outside_trust_region():
    mu = torch.tensor([[2.0]], requires_grad=True)
    ls = torch.zeros(1, 1)
    a = torch.tensor([[2.0]])
    logp_old = oracle.gaussian_logp(a, torch.tensor([[0.0]]), ls)   # ratio = e^2 >> 1.2
    out = oracle.ppo_loss(mu, ls, torch.zeros(1, 1), a, logp_old, torch.tensor([1.0]), torch.zeros(1),
                          None, clip=0.2, ent_coeff=0.0)
    out["loss_clip"].backward()
    assert mu.grad.abs().item() == 0.0


def test_dppo_ref_loss_matches_reference_formulas():
    g = torch.Generator().manual_seed(2)
    B, A = 20, 3
    mu = torch.randn(B, A, generator=g)
    ls = torch.randn(1, A, generator=g) * 0.2
    v = torch.randn(B, 1, generator=g)
    mu_o, ls_o, v_o = mu + 0.1, ls - 0.05, v + 0.3
    a = torch.randn(B, A, generator=g)
    adv = torch.randn(B, generator=g)
    ret = torch.randn(B, generator=g)
    out = oracle.dppo_ref_loss(mu, ls, v, mu_o, ls_o, v_o, a, adv, ret, clip=0.2, ent_coeff=0.1)
    # independent restatement of train.py:142-161
    p_old = torch.exp(-(a - mu_o) ** 2 / (2 * torch.exp(ls_o))) / torch.sqrt(2 * torch.exp(ls_o) * math.pi)
    p = torch.exp(-(a - mu) ** 2 / (2 * torch.exp(ls))) / torch.sqrt(2 * torch.exp(ls) * math.pi)
    ratio = p / (1e-10 + p_old)
    advA = torch.cat([adv[:, None]] * A, 1)
    lc = -torch.mean(torch.min(ratio * advA, ratio.clamp(0.8, 1.2) * advA))
    vf1 = (v - ret[:, None]) ** 2
    vf2 = (v_o + (v - v_o).clamp(-0.2, 0.2) - ret[:, None]) ** 2
    lv = 0.5 * torch.mean(torch.max(vf1, vf2))
    le = -0.1 * torch.mean(p * torch.log(p + 1e-5))
    assert torch.allclose(out["loss"], lc + lv + le, atol=1e-6)


def test_adam_matches_torch_optim():
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(100, generator=g)
    p_ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([p_ref], lr=3e-4)
    p = p0.clone()
    m = torch.zeros(100)
    v = torch.zeros(100)
    for step in range(1, 6):
        grad = torch.randn(100, generator=g)
        p_ref.grad = grad.clone()
        opt.step()
        oracle.adam_step_(p, grad, m, v, step, 3e-4)
    assert torch.allclose(p, p_ref.detach(), atol=1e-7)


def test_clip_grad_norm_matches_torch():
    g = torch.randn(1000) * 3
    p = torch.nn.Parameter(torch.zeros(1000))
    p.grad = g.clone()
    torch.nn.utils.clip_grad_norm_([p], 0.5)
    g2 = g.clone()
    oracle.clip_grad_norm_(g2, 0.5)
    assert torch.allclose(g2, p.grad, atol=1e-7)
