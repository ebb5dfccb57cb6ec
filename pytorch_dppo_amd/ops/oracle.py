"""Pure-PyTorch math: the CPU execution path and the numerical oracle for every HIP kernel.

Each function documents which reference lines it reproduces.  GPU kernels in ``csrc/`` are
tested against these at fp32 (tight) and bf16/fp8 (loose) tolerances.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import torch

LOG_2PI = math.log(2.0 * math.pi)


def sigma_from_log_std(log_std: torch.Tensor, convention: str) -> torch.Tensor:
    """'std': sigma = exp(log_std) (ppo.py:93).  'var': exp(log_std) is sigma^2 (train.py:89)."""
    return torch.exp(log_std) if convention == "std" else torch.exp(0.5 * log_std)


def gaussian_logp(a: torch.Tensor, mu: torch.Tensor, log_std: torch.Tensor,
                  convention: str = "std") -> torch.Tensor:
    """joint diagonal-Gaussian log-density [B,1] (ppo.py:95-97 for 'std')."""
    log_sigma = log_std if convention == "std" else 0.5 * log_std
    z = (a - mu) * torch.exp(-log_sigma)
    return (-0.5 * z * z - 0.5 * LOG_2PI - log_sigma).sum(-1, keepdim=True)


def gaussian_entropy(log_std: torch.Tensor, convention: str = "std") -> torch.Tensor:
    """analytic entropy sum_j (0.5 + 0.5 log 2pi + log sigma_j) (ppo.py:152-153)."""
    log_sigma = log_std if convention == "std" else 0.5 * log_std
    return (0.5 + 0.5 * LOG_2PI + log_sigma).sum(-1)


def normal_pdf_var(x: torch.Tensor, mu: torch.Tensor, var: torch.Tensor) -> torch.Tensor:
    """per-dim density whose 3rd arg is the VARIANCE (train.py:41-44)."""
    return torch.exp(-(x - mu) ** 2 / (2 * var)) / torch.sqrt(2 * var * math.pi)


def gae(rewards: torch.Tensor, values: torch.Tensor, dones: torch.Tensor, gamma: float,
        lam: float, segment: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """GAE(lambda) over a [T,E] rollout (train.py:109-122, ppo.py:119-133, vectorised).

    ``values`` is [T+1,E] (row T = bootstrap V(s_T)); ``dones[t]`` = episode ended at step t
    (so V_{t+1} and A_{t+1} are masked, which is the reference's segment break + R=0).
    ``segment`` > 0 (the reference's ``num_steps``, train.py:82-106 / ppo.py:87): a segment
    ends at a done OR after ``segment`` steps, and the next segment starts fresh (its step count
    restarts after a done).  Where a segment ends by length without a done the recursion
    restarts (A_{t+1} masked) while the bootstrap V_{t+1} of the not-done state is kept
    (train.py:109-112 per segment).
    Returns (advantages [T,E], returns [T,E]) with returns = A + V.
    """
    T = rewards.shape[0]
    cont = torch.ones_like(rewards)
    if segment > 0:
        # forward: steps since the current segment started, per env (train.py:82 `for step`)
        s = torch.zeros_like(rewards[0], dtype=torch.int64)
        for t in range(T):
            d = dones[t] != 0
            end_len = (s + 1 == segment) & ~d
            cont[t] = torch.where(end_len, torch.zeros_like(cont[t]), cont[t])
            s = torch.where(d | (s + 1 == segment), torch.zeros_like(s), s + 1)
    adv = torch.zeros_like(rewards)
    nxt = torch.zeros_like(rewards[0])
    for t in range(T - 1, -1, -1):
        nonterm = 1.0 - dones[t].to(rewards.dtype)
        delta = rewards[t] + gamma * values[t + 1] * nonterm - values[t]
        nxt = delta + gamma * lam * nonterm * cont[t] * nxt
        adv[t] = nxt
    return adv, adv + values[:T]


def ppo_loss(mu, log_std, v, actions, logp_old, adv, ret, v_old, *, clip: float,
             ent_coeff: float, value_loss: str = "mse", convention: str = "std") -> Dict[str, torch.Tensor]:
    """Corrected PPO loss (ppo.py:148-167).

    ratio = exp(logp - logp_old) with logp_old recorded at rollout; clipped surrogate;
    value loss 'mse' = mean((v-R)^2) (ppo.py:164) or 'clipped_half' =
    0.5*mean(max((v-R)^2, (v_old+clip(v-v_old,+-eps)-R)^2)) (train.py:154-157);
    entropy bonus -ent_coeff * H (ppo.py:167).
    """
    adv = adv.reshape(-1, 1)
    ret = ret.reshape(-1, 1)
    logp = gaussian_logp(actions, mu, log_std, convention)
    ratio = torch.exp(logp - logp_old.reshape(-1, 1))
    surr1 = ratio * adv
    surr2 = ratio.clamp(1.0 - clip, 1.0 + clip) * adv
    loss_clip = -torch.min(surr1, surr2).mean()
    v = v.reshape(-1, 1)
    if value_loss == "mse":
        loss_value = ((v - ret) ** 2).mean()
    else:
        v_old = v_old.reshape(-1, 1)
        vc = v_old + (v - v_old).clamp(-clip, clip)
        loss_value = 0.5 * torch.max((v - ret) ** 2, (vc - ret) ** 2).mean()
    ent = gaussian_entropy(log_std, convention).mean()
    loss_ent = -ent_coeff * ent
    with torch.no_grad():
        lr = (logp - logp_old.reshape(-1, 1))
        approx_kl = ((torch.exp(lr) - 1.0) - lr).mean()
        clipfrac = ((ratio - 1.0).abs() > clip).float().mean()
    return {"loss": loss_clip + loss_value + loss_ent, "loss_clip": loss_clip,
            "loss_value": loss_value, "loss_ent": loss_ent, "approx_kl": approx_kl,
            "clipfrac": clipfrac}


def dppo_ref_loss(mu, log_std, v, mu_old, log_std_old, v_old, actions, adv, ret, *, clip: float,
                  ent_coeff: float) -> Dict[str, torch.Tensor]:
    """The reference DPPO worker loss, verbatim semantics (train.py:142-161).

    sigma_sq = exp(log_std) is used as a VARIANCE; ratio is per action dim
    p/(1e-10+p_old) of the per-dim densities; advantages broadcast over action dims;
    clipped value loss with the same clip eps; entropy term -c*mean(p log(p+1e-5)).
    """
    var = torch.exp(log_std)
    var_old = torch.exp(log_std_old)
    p_old = normal_pdf_var(actions, mu_old, var_old)
    p = normal_pdf_var(actions, mu, var)
    ratio = p / (1e-10 + p_old)
    A = adv.reshape(-1, 1).expand_as(ratio)
    surr1 = ratio * A
    surr2 = ratio.clamp(1.0 - clip, 1.0 + clip) * A
    loss_clip = -torch.min(surr1, surr2).mean()
    v = v.reshape(-1, 1)
    ret = ret.reshape(-1, 1)
    v_old = v_old.reshape(-1, 1)
    vf1 = (v - ret) ** 2
    vc = v_old + (v - v_old).clamp(-clip, clip)
    vf2 = (vc - ret) ** 2
    loss_value = 0.5 * torch.max(vf1, vf2).mean()
    loss_ent = -ent_coeff * (p * torch.log(p + 1e-5)).mean()
    with torch.no_grad():
        clipfrac = ((ratio - 1.0).abs() > clip).float().mean()
    return {"loss": loss_clip + loss_value + loss_ent, "loss_clip": loss_clip,
            "loss_value": loss_value, "loss_ent": loss_ent,
            "approx_kl": torch.zeros((), device=mu.device), "clipfrac": clipfrac}


def clip_grad_norm_(g: torch.Tensor, max_norm: float) -> torch.Tensor:
    """global-norm clip on a flat gradient (nn.utils.clip_grad_norm, ppo.py:173)."""
    norm = torch.linalg.vector_norm(g)
    coef = max_norm / (norm + 1e-6)
    if coef < 1.0:
        g.mul_(coef)
    return norm


def adam_step_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
               lr: float, betas=(0.9, 0.999), eps: float = 1e-8) -> None:
    """torch.optim.Adam (default, non-amsgrad, no weight decay) on flat buffers."""
    b1, b2 = betas
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
