"""Eager-PyTorch engine: the CPU execution path (BASELINE config 1) and the end-to-end oracle
for the HIP engine.

One *engine* owns the device-side state of one DPPO worker — the vectorised envs, the
``[T,E]`` rollout buffer, the flat parameters / gradient / Adam moments — and exposes the
phases the worker loop (``runtime/worker.py``) sequences:

    rollout()  ->  values()  ->  gae()  ->  for each minibatch: grad(idx) -> [all-reduce] -> apply()

Reference mapping: rollout = ``train.py:60-106``; values/bootstrap = ``train.py:109-112``;
gae = ``train.py:117-122``; grad = ``train.py:140-166``; apply = ``chief.py:15-19``.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

from ..config import Params
from ..models.actor_critic import ActorCritic
from ..ops import oracle
from ..utils import rng
from ..utils.obs_stats import RunningObsStats


class TorchEngine:
    name = "torch"

    def __init__(self, params: Params, model: ActorCritic, env, stats: RunningObsStats,
                 device: torch.device, action_rank: int):
        self.p = params
        self.model = model
        self.env = env
        self.stats = stats
        self.device = device
        T, E = params.rollout_len, env.E
        O, A = env.O, env.A
        self.T, self.E, self.O, self.A = T, E, O, A
        f32 = dict(device=device, dtype=torch.float32)
        self.x = torch.zeros(T + 1, E, O, **f32)         # normalised observations (update input)
        self.raw_last = torch.zeros(E, O, **f32)          # raw bootstrap obs (compat Q8)
        self.actions = torch.zeros(T, E, A, **f32)
        self.logp = torch.zeros(T, E, **f32)
        self.values_buf = torch.zeros(T + 1, E, **f32)
        self.rewards = torch.zeros(T, E, **f32)
        self.dones = torch.zeros(T, E, **f32)
        self.adv = torch.zeros(T, E, **f32)
        self.ret = torch.zeros(T, E, **f32)
        n = model.num_params
        self.grad_flat = torch.zeros(n, **f32)
        self.adam_m = torch.zeros(n, **f32)
        self.adam_v = torch.zeros(n, **f32)
        self.adam_step = 0
        self.flat_old = model.flat.detach().clone()  # dppo_ref "model_old" (train.py:128-129,164)
        self.key_action = rng.base_key(params.seed, rng.STREAM_ACTION, action_rank)
        self.obs = env.reset().to(device)
        self.local_stats: Optional[RunningObsStats] = None

    # -- rollout ---------------------------------------------------------------------------
    @torch.no_grad()
    def rollout(self) -> Dict:
        p, T, E = self.p, self.T, self.E
        shift = self.stats.shift().clone()
        s1 = torch.zeros(self.O, dtype=torch.float64, device=self.device)
        s2 = torch.zeros(self.O, dtype=torch.float64, device=self.device)
        count = 0.0
        norm_stats = self.stats
        if p.obs_norm_update == "step":
            self.local_stats = RunningObsStats(self.O, self.device)
            self.local_stats.copy_from(self.stats)
            norm_stats = self.local_stats
        ep_ret_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        ep_count = torch.zeros((), dtype=torch.float64, device=self.device)
        eidx = self.env.env_idx.to(self.device)
        dims = torch.arange(self.A, device=self.device, dtype=torch.int64)
        log_std = self.model.view("log_std")
        log_sigma = log_std if p.std_convention == "std" else 0.5 * log_std
        sigma = torch.exp(log_sigma)
        for t in range(T):
            raw = self.obs
            c, a1, a2 = RunningObsStats.moments(raw, shift)
            count += c
            s1 += a1
            s2 += a2
            if p.obs_norm_update == "step":
                norm_stats.observes(raw)
            x = norm_stats.normalize(raw)
            mu, _, _ = self.model(x)
            eps = rng.gauss(self.key_action, eidx[:, None], self.env.t, dims[None, :])
            a = mu + sigma * eps
            logp = (-0.5 * eps * eps - 0.5 * oracle.LOG_2PI - log_sigma).sum(-1)
            obs, r, done, info = self.env.step(a)
            if p.reward_clip > 0:
                r = r.clamp(-p.reward_clip, p.reward_clip)
            self.x[t] = x
            self.actions[t] = a
            self.logp[t] = logp
            self.rewards[t] = r
            self.dones[t] = done.to(torch.float32)
            ep_ret_sum += info["ep_return_sum"].to(torch.float64)
            ep_count += info["ep_count"].to(torch.float64)
            self.obs = obs.to(self.device)
        self.x[T] = norm_stats.normalize(self.obs)
        self.raw_last.copy_(self.obs)
        return {"count": count, "s1": s1, "s2": s2, "shift": shift,
                "ep_return_sum": float(ep_ret_sum), "ep_count": float(ep_count)}

    @torch.no_grad()
    def values(self) -> None:
        T, E = self.T, self.E
        _, _, v = self.model(self.x.reshape((T + 1) * E, self.O))
        self.values_buf.copy_(v.reshape(T + 1, E))
        if self.p.compat:  # Q8: bootstrap with the raw, un-normalised state (train.py:111)
            _, _, vb = self.model(self.raw_last)
            self.values_buf[T] = vb.reshape(E)

    @torch.no_grad()
    def gae(self) -> None:
        adv, ret = oracle.gae(self.rewards, self.values_buf, self.dones, self.p.gamma, self.p.gae_param,
                              segment=self.p.gae_segment())
        if self.p.normalize_adv:
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        self.adv.copy_(adv)
        self.ret.copy_(ret)

    def current_obs(self) -> torch.Tensor:
        return self.obs

    def env_state(self) -> Dict:
        return self.env.state_dict()

    def load_env_state(self, d: Dict) -> None:
        self.env.load_state_dict(d)
        self.obs = self.env.observe().to(self.device)

    def begin_update(self) -> None:
        self.flat_old.copy_(self.model.flat.detach())

    # -- update ----------------------------------------------------------------------------
    def grad(self, idx: torch.Tensor) -> Dict[str, float]:
        """loss + backward on rows ``idx`` of the flattened [T*E] buffer -> self.grad_flat."""
        p = self.p
        N = self.T * self.E
        if idx is None:
            idx = torch.arange(N, device=self.device)
        x = self.x[:self.T].reshape(N, self.O)[idx]
        a = self.actions.reshape(N, self.A)[idx]
        adv = self.adv.reshape(N)[idx]
        ret = self.ret.reshape(N)[idx]
        self.model.flat.grad = None
        mu, log_std, v = self.model(x)
        if p.loss == "ppo":
            logp_old = self.logp.reshape(N)[idx]
            v_old = self.values_buf[:self.T].reshape(N)[idx]
            out = oracle.ppo_loss(mu, log_std, v, a, logp_old, adv, ret, v_old, clip=p.clip,
                                  ent_coeff=p.ent_coeff, value_loss=p.value_loss,
                                  convention=p.std_convention)
        else:
            with torch.no_grad():
                mu_o, ls_o, v_o = _forward_with(self.model, self.flat_old, x)
            out = oracle.dppo_ref_loss(mu, log_std, v, mu_o, ls_o, v_o, a, adv, ret,
                                       clip=p.clip, ent_coeff=p.ent_coeff)
            # train.py:164 model_old <- model (pre-update params of this step)
            self.flat_old.copy_(self.model.flat.detach())
        out["loss"].backward()
        self.grad_flat.copy_(self.model.flat.grad)
        self._last = {k: float(v.detach()) for k, v in out.items()}
        return self._last

    @torch.no_grad()
    def apply(self, extra_grad: float = 0.0) -> float:
        """clip (optional) + Adam on the flat buffers; returns the pre-clip grad norm."""
        g = self.grad_flat
        if extra_grad:
            g.add_(extra_grad)
        norm = float(torch.linalg.vector_norm(g))
        if self.p.max_grad_norm is not None and self.p.max_grad_norm > 0:
            oracle.clip_grad_norm_(g, self.p.max_grad_norm)
        self.adam_step += 1
        oracle.adam_step_(self.model.flat.data, g, self.adam_m, self.adam_v, self.adam_step,
                          self.p.lr, self.p.adam_betas, self.p.adam_eps)
        self._norm = norm
        return norm

    def last_losses(self) -> Dict[str, float]:
        out = dict(getattr(self, "_last", {}))
        out["grad_norm"] = getattr(self, "_norm", 0.0)
        return out

    def sync(self) -> None:
        pass


def _forward_with(model: ActorCritic, flat: torch.Tensor, x: torch.Tensor):
    saved = model.flat.data
    try:
        model.flat.data = flat
        return model(x)
    finally:
        model.flat.data = saved
