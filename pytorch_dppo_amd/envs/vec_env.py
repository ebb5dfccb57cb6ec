"""Vectorised environments with explicit state tensors.

The reference steps ONE gym env per worker at batch 1 (``train.py:82-106``).  Here a worker
owns ``E`` envs whose whole state lives in tensors (``state [E,S]``, ``ep_len``, ``ep_ret``)
so the GPU rollout kernel (``csrc/rollout.hip``) can step them in-kernel, and the torch
``step`` below is the bit-compatible oracle used on the CPU path and in tests.

Episode semantics follow gym: ``done`` = terminal OR ``ep_len >= min(time_limit,
max_episode_length)`` counted per step (the reference counts per outer iteration, SURVEY Q7;
``compat`` is not needed for that quirk because it almost never fires).  The env resets
in place on ``done`` and returns the post-reset observation, like ``train.py:98-105``.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import torch

from ..utils import rng
from .registry import KIND_PENDULUM, KIND_SYNTHETIC, EnvSpec

SYN_DECAY = 0.9
SYN_DRIVE = 0.1
SYN_NOISE = 0.05
SYN_RESET = 0.1
SYN_TERM_P = 0.002


def syn_weights(obs_dim: int, device) -> torch.Tensor:
    i = torch.arange(obs_dim, device=device)
    return 0.5 + (i % 7).to(torch.float32) / 7.0


class VecEnv:
    """Base: E envs of one spec, keyed RNG (seed, rank)."""

    def __init__(self, spec: EnvSpec, num_envs: int, seed: int = 1, rank: int = 0,
                 device="cpu", max_episode_length: int = 10000):
        self.spec = spec
        self.E = int(num_envs)
        self.O = spec.obs_dim
        self.A = spec.act_dim
        self.kind = spec.kind
        self.seed = int(seed)
        self.rank = int(rank)
        self.device = torch.device(device)
        self.limit = int(min(spec.time_limit, max_episode_length))
        self.t = 0  # global step counter: RNG key, advances once per vector step
        self.env_idx = torch.arange(self.E, device=self.device, dtype=torch.int64)
        self.key_env = rng.base_key(self.seed, rng.STREAM_ENV, self.rank)
        self.key_term = rng.base_key(self.seed, rng.STREAM_TERM, self.rank)
        self.key_reset = rng.base_key(self.seed, rng.STREAM_RESET, self.rank)
        self.state = torch.zeros(self.E, self.state_dim, device=self.device, dtype=torch.float32)
        self.ep_len = torch.zeros(self.E, device=self.device, dtype=torch.int32)
        self.ep_ret = torch.zeros(self.E, device=self.device, dtype=torch.float32)

    # -- subclass API ----------------------------------------------------------------------
    @property
    def state_dim(self) -> int:
        raise NotImplementedError

    def _reset_state(self, step_key: int) -> torch.Tensor:
        raise NotImplementedError

    def observe(self) -> torch.Tensor:
        raise NotImplementedError

    def _dynamics(self, a: torch.Tensor, step_key: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """returns (new_state, reward, terminal)"""
        raise NotImplementedError

    # -- common ------------------------------------------------------------------------------
    def reset(self) -> torch.Tensor:
        self.state = self._reset_state(0xFFFFFFFF)
        self.ep_len.zero_()
        self.ep_ret.zero_()
        return self.observe()

    @torch.no_grad()
    def step(self, actions: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, Dict]:
        a = actions.to(self.device, torch.float32).reshape(self.E, self.A)
        k = self.t & rng.MASK32
        new_state, reward, terminal = self._dynamics(a, k)
        self.ep_len += 1
        self.ep_ret += reward
        done = terminal | (self.ep_len >= self.limit)
        finished_ret = torch.where(done, self.ep_ret, torch.zeros_like(self.ep_ret))
        finished_len = torch.where(done, self.ep_len, torch.zeros_like(self.ep_len))
        reset_state = self._reset_state(k)
        self.state = torch.where(done[:, None], reset_state, new_state)
        self.ep_len = torch.where(done, torch.zeros_like(self.ep_len), self.ep_len)
        self.ep_ret = torch.where(done, torch.zeros_like(self.ep_ret), self.ep_ret)
        self.t += 1
        info = {"ep_return_sum": finished_ret.sum(), "ep_count": done.sum(),
                "finished_ret": finished_ret, "finished_len": finished_len}
        return self.observe(), reward, done, info

    def kernel_params(self) -> Dict:
        return dict(kind=self.kind, limit=self.limit, key_env=self.key_env,
                    key_term=self.key_term, key_reset=self.key_reset)

    def state_dict(self):
        return {"state": self.state.cpu(), "ep_len": self.ep_len.cpu(), "ep_ret": self.ep_ret.cpu(),
                "t": self.t}

    def load_state_dict(self, d):
        self.state = d["state"].to(self.device)
        self.ep_len = d["ep_len"].to(self.device)
        self.ep_ret = d["ep_ret"].to(self.device)
        self.t = int(d["t"])


class SyntheticEnv(VecEnv):
    """Obs/act-dim-faithful synthetic locomotion task (one per MuJoCo/Bullet name).

    state == observation s in R^O.  With a_c = clamp(a, -1, 1) and w_i = 0.5 + (i mod 7)/7:
        r    = 1 - mean_{j<A} (a_c[j] - tanh(s[j]))^2           (learnable: target is a function of s)
        s'_i = 0.9 s_i + 0.1 tanh(w_i a_c[i mod A]) + 0.05 N(0,1)
        terminal with probability 0.002 per step; reset s ~ 0.1 N(0,1)
    All noise is keyed (seed, rank, env, step, dim) — identical in ``csrc/rollout.hip``.
    """

    @property
    def state_dim(self) -> int:
        return self.O

    def _reset_state(self, step_key: int) -> torch.Tensor:
        d = torch.arange(self.O, device=self.device, dtype=torch.int64)
        g = rng.gauss(self.key_reset, self.env_idx[:, None], step_key, d[None, :])
        return SYN_RESET * g

    def observe(self) -> torch.Tensor:
        return self.state.clone()

    def _dynamics(self, a, step_key):
        s = self.state
        ac = a.clamp(-1.0, 1.0)
        na = min(self.A, self.O)
        err = ac[:, :na] - torch.tanh(s[:, :na])
        reward = 1.0 - (err * err).sum(1) / float(na)
        d = torch.arange(self.O, device=self.device, dtype=torch.int64)
        w = syn_weights(self.O, self.device)
        drive = torch.tanh(w[None, :] * ac[:, (d % self.A)])
        noise = rng.gauss(self.key_env, self.env_idx[:, None], step_key, d[None, :])
        new_s = SYN_DECAY * s + SYN_DRIVE * drive + SYN_NOISE * noise
        u = rng.uniform01(rng.keyed(self.key_term, self.env_idx, step_key,
                                    torch.zeros_like(self.env_idx)))
        terminal = u < SYN_TERM_P
        return new_s, reward, terminal


class PendulumEnv(VecEnv):
    """gym Pendulum-v0 dynamics (g=10, m=l=1, dt=.05, max_speed 8, max_torque 2, 200 steps)."""
    G, M, L, DT, MAX_SPEED, MAX_TORQUE = 10.0, 1.0, 1.0, 0.05, 8.0, 2.0

    @property
    def state_dim(self) -> int:
        return 2

    def _reset_state(self, step_key: int) -> torch.Tensor:
        d = torch.zeros(self.E, dtype=torch.int64, device=self.device)
        u0 = rng.uniform01(rng.keyed(self.key_reset, self.env_idx, step_key, d))
        u1 = rng.uniform01(rng.keyed(self.key_reset, self.env_idx, step_key, d + 1))
        th = (2.0 * u0 - 1.0) * math.pi
        thdot = 2.0 * u1 - 1.0
        return torch.stack([th, thdot], 1)

    def observe(self) -> torch.Tensor:
        th, thdot = self.state[:, 0], self.state[:, 1]
        return torch.stack([torch.cos(th), torch.sin(th), thdot], 1)

    def _dynamics(self, a, step_key):
        th, thdot = self.state[:, 0], self.state[:, 1]
        u = a[:, 0].clamp(-self.MAX_TORQUE, self.MAX_TORQUE)
        thn = torch.remainder(th + math.pi, 2.0 * math.pi) - math.pi
        costs = thn * thn + 0.1 * thdot * thdot + 0.001 * u * u
        newthdot = thdot + (-3.0 * self.G / (2.0 * self.L) * torch.sin(th + math.pi)
                            + 3.0 / (self.M * self.L * self.L) * u) * self.DT
        newth = th + newthdot * self.DT
        newthdot = newthdot.clamp(-self.MAX_SPEED, self.MAX_SPEED)
        terminal = torch.zeros(self.E, dtype=torch.bool, device=self.device)
        return torch.stack([newth, newthdot], 1), -costs, terminal


def make_vec_env(spec: EnvSpec, num_envs: int, seed: int = 1, rank: int = 0, device="cpu",
                 max_episode_length: int = 10000, backend: str = "builtin", name: str = ""):
    """``builtin``: the tensor envs above (stepped in-kernel on the GPU engine); ``gym``: real
    gym envs stepped on the host (envs/gym_adapter.py, ``gym.make`` as main.py:45; ``name`` or
    ``spec.name``)."""
    if backend == "gym":
        from .gym_adapter import GymVecEnv
        return GymVecEnv(name or spec.name, num_envs, seed=seed, rank=rank, max_episode_length=max_episode_length)
    if backend != "builtin":
        raise ValueError(f"env backend must be builtin|gym, got {backend!r}")
    cls = PendulumEnv if spec.kind == KIND_PENDULUM else SyntheticEnv
    return cls(spec, num_envs, seed=seed, rank=rank, device=device,
               max_episode_length=max_episode_length)
