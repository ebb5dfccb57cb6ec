"""Optional adapter for real gym envs (``gym.make``, as ``main.py:45`` / ``train.py:48``).

gym / mujoco_py / pybullet are not installed in this image; the adapter is import-gated
and only used when ``--env-backend gym`` is requested and ``gym`` imports.  It exposes the
same ``reset/step`` surface as :class:`~pytorch_dppo_amd.envs.vec_env.VecEnv` (CPU tensors,
E independent gym envs stepped in a python loop, auto-reset on done like ``train.py:98-105``).
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch


def gym_available() -> bool:
    try:
        import gym  # noqa: F401
        return True
    except Exception:
        return False


class GymVecEnv:
    def __init__(self, name: str, num_envs: int, seed: int = 1, rank: int = 0,
                 max_episode_length: int = 10000):
        import gym
        self.envs = [gym.make(name) for _ in range(num_envs)]
        for i, e in enumerate(self.envs):
            try:
                e.seed(seed + 1000 * rank + i)
            except Exception:
                pass
        self.E = num_envs
        self.O = self.envs[0].observation_space.shape[0]
        self.A = self.envs[0].action_space.shape[0]
        self.limit = max_episode_length
        self.device = torch.device("cpu")
        self.ep_len = np.zeros(num_envs, dtype=np.int64)
        self.ep_ret = np.zeros(num_envs, dtype=np.float64)
        self.t = 0

    def _obs(self, o):
        return np.asarray(o[0] if isinstance(o, tuple) else o, dtype=np.float32)

    def reset(self) -> torch.Tensor:
        self._last = np.stack([self._obs(e.reset()) for e in self.envs])
        self.ep_len[:] = 0
        self.ep_ret[:] = 0
        return torch.from_numpy(self._last.copy())

    def step(self, actions: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, Dict]:
        acts = actions.detach().cpu().numpy()
        obs, rew, done = [], [], []
        fin_ret = np.zeros(self.E, dtype=np.float32)
        for i, e in enumerate(self.envs):
            out = e.step(acts[i])
            o, r, d = out[0], out[1], out[2]
            if len(out) == 5:
                d = out[2] or out[3]
            self.ep_len[i] += 1
            self.ep_ret[i] += r
            d = bool(d) or self.ep_len[i] >= self.limit
            if d:
                fin_ret[i] = self.ep_ret[i]
                self.ep_len[i] = 0
                self.ep_ret[i] = 0
                o = e.reset()
            obs.append(self._obs(o))
            rew.append(r)
            done.append(d)
        self.t += 1
        done_t = torch.tensor(done)
        info = {"ep_return_sum": torch.tensor(float(fin_ret.sum())), "ep_count": done_t.sum(),
                "finished_ret": torch.from_numpy(fin_ret)}
        return (torch.from_numpy(np.stack(obs)), torch.tensor(rew, dtype=torch.float32), done_t, info)
