"""Real gym environments (``gym.make``, as the reference builds every env: ``main.py:45``,
``train.py:48``, ``test.py:28``, ``ppo.py:191``) behind the vectorised-env surface.

``--env-backend gym`` routes :func:`~pytorch_dppo_amd.envs.vec_env.make_vec_env` here:
:class:`GymVecEnv` owns E independent gym envs stepped in a host loop, auto-resetting on done
like ``train.py:98-105`` (terminal, gym's ``TimeLimit`` truncation or ``max_episode_length``,
counted per step), and exposes what the engines use — ``E/O/A``, ``t``, ``env_idx`` (action-noise
keys), ``reset/step/observe``, ``state_dict``.  Such an env cannot be stepped inside the GPU
rollout kernel, so ``host_stepped`` tells :class:`~pytorch_dppo_amd.runtime.engine_hip.HipEngine`
to take its host-env rollout path (the update still runs on the HIP kernels).

gym / mujoco_py / pybullet are not installed in this image.  ``gym.make`` is the default env
factory; :func:`register_env` installs another factory for a name (any object with gym's
``reset() -> obs`` / ``step(a) -> (obs, r, done, info)`` API, old or new gym style, and
``observation_space.shape`` / ``action_space.shape``) — the tests use that to exercise this
path with an in-test env.  Parity with the reference's MuJoCo results is unpinned here.
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import numpy as np
import torch

_FACTORIES: Dict[str, Callable[[], object]] = {}


def register_env(name: str, factory: Callable[[], object]) -> None:
    """``GymVecEnv(name)`` builds its envs with ``factory()`` instead of ``gym.make(name)``."""
    _FACTORIES[name] = factory


def gym_available() -> bool:
    try:
        import gym  # noqa: F401
        return True
    except Exception:
        return False


def _make(name: str):
    if name in _FACTORIES:
        return _FACTORIES[name]()
    try:
        import gym
    except Exception as e:
        raise RuntimeError(f"--env-backend gym needs the gym package for {name!r} (not installed here); "
                           "use the builtin backend or register_env() a factory") from e
    return gym.make(name)


class GymVecEnv:
    host_stepped = True        # stepped on the host: no in-kernel dynamics (HipEngine checks it)

    def __init__(self, name: str, num_envs: int, seed: int = 1, rank: int = 0,
                 max_episode_length: int = 10000):
        self.name = name
        self.envs = [_make(name) for _ in range(num_envs)]
        for i, e in enumerate(self.envs):
            try:
                e.seed(seed + 1000 * rank + i)          # old gym API; new API seeds via reset
            except Exception:
                pass
        self.E = int(num_envs)
        self.O = int(self.envs[0].observation_space.shape[0])
        self.A = int(self.envs[0].action_space.shape[0])
        limit = getattr(getattr(self.envs[0], "spec", None), "max_episode_steps", None)
        self.limit = int(min(limit or max_episode_length, max_episode_length))
        self.device = torch.device("cpu")
        self.seed, self.rank = int(seed), int(rank)
        self.env_idx = torch.arange(self.E, dtype=torch.int64)
        self.ep_len = np.zeros(self.E, dtype=np.int64)
        self.ep_ret = np.zeros(self.E, dtype=np.float64)
        self.t = 0
        self._last = np.zeros((self.E, self.O), dtype=np.float32)

    @staticmethod
    def _obs(o) -> np.ndarray:
        # new-style gym returns (obs, info) from reset
        return np.asarray(o[0] if isinstance(o, tuple) else o, dtype=np.float32).reshape(-1)

    def reset(self) -> torch.Tensor:
        self._last = np.stack([self._obs(e.reset()) for e in self.envs])
        self.ep_len[:] = 0
        self.ep_ret[:] = 0
        return self.observe()

    def observe(self) -> torch.Tensor:
        return torch.from_numpy(self._last.copy())

    def step(self, actions: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, Dict]:
        acts = actions.detach().to("cpu", torch.float32).reshape(self.E, self.A).numpy()
        obs, rew, done = [], [], []
        fin_ret = np.zeros(self.E, dtype=np.float32)
        fin_len = np.zeros(self.E, dtype=np.int32)
        for i, e in enumerate(self.envs):
            out = e.step(acts[i])               # unclipped action (train.py:92-93)
            o, r, d = out[0], float(out[1]), bool(out[2])
            if len(out) == 5:                   # new API: (obs, r, terminated, truncated, info)
                d = bool(out[2]) or bool(out[3])
            self.ep_len[i] += 1
            self.ep_ret[i] += r
            d = d or self.ep_len[i] >= self.limit
            if d:
                fin_ret[i] = self.ep_ret[i]
                fin_len[i] = self.ep_len[i]
                self.ep_len[i] = 0
                self.ep_ret[i] = 0.0
                o = e.reset()                   # train.py:98-105
            obs.append(self._obs(o))
            rew.append(r)
            done.append(d)
        self.t += 1
        self._last = np.stack(obs)
        done_t = torch.tensor(done)
        info = {"ep_return_sum": torch.tensor(float(fin_ret.sum())), "ep_count": done_t.sum(),
                "finished_ret": torch.from_numpy(fin_ret), "finished_len": torch.from_numpy(fin_len)}
        return self.observe(), torch.tensor(rew, dtype=torch.float32), done_t, info

    def kernel_params(self) -> Dict:
        raise RuntimeError("a gym env is stepped on the host; it has no in-kernel dynamics")

    def state_dict(self) -> Dict:
        # the simulators' internal state is not serialisable through gym's API: a resumed run
        # resets its envs (episode counters restart), everything else resumes exactly
        return {"t": self.t, "host_env": self.name}

    def load_state_dict(self, d: Dict) -> None:
        self.t = int(d.get("t", 0))
        self.reset()
