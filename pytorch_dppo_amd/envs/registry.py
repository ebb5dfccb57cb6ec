"""Env registry: every env name the reference mentions, with gym's observation/action dims.

The reference picks an env by commenting lines (``main.py:33-39``, ``ppo.py:35-42``) and
runs it through ``gym.make`` (MuJoCo / PyBullet).  Neither is installed in this image, so an
env name resolves to

* ``pendulum`` — a faithful vectorised Pendulum-v0 (gym's dynamics; CPU torch + HIP), or
* ``synthetic`` — an obs/act-dim-faithful synthetic locomotion task (CPU torch + HIP),
  used for every MuJoCo/Bullet name, or
* ``gym`` — the real env through :mod:`pytorch_dppo_amd.envs.gym_adapter` with
  ``--env-backend gym`` (``gym.make``, or a factory installed with ``register_env``); its dims
  come from the env's spaces (:func:`host_spec`).

Dims are gym facts (SURVEY.md §2.6 [ext]).
"""
from __future__ import annotations

from dataclasses import dataclass

KIND_SYNTHETIC = 0
KIND_PENDULUM = 1
KIND_HOST = 2          # a host-stepped env (gym backend): dims come from the env itself


@dataclass(frozen=True)
class EnvSpec:
    name: str
    obs_dim: int
    act_dim: int
    kind: int
    time_limit: int       # gym TimeLimit max_episode_steps


_SPECS = {}


def _reg(names, obs, act, kind, limit):
    for n in names:
        _SPECS[n] = EnvSpec(n, obs, act, kind, limit)


_reg(["Pendulum-v0", "Pendulum-v1"], 3, 1, KIND_PENDULUM, 200)
_reg(["InvertedPendulum-v1", "InvertedPendulum-v2"], 4, 1, KIND_SYNTHETIC, 1000)
_reg(["InvertedDoublePendulum-v1", "InvertedDoublePendulum-v2"], 11, 1, KIND_SYNTHETIC, 1000)
_reg(["Reacher-v1", "Reacher-v2"], 11, 2, KIND_SYNTHETIC, 50)
_reg(["Hopper-v1", "Hopper-v2"], 11, 3, KIND_SYNTHETIC, 1000)
_reg(["HalfCheetah-v1", "HalfCheetah-v2"], 17, 6, KIND_SYNTHETIC, 1000)
_reg(["Walker2d-v1", "Walker2d-v2"], 17, 6, KIND_SYNTHETIC, 1000)
_reg(["Ant-v1", "Ant-v2"], 111, 8, KIND_SYNTHETIC, 1000)
_reg(["Humanoid-v1", "Humanoid-v2"], 376, 17, KIND_SYNTHETIC, 1000)
_reg(["HalfCheetahBulletEnv-v0"], 26, 6, KIND_SYNTHETIC, 1000)
_reg(["HopperBulletEnv-v0"], 15, 3, KIND_SYNTHETIC, 1000)
_reg(["AntBulletEnv-v0"], 28, 8, KIND_SYNTHETIC, 1000)


def host_spec(name: str, obs_dim: int, act_dim: int, limit: int) -> EnvSpec:
    """spec of a host-stepped env (``--env-backend gym``) built from the env's own spaces"""
    return EnvSpec(name, int(obs_dim), int(act_dim), KIND_HOST, int(limit))


def get_spec(name: str) -> EnvSpec:
    if name in _SPECS:
        return _SPECS[name]
    if name.startswith("Synthetic-"):
        # Synthetic-<obs>x<act>
        o, a = name[len("Synthetic-"):].split("x")
        return EnvSpec(name, int(o), int(a), KIND_SYNTHETIC, 1000)
    raise KeyError(f"unknown env {name!r}; known: {sorted(_SPECS)}")


def known_envs():
    return sorted(_SPECS)
