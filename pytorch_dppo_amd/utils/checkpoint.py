"""Checkpoint / resume (the reference has none).

* ``model.pt``          — pure fp32 ``state_dict`` with the reference keys/shapes
                          (``model.py``); loads into the reference ``Model`` with strict=True.
* ``trainer_state.pt``  — Adam moments + step, obs stats (reference names ``n, mean,
                          mean_diff, var``, ``model.py:63-66``), counters, config.
* ``env_rank{r}.pt``    — each rank's vectorised env state (so a resumed run continues the
                          same trajectories).
Everything is plain tensors / python scalars, loadable with ``weights_only=True``.
Writes are atomic (tmp + rename) and done by rank 0 (env files by their rank).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch


def _atomic_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_checkpoint(ckpt_dir: str, model_sd: Dict, trainer_state: Optional[Dict], rank: int,
                    env_state: Optional[Dict] = None) -> None:
    os.makedirs(ckpt_dir, exist_ok=True)
    if rank == 0:
        _atomic_save(model_sd, os.path.join(ckpt_dir, "model.pt"))
        if trainer_state is not None:
            _atomic_save(trainer_state, os.path.join(ckpt_dir, "trainer_state.pt"))
    if env_state is not None:
        _atomic_save(env_state, os.path.join(ckpt_dir, f"env_rank{rank}.pt"))


def load_model_state(ckpt_dir: str) -> Dict:
    return torch.load(os.path.join(ckpt_dir, "model.pt"), map_location="cpu", weights_only=True)


def load_trainer_state(ckpt_dir: str) -> Optional[Dict]:
    p = os.path.join(ckpt_dir, "trainer_state.pt")
    if not os.path.exists(p):
        return None
    return torch.load(p, map_location="cpu", weights_only=True)


def load_env_state(ckpt_dir: str, rank: int) -> Optional[Dict]:
    p = os.path.join(ckpt_dir, f"env_rank{rank}.pt")
    if not os.path.exists(p):
        return None
    return torch.load(p, map_location="cpu", weights_only=True)
