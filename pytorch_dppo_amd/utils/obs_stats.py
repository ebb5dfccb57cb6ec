"""Running observation statistics (the reference ``Shared_obs_stats``, ``model.py:61-80``).

Reference semantics per observation x (``model.py:68-75``)::

    n += 1; mean += (x - mean)/n; mean_diff += (x - mean_old)*(x - mean); var = clamp(mean_diff/n, 1e-2)
    normalize(x) = clamp((x - mean)/sqrt(var), -5, 5)

Here the state is fp64 and updated by exact batched merges (Chan et al.) of batch moments
taken around a shift (the current mean), which equals the sequential Welford recurrence up
to rounding.  The reference's shared-memory RMW races are replaced by one
deterministic merge of every rank's moments (an all-reduce of ``(count, S1, S2)`` about the
common shift — :func:`pytorch_dppo_amd.parallel.dist.allreduce_obs_moments`).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

VAR_FLOOR = 1e-2
CLIP = 5.0


class RunningObsStats:
    def __init__(self, num_inputs: int, device="cpu"):
        self.O = int(num_inputs)
        self.device = torch.device(device)
        self.n = 0.0
        self.mean = torch.zeros(self.O, dtype=torch.float64, device=self.device)
        self.mean_diff = torch.zeros(self.O, dtype=torch.float64, device=self.device)
        # fp32 images consumed by the normalisation prologue of the kernels
        self.mean_f32 = torch.zeros(self.O, dtype=torch.float32, device=self.device)
        self.inv_std_f32 = torch.ones(self.O, dtype=torch.float32, device=self.device)
        # optional fused device merge (set by the HIP engine: csrc/obs.hip obs_merge); called as
        # fn(s1, s2, count, n_a, shift) and updates mean / mean_diff / fp32 images in place
        self.device_merge = None
        self._refresh()

    @property
    def var(self) -> torch.Tensor:
        if self.n <= 0:
            return torch.full_like(self.mean, VAR_FLOOR)
        return torch.clamp(self.mean_diff / self.n, min=VAR_FLOOR)

    def _refresh(self) -> None:
        self.mean_f32.copy_(self.mean.to(torch.float32))
        self.inv_std_f32.copy_(torch.rsqrt(self.var).to(torch.float32))

    # -- moments -------------------------------------------------------------------------
    def shift(self) -> torch.Tensor:
        """the common shift every rank takes its moments about (fp32 current mean)."""
        return self.mean_f32

    @staticmethod
    def moments(x: torch.Tensor, shift: torch.Tensor) -> Tuple[float, torch.Tensor, torch.Tensor]:
        """(count, S1 = sum(x - shift), S2 = sum((x - shift)^2)) in fp64."""
        d = x.reshape(-1, x.shape[-1]).to(torch.float64) - shift.to(torch.float64)
        return float(d.shape[0]), d.sum(0), (d * d).sum(0)

    def merge_moments(self, count: float, s1: torch.Tensor, s2: torch.Tensor,
                      shift: torch.Tensor) -> None:
        """Chan merge of a batch given by its moments about ``shift``."""
        if count <= 0:
            return
        if self.device_merge is not None and s1.is_cuda:
            self.device_merge(s1, s2, float(count), float(self.n), shift)
            self.n = self.n + count
            return
        s1 = s1.to(self.device, torch.float64)
        s2 = s2.to(self.device, torch.float64)
        shift = shift.to(self.device, torch.float64)
        bmean_d = s1 / count
        bmean = shift + bmean_d
        bm2 = torch.clamp(s2 - s1 * bmean_d, min=0.0)
        n_a, n_b = self.n, count
        n = n_a + n_b
        delta = bmean - self.mean
        self.mean = self.mean + delta * (n_b / n)
        self.mean_diff = self.mean_diff + bm2 + delta * delta * (n_a * n_b / n)
        self.n = n
        self._refresh()

    def observes(self, obs: torch.Tensor) -> None:
        """update with a batch [B,O] (or one obs [O] / [1,O]) — model.py:68."""
        x = obs.reshape(-1, self.O)
        c, s1, s2 = self.moments(x, self.shift())
        self.merge_moments(c, s1, s2, self.shift())

    def normalize(self, inputs: torch.Tensor) -> torch.Tensor:
        """clamp((x-mean)/sqrt(var), -5, 5) — model.py:77-80 (fp32)."""
        m = self.mean_f32.to(inputs.device)
        s = self.inv_std_f32.to(inputs.device)
        return torch.clamp((inputs - m) * s, -CLIP, CLIP)

    # -- persistence (reference attribute names, model.py:63-66) -------------------------------
    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {"n": torch.full((self.O,), self.n, dtype=torch.float64),
                "mean": self.mean.cpu().clone(), "mean_diff": self.mean_diff.cpu().clone(),
                "var": self.var.cpu().clone()}

    def load_state_dict(self, d: Dict[str, torch.Tensor]) -> None:
        n = d["n"]
        self.n = float(n.reshape(-1)[0]) if torch.is_tensor(n) else float(n)
        self.mean = d["mean"].to(self.device, torch.float64).clone()
        self.mean_diff = d["mean_diff"].to(self.device, torch.float64).clone()
        self._refresh()

    def copy_from(self, other: "RunningObsStats") -> None:
        self.n = other.n
        self.mean = other.mean.to(self.device).clone()
        self.mean_diff = other.mean_diff.to(self.device).clone()
        self._refresh()
