"""Metrics / observability.

The reference only ``print``s (``test.py:56-59``, ``ppo.py:177``).  Here rank 0 writes one
JSONL record per iteration (iteration, env_steps, steps/s, per-phase ms, loss terms, clip
fraction, approx-KL, mean episode return) and per-phase timing uses HIP events on GPU (no
host sync inside the timed phases) or ``perf_counter`` on CPU.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import torch


class PhaseTimer:
    def __init__(self, device: torch.device):
        self.gpu = device.type == "cuda"
        self._open: Dict[str, object] = {}
        self._done: Dict[str, list] = {}

    def start(self, name: str) -> None:
        if self.gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._open[name] = ev
        else:
            self._open[name] = time.perf_counter()

    def stop(self, name: str) -> None:
        s = self._open.pop(name)
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._done.setdefault(name, []).append((s, e))
        else:
            self._done.setdefault(name, []).append((time.perf_counter() - s) * 1e3)

    def summary(self) -> Dict[str, float]:
        out = {}
        for k, lst in self._done.items():
            if self.gpu:
                torch.cuda.synchronize()
                out[f"ms_{k}"] = sum(s.elapsed_time(e) for s, e in lst)
            else:
                out[f"ms_{k}"] = sum(lst)
        self._done = {}
        return out


class MetricsLogger:
    def __init__(self, path: str = "", enabled: bool = True, stdout: bool = True):
        self.enabled = enabled
        self.stdout = stdout
        self.f = None
        if enabled and path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a")

    def log(self, rec: Dict) -> None:
        if not self.enabled:
            return
        rec = {k: (float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) else v)
               for k, v in rec.items()}
        if self.f:
            self.f.write(json.dumps(rec) + "\n")
            self.f.flush()
        if self.stdout:
            it = int(rec.get("iteration", 0))
            print(f"iter {it} env_steps {int(rec.get('env_steps', 0))} "
                  f"steps/s {rec.get('steps_per_s', 0):.1f} "
                  f"av_reward {rec.get('mean_ep_return', float('nan')):.3f} "
                  f"loss {rec.get('loss', float('nan')):.4f}", flush=True)

    def close(self) -> None:
        if self.f:
            self.f.close()
            self.f = None
