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
    """Per-phase wall time: HIP events on GPU (read once per iteration), perf_counter on CPU.

    With ``annotate`` each phase is also a ``torch.profiler`` range, so the chrome traces of
    ``--profile-dir`` show rollout / obs_stats / values_gae / update around the HIP kernels."""

    def __init__(self, device: torch.device, annotate: bool = False):
        self.gpu = device.type == "cuda"
        self.annotate = annotate
        # off: start/stop record nothing.  Each timed HIP event record costs ~10 us of GPU idle
        # at its position in the stream (rocprofv3 timeline: a gap at every phase boundary), so
        # the worker samples the phases every ``phase_timing`` iterations.
        self.enabled = True
        self._open: Dict[str, object] = {}
        self._ranges: Dict[str, object] = {}
        self._done: Dict[str, list] = {}

    def start(self, name: str) -> None:
        if not self.enabled:
            return
        if self.annotate:
            r = torch.autograd.profiler.record_function(name)
            r.__enter__()
            self._ranges[name] = r
        if self.gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._open[name] = ev
        else:
            self._open[name] = time.perf_counter()

    def stop(self, name: str) -> None:
        if not self.enabled:
            return
        r = self._ranges.pop(name, None)
        if r is not None:
            r.__exit__(None, None, None)
        s = self._open.pop(name)
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._done.setdefault(name, []).append((s, e))
        else:
            self._done.setdefault(name, []).append((time.perf_counter() - s) * 1e3)

    def collect(self):
        """hand over this iteration's finished phases (events are read later, see ``elapsed``)."""
        done, self._done = self._done, {}
        return (self.gpu, done)

    @staticmethod
    def elapsed(collected) -> Dict[str, float]:
        gpu, done = collected
        out = {}
        for k, lst in done.items():
            if gpu:
                for _, e in lst:
                    e.synchronize()
                out[f"ms_{k}"] = sum(s.elapsed_time(e) for s, e in lst)
            else:
                out[f"ms_{k}"] = sum(lst)
        return out

    def summary(self) -> Dict[str, float]:
        return PhaseTimer.elapsed(self.collect())


CSV_COLUMNS = ("iteration", "env_steps", "updates", "steps_per_s", "mean_ep_return", "ep_count", "loss",
               "loss_clip", "loss_value", "loss_ent", "approx_kl", "clipfrac", "grad_norm")


class MetricsLogger:
    """Rank-0 JSONL (every field) + optional learning-curve CSV (fixed columns) + stdout line."""

    def __init__(self, path: str = "", enabled: bool = True, stdout: bool = True, csv_path: str = ""):
        self.enabled = enabled
        self.stdout = stdout
        self.f = None
        self.csv = None
        if enabled and path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a")
        if enabled and csv_path:
            os.makedirs(os.path.dirname(os.path.abspath(csv_path)), exist_ok=True)
            fresh = not os.path.exists(csv_path) or os.path.getsize(csv_path) == 0
            self.csv = open(csv_path, "a")
            if fresh:
                self.csv.write(",".join(CSV_COLUMNS) + "\n")

    def log(self, rec: Dict) -> None:
        if not self.enabled:
            return
        rec = {k: (float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) else v)
               for k, v in rec.items()}
        if self.f:
            self.f.write(json.dumps(rec) + "\n")
            self.f.flush()
        if self.csv:
            self.csv.write(",".join("" if rec.get(c) is None else repr(rec[c]) for c in CSV_COLUMNS) + "\n")
            self.csv.flush()
        if self.stdout:
            it = int(rec.get("iteration", 0))
            print(f"iter {it} env_steps {int(rec.get('env_steps', 0))} "
                  f"steps/s {rec.get('steps_per_s', 0):.1f} "
                  f"av_reward {rec.get('mean_ep_return', float('nan')):.3f} "
                  f"loss {rec.get('loss', float('nan')):.4f}", flush=True)

    def close(self) -> None:
        for name in ("f", "csv"):
            fh = getattr(self, name)
            if fh:
                fh.close()
                setattr(self, name, None)
