"""Hyper-parameters and CLI.

One dataclass carries every knob of both reference programs:

* preset ``dppo`` reproduces ``Params`` of ``main.py:18-39`` (batch 1000, lr 3e-4,
  4 workers, ``update_treshold = N-1`` …),
* preset ``ppo`` reproduces ``Params`` of ``ppo.py:21-42`` (batch 64, lr 7e-4,
  ent 0.01, max grad norm 0.5, 2048 steps …).

Field names are the reference's (``gae_param``, ``ent_coeff``, ``num_epoch``,
``exploration_size``, ``update_treshold`` — sic, ``main.py:30``; the correctly spelled
``update_threshold`` is accepted as an alias).  The fields after the reference block are
the MI355X-native additions listed in SURVEY.md §5.6.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import warnings
from dataclasses import dataclass, field, fields
from typing import Any, Dict, Optional


@dataclass
class Params:
    # ---- reference fields (main.py:18-39 / ppo.py:21-42) -------------------------------
    batch_size: int = 1000
    lr: float = 3e-4
    gamma: float = 0.99
    gae_param: float = 0.95
    clip: float = 0.2
    ent_coeff: float = 0.0
    num_epoch: int = 10
    num_steps: int = 1000
    exploration_size: int = 1000
    num_processes: int = 4
    update_treshold: Optional[int] = None  # sic (main.py:30); None -> num_processes - 1
    max_episode_length: int = 10000
    seed: int = 1
    env_name: str = "InvertedPendulum-v1"
    time_horizon: int = 1000000          # ppo.py:31 (outer iterations)
    max_grad_norm: Optional[float] = None  # ppo.py:33 uses 0.5; DPPO path has no clipping

    # ---- MI355X-native additions --------------------------------------
    device: str = "cpu"                  # cpu | gpu
    env_backend: str = "builtin"         # builtin (tensor envs, in-kernel on GPU) | gym (gym.make, host-stepped)
    num_envs: int = 1                    # E vectorised envs per worker
    dtype: str = "fp32"                  # fp32 | bf16x3 | bf16 | fp8  (GEMM operand precision;
                                         # bf16x3 = fp32-accurate split-bf16 on the bf16 MFMA)
    hidden: tuple = (100, 100)           # model.py:11-12
    value_mult: int = 5                  # model.py:17 (value fc1 = hidden[0]*5)
    loss: str = "ppo"                    # ppo (corrected, ppo.py:148-167) | dppo_ref (train.py:142-161)
    value_loss: str = "mse"              # mse (ppo.py:164) | clipped_half (train.py:154-157)
    std_convention: str = "std"          # std: exp(log_std) is sigma (ppo.py:93) | var: it is sigma^2 (train.py:89)
    compat: bool = False                 # reproduce reference quirks Q1 (ones grad buffers), Q6 (same seed), Q8 (raw bootstrap)
    grad_reduce: str = "sum"             # sum (model.py:55, chief.py:16) | mean
    obs_norm_update: str = "rollout"     # step (model.py:68 per step) | rollout (one merge per rollout)
    reward_clip: float = 1.0             # train.py:96 clips to +-1; <=0 disables
    normalize_adv: bool = False
    minibatches_per_epoch: int = 0       # 0 = buffer // batch_size (full pass); reference ppo.py uses 1
    total_env_steps: int = 0             # 0 = unbounded (use max_iters)
    max_iters: int = 0                   # 0 = unbounded
    eval_every: int = 0                  # evaluator snapshot period in iterations (0 = off)
    eval_episodes: int = 1
    eval_sleep: float = 0.0              # test.py:63 sleeps 10 s per episode; default no sleep
    checkpoint_dir: str = ""
    checkpoint_every: int = 0
    resume: str = ""
    log_jsonl: str = ""
    log_every: int = 1
    # the last gradient all-reduce overlaps the next rollout.  GPU engine: the value
    # head's last step stays pending until after the next rollout (which reads only the policy:
    # exact); CPU engine: the whole last step (option b, a 1-update policy lag)
    overlap_rollout: bool = False
    # GPU engine, in-stream communicator (the default at N > 1): EVERY epoch's value-head all-reduce
    # + Adam on a side stream (second communicator), joined just before the next value kernel, so
    # it runs beside the next epoch's policy Adam + policy kernel (chief.py:13-20's sum -> Adam ->
    # release off the critical path, once per epoch).  Exact (the policy chain reads no value
    # parameter).  False: stream order (only the last epoch's, with overlap_rollout)
    overlap_value_epochs: bool = False
    dist_timeout_s: float = 300.0
    verify_sync_every: int = 0           # debug param-checksum all-reduce period
    adam_betas: tuple = (0.9, 0.999)
    adam_eps: float = 1e-8
    # ---- observability / failure detection ----------------------
    log_csv: str = ""                    # learning-curve CSV (rank 0), the figs/*.png analogue
    profile_dir: str = ""                # torch.profiler chrome traces (host + HIP timeline) per rank
    profile_iters: str = "2:4"           # [start:stop) iterations captured when profile_dir is set
    heartbeat_s: float = -1.0            # per-rank heartbeat in the rendezvous store every N s (<0: auto =
                                         # 5 s whenever world_size > 1; 0: off)
    heartbeat_timeout_s: float = 60.0    # a peer silent this long is reported dead: abort + exit 75
    check_finite: bool = False           # debug: stop with the failing phase when loss/params go non-finite
    phase_timing: int = 1                # per-phase HIP-event timing every N iterations (0 = off; each
                                         # event record idles the GPU ~10 us, see PhaseTimer)
    # ---- execution options (the GPU engine's paths; A/B switches of earlier rounds) ----------
    dist_backend: str = "auto"           # auto: nccl (RCCL) on gpu, gloo on cpu | nccl | gloo (GPU ranks
                                         # sharing one device: the 1-GPU box's multi-rank runs)
    grad_comm: str = "auto"              # auto: in-stream communicator when available (csrc/comm.cpp RCCL;
                                         # gloo adapter) | native (required) | process_group (torch's)
    update_kernels: str = "auto"         # auto | heads (per-head streaming kernels, csrc/mlp_head.hip) |
                                         # tile (one-kernel update, csrc/mlp.hip)
    fused_apply: bool = True             # world size 1: gradient gather + Adam in one launch
    fp8_wgrad_operands: bool = True      # dtype fp8 on the per-head path: e4m3 wgrad operands (else bf16)
    fp8_policy_gemms: bool = False       # dtype fp8: the policy head's fc1 / fc2 on the e4m3 x128 MFMA too (opt-in:
                                         # speed-neutral and 3x the policy-gradient error, profiles/r4/fp8_heads.md)
    stats_stream: str = "off"            # off | on | auto (on when an all-reduce sits in the chain): the
                                         # obs-stat reduce / all-reduce / merge on a side stream
    wgrad_wgs: int = 0                   # wgrad tasks per launch (0: one per CU of the device)
    wgrad_wide: bool = True              # wgrad tiles of up to 16 quadrants, two per wave (split-bf16 / bf16;
                                         # csrc/wgrad.hip)
    phead_kernel: bool = True            # the policy head on the 32x32 kernel (csrc/phead.hip)
    phead_fused_dw2: str = "auto"        # auto | on | off: ... summing p_fc2's weight gradient in the kernel
                                         # (auto: at bf16x3 only, the measured-faster choice per dtype)
    mlp_rows: int = 0                    # diagnostics: force the tile update kernel's row tile (0: auto)

    # ------------------------------------------------------------------------------------
    def __post_init__(self):
        if self.update_treshold is None:
            self.update_treshold = self.num_processes - 1
        elif self.update_treshold != self.num_processes - 1:
            # chief.py:13 fires when counter > threshold, i.e. with threshold+1 of N workers'
            # gradients.  The synchronous RCCL all-reduce always combines all N ranks, so a
            # smaller threshold (straggler tolerance) cannot be honoured: say so, do not no-op.
            warnings.warn(f"update_treshold={self.update_treshold} is inert: the gradient all-reduce is "
                          f"synchronous over all num_processes={self.num_processes} ranks (reference "
                          f"default N-1 = {self.num_processes - 1})", UserWarning, stacklevel=3)
        self.hidden = tuple(int(h) for h in self.hidden)
        self.adam_betas = tuple(float(b) for b in self.adam_betas)
        if self.device not in ("cpu", "gpu"):
            raise ValueError(f"device must be cpu|gpu, got {self.device}")
        if self.env_backend not in ("builtin", "gym"):
            raise ValueError(f"env_backend must be builtin|gym, got {self.env_backend}")
        if self.dtype not in ("fp32", "bf16x3", "bf16", "fp8"):
            raise ValueError(f"dtype must be fp32|bf16x3|bf16|fp8, got {self.dtype}")
        if self.phead_fused_dw2 not in ("auto", "on", "off"):
            raise ValueError(f"phead_fused_dw2 must be auto|on|off, got {self.phead_fused_dw2}")
        if self.loss not in ("ppo", "dppo_ref"):
            raise ValueError(f"loss must be ppo|dppo_ref, got {self.loss}")
        if self.value_loss not in ("mse", "clipped_half"):
            raise ValueError(f"value_loss must be mse|clipped_half, got {self.value_loss}")
        if self.std_convention not in ("std", "var"):
            raise ValueError("std_convention must be std|var")
        if self.grad_reduce not in ("sum", "mean"):
            raise ValueError("grad_reduce must be sum|mean")
        if self.loss == "dppo_ref":
            # train.py:88-89,143-146 treat exp(log_std) as the variance everywhere
            self.std_convention = "var"
        if self.obs_norm_update not in ("step", "rollout"):
            raise ValueError("obs_norm_update must be step|rollout")
        for name, ok in (("dist_backend", ("auto", "nccl", "gloo")), ("grad_comm", ("auto", "native", "process_group")),
                         ("update_kernels", ("auto", "heads", "tile")), ("stats_stream", ("off", "on", "auto"))):
            if getattr(self, name) not in ok:
                raise ValueError(f"{name} must be {'|'.join(ok)}, got {getattr(self, name)}")

    def heartbeat_interval(self, world_size: int) -> float:
        """the heartbeat period in effect: heartbeat_s, or 5 s (auto) whenever there are peers"""
        if self.heartbeat_s >= 0:
            return float(self.heartbeat_s)
        return 5.0 if world_size > 1 else 0.0

    # alias with the correct spelling
    @property
    def update_threshold(self) -> int:
        return self.update_treshold

    @update_threshold.setter
    def update_threshold(self, v: int) -> None:
        self.update_treshold = v

    # rollout geometry: T steps x E envs per worker --------------------------------------
    @property
    def rollout_len(self) -> int:
        """T: steps per env per iteration so that T*E ~= exploration_size."""
        return max(1, -(-self.exploration_size // max(1, self.num_envs)))

    @property
    def buffer_rows(self) -> int:
        return self.rollout_len * self.num_envs

    def gae_segment(self) -> int:
        """the reference's segment length num_steps (train.py:82, ppo.py:87) when it cuts the
        T-step rollout (0 otherwise): GAE restarts after every num_steps steps, bootstrapping
        the not-done state (ops/oracle.gae, csrc/optim.hip gae kernels)"""
        return self.num_steps if 0 < self.num_steps < self.rollout_len else 0

    def minibatch_rows(self) -> int:
        return max(1, min(self.batch_size, self.buffer_rows))

    def num_minibatches(self) -> int:
        if self.minibatches_per_epoch > 0:
            return self.minibatches_per_epoch
        return max(1, self.buffer_rows // self.minibatch_rows())

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d["hidden"] = list(self.hidden)
        d["adam_betas"] = list(self.adam_betas)
        return d

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Params":
        d = dict(d)
        if "update_threshold" in d:
            d["update_treshold"] = d.pop("update_threshold")
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})


def dppo_preset(**overrides) -> Params:
    """``main.py:18-39`` values."""
    p = dict(batch_size=1000, lr=3e-4, gamma=0.99, gae_param=0.95, clip=0.2, ent_coeff=0.0,
             num_epoch=10, num_steps=1000, exploration_size=1000, num_processes=4,
             max_episode_length=10000, seed=1, env_name="InvertedPendulum-v1",
             max_grad_norm=None, loss="ppo", value_loss="clipped_half", std_convention="std")
    p.update(overrides)
    return Params(**p)


def ppo_preset(**overrides) -> Params:
    """``ppo.py:21-42`` values (single process)."""
    p = dict(batch_size=64, lr=7e-4, gamma=0.99, gae_param=0.95, clip=0.2, ent_coeff=0.01,
             num_epoch=10, num_steps=2048, exploration_size=2048, time_horizon=1000000,
             max_episode_length=10000, max_grad_norm=0.5, seed=1, env_name="HalfCheetah-v1",
             num_processes=1, loss="ppo", value_loss="mse", std_convention="std",
             minibatches_per_epoch=1)
    p.update(overrides)
    return Params(**p)


PRESETS = {"dppo": dppo_preset, "ppo": ppo_preset}


def _parse_bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "y", "on")


def build_arg_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="MI355X-native DPPO / PPO trainer")
    ap.add_argument("--preset", choices=sorted(PRESETS), default="dppo")
    for f in fields(Params):
        flag = "--" + f.name.replace("_", "-")
        default = None
        if f.name == "hidden" or f.name == "adam_betas":
            ap.add_argument(flag, type=str, default=default, help=f"comma list (default preset)")
        elif f.type in ("bool", bool):
            ap.add_argument(flag, type=_parse_bool, default=default, nargs="?", const=True)
        elif f.name in ("update_treshold",):
            ap.add_argument(flag, "--update-threshold", type=int, default=default)
        elif f.name == "max_grad_norm":
            ap.add_argument(flag, type=float, default=default)
        else:
            t = {"int": int, "float": float, "str": str}.get(str(f.type), None)
            if t is None:
                t = type(f.default) if f.default is not None else str
            ap.add_argument(flag, type=t, default=default)
    return ap


def params_from_args(argv=None) -> Params:
    ap = build_arg_parser()
    ns = ap.parse_args(argv)
    overrides = {}
    for f in fields(Params):
        v = getattr(ns, f.name, None)
        if v is None:
            continue
        if f.name in ("hidden", "adam_betas"):
            v = tuple(float(x) if f.name == "adam_betas" else int(x) for x in str(v).split(","))
        overrides[f.name] = v
    return PRESETS[ns.preset](**overrides)
