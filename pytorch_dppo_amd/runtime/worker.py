"""The DPPO worker loop (one per process / GPU): the reference's worker + chief fused.

Reference roles:

* ``train.py:46-178`` worker: sync weights → collect ≥1000 steps → GAE → 10 epochs of
  {minibatch loss, backward, push grads, increment counter, spin on the traffic light},
* ``chief.py:7-21``: poll every 1 s, when all N grads are in → Adam step → release.

Here every rank runs the SAME loop: rollout → (obs-stat all-reduce) → values → GAE →
for each epoch/minibatch {grad → all-reduce(sum) → clip → Adam}.  Because the all-reduce
delivers the identical summed gradient to every rank and every rank applies the identical
fused Adam step, parameters stay bit-identical without a chief process or a broadcast
(replicated optimizer; checked by ``verify_sync_every``).  The 1 s chief poll (Q13) and the
busy-spin (Q14) disappear: a step costs compute + one collective.
"""
from __future__ import annotations

import contextlib
import json
import math
import os
import sys
import time
from typing import Dict, Optional

import torch

from ..config import Params
from ..envs import get_spec, host_spec, make_vec_env
from ..models.actor_critic import ActorCritic
from ..parallel.dist import DistContext
from ..utils import rng
from ..utils.metrics import MetricsLogger, PhaseTimer
from ..utils.obs_stats import RunningObsStats


def build_engine(params: Params, model, env, stats, device, action_rank):
    if params.device == "gpu":
        from .engine_hip import HipEngine
        return HipEngine(params, model, env, stats, device, action_rank)
    from .engine_torch import TorchEngine
    return TorchEngine(params, model, env, stats, device, action_rank)


class DPPOWorker:
    def __init__(self, params: Params, ctx: DistContext, log: Optional[MetricsLogger] = None):
        self.p = params
        self.ctx = ctx
        self.device = ctx.device
        if params.env_backend == "gym":
            # real gym envs (main.py:45 / train.py:48): dims from the env's own spaces
            self.env = make_vec_env(None, params.num_envs, seed=params.seed, rank=ctx.rank,
                                    max_episode_length=params.max_episode_length, backend="gym",
                                    name=params.env_name)
            self.spec = host_spec(params.env_name, self.env.O, self.env.A, self.env.limit)
        else:
            self.spec = get_spec(params.env_name)
        torch.manual_seed(params.seed)          # main.py:44 — identical init on every rank
        self.model = ActorCritic(self.spec.obs_dim, self.spec.act_dim, params.hidden,
                                 params.value_mult).to(self.device)
        self.ctx.broadcast_(self.model.flat.data, src=0)   # R3 once at start
        action_rank = 0 if params.compat else ctx.rank     # Q6: reference workers share the seed
        if params.env_backend != "gym":
            self.env = make_vec_env(self.spec, params.num_envs, seed=params.seed, rank=ctx.rank,
                                    device=self.device, max_episode_length=params.max_episode_length)
        self.stats = RunningObsStats(self.spec.obs_dim, self.device)
        self.engine = build_engine(params, self.model, self.env, self.stats, self.device, action_rank)
        if ctx.collective and hasattr(self.engine, "ext"):
            # in-stream communicator (collective: every rank); --overlap-rollout also gets the
            # side-stream one its deferred value step uses
            ctx.init_native_comm(self.engine.ext, side=bool(params.overlap_rollout or params.overlap_value_epochs))
        self.iteration = 0
        self.env_steps = 0            # global (all ranks)
        self.updates = 0
        self.log = log
        self.timer = PhaseTimer(self.device, annotate=bool(params.profile_dir))
        self._stats_initialised = False
        self.last_metrics: Dict = {}
        self._perm_gen = torch.Generator(device="cpu")
        # DPPO_DEBUG_FAULT="rank:iteration:epoch" (fault-injection tests): that rank
        # exits abruptly (status 13) at that epoch, as a crashed worker would
        self._fault = None
        spec = os.environ.get("DPPO_DEBUG_FAULT", "")
        if spec:
            fr, fi, fe = (int(x) for x in spec.split(":"))
            if fr == ctx.rank:
                self._fault = (fi, fe)
        self._pending = None          # (async all-reduce work, extra) under --overlap-rollout
        self._staged = None           # metrics of the last deferred iteration (iteration_step(defer=True))
        # GPU engine: optional side stream for the observation-statistics reduce + all-reduce +
        # merge (Params.stats_stream on, auto: when an all-reduce sits in that chain, off =
        # default).  Measured slower on the 1-GPU box: 26.06-26.35 vs 26.43-26.55 M env steps/s
        # plain, 24.55-24.79 vs 24.85-25.17 M with the RCCL calls forced — the reduce/merge
        # kernels take CU slots from the LDS-bound value forward and the hand-offs cost more
        # than the ~15 us (+ all-reduce latency) they hide.
        want = {"on": True, "off": False}.get(params.stats_stream, bool(ctx.collective))
        self._stats_stream = None
        if want and self.device.type == "cuda" and hasattr(self.engine, "s12"):
            self._stats_stream = torch.cuda.Stream(device=self.device)

    # ---------------------------------------------------------------------------------------
    def _merge_stats(self, count, s1, s2, shift, count_uniform: bool = False, extra=None) -> None:
        count, s1, s2 = self.ctx.allreduce_obs_moments(count, s1, s2, count_uniform=count_uniform, extra=extra)
        self.stats.merge_moments(count, s1, s2, shift)

    def init_stats(self) -> None:
        """Seed the normaliser with the reset observations of every rank (rollout mode),
        so the first rollout is not normalised by empty statistics."""
        if self._stats_initialised:
            return
        obs = self.engine.current_obs()
        shift = self.stats.shift().clone()
        c, s1, s2 = RunningObsStats.moments(obs, shift)
        self._merge_stats(c, s1, s2, shift)
        self._stats_initialised = True

    def _minibatch_plan(self):
        N = self.engine.T * self.engine.E
        mb = self.p.minibatch_rows()
        nmb = self.p.num_minibatches()
        return N, mb, nmb

    def iteration_step(self, defer: bool = False) -> Dict:
        """One DPPO iteration.

        ``defer=False``: returns this iteration's metrics (host sync at the end).
        ``defer=True``: enqueues everything, stages the device-side metrics (loss sums, grad
        norm, all-reduced episode stats, phase events) into pinned host memory behind an event,
        and returns the metrics of the PREVIOUS iteration, which by then are complete — the host
        never waits on the iteration it just launched, so the next rollout is enqueued while the
        GPU still runs this update (no idle gap at the iteration boundary).  ``finish_metrics``
        resolves the last one."""
        p, eng, tm = self.p, self.engine, self.timer
        tm.enabled = p.phase_timing > 0 and self.iteration % p.phase_timing == 0
        self.init_stats()
        t0 = time.perf_counter()
        tm.start("iteration")
        tm.start("rollout")
        side = self._stats_stream if p.obs_norm_update == "rollout" else None
        ro = eng.rollout(stats_stream=side) if side is not None else eng.rollout()
        # --overlap-rollout: the previous iteration's final gradient all-reduce ran on
        # RCCL's stream concurrently with the rollout just enqueued.  GPU engine (per-head
        # chains): only the VALUE head's last step was left pending — the rollout reads only the
        # policy, so this is exact; apply it now, before values() reads the value head.  CPU
        # engine: the whole last step (a 1-update policy lag, safe for PPO because logp_old is
        # recorded at rollout).
        self.flush_pending()
        tm.stop("rollout")
        tm.start("obs_stats")
        # every rank collects exactly T*E steps -> the global count is host-known (no sync)
        stats_done = None
        # the episode [return sum, count] of a device rollout join the moments' all-reduce (R5)
        ep2 = ro.get("ep2")
        ep_extra = ep2 if (torch.is_tensor(ep2) and ep2.dtype == torch.float64 and ep2.device == self.device) else None
        ro["ep2_reduced"] = ep_extra is not None
        if side is not None:
            # rollout-mode stats feed only the NEXT rollout's normalisation: the reduce, the RCCL
            # all-reduce and the Chan merge run on a side stream, overlapping values/GAE/update
            with torch.cuda.stream(side):
                self._merge_stats(ro["count"], ro["s1"], ro["s2"], ro["shift"], count_uniform=True, extra=ep_extra)
                stats_done = torch.cuda.Event()
                stats_done.record(side)
        else:
            self._merge_stats(ro["count"], ro["s1"], ro["s2"], ro["shift"], count_uniform=True, extra=ep_extra)
        if p.obs_norm_update == "step" and hasattr(eng, "after_stats_merge"):
            eng.after_stats_merge()
        tm.stop("obs_stats")
        tm.start("values_gae")
        eng.values()
        eng.gae()
        tm.stop("values_gae")
        tm.start("update")
        eng.begin_update()
        N, mb, nmb = self._minibatch_plan()
        mean = p.grad_reduce == "mean"
        self._perm_gen.manual_seed((p.seed * 1000003 + self.ctx.rank * 7919 + self.iteration) & 0x7FFFFFFF)
        for epoch in range(p.num_epoch):
            if mb >= N and nmb == 1:
                perm = None
            else:
                perm = torch.randperm(N, generator=self._perm_gen)
            for b in range(nmb):
                if perm is None:
                    idx = None
                else:
                    lo = (b * mb) % N
                    idx = perm[lo:lo + mb]
                    if idx.numel() < mb:
                        idx = torch.cat([idx, perm[:mb - idx.numel()]])
                extra = 0.0
                if p.compat and self.updates == 0:
                    extra = 1.0  # Q1: Shared_grad_buffers start at ones (model.py:51)
                last = epoch == p.num_epoch - 1 and b == nmb - 1
                if self._fault == (self.iteration, epoch):
                    print(f"[dppo rank {self.ctx.rank}] DPPO_DEBUG_FAULT: exiting at iteration {self.iteration} "
                          f"epoch {epoch}", file=sys.stderr, flush=True)
                    os._exit(13)
                if hasattr(eng, "step"):
                    # GPU engine: gradient -> all-reduce -> Adam.  In-stream communicator (the
                    # default: native RCCL, or the gloo adapter): in stream order after the joint
                    # gather (the last step's value half on the side stream under
                    # --overlap-rollout); a process-group all-reduce: per-head chains, each head's
                    # async all-reduce overlapping the other head's kernels (HipEngine.step)
                    ar = self.ctx.grad_allreduce_fn(mean)
                    eng.step(idx, extra, allreduce=ar, mean=mean, last=last)
                    self.updates += 1
                    continue
                deferred = p.overlap_rollout and last and not mean and self.ctx.collective
                eng.grad(idx)
                if deferred:
                    work = self.ctx.allreduce_grads(eng.grad_flat, async_op=True)
                    self._pending = (work, extra)      # applied after the next rollout launch
                else:
                    self.ctx.allreduce_grads(eng.grad_flat, mean=mean)
                    eng.apply(extra)
                self.updates += 1
        if hasattr(eng, "finish_steps") and not (p.overlap_rollout and self.ctx.collective):
            eng.finish_steps()        # the last value-head step's all-reduce + Adam
        if stats_done is not None:
            # order the compute stream after the merge: the metrics read the episode stats, and
            # everything after this iteration (next rollout, snapshots, checkpoints) the stats
            torch.cuda.current_stream(self.device).wait_event(stats_done)
        tm.stop("update")
        tm.stop("iteration")
        steps_local = eng.T * eng.E
        self.env_steps += steps_local * self.ctx.world_size
        self.iteration += 1
        staged = self._stage_metrics(ro, t0, steps_local)
        if not defer:
            m = self._resolve_metrics(staged)
            self.last_metrics = m
            return m
        prev, self._staged = self._staged, staged
        m = self._resolve_metrics(prev) if prev is not None else {}
        if m:
            self.last_metrics = m
        return m

    def finish_metrics(self) -> Dict:
        """resolve the metrics still staged by a deferred ``iteration_step`` (or {})."""
        prev, self._staged = self._staged, None
        m = self._resolve_metrics(prev) if prev is not None else {}
        if m:
            self.last_metrics = m
        return m

    def _stage_metrics(self, ro: Dict, t0: float, steps_local: int) -> Dict:
        """Device-side metric values of this iteration -> one pinned host buffer (async)."""
        eng = self.engine
        dev = self.device
        ep2 = ro.get("ep2")
        flat = None
        if ep2 is not None and hasattr(eng, "pack_metrics") and getattr(eng, "_loss_dev", None) is not None:
            # GPU engine: the [return sum, count] pair (R5) was summed over ranks with the
            # observation moments (or is all-reduced here), then one launch packs it with the
            # loss sums and the gradient norm
            flat = eng.pack_metrics(ep2 if ro.get("ep2_reduced") else self.ctx.allreduce_tensor_(ep2))
        if flat is not None:
            loss_dev = flat
        else:
            flat, loss_dev = self._stage_parts(ro)
        if dev.type == "cuda":
            # the stream the metrics were packed on (the side stream while the overlapped value
            # step runs there)
            side = eng.metrics_stream() if hasattr(eng, "metrics_stream") else None
            with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
                host = torch.empty(flat.numel(), dtype=torch.float64, pin_memory=True)
                host.copy_(flat, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
        else:
            host, ev = flat, None
        return {"host": host, "event": ev, "phases": self.timer.collect(), "has_loss": loss_dev is not None,
                "iteration": self.iteration, "env_steps": self.env_steps, "updates": self.updates,
                "host_s": time.perf_counter() - t0, "steps_local": steps_local}

    def _stage_parts(self, ro: Dict):
        """generic staging (CPU engine): [ep return sum, count] (+ loss vector) as one f64 tensor."""
        eng = self.engine
        dev = self.device
        parts = [torch.stack([torch.as_tensor(ro["ep_return_sum"], dtype=torch.float64, device=dev).reshape(()),
                              torch.as_tensor(ro["ep_count"], dtype=torch.float64, device=dev).reshape(())])]
        parts[0] = self.ctx.allreduce_tensor_(parts[0])        # R5: episode stats over ranks
        loss_dev = eng.loss_vector() if hasattr(eng, "loss_vector") else None
        if loss_dev is not None:
            parts.append(loss_dev.to(torch.float64))
        return torch.cat([x.reshape(-1) for x in parts]), loss_dev

    def _resolve_metrics(self, st: Dict) -> Dict:
        p = self.p
        if st["event"] is not None:
            self.ctx.wait_event(st["event"])     # bounded by dist_timeout_s (collective watchdog)
        if hasattr(self.engine, "raise_if_failed"):
            self.engine.raise_if_failed()        # (a timed-out per-step filter launch: never report it)
        v = st["host"].tolist()
        ep_ret, ep_cnt = v[0], v[1]
        if st["has_loss"]:
            losses = self.engine.losses_from_vector(v[2:])
        else:
            losses = self.engine.last_losses()
        gnorm = losses.pop("grad_norm", 0.0)
        phases = PhaseTimer.elapsed(st["phases"])
        it_ms = phases.pop("ms_iteration", None)
        dt = (it_ms / 1e3) if it_ms else st["host_s"]
        m = {"iteration": st["iteration"], "env_steps": st["env_steps"], "updates": st["updates"],
             "iter_s": dt, "steps_per_s": st["steps_local"] * self.ctx.world_size / max(dt, 1e-9),
             "ep_count": ep_cnt, "mean_ep_return": (ep_ret / ep_cnt) if ep_cnt > 0 else float("nan"),
             "grad_norm": gnorm, **losses, **phases}
        if p.verify_sync_every and st["iteration"] % p.verify_sync_every == 0:
            self.quiesce()                       # the checksum reads the value head too
            m["replicas_in_sync"] = self.ctx.verify_replicas(self.model.flat.data)
        if p.check_finite:
            self._check_finite(m)
        return m

    def _check_finite(self, m: Dict) -> None:
        """debug mode: stop at the first iteration whose loss terms, gradient norm or
        parameters are not finite, naming what broke (the phase timings are in ``m``)."""
        bad = [k for k in ("loss", "loss_clip", "loss_value", "loss_ent", "grad_norm")
               if k in m and not math.isfinite(m[k])]
        it = m.get("iteration", self.iteration)
        if not bool(torch.isfinite(self.model.flat.data).all()):
            bad.append("parameters")
        if bool(torch.isfinite(self.stats.mean_f32).all()) is False:
            bad.append("obs_stats.mean")
        if bad:
            raise FloatingPointError(f"rank {self.ctx.rank} iteration {int(it)}: non-finite {bad}")

    def quiesce(self) -> None:
        """the GPU engine's deferred value-head step (side stream / pending all-reduce) applied:
        the parameters are the synchronous ones (snapshots, checksums); the CPU engine's deferred
        whole step (its documented 1-update lag) is left alone"""
        if hasattr(self.engine, "finish_steps"):
            self.engine.finish_steps()

    def flush_pending(self) -> None:
        """complete a deferred (overlapped) all-reduce + Adam step, if any."""
        if hasattr(self.engine, "finish_steps"):
            self.engine.finish_steps()
        pend = getattr(self, "_pending", None)
        if pend is None:
            return
        work, extra = pend
        self._pending = None
        if work is not None:
            work.wait()            # orders the compute stream after RCCL's (no host block on GPU)
        self.engine.apply(extra)

    def should_stop(self) -> bool:
        p = self.p
        if p.max_iters and self.iteration >= p.max_iters:
            return True
        if p.total_env_steps and self.env_steps >= p.total_env_steps:
            return True
        if self.iteration >= p.time_horizon:
            return True
        return False

    # -- checkpoint ---------------------------------------------------------------------------
    def trainer_state(self) -> Dict:
        self.flush_pending()
        eng = self.engine
        return {"adam_m": eng.adam_m.detach().cpu(), "adam_v": eng.adam_v.detach().cpu(),
                "adam_step": eng.adam_step, "obs_stats": self.stats.state_dict(),
                "iteration": self.iteration, "env_steps": self.env_steps, "updates": self.updates,
                "config": self.p.to_dict(), "world_size": self.ctx.world_size,
                # fp8 mode's e4m3 wgrad operands: the gradient-maxima ring the next step's delayed
                # scales come from (a resumed run continues bit-identically)
                **({"q8_amax": eng.q8_amax.detach().cpu(), "q8_next": eng._q8_next}
                   if getattr(eng, "q8", False) else {})}

    def load_trainer_state(self, st: Dict) -> None:
        eng = self.engine
        eng.adam_m.copy_(st["adam_m"].to(eng.adam_m.device))
        eng.adam_v.copy_(st["adam_v"].to(eng.adam_v.device))
        eng.adam_step = int(st["adam_step"])
        self.stats.load_state_dict(st["obs_stats"])
        self.iteration = int(st["iteration"])
        self.env_steps = int(st["env_steps"])
        self.updates = int(st["updates"])
        self._stats_initialised = True
        if getattr(eng, "q8", False) and "q8_amax" in st:
            eng.q8_amax.copy_(st["q8_amax"].to(eng.q8_amax.device))
            eng._q8_next = int(st["q8_next"])
            eng._q8_cal = [True, True]
        if hasattr(eng, "params_changed"):
            eng.params_changed()
