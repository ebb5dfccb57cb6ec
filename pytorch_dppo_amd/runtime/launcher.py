"""Process orchestration — the reference ``main.py:41-73`` (spawn test + chief + N workers,
join forever), re-done as one process per worker (per GPU) with a real termination story.

* under ``torchrun`` (``RANK``/``WORLD_SIZE`` set) the current process IS one worker;
* otherwise ``num_processes`` workers are spawned here (gloo on CPU; RCCL on GPU, one per
  device), rendezvous on 127.0.0.1;
* rank 0 owns logging, checkpoints and the evaluator process;
* every collective has a timeout (``dist_timeout_s``), so a dead rank makes the others exit
  with an error instead of deadlocking forever (reference Q21).
"""
from __future__ import annotations

import os
import socket
import sys
import traceback
from typing import Optional

import torch

from ..config import Params
from ..parallel.dist import DistContext, init_distributed
from ..utils import checkpoint as ckpt
from ..utils.heartbeat import start_heartbeat
from ..utils.metrics import MetricsLogger


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_worker(params: Params, ctx: DistContext, max_iters: Optional[int] = None,
               evaluator: bool = True, quiet: bool = False):
    from .worker import DPPOWorker
    log = MetricsLogger(params.log_jsonl if ctx.is_main else "", enabled=ctx.is_main,
                        stdout=ctx.is_main and not quiet, csv_path=params.log_csv if ctx.is_main else "")
    w = DPPOWorker(params, ctx, log)
    if params.resume:
        sd = ckpt.load_model_state(params.resume)
        w.model.load_state_dict(sd)
        st = ckpt.load_trainer_state(params.resume)
        if st is not None:
            w.load_trainer_state(st)
        es = ckpt.load_env_state(params.resume, ctx.rank)
        if es is not None and hasattr(w.engine, "load_env_state"):
            w.engine.load_env_state(es)
        ctx.broadcast_(w.model.flat.data, src=0)
        if hasattr(w.engine, "params_changed"):
            w.engine.params_changed()
    ev = None
    if evaluator and ctx.is_main and params.eval_every > 0:
        from .evaluator import EvaluatorHandle
        ev = EvaluatorHandle(params)
    history = []
    hb = start_heartbeat(ctx, params.heartbeat_interval(ctx.world_size), params.heartbeat_timeout_s)
    prof = _Profiler(params, ctx)
    try:
        n = 0
        # GPU: metrics are resolved one iteration late, so the host never idles the device at
        # an iteration boundary waiting for numbers it only logs
        defer = ctx.device.type == "cuda"

        def record(m):
            if not m:
                return
            history.append(m)
            if ctx.is_main and params.log_every and int(m["iteration"]) % params.log_every == 0:
                log.log(m)

        while not w.should_stop():
            prof.before(n)
            record(w.iteration_step(defer=defer))
            prof.after(n)
            n += 1
            if ev is not None and w.iteration % params.eval_every == 0:
                w.quiesce()     # a value step still on the side stream writes what the snapshot reads
                ev.push(w.model.state_dict(), w.stats.state_dict(), w.iteration)
            if params.checkpoint_dir and params.checkpoint_every and w.iteration % params.checkpoint_every == 0:
                save(w, ctx, params.checkpoint_dir)
            if max_iters is not None and n >= max_iters:
                break
        record(w.finish_metrics())
        w.flush_pending()
        if params.checkpoint_dir:
            save(w, ctx, params.checkpoint_dir)
    finally:
        prof.close()
        if hb is not None:
            hb.stop()
        if ev is not None:
            ev.close()
        log.close()
    return w, history


class _Profiler:
    """``--profile-dir``: a torch.profiler window over iterations [a, b) (host ops + HIP kernels
    + the PhaseTimer ranges), exported as one chrome trace per rank."""

    def __init__(self, params: Params, ctx: DistContext):
        self.dir = params.profile_dir
        self.rank = ctx.rank
        self.gpu = ctx.device.type == "cuda"
        a, _, b = (params.profile_iters or "0:1").partition(":")
        self.a = int(a or 0)
        self.b = int(b) if b else self.a + 1
        self.p = None

    def before(self, n: int) -> None:
        if self.dir and self.p is None and n == self.a:
            from torch.profiler import ProfilerActivity, profile
            acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.gpu else [])
            self.p = profile(activities=acts, record_shapes=False)
            self.p.__enter__()

    def after(self, n: int) -> None:
        if self.p is not None and n + 1 >= self.b:
            self.close()

    def close(self) -> None:
        if self.p is None:
            return
        if self.gpu:
            torch.cuda.synchronize()
        self.p.__exit__(None, None, None)
        os.makedirs(self.dir, exist_ok=True)
        self.p.export_chrome_trace(os.path.join(self.dir, f"trace_rank{self.rank}.json"))
        self.p = None
        self.dir = ""


def save(w, ctx: DistContext, path: str) -> None:
    # every deferred step applied BEFORE the weights are copied out: model.pt and the Adam state
    # of trainer_state.pt must describe the same step
    w.flush_pending()
    if hasattr(w.engine, "raise_if_failed"):
        w.engine.raise_if_failed(sync=True)   # never checkpoint a step built on a failed launch
    env_state = w.engine.env_state() if hasattr(w.engine, "env_state") else None
    ckpt.save_checkpoint(path, w.model.state_dict(), w.trainer_state(), ctx.rank, env_state)
    ctx.barrier()


def _spawn_entry(rank: int, world: int, port: int, params_dict, ret_q=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("OMP_NUM_THREADS", "1")   # main.py:42
    torch.set_num_threads(1)
    params = Params.from_dict(params_dict)
    ctx = init_distributed(params.device, rank=rank, world_size=world, timeout_s=params.dist_timeout_s,
                           backend=params.dist_backend, grad_comm=params.grad_comm)
    try:
        w, hist = run_worker(params, ctx)
        if ret_q is not None and rank == 0:
            ret_q.put([{k: v for k, v in m.items() if isinstance(v, (int, float, bool))} for m in hist])
    except Exception:
        traceback.print_exc()
        raise
    finally:
        ctx.destroy()


def launch(params: Params) -> None:
    if "WORLD_SIZE" in os.environ and "RANK" in os.environ:
        ctx = init_distributed(params.device, timeout_s=params.dist_timeout_s, backend=params.dist_backend,
                               grad_comm=params.grad_comm)
        try:
            if params.device == "gpu" and ctx.world_size == 1:
                from ..parallel.dist import init_single_rank_collective
                ctx = init_single_rank_collective(ctx.device, timeout_s=params.dist_timeout_s,
                                                  grad_comm=params.grad_comm)
            run_worker(params, ctx)
        finally:
            ctx.destroy()
        return
    world = max(1, int(params.num_processes))
    if params.device == "gpu":
        world = min(world, max(1, torch.cuda.device_count()))
    if world == 1:
        ctx = init_distributed(params.device, rank=0, world_size=1, backend=params.dist_backend)
        if params.device == "gpu":
            from ..parallel.dist import init_single_rank_collective
            ctx = init_single_rank_collective(ctx.device, port=free_port(), timeout_s=params.dist_timeout_s,
                                              grad_comm=params.grad_comm)
        try:
            run_worker(params, ctx)
        finally:
            ctx.destroy()
        return
    import torch.multiprocessing as mp
    port = free_port()
    mp.start_processes(_spawn_entry, args=(world, port, params.to_dict()), nprocs=world,
                       join=True, start_method="spawn")
