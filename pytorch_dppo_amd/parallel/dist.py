"""Process groups and the collectives that replace the reference's shared-memory IPC.

Reference → here:

* R1 grad sum into ``Shared_grad_buffers`` (``model.py:53-55``) + chief ``Adam.step``
  (``chief.py:13-20``)  →  ONE all-reduce of the flat fp32 gradient
  (:meth:`DistContext.allreduce_grads`, async so it can overlap other work), then every
  rank applies the same fused Adam step (replicated optimizer: no parameter broadcast).
* R2 racy shared obs-stat RMW (``model.py:71-74``) → one all-reduce of batch moments about a
  common shift (:meth:`DistContext.allreduce_obs_moments`).
* R3 weight reads from shared memory (``train.py:62,135``) → one broadcast at start / resume.
* R4 Counter + TrafficLight barrier (``utils.py:4-39``) → implicit in the collective.
* R5 ``test_n`` counter → metrics all-reduce (:meth:`DistContext.allreduce_scalars`).

On GPU the backend is ``nccl`` (= RCCL on ROCm, xGMI inside a node); on CPU it is ``gloo``.
There is no custom transport and no multi-backend dispatch on the hot path.

The per-epoch gradient all-reduce and the per-iteration statistics all-reduce of a GPU worker
run on a NATIVE RCCL communicator (:class:`NativeComm`, ``csrc/comm.cpp``) created from the
process group once: its collectives are enqueued on the compute stream itself, in stream order.
torch's ProcessGroupNCCL runs every collective on an internal stream, and each one then costs
two cross-stream event hops the compute queue idles on (~26 us per all-reduce measured with the
collectives forced at world size 1: 5.03 vs 4.21 ms per bench iteration with the two-chain
overlap design that needed them; profiles/r3/rccl_forced_vs_plain.md).
"""
from __future__ import annotations

import contextlib
import datetime
import os
import sys
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


class CollectiveError(RuntimeError):
    """a hot-path collective failed or timed out (dead / hung peer); the communicators are aborted"""


class NativeComm:
    """RCCL communicator over the process group's ranks, collectives on a caller-named stream
    (default: the current one), ``csrc/comm.cpp``.  Non-blocking underneath: creation and a
    stalled enqueue are bounded by ``timeout_s`` (then aborted); ``status()`` is the asynchronous
    error state the host wait loops poll (:meth:`DistContext.wait_event`)."""
    in_stream = True

    def __init__(self, ext, handle: int, world_size: int):
        self.ext = ext
        self.world_size = world_size
        self.handle = handle

    @classmethod
    def create(cls, ext, rank: int, world_size: int, timeout_s: float,
               device: Optional[torch.device] = None) -> Optional["NativeComm"]:
        """Collective over the default group.  Rank 0 ALWAYS takes part in the id broadcast — it
        sends an error token when it cannot make an id — so a failure on any rank is seen by all:
        every rank returns None together (after a MIN all-reduce of the outcome) or every rank
        returns a communicator."""
        token = [None]
        if rank == 0:
            try:
                token[0] = ext.comm_unique_id()
            except Exception as e:   # noqa: BLE001 — the error travels in the token
                token[0] = ("error", f"{type(e).__name__}: {e}")
        dist.broadcast_object_list(token, src=0)
        tok = token[0]
        if isinstance(tok, tuple):
            print(f"[dppo rank {rank}] native RCCL communicator unavailable (rank 0: {tok[1]}); "
                  f"using the process group", flush=True)
            return None
        handle, err = None, None
        try:
            handle = ext.comm_init(tok, world_size, rank, float(timeout_s))   # bounded (comm.cpp)
        except Exception as e:   # noqa: BLE001 — the fallback is collective, the cause is printed
            err = e
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        ok = torch.tensor([0.0 if handle is None else 1.0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() == 1.0:
            return cls(ext, handle, world_size)
        if handle is not None:
            ext.comm_abort(handle)
        print(f"[dppo rank {rank}] native RCCL communicator unavailable "
              f"({err if err is not None else 'on another rank'}); using the process group", flush=True)
        return None

    def allreduce_(self, t: torch.Tensor, mean: bool = False, stream: Optional[torch.cuda.Stream] = None) -> None:
        self.ext.comm_allreduce(self.handle, t, mean, 0 if stream is None else stream.cuda_stream)

    def status(self) -> int:
        """0 ok, 7 in progress, -1 aborted / destroyed, else an RCCL error code"""
        return int(self.ext.comm_status(self.handle)) if self.handle is not None else -1

    def abort(self) -> None:
        if self.handle is not None:
            self.ext.comm_abort(self.handle)

    def destroy(self) -> None:
        if self.handle is not None:
            h, self.handle = self.handle, None
            if self.ext.comm_status(h) == -1:
                return                      # aborted: nothing to finalise
            self.ext.comm_destroy(h)


class GlooStreamComm:
    """The native communicator's interface on a gloo group: the in-stream (production) engine
    branch for ranks that SHARE one GPU (RCCL refuses two ranks on one device), so 2-rank runs
    on the 1-GPU box take the exact code path an N-GPU RCCL run takes — joint kernels → gather →
    all-reduce → whole-vector Adam, and the side-stream value step of ``--overlap-rollout``.
    gloo copies device tensors through the host and its wait blocks: stream order is kept, only
    the overlap is not real.  ``mean``: the sum, then a stream-ordered scale (ncclAvg's result)."""
    in_stream = True

    def __init__(self, world_size: int):
        self.world_size = world_size
        self.handle = 0

    def allreduce_(self, t: torch.Tensor, mean: bool = False, stream: Optional[torch.cuda.Stream] = None) -> None:
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            if mean:
                t.mul_(1.0 / self.world_size)

    def status(self) -> int:
        return 0

    def abort(self) -> None:
        pass

    def destroy(self) -> None:
        pass


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    # run the hot-path collectives even at world size 1, where a sum over one rank is the
    # identity (tests use it to exercise the real RCCL call on the 1-GPU box)
    force_collectives: bool = False
    # the in-stream communicator of the hot path (NativeComm on RCCL, GlooStreamComm on a gloo
    # group of GPU ranks) and the second one the side-stream value step of --overlap-rollout uses
    # (two communicators: their collectives may run concurrently on different streams)
    native: Optional[object] = None
    native_side: Optional[object] = None
    timeout_s: float = 300.0             # Params.dist_timeout_s: the bound of every wait on peers
    grad_comm: str = "auto"              # Params.grad_comm: auto | native | process_group

    def init_native_comm(self, ext, side: bool = False) -> bool:
        """create the in-stream communicator(s) (collective: every rank calls it).  RCCL groups:
        NativeComm (bounded, collective-safe creation; on failure every rank falls back to the
        process group together unless grad_comm == "native").  gloo groups of GPU ranks:
        GlooStreamComm.  ``side``: also the side-stream communicator."""
        if self.native is not None or not self.enabled or self.device.type != "cuda" or self.grad_comm == "process_group":
            return self.native is not None
        if self.backend == "gloo":
            self.native = GlooStreamComm(self.world_size)
            self.native_side = GlooStreamComm(self.world_size) if side else None
        elif self.backend == "nccl" and hasattr(ext, "comm_init"):
            self.native = NativeComm.create(ext, self.rank, self.world_size, self.timeout_s, self.device)
            if self.native is not None and side:
                self.native_side = NativeComm.create(ext, self.rank, self.world_size, self.timeout_s, self.device)
        if self.native is None and self.grad_comm == "native":
            raise RuntimeError("grad_comm=native but the native communicator could not be created")
        return self.native is not None

    def grad_allreduce_fn(self, mean: bool = False):
        """the engines' hot-path all-reduce callback for the flat gradient: None when no collective
        runs; on an in-stream communicator ``ar(t, stream=None)`` — a stream-ordered sum/mean on the
        current stream, or on ``stream`` through the side communicator (attributes ``in_stream``,
        ``side``: a side communicator exists) — else the async process-group all-reduce returning
        its work handle (the engine scales for mean)."""
        if not self.collective:
            return None
        if self.native is not None:
            nat, side = self.native, self.native_side

            def ar(t, stream=None):
                (nat if stream is None else side).allreduce_(t, mean, stream)
            ar.in_stream = True
            ar.side = side is not None
            return ar
        return lambda t: self.allreduce_grads(t, async_op=True)

    # -- failure detection ------------------------------------------------------
    def _comms(self):
        return [c for c in (self.native, self.native_side) if c is not None]

    def comm_error(self) -> Optional[str]:
        """the first asynchronous error of the in-stream communicators, or None"""
        for c in self._comms():
            st = c.status()
            if st not in (0, 7):
                return f"RCCL communicator state {st}" if st != -1 else "communicator aborted"
        return None

    def abort(self, reason: str = "") -> None:
        """abort every communicator of this rank (their kernels exit: nothing stays spinning on
        the GPU for a dead peer) — called before a rank gives up on its peers"""
        if reason:
            print(f"[dppo rank {self.rank}] aborting collectives: {reason}", file=sys.stderr, flush=True)
        for c in self._comms():
            try:
                c.abort()
            except Exception:   # noqa: BLE001 — best effort on the way out
                pass
        if self.backend == "nccl" and self.enabled:
            try:
                from torch.distributed.distributed_c10d import _abort_process_group
                _abort_process_group()
            except Exception:   # noqa: BLE001
                pass

    def wait_event(self, ev, timeout_s: Optional[float] = None) -> None:
        """Host wait for a device event that may sit behind in-stream collectives: the
        communicators' watchdog.  Polls the event and ncclCommGetAsyncError; an asynchronous
        error, or no completion within ``timeout_s`` (default dist_timeout_s), aborts the
        communicators (ncclCommAbort) and raises CollectiveError — the reference's dead-worker
        deadlock (chief.py:13, Q21) becomes a non-zero exit."""
        if ev is None:
            return
        if not self._comms():
            ev.synchronize()
            return
        to = self.timeout_s if timeout_s is None else float(timeout_s)
        t0 = time.monotonic()
        n = 0
        while not ev.query():
            n += 1
            if n % 64 == 0:
                err = self.comm_error()
                if err is not None:
                    self.abort(err)
                    raise CollectiveError(f"rank {self.rank}: {err}")
                el = time.monotonic() - t0
                if el > to:
                    msg = f"rank {self.rank}: device work behind the collectives did not complete in {to:.0f} s"
                    self.abort(msg)
                    raise CollectiveError(msg)
                if el > 0.02:
                    time.sleep(2e-4)     # spin first (latency), then yield the core

    def sync(self) -> None:
        """device synchronise through the watchdog (torch.cuda.synchronize without communicators)"""
        if self.device.type != "cuda":
            return
        if not self._comms():
            torch.cuda.synchronize(self.device)
            return
        ev = torch.cuda.Event()
        ev.record()
        self.wait_event(ev)
        torch.cuda.synchronize(self.device)   # (the other streams: the event covered the current one)

    @property
    def enabled(self) -> bool:
        return dist.is_available() and dist.is_initialized()

    @property
    def collective(self) -> bool:
        """hot-path reductions run: a group exists and has more than one rank (or forced).
        At world size 1 every all-reduce is the identity, and an RCCL call still costs
        ~10 us of stream handoff per epoch (rocprofv3 timeline), so it is skipped."""
        return self.enabled and (self.world_size > 1 or self.force_collectives)

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    # -- collectives -----------------------------------------------------------------------
    def allreduce_grads(self, flat_grad: torch.Tensor, mean: bool = False, async_op: bool = False):
        """Sum (or mean) of the flat gradient over ranks, in place.

        With ``async_op`` the returned work handle's ``wait()`` orders the consumer after
        the collective on the device stream (RCCL runs on its own stream)."""
        if not self.collective:
            return None
        if self.native is not None and flat_grad.dtype == torch.float32:
            self.native.allreduce_(flat_grad, mean)    # in stream order: nothing to wait on
            return None
        work = dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, async_op=async_op)
        if mean:
            if async_op:
                work.wait()
                work = None
            flat_grad.mul_(1.0 / self.world_size)
        return work

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        if self.enabled:
            dist.broadcast(t, src=src)

    def allreduce_obs_moments(self, count: float, s1: torch.Tensor, s2: torch.Tensor,
                              count_uniform: bool = False, extra: Optional[torch.Tensor] = None):
        """global (count, S1, S2) about a shift every rank shares — exact merge (R2).

        ``count_uniform``: every rank contributed the same (host-known) count, so the global
        count is count * world_size and no device->host read is needed (the hot path).
        ``extra`` (count_uniform only): a small fp64 device tensor summed over ranks in the SAME
        all-reduce and written back in place — the iteration's episode [return sum, count] (R5)
        ride along with the moments instead of costing a second collective."""
        if not self.collective:
            return count, s1, s2
        O = s1.numel()
        if count_uniform:
            parts = [s1.reshape(-1).to(self.device, torch.float64), s2.reshape(-1).to(self.device, torch.float64)]
            if extra is not None:
                parts.append(extra.reshape(-1).to(self.device, torch.float64))
            buf = torch.cat(parts)
            if self.native is not None:
                self.native.allreduce_(buf)          # in stream order
            else:
                dist.all_reduce(buf, op=dist.ReduceOp.SUM)
            if extra is not None:
                extra.copy_(buf[2 * O:].view(extra.shape))
            return count * self.world_size, buf[:O], buf[O:2 * O]
        assert extra is None, "extra rides only on the count-uniform all-reduce"
        buf = torch.empty(1 + 2 * O, dtype=torch.float64, device=self.device)
        buf[0] = count
        buf[1:1 + O] = s1.reshape(-1).to(self.device, torch.float64)
        buf[1 + O:] = s2.reshape(-1).to(self.device, torch.float64)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        return float(buf[0].item()), buf[1:1 + O].clone(), buf[1 + O:].clone()

    def allreduce_scalars(self, vals: Dict[str, float], op: str = "sum") -> Dict[str, float]:
        """values may be python numbers or 0-d device tensors (stacked without a host read)."""
        keys = sorted(vals)
        parts = [vals[k].reshape(1).to(self.device, torch.float64) if torch.is_tensor(vals[k])
                 else torch.tensor([float(vals[k])], dtype=torch.float64, device=self.device) for k in keys]
        t = torch.cat(parts)
        if self.collective:
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
        return {k: float(x) for k, x in zip(keys, t.tolist())}

    def allreduce_tensor_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if (self.collective and self.native is not None and op == "sum" and t.is_contiguous()
                and t.dtype in (torch.float32, torch.float64)):
            self.native.allreduce_(t)                # in stream order
            return t
        if self.collective:
            dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                                   "min": dist.ReduceOp.MIN}[op])
        return t

    def verify_replicas(self, flat: torch.Tensor) -> bool:
        """debug checksum all-reduce: True iff every rank holds bit-identical params."""
        if not self.enabled:
            return True
        h = flat.detach().view(torch.int32).to(torch.int64).sum().reshape(1)
        h = h.to(self.device)
        lo, hi = h.clone(), h.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        return bool((lo == hi).item())

    def barrier(self) -> None:
        if self.enabled:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def destroy(self) -> None:
        for c in self._comms():
            try:
                c.destroy()
            except Exception:   # noqa: BLE001
                pass
        self.native = self.native_side = None
        if dist.is_available() and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_distributed(device: str = "cpu", rank: Optional[int] = None, world_size: Optional[int] = None,
                     master_addr: str = "127.0.0.1", master_port: Optional[int] = None,
                     timeout_s: float = 300.0, backend: str = "auto", grad_comm: str = "auto") -> DistContext:
    """Initialise from torchrun env vars or explicit args; one process per GPU.

    ``backend`` (Params.dist_backend): auto = 'nccl' (RCCL over xGMI) on GPU, 'gloo' on CPU;
    'gloo' on GPU is for ranks sharing one GPU (RCCL refuses two ranks on one device: the 1-GPU
    box's multi-rank tests), with the in-stream engine path on GlooStreamComm.  world_size 1 →
    no process group (bench.py / the launcher make a world-1 RCCL group themselves).
    """
    rank = _env_int("RANK", 0) if rank is None else rank
    world_size = _env_int("WORLD_SIZE", 1) if world_size is None else world_size
    local_rank = _env_int("LOCAL_RANK", rank)
    if backend not in ("auto", "nccl", "gloo"):
        raise ValueError(f"unsupported backend {backend}")
    if device == "gpu":
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError("device=gpu but no HIP device visible")
        torch.cuda.set_device(local_rank % ndev)
        dev = torch.device("cuda", local_rank % ndev)
        backend = "nccl" if backend == "auto" else backend
    else:
        dev = torch.device("cpu")
        if backend == "nccl":
            raise ValueError("the nccl (RCCL) backend needs device=gpu")
        backend = "gloo"
    ctx = DistContext(rank=rank, world_size=world_size, local_rank=local_rank, backend=backend,
                      device=dev, timeout_s=float(timeout_s), grad_comm=grad_comm)
    if world_size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", master_addr)
        if master_port is not None:
            os.environ["MASTER_PORT"] = str(master_port)
        os.environ.setdefault("MASTER_PORT", "29531")
        kw = dict(backend=backend, rank=rank, world_size=world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return ctx


def init_single_rank_collective(device: torch.device, port: int = 29541, timeout_s: float = 300.0,
                                grad_comm: str = "auto") -> DistContext:
    """A world-size-1 RCCL group so the real collective path runs on a 1-GPU box."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(port))
    if not dist.is_initialized():
        dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=device,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return DistContext(rank=0, world_size=1, local_rank=device.index or 0, backend="nccl",
                       device=device, timeout_s=float(timeout_s), grad_comm=grad_comm)
