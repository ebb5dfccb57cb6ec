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

import datetime
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


class NativeComm:
    """RCCL communicator over the process group's ranks, collectives on a caller-named stream
    (default: the current one).  Created collectively: rank 0's ncclUniqueId is broadcast over
    the existing group."""

    def __init__(self, ext, rank: int, world_size: int):
        idb = [ext.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(idb, src=0)
        self.ext = ext
        self.world_size = world_size
        self.handle = ext.comm_init(idb[0], world_size, rank)

    def allreduce_(self, t: torch.Tensor, mean: bool = False) -> None:
        self.ext.comm_allreduce(self.handle, t, mean)

    def destroy(self) -> None:
        if self.handle is not None:
            self.ext.comm_destroy(self.handle)
            self.handle = None


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
    native: Optional[NativeComm] = None

    def init_native_comm(self, ext) -> bool:
        """create the in-stream RCCL communicator (RCCL groups only; DPPO_NATIVE_COMM=0: off)"""
        if (self.native is None and self.enabled and self.backend == "nccl" and self.device.type == "cuda"
                and os.environ.get("DPPO_NATIVE_COMM", "1") != "0" and hasattr(ext, "comm_init")):
            # every rank must take the same path (a rank on the process group and another on the
            # native communicator would never meet in a collective): a rank whose communicator
            # fails reports it and ALL ranks fall back to the process group's collectives
            nat, err = None, None
            try:
                nat = NativeComm(ext, self.rank, self.world_size)
            except Exception as e:   # noqa: BLE001 — the fallback is collective, the cause is printed
                err = e
            ok = torch.tensor([0.0 if nat is None else 1.0], device=self.device)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if ok.item() == 1.0:
                self.native = nat
            else:
                if nat is not None:
                    nat.destroy()
                print(f"[dppo rank {self.rank}] native RCCL communicator unavailable "
                      f"({err if err is not None else 'on another rank'}); using the process group", flush=True)
        return self.native is not None

    def grad_allreduce_fn(self, mean: bool = False):
        """the engines' hot-path all-reduce callback for the flat gradient: None when no collective
        runs; on a native communicator an in-stream sum/mean (attribute ``in_stream``), else the
        async process-group all-reduce returning its work handle (the engine scales for mean)."""
        if not self.collective:
            return None
        if self.native is not None:
            nat = self.native

            def ar(t):
                nat.allreduce_(t, mean)
            ar.in_stream = True
            return ar
        return lambda t: self.allreduce_grads(t, async_op=True)

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
        if self.native is not None:
            try:
                self.native.destroy()
            except Exception:
                pass
            self.native = None
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
                     timeout_s: float = 300.0) -> DistContext:
    """Initialise from torchrun env vars or explicit args; one process per GPU.

    GPU → backend 'nccl' (RCCL over xGMI), CPU → 'gloo'.  world_size 1 → no process group
    unless ``force`` is wanted by a caller (RCCL at world size 1 is exercised by bench.py).
    """
    rank = _env_int("RANK", 0) if rank is None else rank
    world_size = _env_int("WORLD_SIZE", 1) if world_size is None else world_size
    local_rank = _env_int("LOCAL_RANK", rank)
    if device == "gpu":
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError("device=gpu but no HIP device visible")
        torch.cuda.set_device(local_rank % ndev)
        dev = torch.device("cuda", local_rank % ndev)
        # DPPO_DIST_BACKEND=gloo: diagnostics only — several ranks sharing one GPU (RCCL refuses
        # two ranks on one device), to exercise the multi-rank GPU engine path on a 1-GPU box
        backend = os.environ.get("DPPO_DIST_BACKEND", "nccl")
    else:
        dev = torch.device("cpu")
        backend = "gloo"
    ctx = DistContext(rank=rank, world_size=world_size, local_rank=local_rank, backend=backend,
                      device=dev)
    if backend not in ("nccl", "gloo"):
        raise ValueError(f"unsupported backend {backend}")
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


def init_single_rank_collective(device: torch.device, port: int = 29541) -> DistContext:
    """A world-size-1 RCCL group so the real collective path runs on a 1-GPU box."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(port))
    if not dist.is_initialized():
        dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=device)
    return DistContext(rank=0, world_size=1, local_rank=device.index or 0, backend="nccl",
                       device=device)
