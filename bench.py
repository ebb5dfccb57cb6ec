#!/usr/bin/env python3
"""Headline benchmark: env steps/sec (whole node), Humanoid-v2 DPPO workers (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Both forms run N ranks: without a torchrun world (no WORLD_SIZE) and N > 1 the first form
starts the N ranks itself as a child torch.distributed.run tree and exits with its status (the
parent makes no HIP call at all: the ranks check the devices); under torchrun WORLD_SIZE must
equal --gpus and every local rank needs its own GPU (RCCL), else the bench exits non-zero
instead of reporting a different world as N GPUs.

Multi-rank runs use the in-stream gradient all-reduce (csrc/comm.cpp: the native RCCL
communicator on the compute stream, bounded by --dist-timeout-s with ncclCommAbort on a dead
peer) and the per-rank heartbeat; ``--dist-backend gloo`` runs the same engine branch for ranks
that share one GPU (the 1-GPU box's rehearsal of the N-GPU path).

One DPPO worker per GPU (one process per GPU, RCCL over xGMI).  A *step* is one full DPPO
iteration of the reference algorithm on every worker (train.py:60-178 + chief.py):
rollout of T x E = 16 x 4096 = 65,536 env steps (Humanoid-v2 dims: obs 376, act 17, synthetic
dynamics), value forward, GAE, then 10 epochs, each ONE synchronous global step on the full
65,536-row batch (reference: batch_size == exploration_size, main.py:20,28), each with the
RCCL all-reduce of the flat gradient and the fused Adam step.  Per-GPU work is fixed as N
grows (weak scaling).  Model: the reference actor-critic (model.py), random init.

Precision: the headline runs at the reference's precision, fp32 (model.py / train.py are fp32
end to end): ``--dtype bf16x3`` = every GEMM on split-bf16 operands (x = hi + lo, three bf16
MFMAs per product, fp32 accumulate; fp32 tolerances in tests/test_gpu_kernels.py), fp32 master
weights, fp32 loss/GAE/Adam.  The reduced-precision modes (bf16, fp8 forward) are timed in the
same invocation on the same config and reported as separately labelled ``variants``.

Timing: W untimed warmup iterations; barrier + device sync; K timed iterations; barrier +
device sync; the max over ranks of the elapsed time.  Rank 0 prints ONE JSON line.  The
per-phase HIP-event instrumentation of the worker is off by default here (--phase-timing N
samples it): it is diagnostics, and each timed event record idles the GPU ~10 us.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pytorch_dppo_amd.config import dppo_preset  # noqa: E402
from pytorch_dppo_amd.parallel.dist import init_distributed, init_single_rank_collective  # noqa: E402
from pytorch_dppo_amd.runtime.worker import DPPOWorker  # noqa: E402
from pytorch_dppo_amd.utils.heartbeat import start_heartbeat  # noqa: E402

METRIC = "env steps/sec (whole node), MuJoCo Humanoid-v2, 8 DPPO workers"
# BASELINE.md derived estimate for the reference on this metric: 0.8-1.6e3 steps/s per node
# (8 workers).  We divide by the UPPER end (conservative).
BASELINE_VALUE = 1.6e3
# JSON "dtype" labels: bf16x3 IS fp32-accurate compute (split-bf16 operands, fp32 accumulate)
DTYPE_LABEL = {"bf16x3": "fp32_3xbf16", "fp32": "fp32", "bf16": "bf16", "fp8": "fp8_e4m3_fwd+wgrad+bf16_update"}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """``python bench.py --gpus N`` without a torchrun world: start the N ranks as ONE child
    process tree (torch.distributed.run, rendezvous on 127.0.0.1) and return its exit status.
    Runs before this process touches the GPU (no HIP call, no exec: the parent only waits), the
    way the reference's main.py:68-71 spawns its N workers."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL over dmabuf IPC on this host driver
    print(f"bench: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def check_world(gpus: int, backend: str) -> None:
    """a torchrun world must be the one --gpus names, with a device per local rank (RCCL: one
    process per GPU).  ``--dist-backend gloo`` (ranks sharing one GPU) skips the device count."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {gpus}: refusing to report a "
                         f"{world}-rank run as {gpus} GPUs")
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    ndev = torch.cuda.device_count()
    if backend != "gloo" and ndev < local:
        raise SystemExit(f"bench: {local} local ranks but only {ndev} visible GPU(s) (RCCL needs one "
                         f"process per GPU)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--env-name", default="Humanoid-v2")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--rollout-len", type=int, default=16)
    ap.add_argument("--num-epoch", type=int, default=10)
    ap.add_argument("--dtype", default="bf16x3",
                    help="headline operand precision: bf16x3 (fp32-accurate, default), fp32 (exact f32 MFMA), "
                         "bf16, fp8")
    ap.add_argument("--variants", default="bf16,fp8",
                    help="comma list of extra dtypes timed after the headline on the same config "
                         "(reported under 'variants'; '' = none)")
    ap.add_argument("--batch-size", type=int, default=0, help="0 = full buffer (reference DPPO)")
    ap.add_argument("--overlap-rollout", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                    help="the last value-head all-reduce + Adam overlap the next rollout on a side stream (exact: "
                         "the rollout reads only the policy); auto = on when the world has more than one rank")
    ap.add_argument("--overlap-value", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                    help="every epoch's value-head all-reduce + Adam on a side stream, joined before the next value "
                         "kernel (exact); auto = the measured default (docs/ARCHITECTURE.md §13: off)")
    ap.add_argument("--force-collectives", action="store_true",
                    help="diagnostics: run the hot-path RCCL collectives even at world size 1")
    ap.add_argument("--phase-timing", type=int, default=0,
                    help="per-phase HIP-event timing every N iterations (0 = off: instrumentation only, "
                         "each timed event record idles the GPU ~10 us)")
    ap.add_argument("--verify-sync", action="store_true",
                    help="after the timed steps, check every rank holds bit-identical parameters")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="auto/nccl: RCCL, one rank per GPU; gloo: ranks sharing one GPU (rehearsal of the "
                         "multi-rank engine path on a 1-GPU box)")
    ap.add_argument("--grad-comm", default="auto", choices=["auto", "native", "process_group"],
                    help="gradient all-reduce: in-stream communicator (auto/native) or torch's process group")
    ap.add_argument("--dist-timeout-s", type=float, default=300.0,
                    help="bound of every wait on peers (collective watchdog; abort + non-zero exit)")
    ap.add_argument("--heartbeat-timeout-s", type=float, default=60.0)
    ap.add_argument("--t32", default="auto", choices=["auto", "off", "policy"],
                    help="policy update head kernel: the 32x32 transposed-chain kernel (csrc/phead.hip) or the "
                         "16x16 head kernel (off); auto = the Params default")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the N-GPU node run from a plain `python bench.py --gpus N`: N child ranks, this process
        # exits with their status.  It makes no HIP call at all — not even a device count: the
        # ranks check the visible devices themselves (check_world) and fail the run if short.
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    check_world(args.gpus, args.dist_backend)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # the north-star configuration at N > 1: the last epoch's value all-reduce + Adam beside the
    # next rollout (bit-identical to stream order: test_head_chains_through_rccl_bit_identical_to_fused)
    args.overlap_rollout = args.overlap_rollout == "on" or (args.overlap_rollout == "auto" and world > 1)
    args.overlap_value = args.overlap_value == "on"
    if world > 1:
        ctx = init_distributed("gpu", timeout_s=args.dist_timeout_s, backend=args.dist_backend,
                               grad_comm=args.grad_comm)
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ctx = init_single_rank_collective(dev, port=int(os.environ.get("MASTER_PORT", "29561")),
                                          timeout_s=args.dist_timeout_s, grad_comm=args.grad_comm)
    ctx.force_collectives = args.force_collectives
    hb = start_heartbeat(ctx, 5.0, args.heartbeat_timeout_s)   # None at world size 1
    E, T = args.num_envs, args.rollout_len
    rows = E * T

    def run(dtype: str):
        """W untimed + K timed iterations at ``dtype``: (elapsed max over ranks, params, worker, metrics)"""
        p = dppo_preset(device="gpu", env_name=args.env_name, num_envs=E, exploration_size=rows,
                        batch_size=args.batch_size or rows, num_epoch=args.num_epoch, dtype=dtype,
                        num_processes=ctx.world_size, seed=1, overlap_rollout=args.overlap_rollout,
                        overlap_value_epochs=args.overlap_value,
                        dist_backend=args.dist_backend, grad_comm=args.grad_comm,
                        dist_timeout_s=args.dist_timeout_s,
                        phase_timing=args.phase_timing if not args.verbose else max(args.phase_timing, 1))
        if args.t32 != "auto":
            p.phead_kernel = args.t32 == "policy"
        w = DPPOWorker(p, ctx)
        m = {}
        for i in range(args.warmup):
            m = w.iteration_step()
            if args.verbose and ctx.rank == 0:
                print(dtype, "warmup", i, json.dumps({k: round(v, 4) if isinstance(v, float) else v
                                                      for k, v in m.items()}), file=sys.stderr, flush=True)
        ctx.barrier()
        ctx.sync()                 # torch.cuda.synchronize, bounded by the collective watchdog
        t0 = time.perf_counter()
        # the production loop (run_worker): each iteration's metrics are read one iteration later,
        # so the host enqueues the next rollout while the device still runs this update.  Every
        # kernel of all K iterations is inside the timed region (closing synchronize below).
        for i in range(args.steps):
            mi = w.iteration_step(defer=True)
            if args.verbose and ctx.rank == 0 and mi:
                print(dtype, "step", i, json.dumps({k: round(v, 4) if isinstance(v, float) else v
                                                    for k, v in mi.items()}), file=sys.stderr, flush=True)
        ctx.barrier()
        ctx.sync()
        el = torch.tensor([time.perf_counter() - t0], device=ctx.device, dtype=torch.float64)
        m = w.finish_metrics() or m
        if args.verify_sync:
            in_sync = ctx.verify_replicas(w.model.flat.data)
            if ctx.rank == 0:
                print(f"{dtype} replicas_in_sync {in_sync}", file=sys.stderr, flush=True)
            if not in_sync:
                raise SystemExit("replicas diverged")
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()), p, w, m

    elapsed, p, w, m = run(args.dtype)
    if ctx.rank == 0 and ctx.world_size > 1:
        print(f"bench: grad_allreduce {'in_stream' if ctx.native is not None else 'process_group'} "
              f"backend {ctx.backend} world {ctx.world_size}", file=sys.stderr, flush=True)
    total_steps = rows * ctx.world_size * args.steps
    value = total_steps / elapsed
    heads = bool(getattr(w.engine, "heads", False))
    # the gradient all-reduce in use: native RCCL on the compute stream (csrc/comm.cpp), the gloo
    # adapter of the same in-stream engine branch, the process group's (per-head chains), or none
    # (world size 1, not forced)
    grad_ar = "none"
    if ctx.collective:
        grad_ar = ("process_group" if ctx.native is None else
                   "rccl_in_stream" if ctx.backend == "nccl" else "gloo_in_stream")
    t32_heads = ["policy"] if getattr(w.engine, "phead", False) else []
    # what the engine DID with the value-head steps (not what the flags asked for): run on the side
    # stream (a second communicator), left pending on a process-group all-reduce, or in stream order
    n_iter = args.warmup + args.steps
    side_steps, pend_steps = int(getattr(w.engine, "side_steps", 0)), int(getattr(w.engine, "pending_steps", 0))
    overlap_value_step = "side_stream" if side_steps else ("pending_work" if pend_steps else "none")
    del w
    variants = {}
    for dt in [d for d in args.variants.split(",") if d and d != args.dtype]:
        el_v, _, wv, _ = run(dt)
        variants[dt] = {"value": total_steps / el_v, "ms_per_step": el_v / args.steps * 1e3,
                        "dtype": DTYPE_LABEL[dt], "vs_headline": (total_steps / el_v) / value}
        del wv
        torch.cuda.empty_cache()
    if ctx.rank == 0:
        out = {"metric": METRIC, "value": value, "unit": "env_steps/s", "n_gpus": ctx.world_size,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": value / BASELINE_VALUE,
               "dtype": DTYPE_LABEL[args.dtype], "data": "synthetic (Humanoid-v2 obs/act dims, random-init weights)",
               "config": {"model": "reference actor-critic MLP (policy 376-100-100-17, value 376-500-100-1)",
                          "global_batch": rows * ctx.world_size, "seq_len": T,
                          "parallelism": f"dp{ctx.world_size}", "env": args.env_name,
                          "dppo_workers": ctx.world_size, "workers_per_gpu": 1, "num_envs_per_gpu": E,
                          "dist_backend": ctx.backend,
                          "rccl_world_size": (dist.get_world_size() if dist.is_initialized()
                                              and ctx.backend == "nccl" else 0),
                          "rollout_len": T, "num_epoch": args.num_epoch,
                          "minibatch_rows": p.minibatch_rows(), "overlap_rollout": args.overlap_rollout,
                          "per_head_kernels": heads, "grad_allreduce": grad_ar,
                          "t32_heads": t32_heads,
                          # counted by the engine: value-head all-reduce + Adam steps that ran on the
                          # side stream (--overlap-rollout: the last epoch's, beside the next rollout;
                          # --overlap-value: every epoch's) or pending on a process-group all-reduce
                          "overlap_value_step": overlap_value_step,
                          "overlapped_value_steps_per_iter": (side_steps + pend_steps) / max(n_iter, 1),
                          "note": ("value = total env steps/s of all n_gpus workers (one DPPO worker per GPU); "
                                   "the 8-worker node figure of the metric is the n_gpus=8 run; vs_baseline "
                                   "divides by the reference's derived 8-worker CPU node estimate (BASELINE.md)"),
                          "last_iter": {k: m[k] for k in ("loss", "mean_ep_return", "ms_rollout", "ms_values_gae",
                                                          "ms_update", "ms_obs_stats") if k in m}},
               "variants": variants}
        print(json.dumps(out), flush=True)
    if hb is not None:
        hb.stop()
    ctx.destroy()


if __name__ == "__main__":
    main()
