#!/usr/bin/env python3
"""What does a fork/join to a side HIP stream cost the compute stream when the side work has
ALREADY finished by the join?  (the round-3 probe, scripts/probe_stream_hop.py,
timed a serial ping-pong — every kernel waiting on the other stream's previous one — i.e. the
dependency latency on the critical path, not the stall of a fork whose side work is off it.)

Compute stream: N steps of a spin kernel of `--step-us` (torch.cuda._sleep).  Variants:
  plain       the N spins alone
  fork_join   per step: record(fork) on the compute stream, the side stream waits for it and runs
              a short kernel (`--side-us`), record(join) there; the compute stream spins, then waits
              for the join — the side work is done long before the join
  fork_only   the same without the join wait (what the fork itself costs)
  pingpong    the round-3 pattern: each spin alternates streams, each waiting on the other's last
Events are created once with timing disabled (hipEventDisableTiming); the elapsed time is taken
between two timing events on the compute stream.  Prints one JSON line per variant: us per step
over `plain` = the per-fork/join cost.
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--step-us", type=float, default=40.0)
    ap.add_argument("--side-us", type=float, default=10.0)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # calibrate torch.cuda._sleep cycles -> microseconds
    comp = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        torch.cuda.synchronize()
        t0.record(comp)
        fn()
        t1.record(comp)
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) * 1e3

    cyc = 100000
    us = min(timed(lambda: torch.cuda._sleep(cyc)) for _ in range(5))
    per_us = cyc / us
    step_c = int(args.step_us * per_us)
    side_c = int(args.side_us * per_us)
    forks = [torch.cuda.Event(enable_timing=False) for _ in range(args.steps)]
    joins = [torch.cuda.Event(enable_timing=False) for _ in range(args.steps)]

    def plain():
        for _ in range(args.steps):
            torch.cuda._sleep(step_c)

    def fork_join(join=True):
        for i in range(args.steps):
            forks[i].record(comp)
            side.wait_event(forks[i])
            with torch.cuda.stream(side):
                torch.cuda._sleep(side_c)
                joins[i].record(side)
            torch.cuda._sleep(step_c)
            if join:
                comp.wait_event(joins[i])

    def pingpong():
        for i in range(args.steps):
            s = side if i % 2 else comp
            o = comp if i % 2 else side
            forks[i].record(o)
            s.wait_event(forks[i])
            with torch.cuda.stream(s):
                torch.cuda._sleep(step_c)
        joins[0].record(side)
        comp.wait_event(joins[0])

    res = {"cycles_per_us": per_us, "steps": args.steps, "step_us": args.step_us, "side_us": args.side_us}
    for name, fn in (("plain", plain), ("fork_join", fork_join), ("fork_only", lambda: fork_join(False)),
                     ("pingpong", pingpong)):
        fn()   # warm
        ts = sorted(timed(fn) for _ in range(args.reps))
        res[f"{name}_us_per_step"] = ts[len(ts) // 2] / args.steps
    base = res["plain_us_per_step"]
    for name in ("fork_join", "fork_only", "pingpong"):
        res[f"{name}_overhead_us"] = res[f"{name}_us_per_step"] - base
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
