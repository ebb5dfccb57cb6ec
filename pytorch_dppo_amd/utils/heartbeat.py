"""Per-rank liveness beacons in the rendezvous store.

The reference has no failure detection: a dead worker leaves the chief polling forever
(``chief.py:13``, Q21) and a dead chief leaves workers busy-spinning (``train.py:174-175``).
Collective timeouts (``dist_timeout_s``) already turn a dead peer into an error at the next
collective; the heartbeat adds detection while a rank is NOT inside a collective (a long
rollout, checkpoint I/O, a hung kernel on one GPU) and names the rank that went silent.

Each rank runs one daemon thread that, every ``interval_s``:

* bumps its own counter key ``<prefix><rank>`` in the store,
* reads every peer's counter and remembers (on its OWN monotonic clock) when it last changed —
  no cross-host clock comparison,
* reports the peers whose counter has not moved for ``timeout_s`` to ``on_dead`` once.

A rank that finishes normally writes ``done`` and is never reported.  The thread talks to the
store through its own client connection when it can open one, so it never shares a socket
with the collectives of the main thread.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from datetime import timedelta
from typing import Callable, Dict, List, Optional

DONE = b"done"


def _own_store_client(default_store, timeout_s: float):
    """A second client connection to the rendezvous TCPStore (MASTER_ADDR/MASTER_PORT), or the
    default store when no such endpoint is known."""
    import torch.distributed as dist
    addr, port = os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")
    if addr and port:
        try:
            return dist.TCPStore(addr, int(port), is_master=False, timeout=timedelta(seconds=timeout_s),
                                 wait_for_workers=False)
        except Exception:   # e.g. an agent-hosted store on another port: fall back
            pass
    return default_store


class Heartbeat:
    def __init__(self, store, rank: int, world_size: int, interval_s: float, timeout_s: float,
                 on_dead: Optional[Callable[[List[int]], None]] = None, prefix: str = "dppo/hb/",
                 abort: Optional[Callable[[str], None]] = None):
        if interval_s <= 0:
            raise ValueError("interval_s must be > 0")
        self.store = store
        self.rank = rank
        self.world_size = world_size
        self.interval_s = float(interval_s)
        self.timeout_s = float(max(timeout_s, 2 * interval_s))
        self.on_dead = on_dead or self._default_on_dead
        self.prefix = prefix
        self.abort = abort
        self.beats = 0
        self.dead: List[int] = []
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name=f"heartbeat-r{rank}", daemon=True)

    # ------------------------------------------------------------------------------------------
    def _key(self, r: int) -> str:
        return f"{self.prefix}{r}"

    def start(self) -> "Heartbeat":
        self.store.set(self._key(self.rank), str(self.beats))
        self._thread.start()
        return self

    def stop(self, done: bool = True) -> None:
        """normal shutdown: peers stop watching this rank (``done=False`` simulates a crash)."""
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=5 * self.interval_s)
        if done:
            try:
                self.store.set(self._key(self.rank), DONE.decode())
            except Exception:
                pass

    def _run(self) -> None:
        peers = [r for r in range(self.world_size) if r != self.rank]
        seen: Dict[int, tuple] = {r: (None, time.monotonic()) for r in peers}
        reported = set()
        while not self._stop.wait(self.interval_s):
            self.beats += 1
            try:
                self.store.set(self._key(self.rank), str(self.beats))
            except Exception:
                # the store itself is gone (rank 0 hosts it): that is a dead rank 0
                self._report([0] if self.rank != 0 else [], reported)
                return
            now = time.monotonic()
            dead = []
            for r in peers:
                if r in reported:
                    continue
                v = None
                try:
                    if self.store.check([self._key(r)]):
                        v = self.store.get(self._key(r))
                except Exception:
                    v = None
                if v == DONE:
                    reported.add(r)         # finished normally: stop watching
                    continue
                if v is not None and v != seen[r][0]:
                    seen[r] = (v, now)
                elif now - seen[r][1] > self.timeout_s:
                    dead.append(r)
            if dead:
                self._report(dead, reported)

    def _report(self, dead: List[int], reported: set) -> None:
        if not dead:
            return
        reported.update(dead)
        self.dead.extend(dead)
        self.on_dead(list(dead))

    def _default_on_dead(self, dead: List[int]) -> None:
        msg = (f"[heartbeat] rank {self.rank}: rank(s) {dead} silent for > {self.timeout_s:.0f} s; "
               f"exiting instead of waiting in a collective")
        print(msg, file=sys.stderr, flush=True)
        if self.abort is not None:
            # ncclCommAbort first: a collective waiting on the dead peer must leave the GPU
            # before this process does
            try:
                self.abort(msg)
            except Exception:   # noqa: BLE001 — exiting regardless
                pass
        os._exit(75)


def start_heartbeat(ctx, interval_s: float, timeout_s: float,
                    on_dead: Optional[Callable[[List[int]], None]] = None) -> Optional[Heartbeat]:
    """Heartbeat on the process group's rendezvous store (None for a single rank / no group)."""
    import torch.distributed as dist
    if interval_s <= 0 or ctx.world_size <= 1 or not (dist.is_available() and dist.is_initialized()):
        return None
    from torch.distributed import distributed_c10d as c10d
    store = _own_store_client(c10d._get_default_store(), timeout_s)
    return Heartbeat(store, ctx.rank, ctx.world_size, interval_s, timeout_s, on_dead,
                     abort=getattr(ctx, "abort", None)).start()
