"""API-parity synchronisation primitives (reference ``utils.py:4-39``), over a c10d Store.

The training hot path never uses these: the reference's Counter + TrafficLight barrier (R4)
is implicit in the RCCL/gloo all-reduce here.  They exist so code written against the
reference API (a chief that waits for ``counter.get() > threshold`` and then
``traffic_light.switch()``) can run unchanged across processes — and across hosts, since a
``TCPStore`` replaces the reference's fork-inherited ``mp.Value`` + ``mp.Lock``.
``Store.add`` is atomic, so unlike the reference there is no read-modify-write race.
"""
from __future__ import annotations

import random
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


class Counter:
    """counter of worker contributions (reference ``utils.py:19-39``)."""

    def __init__(self, store: dist.Store, key: str = "dppo/counter"):
        self.store = store
        self.key = key
        self.store.add(self.key, 0)

    def get(self) -> int:
        return int(self.store.add(self.key, 0))

    def increment(self) -> None:
        self.store.add(self.key, 1)

    def reset(self) -> None:
        cur = self.get()
        self.store.add(self.key, -cur)


class TrafficLight:
    """generation flag toggled by the chief to release workers (reference ``utils.py:4-17``).

    Stored as a monotonically increasing generation number; ``get`` returns its parity, so a
    waiter comparing against the value it saw before waiting behaves exactly like the
    reference boolean."""

    def __init__(self, store: dist.Store, key: str = "dppo/light"):
        self.store = store
        self.key = key
        self.store.add(self.key, 0)

    def get(self) -> bool:
        return bool(int(self.store.add(self.key, 0)) & 1)

    def switch(self) -> None:
        self.store.add(self.key, 1)


class ReplayMemory:
    """tensor rollout memory with the reference API (``train.py:17-33``, ``ppo.py:44-60``):
    ``push(events)`` appends per-step tuples with FIFO eviction at ``capacity``; ``sample(n)``
    draws n distinct steps and concatenates each field; ``clear()``.

    Storage is one list of per-field tensors; sampling uses a seedable generator (the
    reference used the unseeded global ``random``)."""

    def __init__(self, capacity: int, seed: Optional[int] = None):
        self.capacity = int(capacity)
        self.memory: List[tuple] = []
        self._rng = random.Random(seed)

    def push(self, events: Sequence[Sequence[torch.Tensor]]) -> None:
        for ev in zip(*events):
            self.memory.append(ev)
            if len(self.memory) > self.capacity:
                del self.memory[0]

    def clear(self) -> None:
        self.memory = []

    def __len__(self) -> int:
        return len(self.memory)

    def sample(self, batch_size: int):
        batch = self._rng.sample(self.memory, batch_size)
        return [torch.cat(list(field), 0) for field in zip(*batch)]
