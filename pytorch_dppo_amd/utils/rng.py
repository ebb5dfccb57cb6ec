"""Counter-based RNG shared bit-for-bit (up to libm ulps) by the torch path and the HIP kernels.

The reference draws exploration noise with the global ``torch.randn`` (``train.py:88``,
``ppo.py:93``) and minibatches with an unseeded python ``random`` shared by every forked
worker.  Here every random number is a pure function of
``(seed, stream, rank, env, step, dim)``, so a vectorised env running inside a HIP kernel and
its torch twin on the CPU produce the same trajectory, and no RNG state has to be carried
or synchronised between processes.  The mixer is the ``lowbias32`` integer hash; the HIP
side is ``csrc/common.h: hash_u32 / uniform01 / gauss``.
"""
from __future__ import annotations

import math

import torch

MASK32 = 0xFFFFFFFF
GOLDEN = 0x9E3779B9

# stream ids (must match csrc/common.h)
STREAM_ACTION = 1
STREAM_ENV = 2
STREAM_TERM = 3
STREAM_RESET = 4
STREAM_EVAL = 5


def _hash(x: torch.Tensor) -> torch.Tensor:
    x = x & MASK32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & MASK32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & MASK32
    x = x ^ (x >> 16)
    return x


def hash_py(x: int) -> int:
    x &= MASK32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & MASK32
    x ^= x >> 15
    x = (x * 0x846CA68B) & MASK32
    x ^= x >> 16
    return x


def base_key(seed: int, stream: int, rank: int) -> int:
    """Scalar prefix of the key chain (host side, passed to kernels as one u32)."""
    h = hash_py((seed ^ ((GOLDEN * stream) & MASK32)) & MASK32)
    return hash_py(h ^ (rank & MASK32))


def keyed(base: int, env: torch.Tensor, step, dim: torch.Tensor) -> torch.Tensor:
    """u32 hash of (base, env, step, dim); tensors broadcast. step may be int or tensor."""
    h = _hash(env.to(torch.int64) ^ base)
    if isinstance(step, torch.Tensor):
        h = _hash(h ^ (step.to(torch.int64) & MASK32))
    else:
        h = _hash(h ^ (int(step) & MASK32))
    return _hash(h ^ dim.to(torch.int64))


def uniform01(h: torch.Tensor) -> torch.Tensor:
    """(0,1) float32 from a u32 hash: 24 high bits, centred in the bucket."""
    return ((h >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


def gauss(base: int, env: torch.Tensor, step, dim: torch.Tensor) -> torch.Tensor:
    """Standard normal by Box-Muller; dims 2p and 2p+1 share one uniform pair p (keys 2p, 2p+1)
    and take its cosine and sine branch respectively, so a kernel draws two normals per pair."""
    dim = dim.to(torch.int64)
    p2 = (dim >> 1) * 2
    u1 = uniform01(keyed(base, env, step, p2))
    u2 = uniform01(keyed(base, env, step, p2 + 1))
    r = torch.sqrt(-2.0 * torch.log(u1))
    ang = (2.0 * math.pi) * u2
    return r * torch.where((dim & 1) == 0, torch.cos(ang), torch.sin(ang))
