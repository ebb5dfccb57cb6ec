"""Operand storage formats of the HIP kernels (``csrc/common.h`` ``Prec<DT>``), host side.

dt code -> torch storage dtype:

* 0 fp32   ``float32``
* 1 bf16   ``bfloat16``
* 2 fp8    ``uint8`` (OCP e4m3 bytes; forward weight images only)
* 3 bf16x3 ``int32`` — split-bf16, the fp32-accurate mode: one 4-byte slot per logical
  element; in every 8-aligned group of 8 slots (32 bytes) the 8 ``hi = bf16(x)`` come first,
  then the 8 ``lo = bf16(x - hi)``.  ``numel`` counts logical elements, so every shape, offset
  and fragment-major index is the fp32 one.  ``decode(encode(x))`` is ``hi + lo`` (|err| <=
  2^-16 |x|), and ``encode(decode(s)) == s`` exactly.

These are the reference implementations the kernels are tested against (tests/) and the way
host code writes or reads a storage buffer element (constant bias rows, test inputs).
"""
from __future__ import annotations

import torch

STORAGE = {0: torch.float32, 1: torch.bfloat16, 2: torch.uint8, 3: torch.int32}
DT_S3 = 3


def _split(x: torch.Tensor):
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return hi, lo


def encode(x: torch.Tensor, dt: int) -> torch.Tensor:
    """float tensor -> storage tensor of the same shape (bf16x3: groups of 8 consecutive
    elements of the flattened tensor; its numel must be a multiple of 8)."""
    if dt != DT_S3:
        if dt == 2:
            raise ValueError("fp8 images are produced on the device (per-layer scales)")
        return x.to(STORAGE[dt])
    xf = x.float().contiguous().reshape(-1, 8)
    hi, lo = _split(xf)
    return torch.stack([hi, lo], 1).reshape(-1, 16).view(torch.int32).reshape(x.shape)


def decode(s: torch.Tensor, dt: int) -> torch.Tensor:
    """storage tensor -> float32 (bf16x3: hi + lo)."""
    if dt != DT_S3:
        if dt == 2:
            raise ValueError("fp8 images need their per-layer scales")
        return s.float()
    b = s.contiguous().reshape(-1, 8).view(torch.bfloat16).reshape(-1, 2, 8).float()
    return (b[:, 0] + b[:, 1]).reshape(s.shape)


def set_elements(buf: torch.Tensor, idx: torch.Tensor, value: float, dt: int) -> None:
    """buf.view(-1)[idx] = value in the storage format of ``dt`` (in place)."""
    flat = buf.view(-1)
    if dt == 2:       # the e4m3 byte of value (the caller applies the buffer's scale)
        flat[idx] = torch.tensor(float(value)).to(torch.float8_e4m3fn).view(torch.uint8).item()
        return
    if dt != DT_S3:
        flat[idx] = value
        return
    idx = idx.to(torch.int64)
    b = flat.view(torch.bfloat16)
    h = 2 * (idx & ~7) + (idx & 7)
    v = torch.full(idx.shape, float(value), dtype=torch.float32, device=buf.device)
    hi, lo = _split(v)
    b[h] = hi
    b[h + 8] = lo
