"""Loader for the in-tree HIP extension.

GPU code paths call :func:`load`, which imports ``pytorch_dppo_amd/ops/_dppo_hip*.so`` and
raises loudly if it is missing or was not built for gfx950 — there is deliberately no silent
eager fallback on a GPU box (a GPU run that did not execute our kernels must fail, not pass).
"""
from __future__ import annotations

import importlib
import os

_MOD = None

# bf16x3: split-bf16 operands, fp32-accurate on three bf16 MFMAs (ops/storage.py)
DT_CODE = {"fp32": 0, "bf16": 1, "fp8": 2, "bf16x3": 3}


def load(build_if_missing: bool = False):
    global _MOD
    if _MOD is not None:
        return _MOD
    try:
        _MOD = importlib.import_module("pytorch_dppo_amd.ops._dppo_hip")
    except ImportError as e:
        if not build_if_missing:
            raise RuntimeError(
                "HIP extension pytorch_dppo_amd/ops/_dppo_hip*.so is not built; run "
                "`python -m pytorch_dppo_amd.ops._build` (or __graft_entry__.build()) first") from e
        from . import _build
        _build.build()
        _MOD = importlib.import_module("pytorch_dppo_amd.ops._dppo_hip")
    if getattr(_MOD, "arch", None) != "gfx950":
        raise RuntimeError(f"extension built for {getattr(_MOD, 'arch', '?')}, need gfx950")
    if os.environ.get("DPPO_DEBUG_SYNC", "0") == "1":
        # debug mode: every op synchronises after its launch and raises naming the op (HIP
        # kernels are asynchronous: without this a fault surfaces at some later sync point)
        _MOD.set_debug_sync(True)
    return _MOD


def load_variant(name: str):
    """A/B diagnostics: the extension built from another source tree as ``_dppo_hip_<name>``
    (``python -m pytorch_dppo_amd.ops._build --variant <name> --src <dir>``)."""
    mod = importlib.import_module(f"pytorch_dppo_amd.ops._dppo_hip_{name}")
    if getattr(mod, "arch", None) != "gfx950":
        raise RuntimeError(f"variant {name} built for {getattr(mod, 'arch', '?')}")
    return mod


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def so_path() -> str:
    return load().__file__
