"""Actor-critic MLP over ONE flat fp32 parameter buffer.

Architecture = reference ``Model`` (``model.py:8-45``):

* policy ``in -> H1 -> H2 -> A`` with tanh after the two hidden layers and a linear ``mu``,
* value  ``in -> value_mult*H1 -> H2 -> 1`` (tanh, tanh, linear),
* a state-independent ``log_std [1, A]`` initialised to 0 (``model.py:21``),
* Linear weights with torch's default init, biases zeroed (``model.py:24-27``).

Every parameter is a view into ``self.flat`` (one contiguous fp32 tensor): ``log_std`` and
the policy head, then the value head (each head one contiguous range); ``state_dict()`` and
``named_parameters_ref()`` keep the reference's ``named_parameters`` order (``log_std`` first —
root parameters precede sub-modules).  That single buffer is what the RCCL gradient all-reduce, the fused Adam kernel
and checkpointing operate on.  ``state_dict()`` returns exactly the
reference keys/shapes so ``model.pt`` loads into the reference ``Model`` with
``strict=True``.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


def pad32(x: int) -> int:
    return (x + 31) // 32 * 32


@dataclass(frozen=True)
class LayerSpec:
    name: str        # reference module name (p_fc1, p_fc2, mu, v_fc1, v_fc2, v)
    fan_in: int      # K
    fan_out: int     # N
    act: str         # tanh | linear

    @property
    def d_in(self) -> int:
        """padded input width: K real columns + 1 bias column (value 1.0), rounded to 32"""
        return pad32(self.fan_in + 1)

    @property
    def d_out(self) -> int:
        return pad32(self.fan_out + 1)


class ActorCritic(nn.Module):
    def __init__(self, num_inputs: int, num_outputs: int, hidden=(100, 100), value_mult: int = 5):
        super().__init__()
        h1, h2 = int(hidden[0]), int(hidden[1])
        self.num_inputs, self.num_outputs = int(num_inputs), int(num_outputs)
        self.hidden = (h1, h2)
        self.value_mult = int(value_mult)
        O, A, V1 = self.num_inputs, self.num_outputs, h1 * self.value_mult
        self.policy_layers: List[LayerSpec] = [
            LayerSpec("p_fc1", O, h1, "tanh"), LayerSpec("p_fc2", h1, h2, "tanh"),
            LayerSpec("mu", h2, A, "linear")]
        self.value_layers: List[LayerSpec] = [
            LayerSpec("v_fc1", O, V1, "tanh"), LayerSpec("v_fc2", V1, h2, "tanh"),
            LayerSpec("v", h2, 1, "linear")]
        # reference named_parameters order (model.py:21 log_std is a root param -> first)
        order = [("log_std", (1, A))]
        for name in ("p_fc1", "p_fc2", "v_fc1", "v_fc2", "mu", "v"):
            ls = self.layer(name)
            order += [(f"{name}.weight", (ls.fan_out, ls.fan_in)), (f"{name}.bias", (ls.fan_out,))]
        self.param_shapes: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict(order)
        # memory order of the flat buffer: log_std and the policy head first, then the value head,
        # so each head's parameters (and gradient, and Adam state) are ONE contiguous range — the
        # HIP engine updates and all-reduces the two heads as independent chains.  state_dict()
        # keeps the reference key order regardless (it is built from views).
        mem = ["log_std"] + [f"{n}.{s}" for n in ("p_fc1", "p_fc2", "mu", "v_fc1", "v_fc2", "v")
                             for s in ("weight", "bias")]
        self.offsets: Dict[str, Tuple[int, int]] = {}
        off = 0
        for k in mem:
            n = math.prod(self.param_shapes[k])
            self.offsets[k] = (off, n)
            off += n
        self.num_params = off
        # [lo, hi) of each head in the flat buffer (log_std belongs to the policy)
        self.head_ranges: Dict[str, Tuple[int, int]] = {"policy": (0, self.offsets["v_fc1.weight"][0]),
                                                        "value": (self.offsets["v_fc1.weight"][0], off)}
        self.flat = nn.Parameter(torch.zeros(off, dtype=torch.float32))
        self.reset_parameters()

    # ------------------------------------------------------------------------------------
    def layer(self, name: str) -> LayerSpec:
        for ls in self.policy_layers + self.value_layers:
            if ls.name == name:
                return ls
        raise KeyError(name)

    @torch.no_grad()
    def reset_parameters(self) -> None:
        """Default nn.Linear init in the reference construction order (model.py:14-22), so the
        same torch seed yields the same weights as the reference ``Model``; biases -> 0."""
        for name in ("p_fc1", "p_fc2", "v_fc1", "v_fc2", "mu", "v"):
            ls = self.layer(name)
            lin = nn.Linear(ls.fan_in, ls.fan_out)  # consumes RNG exactly like the reference
            self.view(f"{name}.weight").copy_(lin.weight)
            self.view(f"{name}.bias").zero_()
        self.view("log_std").zero_()

    def view(self, key: str, t: torch.Tensor = None) -> torch.Tensor:
        off, n = self.offsets[key]
        base = self.flat if t is None else t
        return base[off:off + n].view(self.param_shapes[key])

    def views(self, t: torch.Tensor = None) -> Dict[str, torch.Tensor]:
        return {k: self.view(k, t) for k in self.param_shapes}

    # --- forward (torch path: CPU trainer and numerical oracle) ---------------------------
    def forward(self, x: torch.Tensor):
        """returns (mu [B,A], log_std [1,A], v [B,1])"""
        p = self.views()
        h = torch.tanh(F.linear(x, p["p_fc1.weight"], p["p_fc1.bias"]))
        h = torch.tanh(F.linear(h, p["p_fc2.weight"], p["p_fc2.bias"]))
        mu = F.linear(h, p["mu.weight"], p["mu.bias"])
        g = torch.tanh(F.linear(x, p["v_fc1.weight"], p["v_fc1.bias"]))
        g = torch.tanh(F.linear(g, p["v_fc2.weight"], p["v_fc2.bias"]))
        v = F.linear(g, p["v.weight"], p["v.bias"])
        return mu, p["log_std"], v

    def reference_forward(self, x: torch.Tensor):
        """(mu, sigma_sq, v) exactly as ``model.py:35-45`` returns them."""
        mu, log_std, v = self.forward(x)
        return mu, torch.exp(log_std), v

    # --- reference-compatible state dict ---------------------------------------------------
    def state_dict(self, *args, **kwargs):  # noqa: D401
        """Reference keys/shapes (model.py), fp32 CPU copies."""
        out = OrderedDict()
        for k in self.param_shapes:
            out[k] = self.view(k).detach().to("cpu", torch.float32).clone()
        return out

    @torch.no_grad()
    def load_state_dict(self, sd, strict: bool = True):
        keys = list(self.param_shapes)
        missing = [k for k in keys if k not in sd]
        unexpected = [k for k in sd if k not in self.param_shapes]
        if strict and (missing or unexpected):
            raise RuntimeError(f"state_dict mismatch: missing={missing} unexpected={unexpected}")
        for k in keys:
            if k in sd:
                src = torch.as_tensor(sd[k])
                if tuple(src.shape) != self.param_shapes[k]:
                    raise RuntimeError(f"shape mismatch for {k}: {tuple(src.shape)} vs {self.param_shapes[k]}")
                self.view(k).copy_(src.to(self.flat.device, torch.float32))
        return None

    def named_parameters_ref(self):
        """(name, view) pairs in the reference order (model.py:24 iteration order)."""
        return [(k, self.view(k)) for k in self.param_shapes]

    # --- packed layout for the HIP kernels ----------------------------------------------------
    def packed_layout(self) -> "PackedLayout":
        return PackedLayout(self)


def fm_index(r: torch.Tensor, c: torch.Tensor, cols: int) -> torch.Tensor:
    """Fragment-major element index of (r, c) in a [rows][cols] matrix — csrc/common.h fm_index.

    16x32 blocks, block-row-major; inside a block lane = (r % 16) + 16 * ((c % 32) // 8) holds
    the 8 elements c % 8 contiguously, so one MFMA operand fragment is one contiguous read."""
    r = r.to(torch.int64)
    c = c.to(torch.int64)
    return (((r // 16) * (cols // 32) + c // 32) * 512 + (((r % 16) + ((c % 32) // 8) * 16) * 8) + (c % 8))


class PackedLayout:
    """Padded weight images consumed by the MFMA kernels (csrc/mlp.hip, csrc/rollout.hip).

    For each layer (order p_fc1, p_fc2, mu, v_fc1, v_fc2, v) in one buffer:
      Wp  [d_out][d_in]: Wp[n][k] = W[n][k] (k < K), Wp[n][K] = b[n], zeros elsewhere
      Wpt [d_in][d_out]: transpose of Wp (dgrad operand) — for every layer but the first of each
                         head: no kernel back-propagates into the observations, so p_fc1 / v_fc1
                         have no transposed image (``wt_off`` aliases their forward image, and
                         ``flat_to_wt`` is -1 there: the Adam kernels skip ~80 % of the scattered
                         transposed-image stores)
    Both are stored FRAGMENT-MAJOR (:func:`fm_index`), so a kernel's B-operand fragment is a
    contiguous 1 KiB read.  The bias sits in column K because every activation tile carries a
    constant-1 column at index K (SURVEY §7.4 hard part 1: padded math == unpadded math),
    which also makes the wgrad GEMM emit the bias gradient as column K.
    ``flat_to_w`` / ``flat_to_wt`` map every flat-buffer index to its element in the two
    images (-1 for log_std); the fused Adam kernel uses them to refresh the images.
    """

    ORDER = ("p_fc1", "p_fc2", "mu", "v_fc1", "v_fc2", "v")
    NO_WT = ("p_fc1", "v_fc1")   # first layer of each head: no dgrad operand

    def __init__(self, model: ActorCritic):
        self.layers = [model.layer(n) for n in self.ORDER]
        self.w_off: Dict[str, int] = {}
        self.wt_off: Dict[str, int] = {}
        off = 0
        for ls in self.layers:
            self.w_off[ls.name] = off
            off += ls.d_out * ls.d_in
            if ls.name in self.NO_WT:
                self.wt_off[ls.name] = self.w_off[ls.name]
                continue
            self.wt_off[ls.name] = off
            off += ls.d_in * ls.d_out
        self.total = off
        n = model.num_params
        w_map = torch.full((n,), -1, dtype=torch.int32)
        wt_map = torch.full((n,), -1, dtype=torch.int32)
        for ls in self.layers:
            woff, wn = model.offsets[f"{ls.name}.weight"]
            nn_ = torch.arange(ls.fan_out).repeat_interleave(ls.fan_in)
            kk = torch.arange(ls.fan_in).repeat(ls.fan_out)
            w_map[woff:woff + wn] = (self.w_off[ls.name] + fm_index(nn_, kk, ls.d_in)).to(torch.int32)
            boff, bn = model.offsets[f"{ls.name}.bias"]
            nb = torch.arange(ls.fan_out)
            kb = torch.full_like(nb, ls.fan_in)
            w_map[boff:boff + bn] = (self.w_off[ls.name] + fm_index(nb, kb, ls.d_in)).to(torch.int32)
            if ls.name in self.NO_WT:
                continue
            wt_map[woff:woff + wn] = (self.wt_off[ls.name] + fm_index(kk, nn_, ls.d_out)).to(torch.int32)
            wt_map[boff:boff + bn] = (self.wt_off[ls.name] + fm_index(kb, nb, ls.d_out)).to(torch.int32)
        self.flat_to_w = w_map
        self.flat_to_wt = wt_map

    def _rowmajor(self, img: torch.Tensor, off: int, rows: int, cols: int) -> torch.Tensor:
        r = torch.arange(rows, device=img.device).repeat_interleave(cols)
        c = torch.arange(cols, device=img.device).repeat(rows)
        return img[off + fm_index(r, c, cols)].view(rows, cols)

    def image_w(self, img: torch.Tensor, name: str) -> torch.Tensor:
        """row-major view [d_out][d_in] of layer ``name``'s forward image (tests/debug)."""
        ls = next(l for l in self.layers if l.name == name)
        return self._rowmajor(img, self.w_off[name], ls.d_out, ls.d_in)

    def image_wt(self, img: torch.Tensor, name: str) -> torch.Tensor:
        ls = next(l for l in self.layers if l.name == name)
        return self._rowmajor(img, self.wt_off[name], ls.d_in, ls.d_out)

    def pack(self, flat: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
        """Reference implementation of the image packing (torch; tests + CPU fallback)."""
        out = torch.zeros(self.total, dtype=torch.float32, device=flat.device)
        m = self.flat_to_w.to(flat.device).long()
        mt = self.flat_to_wt.to(flat.device).long()
        sel = m >= 0
        out[m[sel]] = flat[sel].float()
        selt = mt >= 0
        out[mt[selt]] = flat[selt].float()
        return out.to(dtype)
