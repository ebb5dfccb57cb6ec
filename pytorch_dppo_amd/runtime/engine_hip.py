"""HIP engine: the MI355X execution path of one DPPO worker (one process per GPU).

Per iteration (all device work on the current HIP stream, no host sync until the end):

  rollout   1 launch  csrc/rollout.hip   T env steps of E envs fused (norm, policy MFMA, sample,
                                         log-prob, env physics) -> [T][E] buffer in HBM
  values    1 launch  csrc/mlp.hip       V(s) for all (T+1)*E rows (value head on MFMA)
  gae       1 launch  csrc/optim.hip     one lane per env reverse scan
  per minibatch (= one synchronous global step, train.py:133-175 / chief.py:13-20), step():
    split-bf16 + the reference network (the headline): the two heads are independent chains,
      per head  mlp_head (fwd+loss+dgrad, csrc/mlp_head.hip) -> wgrad (its layers) -> gather+Adam
      world size > 1: gather -> async RCCL all-reduce of the head's flat range -> Adam, with each
      head's all-reduce in flight while the other head's kernels run (policy step e's beside
      value step e's kernels, value step e's beside policy step e+1's)
    otherwise: mlp_train (both heads) -> wgrad -> grad_gather [-> all-reduce] -> Adam
    with clipping (ppo preset): gathers -> all-reduce -> sumsq + Adam over the whole vector

The packed weight images (PackedLayout) hold every layer as [d_out][d_in] and its transpose
in the MFMA operand precision (fp32 / bf16), the bias folded into column K.
"""
from __future__ import annotations

import contextlib
import math
from typing import Dict, Optional

import torch

from ..config import Params
from ..models.actor_critic import ActorCritic, PackedLayout, fm_index
from ..ops import native, storage
from ..utils import rng
from ..utils.obs_stats import RunningObsStats

STORAGE = storage.STORAGE
NPART_FIXED = 8
Q8_SX, Q8_SH = 64.0, 256.0   # fixed e4m3 operand scales of the observations / tanh activations (csrc/common.h)
Q8_SUB = 64                  # sub-slots per tensor of the gradient-amax ring (csrc/kernels.h)
WT = 128            # operand-buffer row padding (csrc/kernels.h WGRAD_TILE)


def wgrad_tile_ok(nq: int, kq: int, wide: bool = False) -> bool:
    """the quadrant tiles the wgrad kernel runs (csrc/wgrad.hip wgrad_task_ok): one quadrant per wave
    of the 8-wave workgroup (nq*kq <= 8, nq + kq <= 6: 24 fragment slots per ring stage), or with
    ``wide`` (split-bf16 / bf16) two per wave (9-16 quadrants, nq even, nq + kq <= 10: 40 slots)"""
    if nq < 1 or kq < 1:
        return False
    if nq * kq <= 8:
        return nq + kq <= 6
    return wide and nq * kq <= 16 and nq % 2 == 0 and nq + kq <= 10


def wgrad_tiles(li: int, n: int, k: int, wide: bool = False):
    """Output tiles of one layer's weight gradient ([n][k], k including the bias column) for the
    wgrad kernel: (layer, n0, k0, nq, kq), a tile = nq x kq quadrants of 64x64 (wgrad_tile_ok).  The
    kernel streams (nq + kq) * 64 operand rows per 32-row k-step, so the (nq, kq) minimising the
    layer's total rows read wins (ties: fewer tasks, then wider n).  Humanoid v_fc1 (512 x 377):
    4x2 tiles, 2304 rows per step instead of 3072 with 128x128 tiles; ``wide``: 4x4 + 4x2 tiles,
    1792 rows per step."""
    N, K = -(-n // 64), -(-k // 64)
    best = None
    for nq in range(1, 17):
        for kq in range(1, 17):
            if nq > N or kq > K or not wgrad_tile_ok(nq, kq, wide):
                continue
            tl = []
            for a in range(0, N, nq):
                for b in range(0, K, kq):
                    tl.append((li, a * 64, b * 64, min(nq, N - a), min(kq, K - b)))
            if not all(wgrad_tile_ok(t[3], t[4], wide) for t in tl):
                continue
            cost = sum(t[3] + t[4] for t in tl)
            key = (cost, len(tl), -nq)
            if best is None or key < best[0]:
                best = (key, tl)
    return best[1]


ROLL_ROWS = 16
WGRAD_TARGET_WGS = 0     # wgrad tasks per launch; 0: one per CU of the device (256 on MI355X)


def _r(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class HipEngine:
    name = "hip"

    def __init__(self, params: Params, model: ActorCritic, env, stats: RunningObsStats,
                 device: torch.device, action_rank: int):
        if device.type != "cuda":
            raise RuntimeError("HipEngine needs a HIP device")
        self.ext = native.load()
        self.p = params
        self.model = model
        self.env = env
        self.stats = stats
        self.device = device
        # dtype fp8 (BASELINE config 5): the forward GEMMs of the rollout policy and of the value
        # pass run on the OCP e4m3 MFMA (v_mfma_f32_16x16x32_fp8_fp8) with per-layer weight
        # scales; on the per-head path the value head's fc1 in the update and every weight-gradient
        # GEMM (e4m3 operands with power-of-two scales, delayed per-tensor for the gradients: self.q8)
        # too; the loss, dgrad and the rest of the update run in bf16.  fp32 / bf16 use one
        # precision throughout.
        self.fp8 = params.dtype == "fp8"
        self.dt = native.DT_CODE["bf16"] if self.fp8 else native.DT_CODE[params.dtype]
        self.dt_fwd = native.DT_CODE[params.dtype]
        self.sdtype = STORAGE[self.dt]
        T, E, O, A = params.rollout_len, env.E, env.O, env.A
        self.T, self.E, self.O, self.A = T, E, O, A
        self.N = T * E
        L = model.packed_layout()
        self.L = L
        ls = L.layers
        self.layout = ([L.w_off[l.name] for l in ls] + [L.wt_off[l.name] for l in ls] +
                       [l.d_in for l in ls] + [l.d_out for l in ls] + [l.fan_out for l in ls])
        self.scales = [1.0] * 6
        dev = dict(device=device)
        f32 = dict(device=device, dtype=torch.float32)
        self.w_map = L.flat_to_w.to(device)
        self.wt_map = L.flat_to_wt.to(device)
        self.wimg = torch.zeros(L.total, dtype=self.sdtype, **dev)
        self.qscale = torch.empty(0, **f32)
        if self.fp8:
            self.wimg_fwd = torch.zeros(L.total, dtype=torch.uint8, **dev)
            self.qscale = torch.ones(6, **f32)
            # layer id of every flat parameter (-1: log_std) for the per-layer amax
            lid = torch.full((model.num_params,), -1, dtype=torch.int64)
            for li, l in enumerate(ls):
                for suffix in ("weight", "bias"):
                    o, n_ = model.offsets[f"{l.name}.{suffix}"]
                    lid[o:o + n_] = li
            # the device refresh indexes qscale[lid]: validate the static map once here
            assert bool(((lid >= 0) == (L.flat_to_w >= 0)).all()) and int(lid.max()) < 6
            self.layer_id = lid.to(torch.int32).to(device)
            self.fp8_part = torch.zeros(128 * 6, **f32)   # per-block layer maxima (fp8_amax_kernel)
        else:
            self.wimg_fwd = self.wimg
        self.d0 = ls[0].d_in
        self.x_buf = torch.zeros((T + 1) * E, self.d0, dtype=self.sdtype, **dev)
        self.actions = torch.zeros(self.N, A, **f32)
        self.logp = torch.zeros(self.N, **f32)
        self.rewards = torch.zeros(self.N, **f32)
        self.dones = torch.zeros(self.N, **f32)
        self.values_buf = torch.zeros((T + 1) * E, **f32)
        self.adv = torch.zeros(self.N, **f32)
        self.ret = torch.zeros(self.N, **f32)
        self.mu_prev = torch.zeros(self.N, A, **f32)
        self.v_prev = torch.zeros(self.N, **f32)
        self.log_std_old = torch.zeros(A, **f32)
        nroll = (E + ROLL_ROWS - 1) // ROLL_ROWS
        self.mom = torch.zeros(nroll, 2, O, **f32)
        self.epstat = torch.zeros(nroll, 2, **f32)
        self.ep_sum = torch.zeros(2, dtype=torch.float64, device=device)
        self._step_bufs = None     # per-step obs-norm mode: the steps' rollout moments / episode stats
        self._sn_cap = None        # per-step obs-norm launch: co-resident grid cap of this device
        self._sn_bufs = None       # its granule buffers, timeout word (+ pinned copy)
        self._sn_epoch = 1         # its next granule tag (never reused)
        self._obs_scratch = None   # obs_observe partials + fp64 sums
        # ---- update geometry ----
        self.mb = params.minibatch_rows()
        # per-head streaming kernels (csrc/mlp_head.hip, 128 rows per workgroup): split-bf16 and
        # the reference network, at minibatches of at least one full round of 128-row workgroups
        # (one per CU): below that the two-head tile kernel's smaller workgroups fill the chip better
        # (measured, 16,384 rows: 0.716 vs 0.836 ms per iteration at bf16, 1.61 vs 1.71 at bf16x3;
        # 65,536 rows: 4.2 vs 4.9 ms at bf16x3).  Params.update_kernels heads / tile force one path.
        mode = params.update_kernels
        ncu = (torch.cuda.get_device_properties(device).multi_processor_count if device.type == "cuda" else 256)
        self.heads = (mode != "tile" and bool(self.ext.head_applies(self.dt, self.layout, A))
                      and (mode == "heads" or params.minibatch_rows() >= 128 * ncu))
        # fp8 mode on the per-head path: the wgrad operands (x^T, h1^T, g1^T, g2^T of both heads)
        # are e4m3 bytes with power-of-two scales — fixed for the activations, delayed per-tensor
        # for the gradients (csrc/common.h Q8) — and the wgrad runs on the e4m3 MFMA: half the
        # operand bytes of the bf16 update's HBM round trip.  fp8_wgrad_operands=False: bf16 operands.
        self.q8 = self.fp8 and self.heads and bool(params.fp8_wgrad_operands)
        # (the value head's update stays on the 16x16 head kernel: its 32x32 one-wave-per-SIMD form
        # measured slower at every step, docs/ARCHITECTURE.md §13)
        # the policy head's update on the transposed-chain kernel too (csrc/phead.hip): h1p / g1p /
        # g2p row-major, and the observation operand of p_fc1 AND v_fc1 row-major — x_buf itself
        # for a full-batch step (no x^T anywhere: the rollout skips writing it), the kernel's
        # gathered rows in xT for a minibatch
        self.phead = (self.heads and not self.fp8 and bool(params.phead_kernel)
                      and bool(self.ext.phead_train_applies(self.dt, self.layout, A)))
        # ... summing p_fc2's weight gradient itself at bf16x3 (h1p / g2p never reach HBM: 4.26 ->
        # 4.15 ms per iteration); at bf16 their round trip is half the bytes and storing them for
        # the wgrad is faster (2.27 vs 2.36 ms; same box, profiles/r5/ab_p2_by_dtype.log)
        fused = params.phead_fused_dw2
        self.phead_p2 = self.phead and (fused == "on" or (fused == "auto" and self.dt == native.DT_CODE["bf16x3"]))
        # the gradient-amax ring: 3 slots x 4 tensors x 64 sub-slot lines of 32 dwords (csrc/kernels.h)
        self.q8_amax = torch.zeros(3 * 4 * Q8_SUB * 32, dtype=torch.int32, device=device)
        self._q8_next = 0          # step counter of the amax ring
        self._q8_step = 0
        self._q8_cal = [False, False]   # per head: the calibration pass ran
        # operand rows: a multiple of the update kernel's row tile (every row it writes has a
        # column) and of 64 (wgrad consumes k-steps in pairs, csrc/wgrad.hip)
        self.ldT = _r(self.mb, 128 if self.heads else 64)
        self.npart = NPART_FIXED + A
        # per-workgroup partials, sized for the smallest row tile (16) so a tile change
        # (set_mlp_rows, A/B diagnostics) never outgrows it
        self.part = torch.zeros(self.ldT // 16, self.npart, **f32)
        # per-head partial rows (one per 128-row workgroup): policy [8 loss terms | A dlog_std],
        # value [8 loss terms]; the loss columns each head's gather owns
        # policy [loss terms (its columns) | A dlog_std | pad | dW_mu [32][128]], value [loss
        # column 1 | .. | dW_v [128]] — the narrow output layers' weight gradients are summed in
        # the head kernels (csrc/mlp_head.hip) instead of streaming two more operand pairs through
        # the wgrad
        self.nhead_blk = self.ldT // 128
        self.part_dw = [_r(8 + A, 4), 8]
        # (the 32x32 policy head at bf16x3 also sums p_fc2's weight gradient [128][128] right after
        # dW_mu: p_fc2 leaves the wgrad, and h1p / g2p their HBM round trip)
        np_pol = self.part_dw[0] + 32 * 128 + (128 * 128 if self.phead_p2 else 0)
        nv_val = 128
        self.part_h = [torch.zeros(self.nhead_blk, np_pol, **f32), torch.zeros(self.nhead_blk, 8 + nv_val, **f32)]
        # world size 1: both head kernels write ONE partial buffer (policy its columns, value
        # column 1 and its dW_v after the policy's block) and one wgrad + gather/Adam launch
        # covers both heads (the observation^T operand is streamed once for p_fc1 and v_fc1)
        self.part_joint = torch.zeros(self.nhead_blk, np_pol + nv_val, **f32)
        self.part_dw_joint = [self.part_dw[0], np_pol]
        self.head_range = [model.head_ranges["policy"], model.head_ranges["value"]]
        self.head_order = (0, 1)     # launch order of the joint head kernels (A/B: scripts/ab_iter.py)
        if params.mlp_rows:                     # diagnostics: force the fused-kernel row tile
            self.ext.set_mlp_rows(int(params.mlp_rows))
        self.sync_tile()
        # transposed operand buffers (feature-major), heights padded to the wgrad tile
        lp1, lp2, lmu, lv1, lv2, lv = ls
        x_rows = [lp1.d_in, lp2.d_in, lmu.d_in, lv1.d_in, lv2.d_in, lv.d_in]
        g_rows = [lp1.fan_out, lp2.fan_out, lmu.fan_out, lv1.fan_out, lv2.fan_out, lv.fan_out]
        self.x_rows = [_r(r, WT) for r in x_rows]
        self.g_rows = [_r(r, WT) for r in g_rows]
        opd = torch.uint8 if self.q8 else self.sdtype
        mk = lambda rows: torch.zeros(rows, self.ldT, dtype=opd, **dev)
        self.xT = mk(self.x_rows[0])                       # shared by p_fc1 and v_fc1
        self.h1pT, self.h2pT = mk(self.x_rows[1]), mk(self.x_rows[2])
        self.h1vT, self.h2vT = mk(self.x_rows[4]), mk(self.x_rows[5])
        self.g1pT, self.g2pT, self.g3pT = mk(self.g_rows[0]), mk(self.g_rows[1]), mk(self.g_rows[2])
        self.g1vT, self.g2vT, self.g3vT = mk(self.g_rows[3]), mk(self.g_rows[4]), mk(self.g_rows[5])
        self.tbufs = [self.xT, self.h1pT, self.h2pT, self.h1vT, self.h2vT,
                      self.g1pT, self.g2pT, self.g3pT, self.g1vT, self.g2vT, self.g3vT]
        self.wg_g = [self.g1pT, self.g2pT, self.g3pT, self.g1vT, self.g2vT, self.g3vT]
        self.wg_x = [self.xT, self.h1pT, self.h2pT, self.xT, self.h1vT, self.h2vT]
        # constant bias rows of the hidden-activation operands (the kernel writes rows < n_out;
        # row n_out == 1 makes the wgrad GEMM emit the bias gradient as column K).  The operand
        # buffers are fragment-major, so "row r" is a scattered index set.
        cols = torch.arange(self.ldT, device=device)
        # (row-major h1v / h1p: the t32 kernels write their bias columns themselves)
        bias_rows = [(self.h2pT, lp2.fan_out), (self.h2vT, lv2.fan_out), (self.h1vT, lv1.fan_out)]
        if not self.phead:
            bias_rows.append((self.h1pT, lp1.fan_out))
        # wgrad operand layout flags (dY side of the 6 layers, then X side; 1 row-major [ldT][features]):
        # under the 32x32 policy head p_fc1's / p_fc2's dY (g1p, g2p), p_fc2's X (h1p) and the
        # observation operand of both fc1 layers
        self.rm = [0] * 12
        self.wg_x_full = self.wg_x
        if self.phead:
            self.rm[0] = self.rm[1] = self.rm[6 + 0] = self.rm[6 + 1] = self.rm[6 + 3] = 1
            assert self.x_rows[0] == self.d0, "row-major observation operand: x_buf rows are d0 wide"
            # a full-batch step reads the observation rows straight from x_buf (rows [0, ldT) of
            # its N + E rows)
            if self.ldT <= self.x_buf.shape[0]:
                xb = self.x_buf.view(-1)
                self.wg_x_full = [xb, self.h1pT, self.h2pT, xb, self.h1vT, self.h2vT]
        # X side of p_fc1 / v_fc1 per step under the 32x32 policy head: "fm" = the rollout's
        # fragment-major x^T (full batch), "buf" = x_buf's rows (full batch without it), "mb" = the
        # rows the policy kernel gathered into xT (minibatch); rm_xfm = the flags of "fm"
        self.rm_xfm = list(self.rm)
        self.rm_xfm[6 + 0] = self.rm_xfm[6 + 3] = 0
        self._x_mode = "fm"
        for buf, r in bias_rows:
            if self.q8:       # e4m3 bytes of the activation scale (Q8_SH = 256: exact)
                storage.set_elements(buf, fm_index(torch.full_like(cols, r), cols, self.ldT), Q8_SH, 2)
            else:
                storage.set_elements(buf, fm_index(torch.full_like(cols, r), cols, self.ldT), 1.0, self.dt)
        # wgrad tiles of up to 16 quadrants, two per wave (csrc/wgrad.hip; split-bf16 / bf16 operands):
        # fewer operand rows streamed per output (v_fc1 1792 instead of 2304 rows per k-step), more
        # slab chunks for the gather; per iteration −0.4 % at bf16x3, −2 % at bf16 (same process,
        # profiles/r6/ab_heads_wide_*.log).  Restricting it to the fc1 layers was slower than both.
        self.wgrad_wide = bool(params.wgrad_wide) and self.dt in (native.DT_CODE["bf16x3"], native.DT_CODE["bf16"]) \
            and not self.q8
        self._build_wgrad_plan(model)
        if self.heads:
            # the joint (one-bucket) plan of world size 1 beside the per-head buckets
            heads_buckets, heads_src = self.buckets, (self.src_off, self.src_meta)
            self._build_wgrad_plan(model, joint=True)
            self.joint_bucket, self.joint_src = self.buckets[0], (self.src_off, self.src_meta)
            self.buckets, (self.src_off, self.src_meta) = heads_buckets, heads_src
        self.items = self._reduce_items(model)
        # ---- optimizer state ----
        n = model.num_params
        self.grad_flat = torch.zeros(n, **f32)
        self.adam_m = torch.zeros(n, **f32)
        self.adam_v = torch.zeros(n, **f32)
        self.adam_state = torch.zeros(4, **f32)
        self.adam_step = 0
        # per-block gradient sums of squares of whichever Adam path ran; the fused gather+Adam
        # launch uses one block per entry: A + 8 reduction blocks plus one per 256 elements
        # launch (one element per thread: a grid-stride second pass would double the load latency
        # chain of the blocks that take it) needs A + 8 reduction blocks plus one per 256 elements
        n_whole = min(4096, (n - self.A + 255) // 256 + self.A + 8)
        # (the fused gather + Adam launch takes one block per 32 reduce items first: with the fused
        # narrow / second-layer weight gradients there are tens of thousands of items)
        # (blocks of 32 items, csrc/kernels.h ITEM_IPB; blocks of 8 measured no faster, profiles/r6/ab_iter_phead_kb_vs_plain_ipb8_*.log)
        n_whole = min(4096, max(n_whole, -(-len(self.items["joint"][0]) // 32) + (n + 255) // 256))
        # per-head regions (fixed: every head launch writes each block of its region): policy
        # [0, np_), value [np_, np_ + nv_)
        (plo, phi), (vlo, vhi) = self.head_range
        np_ = min(4096, self.A + 8 + (phi - self.A + 255) // 256)
        nv_ = min(4096, 8 + (vhi - vlo + 255) // 256)
        self.norm_regions = [(0, np_), (np_, np_ + nv_)]
        self.norm_part = torch.zeros(max(n_whole, np_ + nv_), **f32)
        self.norm_n_whole = n_whole
        self._norm_n = n_whole       # entries the last Adam path wrote (metrics_pack sums them)
        # a value-head step not yet applied: ("work", all-reduce work, step, mean) on the
        # process-group chains, or ("side", None, step, mean) when it runs on the side stream
        self._pending_value = None
        self._side: Optional[torch.cuda.Stream] = None   # the side stream of the overlapped value step
        self.side_steps = 0          # value steps run on the side stream (bench / tests report it)
        self.pending_steps = 0       # value steps left pending on a process-group all-reduce
        # world-size-1 fast path: grad_gather + no-clip Adam in one launch (fused_apply=False: off)
        self.fused_apply = bool(params.fused_apply)
        self.idx_dev = torch.zeros(self.ldT, dtype=torch.int32, **dev)
        self.key_action = rng.base_key(params.seed, rng.STREAM_ACTION, action_rank)
        self.empty = torch.empty(0, dtype=torch.int32, **dev)
        self.no_q = torch.empty(0, **f32)
        self.no_u8 = torch.empty(0, dtype=torch.uint8, **dev)
        self._first_step = True
        self._loss_dev: Optional[torch.Tensor] = None
        self.local_stats: Optional[RunningObsStats] = None
        self.loss_sums = torch.zeros(NPART_FIXED, **f32)
        self.metrics_buf = torch.zeros(2 + NPART_FIXED + 1, dtype=torch.float64, **dev)
        self.empty_x = torch.empty(0, dtype=self.sdtype, **dev)
        self.x_raw: Optional[torch.Tensor] = None   # compat Q8: raw bootstrap rows (values())
        # the rollout can emit the full-batch x^T operand when the update is one full-batch step
        # (Q8: the policy kernel writes the e4m3 x^T in the first full-batch step instead)
        self.xT_from_rollout = (self.mb == self.N and self.ldT == self.N and E % 16 == 0 and self.N % 32 == 0
                                and params.obs_norm_update == "rollout" and not self.q8
                                and not (self.phead and self.wg_x_full is not self.wg_x))
        self._xT_valid = False   # True once a rollout wrote x^T for the current buffer contents
        self.s12 = torch.zeros(2, O, dtype=torch.float64, **dev)
        stats.device_merge = self._device_merge
        # host-stepped env (--env-backend gym): no in-kernel dynamics; rollout() takes the host
        # path (_rollout_host) and the update runs on the HIP kernels as usual
        self.host_env = bool(getattr(env, "host_stepped", False))
        obs0 = env.reset()
        self._host_obs = obs0.to(device) if self.host_env else None
        self.params_changed()

    # ------------------------------------------------------------------------------------------
    def _build_wgrad_plan(self, model: ActorCritic, target_wgs: Optional[int] = None, joint: bool = False) -> None:
        """Task lists of the grouped split-K wgrad launches: (layer, output tile, batch chunk),
        output tiles from wgrad_tiles().

        One *bucket* = one wgrad launch + one gather launch over a contiguous flat range of the
        gradient.  Per-head kernels: bucket 0 = the policy layers p_fc1, p_fc2 (flat
        [A, v_fc1.weight)), bucket 1 = the value layers v_fc1, v_fc2 (flat [v_fc1.weight, n)),
        so each head's chain gathers (and all-reduces) its own range; ``joint`` (world size 1):
        those four layers in ONE bucket over [A, n).  The narrow output layers mu and v, log_std
        and the loss terms are the head kernels' reduce items (partial-row columns, _reduce_items),
        so their elements carry src_meta 0.  One-kernel path: every layer in one bucket.  Each
        bucket is chunked for ~target_wgs workgroups (default Params.wgrad_wgs, 0: one per CU)
        with its own fp32 partial slab."""
        if target_wgs is None:
            target_wgs = int(self.p.wgrad_wgs or WGRAD_TARGET_WGS)
        if target_wgs <= 0:
            target_wgs = (torch.cuda.get_device_properties(self.device).multi_processor_count
                          if self.device.type == "cuda" else 256)
        ls = self.L.layers
        names = [l.name for l in ls]
        # (the 32x32 policy head at bf16x3 sums p_fc2's weight gradient itself)
        pol = ("p_fc1",) if getattr(self, "phead_p2", False) else ("p_fc1", "p_fc2")
        val = ("v_fc1", "v_fc2")
        if self.heads and joint:
            groups = [[names.index(n) for n in pol + val]]
            ranges = [(self.A, model.num_params)]
            partials = [True]
        elif self.heads:
            groups = [[names.index(n) for n in pol], [names.index(n) for n in val]]
            (_, phi), (vlo, vhi) = self.head_range
            ranges = [(self.A, phi), (vlo, vhi)]
            partials = [True, False]
        else:
            groups = [list(range(len(ls)))]
            ranges = [(self.A, model.num_params)]
            partials = [True]
        src = torch.full((model.num_params,), -1, dtype=torch.int64)
        meta = torch.zeros(model.num_params, dtype=torch.int64)
        self.buckets = []
        max_chunks = max(1, self.ldT // 64)            # a task covers >= 64 batch rows
        # Batch chunks PER TILE, in proportion to the tile's operand stream ((nq + kq) * 64 rows
        # per k-step): every task then streams about the same bytes, and the task count is
        # ~target_wgs = one workgroup per CU (the kernel is bound by each CU's operand stream, so
        # every CU gets one equal share; largest-remainder rounding).  The chunk counts are
        # dealt over the tiles of ALL buckets together, so the per-head buckets and the joint one
        # split every tile identically: each weight-gradient element is the same fixed-order sum
        # on every path (the process-group chains == the in-stream joint path, bit for bit).
        # (two quadrants per wave at split-bf16 / bf16: Params.wgrad_wide)
        wide = bool(getattr(self, "wgrad_wide", False))
        all_tiles = []  # (layer, n0, k0, nq, kq)
        for li in sorted({li for layers in groups for li in layers}):
            l = ls[li]
            all_tiles += wgrad_tiles(li, l.fan_out, l.fan_in + 1, wide)
        costs = [t[3] + t[4] for t in all_tiles]
        raw = [target_wgs * c / sum(costs) for c in costs]
        nch_all = [max(1, int(r)) for r in raw]
        rest = sorted(range(len(all_tiles)), key=lambda t: raw[t] - int(raw[t]), reverse=True)
        for t in rest[:max(0, target_wgs - sum(nch_all))]:
            nch_all[t] += 1
        nch_of = {t: min(max_chunks, n) for t, n in zip(all_tiles, nch_all)}
        for bi, (layers, (lo, hi)) in enumerate(zip(groups, ranges)):
            tiles = [t for t in all_tiles if t[0] in layers]
            nch = [nch_of[t] for t in tiles]
            tasks, tile_off, base = [], {}, 0
            for t, n in zip(tiles, nch):
                size = t[3] * t[4] * 64 * 64
                # even number of 32-row k-steps per task (e4m3: a multiple of 4)
                mc = _r(-(-self.ldT // n), 128 if getattr(self, "q8", False) else 64)
                chunks = [(c0, min(c0 + mc, self.ldT)) for c0 in range(0, self.ldT, mc)]
                tile_off[t] = (base, len(chunks), size)
                for ci, (m0, m1) in enumerate(chunks):
                    tasks.append([t[0], t[1], t[2], m0, m1, base + ci * size, t[3], t[4]])
                base += len(chunks) * size
            # XCD-aware order: workgroups b, b+8, b+16, ... are dealt to the same XCD (observed
            # round-robin placement; speed only).  Tasks sorted by batch-row position are cut
            # into 8 runs, one per XCD, so the tasks that share operand rows (all tiles of one
            # row range) run on one XCD and share its L2.
            tasks.sort(key=lambda r: (r[3] + r[4], r[0], r[1], r[2]))
            per_xcd = [[] for _ in range(8)]
            for rank, r in enumerate(tasks):
                per_xcd[rank * 8 // len(tasks)].append(r)
            order = []
            j = 0
            while any(j < len(q) for q in per_xcd):
                for q in per_xcd:
                    if j < len(q):
                        order.append(q[j])
                j += 1
            tasks_host = torch.tensor(order, dtype=torch.int32).reshape(-1).contiguous()
            # flat index -> (offset of its element in its tile's chunk-0 slab, chunk count and
            # slab stride of that tile packed as nch * 32 + size / 4096)
            for li in layers:
                l = ls[li]
                woff, wn = model.offsets[f"{l.name}.weight"]
                nn_ = torch.arange(l.fan_out).repeat_interleave(l.fan_in)
                kk = torch.arange(l.fan_in).repeat(l.fan_out)
                src[woff:woff + wn], meta[woff:woff + wn] = self._slab_index(tile_off, li, nn_, kk)
                boff, bn = model.offsets[f"{l.name}.bias"]
                nb = torch.arange(l.fan_out)
                src[boff:boff + bn], meta[boff:boff + bn] = self._slab_index(tile_off, li, nb,
                                                                             torch.full_like(nb, l.fan_in))
            # every element this bucket gathers from its slab stays inside it (grad_gather relies
            # on it); the elements without a tile (src_meta 0) are reduce items
            so, sm = src[lo:hi], meta[lo:hi]
            has = sm > 0
            reach = so + ((sm >> 5) - 1).clamp(min=0) * ((sm & 31) << 12)
            assert bool((so[has] >= 0).all()) and int(reach[has].max()) < base, "wgrad gather plan exceeds its slab"
            self.buckets.append({
                "tasks_host": tasks_host, "tasks": tasks_host.to(self.device),
                "slab": torch.zeros(base, device=self.device, dtype=torch.float32),
                "lo": lo, "hi": hi, "partials": partials[bi], "runs": self._slab_runs(sm, lo)})
        src[src < 0] = 0  # reduce items (log_std, and with the per-head kernels mu / v)
        self.src_off = src.to(torch.int32).to(self.device)
        self.src_meta = meta.to(torch.int32).to(self.device)

    def q8_maxima(self) -> torch.Tensor:
        """[3 slots][4 tensors] gradient maxima (g1p, g2p, g1v, g2v) of the amax ring (diagnostics)"""
        return self.q8_amax.view(3, 4, Q8_SUB, 32)[..., 0].view(torch.float32).amax(-1)

    def _wgrad_dt(self) -> int:
        return native.DT_CODE["fp8"] if self.q8 else self.dt

    def _q8_args(self) -> tuple:
        if self.q8:
            return (self.q8_amax, self._q8_step, [0, 1, -1, 2, 3, -1], [Q8_SX, Q8_SH, 1.0, Q8_SX, Q8_SH, 1.0])
        return (self.empty, 0, [-1] * 6, [1.0] * 6)

    def _wgrad(self, b: Dict, xmode: str) -> None:
        """one wgrad launch over bucket b's tasks (Q8: e4m3 operands, the step's scales); ``xmode``
        = where the minibatch's observation operand is (_minibatch: "fm" / "buf" / "mb")"""
        wg_x = self.wg_x_full if (self.phead and xmode == "buf") else self.wg_x
        rm = self.rm_xfm if (not self.phead or xmode == "fm") else self.rm
        self.ext.wgrad(self._wgrad_dt(), self.wg_g, wg_x, self.g_rows, self.x_rows, self.ldT, b["tasks"],
                       b["tasks_host"], b["slab"], *self._q8_args(), rm)

    def _w8(self):
        """fp8 mode: (e4m3 image, per-layer scales) for the value head's e4m3 fc1; else off"""
        return (self.wimg_fwd, self.qscale) if self.fp8 else (self.no_u8, self.no_q)

    def _f8(self, lo: int = 0, hi: Optional[int] = None):
        """fp8 mode: the Adam kernels' shadow e4m3 image (the update's fc1 reads it, csrc/mlp_head.hip
        F8) — (image, per-element layer id of the flat slice [lo, hi), per-layer scales); else off"""
        if not self.fp8:
            return (self.no_u8, self.empty, self.no_q)
        return (self.wimg_fwd, self.layer_id[lo:hi], self.qscale)

    @staticmethod
    def _slab_runs(meta_slice: torch.Tensor, lo: int) -> list:
        """the gathers' slab runs (csrc/kernels.h SlabRuns): the maximal index runs of a bucket's
        flat range [lo, hi) whose elements all have a slab source (src_meta > 0), flattened
        [lo0, hi0, ...] in absolute flat indices; the reduce items between them are not visited"""
        has = (meta_slice > 0).to(torch.int8).tolist()
        runs, start = [], None
        for k, h in enumerate(has + [0]):
            if h and start is None:
                start = k
            elif not h and start is not None:
                runs += [lo + start, lo + k]
                start = None
        assert 2 <= len(runs) <= 8, "a gather takes 1-4 slab runs"
        return runs

    def _reduce_items(self, model: ActorCritic) -> Dict[str, tuple]:
        """Reduce items of the gather launches: (partial-row column, destination) pairs, the
        destination a flat index of the gathered range or -1 - q for the loss term q.  "legacy":
        the one-kernel update's [8 loss terms | A dlog_std] rows; "policy" / "value": one head's
        partial buffer (its loss columns, log_std, and mu / v from the fused dW blocks), the value
        destinations relative to its slice; "joint": both heads in the shared buffer."""
        A = self.A
        cols: Dict[str, list] = {k: [] for k in ("legacy", "policy", "value", "joint")}
        dsts: Dict[str, list] = {k: [] for k in cols}

        def add(kind, c, d):
            cols[kind].append(int(c))
            dsts[kind].append(int(d))
        for q in range(8):
            add("legacy", q, -1 - q)
        for j in range(A):
            add("legacy", 8 + j, j)
        vlo = self.head_range[1][0]

        def narrow(kind, layer, dw, base, stride=128):
            """the weight gradient of a layer summed in a head kernel, [out][stride] at partial column
            dw (rows j, k <= fan_in: k == fan_in is the bias)"""
            l = model.layer(layer)
            wo, bo = model.offsets[f"{layer}.weight"][0], model.offsets[f"{layer}.bias"][0]
            for j in range(l.fan_out):
                for k in range(l.fan_in):
                    add(kind, dw + j * stride + k, wo - base + j * l.fan_in + k)
                add(kind, dw + j * stride + l.fan_in, bo - base + j)
        for kind, dwp, dwv, vbase in (("policy", self.part_dw[0], None, None),
                                      ("value", None, self.part_dw[1], vlo),
                                      ("joint", self.part_dw_joint[0], self.part_dw_joint[1], 0)):
            if dwp is not None:
                for q in (0, 2, 3, 4, 5, 6, 7):
                    add(kind, q, -1 - q)
                for j in range(A):
                    add(kind, 8 + j, j)
                narrow(kind, "mu", dwp, 0)
                if self.phead_p2:
                    narrow(kind, "p_fc2", dwp + 32 * 128, 0)
            if dwv is not None:
                add(kind, 1, -2)
                narrow(kind, "v", dwv, vbase)
        out = {}
        for kind in cols:
            c = torch.tensor(cols[kind], dtype=torch.int32)
            d = torch.tensor(dsts[kind], dtype=torch.int32)
            # the gather kernels index part rows and flat slices by these without a device check
            lim = {"legacy": self.npart, "policy": self.part_h[0].shape[1], "value": self.part_h[1].shape[1],
                   "joint": self.part_joint.shape[1]}[kind]
            assert int(c.min()) >= 0 and int(c.max()) < lim, kind
            assert len(set(d[d >= 0].tolist())) == int((d >= 0).sum()), kind   # one item per element
            out[kind] = (c.to(self.device), d.to(self.device))
        return out

    @staticmethod
    def _slab_index(tile_off, li, n, k):
        """dW[n][k] of layer li -> (slab offset in its tile's chunk-0 slab: tile base +
        (n - n0) * (kq * 64) + (k - k0); packed chunk count / stride of the tile)"""
        out = torch.full_like(n, -1)
        meta = torch.zeros_like(n)
        for (tl, n0, k0, nq, kq), (base, nch, size) in tile_off.items():
            if tl != li:
                continue
            m = (n >= n0) & (n < n0 + 64 * nq) & (k >= k0) & (k < k0 + 64 * kq)
            out[m] = base + (n[m] - n0) * (64 * kq) + (k[m] - k0)
            meta[m] = nch * 32 + size // 4096
        assert bool((out >= 0).all()), "wgrad tiles do not cover the layer"
        return out, meta

    # ------------------------------------------------------------------------------------------
    def sync_tile(self) -> None:
        """Row tile of the fused update kernel (64 rows when the layer set fits LDS, else 32;
        16 at fp32) and the partial-sum rows it produces; re-query after ext.set_mlp_rows."""
        xb = self.x_buf.numel() * self.x_buf.element_size()
        self.train_rows = int(self.ext.train_rows(self.dt, self.layout, self.A, xb))
        self.ntrain_blk = self.ldT // self.train_rows

    def params_changed(self) -> None:
        """re-pack the weight images from the fp32 master (after init / load / broadcast)."""
        self.ext.pack(self.model.flat.data, self.wimg, self.w_map, self.wt_map, self.dt, self.no_q)
        self.adam_state[0] = float(self.adam_step)
        self.refresh_fwd_image()

    @torch.no_grad()
    def refresh_fwd_image(self) -> None:
        """fp8 only: per-layer amax scales + e4m3 image of the current weights, on the device in
        two launches (csrc/optim.hip fp8_amax_kernel + pack_fp8_kernel; no host sync).
        s_l = amax_l / 416 keeps every weight inside e4m3's finite range (448) with headroom;
        the kernels multiply each layer's accumulator by s_l."""
        if not self.fp8:
            return
        self.ext.fp8_refresh(self.model.flat.data, self.layer_id, self.qscale, self.fp8_part, self.wimg_fwd, self.w_map,
                             self.wt_map)

    def decode(self, t: torch.Tensor) -> torch.Tensor:
        """a storage-precision buffer of this engine (x_buf, an operand buffer) as fp32"""
        return storage.decode(t, self.dt)

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        return storage.encode(x, self.dt)

    def current_obs(self) -> torch.Tensor:
        return self._host_obs if self.host_env else self.env.observe()

    def _device_merge(self, s1, s2, count, n_a, shift) -> None:
        """RunningObsStats merge on the device (csrc/obs.hip): one launch instead of ~15 ops."""
        st = self.stats
        if s1.data_ptr() == self.s12.data_ptr() and s2.data_ptr() == self.s12[1].data_ptr():
            s12 = self.s12
        else:
            s12 = torch.stack([s1.to(torch.float64), s2.to(torch.float64)]).contiguous()
        self.ext.obs_merge(s12, count, n_a, shift.contiguous(), st.mean, st.mean_diff, st.mean_f32,
                           st.inv_std_f32, 1e-2)

    def env_state(self) -> Dict:
        return self.env.state_dict()

    def load_env_state(self, d: Dict) -> None:
        self.env.load_state_dict(d)
        if self.host_env:
            # the host envs were restored (and reset): the next rollout acts on their observation,
            # not on the one the constructor's reset left (TorchEngine.load_env_state does the same)
            self._host_obs = self.env.observe().to(self.device, torch.float32)

    # ------------------------------------------------------------------------------------------
    def _launch_rollout(self, T: int, t_base: int, t0: int, norm: RunningObsStats, shift: torch.Tensor,
                        xT: Optional[torch.Tensor] = None, mom: Optional[torch.Tensor] = None,
                        epstat: Optional[torch.Tensor] = None):
        e = self.env
        kp = e.kernel_params()
        ints = [kp["kind"], self.E, self.O, self.A, e.state_dim, T, t_base, self.E, t0 & 0xFFFFFFFF,
                kp["limit"], 1 if self.p.std_convention == "var" else 0]
        keys = [kp["key_env"], kp["key_term"], kp["key_reset"], self.key_action]
        xt = xT if xT is not None else self.empty_x
        self.ext.rollout(self.dt_fwd, ROLL_ROWS, e.state, e.ep_len, e.ep_ret, self.wimg_fwd, self.layout,
                         self.scales, self.model.flat.data, norm.mean_f32, norm.inv_std_f32, shift, self.x_buf,
                         self.actions, self.logp, self.rewards, self.dones,
                         self.mom if mom is None else mom, self.epstat if epstat is None else epstat, ints, keys,
                         float(self.p.reward_clip), self.qscale, xt, self.x_rows[0])

    def _stepnorm_fits(self) -> bool:
        """the per-step normalisation launch holds every env tile co-resident on this device"""
        if self._sn_cap is None:
            e = self.env
            self._sn_cap = int(self.ext.rollout_stepnorm_cap(self.dt_fwd, ROLL_ROWS, self.layout, self.O, self.A,
                                                              e.state_dim))
        return self.mom.shape[0] <= self._sn_cap

    def _launch_stepnorm(self, ls: RunningObsStats, shift: torch.Tensor) -> None:
        """obs_norm_update='step' as one cooperative rollout launch: every step merges its batch
        into ``ls`` (in place, fp64) before normalising it (csrc/rollout.hip sn_step)."""
        if self._sn_bufs is None:
            nroll = self.mom.shape[0]
            # (csrc/kernels.h sn_g1_elems: 4-feature x 4-workgroup line blocks)
            g1n = 2 * (-(-self.O // 4)) * (-(-nroll // 4)) * 16
            self._sn_bufs = (torch.zeros(g1n, dtype=torch.int64, device=self.device),
                             torch.zeros(2 * self.O, dtype=torch.int64, device=self.device),
                             torch.zeros(1, dtype=torch.int32, device=self.device),
                             torch.zeros(1, dtype=torch.int32, pin_memory=True))
        g1, g2, err, err_host = self._sn_bufs
        if int(err_host[0]) != 0:   # (staged after an earlier launch: no sync here)
            raise RuntimeError("per-step observation normalisation launch timed out waiting for a workgroup")
        e = self.env
        kp = e.kernel_params()
        ints = [kp["kind"], self.E, self.O, self.A, e.state_dim, self.T, 0, self.E, e.t & 0xFFFFFFFF,
                kp["limit"], 1 if self.p.std_convention == "var" else 0]
        keys = [kp["key_env"], kp["key_term"], kp["key_reset"], self.key_action]
        self.ext.rollout_stepnorm(self.dt_fwd, ROLL_ROWS, e.state, e.ep_len, e.ep_ret, self.wimg_fwd, self.layout,
                                  self.scales, self.model.flat.data, shift, self.x_buf, self.actions, self.logp,
                                  self.rewards, self.dones, self.mom, self.epstat, ints, keys,
                                  float(self.p.reward_clip), self.qscale,
                                  [ls.mean, ls.mean_diff, ls.mean_f32, ls.inv_std_f32], g1, g2, err, float(ls.n),
                                  self._sn_epoch, 1e-2)
        self._sn_epoch += self.T
        ls.n += float(self.N)
        err_host.copy_(err, non_blocking=True)

    def raise_if_failed(self, sync: bool = False) -> None:
        """A per-step normalisation launch that timed out waiting for a workgroup left its buffers
        partly written: raise before anything built on them is reported or saved.  The host copy
        of the timeout word is staged behind each launch; ``sync`` waits for it (checkpoints), the
        worker's metrics resolution calls it after the iteration's event has completed."""
        if self._sn_bufs is None:
            return
        if sync:
            torch.cuda.synchronize(self.device)
        if int(self._sn_bufs[3][0]) != 0:
            raise RuntimeError("per-step observation normalisation launch timed out waiting for a workgroup: "
                               "the iteration's rollout is incomplete")

    def _observe_step(self, norm: RunningObsStats, obs: torch.Tensor, shift: torch.Tensor) -> None:
        """norm.observes(obs) as three device launches (csrc/obs.hip obs_observe), moments about
        the iteration's shift snapshot."""
        if self._obs_scratch is None:
            self._obs_scratch = (torch.zeros(int(self.ext.obs_moments_nblk(self.E)), 2, self.O,
                                             dtype=torch.float32, device=self.device),
                                 torch.zeros(2, self.O, dtype=torch.float64, device=self.device))
        part, s12 = self._obs_scratch
        self.ext.obs_observe(obs.to(self.device, torch.float32).contiguous(), shift, norm.mean, norm.mean_diff,
                             norm.mean_f32, norm.inv_std_f32, float(norm.n), part, s12, 1e-2)
        norm.n += float(obs.shape[0])

    @torch.no_grad()
    def _rollout_host(self) -> Dict:
        """T steps of a host-stepped env (gym backend, train.py:82-106 vectorised): the env runs
        on the host, so the fused rollout kernel (which steps the builtin dynamics in-kernel)
        cannot; per step the E observations are normalised and the policy head evaluated as
        device tensor ops (E rows; the env's host loop is the bottleneck here), the action noise
        and log-prob use the same keyed RNG as the kernel, and the buffer rows are written in
        the storage precision.  The rollout-time x^T operand is not emitted (the update kernel
        transposes X itself)."""
        from ..ops import oracle
        p, T, E, O = self.p, self.T, self.E, self.O
        shift = self.stats.shift().clone()
        s1 = torch.zeros(O, dtype=torch.float64, device=self.device)
        s2 = torch.zeros_like(s1)
        ep = torch.zeros(2, dtype=torch.float64, device=self.device)
        norm = self.stats
        if p.obs_norm_update == "step":
            self.local_stats = RunningObsStats(O, self.device)
            self.local_stats.copy_from(self.stats)
            norm = self.local_stats
        log_std = self.model.view("log_std")
        log_sigma = log_std if p.std_convention == "std" else 0.5 * log_std
        sigma = torch.exp(log_sigma)
        eidx = torch.arange(E, device=self.device, dtype=torch.int64)
        dims = torch.arange(self.A, device=self.device, dtype=torch.int64)
        X = torch.zeros(T + 1, E, self.d0, device=self.device)
        X[..., O] = 1.0
        obs = self._host_obs
        for t in range(T):
            _, a1, a2 = RunningObsStats.moments(obs, shift)
            s1 += a1
            s2 += a2
            if p.obs_norm_update == "step":
                self._observe_step(norm, obs, shift)
            x = norm.normalize(obs)
            mu, _, _ = self.model(x)
            eps = rng.gauss(self.key_action, eidx[:, None], self.env.t, dims[None, :])
            a = mu + sigma * eps
            logp = (-0.5 * eps * eps - 0.5 * oracle.LOG_2PI - log_sigma).sum(-1)
            nobs, r, done, info = self.env.step(a)
            r = r.to(self.device)
            if p.reward_clip > 0:
                r = r.clamp(-p.reward_clip, p.reward_clip)
            X[t, :, :O] = x
            rows = slice(t * E, (t + 1) * E)
            self.actions[rows] = a
            self.logp[rows] = logp
            self.rewards[rows] = r
            self.dones[rows] = done.to(self.device, torch.float32)
            ep[0] += float(info["ep_return_sum"])
            ep[1] += float(info["ep_count"])
            obs = nobs.to(self.device, torch.float32)
        X[T, :, :O] = norm.normalize(obs)
        self._host_obs = obs
        self.x_buf.copy_(self.encode(X.view(-1, self.d0)))
        self._xT_valid = False
        return {"count": float(self.N), "s1": s1, "s2": s2, "shift": shift,
                "ep_return_sum": ep[0], "ep_count": ep[1], "ep2": ep}

    @torch.no_grad()
    def rollout(self, stats_stream: Optional[torch.cuda.Stream] = None) -> Dict:
        """T env steps for every env.  ``stats_stream`` (rollout-mode obs stats only): the
        one-launch moment/episode-stat reduce runs there, ordered after the rollout kernel, so
        it (and the caller's merge, issued on the same stream) overlaps the value forward and
        the update; the caller orders its stream after that work before reading the stats."""
        # fp8: the weights changed during the previous update (Adam rewrites only the bf16 image);
        # before either path, so values() / GAE of a host-env rollout see the current weights too.
        # The refresh reads every layer: a value step still running on the side stream
        # (--overlap-rollout) is joined first, so fp8 runs that step in order.
        if self.fp8 or self.host_env:
            self._flush_value()
        self.refresh_fwd_image()
        if self.host_env:
            ro = self._rollout_host()
            if stats_stream is not None:
                # the caller merges the moments on stats_stream: order it after the host rollout's
                # device work, which produced them (and reads the stats the merge overwrites)
                stats_stream.wait_stream(torch.cuda.current_stream(self.device))
            return ro
        p = self.p
        if p.obs_norm_update == "rollout":
            # the shift IS the fp32 mean, no snapshot copy: its readers are the rollout kernel
            # and obs_merge, which reads shift[d] before writing mean_f32[d] in the same thread
            shift = self.stats.shift()
            # full-batch update: the rollout also writes the fragment-major x^T wgrad operand once,
            # so the 10 epochs' fused kernels skip re-transposing X (xT_ready)
            self._launch_rollout(self.T, 0, self.env.t, self.stats, shift,
                                 self.xT if self.xT_from_rollout else None)
            self._xT_valid = self.xT_from_rollout
            self.env.t += self.T
            # --overlap-rollout: the previous iteration's last value-head step (side stream) ran
            # beside the rollout kernel just enqueued (which reads only the policy); join it here,
            # before the reduce rewrites the episode stats its metrics pack read
            self._flush_value()
            # one launch: moments [nblk][2][O] -> s12, episode stats [nblk][2] -> ep_sum
            if stats_stream is not None:
                stats_stream.wait_stream(torch.cuda.current_stream(self.device))
                shift.record_stream(stats_stream)
                with torch.cuda.stream(stats_stream):
                    self.ext.obs_reduce(self.mom, self.mom.shape[0], self.O, self.s12, self.epstat, self.ep_sum)
            else:
                self.ext.obs_reduce(self.mom, self.mom.shape[0], self.O, self.s12, self.epstat, self.ep_sum)
            s1, s2 = self.s12[0], self.s12[1]
            ep = self.ep_sum
        else:
            # per-step obs-norm mode (the reference's filter updates with every observation before
            # normalising it, model.py:68 / train.py:84): step t's normalisation needs the stats of
            # step t's batch, a grid-wide dependency.  Default: ONE cooperative launch whose
            # workgroups exchange each step's moments and merged stats in-kernel
            # (csrc/rollout.hip sn_step), into the worker-local stats.  Fallback (the env tiles do
            # not fit co-resident): per step one observe (csrc/obs.hip: moments -> reduce -> merge)
            # + a one-step rollout launch, the steps' moments / episode stats in per-step slices
            # and ONE reduce after the loop.  No host sync either way.
            self._flush_value()
            shift = self.stats.shift().clone()
            ls = self.local_stats = RunningObsStats(self.O, self.device)
            ls.copy_from(self.stats)
            if self._stepnorm_fits():
                self._launch_stepnorm(ls, shift)
                self.env.t += self.T
                self.ext.obs_reduce(self.mom, self.mom.shape[0], self.O, self.s12, self.epstat, self.ep_sum)
                return {"count": float(self.N), "s1": self.s12[0], "s2": self.s12[1], "shift": shift,
                        "ep_return_sum": self.ep_sum[0], "ep_count": self.ep_sum[1], "ep2": self.ep_sum}
            T, nroll = self.T, self.mom.shape[0]
            if self._step_bufs is None or self._step_bufs[0].shape[0] != T:
                f32 = dict(dtype=torch.float32, device=self.device)
                self._step_bufs = (torch.zeros(T, nroll, 2, self.O, **f32), torch.zeros(T, nroll, 2, **f32))
            mom_t, ep_t = self._step_bufs
            for t in range(T):
                self._observe_step(ls, self.current_obs(), shift)
                self._launch_rollout(1, t, self.env.t, ls, shift, mom=mom_t[t], epstat=ep_t[t])
                self.env.t += 1
            self.ext.obs_reduce(mom_t, T * nroll, self.O, self.s12, ep_t, self.ep_sum)
            s1, s2 = self.s12[0], self.s12[1]
            ep = self.ep_sum
        # everything stays on the device: no host sync inside the iteration
        return {"count": float(self.N), "s1": s1, "s2": s2, "shift": shift,
                "ep_return_sum": ep[0], "ep_count": ep[1], "ep2": ep}

    @torch.no_grad()
    def values(self) -> None:
        self._flush_value()          # the value head must hold its last step
        M = (self.T + 1) * self.E
        if self.fp8 and self.heads:
            # fp8 mode on the per-head path: the value head's streaming forward with the e4m3 fc1
            # (fc2 / fc3 on the bf16 image; csrc/mlp_head.hip F8)
            self.ext.mlp_value(self.dt, self.x_buf, self.empty, 0, M, self.wimg, self.layout, self.scales,
                               self.model.flat.data, self.A, self.values_buf, False, self.qscale, self.wimg_fwd)
        else:
            self.ext.mlp_value(self.dt_fwd, self.x_buf, self.empty, 0, M, self.wimg_fwd, self.layout, self.scales,
                               self.model.flat.data, self.A, self.values_buf, False, self.qscale, self.no_u8)
        if self.p.compat:
            # Q8 (train.py:109-112, ppo.py:119-122): the reference bootstraps R = V(s_T) from the
            # RAW, un-normalised last state.  Rows [T*E, (T+1)*E) of values_buf get V of the env's
            # current raw observation (the rollout left the env after its last step).
            raw = self.env.observe().to(self.device, torch.float32)
            xr = torch.zeros(self.E, self.d0, device=self.device)
            xr[:, :self.O] = raw
            xr[:, self.O] = 1.0
            if self.x_raw is None:
                self.x_raw = torch.empty(self.E, self.d0, dtype=self.sdtype, device=self.device)
            self.x_raw.copy_(self.encode(xr))
            self.ext.mlp_value(self.dt_fwd, self.x_raw, self.empty, 0, self.E, self.wimg_fwd, self.layout,
                               self.scales, self.model.flat.data, self.A, self.values_buf[self.N:], False,
                               self.qscale, self.no_u8)

    @torch.no_grad()
    def gae(self) -> None:
        T, E = self.T, self.E
        self.ext.gae(self.rewards.view(T, E), self.values_buf.view(T + 1, E), self.dones.view(T, E),
                     self.adv.view(T, E), self.ret.view(T, E), float(self.p.gamma), float(self.p.gae_param), 0,
                     self.p.gae_segment())
        if self.p.normalize_adv:
            m, s = self.adv.mean(), self.adv.std()
            self.adv.sub_(m).div_(s + 1e-8)

    def begin_update(self) -> None:
        if self.p.loss == "dppo_ref":   # only the reference loss reads the previous log_std
            self.log_std_old.copy_(self.model.flat.data[:self.A])
        self._first_step = True

    # ------------------------------------------------------------------------------------------
    def _minibatch(self, idx: Optional[torch.Tensor]):
        """(index tensor, first-step flag, x^T-ready flag, x-mode) of one minibatch call.

        x-mode: where the observation operand of p_fc1 / v_fc1's weight gradient is — "fm" the
        rollout's fragment-major x^T (full batch), "buf" x_buf's own rows (full batch under the
        32x32 policy head: no x^T written), "mb" the rows the policy kernel gathers into xT
        (minibatch).  Decided here, from the minibatch alone, and passed to both the head
        kernels and the wgrad (no engine state couples them)."""
        M = self.mb
        if idx is None:
            assert M == self.N, "full-batch call needs minibatch == buffer"
            idx_t = self.empty
        else:
            idx = idx.reshape(-1)
            if idx.numel() != M:
                raise ValueError(f"minibatch has {idx.numel()} rows, engine was planned for {M}")
            lo, hi = int(idx.min()), int(idx.max())
            if lo < 0 or hi >= self.N:   # host-side range check (the launch skips the device check)
                raise IndexError(f"minibatch indices out of range [0, {self.N}): {lo}..{hi}")
            self.idx_dev[:M].copy_(idx.to(torch.int32), non_blocking=True)
            idx_t = self.idx_dev
        first, xt_ready = bool(self._first_step), bool(idx is None and self._xT_valid)
        xmode = "fm"
        if self.phead:
            # (measured: the fragment-major x^T beside the row-major policy operands made the
            # wgrad slower than x_buf's rows — 4.378 vs 4.214 ms per bf16x3 iteration, profiles/r5 —
            # so x_buf's rows come first and the rollout writes no x^T when they can serve)
            full = idx is None
            if full and self.wg_x_full is not self.wg_x:
                xmode, xt_ready = "buf", True
            elif not (full and xt_ready):
                xmode, xt_ready = "mb", False
        self._x_mode = xmode      # (diagnostics / tests only)
        self._first_step = False
        self._q8_step, self._q8_next = self._q8_next, self._q8_next + 1
        self._loss_dev = self.loss_sums
        return idx_t, first, xt_ready, xmode

    def can_fuse_apply(self, extra_grad: float = 0.0) -> bool:
        """the one-kernel path's grad(idx, apply=True): one gradient range, no clipping (the Adam
        step needs no global norm first), eager launches (the host knows the step number), and
        no all-reduce between the gradient and the update (the caller checks: world size 1)."""
        p = self.p
        clip = p.max_grad_norm is not None and p.max_grad_norm > 0
        return (self.fused_apply and not extra_grad and not clip
                and (self.heads or (len(self.buckets) == 1 and self.buckets[0]["partials"])))

    def step(self, idx: Optional[torch.Tensor], extra_grad: float = 0.0, allreduce=None,
             mean: bool = False, last: bool = False) -> None:
        """ONE synchronous global step (train.py:133-175 + chief.py:13-20): the minibatch
        gradient, its sum (``mean``: average) over ranks, and the Adam step.

        ``allreduce``: the worker's collective (parallel/dist.py grad_allreduce_fn), None at world
        size 1.  In-stream communicators (``allreduce.in_stream``: the native RCCL one — the
        default on an RCCL group — or the gloo adapter) reduce in stream order and do the mean
        themselves: joint kernels (one wgrad, one gather) → all-reduce → whole-vector Adam.
        With a side communicator, the value head's all-reduce + Adam go to a side stream instead:
        every epoch's under ``overlap_value_epochs`` (joined right before the next value kernel,
        so they overlap the policy Adam and the next policy kernel), and the iteration's last
        (``last``) under --overlap-rollout (overlapping the next rollout, which reads only the
        policy; joined in rollout()/values()).  Exact either way.

        Process-group collectives (``allreduce(t)`` returns an async work handle): per-head
        chains.  The policy range's all-reduce is issued as soon as it is gathered and runs while
        the value head's kernels compute; the value range's all-reduce runs while the policy Adam
        and the NEXT step's policy kernels compute — its Adam is applied just before the value
        kernel of the next step (or by finish_steps()).  Each head's Adam step e still precedes
        that head's kernel of step e+1, so the parameters are exactly the synchronous ones.
        Clipping (a global norm over both heads), the Q1 extra gradient and the one-kernel tile
        update take the whole-vector path."""
        p = self.p
        clip = p.max_grad_norm is not None and p.max_grad_norm > 0
        if allreduce is None and self.can_fuse_apply(extra_grad):
            self.grad(idx, apply=True)          # world size 1: gather + Adam in one launch
            return
        if getattr(allreduce, "in_stream", False):
            if self.heads:
                # (a value step of the previous epoch still on the side stream is joined inside,
                # right before the value kernel: it ran beside this epoch's policy kernel)
                self._joint_grad(*self._minibatch(idx))
            else:
                self._flush_value()
                self.grad(idx)
            if (self.heads and getattr(allreduce, "side", False) and not clip and not extra_grad
                    and (p.overlap_value_epochs or (last and p.overlap_rollout))):
                self._split_step_side(allreduce)
                return
            self._flush_value()
            allreduce(self.grad_flat)           # sum / mean in stream order: no host-side scaling
            self.apply(extra_grad)
            return
        if not self.heads:
            self.grad(idx)
            if allreduce is not None:
                self._reduce_wait(allreduce(self.grad_flat), self.grad_flat, mean)
            self.apply(extra_grad)
            return
        mbt = self._minibatch(idx)
        if clip or extra_grad:
            self._flush_value()
            self._heads_grad(*mbt)
            if allreduce is not None:
                self._reduce_wait(allreduce(self.grad_flat), self.grad_flat, mean)
            self.apply(extra_grad)
            return
        if allreduce is None:                   # (fused_apply=False: the two-launch chains, no collective)
            allreduce = lambda t: None          # noqa: E731
        step_no = self.adam_step + 1
        (plo, phi), (vlo, vhi) = self.head_range
        self._head_chain(0, *mbt)
        wp = allreduce(self.grad_flat[plo:phi])
        self._flush_value()
        self._head_chain(1, *mbt)
        self._pending_value = ("work", allreduce(self.grad_flat[vlo:vhi]), step_no, mean)
        self.pending_steps += 1
        self._reduce_wait(wp, self.grad_flat[plo:phi], mean)
        self._head_adam(0, step_no)
        self.adam_step += 1
        self._norm_n = self.norm_regions[1][1]

    def _split_step_side(self, allreduce) -> None:
        """the joint gradient is gathered: the value range's all-reduce (the side communicator) +
        Adam are forked to the side stream right away, then the policy range's all-reduce + Adam
        run in stream order (the two collectives on two communicators may run concurrently).  The
        next value kernel (_joint_heads), rollout() / values() / finish_steps() join it
        (_flush_value): it overlaps the policy Adam and the next epoch's policy kernel, or the next
        rollout after the last epoch."""
        (plo, phi), (vlo, vhi) = self.head_range
        step_no = self.adam_step + 1
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        side = self._side
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            allreduce(self.grad_flat[vlo:vhi], stream=side)
            self._head_adam(1, step_no)
        allreduce(self.grad_flat[plo:phi])
        self._head_adam(0, step_no)
        self._pending_value = ("side", None, step_no, False)
        self.side_steps += 1
        self.adam_step += 1
        self._norm_n = self.norm_regions[1][1]

    def finish_steps(self) -> None:
        """apply a value-head step still waiting for its all-reduce (end of the epochs)"""
        self._flush_value()

    def metrics_stream(self) -> Optional[torch.cuda.Stream]:
        """the stream the iteration's metrics are packed and staged on: the side stream while the
        last value step runs there (its Adam writes the value head's norm partials), else None"""
        pend = self._pending_value
        return self._side if (pend is not None and pend[0] == "side") else None

    def _flush_value(self) -> None:
        pend, self._pending_value = self._pending_value, None
        if pend is None:
            return
        kind, work, step_no, mean = pend
        if kind == "side":
            # everything enqueued on the side stream so far: the value step AND the metrics
            # pack / staging copy behind it (their buffers are rewritten after this point)
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            return
        vlo, vhi = self.head_range[1]
        self._reduce_wait(work, self.grad_flat[vlo:vhi], mean)
        self._head_adam(1, step_no)

    def _reduce_wait(self, work, t: torch.Tensor, mean: bool) -> None:
        if work is not None:
            work.wait()          # orders the compute stream after RCCL's (no host block on GPU)
        if mean:
            t.mul_(1.0 / torch.distributed.get_world_size())

    def _heads_grad(self, idx_t, first: bool, xt_ready: bool, xmode: str) -> None:
        for h in (0, 1):
            self._head_chain(h, idx_t, first, xt_ready, xmode)

    def _head_kernel(self, h: int, idx_t, first: bool, xt_ready: bool, part: torch.Tensor, part_dw: int) -> None:
        p, M = self.p, self.mb
        t32 = h == 0 and self.phead
        opts = [0 if p.loss == "ppo" else 1, 0 if p.value_loss == "mse" else 1,
                1 if p.std_convention == "var" else 0, 1 if first else 0, part.shape[1], h, part_dw,
                (1 if self.phead_p2 else 2) if t32 else 0]
        # (the 32x32 policy kernel: xt_ready as _minibatch resolved it — it writes X rows into xT
        # only for x-mode "mb", a minibatch)
        # fp8: the value head's fc1 on the e4m3 image; the policy's GEMMs only with fp8_policy_gemms
        w8 = self._w8() if (h == 1 or p.fp8_policy_gemms) else (self.no_u8, self.no_q)

        def launch(q8_step):
            self.ext.mlp_train(self.dt, self.x_buf, idx_t, 0, M, self.wimg, self.layout, self.scales,
                               self.model.flat.data, self.log_std_old, self.A, self.actions, self.logp, self.adv,
                               self.ret, self.values_buf, self.mu_prev, self.v_prev, opts,
                               [float(p.clip), float(p.ent_coeff)], self.tbufs, self.ldT, part, False, xt_ready,
                               *w8, self.q8_amax if self.q8 else self.empty, q8_step)
        if self.q8 and not self._q8_cal[h]:
            # the first step of this engine: one pass as step -1 only to record the gradient maxima
            # the step-0 scales come from (its stores and partials are overwritten by the real one;
            # the reference loss's mu_prev / v_prev writes are idempotent)
            launch(-1)
            self._q8_cal[h] = True
        launch(self._q8_step)
        if h == 0 and idx_t is self.empty and not self.phead:
            self._xT_valid = True   # the policy kernel wrote x^T of this buffer (full batch)
        if h == 0 and p.loss == "dppo_ref":
            self.log_std_old.copy_(self.model.flat.data[:self.A])   # train.py:164, before Adam moves it

    def _joint_heads(self, idx_t, first: bool, xt_ready: bool, xmode: str) -> None:
        """both head kernels into the shared partial buffer (disjoint columns and operands), in
        stream order.  (Measured: the policy kernel on a side stream concurrent with the value
        kernel, joined before the wgrad: 4.57 vs 4.39 ms per iteration, same box — each kernel
        fills a CU's LDS, so they only time-slice the CUs and the stream hand-offs are extra.)"""
        for h in self.head_order:
            if h == 1:
                self._flush_value()   # the previous step's value Adam (side stream) lands first
            self._head_kernel(h, idx_t, first, xt_ready, self.part_joint, self.part_dw_joint[h])

    def _joint_grad(self, idx_t, first: bool, xt_ready: bool, xmode: str) -> None:
        """both head kernels (one shared partial buffer), ONE wgrad over both heads' layers, ONE
        gather of the whole gradient into grad_flat (no optimizer step)"""
        self._joint_heads(idx_t, first, xt_ready, xmode)
        b = self.joint_bucket
        self._wgrad(b, xmode)
        src_off, src_meta = self.joint_src
        rc, rd = self.items["joint"]
        self.ext.grad_gather(b["slab"], src_off, src_meta, self.part_joint, self.nhead_blk, self.part_joint.shape[1],
                             rc, rd, 1.0 / self.mb, self.grad_flat, self.loss_sums, b["runs"])

    def _joint_step(self, idx_t, first: bool, xt_ready: bool, xmode: str) -> None:
        """world size 1: policy kernel, value kernel (one shared partial buffer), ONE wgrad over
        both heads' layers, ONE gather + Adam launch over the whole flat vector"""
        p, M = self.p, self.mb
        self._joint_heads(idx_t, first, xt_ready, xmode)
        b = self.joint_bucket
        self._wgrad(b, xmode)
        b1, b2 = p.adam_betas
        src_off, src_meta = self.joint_src
        rc, rd = self.items["joint"]
        self.ext.gather_adam(b["slab"], src_off, src_meta, self.part_joint, self.nhead_blk, self.part_joint.shape[1],
                             rc, rd, b["runs"], 1.0 / M, self.loss_sums, self.grad_flat, self.model.flat.data,
                             self.adam_m, self.adam_v, float(p.lr), float(b1), float(b2), float(p.adam_eps),
                             self.adam_step + 1, self.adam_state, self.norm_part[:self.norm_n_whole], self.wimg,
                             self.w_map, self.wt_map, self.dt, self.no_q, *self._f8())
        self.adam_step += 1
        self._norm_n = self.norm_n_whole

    def _head_chain(self, h: int, idx_t, first: bool, xt_ready: bool, xmode: str) -> None:
        """head h's kernel -> its wgrad -> its gather into its flat range of grad_flat"""
        M = self.mb
        self._head_kernel(h, idx_t, first, xt_ready, self.part_h[h], self.part_dw[h])
        b = self.buckets[h]
        self._wgrad(b, xmode)
        lo, hi = self.head_range[h]
        part = self.part_h[h]
        rc, rd = self.items["policy" if h == 0 else "value"]
        self.ext.grad_gather(b["slab"], self.src_off[lo:hi], self.src_meta[lo:hi], part, self.nhead_blk,
                             part.shape[1], rc, rd, 1.0 / M, self.grad_flat[lo:hi], self.loss_sums,
                             [r - lo for r in b["runs"]])

    def _head_adam(self, h: int, step_no: int) -> None:
        """no-clip Adam over head h's flat range (after its all-reduce); its norm region"""
        p = self.p
        lo, hi = self.head_range[h]
        r0, r1 = self.norm_regions[h]
        b1, b2 = p.adam_betas
        self.ext.adam(self.model.flat.data[lo:hi], self.grad_flat[lo:hi], self.adam_m[lo:hi], self.adam_v[lo:hi],
                      float(p.lr), float(b1), float(b2), float(p.adam_eps), 0.0, self.adam_state,
                      self.norm_part[r0:r1], self.wimg, self.w_map[lo:hi], self.wt_map[lo:hi], self.dt, self.no_q,
                      step_no, *self._f8(lo, hi))

    def grad(self, idx: Optional[torch.Tensor], apply: bool = False) -> None:
        """one minibatch gradient into grad_flat (no optimizer step; tests / the whole-vector
        path).  ``apply=True`` (one-kernel path, only when can_fuse_apply()): the gather and the
        Adam step run as ONE launch — the same update as grad() then apply()."""
        if self.heads:
            self._flush_value()
            mbt = self._minibatch(idx)
            if apply:
                assert self.can_fuse_apply(), "fused gather + Adam is not available here"
                self._joint_step(*mbt)
            else:
                self._heads_grad(*mbt)
            return None
        idx_t, first, xt_ready, xmode = self._minibatch(idx)
        if apply:
            assert self.can_fuse_apply(), "fused gather + Adam is not available here"
            self._launch_grad(idx_t, first, xt_ready, fused_apply=True)
            self.adam_step += 1
            self._norm_n = self.norm_n_whole
        else:
            self._launch_grad(idx_t, first, xt_ready)
        return None

    def _launch_grad(self, idx_t: torch.Tensor, first: bool, xt_ready: bool, fused_apply: bool = False) -> None:
        p, M = self.p, self.mb
        opts = [0 if p.loss == "ppo" else 1, 0 if p.value_loss == "mse" else 1,
                1 if p.std_convention == "var" else 0, 1 if first else 0, self.npart]
        fopts = [float(p.clip), float(p.ent_coeff)]
        self.ext.mlp_train(self.dt, self.x_buf, idx_t, 0, M, self.wimg, self.layout, self.scales,
                           self.model.flat.data, self.log_std_old, self.A, self.actions, self.logp, self.adv,
                           self.ret, self.values_buf, self.mu_prev, self.v_prev, opts, fopts, self.tbufs,
                           self.ldT, self.part, False, xt_ready, self.no_u8, self.no_q, self.empty, 0)
        b = self.buckets[0]
        self._wgrad(b, "fm")
        if fused_apply:
            if p.loss == "dppo_ref":   # train.py:164: the pre-update log_std, before Adam moves it
                self.log_std_old.copy_(self.model.flat.data[:self.A])
            b1, b2 = p.adam_betas
            rc, rd = self.items["legacy"]
            self.ext.gather_adam(b["slab"], self.src_off, self.src_meta, self.part, self.ntrain_blk,
                                 self.npart, rc, rd, b["runs"], 1.0 / M, self.loss_sums, self.grad_flat,
                                 self.model.flat.data, self.adam_m, self.adam_v, float(p.lr), float(b1),
                                 float(b2), float(p.adam_eps), self.adam_step + 1, self.adam_state,
                                 self.norm_part[:self.norm_n_whole], self.wimg, self.w_map, self.wt_map, self.dt,
                                 self.no_q, *self._f8())
            return
        rc, rd = self.items["legacy"]
        self.ext.grad_gather(b["slab"], self.src_off, self.src_meta, self.part, self.ntrain_blk, self.npart,
                             rc, rd, 1.0 / M, self.grad_flat, self.loss_sums, b["runs"])
        if p.loss == "dppo_ref":
            self.log_std_old.copy_(self.model.flat.data[:self.A])  # train.py:164

    @torch.no_grad()
    def apply(self, extra_grad: float = 0.0) -> None:
        """whole-vector Adam (+ clip) after grad() [+ the all-reduce]"""
        p = self.p
        self._flush_value()
        if extra_grad:
            self.grad_flat.add_(extra_grad)
        mx = float(p.max_grad_norm) if (p.max_grad_norm is not None and p.max_grad_norm > 0) else 0.0
        b1, b2 = p.adam_betas
        # the host knows the step number: one fused kernel without clipping
        self.ext.adam(self.model.flat.data, self.grad_flat, self.adam_m, self.adam_v, float(p.lr), float(b1),
                      float(b2), float(p.adam_eps), mx, self.adam_state, self.norm_part[:self.norm_n_whole], self.wimg,
                      self.w_map, self.wt_map, self.dt, self.no_q, self.adam_step + 1, *self._f8())
        self.adam_step += 1
        self._norm_n = self.norm_n_whole
        return None

    def pack_metrics(self, ep2: torch.Tensor) -> Optional[torch.Tensor]:
        """device f64[11] = [episode return sum, count | loss sums (8) | grad norm], written by ONE
        launch (csrc/optim.hip metrics_pack, 256 threads over the Adam partials) instead of ~6
        small torch ops per iteration; the buffer is reused (stream order keeps the previous D2H
        copy ahead of the next pack)."""
        if self._loss_dev is None:
            return None
        # every Adam path (fused no-clip, sumsq + clip, per head) leaves the per-block
        # sums of squares of the gradient it applied in norm_part[:_norm_n].  A value step left
        # pending on the process-group chains has not written its region yet: the norm is the
        # policy head's for that step.  One on the side stream: the pack runs there, after it.
        pend = self._pending_value
        n = self.norm_regions[0][1] if (pend is not None and pend[0] == "work") else self._norm_n
        side = self.metrics_stream()
        if side is not None:
            # everything the pack reads that the compute stream wrote after the value step was
            # forked (the side-stream obs-stat merge's episode sums are joined there at the end)
            side.wait_stream(torch.cuda.current_stream(self.device))
        with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
            self.ext.metrics_pack(ep2, self._loss_dev, self.norm_part[:n], self.metrics_buf)
        return self.metrics_buf

    def loss_vector(self) -> Optional[torch.Tensor]:
        """device [loss sums of the last minibatch (8) | grad norm of the last Adam step] — staged
        into host memory by the worker without a sync (``losses_from_vector`` decodes it)."""
        if self._loss_dev is None:
            return None
        if self.p.max_grad_norm is not None and self.p.max_grad_norm > 0:
            gn = self.adam_state[2:3]              # the clip pass computed it
        else:                                      # no-clip Adam skips the norm: last step's gradient
            gn = torch.linalg.vector_norm(self.grad_flat).reshape(1)
        return torch.cat([self._loss_dev.reshape(-1), gn])

    @staticmethod
    def losses_from_vector(v) -> Dict[str, float]:
        n = max(v[5], 1.0)
        out = {"loss_clip": v[0] / n, "loss_value": v[1] / n, "loss_ent": v[2] / n,
               "approx_kl": v[3] / n, "clipfrac": v[4] / n}
        out["loss"] = out["loss_clip"] + out["loss_value"] + out["loss_ent"]
        out["grad_norm"] = float(v[NPART_FIXED])
        return out

    def last_losses(self) -> Dict[str, float]:
        vec = self.loss_vector()
        return {} if vec is None else self.losses_from_vector(vec.tolist())

    def sync(self) -> None:
        torch.cuda.synchronize(self.device)
