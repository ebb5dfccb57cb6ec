// Weight-gradient GEMM for all six layers in ONE launch (grouped, split-K over the batch).
//
//   dW_aug[n][k] = sum_m dY[m][n] * X[m][k]      (k == K is the bias column: X^T row K == 1)
//
// Both operands are feature-major (written transposed by mlp_train_kernel), so every MFMA
// fragment is one 16-byte load along m, the reduction axis.  A task = (layer, output tile,
// batch chunk).  The tile is nq x kq QUADRANTS of 64x64 (nq * kq <= 8, nq + kq <= 6), one per
// wave of the 8-wave workgroup, or at split-bf16 / bf16 up to 16 quadrants, two per wave
// (wgrad_task_ok); each quadrant = 4x4 MFMA tiles of 16x16 (64 f32 accumulator registers).  The host plan picks (nq, kq) per layer to minimise operand rows read per
// k-step: the kernel is bound by the operand stream (HBM / MALL), and a 256x128 tile reads
// 384 rows per step for 2x the outputs of a 128x128 tile's 256 (v_fc1: 2304 instead of 3072
// rows per step).  Results go to per-chunk fp32 slabs ([nq*64][kq*64] per task) that
// grad_gather sums in a fixed order — deterministic, no float atomics (SURVEY §7.4 part 2).
#include "kernels.h"
#include "mlp_core.h"

namespace {

constexpr int WG_WAVES = 8;

// The workgroup stages each k-step's distinct fragments (4*nq of dY^T, 4*kq of X^T) ONCE into
// LDS with LDS-DMA (global_load_lds_dwordx4): an FM fragment is 64 lanes x 16 B per KiB in lane
// order, exactly the lane-linear image the DMA writes, so the fragment reads are conflict-free
// ds_read_b128 at lane*16.  A split-bf16 fragment (32 B per lane: hi | lo) is two DMA
// instructions, instruction h moving the fragment's h-th KiB (lanes 32h .. 32h+31) so it lands
// as [their hi][their lo] (the dense layout of mlp_stream.hip frag_lane_off).  Each wave DMAs C
// fixed slots per stage (C = 2 when the task has <= 16 fragments, 3 <= 24, 4 <= 32, 5 <= 40; slots past the task's
// fragment count re-load one of its fragments, an L2 hit, so every wave's DMA count — and with
// it the vmcnt arithmetic — is task-independent).  S-deep ring, counted vmcnt and a raw
// s_barrier keep S-1 steps of DMA in flight across the barrier (cdna_hip_programming.md
// 'Pipelining across barriers'): no VGPRs hold in-flight data.
// bytes per operand slot: one fragment (32 batch rows of 16 features); e4m3 (DT_FP8) four
// fragments of consecutive k-steps (128 batch rows, 2 KiB: two DMA instructions; they are
// contiguous in the FM layout), one v_mfma_scale_f32_16x16x128_f8f6f4 per tile pair — twice the
// bf16 MFMA rate — so a kernel "k-step" there covers 128 rows
template <int DT>
constexpr int wgrad_frag_bytes() { return DT == DT_FP8 ? 2048 : 512 * Prec<DT>::BYTES; }
template <int DT>
constexpr int wgrad_step_rows() { return DT == DT_FP8 ? 128 : 32; }
typedef __attribute__((ext_vector_type(8))) int i32x8;

// the 16-byte chunk swizzle of a row-major operand image (128-byte rows): even XOR values keep the two
// chunks of a 16-feature column group adjacent; rows r, r + 2, r + 8, r + 10 (the rows of a 32-lane
// half's transposed reads that share banks) get distinct chunk pairs — conflict-free
__host__ __device__ inline int wgrad_swz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

// Row-major operands: lane l's MFMA operand (feature 16 s + (l & 15) of a quadrant, rows 8 (l >> 4)
// .. + 7) is two ds_read_b64_tr_b16 of 4 rows each (lane 4 q' + p' of a 16-lane group addresses row
// q', columns 4 p' .. 4 p' + 3; lane i receives column i) per precision part.  rm_off: the byte
// offset (within a stage) of read `sub` of slot f (quadrant slots f & ~3 .. + 3, s = f & 3)
DEV unsigned rm_off(int f, int sub, int lane, int FB) {
  const int li = lane & 15, g = lane >> 4;
  const int row = 8 * g + 4 * sub + (li >> 2), col = 16 * (f & 3) + 4 * (li & 3);
  return (unsigned)((f & ~3) * FB + row * 128 + (((col >> 3) ^ wgrad_swz(row)) << 4) + (col & 7) * 2);
}
// Split-bf16 row-major quadrants keep the memory's [8 hi | 8 lo] groups: a row's 64 features are 256
// contiguous bytes, DMA'd 4 rows per instruction (16 lanes x 16 B per row: whole 256-byte row
// segments, not 16-byte pieces at a 32-byte stride), the 16 chunks of a row XOR-swizzled by
// wgrad_swz16(row) so the 16 rows of a transposed read meet each 16-byte bank group at most twice
// (the 2-cycle minimum of a 512-byte read)
__host__ __device__ inline int wgrad_swz16(int row) { return ((row & 3) << 2) | ((row >> 3) & 3); }
DEV unsigned rm_off_s3(int f, int sub, int part, int lane, int FB) {
  const int li = lane & 15, g = lane >> 4;
  const int row = 8 * g + 4 * sub + (li >> 2), col = 16 * (f & 3) + 4 * (li & 3);
  const int pos = ((col >> 3) * 2 + part) ^ wgrad_swz16(row);
  return (unsigned)((f & ~3) * FB + row * 256 + pos * 16 + (col & 7) * 2);
}
// the operand from its precomputed read offsets (split: hi reads o[0], o[1], lo reads o[2], o[3])
template <int DT>
DEV typename Prec<DT>::Frag rm_frag_at(const char* st, const unsigned (&o)[4]) {
  typedef __attribute__((ext_vector_type(4))) short s16x4;
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  auto rd = [&](unsigned off) __attribute__((always_inline)) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(st + off));
  };
  auto cat = [&](s16x4 a0, s16x4 a1) __attribute__((always_inline)) {
    const s16x8 v{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    return *reinterpret_cast<const bf16x8*>(&v);
  };
  if constexpr (IsSplit<DT>::value) {
    return S3Frag{cat(rd(o[0]), rd(o[1])), cat(rd(o[2]), rd(o[3]))};
  } else {
    return cat(rd(o[0]), rd(o[1]));
  }
}

// Tasks of up to 8 quadrants run one quadrant per wave (QW 1: 24 fragment slots per stage); split-bf16
// and bf16 tasks of 9-16 quadrants (nq even) run TWO per wave (QW 2: 40 slots, nq + kq <= 10), the
// wave's quadrants (wn, wk) and (wn + nq / 2, wk) sharing its X fragments — a wider tile streams fewer
// operand rows per output (Humanoid v_fc1 as four 4x3 quadrant tiles: 28 x 64 rows per k-step
// instead of 36 x 64 with six 4x2 tiles) and a wave reads 12 fragments per 32 MFMA tiles instead of
// 8 per 16.  The ring depth follows the stage size: split-bf16 3 stages of 24 slots or 2 of 40 (one
// stage in flight: a 4x3 tile's 3-stage ring would need 168 KiB; the wait share grows, 0.46 -> 0.52
// of the wave cycles, docs/ARCHITECTURE.md §13), bf16 4 of either.
template <int DT, int QW>
struct WgCfg {
  static constexpr int SLOTS = QW == 1 ? 24 : 40;
  static constexpr int S = DT == DT_BF16 ? 4 : (QW == 1 ? 3 : 2);
};
template <int DT, bool WIDE>
constexpr size_t wgrad_lds_bytes() {
  constexpr size_t one = (size_t)WgCfg<DT, 1>::S * WgCfg<DT, 1>::SLOTS * wgrad_frag_bytes<DT>();
  constexpr size_t two = (size_t)WgCfg<DT, 2>::S * WgCfg<DT, 2>::SLOTS * wgrad_frag_bytes<DT>();
  return WIDE && two > one ? two : one;
}
static_assert(wgrad_lds_bytes<DT_S3, true>() <= 160 * 1024 && wgrad_lds_bytes<DT_BF16, true>() <= 160 * 1024, "wgrad LDS");

template <int DT, int QW, int C>
DEV void wgrad_lds_body(const WgradArgs& a, const WgradTask& tk, char* smem) {
  using P = Prec<DT>;
  using T = typename P::T;
  using Frag = typename P::Frag;
  constexpr int FB = wgrad_frag_bytes<DT>();     // bytes per fragment
  constexpr int NI = FB / 1024;                  // DMA instructions per fragment (64 lanes x 16 B)
  constexpr int S = WgCfg<DT, QW>::S;
  constexpr int SB = WgCfg<DT, QW>::SLOTS * FB;  // bytes per stage
  static_assert(QW == 1 || DT == DT_S3 || DT == DT_BF16, "two quadrants per wave: split-bf16 / bf16");
  static_assert(C * WG_WAVES <= WgCfg<DT, QW>::SLOTS, "slots");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const char* g = reinterpret_cast<const char*>(a.gT[tk.layer]);
  const char* x = reinterpret_cast<const char*>(a.xT[tk.layer]);
  const int nk = (tk.m1 - tk.m0) / wgrad_step_rows<DT>();
  const int ks0 = tk.m0 >> 5;
  const int NF = 4 * tk.nq, F = NF + 4 * tk.kq;
  // slot f of a stage holds fragment f: f < NF -> dY^T row tile n0/16 + f, else X^T row tile
  // k0/16 + f - NF.  Wave w DMAs slots C*w .. C*w + C-1 (a slot >= F re-loads fragment f mod F).
  // FM operands: a fragment is contiguous (FB bytes per k-step).  Row-major operands (the 32x32
  // policy head's g1p / g2p / h1p and the observation rows, csrc/phead.hip; row length a.g_rm /
  // a.x_rm): a quadrant's 4 slots hold its [32 rows][64 features] image per k-step — bf16: 128-byte
  // rows, the 16-byte chunks XOR-swizzled by wgrad_swz(row), 8 rows per DMA instruction;
  // split-bf16: the memory's 256-byte [8 hi | 8 lo] rows, wgrad_swz16, 4 rows per instruction —
  // read back transposed (ds_read_b64_tr_b16).
  const char* srcp[C][NI];
  size_t kstride[C];
  int dst[C];
#pragma unroll
  for (int q = 0; q < C; ++q) {
    const int f = wave * C + q;
    const int ff = f < F ? f : f % F;   // dummy slot: re-load one of the task's fragments
    const bool gs = ff < NF;
    const int fl = gs ? ff : ff - NF;
    const int feat0 = (gs ? tk.n0 : tk.k0) + 16 * fl;
    // rm: 0 fragment-major; > 0 row-major rows of rm elements
    const int rm = (DT == DT_S3 || DT == DT_BF16) ? (gs ? a.g_rm[tk.layer] : a.x_rm[tk.layer]) : 0;
    const char* ob = gs ? g : x;
    if (rm == 0) {
      const char* src = ob + fm_frag(feat0 >> 4, ks0, a.ld, 0) * sizeof(T);
#pragma unroll
      for (int hh = 0; hh < NI; ++hh)
        srcp[q][hh] = src + (IsSplit<DT>::value ? (size_t)hh * 1024 + (lane & 31) * 32 + (lane >> 5) * 16
                                                 : (size_t)hh * 1024 + lane * 16);
      kstride[q] = FB;
    } else {
      const int sq = fl & 3, f0 = feat0 - 16 * sq;   // slot in the quadrant, the quadrant's first feature
#pragma unroll
      for (int hh = 0; hh < NI; ++hh) {
        const int n = NI * sq + hh;                   // 1 KiB DMA instruction of the quadrant image
        if constexpr (IsSplit<DT>::value) {           // rows 4 n .. 4 n + 3, 256 bytes each
          const int row = 4 * n + (lane >> 4);
          const int c = (lane & 15) ^ wgrad_swz16(row);
          srcp[q][hh] = ob + ((size_t)(tk.m0 + row) * rm + f0) * sizeof(T) + 16 * c;
        } else {                                      // rows 8 n .. 8 n + 7, 128 bytes each
          const int row = 8 * n + (lane >> 3);
          const int c = (lane & 7) ^ wgrad_swz(row);
          srcp[q][hh] = ob + ((size_t)(tk.m0 + row) * rm + f0 + 8 * c) * sizeof(T);
        }
      }
      kstride[q] = (size_t)32 * rm * sizeof(T);
    }
    dst[q] = f * FB;
  }
  auto issue = [&](int k) {
    const int kk = min(k, nk - 1);            // past the end: re-load valid data (count stays fixed)
    char* st = smem + (k % S) * SB;
#pragma unroll
    for (int q = 0; q < C; ++q)
#pragma unroll
      for (int h = 0; h < NI; ++h) glds16(srcp[q][h] + (size_t)kk * kstride[q], st + dst[q] + h * 1024);
  };
  // Q8: this lane's sub-slot maximum of the layer's gradient tensor, loaded before any DMA (the
  // oldest vector-memory op: it never holds up a counted wait), folded in the epilogue
  uint32_t q8v = 0;
  if constexpr (DT == DT_FP8) q8v = a.q8_rd[(a.q8_t[tk.layer] * Q8_SUB + lane) * Q8_LINE];
  // QW 2: waves (wn, wk) for wn < nq / 2, quadrant rows wn and wn + nq / 2
  const int nqw = QW == 1 ? tk.nq : tk.nq >> 1;
  const bool active = wave < nqw * tk.kq;
  constexpr bool RMOK = DT == DT_S3 || DT == DT_BF16;   // (fp32 / e4m3 operands are fragment-major only)
  const bool g_rm = RMOK && a.g_rm[tk.layer] != 0, x_rm = RMOK && a.x_rm[tk.layer] != 0;
  const int wn = wave / tk.kq, wk = wave - (wave / tk.kq) * tk.kq;
  // per-lane byte offsets within a quadrant's 4 slots: fragment-major, the lane's 16 bytes of slot i
  // at fmo + i * FB; row-major, the two 4-row transposed reads (rm_off) of slot i (split: hi, lo) —
  // the same pattern for every quadrant and side (a quadrant adds its uniform slot base)
  const unsigned fmo = IsSplit<DT>::value ? (unsigned)((lane >> 5) * 1024 + (lane & 31) * 16)
                                          : (unsigned)(lane * 8 * (int)sizeof(T));
  unsigned pat[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pat[i][0] = pat[i][1] = pat[i][2] = pat[i][3] = 0;
    if constexpr (IsSplit<DT>::value) {
      for (int j = 0; j < 4; ++j) pat[i][j] = rm_off_s3(i, j & 1, j >> 1, lane, FB);
    } else if constexpr (RMOK) {
      pat[i][0] = rm_off(i, 0, lane, FB);
      pat[i][1] = rm_off(i, 1, lane, FB);
    }
  }
  // slot i of the quadrant whose first slot is `slot` in stage st
  auto frag = [&](const char* st, int slot, bool rm, int i) __attribute__((always_inline)) -> Frag {
    const char* qb = st + slot * FB;
    if constexpr (RMOK)
      if (rm) return rm_frag_at<DT>(qb, pat[i]);
    const char* b = qb + fmo + i * FB;
    if constexpr (IsSplit<DT>::value) {
      return Frag{*reinterpret_cast<const bf16x8*>(b), *reinterpret_cast<const bf16x8*>(b + 512)};
    } else {
      return P::load(reinterpret_cast<const T*>(b));
    }
  };
  f32x4 acc[QW][4][4];
#pragma unroll
  for (int u = 0; u < QW; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[u][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  for (int k = 0; k < nk; ++k) {
    WAIT_VMCNT(C * NI * (S - 2));             // this wave's part of stage k has landed
    __builtin_amdgcn_s_barrier();              // ... everyone's; and stage k-1 is no longer read
    // refill the slot stage k-1 used: split-bf16 / bf16 after this step's fragment reads (the DMA
    // issue cost then overlaps their latency: 4.16 vs 4.22 ms per bf16x3 iteration, 2.30 vs 2.32
    // bf16, same box); e4m3 right here (2.01 vs 1.99 the other way; profiles/r4/ab_late_issue_*.json)
    constexpr bool LATE = DT != DT_FP8;
    if (!LATE || !active) issue(k + S - 1);
    if (active) {
      const char* st = smem + (k % S) * SB;
      if constexpr (DT == DT_FP8) {
        // four e4m3 k-steps per slot: lane l's 8 bytes of k-step 4kk + j at j * 512 + l * 8.  The
        // 16x16x128 operand of lane l is those 32 bytes in j order — rows {32 j + 8 (l >> 4) + e}
        // for BOTH operands, so the MFMA's k sum runs over every row of the 128 exactly once
        // (E8M0 scales 127 = 1: the power-of-two operand scales are undone in the epilogue)
        auto rd = [&](int f) {
          const char* p = st + f * FB + lane * 8;
          const long x0 = *reinterpret_cast<const long*>(p), x1 = *reinterpret_cast<const long*>(p + 512);
          const long x2 = *reinterpret_cast<const long*>(p + 1024), x3 = *reinterpret_cast<const long*>(p + 1536);
          return i32x8{(int)x0, (int)(x0 >> 32), (int)x1, (int)(x1 >> 32), (int)x2, (int)(x2 >> 32), (int)x3,
                       (int)(x3 >> 32)};
        };
        i32x8 a8[4], b8[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a8[i] = rd(wn * 4 + i);
          b8[i] = rd(NF + wk * 4 + i);
        }

#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[0][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8[i], b8[j], acc[0][i][j], 0, 0, 0, 127, 0, 127);
        continue;
      }
      Frag af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = frag(st, 4 * wn, g_rm, i);
        bf[i] = frag(st, NF + 4 * wk, x_rm, i);
      }
      if constexpr (LATE) issue(k + S - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[0][i][j] = P::mma(acc[0][i][j], af[i], bf[j]);
      if constexpr (QW == 2) {
        // the second quadrant's dY fragments (its X fragments are the first's)
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag(st, 4 * (wn + nqw), g_rm, i);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[QW - 1][i][j] = P::mma(acc[QW - 1][i][j], af[i], bf[j]);
      }
    }
  }
  WAIT_VMCNT(0);                               // no DMA may outlive the workgroup's LDS
  if (!active) return;
  const int KE = tk.kq * 64;
  float* out = a.slab + tk.slab;
  if constexpr (DT == DT_FP8) {   // undo the operands' scales (powers of two: exact)
    const float inv = q8_pow2(-q8_exp(wave_umax(q8v))) / a.q8_xs[tk.layer];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[0][i][j] *= inv;
  }
  const int col = wk * 64 + (lane & 15);
#pragma unroll
  for (int u = 0; u < QW; ++u) {
    const int rbase = (wn + u * nqw) * 64 + (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) out[(rbase + 16 * i + q) * KE + col + 16 * j] = acc[u][i][j][q];
  }
}

// WIDE: the launch holds two-quadrant-per-wave tasks (wgrad_task_ok), the LDS of either ring
template <int DT, bool WIDE>
__global__ __launch_bounds__(WG_WAVES * 64) void wgrad_kernel(WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];   // the kernel's ONLY LDS object
  const WgradTask tk = a.tasks[blockIdx.x];
  const int F = 4 * (tk.nq + tk.kq);
  if constexpr (WIDE) {
    if (tk.nq * tk.kq > WG_WAVES) {
      if (F <= 4 * WG_WAVES) wgrad_lds_body<DT, 2, 4>(a, tk, smem);
      else wgrad_lds_body<DT, 2, 5>(a, tk, smem);
      return;
    }
  }
  if (F <= 2 * WG_WAVES) wgrad_lds_body<DT, 1, 2>(a, tk, smem);
  else wgrad_lds_body<DT, 1, 3>(a, tk, smem);
}

template <int DT, bool WIDE>
void launch_wgrad_lds(const WgradArgs& a, hipStream_t s) {
  const size_t lds = wgrad_lds_bytes<DT, WIDE>();
  set_max_lds_once<wgrad_kernel<DT, WIDE>>(lds);
  hipLaunchKernelGGL((wgrad_kernel<DT, WIDE>), dim3(a.ntasks), dim3(WG_WAVES * 64), lds, s, a);
}

// Blocks [0, item_blocks(nitems)): the reduce items (log_std, loss-term sums, the per-head
// kernels' fused narrow-layer weight gradients): column sums of the per-workgroup partial rows in
// a fixed order (item_reduce), grad[d] = scale * sum or loss_out[q] (red_dst).
// Blocks past them: grad[i] = scale * sum_{c < nch} slab[src_off[i] + c * stride] for the slab
// elements i of `runs` (src_meta[i] = nch * 32 + stride / 4096, each tile has its own batch-chunk
// count).  Fixed chunk order: deterministic; no float atomics anywhere.
__global__ __launch_bounds__(256) void grad_gather_kernel(const float* __restrict__ slab,
                                                          const int* __restrict__ src_off,
                                                          const int* __restrict__ src_meta,
                                                          const float* __restrict__ part,
                                                          int nblk, int npart, const int* __restrict__ red_col,
                                                          const int* __restrict__ red_dst, int nitems,
                                                          float scale, float* __restrict__ grad, SlabRuns runs,
                                                          float* __restrict__ loss_out) {
  const int nrb = item_blocks(nitems);
  if ((int)blockIdx.x < nrb) {
    __shared__ float red[256];
    float tot = 0.f;
    int j;
    if (item_reduce(part, nblk, npart, red_col, nitems, blockIdx.x, red, tot, j)) {
      const int d = red_dst[j];
      if (d >= 0) grad[d] = tot * scale;
      else loss_out[-1 - d] = tot;
    }
    return;
  }
  const int nb = gridDim.x - nrb;
  for (int j = (blockIdx.x - nrb) * 256 + threadIdx.x; j < runs.total; j += nb * 256) {
    const int i = runs.flat(j);
    const int mt = src_meta[i];
    const int o = src_off[i];
    const int nch = mt >> 5;
    const size_t st = (size_t)(mt & 31) << 12;
    const float s = slab_sum(slab + o, nch, st);
    grad[i] = s * scale;
  }
}

}  // namespace

// a task's quadrant tile: one quadrant per wave (nq * kq <= 8, nq + kq <= 6: 24 slots), or at
// split-bf16 / bf16 two per wave (9-16 quadrants, nq even, nq + kq <= 10: 40 slots)
extern "C" int wgrad_task_ok(int dt, int nq, int kq) {
  if (nq < 1 || kq < 1) return 0;
  if (nq * kq <= WG_WAVES) return nq + kq <= 6;
  return (dt == DT_S3 || dt == DT_BF16) && nq * kq <= 2 * WG_WAVES && nq % 2 == 0 && nq + kq <= 10;
}

extern "C" void launch_wgrad(int dt, const WgradArgs& a, hipStream_t s) {
  if (a.ntasks <= 0) return;
  if (dt == DT_F32) launch_wgrad_lds<DT_F32, false>(a, s);
  else if (dt == DT_FP8) launch_wgrad_lds<DT_FP8, false>(a, s);
  else if (dt == DT_S3) {
    if (a.wide) launch_wgrad_lds<DT_S3, true>(a, s);
    else launch_wgrad_lds<DT_S3, false>(a, s);
  } else {
    if (a.wide) launch_wgrad_lds<DT_BF16, true>(a, s);
    else launch_wgrad_lds<DT_BF16, false>(a, s);
  }
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_grad_gather(const float* slab, const int* src_off, const int* src_meta, const float* part,
                                   int nblk, int npart, const int* red_col, const int* red_dst, int nitems,
                                   float scale, float* grad, const SlabRuns& runs, float* loss_out, hipStream_t s) {
  int grid = (runs.total + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  grid += item_blocks(nitems);
  hipLaunchKernelGGL(grad_gather_kernel, dim3(grid), dim3(256), 0, s, slab, src_off, src_meta, part, nblk, npart,
                     red_col, red_dst, nitems, scale, grad, runs, loss_out);
  HIP_CHECK_LAUNCH();
}
