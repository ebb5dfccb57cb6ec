// Dense-layer building block shared by the rollout kernel and the fused update kernel.
//
//   out[r][c] = EPI( sum_k A[r][k] * B[c][k] )     r < ROWS, c < n_real, k < kdim (mult. of 32)
//
// A is a row tile in LDS (activations, or upstream gradients for dgrad), B is a row-major
// weight image in global memory (L2-resident; Wp [d_out][d_in] for forward, Wpt [d_in][d_out]
// for dgrad).  The bias is column K of Wp and the activation tiles carry a constant 1 in
// column K, so no separate bias add exists anywhere (PackedLayout in models/actor_critic.py).
//
// Work split: the NW waves of the workgroup stride over PAIRS of 16-wide output column tiles;
// each wave computes ALL ROWS/16 row blocks of its tiles, so one 16-byte B fragment (weights,
// the operand that streams from L2) feeds ROWS/16 MFMAs.  B fragments are register
// double-buffered in chunks of KC k-steps: while the MFMAs of chunk j run, the 2*KC loads of
// chunk j+1 are in flight (PMC showed the 1-step prefetch left waves parked on L2 latency
// ~60% of their cycles).
//
// Optional transposed store: with outT != nullptr the epilogue ALSO writes the value to the
// feature-major buffer outT[c][m0 + r] that feeds the wgrad GEMM.  In the MFMA C/D layout a
// lane holds 4 consecutive rows of one column, i.e. 4 contiguous m of one feature: one
// 4-element store per lane per row block, straight from registers (no LDS gather).
#pragma once
#include "common.h"

// EPI_DTANH_GLOBAL: like EPI_DTANH_INPLACE but the result is only needed as the wgrad
// operand, so it goes to outT alone (no LDS write-back) — used for the last dgrad layers.
enum { EPI_TANH = 0, EPI_LINEAR_F32 = 1, EPI_DTANH_INPLACE = 2, EPI_LINEAR_T = 3, EPI_DTANH_GLOBAL = 4 };

// tanh for the MFMA epilogues: exp + reciprocal on the transcendental unit (v_exp_f32,
// v_rcp_f32) instead of the libm polynomial; |err| ~1e-7.  The fp32 path keeps tanhf (it is
// the near-exact path the numerics tests compare against the torch oracle).
template <int DT>
DEV float act_tanh(float x) {
  if constexpr (DT == DT_F32) {
    return tanhf(x);
  } else {
    // tanh x = 1 - 2 / (1 + 2^(2 log2(e) x)): v_mul, v_exp, v_add, v_rcp, v_fma — 5 VALU, no
    // abs / sign fix-up (the previous form took 8: the compiler does not fold -2 * log2 e).
    // Saturates exactly (exp2 -> inf gives 1, -> 0 gives -1); absolute error ~1e-7, far below
    // the bf16 / fp8 rounding of the stored activation.
    const float e = __builtin_amdgcn_exp2f(x * (2.0f * 1.4426950408889634f));
    return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
  }
}

// k-steps per prefetch chunk: 2, so two register sets plus the cross-barrier BPre set stay
// inside the 2-waves/SIMD VGPR budget at every row tile (4 spilled once BPre was added).
// 4-wide tanh for the epilogues: f32x4 arithmetic lowers to packed 2-wide f32 VALU ops.
template <int DT>
DEV f32x4 act_tanh4(f32x4 x) {
  if constexpr (DT == DT_F32) {
    return f32x4{tanhf(x[0]), tanhf(x[1]), tanhf(x[2]), tanhf(x[3])};
  } else {
    const f32x4 y = x * (2.0f * 1.4426950408889634f);
    f32x4 e;
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = __builtin_amdgcn_exp2f(y[i]);
    e = e + 1.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = __builtin_amdgcn_rcpf(e[i]);
    return __builtin_elementwise_fma(e, f32x4{-2.f, -2.f, -2.f, -2.f}, f32x4{1.f, 1.f, 1.f, 1.f});
  }
}

// f32x4 -> 4 storage elements (bf16: two v_cvt_pk_bf16_f32)
template <int DT>
DEV void cvt4(const f32x4& v, typename Prec<DT>::T (&q)[4]) {
  using P = Prec<DT>;
  if constexpr (DT == DT_BF16) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    *reinterpret_cast<bf16x4*>(q) = __builtin_convertvector(v, bf16x4);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = P::cvt(v[i]);
  }
}

// 4 converted values -> 4 consecutive elements of a transposed (FM) operand row.  Non-temporal
// (streaming) stores: the wgrad operands (~200 MB per epoch) are read back only by the next
// kernel, long after they would have left L2, and with normal stores they evict the weight
// images every layer re-reads from L2.
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4s;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4v;
template <int DT>
DEV void store4q_T(typename Prec<DT>::T* dst, const typename Prec<DT>::T (&q)[4]) {
  if constexpr (DT == DT_F32) {
    opnd_store(f32x4s{q[0], q[1], q[2], q[3]}, reinterpret_cast<f32x4s*>(dst));
  } else if constexpr (DT == DT_BF16) {
    opnd_store(*reinterpret_cast<const u32x2*>(q), reinterpret_cast<u32x2*>(dst));
  } else {
    opnd_store(*reinterpret_cast<const uint32_t*>(q), reinterpret_cast<uint32_t*>(dst));
  }
}

// (split-bf16 fragments are twice the registers: one k-step per chunk keeps the 8-wave, 2-waves-
// per-SIMD form inside 256 VGPRs; the second wave per SIMD hides the latency instead)
// register sets in the layer_gemm rotation (prefetch distance NB - 1 steps).  split-bf16 at 8
// waves runs one k-step per chunk with VGPRs to spare, so it prefetches deeper: a step is only
// 12 MFMAs there, far shorter than the L2 latency of the weight fragments it waits for.
// (3 sets for split-bf16 at 8 waves measured neutral: profiles/r4/ab_rollout_nb3/)
template <int DT, int NW> struct GemmDepth { static constexpr int NB = 2; };

template <int DT, int RB> struct KChunk { static constexpr int KC = IsSplit<DT>::value ? 1 : 2; };

// B fragments of a wave's FIRST (tile pair, k-chunk) step of one layer_gemm call, loaded ahead
// of time by layer_prefetch: weights do not depend on the previous layer, so their L2 latency
// can overlap a barrier wait or another phase instead of stalling the layer's first MFMA.
// (one type per k-chunk size, so 32- and 64-row calls with the same KC share a prefetch set)
template <int DT, int KC> struct BPreK {
  typename Prec<DT>::Frag b0[KC], b1[KC];
};
template <int DT, int RB> using BPre = BPreK<DT, KChunk<DT, RB>::KC>;

template <int DT, int ROWS, int NW>
DEV void layer_prefetch(BPre<DT, ROWS / 16>& pre, const typename Prec<DT>::T* __restrict__ B, int kdim,
                        int n_real, int wave, int lane, int wrot = 0) {
  using P = Prec<DT>;
  constexpr int KC = KChunk<DT, ROWS / 16>::KC;
  wave = __builtin_amdgcn_readfirstlane((wave + wrot) & (NW - 1));
  const int ksteps = kdim >> 5;
  const int first_pair = wave * 2;
  if (first_pair >= ((n_real + 15) >> 4)) return;
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    const typename P::T* p0 = B + fm_frag(first_pair, min(j, ksteps - 1), kdim, lane);
    pre.b0[j] = P::load(p0);
    pre.b1[j] = P::load(p0 + (size_t)ksteps * 512);
  }
}

template <int DT, int ROWS, int NW, int EPI, bool PRE = false, typename OutT>
DEV void layer_gemm(const typename Prec<DT>::T* __restrict__ A, int lda, int kdim,
                    const typename Prec<DT>::T* __restrict__ B, int n_real,
                    OutT* out, int ldo, float scale, int wave, int lane,
                    typename Prec<DT>::T* __restrict__ outT = nullptr, int ldT = 0, int m0 = 0, int wrot = 0,
                    const BPre<DT, ROWS / 16>* pre = nullptr) {
  using P = Prec<DT>;
  using T = typename P::T;
  using Frag = typename P::Frag;
  constexpr int RB = ROWS / 16;
  constexpr int KC = KChunk<DT, RB>::KC;
  constexpr int NT2 = 2;
  // every quantity that steers control flow is wave-uniform and must live in SGPRs: with a
  // VGPR `wave` the compiler turns the step loop into EXEC-masked regions and waits for ALL
  // outstanding loads (vmcnt(0)) at each merge — the prefetch below would never overlap
  // wrot rotates the wave -> tile-pair map so two back-to-back narrow layers (policy and
  // value head, 4 pairs each) land on disjoint waves when NW = 8
  wave = __builtin_amdgcn_readfirstlane((wave + wrot) & (NW - 1));
  const int ksteps = kdim >> 5;
  const int nchunks = (ksteps + KC - 1) / KC;
  const int ntiles = (n_real + 15) >> 4;
  const int lr = lane & 15;
  const T* ap = A + lr * lda + (lane >> 4) * 8;
  // This wave's work is a flat stream of (tile pair, k-chunk) steps; the A (LDS) and B (L2)
  // fragments of step s+1 — including the FIRST chunk of the wave's next tile pair — are
  // loaded while step s computes.  Two register sets alternate (s even: set 0 computes, set 1
  // loads), so no fragment is ever copied between registers.
  const int first_pair = wave * NT2;
  if (first_pair >= ntiles) return;
  const int npairs = (ntiles - first_pair + NW * NT2 - 1) / (NW * NT2);
  const int nsteps = npairs * nchunks;
  struct Buf { Frag b0[KC], b1[KC], a[KC][RB]; };
  // The partner tile nt+1 of an (even) nt always exists in memory: every image's row count is
  // a multiple of 32 (PackedLayout pads d_out / d_in to P32), so past n_real it is zero padding
  // and its MFMA results are simply not stored.  Loading it unconditionally keeps the loads
  // branch-free (a select between "reload" and "reuse" made the compiler wait vmcnt(0)).
  auto load = [&](Buf& d, int nt, int kc_) {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const int ks = min(kc_ * KC + j, ksteps - 1);   // past-the-end steps re-load the last one
      const T* p0 = B + fm_frag(nt, ks, kdim, lane);
      d.b0[j] = P::load(p0);
      d.b1[j] = P::load(p0 + (size_t)ksteps * 512);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) d.a[j][rb] = P::load(ap + rb * 16 * lda + ks * 32);
    }
  };
  auto load_a0 = [&](Buf& d) {   // A fragments of chunk 0 (the B half came from layer_prefetch)
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const int ks = min(j, ksteps - 1);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) d.a[j][rb] = P::load(ap + rb * 16 * lda + ks * 32);
    }
  };
  f32x4 acc[NT2][RB];
#pragma unroll
  for (int t = 0; t < NT2; ++t)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) acc[t][rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const Buf& c, int kc_) {
    if ((kc_ + 1) * KC <= ksteps) {   // full chunk: straight-line, no per-step branch
#pragma unroll
      for (int j = 0; j < KC; ++j)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          acc[0][rb] = P::mma(acc[0][rb], c.a[j][rb], c.b0[j]);
          acc[1][rb] = P::mma(acc[1][rb], c.a[j][rb], c.b1[j]);
        }
    } else {                           // ragged last chunk (kdim not a multiple of 32*KC)
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        if (kc_ * KC + j < ksteps) {
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) {
            acc[0][rb] = P::mma(acc[0][rb], c.a[j][rb], c.b0[j]);
            acc[1][rb] = P::mma(acc[1][rb], c.a[j][rb], c.b1[j]);
          }
        }
      }
    }
  };
  // Epilogue of one tile pair: per (tile, row block) a lane holds 4 consecutive rows of one
  // column.  The 4 values go through the activation with packed 2-wide f32 math (v_pk_mul /
  // v_pk_add / v_pk_fma; exp2 / rcp stay scalar on the transcendental unit), are converted to
  // the storage type ONCE, and that one conversion feeds both the LDS tile (2-byte row stores)
  // and the 8-byte transposed wgrad-operand store.
  auto epilogue = [&](int nt0) {
    const bool two = (nt0 + 1) < ntiles;
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const int c = (nt0 + t) * 16 + lr;
      if (c < n_real && (t == 0 || two)) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const int r0 = rb * 16 + (lane >> 4) * 4;
          f32x4 v = acc[t][rb];
          if constexpr (DT == DT_FP8) v *= scale;   // e4m3 weight scale; 1 for bf16 / fp32
          if constexpr (EPI == EPI_LINEAR_F32) {
#pragma unroll
            for (int i = 0; i < 4; ++i) out[(r0 + i) * ldo + c] = v[i];
          } else {
            if constexpr (EPI == EPI_TANH) {
              v = act_tanh4<DT>(v);
            } else if constexpr (EPI == EPI_DTANH_INPLACE || EPI == EPI_DTANH_GLOBAL) {
              // out holds h = tanh(pre) of this layer's input; dpre = v * (1 - h^2)
              f32x4 h;
              if constexpr (IsSplit<DT>::value) {
                // rows r0..r0+3 of column c: one per-lane base, then a fixed row stride (ldo is
                // a multiple of 8, so the hi|lo group arithmetic is per column only)
                const __bf16* hp = P::hi_ptr(out, (size_t)r0 * ldo + c);
#pragma unroll
                for (int i = 0; i < 4; ++i) h[i] = (float)hp[2 * i * ldo] + (float)hp[2 * i * ldo + 8];
              } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) h[i] = P::get(out, (r0 + i) * ldo + c);
              }
              v = v * (1.0f - h * h);
            }
            if constexpr (IsSplit<DT>::value) {
              // split-bf16: hi = bf16(v), lo = bf16(v - hi), 4-wide (packed converts); LDS row
              // stores per element, and the transposed operand's 4 consecutive m as one 8-byte
              // hi store + one 8-byte lo store (the 4 slots share one 8-group: m0 + r0 % 4 == 0)
              const bf16x4v hv = __builtin_convertvector(v, bf16x4v);
              const bf16x4v lv = __builtin_convertvector(v - __builtin_convertvector(hv, f32x4), bf16x4v);
              if constexpr (EPI != EPI_DTANH_GLOBAL) {
                __bf16* p = P::hi_ptr(out, (size_t)r0 * ldo + c);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  p[2 * i * ldo] = hv[i];
                  p[2 * i * ldo + 8] = lv[i];
                }
              }
              if (outT != nullptr) {
                __bf16* p = P::hi_ptr(outT, fm_index(c, m0 + r0, ldT));
                opnd_store(*reinterpret_cast<const u32x2*>(&hv), reinterpret_cast<u32x2*>(p));
                opnd_store(*reinterpret_cast<const u32x2*>(&lv), reinterpret_cast<u32x2*>(p + 8));
              }
            } else {
              typename P::T q[4];
              cvt4<DT>(v, q);
              if constexpr (EPI != EPI_DTANH_GLOBAL) {
                if constexpr (DT == DT_BF16) {
                  // 2-byte row stores straight from the two packed dwords (ds_write_b16 /
                  // ds_write_b16_d16_hi): no second per-value conversion
                  uint32_t wx = reinterpret_cast<const uint32_t*>(q)[0];
                  uint32_t wy = reinterpret_cast<const uint32_t*>(q)[1];
                  // opaque: otherwise LLVM folds trunc(cvt_pk(a, b)) back into a per-value cvt
                  asm volatile("" : "+v"(wx), "+v"(wy));
                  const uint2 w = make_uint2(wx, wy);
                  uint16_t* o16 = reinterpret_cast<uint16_t*>(out);
                  o16[(r0 + 0) * ldo + c] = (uint16_t)w.x;
                  o16[(r0 + 1) * ldo + c] = (uint16_t)(w.x >> 16);
                  o16[(r0 + 2) * ldo + c] = (uint16_t)w.y;
                  o16[(r0 + 3) * ldo + c] = (uint16_t)(w.y >> 16);
                } else {
#pragma unroll
                  for (int i = 0; i < 4; ++i) out[(r0 + i) * ldo + c] = q[i];
                }
              }
              if (outT != nullptr)   // FM wgrad operand: 4 consecutive m of feature c are contiguous
                store4q_T<DT>(outT + fm_index(c, m0 + r0, ldT), q);
            }
          }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT2; ++t)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[t][rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // NB register sets in rotation: the loads of step s + NB - 1 are issued while step s
  // computes (prefetch distance NB - 1 steps).  Past the end, a load re-reads the last step's
  // (valid) addresses, so every step issues the same loads and the compiler's vmcnt waits stay
  // exact.  The load cursor (ntl, kcl, sl) runs NB - 1 steps ahead of the compute cursor.
  constexpr int NB = GemmDepth<DT, NW>::NB;
  if constexpr (NB == 2) {
    // the two-set form: prefetch step s+1 into `nx` (unconditionally: past the end it re-loads
    // valid addresses), compute step s from `cur`, epilogue at the end of a pair
    Buf buf0, buf1;
    int nt0 = first_pair, kc = 0;
    if constexpr (PRE) {
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        buf0.b0[j] = pre->b0[j];
        buf0.b1[j] = pre->b1[j];
      }
      load_a0(buf0);
    } else {
      load(buf0, nt0, 0);
    }
    auto step = [&](int s, const Buf& cur, Buf& nx) {
      int nt1 = nt0, kc1 = kc + 1;
      if (kc1 == nchunks) { kc1 = 0; nt1 = nt0 + NW * NT2; }
      if (s + 1 >= nsteps) { nt1 = nt0; kc1 = kc; }
      load(nx, nt1, kc1);
      compute(cur, kc);
      if (++kc == nchunks) {
        epilogue(nt0);
        kc = 0;
        nt0 += NW * NT2;
      }
    };
    int s = 0;
    for (; s + 1 < nsteps; s += 2) {
      step(s, buf0, buf1);
      step(s + 1, buf1, buf0);
    }
    if (s < nsteps) step(s, buf0, buf1);
    return;
  }
  Buf buf[NB];
  int nt0 = first_pair, kc = 0;
  int ntl = first_pair, kcl = 0, sl = 0;
  const int nt_last = first_pair + (npairs - 1) * NW * NT2, kc_last = nchunks - 1;
  auto load_next = [&](Buf& d) {
    const bool v = sl < nsteps;
    load(d, v ? ntl : nt_last, v ? kcl : kc_last);
    if (++kcl == nchunks) { kcl = 0; ntl += NW * NT2; }
    ++sl;
  };
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      buf[0].b0[j] = pre->b0[j];
      buf[0].b1[j] = pre->b1[j];
    }
    load_a0(buf[0]);
    if (++kcl == nchunks) { kcl = 0; ntl += NW * NT2; }
    ++sl;
  } else {
    load_next(buf[0]);
  }
#pragma unroll
  for (int j = 1; j < NB - 1; ++j) load_next(buf[j]);
  // one step: prefetch into the set NB - 1 ahead, compute the current set, epilogue at the end
  // of a tile pair
  auto step = [&](const Buf& cur, Buf& nx) {
    load_next(nx);
    compute(cur, kc);
    if (++kc == nchunks) {
      epilogue(nt0);
      kc = 0;
      nt0 += NW * NT2;
    }
  };
  int s = 0;
  for (; s + NB <= nsteps; s += NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u) step(buf[u], buf[(u + NB - 1) % NB]);
  }
#pragma unroll
  for (int u = 0; u < NB - 1; ++u)
    if (s + u < nsteps) step(buf[u], buf[(u + NB - 1) % NB]);
}

__host__ __device__ inline size_t al16(size_t b) { return (b + 15) & ~size_t(15); }

// 16-byte aligned carve of the dynamic LDS region (Guideline 17: keep the base 16-B aligned).
struct LdsCarve {
  char* base;
  size_t off;
  DEV explicit LdsCarve(char* b) : base(b), off(0) {}
  template <typename T>
  DEV T* take(size_t n) {
    T* p = reinterpret_cast<T*>(base + off);
    off += (n * sizeof(T) + 15) & ~size_t(15);
    return p;
  }
};

// Columns [c0, ld) of a rows x ld activation tile: column c0 = 1 (the constant bias input of
// the next layer), the rest 0.  Written as whole 16-byte chunks (split-bf16: 32-byte hi|lo
// groups) from the chunk holding c0 on, so the columns of that chunk below c0 are zeroed too:
// callers preset BEFORE the producing layer's epilogue writes every row of the columns
// c < n_real (layer_gemm stores all ROWS rows of each of them), behind a barrier.
template <int DT>
DEV void preset_pad(typename Prec<DT>::T* H, int ld, int rows, int c0, int tid, int nthreads) {
  using P = Prec<DT>;
  constexpr bool SPLIT = IsSplit<DT>::value;
  constexpr int G = SPLIT ? 8 : 16 / P::BYTES;   // logical elements per chunk (ld % G == 0)
  const int g0 = c0 / G, ng = ld / G - g0;
  for (int i = tid; i < rows * ng; i += nthreads) {
    const int r = i / ng, g = g0 + (i - r * ng);
    const int one = c0 - g * G;                   // column c0 inside this chunk, if it is here
    // the 1.0 bit pattern of the storage type, placed in dword `wi` at bit `sh` (register
    // selects only: a dynamically indexed local array would live in scratch)
    constexpr int EPW = 4 / (SPLIT ? 2 : P::BYTES);   // elements per dword
    constexpr uint32_t ONE = (SPLIT || DT == DT_BF16) ? 0x3F80u : (DT == DT_F32 ? 0x3F800000u : 0x38u);
    const bool here = one >= 0 && one < G;
    const int wi = one / EPW, sh = (one - wi * EPW) * (32 / EPW);
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (here && wi == k) ? (ONE << sh) : 0u;
    uint4* dst = reinterpret_cast<uint4*>(H + (size_t)r * ld + (size_t)g * G);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    if constexpr (SPLIT) dst[1] = make_uint4(0, 0, 0, 0);             // lo of the group
  }
}

// Zero a whole rows x ld tile with 16-byte stores (ld * sizeof(T) is a multiple of 16 for
// every Lds<DT>::stride of a P32 width, and LdsCarve keeps tile bases 16-byte aligned).
template <int DT>
DEV void zero_tile(typename Prec<DT>::T* H, int ld, int rows, int tid, int nthreads) {
  const int n16 = rows * ld * Prec<DT>::BYTES / 16;
  uint4* h = reinterpret_cast<uint4*>(H);
  for (int i = tid; i < n16; i += nthreads) h[i] = make_uint4(0, 0, 0, 0);
}
