// Device helpers of the transposed-chain 32x32x16 MFMA kernel (csrc/phead.hip).
//
// In the transposed chain every layer computes out^T = W . in^T: A = a weight fragment (32 output
// features x 16 k from an LDS ring), B = the activations (16 k x 32 batch rows, in registers).  The
// accumulator has the batch row on the lane (col = lane & 31) and 16 output features in its
// registers (feature (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)); b_operand turns 8 of them into the
// next layer's B operand with one v_permlane32_swap per dword.
#pragma once
#include <type_traits>

#include "kernels.h"
#include "common.h"

namespace t32 {

constexpr float T32_LOG_2PI = 1.8378770664093453f;

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2v;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v;

template <int DT> struct VT;
template <> struct VT<DT_S3> {           // split-bf16: fragment = hi 1 KiB | lo 1 KiB
  using Frag = S3Frag;
  static constexpr int FB = 2048, KPS = 1, EB = 4;
  DEV static f32x16 mma(f32x16 c, const Frag& a, const Frag& b) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, c, 0, 0, 0);
  }
  // ring slot u of a stage (lane l: hi at (l / 32) KiB + 16 (l % 32), lo 512 B on)
  DEV static Frag ring(const char* stg, int u, int lane) {
    const char* p = stg + u * FB + (lane >> 5) * 1024 + (lane & 31) * 16;
    return Frag{*reinterpret_cast<const bf16x8*>(p), *reinterpret_cast<const bf16x8*>(p + 512)};
  }
  // the element (n, k) of a packed image, as fp32
  DEV static float img(const void* W, size_t i) {
    const __bf16* p = reinterpret_cast<const __bf16*>(W) + 2 * (i & ~size_t(7)) + (i & 7);
    return (float)p[0] + (float)p[8];
  }
};
template <> struct VT<DT_BF16> {
  using Frag = bf16x8;
  static constexpr int FB = 1024, KPS = 2, EB = 2;
  DEV static f32x16 mma(f32x16 c, const Frag& a, const Frag& b) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  DEV static Frag ring(const char* stg, int u, int lane) {
    return *reinterpret_cast<const bf16x8*>(stg + u * FB + lane * 16);
  }
  DEV static float img(const void* W, size_t i) { return (float)reinterpret_cast<const __bf16*>(W)[i]; }
};

DEV f32x16 tanh16(f32x16 x) {
  // tanh x = 1 - 2 / (1 + 2^(2 log2(e) x)) (csrc/mlp_core.h act_tanh: exp + rcp, |err| ~1e-7)
  f32x16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float e = __builtin_amdgcn_exp2f(x[i] * (2.0f * 1.4426950408889634f));
    r[i] = __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
  }
  return r;
}

// 4 fp32 -> 4 bf16 in 2 dwords
DEV u32x2v pk4(float a, float b, float c, float d) {
  const bf16x4 h = __builtin_convertvector((f32x4){a, b, c, d}, bf16x4);
  return *reinterpret_cast<const u32x2v*>(&h);
}
DEV f32x4 unpk4(u32x2v v) {
  const bf16x4 h = *reinterpret_cast<const bf16x4*>(&v);
  return __builtin_convertvector(h, f32x4);
}

// The B operand of k-step s (features 16 s .. 16 s + 15 of a 32-feature accumulator tile x) in
// natural k order: lanes 0-31 need features 0-7, lanes 32-63 features 8-15; each lane holds
// P = features 4h + 0..3 (regs 8s .. 8s+3) and Q = 8 + 4h + 0..3 (regs 8s+4 .. 8s+7), so ONE
// v_permlane32_swap per dword (P of the upper half <-> Q of the lower half) completes both.
DEV bf16x8 swap_b(u32x2v P, u32x2v Q) {
  u32x4v o;
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto r = __builtin_amdgcn_permlane32_swap(P[d], Q[d], false, false);
    o[d] = r[0];
    o[2 + d] = r[1];
  }
  return *reinterpret_cast<const bf16x8*>(&o);
}
template <int DT>
DEV typename VT<DT>::Frag b_operand(const f32x16& x, int s) {
  const f32x4 p{x[8 * s], x[8 * s + 1], x[8 * s + 2], x[8 * s + 3]};
  const f32x4 q{x[8 * s + 4], x[8 * s + 5], x[8 * s + 6], x[8 * s + 7]};
  const u32x2v ph = pk4(p[0], p[1], p[2], p[3]), qh = pk4(q[0], q[1], q[2], q[3]);
  if constexpr (DT == DT_S3) {
    const f32x4 pr = p - unpk4(ph), qr = q - unpk4(qh);
    const u32x2v pl = pk4(pr[0], pr[1], pr[2], pr[3]), ql = pk4(qr[0], qr[1], qr[2], qr[3]);
    return S3Frag{swap_b(ph, qh), swap_b(pl, ql)};
  } else {
    return swap_b(ph, qh);
  }
}

// s_waitcnt vmcnt(n) for a runtime n (counts past 23 wait for 23: undercounting only waits longer)
DEV void wait_vm_rt(int n) {
  switch (n) {
#define T32_VMC(k) \
  case k: WAIT_VMCNT(k); break;
    T32_VMC(0) T32_VMC(1) T32_VMC(2) T32_VMC(3) T32_VMC(4) T32_VMC(5) T32_VMC(6) T32_VMC(7)
    T32_VMC(8) T32_VMC(9) T32_VMC(10) T32_VMC(11) T32_VMC(12) T32_VMC(13) T32_VMC(14) T32_VMC(15)
    T32_VMC(16) T32_VMC(17) T32_VMC(18) T32_VMC(19) T32_VMC(20) T32_VMC(21) T32_VMC(22)
#undef T32_VMC
    default: WAIT_VMCNT(23); break;
  }
}

// Counted-wait bookkeeping of a 3-stage ring past its runtime-length prologue: n counts every
// vector-memory instruction the wave issues (refills, X loads AND operand stores); ma / mb are
// the counts right after the two pending ring batches (stage st, st + 1).  The sync of stage st
// waits with exactly the instructions issued after its batch still in flight (vmcnt counts in
// issue order on gfx9-family parts): a wait that left the younger stores out would wait for them
// to reach memory, an op left uncounted only makes the wait longer.  In straight-line (unrolled)
// code every count folds to a constant: one s_waitcnt, no switch.
struct VmTrack {
  int n, ma, mb;
  // entering with stage st's batch `older` instructions back and stage st + 1's `older1`
  DEV explicit VmTrack(int older, int older1 = 0) : n(0), ma(-older), mb(-older1) {}
  DEV void add(int k) { n += k; }
  DEV int younger() const { return n - ma; }
  // after stage st's sync: the refill (stage st + 2, `k` instructions) or none
  DEV void advance(int k) {
    n += k;
    ma = mb;
    mb = n;
  }
};

template <int B, int E, typename F>
DEV void static_for_vh(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for_vh<B + 1, E>(f);
  }
}

// MFMAs over N ring fragments slot(0 .. N-1) of a stage, read in groups of G: group g + 1's LDS
// reads are in flight while group g's MFMAs run.  f(i, fragment).
template <int DT, int N, int G, typename SLOT, typename F>
DEV void ring_mma(const char* stg, int lane, SLOT&& slot, F&& f) {
  using Frag = typename VT<DT>::Frag;
  constexpr int NG = N / G;
  static_assert(N % G == 0, "groups");
  Frag b[2][G];
  static_for_vh<0, G>([&](auto ic) __attribute__((always_inline)) {
    b[0][decltype(ic)::value] = VT<DT>::ring(stg, slot(decltype(ic)::value), lane);
  });
  static_for_vh<0, NG>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    if constexpr (g + 1 < NG) {
      static_for_vh<0, G>([&](auto ic) __attribute__((always_inline)) {
        b[(g + 1) & 1][decltype(ic)::value] = VT<DT>::ring(stg, slot((g + 1) * G + decltype(ic)::value), lane);
      });
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for_vh<0, G>([&](auto ic) __attribute__((always_inline)) {
      f(g * G + decltype(ic)::value, b[g & 1][decltype(ic)::value]);
    });
  });
}

// one lane's 16 features of an operand row (natural order: the b_operand / swap_b layout) ->
// the row-major wgrad operand (split: the 32-byte [8 hi | 8 lo] group of each 8 features) by a
// non-temporal buffer store: vrow = the lane's row byte offset + its 8-feature group, fsoff = the
// wave-uniform feature offset (bytes) — no 64-bit address registers live across the chain.
//
// The store's data registers stay untouched for two wait states after it issues: a VALU write
// of a 16-byte store's data right behind the store replaced what it stored for the last 4 lanes
// of each 16-lane group (measured: the bf16 value head's g1 rows, scripts/debug_t32_nan.py), a
// store-data WAR the compiler did not pad here
DEV void st_b128(u32x4v v, __amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, 0);
  asm volatile("s_nop 1" ::"v"(v));
}
template <int DT>
DEV void st_op(__amdgpu_buffer_rsrc_t rs, unsigned vrow, unsigned fsoff, const typename VT<DT>::Frag& f) {
  if constexpr (DT == DT_S3) {
    st_b128(*reinterpret_cast<const u32x4v*>(&f.h), rs, vrow, fsoff);
    st_b128(*reinterpret_cast<const u32x4v*>(&f.l), rs, vrow + 16, fsoff);
  } else {
    st_b128(*reinterpret_cast<const u32x4v*>(&f), rs, vrow, fsoff);
  }
}

// sum over the 32 lanes of each half-wave of 32 values per lane (a butterfly: each level keeps half
// the values, so 31 shuffles instead of 5 x 32); lane l ends with the sum of value l & 31 (fixed order)
DEV float half_sum32(float (&v)[32], int lane) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) {
    const bool up = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < m; ++i) {
      const float send = up ? v[i] : v[i + m];
      const float got = __shfl_xor(send, m, 64);
      v[i] = (up ? v[i + m] : v[i]) + got;
    }
  }
  return v[0];
}

// the same over 16 values per lane: lanes l and l ^ 16 first add (the 32-lane sum then halves
// over 4 levels); lane l ends with the sum of value l & 15
DEV float half_sum16(float (&v)[16], int lane) {
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] += __shfl_xor(v[i], 16, 64);
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) {
    const bool up = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < m; ++i) {
      const float send = up ? v[i] : v[i + m];
      const float got = __shfl_xor(send, m, 64);
      v[i] = (up ? v[i + m] : v[i]) + got;
    }
  }
  return v[0];
}

}  // namespace t32
