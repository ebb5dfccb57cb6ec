// Dense-layer building block shared by the rollout kernel and the fused update kernel.
//
//   out[r][c] = EPI( sum_k A[r][k] * B[c][k] )     r < ROWS, c < n_real, k < kdim (mult. of 32)
//
// A is a row tile in LDS (activations, or upstream gradients for dgrad), B is a row-major
// weight image in global memory (L2-resident; Wp [d_out][d_in] for forward, Wpt [d_in][d_out]
// for dgrad).  The bias is column K of Wp and the activation tiles carry a constant 1 in
// column K, so no separate bias add exists anywhere (PackedLayout in models/actor_critic.py).
//
// Work split: the 4 (or NW) waves of the workgroup stride over 16-wide output column tiles;
// each wave computes ALL ROWS/16 row blocks of its column tile, so one 16-byte B fragment
// (weights, the operand that comes from L2) feeds ROWS/16 MFMAs.  The next k-step's B
// fragment is requested before the current MFMAs issue (one tile of prefetch).
#pragma once
#include "common.h"

enum { EPI_TANH = 0, EPI_LINEAR_F32 = 1, EPI_DTANH_INPLACE = 2, EPI_LINEAR_T = 3 };

template <int DT, int ROWS, int NW, int EPI, typename OutT>
DEV void layer_gemm(const typename Prec<DT>::T* __restrict__ A, int lda, int kdim,
                    const typename Prec<DT>::T* __restrict__ B, int n_real,
                    OutT* out, int ldo, float scale, int wave, int lane) {
  using P = Prec<DT>;
  using Frag = typename P::Frag;
  constexpr int RB = ROWS / 16;
  const int ksteps = kdim >> 5;
  const int ntiles = (n_real + 15) >> 4;
  const int lr = lane & 15;
  const int lk = (lane >> 4) * 8;
  // each pass of a wave covers NT2 = 2 adjacent column tiles: 2 B fragments + RB A fragments
  // per k-step feed 2*RB MFMAs, and the next k-step's B fragments are already in flight.
  constexpr int NT2 = 2;
  for (int nt0 = wave * NT2; nt0 < ntiles; nt0 += NW * NT2) {
    const bool two = (nt0 + 1) < ntiles;
    f32x4 acc[NT2][RB];
#pragma unroll
    for (int t = 0; t < NT2; ++t)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[t][rb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const typename P::T* bp0 = B + (size_t)(nt0 * 16 + lr) * kdim + lk;
    // the second tile's pointer is clamped to the first when it does not exist (loads stay in
    // bounds; its results are discarded)
    const typename P::T* bp1 = two ? bp0 + (size_t)16 * kdim : bp0;
    const typename P::T* ap = A + lr * lda + lk;
    Frag bn0 = P::load(bp0), bn1 = P::load(bp1);
    for (int ks = 0; ks < ksteps; ++ks) {
      Frag b0 = bn0, b1 = bn1;
      if (ks + 1 < ksteps) {
        bn0 = P::load(bp0 + (ks + 1) * 32);
        bn1 = P::load(bp1 + (ks + 1) * 32);
      }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        Frag a = P::load(ap + rb * 16 * lda + ks * 32);
        acc[0][rb] = P::mma(acc[0][rb], a, b0);
        acc[1][rb] = P::mma(acc[1][rb], a, b1);
      }
    }
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const int c = (nt0 + t) * 16 + lr;
      if (c < n_real && (t == 0 || two)) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = rb * 16 + (lane >> 4) * 4 + i;
            float v = acc[t][rb][i] * scale;
            if constexpr (EPI == EPI_TANH) {
              out[r * ldo + c] = P::cvt(tanhf(v));
            } else if constexpr (EPI == EPI_LINEAR_F32) {
              out[r * ldo + c] = v;
            } else if constexpr (EPI == EPI_LINEAR_T) {
              out[r * ldo + c] = P::cvt(v);
            } else {  // EPI_DTANH_INPLACE: out holds h = tanh(pre); write dpre = v * (1 - h^2)
              float h = P::tof(out[r * ldo + c]);
              out[r * ldo + c] = P::cvt(v * (1.0f - h * h));
            }
          }
        }
      }
    }
  }
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
