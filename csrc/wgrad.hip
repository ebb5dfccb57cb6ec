// Weight-gradient GEMM for all six layers in ONE launch (grouped, split-K over the batch).
//
//   dW_aug[n][k] = sum_m dY[m][n] * X[m][k]      (k == K is the bias column: X^T row K == 1)
//
// Both operands are feature-major (written transposed by mlp_train_kernel), so every MFMA
// fragment is one 16-byte load along m, the reduction axis.  A task = (layer, 64x64 output
// tile, batch chunk); each of the 4 waves owns a 32x32 quadrant (2x2 16x16 MFMA tiles, f32
// accumulate).  Results go to per-chunk fp32 slabs that grad_gather sums in a fixed order —
// deterministic, no float atomics (SURVEY §7.4 hard part 2).
#include "kernels.h"
#include "mlp_core.h"

namespace {

template <int DT>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  using Frag = typename P::Frag;
  const WgradTask tk = a.tasks[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const T* g = reinterpret_cast<const T*>(a.gT[tk.layer]);
  const T* x = reinterpret_cast<const T*>(a.xT[tk.layer]);
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const T* ga0 = g + (size_t)(tk.n0 + wn * 32 + lr) * a.ld + lk;
  const T* ga1 = ga0 + (size_t)16 * a.ld;
  const T* xb0 = x + (size_t)(tk.k0 + wk * 32 + lr) * a.ld + lk;
  const T* xb1 = xb0 + (size_t)16 * a.ld;
  f32x4 acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
  int m = tk.m0;
  // two 32-deep k-steps per iteration: 8 independent 16-byte loads in flight per lane
  for (; m + 64 <= tk.m1; m += 64) {
    Frag a0 = P::load(ga0 + m), a1 = P::load(ga1 + m);
    Frag b0 = P::load(xb0 + m), b1 = P::load(xb1 + m);
    Frag c0 = P::load(ga0 + m + 32), c1 = P::load(ga1 + m + 32);
    Frag d0 = P::load(xb0 + m + 32), d1 = P::load(xb1 + m + 32);
    acc00 = P::mma(acc00, a0, b0);
    acc01 = P::mma(acc01, a0, b1);
    acc10 = P::mma(acc10, a1, b0);
    acc11 = P::mma(acc11, a1, b1);
    acc00 = P::mma(acc00, c0, d0);
    acc01 = P::mma(acc01, c0, d1);
    acc10 = P::mma(acc10, c1, d0);
    acc11 = P::mma(acc11, c1, d1);
  }
  for (; m < tk.m1; m += 32) {
    Frag a0 = P::load(ga0 + m), a1 = P::load(ga1 + m);
    Frag b0 = P::load(xb0 + m), b1 = P::load(xb1 + m);
    acc00 = P::mma(acc00, a0, b0);
    acc01 = P::mma(acc01, a0, b1);
    acc10 = P::mma(acc10, a1, b0);
    acc11 = P::mma(acc11, a1, b1);
  }
  float* out = a.slab + tk.slab;
  const int col = wk * 32 + lr;
  const int rbase = wn * 32 + (lane >> 4) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    out[(rbase + q) * 64 + col] = acc00[q];
    out[(rbase + q) * 64 + col + 16] = acc01[q];
    out[(rbase + 16 + q) * 64 + col] = acc10[q];
    out[(rbase + 16 + q) * 64 + col + 16] = acc11[q];
  }
}

// grad[i] = scale * sum_c slab[c*stride + src_off[i]]   (fixed chunk order: deterministic)
// i < A (log_std): grad[i] = scale * sum_b part[b*npart + 8 + i]
__global__ __launch_bounds__(256) void grad_gather_kernel(const float* __restrict__ slab,
                                                          const int* __restrict__ src_off, int nchunks,
                                                          int stride, const float* __restrict__ part,
                                                          int nblk, int npart, int A, float scale,
                                                          float* __restrict__ grad, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    float s = 0.f;
    if (i < A) {
      for (int b = 0; b < nblk; ++b) s += part[(size_t)b * npart + 8 + i];
    } else {
      const int o = src_off[i];
      for (int c = 0; c < nchunks; ++c) s += slab[(size_t)c * stride + o];
    }
    grad[i] = s * scale;
  }
}

}  // namespace

extern "C" void launch_wgrad(int dt, const WgradArgs& a, hipStream_t s) {
  if (a.ntasks <= 0) return;
  if (dt == DT_F32) hipLaunchKernelGGL(wgrad_kernel<DT_F32>, dim3(a.ntasks), dim3(256), 0, s, a);
  else if (dt == DT_BF16) hipLaunchKernelGGL(wgrad_kernel<DT_BF16>, dim3(a.ntasks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(wgrad_kernel<DT_FP8>, dim3(a.ntasks), dim3(256), 0, s, a);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_grad_gather(const float* slab, const int* src_off, int nchunks, int chunk_stride,
                                   const float* part, int nblk, int npart, int A, float scale, float* grad,
                                   int n, hipStream_t s) {
  int grid = (n + 255) / 256;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(grad_gather_kernel, dim3(grid), dim3(256), 0, s, slab, src_off, nchunks, chunk_stride,
                     part, nblk, npart, A, scale, grad, n);
  HIP_CHECK_LAUNCH();
}
