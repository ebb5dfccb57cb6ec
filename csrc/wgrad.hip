// Weight-gradient GEMM for all six layers in ONE launch (grouped, split-K over the batch).
//
//   dW_aug[n][k] = sum_m dY[m][n] * X[m][k]      (k == K is the bias column: X^T row K == 1)
//
// Both operands are feature-major (written transposed by mlp_train_kernel), so every MFMA
// fragment is one 16-byte load along m, the reduction axis.  A task = (layer, 128x128 output
// tile, batch chunk); each of the 4 waves owns a 64x64 quadrant = 4x4 tiles of 16x16 MFMA
// (64 f32 accumulator registers), so one k-step issues 8 fragment loads for 16 MFMAs.
// Results go to per-chunk fp32 slabs that grad_gather sums in a fixed order —
// deterministic, no float atomics (SURVEY §7.4 hard part 2).
#include "kernels.h"
#include "mlp_core.h"

namespace {

template <int DT>
__global__ __launch_bounds__(256) void wgrad_reg_kernel(WgradArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  using Frag = typename P::Frag;
  const WgradTask tk = a.tasks[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const T* g = reinterpret_cast<const T*>(a.gT[tk.layer]);
  const T* x = reinterpret_cast<const T*>(a.xT[tk.layer]);
  // operands are fragment-major (FM): the fragment of (row tile, k-step) is 512 contiguous
  // elements, so each of the 8 loads per k-step is one contiguous 1 KiB wave read
  const size_t blk_row = (size_t)(a.ld >> 5) * 512;  // elements per 16-row block-row
  const T* gp = g + fm_frag((tk.n0 + wn * 64) >> 4, tk.m0 >> 5, a.ld, lane);
  const T* xp = x + fm_frag((tk.k0 + wk * 64) >> 4, tk.m0 >> 5, a.ld, lane);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Two register slots in ping-pong, the loop unrolled by two so each slot keeps fixed
  // registers (no copies).  Every prefetch is unconditional (clamped to the last step; its
  // data unused) and every MFMA in the loop is unconditional, so the number of loads in flight
  // is path-independent and the compiler's waits stay partial (vmcnt(8): the next step's loads
  // remain in flight while this step's MFMAs run).  The copy-rotation form this replaces
  // drained vmcnt(0) at the top of every step.
  const int nk = (tk.m1 - tk.m0) >> 5;
  struct Slot { Frag a[4], b[4]; };
  auto fetch = [&](Slot& d, int k) {
    const size_t ko = (size_t)min(k, nk - 1) * 512;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      d.a[i] = P::load(gp + i * blk_row + ko);
      d.b[i] = P::load(xp + i * blk_row + ko);
    }
  };
  auto mma = [&](const Slot& c) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = P::mma(acc[i][j], c.a[i], c.b[j]);
  };
  // the host plan makes every chunk a multiple of 64 rows (two steps; checked in bindings.cpp)
  Slot r0, r1;
  fetch(r0, 0);
  // sched_barrier pins the order "issue next step's loads, then this step's MFMAs" (the
  // scheduler otherwise sinks each load next to its first use, which serialises on latency)
  for (int k = 0; k < nk; k += 2) {
    fetch(r1, k + 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(r0);
    __builtin_amdgcn_sched_barrier(0);
    fetch(r0, k + 2);
    __builtin_amdgcn_sched_barrier(0);
    mma(r1);
    __builtin_amdgcn_sched_barrier(0);
  }
  const int lr = lane & 15;
  float* out = a.slab + tk.slab;
  const int col = wk * 64 + lr;
  const int rbase = wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) out[(rbase + 16 * i + q) * WGRAD_TILE + col + 16 * j] = acc[i][j][q];
}

// ---- LDS-DMA staged variant (default) ----------------------------------------------------
// The register-streamed kernel above is L2->CU bandwidth bound: each of the 4 waves loads its
// own 64-row A and B fragments, so the WG moves 32 KiB per k-step for 16 KiB of distinct data
// (measured ~11 TB/s of L2->CU traffic, near the ~34 TB/s chip ceiling at its occupancy).
// Here the WG stages each k-step's 16 distinct fragments (8 of dY^T, 8 of X^T, 1 KiB each at
// bf16) ONCE into LDS with global_load_lds_dwordx4: an FM fragment is 64 lanes x 16 B in lane
// order, exactly the lane-linear image glds writes, so each fragment is one DMA instruction and
// the fragment reads are conflict-free ds_read_b128 at lane*16.  WG_STAGES-deep ring, counted
// vmcnt and a raw s_barrier keep WG_STAGES-1 steps of DMA in flight across the barrier
// (cdna_hip_programming.md 'Pipelining across barriers'): no VGPRs hold in-flight data.
template <int DT> struct WgStages { static constexpr int S = (DT == DT_F32) ? 3 : 4; };

template <int DT>
constexpr int wgrad_frag_bytes() { return 512 * Prec<DT>::BYTES; }
template <int DT>
constexpr size_t wgrad_lds_bytes() { return (size_t)WgStages<DT>::S * 16 * wgrad_frag_bytes<DT>(); }

DEV void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 |
// lgkmcnt[11:8]=15 | vmcnt[5:4] in [15:14])
#define WAIT_VMCNT(n) __builtin_amdgcn_s_waitcnt((((n) & 15) | (7 << 4) | (15 << 8) | ((((n) >> 4) & 3) << 14)))

template <int DT>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  using Frag = typename P::Frag;
  constexpr int S = WgStages<DT>::S;
  constexpr int FB = wgrad_frag_bytes<DT>();     // bytes per fragment
  constexpr int NI = FB / 1024;                  // glds instructions per fragment (64 lanes x 16 B)
  constexpr int SB = 16 * FB;                    // bytes per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];   // the kernel's ONLY LDS object
  const WgradTask tk = a.tasks[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 1, wk = wave & 1;
  const char* g = reinterpret_cast<const char*>(a.gT[tk.layer]);
  const char* x = reinterpret_cast<const char*>(a.xT[tk.layer]);
  const int nk = (tk.m1 - tk.m0) >> 5;
  const int ks0 = tk.m0 >> 5;
  // fragment f of a stage: f < 8 -> dY^T row tile n0/16 + f, else X^T row tile k0/16 + f - 8.
  // Wave w DMAs fragments 4w .. 4w+3 of every stage.
  const char* src[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = wave * 4 + q;
    src[q] = (f < 8) ? g + fm_frag((tk.n0 >> 4) + f, ks0, a.ld, 0) * sizeof(T)
                     : x + fm_frag((tk.k0 >> 4) + f - 8, ks0, a.ld, 0) * sizeof(T);
  }
  auto issue = [&](int k) {
    const int kk = min(k, nk - 1);            // past the end: re-load valid data (count stays fixed)
    char* st = smem + (k % S) * SB;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int h = 0; h < NI; ++h)
        glds16(src[q] + (size_t)kk * FB + h * 1024 + lane * 16, st + (wave * 4 + q) * FB + h * 1024);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  for (int k = 0; k < nk; ++k) {
    WAIT_VMCNT(4 * NI * (S - 2));             // this wave's part of stage k has landed
    __builtin_amdgcn_s_barrier();              // ... everyone's; and stage k-1 is no longer read
    issue(k + S - 1);                          // refill the slot stage k-1 used
    const char* st = smem + (k % S) * SB;
    Frag af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i] = P::load(reinterpret_cast<const T*>(st + (wn * 4 + i) * FB) + lane * 8);
      bf[i] = P::load(reinterpret_cast<const T*>(st + (8 + wk * 4 + i) * FB) + lane * 8);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = P::mma(acc[i][j], af[i], bf[j]);
  }
  WAIT_VMCNT(0);                               // no DMA may outlive the workgroup's LDS
  float* out = a.slab + tk.slab;
  const int col = wk * 64 + (lane & 15);
  const int rbase = wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) out[(rbase + 16 * i + q) * WGRAD_TILE + col + 16 * j] = acc[i][j][q];
}

// With the partials pass (nred = A + 8 > 0):
//   Workgroups [0, A): grad[j] = scale * sum_b part[b*npart + 8 + j]  (log_std, one WG per dim,
//                      strided partial sums + LDS tree: fixed order, deterministic)
//   Workgroups [A, A+8): loss_out[q] = sum_b part[b*npart + q] (loss-term sums for logging).
// Workgroups [nred, grid): grad[i] = scale * sum_c slab[c*stride + src_off[i]], i in [i_lo, i_hi)
//                    (fixed chunk order: deterministic; no float atomics anywhere).  A bucketed
//                    gradient (all-reduce of one flat range overlapping the next range's wgrad)
//                    gathers each range with its own launch.
__global__ __launch_bounds__(256) void grad_gather_kernel(const float* __restrict__ slab,
                                                          const int* __restrict__ src_off, int nchunks,
                                                          int stride, const float* __restrict__ part,
                                                          int nblk, int npart, int A, float scale,
                                                          float* __restrict__ grad, int i_lo, int i_hi,
                                                          int nred, float* __restrict__ loss_out) {
  if ((int)blockIdx.x < nred) {
    __shared__ float red[256];
    const int j = blockIdx.x;
    const int col = j < A ? 8 + j : j - A;
    float s = 0.f;
    for (int b = threadIdx.x; b < nblk; b += 256) s += part[(size_t)b * npart + col];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (j < A) grad[j] = red[0] * scale;
      else loss_out[j - A] = red[0];
    }
    return;
  }
  const int nb = gridDim.x - nred;
  for (int i = i_lo + (blockIdx.x - nred) * 256 + threadIdx.x; i < i_hi; i += nb * 256) {
    const int o = src_off[i];
    float s = 0.f;
    for (int c = 0; c < nchunks; ++c) s += slab[(size_t)c * stride + o];
    grad[i] = s * scale;
  }
}

}  // namespace

extern "C" void launch_wgrad(int dt, const WgradArgs& a, hipStream_t s) {
  if (a.ntasks <= 0) return;
  if (a.impl == 1) {
    if (dt == DT_F32) hipLaunchKernelGGL(wgrad_reg_kernel<DT_F32>, dim3(a.ntasks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(wgrad_reg_kernel<DT_BF16>, dim3(a.ntasks), dim3(256), 0, s, a);
  } else if (dt == DT_F32) {
    const size_t lds = wgrad_lds_bytes<DT_F32>();
    set_max_lds_once<wgrad_kernel<DT_F32>>(lds);
    hipLaunchKernelGGL(wgrad_kernel<DT_F32>, dim3(a.ntasks), dim3(256), lds, s, a);
  } else {
    const size_t lds = wgrad_lds_bytes<DT_BF16>();
    set_max_lds_once<wgrad_kernel<DT_BF16>>(lds);
    hipLaunchKernelGGL(wgrad_kernel<DT_BF16>, dim3(a.ntasks), dim3(256), lds, s, a);
  }
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_grad_gather(const float* slab, const int* src_off, int nchunks, int chunk_stride,
                                   const float* part, int nblk, int npart, int A, float scale, float* grad,
                                   int i_lo, int i_hi, int with_partials, float* loss_out, hipStream_t s) {
  int grid = (i_hi - i_lo + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  const int nred = with_partials ? A + 8 : 0;
  grid += nred;
  hipLaunchKernelGGL(grad_gather_kernel, dim3(grid), dim3(256), 0, s, slab, src_off, nchunks, chunk_stride,
                     part, nblk, npart, A, scale, grad, i_lo, i_hi, nred, loss_out);
  HIP_CHECK_LAUNCH();
}
