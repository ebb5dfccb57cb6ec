// Running observation statistics on the device (reference model.py:68-75).
//
// The rollout kernel leaves per-workgroup moments about a common shift (sum(x - shift),
// sum((x - shift)^2)) for its T*ROWS samples.  Here:
//   obs_reduce : [nblk][2][O] fp32 partials -> [2][O] fp64 sums (fixed order: deterministic)
//   [RCCL all-reduce of the [2][O] fp64 sums across ranks — done by the worker]
//   obs_merge  : Chan et al. merge of the batch into (n, mean, M2) fp64 and the fp32 images
//                (mean, 1/sqrt(max(M2/n, 1e-2))) read by the normalisation prologue.
//   obs_moments: the same [nblk][2][O] partials from an [E][O] observation batch — the per-step
//                obs-norm mode (model.py:68 per observation) observes each step's batch before
//                the step's one-step rollout launch normalises it: moments -> reduce -> merge.
// Two launches replace ~25 small torch ops (measured ~230 us per iteration).
#include "kernels.h"
#include "common.h"

namespace {

// One workgroup per 64 consecutive (q, d) columns: lane = column (coalesced 256-B rows), the
// OR_WAVES waves split the blocks (b = wave, wave + OR_WAVES, ...) with 4 rows' loads in flight
// per lane, then a fixed-order LDS combine — deterministic.  Only ~13 workgroups exist (2*O/64),
// so the per-lane chain of dependent loads is the kernel's time: 16 waves x 4 loads in flight
// walk 256 blocks in 4 round trips (4 waves x 2 loads took 32: 11.6 us).
// The last workgroup also sums the per-block episode stats [nblk][2] -> ep[2] (fp64).
constexpr int OR_WAVES = 16;
__global__ __launch_bounds__(OR_WAVES * 64) void obs_reduce_kernel(const float* __restrict__ part, int nblk, int O,
                                                                   double* __restrict__ s12,
                                                                   const float* __restrict__ epstat,
                                                                   double* __restrict__ ep) {
  __shared__ double red[OR_WAVES][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ncol = 2 * O;
  const int ngrp = (ncol + 63) / 64;
  if ((int)blockIdx.x == ngrp) {   // episode stats (launched only when ep is given)
    if (wave == 0) {
      double a = 0.0, c = 0.0;
      for (int b = lane; b < nblk; b += 64) { a += epstat[2 * b]; c += epstat[2 * b + 1]; }
      red[0][lane] = a;
      red[1][lane] = c;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
      double t = 0.0;
      for (int l = 0; l < 64; ++l) t += red[threadIdx.x][l];
      ep[threadIdx.x] = t;
    }
    return;
  }
  const int i = blockIdx.x * 64 + lane;       // column i = q * O + d of the [2][O] partial
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (i < ncol) {
    const float* p = part + i;
    const size_t stride = (size_t)ncol;
    int b = wave;
    for (; b + 3 * OR_WAVES < nblk; b += 4 * OR_WAVES) {
      const float x0 = p[(size_t)b * stride], x1 = p[(size_t)(b + OR_WAVES) * stride];
      const float x2 = p[(size_t)(b + 2 * OR_WAVES) * stride], x3 = p[(size_t)(b + 3 * OR_WAVES) * stride];
      a0 += x0;
      a1 += x1;
      a2 += x2;
      a3 += x3;
    }
    for (; b < nblk; b += OR_WAVES) a0 += p[(size_t)b * stride];
  }
  red[wave][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wave == 0 && i < ncol) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < OR_WAVES; ++w) t += red[w][lane];
    s12[i] = t;
  }
}

__global__ __launch_bounds__(256) void obs_merge_kernel(const double* __restrict__ s12, int O, double count,
                                                        double n_a, const float* shift,
                                                        double* __restrict__ mean, double* __restrict__ m2,
                                                        float* mean_f32, float* __restrict__ inv_std,
                                                        double var_floor) {
  // shift may alias mean_f32 (the rollout takes its moments about the current fp32 mean):
  // each thread reads shift[d] before it writes mean_f32[d], so neither is __restrict__
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d >= O) return;
  const double s1 = s12[d], s2 = s12[O + d];
  const double bmean_d = s1 / count;
  const double bmean = (double)shift[d] + bmean_d;
  double bm2 = s2 - s1 * bmean_d;
  if (bm2 < 0.0) bm2 = 0.0;
  const double n = n_a + count;
  const double delta = bmean - mean[d];
  const double mu = mean[d] + delta * (count / n);
  const double M2 = m2[d] + bm2 + delta * delta * (n_a * count / n);
  mean[d] = mu;
  m2[d] = M2;
  double var = M2 / n;
  if (var < var_floor) var = var_floor;
  mean_f32[d] = (float)mu;
  inv_std[d] = (float)(1.0 / sqrt(var));
}

// One workgroup per OM_ROWS consecutive observations: thread = column (coalesced rows), the
// workgroup's columns in 256-wide passes, OM_ROWS rows summed in order (fp32, about the shift,
// like the rollout kernel's partials).
constexpr int OM_ROWS = 64;
__global__ __launch_bounds__(256) void obs_moments_kernel(const float* __restrict__ obs, int E, int O,
                                                          const float* __restrict__ shift, float* __restrict__ part) {
  const int r0 = blockIdx.x * OM_ROWS;
  const int r1 = min(E, r0 + OM_ROWS);
  for (int d = threadIdx.x; d < O; d += 256) {
    const float sh = shift[d];
    float s1 = 0.f, s2 = 0.f;
    for (int r = r0; r < r1; ++r) {
      const float v = obs[(size_t)r * O + d] - sh;
      s1 += v;
      s2 = fmaf(v, v, s2);
    }
    part[((size_t)blockIdx.x * 2) * O + d] = s1;
    part[((size_t)blockIdx.x * 2 + 1) * O + d] = s2;
  }
}

}  // namespace

extern "C" int obs_moments_blocks(int E) { return (E + OM_ROWS - 1) / OM_ROWS; }

extern "C" void launch_obs_moments(const float* obs, int E, int O, const float* shift, float* part, hipStream_t s) {
  hipLaunchKernelGGL(obs_moments_kernel, dim3(obs_moments_blocks(E)), dim3(256), 0, s, obs, E, O, shift, part);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_obs_reduce(const float* part, int nblk, int O, double* s12, const float* epstat, double* ep,
                                  hipStream_t s) {
  // the extra workgroup (episode stats) only when ep is given
  hipLaunchKernelGGL(obs_reduce_kernel, dim3((2 * O + 63) / 64 + (ep != nullptr ? 1 : 0)), dim3(OR_WAVES * 64), 0, s,
                     part, nblk, O, s12, epstat, ep);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_obs_merge(const double* s12, int O, double count, double n_a, const float* shift,
                                 double* mean, double* m2, float* mean_f32, float* inv_std, double var_floor,
                                 hipStream_t s) {
  hipLaunchKernelGGL(obs_merge_kernel, dim3((O + 255) / 256), dim3(256), 0, s, s12, O, count, n_a, shift, mean, m2,
                     mean_f32, inv_std, var_floor);
  HIP_CHECK_LAUNCH();
}
