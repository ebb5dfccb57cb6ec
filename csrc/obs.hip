// Running observation statistics on the device (reference model.py:68-75).
//
// The rollout kernel leaves per-workgroup moments about a common shift (sum(x - shift),
// sum((x - shift)^2)) for its T*ROWS samples.  Here:
//   obs_reduce : [nblk][2][O] fp32 partials -> [2][O] fp64 sums (fixed order: deterministic)
//   [RCCL all-reduce of the [2][O] fp64 sums across ranks — done by the worker]
//   obs_merge  : Chan et al. merge of the batch into (n, mean, M2) fp64 and the fp32 images
//                (mean, 1/sqrt(max(M2/n, 1e-2))) read by the normalisation prologue.
// Two launches replace ~25 small torch ops (measured ~230 us per iteration).
#include "kernels.h"
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void obs_reduce_kernel(const float* __restrict__ part, int nblk, int O,
                                                         double* __restrict__ s12) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // i in [0, 2*O): (q, d) = (i / O, i % O)
  if (i >= 2 * O) return;
  const int q = i / O, d = i - q * O;
  const float* p = part + (size_t)q * O + d;
  const size_t stride = (size_t)2 * O;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int b = 0;
  for (; b + 4 <= nblk; b += 4) {
    a0 += p[(size_t)(b + 0) * stride];
    a1 += p[(size_t)(b + 1) * stride];
    a2 += p[(size_t)(b + 2) * stride];
    a3 += p[(size_t)(b + 3) * stride];
  }
  for (; b < nblk; ++b) a0 += p[(size_t)b * stride];
  s12[i] = (a0 + a1) + (a2 + a3);
}

__global__ __launch_bounds__(256) void obs_merge_kernel(const double* __restrict__ s12, int O, double count,
                                                        double n_a, const float* __restrict__ shift,
                                                        double* __restrict__ mean, double* __restrict__ m2,
                                                        float* __restrict__ mean_f32, float* __restrict__ inv_std,
                                                        double var_floor) {
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

}  // namespace

extern "C" void launch_obs_reduce(const float* part, int nblk, int O, double* s12, hipStream_t s) {
  hipLaunchKernelGGL(obs_reduce_kernel, dim3((2 * O + 255) / 256), dim3(256), 0, s, part, nblk, O, s12);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_obs_merge(const double* s12, int O, double count, double n_a, const float* shift,
                                 double* mean, double* m2, float* mean_f32, float* inv_std, double var_floor,
                                 hipStream_t s) {
  hipLaunchKernelGGL(obs_merge_kernel, dim3((O + 255) / 256), dim3(256), 0, s, s12, O, count, n_a, shift, mean, m2,
                     mean_f32, inv_std, var_floor);
  HIP_CHECK_LAUNCH();
}
