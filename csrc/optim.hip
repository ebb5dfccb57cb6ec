// GAE scan and fused Adam + global-norm clip + weight-image refresh (K12, K16).
#include <stdio.h>

#include "adam_core.h"
#include "kernels.h"
#include "mlp_core.h"

namespace {

// One lane per env, reverse recurrence over T (train.py:117-122):
//   delta_t = r_t + gamma*V_{t+1}*(1-d_t) - V_t ;  A_t = delta_t + gamma*lam*(1-d_t)*A_{t+1}
// [T][E] layout: lanes of a wave read consecutive envs -> coalesced.
// 64-thread workgroups (E/64 of them, spread over more CUs than E/256), and the loads of 8
// steps are issued before their part of the recurrence (same arithmetic in the same order): the
// step-at-a-time loop was a chain of T dependent load round trips per lane.
// seg > 0: the reference's segment length num_steps (train.py:82-106): a segment ends at a done
// or after seg steps, and the next one starts fresh — so after the last done t_d before t the
// segments are [t_d+1, t_d+1+seg), ...  A segment that ends by length without a done restarts the
// recursion (A_{t+1} masked) while the not-done bootstrap V_{t+1} stays in delta.  The cut flags
// depend on the dones BEFORE t, so a forward pass over the env's dones writes them into adv (as
// scratch: each element is read back by the same thread before the reverse pass overwrites it).
DEV bool seg_cut(int t, int td, int seg, float d) { return d == 0.f && (t - td) % seg == 0; }
__global__ __launch_bounds__(64) void gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                 const float* __restrict__ done, float* __restrict__ adv,
                                                 float* __restrict__ ret, int T, int E, float gamma, float lam,
                                                 int seg) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  if (e >= E) return;
  if (seg > 0) {
    int td = -1;
    for (int t = 0; t < T; ++t) {
      const size_t o = (size_t)t * E + e;
      const float d = done[o];
      adv[o] = seg_cut(t, td, seg, d) ? 0.f : 1.f;   // continuation factor of A_{t+1}
      if (d != 0.f) td = t;
    }
  }
  float nxt = 0.f;
  float vnext = val[(size_t)T * E + e];
  auto step = [&](size_t o, float r, float v, float d, float cont) {
    const float nt = 1.f - d;
    const float delta = r + gamma * vnext * nt - v;
    nxt = delta + gamma * lam * nt * cont * nxt;
    adv[o] = nxt;
    ret[o] = nxt + v;
    vnext = v;
  };
  int t = T - 1;
  for (; t >= 7; t -= 8) {
    float r[8], v[8], d[8], c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const size_t o = (size_t)(t - k) * E + e;
      r[k] = rew[o];
      v[k] = val[o];
      d[k] = done[o];
      c[k] = seg > 0 ? adv[o] : 1.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) step((size_t)(t - k) * E + e, r[k], v[k], d[k], c[k]);
  }
  for (; t >= 0; --t) {
    const size_t o = (size_t)t * E + e;
    step(o, rew[o], val[o], done[o], seg > 0 ? adv[o] : 1.f);
  }
}

// Parallel-in-time GAE for few envs and long rollouts (T >> E, e.g. ppo.py: 1 env x 2048 steps),
// SURVEY K9.  The recurrence A_t = delta_t + c_t * A_{t+1}, c_t = gamma*lam*(1-d_t), is a chain
// of affine maps x -> delta_t + c_t x; composition is associative:
//   (D1, C1) o (D2, C2) = (D1 + C1*D2, C1*C2).
// One workgroup per env: thread j composes the maps of its contiguous chunk of steps, a reverse
// exclusive scan over the 256 chunk maps (in LDS, Hillis-Steele) gives each chunk its incoming
// A_{t1}, and every thread replays its chunk to write adv / ret.  Same arithmetic per step as
// gae_kernel; only the association of the products differs (fp32 rounding-level).
__global__ __launch_bounds__(256) void gae_scan_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                       const float* __restrict__ done, float* __restrict__ adv,
                                                       float* __restrict__ ret, int T, int E, float gamma,
                                                       float lam, int seg) {
  __shared__ float sD[256], sC[256];
  __shared__ int sT[256];
  const int e = blockIdx.x, j = threadIdx.x;
  const int chunk = (T + 255) / 256;
  const int t0 = min(T, j * chunk), t1 = min(T, t0 + chunk);
  if (seg > 0) {
    // the last done before this chunk: an exclusive max-scan of the chunks' last dones, then a
    // forward pass over the chunk writes its cut flags into adv (scratch, see seg_cut)
    int last = -1;
    for (int t = t0; t < t1; ++t)
      if (done[(size_t)t * E + e] != 0.f) last = t;
    sT[j] = last;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      const int o = j >= off ? sT[j - off] : -1;
      __syncthreads();
      sT[j] = max(sT[j], o);
      __syncthreads();
    }
    int td = j > 0 ? sT[j - 1] : -1;
    for (int t = t0; t < t1; ++t) {
      const size_t o = (size_t)t * E + e;
      const float d = done[o];
      adv[o] = seg_cut(t, td, seg, d) ? 0.f : 1.f;
      if (d != 0.f) td = t;
    }
  }
  auto delta_c = [&](int t, float& delta, float& c) {
    const size_t o = (size_t)t * E + e;
    const float nt = 1.f - done[o];
    delta = rew[o] + gamma * val[o + E] * nt - val[o];
    c = gamma * lam * nt * (seg > 0 ? adv[o] : 1.f);
  };
  float D = 0.f, C = 1.f;
  for (int t = t1 - 1; t >= t0; --t) {
    float d, c;
    delta_c(t, d, c);
    D = d + c * D;
    C = c * C;
  }
  sD[j] = D;
  sC[j] = C;
  __syncthreads();
  // inclusive scan from the right: after it, (sD[j], sC[j]) = map_j o map_{j+1} o ... o map_255
  for (int off = 1; off < 256; off <<= 1) {
    float d2 = 0.f, c2 = 1.f;
    const bool has = j + off < 256;
    if (has) { d2 = sD[j + off]; c2 = sC[j + off]; }
    __syncthreads();
    if (has) {
      sD[j] = sD[j] + sC[j] * d2;
      sC[j] = sC[j] * c2;
    }
    __syncthreads();
  }
  // A at the end of this chunk = (maps of chunks j+1..255) applied to A_T = 0
  float a = (j + 1 < 256) ? sD[j + 1] : 0.f;
  for (int t = t1 - 1; t >= t0; --t) {
    float d, c;
    delta_c(t, d, c);
    a = d + c * a;
    const size_t o = (size_t)t * E + e;
    adv[o] = a;
    ret[o] = a + val[o];
  }
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, int n, float* __restrict__ part,
                                                    float* __restrict__ state) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) s += g[i] * g[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x] = red[0];
    if (blockIdx.x == 0) state[1] = state[0] + 1.f;  // staged step counter (graph-replay safe)
  }
}

template <int DT>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int n, float lr,
                                                   float b1, float b2, float eps, float max_norm,
                                                   float* __restrict__ state, const float* __restrict__ part,
                                                   int nblk, typename Prec<DT>::T* __restrict__ wimg,
                                                   const int* __restrict__ w_map, const int* __restrict__ wt_map,
                                                   const float* __restrict__ qmul, F8Shadow f8) {
  using P = Prec<DT>;
  __shared__ float red[256];
  float s = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) s += part[b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float norm = sqrtf(red[0]);
  float coef = 1.f;
  if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
  const float step = state[1];
  const float bc1 = 1.f - powf(b1, step);
  const float bc2 = 1.f - powf(b2, step);
  const float step_size = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    float mi = m[i], vi = v[i];
    const float pi = adam_elem(mi, vi, p[i], g[i] * coef, b1, b2, step_size, rbc2, eps);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    const int wi = w_map[i];
    if (wi >= 0) {
      const float q = qmul ? pi * qmul[i] : pi;
      const int wti = wt_map[i];   // -1: no transposed image (first layer of a head)
      P::put(wimg, wi, q);
      if (wti >= 0) P::put(wimg, wti, q);
      f8_put(f8, i, wi, wti, pi);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    state[0] = step;
    state[2] = norm;
  }
}

// No-clip Adam (the DPPO preset: chief.py:17 has no clipping): no norm is needed before the
// update, so there is no sumsq pass; each block leaves the partial sum of squares of the
// gradient it consumed in norm_part (fixed-order block tree), which metrics_pack sums once per
// iteration for the reported gradient norm.  The step number comes from the host (eager
// launches); block 0 mirrors it into state[0] for the device-counter path.  Graph replay keeps
// the sumsq + adam pair, whose step counter lives on the device.
template <int DT>
__global__ __launch_bounds__(256) void adam_noclip_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v, int n,
                                                          float lr, float b1, float b2, float eps, float step,
                                                          float* __restrict__ state, float* __restrict__ norm_part,
                                                          typename Prec<DT>::T* __restrict__ wimg,
                                                          const int* __restrict__ w_map,
                                                          const int* __restrict__ wt_map,
                                                          const float* __restrict__ qmul, F8Shadow f8) {
  using P = Prec<DT>;
  const float bc1 = 1.f - powf(b1, step);
  const float bc2 = 1.f - powf(b2, step);
  const float step_size = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  float ss = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    float mi = m[i], vi = v[i];
    const float gi = g[i];
    ss = fmaf(gi, gi, ss);
    const float pi = adam_elem(mi, vi, p[i], gi, b1, b2, step_size, rbc2, eps);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    const int wi = w_map[i];
    if (wi >= 0) {
      const float q = qmul ? pi * qmul[i] : pi;
      const int wti = wt_map[i];   // -1: no transposed image (first layer of a head)
      P::put(wimg, wi, q);
      if (wti >= 0) P::put(wimg, wti, q);
      f8_put(f8, i, wi, wti, pi);
    }
  }
  __shared__ float red[256];
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) norm_part[blockIdx.x] = red[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    state[0] = step;
    state[1] = step;
  }
}

// Gradient gather + no-clip Adam in ONE launch (world size 1: no all-reduce sits between the
// two, SURVEY K11+K12).  Element i's gradient is formed exactly as grad_gather_kernel forms it
// (same fixed chunk order, same scale) and handed straight to adam_elem, so the parameters are
// bit-identical to the grad_gather -> adam_noclip pair; the gradient is still written to g (the
// metrics fallback reads it).  Grid = norm_part size: blocks [0, ceil(nitems / 64)) reduce the
// partial-row columns of the reduce items (log_std, the loss terms, the per-head kernels' fused
// narrow-layer weight gradients; item_reduce) and update their parameters; the rest grid-stride
// over the slab elements of [i_lo, n) — the range may be one head's slice of the flat vectors
// (runtime/engine_hip.py).  Every block leaves its sum of squares in norm_part.
template <int DT>
__global__ __launch_bounds__(256) void gather_adam_kernel(
    const float* __restrict__ slab, const int* __restrict__ src_off, const int* __restrict__ src_meta,
    const float* __restrict__ part, int npblk, int npart, const int* __restrict__ red_col,
    const int* __restrict__ red_dst, int nitems, SlabRuns runs, float scale, float* __restrict__ loss_out,
    float* __restrict__ g, float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, int n, float lr,
    float b1, float b2, float eps, float step, float* __restrict__ state, float* __restrict__ norm_part,
    typename Prec<DT>::T* __restrict__ wimg, const int* __restrict__ w_map, const int* __restrict__ wt_map,
    const float* __restrict__ qmul, F8Shadow f8) {
  using P = Prec<DT>;
  __shared__ float red[256];
  const float bc1 = 1.f - powf(b1, step);
  const float bc2 = 1.f - powf(b2, step);
  const float step_size = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  const int nrb = item_blocks(nitems);   // reduce blocks
  float ss = 0.f;
  // the optimizer-state loads are issued before the gradient is formed (they do not depend on
  // it), so their latency overlaps the slab loads'
  auto update = [&](int i, float gi, float mi, float vi, float pv, int wi, int wti) {
    adam_apply<DT>(i, gi, mi, vi, pv, wi, wti, g, p, m, v, b1, b2, step_size, rbc2, eps, wimg, qmul, f8);
  };
  if ((int)blockIdx.x < nrb) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      state[0] = step;
      state[1] = step;
    }
    float tot = 0.f;
    int j;
    // the item's optimizer state, loaded before the column sums (its latency overlaps theirs)
    const int jj = ITEM_IPB * (int)blockIdx.x + (int)threadIdx.x;
    int d = -1, wi = 0, wti = 0;
    float mi = 0.f, vi = 0.f, pv = 0.f;
    if ((int)threadIdx.x < ITEM_IPB && jj < nitems) {
      d = red_dst[jj];
      if (d >= 0) {
        mi = m[d];
        vi = v[d];
        pv = p[d];
        wi = w_map[d];
        wti = wt_map[d];
      }
    }
    if (item_reduce(part, npblk, npart, red_col, nitems, blockIdx.x, red, tot, j)) {
      if (d >= 0) {
        const float gi = tot * scale;
        update(d, gi, mi, vi, pv, wi, wti);
        ss = gi * gi;
      } else {
        loss_out[-1 - d] = tot;
      }
    }
    __syncthreads();
    red[threadIdx.x] = threadIdx.x < ITEM_IPB ? ss : 0.f;
    __syncthreads();
    for (int w = 32; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) norm_part[blockIdx.x] = red[0];
    return;
  }
  const int nb = gridDim.x - nrb;
  for (int j = (blockIdx.x - nrb) * 256 + threadIdx.x; j < runs.total; j += nb * 256) {
    // no data-dependent branch: every per-element load issues in one round trip, then the slab
    // chunk loads (their addresses need src_off)
    const int i = runs.flat(j);
    const int mt = src_meta[i];
    const int o = src_off[i];
    const float mi = m[i], vi = v[i], pv = p[i];
    const int wi = w_map[i], wti = wt_map[i];
    const int nch = mt >> 5;
    const size_t st = (size_t)(mt & 31) << 12;
    const float s = slab_sum(slab + o, nch, st);
    const float gi = s * scale;
    ss = fmaf(gi, gi, ss);
    update(i, gi, mi, vi, pv, wi, wti);
  }
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) norm_part[blockIdx.x] = red[0];
}

template <int DT>
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ p, int n,
                                                   typename Prec<DT>::T* __restrict__ wimg,
                                                   const int* __restrict__ w_map, const int* __restrict__ wt_map,
                                                   const float* __restrict__ qmul) {
  using P = Prec<DT>;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int wi = w_map[i];
    if (wi >= 0) {
      const float q = qmul ? p[i] * qmul[i] : p[i];
      P::put(wimg, wi, q);
      if (wt_map[i] >= 0) P::put(wimg, wt_map[i], q);
    }
  }
}

// fp8 forward image refresh (dtype fp8), step 1: per-block, per-layer amax of the fp32 master
// weights -> part[block][6] (max is order-independent: no atomics).  Step 2 (pack_fp8_kernel):
// every block folds the partials into qscale[l] = amax_l / 416 (e4m3's largest finite value is
// 448: ~7 % headroom) and quantises its elements with it.  Two launches replace ~20 small torch
// ops per iteration (~200 us host-bound back to back).
constexpr int FP8_AMAX_BLOCKS = 128;

__global__ __launch_bounds__(256) void fp8_amax_kernel(const float* __restrict__ p, const int* __restrict__ lid,
                                                        int n, float* __restrict__ part) {
  float m[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int l = lid[i];
    const float a = fabsf(p[i]);
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if (l == k) m[k] = fmaxf(m[k], a);
  }
  __shared__ float red[4][6];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    float v = m[k];
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    if (lane == 0) red[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 6)
    part[blockIdx.x * 6 + threadIdx.x] =
        fmaxf(fmaxf(red[0][threadIdx.x], red[1][threadIdx.x]), fmaxf(red[2][threadIdx.x], red[3][threadIdx.x]));
}

// step 2: e4m3 images of every weight with its layer's scale (x / qscale[l]); kernels multiply
// the accumulator by qscale[l].  IEEE divisions (__fdiv_rn): the tests compare with torch.
__global__ __launch_bounds__(256) void pack_fp8_kernel(const float* __restrict__ p, int n, uint8_t* __restrict__ wimg,
                                                        const int* __restrict__ w_map, const int* __restrict__ wt_map,
                                                        const int* __restrict__ lid, const float* __restrict__ part,
                                                        int npart, float* __restrict__ qscale) {
  using P = Prec<DT_FP8>;
  __shared__ float sc[6];
  __shared__ float red[6][32];
  // fold the npart x 6 block maxima: 32 lanes per layer stride the blocks (independent loads in
  // flight), then one lane per layer folds its 32 (max: order-independent)
  if (threadIdx.x < 6 * 32) {
    const int l = threadIdx.x >> 5, k = threadIdx.x & 31;
    float v = 0.f;
    for (int b = k; b < npart; b += 32) v = fmaxf(v, part[b * 6 + l]);
    red[l][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) v = fmaxf(v, red[threadIdx.x][k]);
    sc[threadIdx.x] = fmaxf(__fdiv_rn(v, 416.f), 1e-12f);
    if (blockIdx.x == 0) qscale[threadIdx.x] = sc[threadIdx.x];
  }
  __syncthreads();
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int wi = w_map[i];
    if (wi >= 0) {
      const float q = __fdiv_rn(p[i], sc[lid[i]]);
      P::put(wimg, wi, q);
      if (wt_map[i] >= 0) P::put(wimg, wt_map[i], q);
    }
  }
}

}  // namespace

extern "C" void launch_fp8_refresh(const float* p, const int* lid, int n, float* qscale, float* part, void* wimg,
                                   const int* w_map, const int* wt_map, hipStream_t s) {
  hipLaunchKernelGGL(fp8_amax_kernel, dim3(FP8_AMAX_BLOCKS), dim3(256), 0, s, p, lid, n, part);
  HIP_CHECK_LAUNCH();
  int grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(pack_fp8_kernel, dim3(grid), dim3(256), 0, s, p, n, (uint8_t*)wimg, w_map, wt_map, lid, part,
                     FP8_AMAX_BLOCKS, qscale);
  HIP_CHECK_LAUNCH();
}

// Per-iteration metric staging in ONE launch (replaces ~6 small torch ops at the iteration tail):
// out[0..1] = episode (return sum, count), out[2..9] = the 8 loss-term sums of the last
// minibatch, out[10] = L2 norm of the last gradient, from the per-block sums of squares every
// Adam path leaves in norm_part (fixed order: deterministic).
__global__ __launch_bounds__(256) void metrics_pack_kernel(const double* __restrict__ ep,
                                                           const float* __restrict__ loss8,
                                                           const float* __restrict__ norm_part, int nblk,
                                                           double* __restrict__ out) {
  __shared__ double red[256];
  const int t = threadIdx.x;
  double s = 0.0;
  for (int b = t; b < nblk; b += 256) s += (double)norm_part[b];
  red[t] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) out[10] = sqrt(red[0]);
  if (t < 2) out[t] = ep[t];
  if (t < 8) out[2 + t] = (double)loss8[t];
}

namespace {
hipError_t g_err = hipSuccess;
char g_err_where[160];
}  // namespace

extern "C" void dppo_note_error(hipError_t e, const char* file, int line) {
  if (g_err != hipSuccess) return;   // keep the first one
  g_err = e;
  snprintf(g_err_where, sizeof(g_err_where), "%s at %s:%d", hipGetErrorString(e), file, line);
}

extern "C" int dppo_take_error(char* msg, int cap) {
  const int code = (int)g_err;
  if (code != 0 && msg != nullptr && cap > 0) snprintf(msg, (size_t)cap, "%s", g_err_where);
  g_err = hipSuccess;
  return code;
}

// test hook (tests/test_gpu_kernels.py): a launch the runtime refuses (2048-thread workgroup,
// the limit is 1024) — nothing reaches the GPU; exercises the launch-error channel end to end
__global__ void noop_kernel() {}

extern "C" void launch_debug_invalid(double* out, hipStream_t s) {
  (void)out;
  hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(2048), 0, s);   // empty body: nothing to fault
  HIP_CHECK_LAUNCH();
}

// DIAGNOSTIC (scripts/probe_side_kernel.py): a stand-in for an RCCL all-reduce kernel's CU
// footprint — nblk workgroups of nthreads with lds bytes of LDS, each spinning until the 100 MHz
// real-time counter has advanced `ticks` since ITS OWN start (so a workgroup that waits for a CU
// still runs its full time once admitted) — to see whether a collective launched on a side stream
// gets CUs while the update kernels hold them (docs/ARCHITECTURE.md §13).  Every wave exits after
// its bounded spin.
__global__ void probe_spin_kernel(unsigned long long ticks, int* __restrict__ sink) {
  extern __shared__ int probe_lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  int n = 0;
  while (t - t0 < ticks && n < (1 << 24)) {
    __builtin_amdgcn_s_sleep(2);
    t = __builtin_amdgcn_s_memrealtime();
    ++n;
  }
  probe_lds[threadIdx.x] = n;
  if (threadIdx.x == 0 && n < 0) sink[blockIdx.x] = probe_lds[0];   // (never: keeps the loop)
}

extern "C" void launch_probe_spin(int nblk, int nthreads, int lds, double us, int* sink, hipStream_t s) {
  const unsigned long long ticks = (unsigned long long)(us * 100.0);   // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(probe_spin_kernel, dim3(nblk), dim3(nthreads), (size_t)lds, s, ticks, sink);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_metrics_pack(const double* ep, const float* loss8, const float* norm_part, int nblk,
                                    double* out, hipStream_t s) {
  hipLaunchKernelGGL(metrics_pack_kernel, dim3(1), dim3(256), 0, s, ep, loss8, norm_part, nblk, out);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_gae(const float* rewards, const float* values, const float* dones, float* adv, float* ret,
                           int T, int E, float gamma, float lam, int mode, int seg, hipStream_t s) {
  // mode 0 = auto: the per-env lane scan keeps >= 1 full wave busy per env batch; with few envs
  // and a long horizon its single dependent chain per lane is the latency, so scan in time.
  const bool scan = mode == 2 || (mode == 0 && E <= 64 && T >= 512);
  if (scan)
    hipLaunchKernelGGL(gae_scan_kernel, dim3(E), dim3(256), 0, s, rewards, values, dones, adv, ret, T, E, gamma, lam,
                       seg);
  else
    hipLaunchKernelGGL(gae_kernel, dim3((E + 63) / 64), dim3(64), 0, s, rewards, values, dones, adv, ret, T, E,
                       gamma, lam, seg);
  HIP_CHECK_LAUNCH();
}

static int g_adam_fused = 1;   // A/B switch (set_adam_fused): 0 forces the sumsq + adam pair
extern "C" void set_adam_fused(int on) { g_adam_fused = on; }

extern "C" void launch_adam(float* p, const float* g, float* m, float* v, int n, float lr, float b1, float b2,
                            float eps, float max_norm, float* state, float* norm_part, int nblk, void* wimg,
                            const int* w_map, const int* wt_map, int dt, const float* img_scale, int host_step,
                            const F8Shadow& f8, hipStream_t s) {
  if (max_norm <= 0.f && g_adam_fused && host_step > 0) {
    const float step = (float)host_step;
    if (dt == DT_F32)
      hipLaunchKernelGGL(adam_noclip_kernel<DT_F32>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps,
                         step, state, norm_part, (float*)wimg, w_map, wt_map, img_scale, f8);
    else if (dt == DT_BF16)
      hipLaunchKernelGGL(adam_noclip_kernel<DT_BF16>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps,
                         step, state, norm_part, (__bf16*)wimg, w_map, wt_map, img_scale, f8);
    else if (dt == DT_S3)
      hipLaunchKernelGGL(adam_noclip_kernel<DT_S3>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps,
                         step, state, norm_part, (S3Slot*)wimg, w_map, wt_map, img_scale, f8);
    else
      hipLaunchKernelGGL(adam_noclip_kernel<DT_FP8>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps,
                         step, state, norm_part, (uint8_t*)wimg, w_map, wt_map, img_scale, f8);
    HIP_CHECK_LAUNCH();
    return;
  }
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, s, g, n, norm_part, state);
  if (dt == DT_F32)
    hipLaunchKernelGGL(adam_kernel<DT_F32>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, max_norm,
                       state, norm_part, nblk, (float*)wimg, w_map, wt_map, img_scale, f8);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL(adam_kernel<DT_BF16>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, max_norm,
                       state, norm_part, nblk, (__bf16*)wimg, w_map, wt_map, img_scale, f8);
  else if (dt == DT_S3)
    hipLaunchKernelGGL(adam_kernel<DT_S3>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, max_norm,
                       state, norm_part, nblk, (S3Slot*)wimg, w_map, wt_map, img_scale, f8);
  else
    hipLaunchKernelGGL(adam_kernel<DT_FP8>, dim3(nblk), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, max_norm,
                       state, norm_part, nblk, (uint8_t*)wimg, w_map, wt_map, img_scale, f8);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_gather_adam(const float* slab, const int* src_off, const int* src_meta, const float* part,
                                   int npblk, int npart, const int* red_col, const int* red_dst, int nitems,
                                   const SlabRuns& runs, float scale, float* loss_out, float* g, float* p,
                                   float* m, float* v, int n, float lr, float b1, float b2, float eps, int step,
                                   float* state, float* norm_part, int nblk, void* wimg, const int* w_map,
                                   const int* wt_map, int dt, const float* img_scale, const F8Shadow& f8,
                                   hipStream_t s) {
#define GA_ARGS slab, src_off, src_meta, part, npblk, npart, red_col, red_dst, nitems, runs, scale, loss_out, g, p, m, \
                v, n, lr, b1, b2, eps, \
                (float)step, state, norm_part
  if (dt == DT_F32)
    hipLaunchKernelGGL(gather_adam_kernel<DT_F32>, dim3(nblk), dim3(256), 0, s, GA_ARGS, (float*)wimg, w_map, wt_map,
                       img_scale, f8);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL(gather_adam_kernel<DT_BF16>, dim3(nblk), dim3(256), 0, s, GA_ARGS, (__bf16*)wimg, w_map,
                       wt_map, img_scale, f8);
  else if (dt == DT_S3)
    hipLaunchKernelGGL(gather_adam_kernel<DT_S3>, dim3(nblk), dim3(256), 0, s, GA_ARGS, (S3Slot*)wimg, w_map,
                       wt_map, img_scale, f8);
  else
    hipLaunchKernelGGL(gather_adam_kernel<DT_FP8>, dim3(nblk), dim3(256), 0, s, GA_ARGS, (uint8_t*)wimg, w_map,
                       wt_map, img_scale, f8);
#undef GA_ARGS
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_pack(const float* p, int n, void* wimg, const int* w_map, const int* wt_map, int dt,
                            const float* img_scale, hipStream_t s) {
  int grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  if (dt == DT_F32)
    hipLaunchKernelGGL(pack_kernel<DT_F32>, dim3(grid), dim3(256), 0, s, p, n, (float*)wimg, w_map, wt_map, img_scale);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL(pack_kernel<DT_BF16>, dim3(grid), dim3(256), 0, s, p, n, (__bf16*)wimg, w_map, wt_map, img_scale);
  else if (dt == DT_S3)
    hipLaunchKernelGGL(pack_kernel<DT_S3>, dim3(grid), dim3(256), 0, s, p, n, (S3Slot*)wimg, w_map, wt_map, img_scale);
  else
    hipLaunchKernelGGL(pack_kernel<DT_FP8>, dim3(grid), dim3(256), 0, s, p, n, (uint8_t*)wimg, w_map, wt_map, img_scale);
  HIP_CHECK_LAUNCH();
}
