// Actor-critic forward / fused loss+backward on MFMA.
//
// mlp_value_kernel: V(x) for every buffer row (GAE input, train.py:87,109-112).
// mlp_train_kernel: ONE launch per minibatch does, per ROWS-row tile, fully on-chip:
//   gather rows by index (K10)  ->  policy head fwd (3 layers)  ->  value head fwd (3 layers)
//   -> PPO loss (corrected ppo.py:148-167, or the reference DPPO loss train.py:142-161)
//      and its gradient w.r.t. mu / log_std / v  (K11 fwd)
//   -> dgrad chain through mu/v and the two tanh layers of both heads (K11 bwd)
// Activations never leave LDS except as the feature-major (transposed) operands of the
// weight-gradient GEMM (wgrad.hip), which sums over the batch with fp32 accumulation.
// The dgrad outputs overwrite the forward activations in place: dpre = (dY W) * (1 - h^2)
// reads h and writes dpre at the same (row, col) from the same lane.
#include "kernels.h"
#include "mlp_core.h"

namespace {

constexpr float LOG_2PI_F = 1.8378770664093453f;
constexpr int NPART_FIXED = 8;

template <int DT>
DEV void load_rows(const typename Prec<DT>::T* xb, const int* idx, int row0, int m0, int nvalid,
                   int d, typename Prec<DT>::T* X, int ldx, int ROWS, int tid) {
  using T = typename Prec<DT>::T;
  constexpr int E16 = 16 / Prec<DT>::BYTES;
  const int chunks = d / E16;
  // (row, chunk) walk with one division per thread instead of one per element
  int r = tid / chunks, c = tid - r * chunks;
  const int step_r = 256 / chunks, step_c = 256 - step_r * chunks;
  while (r < ROWS) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nvalid) {
      int src = idx ? idx[m0 + r] : row0 + m0 + r;
      v = *reinterpret_cast<const uint4*>(xb + (size_t)src * d + c * E16);
    }
    *reinterpret_cast<uint4*>(X + r * ldx + c * E16) = v;
    r += step_r;
    c += step_c;
    if (c >= chunks) { c -= chunks; ++r; }
  }
}

// fp8 value forward: the observation buffer is bf16 (shared with the bf16 update); convert
// 8 elements (16 B) per item into the fp8 LDS tile.
DEV void load_rows_bf16_to_fp8(const __bf16* xb, const int* idx, int row0, int m0, int nvalid, int d,
                               uint8_t* X, int ldx, int ROWS, int tid) {
  const int chunks = d / 8;
  for (int i = tid; i < ROWS * chunks; i += 256) {
    const int r = i / chunks, c = i - r * chunks;
    uint8_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < nvalid) {
      const int src = idx ? idx[m0 + r] : row0 + m0 + r;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(xb + (size_t)src * d + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = Prec<DT_FP8>::cvt((float)v[j]);
    }
    *reinterpret_cast<uint2*>(X + r * ldx + c * 8) = *reinterpret_cast<const uint2*>(q);
  }
}

// dst^T (fragment-major, [rows][ldT]) row f, columns m0 + r  <-  tile[r][f],  f < nfeat, r < ROWS.
// One item = 8 consecutive m of one feature = one contiguous 8-element group of the FM layout.
template <int DT, int ROWS>
DEV void write_transposed(const typename Prec<DT>::T* tile, int ld, int nfeat, void* dstv, int ldT,
                          int m0, int tid) {
  using T = typename Prec<DT>::T;
  constexpr int CH = ROWS / 8;
  T* dst = reinterpret_cast<T*>(dstv);
  for (int i = tid; i < nfeat * CH; i += 256) {
    const int f = i / CH, c = i - f * CH;
    T buf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) buf[j] = tile[(c * 8 + j) * ld + f];
    T* o = dst + fm_index(f, m0 + c * 8, ldT);
    if constexpr (DT == DT_F32) {
      reinterpret_cast<uint4*>(o)[0] = reinterpret_cast<const uint4*>(buf)[0];
      reinterpret_cast<uint4*>(o)[1] = reinterpret_cast<const uint4*>(buf)[1];
    } else if constexpr (DT == DT_BF16) {
      *reinterpret_cast<uint4*>(o) = *reinterpret_cast<const uint4*>(buf);
    } else {
      *reinterpret_cast<uint2*>(o) = *reinterpret_cast<const uint2*>(buf);
    }
  }
}

// bytes of the shared region that first holds X, then H2p | H2v | DMU | DV
template <int DT, int ROWS>
__host__ __device__ size_t train_region_bytes(const MlpArgs& a) {
  using T = typename Prec<DT>::T;
  const size_t x = al16(sizeof(T) * ROWS * Lds<DT>::stride(a.d_in[0]));
  const size_t rest = al16(sizeof(T) * ROWS * Lds<DT>::stride(a.d_in[2])) +
                      al16(sizeof(T) * ROWS * Lds<DT>::stride(a.d_in[5])) +
                      al16(sizeof(T) * ROWS * Lds<DT>::stride(a.d_out[2])) +
                      al16(sizeof(T) * ROWS * Lds<DT>::stride(a.d_out[5]));
  return x > rest ? x : rest;
}

template <int DT, int ROWS>
__global__ __launch_bounds__(256) void mlp_value_kernel(MlpArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  constexpr int NW = 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * ROWS;
  const int nvalid = min(ROWS, a.M - m0);
  const int ldx = Lds<DT>::stride(a.d_in[3]);
  const int ld1 = Lds<DT>::stride(a.d_in[4]);
  const int ld2 = Lds<DT>::stride(a.d_in[5]);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  LdsCarve cv(smem);
  T* X = cv.take<T>(ROWS * ldx);
  T* H1 = cv.take<T>(ROWS * ld1);
  T* H2 = cv.take<T>(ROWS * ld2);
  float* V = cv.take<float>(ROWS);
  const T* W = reinterpret_cast<const T*>(a.W);
  if constexpr (DT == DT_FP8) {
    load_rows_bf16_to_fp8(reinterpret_cast<const __bf16*>(a.x_buf), a.idx, a.row0, m0, nvalid, a.d_in[3], X, ldx,
                          ROWS, tid);
  } else {
    load_rows<DT>(reinterpret_cast<const T*>(a.x_buf), a.idx, a.row0, m0, nvalid, a.d_in[3], X, ldx, ROWS, tid);
  }
  preset_tile<DT>(H1, ld1, ROWS, a.n_out[3], tid, 256);
  preset_tile<DT>(H2, ld2, ROWS, a.n_out[4], tid, 256);
  const float sc3 = a.qscale ? a.qscale[3] : a.scale[3];
  const float sc4 = a.qscale ? a.qscale[4] : a.scale[4];
  const float sc5 = a.qscale ? a.qscale[5] : a.scale[5];
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_TANH>(X, ldx, a.d_in[3], W + a.off_w[3], a.n_out[3], H1, ld1, sc3, wave, lane);
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_TANH>(H1, ld1, a.d_in[4], W + a.off_w[4], a.n_out[4], H2, ld2, sc4, wave, lane);
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_LINEAR_F32>(H2, ld2, a.d_in[5], W + a.off_w[5], 1, V, 1, sc5, wave, lane);
  __syncthreads();
  if (tid < nvalid) a.v_out[m0 + tid] = V[tid];
}

template <int DT, int ROWS>
__global__ __launch_bounds__(256) void mlp_train_kernel(MlpArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  constexpr int NW = 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * ROWS;
  const int nvalid = min(ROWS, a.M - m0);
  const int A = a.A;
  const int ldx = Lds<DT>::stride(a.d_in[0]);
  const int ld1p = Lds<DT>::stride(a.d_in[1]);
  const int ld2p = Lds<DT>::stride(a.d_in[2]);
  const int ld1v = Lds<DT>::stride(a.d_in[4]);
  const int ld2v = Lds<DT>::stride(a.d_in[5]);
  const int ldmu = Lds<DT>::stride(a.d_out[2]);
  const int ldv = Lds<DT>::stride(a.d_out[5]);

  // LDS plan: X is dead after the two first layers, so H2p/H2v/DMU/DV live inside X's region
  // (train_lds sizes the region as the max of the two uses) -> 2 workgroups per CU at bf16.
  extern __shared__ __attribute__((aligned(16))) char smem[];
  LdsCarve cv(smem);
  char* region = cv.base;
  cv.off = train_region_bytes<DT, ROWS>(a);
  T* X = reinterpret_cast<T*>(region);
  LdsCarve rc(region);
  T* H2p = rc.take<T>(ROWS * ld2p);
  T* H2v = rc.take<T>(ROWS * ld2v);
  T* DMU = rc.take<T>(ROWS * ldmu);
  T* DV = rc.take<T>(ROWS * ldv);
  T* H1p = cv.take<T>(ROWS * ld1p);
  T* H1v = cv.take<T>(ROWS * ld1v);
  float* MU = cv.take<float>(ROWS * A);
  float* V = cv.take<float>(ROWS);
  float* DLS = cv.take<float>(ROWS * A);
  float* LOSS = cv.take<float>(ROWS * NPART_FIXED);

  const T* W = reinterpret_cast<const T*>(a.W);
  load_rows<DT>(reinterpret_cast<const T*>(a.x_buf), a.idx, a.row0, m0, nvalid, a.d_in[0], X, ldx, ROWS, tid);
  preset_tile<DT>(H1p, ld1p, ROWS, a.n_out[0], tid, 256);
  preset_tile<DT>(H1v, ld1v, ROWS, a.n_out[3], tid, 256);
  __syncthreads();
  // ---------------- forward ----------------
  // Activations go to the feature-major wgrad operands straight from the MFMA accumulators
  // (rows < n_real; the constant-1 bias row of each buffer is preset once by the host).
  const bool no_T = (a.ablate & 1) != 0;   // diagnostics only (see MlpArgs::ablate)
  T* h1pT = no_T ? nullptr : reinterpret_cast<T*>(a.h1pT);
  T* h2pT = no_T ? nullptr : reinterpret_cast<T*>(a.h2pT);
  T* h1vT = no_T ? nullptr : reinterpret_cast<T*>(a.h1vT);
  T* h2vT = no_T ? nullptr : reinterpret_cast<T*>(a.h2vT);
  if (!a.xT_ready && !no_T) write_transposed<DT, ROWS>(X, ldx, a.d_in[0], a.xT, a.ldT, m0, tid);  // else: rollout wrote it
  layer_gemm<DT, ROWS, NW, EPI_TANH>(X, ldx, a.d_in[0], W + a.off_w[0], a.n_out[0], H1p, ld1p, a.scale[0], wave, lane,
                                     h1pT, a.ldT, m0);
  if (!(a.ablate & 2))
    layer_gemm<DT, ROWS, NW, EPI_TANH>(X, ldx, a.d_in[3], W + a.off_w[3], a.n_out[3], H1v, ld1v, a.scale[3], wave,
                                       lane, h1vT, a.ldT, m0);
  __syncthreads();
  // X is dead: preset the tiles that alias its region
  preset_tile<DT>(H2p, ld2p, ROWS, a.n_out[1], tid, 256);
  preset_tile<DT>(H2v, ld2v, ROWS, a.n_out[4], tid, 256);
  preset_tile<DT>(DMU, ldmu, ROWS, -1, tid, 256);
  preset_tile<DT>(DV, ldv, ROWS, -1, tid, 256);
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_TANH>(H1p, ld1p, a.d_in[1], W + a.off_w[1], a.n_out[1], H2p, ld2p, a.scale[1], wave, lane,
                                     h2pT, a.ldT, m0);
  layer_gemm<DT, ROWS, NW, EPI_TANH>(H1v, ld1v, a.d_in[4], W + a.off_w[4], a.n_out[4], H2v, ld2v, a.scale[4], wave, lane,
                                     h2vT, a.ldT, m0);
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_LINEAR_F32>(H2p, ld2p, a.d_in[2], W + a.off_w[2], A, MU, A, a.scale[2], wave, lane);
  layer_gemm<DT, ROWS, NW, EPI_LINEAR_F32>(H2v, ld2v, a.d_in[5], W + a.off_w[5], 1, V, 1, a.scale[5], wave, lane);
  __syncthreads();
  // ---------------- loss + dL/d(mu, log_std, v) per row ----------------
  if (tid < ROWS && !(a.ablate & 8)) {
    const int r = tid;
    float* lrow = LOSS + r * NPART_FIXED;
#pragma unroll
    for (int q = 0; q < NPART_FIXED; ++q) lrow[q] = 0.f;
    if (r < nvalid) {
      const int src = a.idx ? a.idx[m0 + r] : a.row0 + m0 + r;
      const float* act = a.actions + (size_t)src * A;
      const float advv = a.adv[src], retv = a.ret[src];
      const float v = V[r];
      const float cvar = a.std_var ? 0.5f : 1.f;
      float dv = 0.f, lv = 0.f, lclip = 0.f, lent = 0.f, kl = 0.f, cf = 0.f;
      float vold;
      if (a.loss_kind == 0) {
        // ---- corrected PPO (ppo.py:148-167) ----
        float logp = 0.f;
        for (int j = 0; j < A; ++j) {
          float lsig = cvar * a.log_std[j];
          float z = (act[j] - MU[r * A + j]) * __expf(-lsig);
          logp += -0.5f * z * z - 0.5f * LOG_2PI_F - lsig;
        }
        float lr = logp - a.logp_old[src];
        float ratio = __expf(lr);
        float s1 = ratio * advv;
        float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * advv;
        lclip = -fminf(s1, s2);
        float dlogp = (s1 <= s2) ? -advv * ratio : 0.f;
        kl = (ratio - 1.f) - lr;
        cf = (fabsf(ratio - 1.f) > a.clip) ? 1.f : 0.f;
        for (int j = 0; j < A; ++j) {
          float lsig = cvar * a.log_std[j];
          float isig = __expf(-lsig);
          float z = (act[j] - MU[r * A + j]) * isig;
          DMU[r * ldmu + j] = P::cvt(dlogp * z * isig);
          // d/dlog_std: logp term + entropy bonus (-ent_coeff * sum_j log sigma_j)
          DLS[r * A + j] = (dlogp * (z * z - 1.f) - a.ent_coeff) * cvar;
          lent += -a.ent_coeff * (0.5f + 0.5f * LOG_2PI_F + lsig);
        }
        vold = a.v_old[src];
      } else {
        // ---- reference DPPO loss (train.py:142-161): per-dim pdf ratio, variance convention ----
        const float invA = 1.f / (float)A;
        const bool first = a.first_step != 0;
        for (int j = 0; j < A; ++j) {
          float mu = MU[r * A + j];
          float var = __expf(a.log_std[j]);
          float mu_o = first ? mu : a.mu_prev[(size_t)src * A + j];
          float var_o = first ? var : __expf(a.log_std_old[j]);
          float x = act[j];
          float p = __expf(-(x - mu) * (x - mu) / (2.f * var)) * rsqrtf(2.f * var * 3.14159265358979f);
          float po = __expf(-(x - mu_o) * (x - mu_o) / (2.f * var_o)) * rsqrtf(2.f * var_o * 3.14159265358979f);
          float ratio = p / (1e-10f + po);
          float s1 = ratio * advv;
          float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * advv;
          lclip += -fminf(s1, s2) * invA;
          float dratio = (s1 <= s2) ? -advv * invA : 0.f;
          float dp = dratio / (1e-10f + po);
          float lg = logf(p + 1e-5f);
          lent += -a.ent_coeff * p * lg * invA;
          dp += -a.ent_coeff * invA * (lg + p / (p + 1e-5f));
          DMU[r * ldmu + j] = P::cvt(dp * p * (x - mu) / var);
          DLS[r * A + j] = dp * p * ((x - mu) * (x - mu) / (2.f * var) - 0.5f);
          cf += (fabsf(ratio - 1.f) > a.clip) ? invA : 0.f;
          a.mu_prev[(size_t)src * A + j] = mu;   // train.py:164 model_old <- model
        }
        vold = first ? v : a.v_prev[src];
        a.v_prev[src] = v;
      }
      if (a.value_loss == 0) {
        float d = v - retv;
        lv = d * d;
        dv = 2.f * d;
      } else {
        float d1 = v - retv;
        float dd = v - vold;
        float vc = vold + fminf(fmaxf(dd, -a.clip), a.clip);
        float d2 = vc - retv;
        float f1 = d1 * d1, f2 = d2 * d2;
        float inr = (dd >= -a.clip && dd <= a.clip) ? 1.f : 0.f;
        lv = 0.5f * fmaxf(f1, f2);
        if (f1 > f2) dv = d1;
        else if (f2 > f1) dv = d2 * inr;
        else dv = 0.5f * d1 + 0.5f * d2 * inr;
      }
      DV[r * ldv] = P::cvt(dv);
      lrow[0] = lclip; lrow[1] = lv; lrow[2] = lent; lrow[3] = kl; lrow[4] = cf; lrow[5] = 1.f;
    } else {
      for (int j = 0; j < A; ++j) DLS[r * A + j] = 0.f;
    }
  }
  __syncthreads();
  // ---------------- per-workgroup partials + dY^T of the output layers ----------------
  if (tid < NPART_FIXED + A) {
    float s = 0.f;
    if (tid < NPART_FIXED) for (int r = 0; r < ROWS; ++r) s += LOSS[r * NPART_FIXED + tid];
    else for (int r = 0; r < ROWS; ++r) s += DLS[r * A + (tid - NPART_FIXED)];
    a.part[(size_t)blockIdx.x * a.npart + tid] = s;
  }
  write_transposed<DT, ROWS>(DMU, ldmu, A, a.g3pT, a.ldT, m0, tid);
  write_transposed<DT, ROWS>(DV, ldv, 1, a.g3vT, a.ldT, m0, tid);
  // ---------------- dgrad chain (dY^T of every layer stored from the accumulators) --------
  if (a.ablate & 4) return;   // diagnostics only
  T* g2pT = no_T ? nullptr : reinterpret_cast<T*>(a.g2pT);
  T* g2vT = no_T ? nullptr : reinterpret_cast<T*>(a.g2vT);
  layer_gemm<DT, ROWS, NW, EPI_DTANH_INPLACE>(DMU, ldmu, a.d_out[2], W + a.off_wt[2], a.n_out[1], H2p, ld2p, a.scale[2],
                                              wave, lane, g2pT, a.ldT, m0);
  layer_gemm<DT, ROWS, NW, EPI_DTANH_INPLACE>(DV, ldv, a.d_out[5], W + a.off_wt[5], a.n_out[4], H2v, ld2v, a.scale[5],
                                              wave, lane, g2vT, a.ldT, m0);
  __syncthreads();
  // EPI_DTANH_GLOBAL's only output is the wgrad operand, so it always stores (ablation bit0
  // does not apply here or the MFMAs would be dead code)
  layer_gemm<DT, ROWS, NW, EPI_DTANH_GLOBAL>(H2p, ld2p, a.d_out[1], W + a.off_wt[1], a.n_out[0], H1p, ld1p, a.scale[1],
                                              wave, lane, reinterpret_cast<T*>(a.g1pT), a.ldT, m0);
  layer_gemm<DT, ROWS, NW, EPI_DTANH_GLOBAL>(H2v, ld2v, a.d_out[4], W + a.off_wt[4], a.n_out[3], H1v, ld1v, a.scale[4],
                                              wave, lane, reinterpret_cast<T*>(a.g1vT), a.ldT, m0);
}

template <int DT, int ROWS>
size_t train_lds(const MlpArgs& a) {
  using T = typename Prec<DT>::T;
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  auto ld = [](int d) { return (size_t)Lds<DT>::stride(d); };
  size_t b = train_region_bytes<DT, ROWS>(a);
  b += al(sizeof(T) * ROWS * ld(a.d_in[1]));
  b += al(sizeof(T) * ROWS * ld(a.d_in[4]));
  b += al(sizeof(float) * ROWS * a.A) * 2 + al(sizeof(float) * ROWS) + al(sizeof(float) * ROWS * NPART_FIXED);
  return b;
}

template <int DT, int ROWS>
size_t value_lds(const MlpArgs& a) {
  using T = typename Prec<DT>::T;
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  auto ld = [](int d) { return (size_t)Lds<DT>::stride(d); };
  return al(sizeof(T) * ROWS * ld(a.d_in[3])) + al(sizeof(T) * ROWS * ld(a.d_in[4])) +
         al(sizeof(T) * ROWS * ld(a.d_in[5])) + al(sizeof(float) * ROWS);
}

constexpr int VALUE_ROWS = 32;

template <int DT>
void train_t(const MlpArgs& a, hipStream_t s) {
  constexpr int TRAIN_ROWS = train_rows_for(DT);
  size_t lds = train_lds<DT, TRAIN_ROWS>(a);
  (void)hipFuncSetAttribute((const void*)mlp_train_kernel<DT, TRAIN_ROWS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int nblk = (a.M + TRAIN_ROWS - 1) / TRAIN_ROWS;
  hipLaunchKernelGGL((mlp_train_kernel<DT, TRAIN_ROWS>), dim3(nblk), dim3(256), lds, s, a);
  HIP_CHECK_LAUNCH();
}

template <int DT>
void value_t(const MlpArgs& a, hipStream_t s) {
  size_t lds = value_lds<DT, VALUE_ROWS>(a);
  (void)hipFuncSetAttribute((const void*)mlp_value_kernel<DT, VALUE_ROWS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int nblk = (a.M + VALUE_ROWS - 1) / VALUE_ROWS;
  hipLaunchKernelGGL((mlp_value_kernel<DT, VALUE_ROWS>), dim3(nblk), dim3(256), lds, s, a);
  HIP_CHECK_LAUNCH();
}

}  // namespace

extern "C" void launch_mlp_train(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_F32) train_t<DT_F32>(a, s);
  else if (dt == DT_BF16) train_t<DT_BF16>(a, s);
  else train_t<DT_FP8>(a, s);
}

extern "C" void launch_mlp_value(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_F32) value_t<DT_F32>(a, s);
  else if (dt == DT_BF16) value_t<DT_BF16>(a, s);
  else value_t<DT_FP8>(a, s);
}

extern "C" size_t mlp_train_lds_bytes(int dt, const MlpArgs& a) {
  if (dt == DT_F32) return train_lds<DT_F32, train_rows_for(DT_F32)>(a);
  if (dt == DT_BF16) return train_lds<DT_BF16, train_rows_for(DT_BF16)>(a);
  return train_lds<DT_FP8, train_rows_for(DT_FP8)>(a);
}
