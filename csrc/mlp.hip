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

// phase timeline (diagnostics): lane 0 of each wave of every tstamp_every-th workgroup records
// the shader clock at phase boundaries; one scalar branch per boundary when off
#define STAMP(i)                                                                                  \
  do {                                                                                            \
    if (a.tstamp != nullptr && (blockIdx.x % a.tstamp_every) == 0 && lane == 0)                   \
      a.tstamp[((size_t)(blockIdx.x / a.tstamp_every) * NW + wave) * 16 + (i)] =                  \
          __builtin_amdgcn_s_memtime();                                                           \
  } while (0)

// sum over the G consecutive lanes of a group (G a power of two <= 64), result in every lane
template <int G>
DEV float group_sum(float x) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, G);
  return x;
}

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// Gather ROWS rows of the [*][d] observation buffer into the LDS tile X (row stride ldx).
// Loads go out in batches of B per thread and ALL of a batch's loads are issued before any
// of its LDS stores; `between()` (LDS presets that do not depend on X) runs while the first
// batch is in flight, so the HBM latency is paid once per tile instead of once per item.
template <int DT, int NT, typename F>
DEV void load_rows(const typename Prec<DT>::T* xb, const int* idx, int row0, int m0, int nvalid,
                   int d, typename Prec<DT>::T* X, int ldx, int ROWS, int tid, F&& between, bool stream = false) {
  constexpr int E16 = 16 / Prec<DT>::BYTES;
  constexpr int B = 8;
  const int chunks = d / E16;
  // (row, chunk) walk with one division per thread instead of one per element
  int r = tid / chunks, c = tid - r * chunks;
  const int step_r = NT / chunks, step_c = NT - step_r * chunks;
  bool first = true;
  for (;;) {
    uint4 v[B];
    int off[B];
#pragma unroll
    for (int j = 0; j < B; ++j) {
      off[j] = -1;
      v[j] = make_uint4(0, 0, 0, 0);
      if (r < ROWS) {
        off[j] = r * ldx + c * E16;
        if (r < nvalid) {
          const int src = idx ? idx[m0 + r] : row0 + m0 + r;
          // plain (cached) load: the observation buffer (100 MB at split-bf16) is re-read by every
          // epoch and stays in the 256 MB Infinity Cache between them; measured at the bench
          // geometry, split-bf16 update 299 -> 269 us (the X gather fell from ~38 to ~5 us) and the
          // value forward 162 -> 147 us vs non-temporal loads; bf16 neutral (134-138 us)
          const u32x4* sp = reinterpret_cast<const u32x4*>(xb + (size_t)src * d + c * E16);
          const u32x4 t = stream ? __builtin_nontemporal_load(sp) : *sp;
          v[j] = make_uint4(t.x, t.y, t.z, t.w);
        }
      }
      r += step_r;
      c += step_c;
      if (c >= chunks) { c -= chunks; ++r; }
    }
    if (first) {
      between();
      first = false;
    }
#pragma unroll
    for (int j = 0; j < B; ++j)
      if (off[j] >= 0) *reinterpret_cast<uint4*>(X + off[j]) = v[j];
    if (r >= ROWS) break;
  }
}

// fp8 value forward: the observation buffer is bf16 (shared with the bf16 update); convert
// 8 elements (16 B) per item into the fp8 LDS tile.
template <int NT>
DEV void load_rows_bf16_to_fp8(const __bf16* xb, const int* idx, int row0, int m0, int nvalid, int d,
                               uint8_t* X, int ldx, int ROWS, int tid) {
  const int chunks = d / 8;
  for (int i = tid; i < ROWS * chunks; i += NT) {
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
template <int DT, int ROWS, int NT>
DEV void write_transposed(const typename Prec<DT>::T* tile, int ld, int nfeat, void* dstv, int ldT,
                          int m0, int tid) {
  using T = typename Prec<DT>::T;
  constexpr int CH = ROWS / 8;
  T* dst = reinterpret_cast<T*>(dstv);
  if constexpr (IsSplit<DT>::value) {
    // 8 consecutive m of feature f: their 8 hi then 8 lo bf16 values are one 32-byte FM group
    using P = Prec<DT>;
    for (int i = tid; i < nfeat * CH; i += NT) {
      const int f = i / CH, c = i - f * CH;
      bf16x8 h, l;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16* p = P::hi_ptr(tile, (c * 8 + j) * ld + f);
        h[j] = p[0];
        l[j] = p[8];
      }
      u32x4* o = reinterpret_cast<u32x4*>(P::hi_ptr(dst, fm_index(f, m0 + c * 8, ldT)));
      opnd_store(*reinterpret_cast<const u32x4*>(&h), o);
      opnd_store(*reinterpret_cast<const u32x4*>(&l), o + 1);
    }
    return;
  }
  for (int i = tid; i < nfeat * CH; i += NT) {
    const int f = i / CH, c = i - f * CH;
    T buf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) buf[j] = tile[(c * 8 + j) * ld + f];
    T* o = dst + fm_index(f, m0 + c * 8, ldT);
    if constexpr (DT == DT_F32) {
      reinterpret_cast<uint4*>(o)[0] = reinterpret_cast<const uint4*>(buf)[0];
      reinterpret_cast<uint4*>(o)[1] = reinterpret_cast<const uint4*>(buf)[1];
    } else if constexpr (DT == DT_BF16) {   // streaming store: see store4q_T
      opnd_store(*reinterpret_cast<const u32x4*>(buf), reinterpret_cast<u32x4*>(o));
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

template <int DT, int ROWS, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void mlp_value_kernel(MlpArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  constexpr int NT = NW * 64;
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
  BPre<DT, ROWS / 16> pf;   // cross-barrier weight prefetch (see mlp_train_kernel)
  layer_prefetch<DT, ROWS, NW>(pf, W + a.off_w[3], a.d_in[3], a.n_out[3], wave, lane);
  if constexpr (DT == DT_FP8) {
    load_rows_bf16_to_fp8<NT>(reinterpret_cast<const __bf16*>(a.x_buf), a.idx, a.row0, m0, nvalid, a.d_in[3], X,
                              ldx, ROWS, tid);
  } else {
    load_rows<DT, NT>(reinterpret_cast<const T*>(a.x_buf), a.idx, a.row0, m0, nvalid, a.d_in[3], X, ldx, ROWS, tid,
                      [] {}, a.x_stream != 0);
  }
  preset_pad<DT>(H1, ld1, ROWS, a.n_out[3], tid, NT);
  preset_pad<DT>(H2, ld2, ROWS, a.n_out[4], tid, NT);
  const float sc3 = a.qscale ? a.qscale[3] : a.scale[3];
  const float sc4 = a.qscale ? a.qscale[4] : a.scale[4];
  const float sc5 = a.qscale ? a.qscale[5] : a.scale[5];
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_TANH, true>(X, ldx, a.d_in[3], W + a.off_w[3], a.n_out[3], H1, ld1, sc3, wave, lane,
                                           nullptr, 0, 0, 0, &pf);
  layer_prefetch<DT, ROWS, NW>(pf, W + a.off_w[4], a.d_in[4], a.n_out[4], wave, lane);
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_TANH, true>(H1, ld1, a.d_in[4], W + a.off_w[4], a.n_out[4], H2, ld2, sc4, wave, lane,
                                           nullptr, 0, 0, 0, &pf);
  layer_prefetch<DT, ROWS, NW>(pf, W + a.off_w[5], a.d_in[5], 1, wave, lane);
  __syncthreads();
  layer_gemm<DT, ROWS, NW, EPI_LINEAR_F32, true>(H2, ld2, a.d_in[5], W + a.off_w[5], 1, V, 1, sc5, wave, lane,
                                                 nullptr, 0, 0, 0, &pf);
  __syncthreads();
  if (tid < nvalid) a.v_out[m0 + tid] = V[tid];
}

// (split-bf16 at 4 waves: the 32-row tile needs ~134 KiB of LDS at Humanoid dims, one workgroup
// per CU, so each wave may take the whole 512-VGPR budget of its SIMD instead of spilling)
template <int DT, int NW> struct TrainOcc { static constexpr int V = (DT == DT_S3 && NW == 4) ? 1 : 8 / NW; };

template <int DT, int ROWS, int NW>
__global__ __launch_bounds__(NW * 64, (TrainOcc<DT, NW>::V)) void mlp_train_kernel(MlpArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  constexpr int NT = NW * 64;
  constexpr int VR = NW / 2;   // value-head wave rotation (disjoint waves for paired narrow layers)
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
  STAMP(0);
  // Cross-barrier weight prefetch: before each barrier every wave loads the B fragments of its
  // first step of the next layer(s) (layer_prefetch / BPre), so the L2 latency overlaps the
  // barrier wait and the presets instead of stalling the first MFMA after it.
  constexpr int RB = ROWS / 16;
  BPre<DT, RB> pf_p, pf_v;
  // Optional wave balance at 8 waves: a narrow layer (4 tile pairs) split into (pair, row-half)
  // items — wave w takes pair w & 3 of rows 32*(w >> 2) .. +31 — for the policy head's fc1/fc2/
  // dgrad-fc2 and the value head's fc2.  Off: the phase timeline (scripts/phase_timeline.py)
  // showed the layers are latency-, not balance-bound, and fc1 lost more to the doubled weight
  // traffic of 32-row items than the barriers gained (18.4M vs 19.1M env steps/s).
  // split-bf16 at 8 waves (32 rows): fc1 = 4 policy + 16 value tile pairs on 8 waves (3 vs 2 per
  // wave whole); as policy half-pair items every wave takes 2 value pairs + 1 policy half
  // (phase timeline: fc1 barrier wait 7.3 k -> 4.1 k cycles per tile)
  constexpr bool SPLIT = IsSplit<DT>::value && NW == 8;
  constexpr int HR = SPLIT ? ROWS / 2 : ROWS;     // rows of one split item
  constexpr int SNW = SPLIT ? 4 : NW;             // "waves" of a split call
  const int sw = SPLIT ? (wave & 3) : wave;       // wave index inside a split call
  const int sh = SPLIT ? (wave >> 2) * HR : 0;    // first row of this wave's half
  // fc2 alone IS split at 8 waves: value fc2 has 4x the K of policy fc2, so with whole pairs
  // four waves idle at the barrier; as (pair, row-half) items every wave takes one policy and
  // one value half-pair (phase timeline: fc2 + barrier 18.1 k -> 16.1 k cycles per tile).
  constexpr bool SPLIT2 = (NW == 8);
  constexpr int HR2 = SPLIT2 ? ROWS / 2 : ROWS;
  constexpr int SNW2 = SPLIT2 ? 4 : NW;
  const int sw2 = SPLIT2 ? (wave & 3) : wave;
  const int sh2 = SPLIT2 ? (wave >> 2) * HR2 : 0;
  load_rows<DT, NT>(reinterpret_cast<const T*>(a.x_buf), a.idx, a.row0, m0, nvalid, a.d_in[0], X, ldx, ROWS, tid,
                    [&] {
                      layer_prefetch<DT, HR, SNW>(pf_p, W + a.off_w[0], a.d_in[0], a.n_out[0], sw, lane);
                      layer_prefetch<DT, ROWS, NW>(pf_v, W + a.off_w[3], a.d_in[3], a.n_out[3], wave, lane, VR);
                      preset_pad<DT>(H1p, ld1p, ROWS, a.n_out[0], tid, NT);
                      preset_pad<DT>(H1v, ld1v, ROWS, a.n_out[3], tid, NT);
                    },
                    a.x_stream != 0);
  __syncthreads();
  STAMP(1);
  // ---------------- forward ----------------
  // Activations go to the feature-major wgrad operands straight from the MFMA accumulators
  // (rows < n_real; the constant-1 bias row of each buffer is preset once by the host).
  T* h1pT = reinterpret_cast<T*>(a.h1pT);
  T* h2pT = reinterpret_cast<T*>(a.h2pT);
  T* h1vT = reinterpret_cast<T*>(a.h1vT);
  T* h2vT = reinterpret_cast<T*>(a.h2vT);
  if (!a.xT_ready) write_transposed<DT, ROWS, NT>(X, ldx, a.d_in[0], a.xT, a.ldT, m0, tid);  // else: rollout wrote it
  layer_gemm<DT, HR, SNW, EPI_TANH, true>(X + sh * ldx, ldx, a.d_in[0], W + a.off_w[0], a.n_out[0], H1p + sh * ld1p,
                                          ld1p, a.scale[0], sw, lane, h1pT, a.ldT, m0 + sh, 0, &pf_p);
  layer_gemm<DT, ROWS, NW, EPI_TANH, true>(X, ldx, a.d_in[3], W + a.off_w[3], a.n_out[3], H1v, ld1v, a.scale[3],
                                           wave, lane, h1vT, a.ldT, m0, VR, &pf_v);
  STAMP(2);
  layer_prefetch<DT, HR2, SNW2>(pf_p, W + a.off_w[1], a.d_in[1], a.n_out[1], sw2, lane);
  layer_prefetch<DT, HR2, SNW2>(pf_v, W + a.off_w[4], a.d_in[4], a.n_out[4], sw2, lane, SPLIT2 ? 0 : VR);
  __syncthreads();
  STAMP(3);
  // X is dead: preset the tiles that alias its region
  preset_pad<DT>(H2p, ld2p, ROWS, a.n_out[1], tid, NT);
  preset_pad<DT>(H2v, ld2v, ROWS, a.n_out[4], tid, NT);
  zero_tile<DT>(DMU, ldmu, ROWS, tid, NT);
  zero_tile<DT>(DV, ldv, ROWS, tid, NT);
  __syncthreads();
  STAMP(4);
  layer_gemm<DT, HR2, SNW2, EPI_TANH, true>(H1p + sh2 * ld1p, ld1p, a.d_in[1], W + a.off_w[1], a.n_out[1],
                                            H2p + sh2 * ld2p, ld2p, a.scale[1], sw2, lane, h2pT, a.ldT, m0 + sh2, 0,
                                            &pf_p);
  layer_gemm<DT, HR2, SNW2, EPI_TANH, true>(H1v + sh2 * ld1v, ld1v, a.d_in[4], W + a.off_w[4], a.n_out[4],
                                            H2v + sh2 * ld2v, ld2v, a.scale[4], sw2, lane, h2vT, a.ldT, m0 + sh2,
                                            SPLIT2 ? 0 : VR, &pf_v);
  STAMP(5);
  layer_prefetch<DT, ROWS, NW>(pf_p, W + a.off_w[2], a.d_in[2], A, wave, lane);
  layer_prefetch<DT, ROWS, NW>(pf_v, W + a.off_w[5], a.d_in[5], 1, wave, lane, VR);
  // loss inputs of this thread's row / action dims: issued now, consumed after fc3
  constexpr int TPR = NT / ROWS;
  constexpr int JMAX = 4;   // dims held in registers per lane (A <= JMAX * TPR; the rest re-load)
  const int lrow_r = tid / TPR, lsub = tid % TPR;
  const bool lvalid = lrow_r < nvalid;
  const int lsrc = lvalid ? (a.idx ? a.idx[m0 + lrow_r] : a.row0 + m0 + lrow_r) : (a.idx ? a.idx[m0] : a.row0 + m0);
  float actv[JMAX];
#pragma unroll
  for (int q = 0; q < JMAX; ++q) {
    const int j = lsub + q * TPR;
    actv[q] = j < A ? a.actions[(size_t)lsrc * A + j] : 0.f;
  }
  const float l_adv = a.adv[lsrc], l_ret = a.ret[lsrc];
  const float l_lpo = a.loss_kind == 0 ? a.logp_old[lsrc] : 0.f;
  const float l_vold = a.loss_kind == 0 ? a.v_old[lsrc] : 0.f;
  __syncthreads();
  STAMP(6);
  layer_gemm<DT, ROWS, NW, EPI_LINEAR_F32, true>(H2p, ld2p, a.d_in[2], W + a.off_w[2], A, MU, A, a.scale[2], wave, lane,
                                                 nullptr, 0, 0, 0, &pf_p);
  layer_gemm<DT, ROWS, NW, EPI_LINEAR_F32, true>(H2v, ld2v, a.d_in[5], W + a.off_w[5], 1, V, 1, a.scale[5], wave, lane,
                                                 nullptr, 0, 0, VR, &pf_v);
  // dgrad fc3 weights (mu / v heads, transposed images)
  layer_prefetch<DT, ROWS, NW>(pf_p, W + a.off_wt[2], a.d_out[2], a.n_out[1], wave, lane);
  layer_prefetch<DT, ROWS, NW>(pf_v, W + a.off_wt[5], a.d_out[5], a.n_out[4], wave, lane, VR);
  __syncthreads();
  STAMP(7);
  // ---------------- loss + dL/d(mu, log_std, v): TPR lanes per row ----------------
  // Every thread works: the TPR consecutive lanes of a row split its A action dims and
  // combine their partial sums (log-prob, clip/entropy terms) with xor-shuffles inside the
  // group, so the per-row serial chain is ceil(A / TPR) dims long instead of A.
  {
    const int r = lrow_r, sub = lsub, src = lsrc;
    const bool valid = lvalid;
    const float* act = a.actions + (size_t)src * A;
    // action dim j = sub + q*TPR: registers for q < JMAX, re-loaded beyond
    auto act_at = [&](int q, int j) {
      if (q >= JMAX) return act[j];
      float x = actv[0];
#pragma unroll
      for (int u = 1; u < JMAX; ++u)
        if (q == u) x = actv[u];
      return x;
    };
    const float advv = l_adv;
    const float v = V[r];
    const float cvar = a.std_var ? 0.5f : 1.f;
    float lclip = 0.f, lent = 0.f, kl = 0.f, cf = 0.f, vold;
    if (a.loss_kind == 0) {
      // ---- corrected PPO (ppo.py:148-167) ----
      float logp = 0.f;
      for (int j = sub, q = 0; j < A; j += TPR, ++q) {
        const float lsig = cvar * a.log_std[j];
        const float z = (act_at(q, j) - MU[r * A + j]) * __expf(-lsig);
        logp += -0.5f * z * z - 0.5f * LOG_2PI_F - lsig;
      }
      logp = group_sum<TPR>(logp);
      const float lr = logp - l_lpo;
      const float ratio = __expf(lr);
      const float s1 = ratio * advv;
      const float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * advv;
      lclip = -fminf(s1, s2);
      const float dlogp = (s1 <= s2) ? -advv * ratio : 0.f;
      kl = (ratio - 1.f) - lr;
      cf = (fabsf(ratio - 1.f) > a.clip) ? 1.f : 0.f;
      for (int j = sub, q = 0; j < A; j += TPR, ++q) {
        const float lsig = cvar * a.log_std[j];
        const float isig = __expf(-lsig);
        const float z = (act_at(q, j) - MU[r * A + j]) * isig;
        P::put(DMU, r * ldmu + j, valid ? dlogp * z * isig : 0.f);
        // d/dlog_std: logp term + entropy bonus (-ent_coeff * sum_j log sigma_j)
        DLS[r * A + j] = valid ? (dlogp * (z * z - 1.f) - a.ent_coeff) * cvar : 0.f;
        lent += -a.ent_coeff * (0.5f + 0.5f * LOG_2PI_F + lsig);
      }
      lent = group_sum<TPR>(lent);
      vold = l_vold;
    } else {
      // ---- reference DPPO loss (train.py:142-161): per-dim pdf ratio, variance convention ----
      const float invA = 1.f / (float)A;
      const bool first = a.first_step != 0;
      for (int j = sub, q = 0; j < A; j += TPR, ++q) {
        const float mu = MU[r * A + j];
        const float var = __expf(a.log_std[j]);
        const float mu_o = first ? mu : a.mu_prev[(size_t)src * A + j];
        const float var_o = first ? var : __expf(a.log_std_old[j]);
        const float x = act_at(q, j);
        const float p = __expf(-(x - mu) * (x - mu) / (2.f * var)) * rsqrtf(2.f * var * 3.14159265358979f);
        const float po = __expf(-(x - mu_o) * (x - mu_o) / (2.f * var_o)) * rsqrtf(2.f * var_o * 3.14159265358979f);
        const float ratio = p / (1e-10f + po);
        const float s1 = ratio * advv;
        const float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * advv;
        lclip += -fminf(s1, s2) * invA;
        const float dratio = (s1 <= s2) ? -advv * invA : 0.f;
        float dp = dratio / (1e-10f + po);
        const float lg = logf(p + 1e-5f);
        lent += -a.ent_coeff * p * lg * invA;
        dp += -a.ent_coeff * invA * (lg + p / (p + 1e-5f));
        P::put(DMU, r * ldmu + j, valid ? dp * p * (x - mu) / var : 0.f);
        DLS[r * A + j] = valid ? dp * p * ((x - mu) * (x - mu) / (2.f * var) - 0.5f) : 0.f;
        cf += (fabsf(ratio - 1.f) > a.clip) ? invA : 0.f;
        if (valid) a.mu_prev[(size_t)src * A + j] = mu;   // train.py:164 model_old <- model
      }
      lclip = group_sum<TPR>(lclip);
      lent = group_sum<TPR>(lent);
      cf = group_sum<TPR>(cf);
      vold = first ? v : a.v_prev[src];
    }
    if (sub == 0) {
      const float retv = l_ret;
      float dv, lv;
      if (a.value_loss == 0) {
        const float d = v - retv;
        lv = d * d;
        dv = 2.f * d;
      } else {
        const float d1 = v - retv;
        const float dd = v - vold;
        const float vc = vold + fminf(fmaxf(dd, -a.clip), a.clip);
        const float d2 = vc - retv;
        const float f1 = d1 * d1, f2 = d2 * d2;
        const float inr = (dd >= -a.clip && dd <= a.clip) ? 1.f : 0.f;
        lv = 0.5f * fmaxf(f1, f2);
        if (f1 > f2) dv = d1;
        else if (f2 > f1) dv = d2 * inr;
        else dv = 0.5f * d1 + 0.5f * d2 * inr;
      }
      if (a.loss_kind != 0 && valid) a.v_prev[src] = v;
      P::put(DV, r * ldv, valid ? dv : 0.f);
      float* lrow = LOSS + r * NPART_FIXED;
      const float vm = valid ? 1.f : 0.f;
      lrow[0] = lclip * vm; lrow[1] = lv * vm; lrow[2] = lent * vm; lrow[3] = kl * vm; lrow[4] = cf * vm;
      lrow[5] = vm; lrow[6] = 0.f; lrow[7] = 0.f;
    }
  }
  __syncthreads();
  STAMP(8);
  // ---------------- per-workgroup partials + dY^T of the output layers ----------------
  {
    // column q of [loss terms | dlog_std] summed over the tile's rows by a group of PG lanes
    // (fixed order: strided partials, then an xor tree) — deterministic
    constexpr int PG = 16;
    for (int q0 = 0; q0 < NPART_FIXED + A; q0 += NT / PG) {
      const int q = q0 + tid / PG, g = tid % PG;
      float s = 0.f;
      if (q < NPART_FIXED + A) {
        if (q < NPART_FIXED) for (int r = g; r < ROWS; r += PG) s += LOSS[r * NPART_FIXED + q];
        else for (int r = g; r < ROWS; r += PG) s += DLS[r * A + (q - NPART_FIXED)];
      }
      s = group_sum<PG>(s);
      if (q < NPART_FIXED + A && g == 0) a.part[(size_t)blockIdx.x * a.npart + q] = s;
    }
  }
  write_transposed<DT, ROWS, NT>(DMU, ldmu, A, a.g3pT, a.ldT, m0, tid);
  write_transposed<DT, ROWS, NT>(DV, ldv, 1, a.g3vT, a.ldT, m0, tid);
  STAMP(9);
  // ---------------- dgrad chain (dY^T of every layer stored from the accumulators) --------
  T* g2pT = reinterpret_cast<T*>(a.g2pT);
  T* g2vT = reinterpret_cast<T*>(a.g2vT);
  layer_gemm<DT, ROWS, NW, EPI_DTANH_INPLACE, true>(DMU, ldmu, a.d_out[2], W + a.off_wt[2], a.n_out[1], H2p, ld2p,
                                                    a.scale[2], wave, lane, g2pT, a.ldT, m0, 0, &pf_p);
  layer_gemm<DT, ROWS, NW, EPI_DTANH_INPLACE, true>(DV, ldv, a.d_out[5], W + a.off_wt[5], a.n_out[4], H2v, ld2v,
                                                    a.scale[5], wave, lane, g2vT, a.ldT, m0, VR, &pf_v);
  STAMP(10);
  layer_prefetch<DT, HR, SNW>(pf_p, W + a.off_wt[1], a.d_out[1], a.n_out[0], sw, lane);
  layer_prefetch<DT, ROWS, NW>(pf_v, W + a.off_wt[4], a.d_out[4], a.n_out[3], wave, lane, VR);
  __syncthreads();
  STAMP(11);
  // EPI_DTANH_GLOBAL's only output is the wgrad operand, so it always stores (ablation bit0
  // does not apply here or the MFMAs would be dead code)
  layer_gemm<DT, HR, SNW, EPI_DTANH_GLOBAL, true>(H2p + sh * ld2p, ld2p, a.d_out[1], W + a.off_wt[1], a.n_out[0],
                                                  H1p + sh * ld1p, ld1p, a.scale[1], sw, lane,
                                                  reinterpret_cast<T*>(a.g1pT), a.ldT, m0 + sh, 0, &pf_p);
  layer_gemm<DT, ROWS, NW, EPI_DTANH_GLOBAL, true>(H2v, ld2v, a.d_out[4], W + a.off_wt[4], a.n_out[3], H1v, ld1v,
                                                   a.scale[4], wave, lane, reinterpret_cast<T*>(a.g1vT), a.ldT, m0, VR,
                                                   &pf_v);
  STAMP(12);
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

constexpr size_t LDS_MAX = 160 * 1024;
// 0: auto (largest tile that fits LDS), else force 16 / 32 / 64 rows (A/B diagnostics; a
// forced tile that does not fit falls back to auto)
int g_rows_override = 0;

// Row tile of the fused kernels.  A weight fragment loaded from L2 feeds ROWS/16 MFMAs, so the
// 64-row tile (8 waves, 512 threads, one workgroup per CU) halves the L2->CU weight traffic of
// the 32-row tile (4 waves, two workgroups per CU) at the same 8 waves per CU.  fp32 operands
// are twice the bytes: 16 rows.
template <int DT>
int train_rows_t(const MlpArgs& a) {
  if constexpr (DT == DT_F32) {
    return 16;
  } else if constexpr (DT == DT_S3) {
    // split-bf16 fragments are fp32-sized: the 64-row / 8-wave form spills (2 x 256 VGPRs per
    // SIMD is not enough), and at Humanoid dims only the 32-row tile fits LDS anyway (the
    // reference network's update runs on the per-head kernels, csrc/mlp_head.hip)
    return g_rows_override == 16 ? 16 : 32;
  } else {
    const int want = g_rows_override;
    if ((want == 0 || want == 64) && train_lds<DT, 64>(a) <= LDS_MAX) return 64;
    if (want == 16) return 16;
    return 32;
  }
}

// value-only forward: the 64-row tile measured no better (73 vs 77 us, scripts/ab_kernels.py):
// with 3 layers and no backward there is less latency for the second workgroup to hide, so
// the 32-row tile stays the default and 64 is an explicit choice
template <int DT>
int value_rows_t(const MlpArgs& a) {
  if constexpr (DT == DT_F32) {
    return 32;
  } else {
    if (g_rows_override == 64 && value_lds<DT, 64>(a) <= LDS_MAX) return 64;
    return 32;
  }
}

template <int DT, int ROWS, int NW>
void train_launch(const MlpArgs& a, hipStream_t s) {
  const size_t lds = train_lds<DT, ROWS>(a);
  set_max_lds_once<mlp_train_kernel<DT, ROWS, NW>>(lds);
  const int nblk = (a.M + ROWS - 1) / ROWS;
  hipLaunchKernelGGL((mlp_train_kernel<DT, ROWS, NW>), dim3(nblk), dim3(NW * 64), lds, s, a);
  HIP_CHECK_LAUNCH();
}

template <int DT, int ROWS, int NW>
void value_launch(const MlpArgs& a, hipStream_t s) {
  const size_t lds = value_lds<DT, ROWS>(a);
  set_max_lds_once<mlp_value_kernel<DT, ROWS, NW>>(lds);
  const int nblk = (a.M + ROWS - 1) / ROWS;
  hipLaunchKernelGGL((mlp_value_kernel<DT, ROWS, NW>), dim3(nblk), dim3(NW * 64), lds, s, a);
  HIP_CHECK_LAUNCH();
}

// waves of the 32-row split-bf16 workgroup: 4 (one wave per SIMD, 512 VGPRs each) or 8 (two
// per SIMD at <= 256 VGPRs: the second wave hides the first's L2 / LDS latency).  Measured
// (scripts/ab_train.py, bench geometry): 8 waves 290 us vs 4 waves 361 us per call.
int g_s3_train_waves = 8;

template <int DT>
int train_waves_t(const MlpArgs& a) {
  const int rows = train_rows_t<DT>(a);
  if (rows == 64) return 8;
  if (DT == DT_S3 && rows == 32 && g_s3_train_waves == 8) return 8;
  return 4;
}

template <int DT>
void train_t(const MlpArgs& a, hipStream_t s) {
  if constexpr (DT == DT_F32) {
    train_launch<DT, 16, 4>(a, s);
  } else {
    const int rows = train_rows_t<DT>(a);
    if constexpr (DT == DT_S3) {
      if (rows == 32 && train_waves_t<DT>(a) == 8) {
        train_launch<DT, 32, 8>(a, s);
        return;
      }
    }
    if (rows == 64) train_launch<DT, 64, 8>(a, s);
    else if (rows == 16) train_launch<DT, 16, 4>(a, s);
    else train_launch<DT, 32, 4>(a, s);
  }
}

int g_s3_value_waves = 8;   // split-bf16 value forward: 4 or 8 waves per 32-row workgroup (A/B)

int cu_count() {
  static int n = 0;
  if (n <= 0) {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

template <int DT>
void value_t(const MlpArgs& a, hipStream_t s);

// The reference network's value forward on the value head's 128-row streaming kernel in forward
// mode (csrc/mlp_head.hip; set_head_kernels(0) keeps the tile kernels).  One workgroup per CU at a
// time, so a launch costs whole rounds of ncu workgroups: the bench's T*E + E = 69,632 rows are
// 2.125 rounds, and the 32-workgroup third round costs as much as a full one.  Rows past the last
// full round (when they are at most a quarter round) go to the 32-row tile kernel instead, whose
// small workgroups spread over all CUs.
// (rounds 5-6 ran these rows on a 32x32 transposed-chain kernel, csrc/vhead.hip: at par in round 5,
// 128 vs 116 us per values() call at bf16x3 in its round-6 one-wave-per-SIMD form; removed)
template <int DT>
void head_fwd(const MlpArgs& a, hipStream_t s) {
  launch_mlp_head_value(DT, a, s);
}

template <int DT>
void value_head_t(const MlpArgs& a, hipStream_t s) {
  const int round = mlp_head_rows() * cu_count();
  const int full = a.M / round * round;
  if (full > 0 && full < a.M && a.M - full <= round / 4) {
    MlpArgs h = a;
    h.M = full;
    head_fwd<DT>(h, s);
    MlpArgs t = a;
    t.M = a.M - full;
    if (t.idx) t.idx += full;
    else t.row0 += full;
    t.v_out += full;
    value_t<DT>(t, s);   // (t.M < one round: takes the tile kernel below)
    return;
  }
  head_fwd<DT>(a, s);
}

template <int DT>
void value_t(const MlpArgs& a, hipStream_t s) {
  // (at least one full round of head workgroups: below it the 32-row kernel's small workgroups
  // fill the chip better)
  const bool head = DT != DT_F32 && DT != DT_FP8 && mlp_head_applies(a) && a.M >= mlp_head_rows() * cu_count();
  if constexpr (DT == DT_F32) {
    value_launch<DT, 32, 4>(a, s);
  } else if constexpr (DT == DT_S3) {
    if (head) {
      value_head_t<DT>(a, s);
      return;
    }
    // like the update: the 32-row tile takes most of LDS (one workgroup per CU), so a second
    // wave per SIMD is the latency hiding (scripts/ab_train.py: 162 vs 217 us per call)
    if (g_s3_value_waves == 8) value_launch<DT, 32, 8>(a, s);
    else value_launch<DT, 32, 4>(a, s);
  } else {
    if constexpr (DT == DT_BF16) {
      if (head) {
        value_head_t<DT>(a, s);
        return;
      }
    }
    if (value_rows_t<DT>(a) == 64) value_launch<DT, 64, 8>(a, s);
    else value_launch<DT, 32, 4>(a, s);
  }
}

template <int DT>
size_t train_lds_any(const MlpArgs& a) {
  const int rows = train_rows_t<DT>(a);
  return rows == 64 ? train_lds<DT, 64>(a) : rows == 32 ? train_lds<DT, 32>(a) : train_lds<DT, 16>(a);
}

}  // namespace

extern "C" void launch_mlp_train(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_F32) train_t<DT_F32>(a, s);
  else if (dt == DT_BF16) train_t<DT_BF16>(a, s);
  else if (dt == DT_S3) train_t<DT_S3>(a, s);
  else train_t<DT_FP8>(a, s);
}

extern "C" void launch_mlp_value(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_F32) value_t<DT_F32>(a, s);
  else if (dt == DT_BF16) value_t<DT_BF16>(a, s);
  else if (dt == DT_S3) value_t<DT_S3>(a, s);
  else value_t<DT_FP8>(a, s);
}

extern "C" size_t mlp_train_lds_bytes(int dt, const MlpArgs& a) {
  if (dt == DT_F32) return train_lds_any<DT_F32>(a);
  if (dt == DT_BF16) return train_lds_any<DT_BF16>(a);
  if (dt == DT_S3) return train_lds_any<DT_S3>(a);
  return train_lds_any<DT_FP8>(a);
}

extern "C" int mlp_train_rows(int dt, const MlpArgs& a) {
  if (dt == DT_F32) return train_rows_t<DT_F32>(a);
  if (dt == DT_BF16) return train_rows_t<DT_BF16>(a);
  if (dt == DT_S3) return train_rows_t<DT_S3>(a);
  return train_rows_t<DT_FP8>(a);
}

extern "C" void set_mlp_rows_override(int rows) { g_rows_override = rows; }
extern "C" void set_s3_train_waves(int nw) { g_s3_train_waves = nw == 8 ? 8 : 4; }
extern "C" void set_s3_value_waves(int nw) { g_s3_value_waves = nw == 8 ? 8 : 4; }
extern "C" int mlp_train_waves(int dt, const MlpArgs& a) {
  if (dt == DT_F32) return 4;
  if (dt == DT_BF16) return train_waves_t<DT_BF16>(a);
  if (dt == DT_S3) return train_waves_t<DT_S3>(a);
  return train_waves_t<DT_FP8>(a);
}
