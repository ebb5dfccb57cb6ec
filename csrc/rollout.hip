// Fused rollout kernel (SURVEY K1+K2/K3+K4+K6+K7+K8+K15): one launch collects T steps.
//
// Each workgroup owns ROWS envs for the whole launch.  Per step, entirely on-chip:
//   obs (from the env state in LDS) -> running-stat moments (K2) -> normalise + clamp (K3)
//   -> policy MLP on MFMA (K4; activations stay in LDS, weights stream from L2)
//   -> Gaussian sample + log-prob with in-kernel counter RNG (K6-K8)
//   -> env physics + reward clip + done/reset (K1, K15)
// and writes the update inputs (normalised obs in the MFMA storage precision, action, logp,
// clipped reward, done) to the HBM-resident [T][E] buffer.  The value head is NOT evaluated
// here: V(s_t) for GAE is computed afterwards by one big batched forward over all (T+1)*E
// rows (mlp.hip), which is far more MFMA-efficient than T small ones.
//
// Reference: train.py:82-106 (one env, batch 1, python loop) and model.py:68-80.
#include <type_traits>

#include "kernels.h"
#include "mlp_core.h"

namespace {

constexpr float LOG_2PI_F = 1.8378770664093453f;
constexpr float SYN_DECAY = 0.9f, SYN_DRIVE = 0.1f, SYN_NOISE = 0.05f, SYN_RESET = 0.1f;
constexpr float SYN_TERM_P = 0.002f;

// observation of env r, dim d.  KIND is a template parameter: with a runtime kind the
// pendulum's libm cosf/sinf (Payne-Hanek reduction, divergent per lane) was inlined into each
// of the ROWS unrolled iterations of the synthetic env's observe loop (~2,500 dead
// instructions per step and a 3x slower phase).
template <int KIND>
DEV float env_obs(const float* st, int S, int r, int d) {
  if constexpr (KIND == 1) {  // pendulum: (cos th, sin th, thdot)
    const float th = st[r * S + 0];
    return d == 0 ? cosf(th) : (d == 1 ? sinf(th) : st[r * S + 1]);
  } else {
    return st[r * S + d];
  }
}

// ---- per-step observation normalisation inside the launch (RolloutArgs sn_*) ----
// 8-byte {tag, fp32 bits} granules, stored and loaded relaxed at agent scope (sc1 vector accesses:
// MI355X_MICROARCH.md "granule"): the data is its own flag, so a hand-off needs no fence and no
// separate flag word.  Every spin is bounded: on a timeout the launch gives up (sn_err) instead of
// leaving waves that never finish.
typedef unsigned long long u64;
constexpr unsigned SN_SPIN_MAX = 1u << 21;   // >= ~1 s of polling per hand-off
constexpr int SN_MAX_BLOCKS = 256;           // grid cap of the per-step normalisation launch
DEV void sn_put(u64* g, unsigned tag, float v) {
  __hip_atomic_store(g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV u64 sn_get(const u64* g) {
  return __hip_atomic_load(const_cast<u64*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV float sn_val(u64 x) { return __uint_as_float((unsigned)x); }

// Workgroup `blk`: the step's Chan merge of the 4-feature units u = blk, blk + nblk, ...
// sn_g1 is line-blocked (kernels.h sn_g1_index): a 128-byte line holds one moment of 4 features x
// 4 workgroups, so a publisher writes 2 O / 4 partial lines and a unit is 2 nblk / 4 lines.
// (One reducer wave per feature over a workgroup-major layout polled one line per workgroup —
// 512 per feature, shared with 15 other features' reducers — and took 3-8 us per hand-off at 256
// workgroups; the idle cross-XCD hop is 0.41 us, scripts/probes/xcd_latency.hip.)  All NW waves
// poll a unit: wave w moment w & 1, line rows 4 ((w >> 1) RL + i) + (l >> 4), i < RL; lane
// l holds granule l & 15 (workgroup offset (l >> 2) & 3, feature fi = l & 3) and sums its rows
// in fp64 in order, then an xor butterfly over the lanes of one fi (the same bits in every lane:
// a fixed order) leaves the wave's partial in lanes 0-3; wave 0 adds the NW / 2 parts of each
// moment (fixed order), merges into the running (mean, M2) — csrc/obs.hip obs_merge's formulas —
// and publishes the (mean, 1/std) granules.  The values of a poll pass whose tags all match are
// the values.  (pf: the first unit's running (mean, M2), loaded by wave 0's lanes 0-3 at the
// start of the step — off the hand-off's critical path.)  Returns false on a timeout (after the
// workgroup's barriers).  Measured per rollout at 4,096 envs (profiles/r5/filter_probe_*): one
// reducer wave per feature 0.50 ms; one workgroup per 16-feature line block 0.60 ms (4 us per poll
// pass of 512 lines); 4x4 lines on waves 0-3 0.449 ms; on all 8 waves 0.415 ms; 2 features x 8
// workgroups per line 0.425 ms — the pass time follows each wave's outstanding line loads.
template <int NW>
DEV bool sn_reduce(const RolloutArgs& a, int nblk, int step, int wave, int lane, const float* shs,
                   double* red, double pmean, double pm2, unsigned& npoll) {
  const int O = a.O, nfu = (O + 3) >> 2, nwb = (nblk + 3) >> 2;
  const unsigned tag = a.sn_epoch0 + (unsigned)step;
  const int gp = lane & 15, fi = lane & 3, wi = (lane >> 2) & 3, lq = lane >> 4;
  constexpr int RL = SN_MAX_BLOCKS / 4 / 4 / (NW / 2);   // line rows per lane (64 rows in NW / 2 parts)
  const int m = wave & 1, part = wave >> 1;
  bool fail = false;
  for (int u = (int)blockIdx.x; u < nfu; u += nblk) {
    const int d = 4 * u + fi;
    {
      const u64* g = a.sn_g1 + (size_t)(m * nfu + u) * nwb * 16 + gp;
      float v[RL];
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < RL; ++i) {
          const int wb = lq + 4 * (RL * part + i);
          v[i] = 0.f;
          if (wb < nwb && 4 * wb + wi < nblk && d < O) {
            const u64 x = sn_get(g + (size_t)wb * 16);
            ok &= (unsigned)(x >> 32) == tag;
            v[i] = sn_val(x);
          }
        }
        npoll = spins + 1;
        if (__all(ok)) break;
        if (spins > SN_SPIN_MAX) { fail = true; break; }
        if (spins > 8) __builtin_amdgcn_s_sleep(1);
      }
      double p = 0.0;
#pragma unroll
      for (int i = 0; i < RL; ++i) p += (double)v[i];
#pragma unroll
      for (int x = 4; x < 64; x <<= 1) p += __shfl_xor(p, x);
      if (lane < 4) red[4 * wave + lane] = p;
    }
    __syncthreads();
    if (wave == 0 && lane < 4 && d < O) {
      double p1 = 0.0, p2 = 0.0;
#pragma unroll
      for (int q = 0; q < NW / 2; ++q) {
        p1 += red[8 * q + lane];
        p2 += red[8 * q + 4 + lane];
      }
      const bool pf = u == (int)blockIdx.x;
      const double count = (double)a.E, n_a = a.sn_n0 + (double)step * count;
      const double bmean_d = p1 / count;
      const double bmean = (double)shs[d] + bmean_d;
      double bm2 = p2 - p1 * bmean_d;
      if (bm2 < 0.0) bm2 = 0.0;
      const double n = n_a + count;
      const double mean0 = pf ? pmean : a.sn_mean[d];
      const double delta = bmean - mean0;
      const double mu = mean0 + delta * (count / n);
      const double M2 = (pf ? pm2 : a.sn_m2[d]) + bm2 + delta * delta * (n_a * count / n);
      double var = M2 / n;
      if (var < a.sn_var_floor) var = a.sn_var_floor;
      const float muf = (float)mu, inv = (float)(1.0 / sqrt(var));
      a.sn_mean[d] = mu;
      a.sn_m2[d] = M2;
      a.sn_mean_f32[d] = muf;
      a.sn_inv_std[d] = inv;
      sn_put(a.sn_g2 + d, tag, muf);
      sn_put(a.sn_g2 + O + d, tag, inv);
    }
    if (u + nblk < nfu) __syncthreads();   // (red is reused by the next unit)
  }
  return !fail;
}

// Every wave: gather its share of the step's (mean, 1/std) granules into LDS (granules tid,
// tid + NTHR, ... of the 2 O; the values of the poll pass whose tags all match; O <= SN_MAX_O)
constexpr int SN_MAX_O = 384;
template <int NTHR>
DEV bool sn_gather(const RolloutArgs& a, int step, int tid, float* nm, float* ninv, unsigned& npoll) {
  constexpr int GU = (2 * SN_MAX_O + NTHR - 1) / NTHR;
  const int O = a.O;
  const unsigned tag = a.sn_epoch0 + (unsigned)step;
  float v[GU];
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int i = tid + NTHR * u;
      if (i < 2 * O) {
        const u64 x = sn_get(a.sn_g2 + i);
        ok &= (unsigned)(x >> 32) == tag;
        v[u] = sn_val(x);
      }
    }
    npoll = spins + 1;
    if (__all(ok)) break;
    if (spins > SN_SPIN_MAX) return false;
    if (spins > 8) __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int u = 0; u < GU; ++u) {
    const int i = tid + NTHR * u;
    if (i < O) nm[i] = v[u];
    else if (i < 2 * O) ninv[i - O] = v[u];
  }
  return true;
}

// NW waves per workgroup: a 16-env tile is one workgroup per CU at E = 4096, so the 8-wave
// form (2 waves per SIMD) doubles the threads of the VALU-heavy observe / sample / env phases
// and gives the SIMDs a second wave to hide latency with; the MFMA layers use the first waves.
// SN: per-step observation normalisation inside the launch (RolloutArgs sn_*; cooperative launch)
template <int DT, int ROWS, int NW, bool SN>
__global__ __launch_bounds__(NW * 64) void rollout_kernel(RolloutArgs a) {
  using P = Prec<DT>;
  using T = typename P::T;
  constexpr int NTHR = 64 * NW;
  static_assert(ROWS % 4 == 0 && NTHR % ROWS == 0 && (NTHR / ROWS) <= 64, "rollout tiling");
  static_assert(!SN || NW >= 4, "the per-step filter's reduce polls with waves 0-3");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int e0 = blockIdx.x * ROWS;
  const int nvalid = min(ROWS, a.E - e0);
  const int O = a.O, A = a.A, S = a.S;
  const int ld1 = Lds<DT>::stride(a.d1), ld2 = Lds<DT>::stride(a.d2), ld3 = Lds<DT>::stride(a.d3);

  extern __shared__ __attribute__((aligned(16))) char smem[];
  LdsCarve cv(smem);
  float* st = cv.take<float>(ROWS * S);
  T* xs = cv.take<T>(ROWS * ld1);
  T* h1 = cv.take<T>(ROWS * ld2);
  T* h2 = cv.take<T>(ROWS * ld3);
  float* mu = cv.take<float>(ROWS * A);
  float* act = cv.take<float>(ROWS * A);
  float* epsb = cv.take<float>(ROWS * A);
  float* s1 = cv.take<float>(O);
  float* s2 = cv.take<float>(O);
  float* done_s = cv.take<float>(ROWS);
  int* eplen = cv.take<int>(ROWS);
  float* epret = cv.take<float>(ROWS);
  float* epacc = cv.take<float>(2 * ROWS);
  uint32_t* kes = cv.take<uint32_t>(3 * ROWS);   // per-env key prefixes of this step: action, env, reset
  float* wdrv = cv.take<float>(S);                // synthetic dynamics: drive weight of state dim d
  int* jdx = cv.take<int>(S);                     //                     action index driving dim d
  float* lsg = cv.take<float>(2 * A);             // per action dim: log sigma [0, A), sigma [A, 2A)
  // SN: the iteration shift and this step's (mean, 1/std) of every feature; the timeout flag
  float* shs = SN ? cv.take<float>(O) : nullptr;
  float* nm = SN ? cv.take<float>(O) : nullptr;
  float* ninv = SN ? cv.take<float>(O) : nullptr;
  int* sn_fail = SN ? cv.take<int>(1) : nullptr;
  double* sn_red = SN ? cv.take<double>(32) : nullptr;   // the reduce's per-wave partials
  // fp8: the MFMA tile is e4m3 but the buffer rows are bf16 — a bf16 staging tile lets them
  // leave as 16-byte row chunks (element stores strided by the row length were 2.6x the bf16
  // kernel's time)
  using XB = typename Prec<XStore<DT>::DTX>::T;
  constexpr bool STAGE = DT == DT_FP8;
  XB* xsb = STAGE ? cv.take<XB>(ROWS * a.d1) : nullptr;

  const T* W = reinterpret_cast<const T*>(a.W);
  const T* W1 = W + a.off_w1;
  const T* W2 = W + a.off_w2;
  const T* W3 = W + a.off_w3;
  using PX = Prec<XStore<DT>::DTX>;              // buffer precision (bf16 when DT is fp8)
  typename PX::T* xo = reinterpret_cast<typename PX::T*>(a.x_out);
  // per-layer dequant scales: device array (fp8 images, refreshed on-device) or kernel args
  const float sc1 = a.qscale ? a.qscale[0] : a.s1;
  const float sc2 = a.qscale ? a.qscale[1] : a.s2;
  const float sc3 = a.qscale ? a.qscale[2] : a.s3;

  // ---- load state, zero the padded activation tiles (pad columns stay constant) ----
  for (int i = tid; i < ROWS * S; i += NTHR) {
    int r = i / S, d = i - r * S;
    st[i] = (r < nvalid) ? a.state[(size_t)(e0 + r) * S + d] : 0.f;
  }
  preset_pad<DT>(h1, ld2, ROWS, a.n1, tid, NTHR);   // the layers' epilogues write columns < n
  preset_pad<DT>(h2, ld3, ROWS, a.n2, tid, NTHR);
  for (int d = tid; d < O; d += NTHR) { s1[d] = 0.f; s2[d] = 0.f; }
  if constexpr (SN) {
    for (int d = tid; d < O; d += NTHR) shs[d] = a.shift[d];
    if (tid == 0) *sn_fail = 0;
  }
  for (int d = tid; d < S; d += NTHR) {   // per-dim constants once per launch (no per-step modulo)
    wdrv[d] = 0.5f + (float)(d % 7) / 7.0f;
    jdx[d] = d % A;
  }
  // log_std is fixed during a rollout: log sigma and sigma once per launch, not a global load
  // (and an exp) per sampled dim and step
  for (int j = tid; j < A; j += NTHR) {
    const float ls = a.log_std[j];
    const float lsig = a.std_var ? 0.5f * ls : ls;
    lsg[j] = lsig;
    lsg[A + j] = __expf(lsig);
  }
  if (tid < ROWS) {
    int e = e0 + tid;
    eplen[tid] = (tid < nvalid) ? a.ep_len[e] : 0;
    epret[tid] = (tid < nvalid) ? a.ep_ret[e] : 0.f;
    epacc[2 * tid] = 0.f;
    epacc[2 * tid + 1] = 0.f;
  }
  __syncthreads();

  // normalisation constants of this thread's first feature: fixed for the whole launch, so
  // loaded once instead of once per step (the compiler cannot hoist them past the stores)
  float hm = 0.f, his = 1.f, hsh = 0.f;
  if (tid < O) { hm = a.mean[tid]; his = a.inv_std[tid]; hsh = a.shift[tid]; }
  BPre<DT, ROWS / 16> pf;   // cross-barrier weight prefetch of each layer's first k-chunk
  // bf16 / fp32: the LDS tile and the buffer share the element type (fp8 tiles feed a bf16 buffer)
  // (split-bf16: the LDS tile and the buffer share the 32-byte hi|lo group layout too)
  constexpr bool SPLIT = IsSplit<DT>::value;
  constexpr bool XO_FROM_LDS = std::is_same_v<T, typename PX::T> || SPLIT || STAGE;
  // the observe loop keeps this feature's ROWS values in the buffer type, or as fp32 for split
  // storage (split once, at the 32-byte x^T group store)
  using GT = std::conditional_t<SPLIT, float, typename PX::T>;
  // phase timeline (diagnostics, a.tstamp != null): per-wave shader-clock cycles summed over
  // the steps for each phase, written by lane 0 of every wave of every workgroup
  // (slots 7-10: the per-step filter's moments / reduce / gather / barrier, SN only)
  // (slots 11-14: absolute s_memrealtime of step 8's filter entry / moments published / reduce
  // done / gather done — the cross-workgroup skew of the hand-offs)
  // (slot 15: step 8's poll passes, gather << 32 | reduce)
  unsigned long long ph_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long ph_t = a.tstamp ? __builtin_amdgcn_s_memtime() : 0ull;
#define PH(i)                                                     \
  do {                                                            \
    if (a.tstamp != nullptr) {                                    \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
      ph_acc[i] += t_ - ph_t;                                     \
      ph_t = t_;                                                  \
    }                                                             \
  } while (0)
#define PH_ABS(i)                                                                  \
  do {                                                                             \
    if (a.tstamp != nullptr && step == 8) ph_acc[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  for (int step = 0; step <= a.T; ++step) {
    const int tb = a.t_base + step;
    const bool last = (step == a.T);  // bootstrap observation only
    // ---- (a) observe, moments, normalise -> LDS tile + global buffer row ----
    auto observe = [&](auto kind_tag) {
      constexpr int KIND = decltype(kind_tag)::value;
      for (int d = tid; d < a.d1; d += NTHR) {
        float m = hm, is = his, sh = hsh;
        if constexpr (SN) {
          if (d < O) { m = nm[d]; is = ninv[d]; }
        } else {
          if (d != tid && d < O) { m = a.mean[d]; is = a.inv_std[d]; sh = a.shift[d]; }
        }
        float ls1 = 0.f, ls2 = 0.f;
        GT grp[ROWS];   // this feature's ROWS consecutive buffer rows (xT groups of 8)
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
          float xv;
          if (d < O) {
            float o = env_obs<KIND>(st, S, r, d);
            if (!SN && !last && r < nvalid) { float dd = o - sh; ls1 += dd; ls2 += dd * dd; }
            xv = fminf(fmaxf((o - m) * is, -5.f), 5.f);
          } else {
            xv = (d == O) ? 1.f : 0.f;
          }
          P::put(xs, r * ld1 + d, xv);
          if constexpr (SPLIT) grp[r] = xv;
          else grp[r] = PX::cvt(xv);
          if constexpr (STAGE) xsb[r * a.d1 + d] = grp[r];
        }
        if (!SN && d < O) { s1[d] += ls1; s2[d] += ls2; }
        // full-batch update operand: rows m = tb*E + e0 + r are contiguous 8-groups of the FM
        // layout (host guarantees E % 16 == 0), written once per rollout instead of per epoch
        if (a.xT_out != nullptr && !last) {
          typename PX::T* xT = reinterpret_cast<typename PX::T*>(a.xT_out);
          const int mrow = tb * a.buf_E + e0;
#pragma unroll
          for (int g = 0; g < ROWS / 8; ++g) {
            typename PX::T* o = xT + fm_index(d, mrow + 8 * g, a.ldT);
            if constexpr (SPLIT) {
              bf16x8 hv, lv;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                __bf16 h, l;
                Prec<DT_S3>::split(grp[8 * g + j], h, l);
                hv[j] = h;
                lv[j] = l;
              }
              uint4* o4 = reinterpret_cast<uint4*>(o);
              o4[0] = *reinterpret_cast<const uint4*>(&hv);
              o4[1] = *reinterpret_cast<const uint4*>(&lv);
            } else if constexpr (sizeof(typename PX::T) == 2) {
              *reinterpret_cast<uint4*>(o) = *reinterpret_cast<const uint4*>(&grp[8 * g]);
            } else {
              reinterpret_cast<uint4*>(o)[0] = reinterpret_cast<const uint4*>(&grp[8 * g])[0];
              reinterpret_cast<uint4*>(o)[1] = reinterpret_cast<const uint4*>(&grp[8 * g])[1];
            }
          }
        }
      }
    };
    if constexpr (SN) {
      if (!last) {
        // this step's batch moments about the iteration shift -> the iteration's moments (as in
        // rollout mode) and this workgroup's granules; its waves merge the features it owns
        // (sn_reduce), every wave gathers its share of the new stats of every feature (sn_gather)
        const unsigned tag = a.sn_epoch0 + (unsigned)step;
        auto moments = [&](auto kind_tag) {
          constexpr int KIND = decltype(kind_tag)::value;
          for (int d = tid; d < O; d += NTHR) {
            const float sh = shs[d];
            float ls1 = 0.f, ls2 = 0.f;
            // every row read unconditionally (st holds ROWS rows), the invalid ones masked: a
            // per-row branch kept the compiler from batching the LDS reads (one round trip each)
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
              const float o = env_obs<KIND>(st, S, r, d);
              const float dd = r < nvalid ? o - sh : 0.f;
              ls1 += dd;
              ls2 += dd * dd;
            }
            s1[d] += ls1;
            s2[d] += ls2;
            sn_put(a.sn_g1 + sn_g1_index(0, d, (int)blockIdx.x, O, (int)gridDim.x), tag, ls1);
            sn_put(a.sn_g1 + sn_g1_index(1, d, (int)blockIdx.x, O, (int)gridDim.x), tag, ls2);
          }
        };
        // the running (mean, M2) of this workgroup's first unit (4 features), loaded now:
        // consumed after the hand-off (wave 0, lanes 0-3)
        const int dfirst = 4 * (int)blockIdx.x + lane;
        double pmean = 0.0, pm2 = 0.0;
        if (wave == 0 && lane < 4 && dfirst < O) {
          pmean = a.sn_mean[dfirst];
          pm2 = a.sn_m2[dfirst];
        }
        PH_ABS(11);
        if (a.kind == 1) moments(std::integral_constant<int, 1>{});
        else moments(std::integral_constant<int, 0>{});
        PH(7);
        PH_ABS(12);
        unsigned npr = 0, npg = 0;
        if (!sn_reduce<NW>(a, (int)gridDim.x, step, wave, lane, shs, sn_red, pmean, pm2, npr) && lane == 0)
          *sn_fail = 1;
        PH(8);
        PH_ABS(13);
        // the gather polls start once this workgroup's reducers are done: polling from the
        // other waves during the reduce queued ahead of the reducers' own loads on the CU
        __syncthreads();
        if (!sn_gather<NTHR>(a, step, tid, nm, ninv, npg) && lane == 0) *sn_fail = 1;
        PH(9);
        PH_ABS(14);
        if (a.tstamp != nullptr && step == 8) ph_acc[15] = ((unsigned long long)npg << 32) | npr;
        __syncthreads();
        PH(10);
        if (*sn_fail) {   // a peer never published: give up (the host raises)
          if (tid == 0) __hip_atomic_store(a.sn_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;
        }
      }
    }
    if (a.kind == 1) observe(std::integral_constant<int, 1>{});
    else observe(std::integral_constant<int, 0>{});
    if (!last) layer_prefetch<DT, ROWS, NW>(pf, W1, a.d1, a.n1, wave, lane);
    __syncthreads();
    if constexpr (XO_FROM_LDS) {
      // row-major buffer rows from the normalised LDS tile: one 16-byte store per 16 bytes of
      // features instead of ROWS element stores per feature (fire-and-forget, overlaps the MFMA
      // layers)
      constexpr int EPC = 16 / sizeof(XB);
      const int ch = a.d1 / EPC;
      for (int i = tid; i < nvalid * ch; i += NTHR) {
        const int r = i / ch, c = i - r * ch;
        const void* src = STAGE ? static_cast<const void*>(xsb + r * a.d1 + c * EPC)
                                : static_cast<const void*>(xs + r * ld1 + c * EPC);
        *reinterpret_cast<uint4*>(xo + ((size_t)tb * a.buf_E + e0 + r) * a.d1 + c * EPC) =
            *reinterpret_cast<const uint4*>(src);
      }
    }
    if (last) break;
    // (env, step) key prefixes of the sample / env phases, shared by every dim of the step:
    // hashed by the last wave's lanes (idle in the narrow policy layers) before fc1, so the
    // layers' barriers publish them and the sample phase needs no barrier of its own (the
    // previous step's env phase, their last reader, ended in a barrier)
    const uint32_t kstep = a.t0 + (uint32_t)step;
    if (tid >= NTHR - ROWS) {
      const int r = tid - (NTHR - ROWS);
      const uint32_t e = (uint32_t)(e0 + r);
      kes[r] = key_es(a.key_action, e, kstep);
      kes[ROWS + r] = key_es(a.key_env, e, kstep);
      kes[2 * ROWS + r] = key_es(a.key_reset, e, kstep);
    }
    PH(0);   // (a) observe -> after its barrier
    // ---- (b) policy MLP ----
    layer_gemm<DT, ROWS, NW, EPI_TANH, true>(xs, ld1, a.d1, W1, a.n1, h1, ld2, sc1, wave, lane, nullptr, 0, 0, 0, &pf);
    layer_prefetch<DT, ROWS, NW>(pf, W2, a.d2, a.n2, wave, lane);
    __syncthreads();
    PH(1);
    layer_gemm<DT, ROWS, NW, EPI_TANH, true>(h1, ld2, a.d2, W2, a.n2, h2, ld3, sc2, wave, lane, nullptr, 0, 0, 0, &pf);
    layer_prefetch<DT, ROWS, NW>(pf, W3, a.d3, a.n3, wave, lane);
    __syncthreads();
    PH(2);
    layer_gemm<DT, ROWS, NW, EPI_LINEAR_F32, true>(h2, ld3, a.d3, W3, a.n3, mu, A, sc3, wave, lane, nullptr, 0, 0, 0,
                                                   &pf);
    __syncthreads();
    PH(3);   // fc1, fc2, fc3 (each incl. barrier)
    // ---- (c) sample a = mu + sigma * eps (one Box-Muller pair -> two action dims) ----
    const int npa = (A + 1) >> 1;
    for (int i = tid; i < ROWS * npa; i += NTHR) {
      const int r = i / npa, q = i - r * npa;
      const float2 g = gauss_pair(kes[r], (uint32_t)q);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * q + h;
        if (j < A) {
          const float eps = h ? g.y : g.x;
          const float av = mu[r * A + j] + lsg[A + j] * eps;
          act[r * A + j] = av;
          epsb[r * A + j] = eps;
          if (r < nvalid) a.actions[((size_t)tb * a.buf_E + e0 + r) * A + j] = av;
        }
      }
    }
    __syncthreads();
    PH(4);   // (c) sample
    // ---- (d) per-env: logp, reward, termination, episode bookkeeping ----
    // LPE lanes per env (contiguous inside a wave) share the per-dim sums, then reduce by shuffles
    {
      constexpr int LPE = NTHR / ROWS;
      const int r = tid / LPE, l = tid - r * LPE;
      const int e = e0 + r;
      float lp = 0.f, err = 0.f;
      const int na = min(A, O);
      for (int j = l; j < A; j += LPE) {
        const float ep = epsb[r * A + j];
        lp += -0.5f * ep * ep - lsg[j];
        if (a.kind != 1 && j < na) {
          const float ac = fminf(fmaxf(act[r * A + j], -1.f), 1.f);
          const float d = ac - fast_tanh(st[r * S + j]);
          err += d * d;
        }
      }
#pragma unroll
      for (int o = LPE / 2; o > 0; o >>= 1) {
        lp += __shfl_xor(lp, o, LPE);
        err += __shfl_xor(err, o, LPE);
      }
      if (l == 0) {
        lp -= 0.5f * LOG_2PI_F * (float)A;
        float rew;
        bool term = false;
        if (a.kind == 1) {
          float th = st[r * S], thd = st[r * S + 1];
          float u = fminf(fmaxf(act[r * A], -2.f), 2.f);
          float thn = fmodf(th + 3.14159265358979f, 6.28318530717959f);
          if (thn < 0.f) thn += 6.28318530717959f;
          thn -= 3.14159265358979f;
          rew = -(thn * thn + 0.1f * thd * thd + 0.001f * u * u);
        } else {
          rew = 1.f - err / (float)na;
          term = uniform01(keyed(a.key_term, (uint32_t)e, kstep, 0u)) < SYN_TERM_P;
        }
        int el = eplen[r] + 1;
        float er_ = epret[r] + rew;
        bool done = term || (el >= a.limit);
        if (done) {
          if (r < nvalid) { epacc[2 * r] += er_; epacc[2 * r + 1] += 1.f; }
          el = 0;
          er_ = 0.f;
        }
        eplen[r] = el;
        epret[r] = er_;
        done_s[r] = done ? 1.f : 0.f;
        if (r < nvalid) {
          size_t o = (size_t)tb * a.buf_E + e;
          float rc = rew;
          if (a.reward_clip > 0.f) rc = fminf(fmaxf(rc, -a.reward_clip), a.reward_clip);
          a.logp[o] = lp;
          a.rewards[o] = rc;
          a.dones[o] = done ? 1.f : 0.f;
        }
      }
    }
    __syncthreads();
    PH(5);   // (d) logp / reward
    // ---- (e) state transition (+ in-place reset on done) ----
    if (a.kind == 1) {
      if (tid < ROWS) {
        const int r = tid, e = e0 + r;
        if (done_s[r] > 0.5f) {
          float u0 = uniform01(keyed(a.key_reset, (uint32_t)e, kstep, 0u));
          float u1 = uniform01(keyed(a.key_reset, (uint32_t)e, kstep, 1u));
          st[r * S] = (2.f * u0 - 1.f) * 3.14159265358979f;
          st[r * S + 1] = 2.f * u1 - 1.f;
        } else {
          float th = st[r * S], thd = st[r * S + 1];
          float u = fminf(fmaxf(act[r * A], -2.f), 2.f);
          float nthd = thd + (-3.f * 10.f / 2.f * sinf(th + 3.14159265358979f) + 3.f * u) * 0.05f;
          float nth = th + nthd * 0.05f;
          nthd = fminf(fmaxf(nthd, -8.f), 8.f);
          st[r * S] = nth;
          st[r * S + 1] = nthd;
        }
      }
    } else {
      // item = (row r, dim pair p), consecutive threads on consecutive pairs of one row: the
      // 16 x S/2 items spread evenly over the threads (one Box-Muller pair per item) and the
      // per-dim constants come from LDS tables filled once per launch.  Two items per turn with
      // every LDS read of both issued before any state store (items never share a state slot),
      // so the second item's loads, hashes and transcendentals overlap the first's instead of
      // waiting behind its stores; the reset / step choice is a select, not a branch.
      const int np = (S + 1) >> 1;
      int r = tid / np, p = tid - r * np;
      const int sr = NTHR / np, sp = NTHR - sr * np;
      struct In { float st0, st1, a0, a1, w0, w1; uint32_t key; bool done, has1; int d0; };
      auto load = [&](int rr, int pp) {
        In q;
        q.d0 = 2 * pp;
        q.has1 = q.d0 + 1 < S;
        const int d1 = q.has1 ? q.d0 + 1 : q.d0;
        q.done = done_s[rr] > 0.5f;
        q.key = q.done ? kes[2 * ROWS + rr] : kes[ROWS + rr];
        q.st0 = st[rr * S + q.d0];
        q.st1 = st[rr * S + d1];
        q.a0 = act[rr * A + jdx[q.d0]];
        q.a1 = act[rr * A + jdx[d1]];
        q.w0 = wdrv[q.d0];
        q.w1 = wdrv[d1];
        return q;
      };
      auto step_item = [&](const In& q, int pp, float& n0, float& n1) {
        const float2 g = gauss_pair(q.key, (uint32_t)pp);
        if (q.done) {
          n0 = SYN_RESET * g.x;
          n1 = SYN_RESET * g.y;
        } else {
          const float a0 = fminf(fmaxf(q.a0, -1.f), 1.f);
          const float a1 = fminf(fmaxf(q.a1, -1.f), 1.f);
          n0 = SYN_DECAY * q.st0 + SYN_DRIVE * fast_tanh(q.w0 * a0) + SYN_NOISE * g.x;
          n1 = SYN_DECAY * q.st1 + SYN_DRIVE * fast_tanh(q.w1 * a1) + SYN_NOISE * g.y;
        }
      };
      while (r < ROWS) {
        int r2 = r + sr, p2 = p + sp;
        if (p2 >= np) { p2 -= np; ++r2; }
        const bool v2 = r2 < ROWS;
        const In q1 = load(r, p);
        const In q2 = load(v2 ? r2 : r, v2 ? p2 : p);   // past the end: re-read item 1 (unused)
        float n10, n11, n20, n21;
        step_item(q1, p, n10, n11);
        step_item(q2, v2 ? p2 : p, n20, n21);
        st[r * S + q1.d0] = n10;
        if (q1.has1) st[r * S + q1.d0 + 1] = n11;
        if (v2) {
          st[r2 * S + q2.d0] = n20;
          if (q2.has1) st[r2 * S + q2.d0 + 1] = n21;
        }
        r = r2 + sr;
        p = p2 + sp;
        if (p >= np) { p -= np; ++r; }
      }
    }
    __syncthreads();
    PH(6);   // (e) env transition
  }
  __syncthreads();
  if (a.tstamp != nullptr && lane == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a.tstamp[((size_t)blockIdx.x * NW + wave) * 16 + i] = ph_acc[i];
  }
#undef PH
#undef PH_ABS
  // ---- write back env state, episode trackers, partial moments / episode stats ----
  for (int i = tid; i < nvalid * S; i += NTHR) a.state[(size_t)e0 * S + i] = st[i];
  if (tid < nvalid) {
    a.ep_len[e0 + tid] = eplen[tid];
    a.ep_ret[e0 + tid] = epret[tid];
  }
  float* mom = a.mom + (size_t)blockIdx.x * 2 * O;
  for (int d = tid; d < O; d += NTHR) { mom[d] = s1[d]; mom[O + d] = s2[d]; }
  if (tid == 0) {
    float sr = 0.f, sc = 0.f;
    for (int r = 0; r < ROWS; ++r) { sr += epacc[2 * r]; sc += epacc[2 * r + 1]; }
    a.epstat[2 * blockIdx.x] = sr;
    a.epstat[2 * blockIdx.x + 1] = sc;
  }
}

template <int DT, int ROWS>
size_t rollout_lds(const RolloutArgs& a) {
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  using T = typename Prec<DT>::T;
  size_t b = 0;
  b += al(sizeof(float) * ROWS * a.S);
  b += al(sizeof(T) * ROWS * Lds<DT>::stride(a.d1));
  b += al(sizeof(T) * ROWS * Lds<DT>::stride(a.d2));
  b += al(sizeof(T) * ROWS * Lds<DT>::stride(a.d3));
  b += 3 * al(sizeof(float) * ROWS * a.A);
  b += 2 * al(sizeof(float) * a.O);
  b += al(sizeof(float) * ROWS) + al(sizeof(int) * ROWS) + al(sizeof(float) * ROWS) + al(sizeof(float) * 2 * ROWS);
  b += al(sizeof(uint32_t) * 3 * ROWS);
  b += al(sizeof(float) * a.S) + al(sizeof(int) * a.S);
  b += al(sizeof(float) * 2 * a.A);
  if (a.sn_g1 != nullptr) b += 3 * al(sizeof(float) * a.O) + al(sizeof(int)) + al(sizeof(double) * 32);
  if (DT == DT_FP8) b += al(sizeof(__bf16) * ROWS * a.d1);   // bf16 staging tile of the buffer rows
  return b;
}

int g_rollout_waves = 8;   // 4 or 8 (set_rollout_waves: A/B diagnostics)

template <int DT, int ROWS, int NW>
void launch_nw(const RolloutArgs& a, hipStream_t s) {
  const size_t lds = rollout_lds<DT, ROWS>(a);
  const int nblk = (a.E + ROWS - 1) / ROWS;
  if (a.sn_g1 == nullptr) {
    if (lds > 65536) set_max_lds_once<rollout_kernel<DT, ROWS, NW, false>>(lds);
    hipLaunchKernelGGL((rollout_kernel<DT, ROWS, NW, false>), dim3(nblk), dim3(NW * 64), lds, s, a);
    HIP_CHECK_LAUNCH();
    return;
  }
  // per-step normalisation: every workgroup must be resident at once (the hand-offs wait on all
  // of them).  Cooperative launch: the runtime refuses a grid that cannot be co-resident; the
  // grid is also kept one workgroup per CU below the occupancy answer (MI355X_MICROARCH.md:
  // the API can overstate residency by one per CU)
  auto kfn = rollout_kernel<DT, ROWS, NW, true>;
  if (lds > 65536) set_max_lds_once<rollout_kernel<DT, ROWS, NW, true>>(lds);
  int per_cu = 0, dev = 0, ncu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kfn), NW * 64, lds);
  if (e == hipSuccess) e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) {
    dppo_note_error(e, __FILE__, __LINE__);
    return;
  }
  const int cap = ncu * (per_cu > 1 ? per_cu - 1 : per_cu);
  if (nblk > cap || nblk > SN_MAX_BLOCKS || a.O > SN_MAX_O) {
    dppo_note_error(hipErrorCooperativeLaunchTooLarge, __FILE__, __LINE__);
    return;
  }
  RolloutArgs aa = a;
  void* args[] = {&aa};
  e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kfn), dim3(nblk), dim3(NW * 64), args, (unsigned)lds, s);
  if (e != hipSuccess) dppo_note_error(e, __FILE__, __LINE__);
}

// the largest grid the per-step normalisation launch accepts (0: none)
template <int DT, int ROWS, int NW>
int stepnorm_cap(const RolloutArgs& a) {
  const size_t lds = rollout_lds<DT, ROWS>(a);
  auto kfn = rollout_kernel<DT, ROWS, NW, true>;
  if (lds > 65536) set_max_lds_once<rollout_kernel<DT, ROWS, NW, true>>(lds);
  int per_cu = 0, dev = 0, ncu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kfn), NW * 64, lds) !=
          hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  if (a.O > SN_MAX_O) return 0;   // the gather holds 2 O granules in registers
  const int cap = ncu * (per_cu > 1 ? per_cu - 1 : per_cu);
  return cap < SN_MAX_BLOCKS ? cap : SN_MAX_BLOCKS;
}

template <int DT, int ROWS>
void launch_t(const RolloutArgs& a, hipStream_t s) {
  // fp32 operands and 32-env tiles: the 8-wave form spills (twice the fragment registers)
  if (g_rollout_waves == 4 || DT == DT_F32 || ROWS > 16) launch_nw<DT, ROWS, 4>(a, s);
  else launch_nw<DT, ROWS, 8>(a, s);
}
template <int DT, int ROWS>
int cap_t(const RolloutArgs& a) {
  if (g_rollout_waves == 4 || DT == DT_F32 || ROWS > 16) return stepnorm_cap<DT, ROWS, 4>(a);
  return stepnorm_cap<DT, ROWS, 8>(a);
}

}  // namespace

extern "C" void set_rollout_waves(int nw) { g_rollout_waves = nw; }

// workgroups the per-step normalisation launch can hold co-resident (its grid must not exceed it)
extern "C" int rollout_stepnorm_cap(int dt, const RolloutArgs& a, int rows) {
  if (rows == 32) {
    if (dt == DT_F32) return cap_t<DT_F32, 32>(a);
    if (dt == DT_BF16) return cap_t<DT_BF16, 32>(a);
    if (dt == DT_S3) return cap_t<DT_S3, 32>(a);
    return cap_t<DT_FP8, 32>(a);
  }
  if (dt == DT_F32) return cap_t<DT_F32, 16>(a);
  if (dt == DT_BF16) return cap_t<DT_BF16, 16>(a);
  if (dt == DT_S3) return cap_t<DT_S3, 16>(a);
  return cap_t<DT_FP8, 16>(a);
}

extern "C" void launch_rollout(int dt, const RolloutArgs& a, int rows, hipStream_t s) {
  if (rows == 32) {
    if (dt == DT_F32) launch_t<DT_F32, 32>(a, s);
    else if (dt == DT_BF16) launch_t<DT_BF16, 32>(a, s);
    else if (dt == DT_S3) launch_t<DT_S3, 32>(a, s);
    else launch_t<DT_FP8, 32>(a, s);
  } else {
    if (dt == DT_F32) launch_t<DT_F32, 16>(a, s);
    else if (dt == DT_BF16) launch_t<DT_BF16, 16>(a, s);
    else if (dt == DT_S3) launch_t<DT_S3, 16>(a, s);
    else launch_t<DT_FP8, 16>(a, s);
  }
}
