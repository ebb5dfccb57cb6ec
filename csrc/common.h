// Shared device helpers for the DPPO kernels (gfx950 / CDNA4, wave64).
//
// * Prec<DT>: one MFMA "fragment" abstraction for the four operand precisions (fp32, bf16,
//   fp8 e4m3, and split-bf16 "bf16x3" = fp32-accurate on three bf16 MFMAs).
//   Every fragment holds 8 consecutive K-elements per lane: lane l owns rows/cols (l & 15)
//   and k = 8*(l >> 4) + j, j = 0..7 — the native operand map of
//   v_mfma_f32_16x16x32_{bf16,fp8} (cdna_hip_programming.md §3).  The fp32 path issues
//   eight v_mfma_f32_16x16x4_f32 (exact f32) over the SAME fragment by permuting k inside
//   the 32-deep step (both operands use the same permutation, so the sum is unchanged).
//   C/D map (dtype independent on gfx950): col = lane & 15, row = 4*(lane >> 4) + i.
// * counter-based RNG identical to pytorch_dppo_amd/utils/rng.py (lowbias32 + Box-Muller).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp8.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

#define DEV __device__ __forceinline__
typedef __attribute__((ext_vector_type(8))) float f32x8v;
// Elementwise fp32 vector arithmetic of the MFMA epilogues / operand splits (packed v_pk_* f32 ops;
// scalar spellings measured mixed in round 4, profiles/r4/ab_nopk/)
DEV f32x4 ew_sub(const f32x4& a, const f32x4& b) { return a - b; }
DEV f32x8v ew_sub(const f32x8v& a, const f32x8v& b) { return a - b; }
DEV f32x8v ew_add(const f32x8v& a, const f32x8v& b) { return a + b; }
DEV f32x4 ew_mul(const f32x4& a, float s) { return a * s; }
// a * (1 - h * h) (the tanh derivative)
DEV f32x4 ew_dtanh(const f32x4& a, const f32x4& h) { return a * (1.0f - h * h); }

enum { DT_F32 = 0, DT_BF16 = 1, DT_FP8 = 2, DT_S3 = 3 };

template <int DT> struct Prec;

template <> struct Prec<DT_F32> {
  using T = float;
  struct Frag { float4 lo, hi; };
  static constexpr int BYTES = 4;
  DEV static Frag load(const T* p) {
    Frag f; f.lo = reinterpret_cast<const float4*>(p)[0]; f.hi = reinterpret_cast<const float4*>(p)[1];
    return f;
  }
  DEV static f32x4 mma(f32x4 c, const Frag& a, const Frag& b) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.x, b.lo.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.y, b.lo.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.z, b.lo.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.w, b.lo.w, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.x, b.hi.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.y, b.hi.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.z, b.hi.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.w, b.hi.w, c, 0, 0, 0);
    return c;
  }
  DEV static T cvt(float x) { return x; }
  DEV static float tof(T x) { return x; }
  DEV static void put(T* b, size_t i, float x) { b[i] = x; }
  DEV static float get(const T* b, size_t i) { return b[i]; }
};

template <> struct Prec<DT_BF16> {
  using T = __bf16;
  using Frag = bf16x8;
  static constexpr int BYTES = 2;
  DEV static Frag load(const T* p) { return *reinterpret_cast<const bf16x8*>(p); }
  DEV static f32x4 mma(f32x4 c, const Frag& a, const Frag& b) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  DEV static T cvt(float x) { return (__bf16)x; }
  DEV static float tof(T x) { return (float)x; }
  DEV static void put(T* b, size_t i, float x) { b[i] = (__bf16)x; }
  DEV static float get(const T* b, size_t i) { return (float)b[i]; }
};

// Split-bf16 "fp32-accurate" operands (DT_S3): x = hi + lo with hi = bf16(x), lo = bf16(x - hi),
// and a . b ~= hi_a.hi_b + hi_a.lo_b + lo_a.hi_b on three v_mfma_f32_16x16x32_bf16 with fp32
// accumulation.  The residual (lo_a.lo_b plus each operand's lost tail) is ~2^-16 relative per
// product; a dot product's error is ~1e-5 relative — the fp32 GEMM tolerances of the tests
// (2e-5 value forward, 1e-4 gradients) hold at 3x the bf16 MFMA cost, where gfx950's exact
// v_mfma_f32_16x16x4_f32 runs at 1/16 of the bf16 rate (no xf32 MFMA on CDNA4).
// Storage: a logical element is a 4-byte slot (T), so every block-level address (row strides,
// fragment-major fragments, LDS carving) is the fp32 one; inside each 8-aligned group of 8
// slots (32 bytes) the 8 hi values come first (16 B), then the 8 lo values (16 B).  A fragment
// (8 consecutive k of one lane) is therefore 32 contiguous bytes: hi | lo, two 16-byte loads.
// Element i: hi at bf16 index 2*(i & ~7) + (i & 7), lo 8 further.  split(hi + lo) == (hi, lo)
// exactly (hi + lo is exact in fp32 and RNE ties can only have left hi even), so re-splitting a
// stored value is lossless.
struct S3Slot { uint32_t raw; };
struct S3Frag { bf16x8 h, l; };
template <> struct Prec<DT_S3> {
  using T = S3Slot;
  using Frag = S3Frag;
  static constexpr int BYTES = 4;
  DEV static Frag load(const T* p) {
    const bf16x8* q = reinterpret_cast<const bf16x8*>(p);
    return Frag{q[0], q[1]};
  }
  DEV static f32x4 mma(f32x4 c, const Frag& a, const Frag& b) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, c, 0, 0, 0);
  }
  DEV static __bf16* hi_ptr(T* b, size_t i) { return reinterpret_cast<__bf16*>(b) + 2 * (i & ~size_t(7)) + (i & 7); }
  DEV static const __bf16* hi_ptr(const T* b, size_t i) {
    return reinterpret_cast<const __bf16*>(b) + 2 * (i & ~size_t(7)) + (i & 7);
  }
  DEV static void split(float x, __bf16& h, __bf16& l) {
    h = (__bf16)x;
    l = (__bf16)(x - (float)h);
  }
  DEV static void put(T* b, size_t i, float x) {
    __bf16* p = hi_ptr(b, i);
    split(x, p[0], p[8]);
  }
  DEV static float get(const T* b, size_t i) {
    const __bf16* p = hi_ptr(b, i);
    return (float)p[0] + (float)p[8];
  }
};
template <int DT> struct IsSplit { static constexpr bool value = DT == DT_S3; };

// OCP e4m3fn (gfx950 native; NOT the MI300 fnuz encoding)
template <> struct Prec<DT_FP8> {
  using T = uint8_t;
  using Frag = long;
  static constexpr int BYTES = 1;
  DEV static Frag load(const T* p) { return *reinterpret_cast<const long*>(p); }
  DEV static f32x4 mma(f32x4 c, const Frag& a, const Frag& b) {
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
  }
  DEV static T cvt(float x) {
    // saturate to the largest finite e4m3 value instead of producing NaN
    __hip_fp8_e4m3 q(fminf(fmaxf(x, -448.f), 448.f));
    return *reinterpret_cast<uint8_t*>(&q);
  }
  DEV static float tof(T x) {
    __hip_fp8_e4m3 q;
    *reinterpret_cast<uint8_t*>(&q) = x;
    return float(q);
  }
  DEV static void put(T* b, size_t i, float x) { b[i] = cvt(x); }
  DEV static float get(const T* b, size_t i) { return tof(b[i]); }
};

// Fragment-major ("FM") layout of a [rows][cols] matrix (rows % 16 == 0, cols % 32 == 0):
// 16x32 blocks stored block-row-major, and inside a block lane l = (r & 15) + 16*((c & 31) >> 3)
// holds elements c & 7 = 0..7 contiguously — exactly the MFMA operand map.  A fragment load
// of block (rt, ks) is then ONE contiguous 512-element read (1 KiB at bf16) per wave:
// base + 8*lane, instead of 16 rows x 64 B (TA-bound, cdna_hip_programming.md §5 table).
// Used for the packed weight images and the feature-major wgrad operands.
__host__ __device__ inline size_t fm_index(int r, int c, int cols) {
  return ((size_t)(r >> 4) * (size_t)(cols >> 5) + (size_t)(c >> 5)) * 512u +
         (size_t)((((r & 15) + (((c & 31) >> 3) << 4)) << 3) + (c & 7));
}
// element offset of lane `lane`'s fragment of block (rt, ks) in an FM matrix with `cols` columns
__host__ __device__ inline size_t fm_frag(int rt, int ks, int cols, int lane) {
  return ((size_t)rt * (size_t)(cols >> 5) + (size_t)ks) * 512u + (size_t)lane * 8u;
}

// Store of a wgrad operand (the feature-major activations / gradients the fused update writes
// and the wgrad kernel reads back): non-temporal (streaming: keeps the weight images in L2; cached
// stores measured neutral, round 2)
template <typename V>
DEV void opnd_store(const V& v, V* p) {
  __builtin_nontemporal_store(v, p);
}

// ---- fp8 mode's e4m3 wgrad operands ("Q8", csrc/mlp_head.hip + csrc/wgrad.hip) ----
// The update writes every wgrad operand (x^T, h1^T, g1^T, g2^T of both heads) as OCP e4m3 bytes
// scaled by a power of two, and the wgrad kernel multiplies each product tile by the exact
// inverse.  Activations have fixed ranges: tanh outputs and the bias 1 (x 256 <= 256), the
// normalised observations clamped to +-5 (x 64 <= 320).  The gradients' scales are DELAYED
// per-tensor scales: step e stores with the scale of step e-1's amax (the head kernels
// atomic-max |g| into a 3-slot ring: accumulate e % 3, read (e-1) % 3, clear (e+1) % 3), chosen
// so the previous amax lands in [64, 128): 3.5x headroom below e4m3's 448 before saturation.
// The ring is [3 slots][4 tensors][Q8_SUB sub-slots][32 dwords]: each wave max-es into sub-slot
// (wave id) % Q8_SUB, one 128-byte line each, so the device-scope atomics of ~8k waves spread
// over 64 lines instead of serialising on one address (measured: one address per tensor made the
// head kernels 2.7x slower); a reader folds the 64 sub-slots with one load per lane.
// (ring geometry Q8_SUB / Q8_LINE / Q8_SLOT: csrc/kernels.h, shared with the bindings)
constexpr float Q8_SX = 64.f, Q8_SH = 256.f;
DEV uint32_t wave_umax(uint32_t v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__host__ __device__ inline float q8_pow2(int e) {   // 2^e, |e| <= 120, exact
  const uint32_t b = (uint32_t)(e + 127) << 23;
  float f;
  __builtin_memcpy(&f, &b, 4);
  return f;
}
// the exponent e of the store scale 2^e for a tensor of max |g| = amax (fp32 bits)
__host__ __device__ inline int q8_exp(uint32_t amax_bits) {
  const int ex = (int)((amax_bits >> 23) & 0xffu);
  if (ex == 0 || ex == 255) return 0;            // zero / denormal / non-finite: scale 1
  const int e = 6 - (ex - 127);
  return e < -120 ? -120 : (e > 120 ? 120 : e);
}
// 4 fp32 -> 4 e4m3 bytes (x s, saturated to +-448) in one dword, element 0 in the low byte
DEV uint32_t q8_pack4(const f32x4& v, float s) {
  const float a = fminf(fmaxf(v[0] * s, -448.f), 448.f), b = fminf(fmaxf(v[1] * s, -448.f), 448.f);
  const float c = fminf(fmaxf(v[2] * s, -448.f), 448.f), d = fminf(fmaxf(v[3] * s, -448.f), 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
// the same for values known to stay inside e4m3's range after scaling (activations)
DEV uint32_t q8_pack4u(const f32x4& v, float s) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * s, v[1] * s, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v[2] * s, v[3] * s, w, true);
}
DEV float absmax4(const f32x4& v) { return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))); }

// storage precision of the normalised-observation buffer written by the rollout and read by
// the value/update kernels: fp8 forward kernels keep it in bf16 (the update runs in bf16)
template <int DT> struct XStore { static constexpr int DTX = (DT == DT_FP8) ? DT_BF16 : DT; };

// LDS row padding of the activation tiles (row-major, width d a multiple of 32).  An A fragment
// is read with ds_read_b128: lane l takes row l & 15, 16 bytes at k-group l >> 4, and the LDS
// services the wave in four non-contiguous 16-lane groups ({0-3,12-15,20-27}, ...;
// MI355X_MICROARCH.md §LDS), bank = (byte / 4) mod 64.  With row stride S dwords the lane's
// first bank is 4 * (r * S / 4 + kg) mod 64: a 16-byte pad (S = 4 mod 64) puts two lanes of every
// group on the same 4 banks (2-way, the ds_read_b128 costs 8 instead of 4 LDS cycles — 38 % of
// the fused update's LDS cycles were conflicts); a 32-byte pad (S = 8 mod 64) is conflict-free
// for every group and every tile width here.  (fp8 tiles feed 8-byte operand reads: 16 bytes.)
template <int DT> struct Lds {
  static constexpr int PAD = (DT == DT_FP8 ? 16 : 32) / Prec<DT>::BYTES;
  __host__ __device__ static constexpr int stride(int d) { return d + PAD; }
};

// tanh from one v_exp_f32 and one v_rcp_f32 (no IEEE division); |err| ~1e-7, saturates cleanly
// (e -> 0 as |x| grows).  Used by the env dynamics inside the rollout kernel.
DEV float fast_tanh(float x) {
  const float e = __expf(-2.0f * fabsf(x));
  return copysignf((1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e), x);
}

// ---- counter RNG (must match utils/rng.py) -------------------------------------------------
DEV uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
// key chain: keyed = hash(hash(hash(env ^ base) ^ step) ^ dim).  key_es is the (env, step)
// prefix, shared by every dim of one env step: kernels compute it once per env and step.
DEV uint32_t key_es(uint32_t base, uint32_t env, uint32_t step) { return hash_u32(hash_u32(env ^ base) ^ step); }
DEV uint32_t keyed(uint32_t base, uint32_t env, uint32_t step, uint32_t dim) {
  return hash_u32(key_es(base, env, step) ^ dim);
}
DEV float uniform01(uint32_t h) { return ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f); }
// Box-Muller pair p: (r cos 2pi u2, r sin 2pi u2) = the normals of dims 2p and 2p+1
// (utils/rng.py: gauss).  Hardware transcendentals: v_log_f32, v_sqrt_f32, and v_sin/v_cos,
// which take the angle in revolutions, so 2*pi*u2 is never formed.
DEV float2 gauss_pair(uint32_t kes, uint32_t p) {
  const float u1 = uniform01(hash_u32(kes ^ (2u * p)));
  const float u2 = uniform01(hash_u32(kes ^ (2u * p + 1u)));
  const float r = __builtin_sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1));
  return make_float2(r * __builtin_amdgcn_cosf(u2), r * __builtin_amdgcn_sinf(u2));
}
DEV float gauss(uint32_t base, uint32_t env, uint32_t step, uint32_t dim) {
  const float2 g = gauss_pair(key_es(base, env, step), dim >> 1);
  return (dim & 1u) ? g.y : g.x;
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4): `lds` is the wave-uniform base, lane l
// lands at lds + 16 * l; the global source address is per lane.
DEV void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 |
// lgkmcnt[11:8]=15 | vmcnt[5:4] in [15:14])
#define WAIT_VMCNT(n) __builtin_amdgcn_s_waitcnt((((n) & 15) | (7 << 4) | (15 << 8) | ((((n) >> 4) & 3) << 14)))

// Launch-error channel (optim.hip): every launcher records the first failed launch or
// attribute call; every binding (bindings.cpp after_launch) takes it after its launch and raises
// a Python exception naming the op — a refused launch never leaves a silently stale result.
extern "C" void dppo_note_error(hipError_t e, const char* file, int line);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is a driver call (~µs of host time): issue it
// once per kernel instantiation and only raise it (the attribute is a per-function maximum).
template <auto Kernel>
inline void set_max_lds_once(size_t bytes) {
  static size_t set = 0;   // one static per kernel (template on the function pointer itself)
  if (bytes > set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(Kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) dppo_note_error(e, __FILE__, __LINE__);
    else set = bytes;
  }
}

#define HIP_CHECK_LAUNCH()                                          \
  do {                                                              \
    hipError_t e__ = hipGetLastError();                             \
    if (e__ != hipSuccess) dppo_note_error(e__, __FILE__, __LINE__); \
  } while (0)

// sum_{c < nch} p[c * st] in that fixed order (the split-K slab reduction of the weight gradient):
// the loads of 16 chunks are issued before the first add, instead of one load -> wait -> add
// round trip per chunk that a variable trip count otherwise compiles to.
__device__ __forceinline__ float slab_sum(const float* __restrict__ p, int nch, size_t st) {
  constexpr int B = 16;   // (24 / 32 in flight: 106 / 131 VGPRs, no faster; profiles/r6/ab_iter_slab_batch.log)
  float s = 0.f;
  for (int c0 = 0; c0 < nch; c0 += B) {
    float x[B];
#pragma unroll
    for (int c = 0; c < B; ++c) x[c] = (c0 + c < nch) ? p[(size_t)(c0 + c) * st] : 0.f;
#pragma unroll
    for (int c = 0; c < B; ++c)
      if (c0 + c < nch) s += x[c];
  }
  return s;
}

// Column sums of the per-workgroup partial rows (the reduce items of the gather kernels): the
// 256 threads of a block take items j = IPB b + (tid % IPB) (consecutive items are consecutive
// columns: one 128-byte segment per row) in RG = 256 / IPB row groups; row group g sums rows
// g, g + RG, ... in order (16 loads in flight: 512 partial rows are 4 dependent batches; 32 in
// flight took the gather kernel from 80 to 113 VGPRs, 6 to 4 waves per SIMD: fewer than its grid), then
// thread tid < IPB adds the RG groups in order — fixed order, deterministic.  Returns true on the
// threads that own an item (tid < IPB, j < nitems) with its sum in `out`.
// red_dst[j] >= 0: flat gradient index (of the gathered slice); -1 - q: loss_out[q].
__device__ __forceinline__ bool item_reduce(const float* __restrict__ part, int nprow, int npart,
                                            const int* __restrict__ red_col, int nitems, int b,
                                            float* red, float& out, int& j) {
  constexpr int RG = 256 / ITEM_IPB;
  const int tid = threadIdx.x, c = tid % ITEM_IPB, rg = tid / ITEM_IPB;
  j = ITEM_IPB * b + c;
  float s = 0.f;
  if (j < nitems && tid < 256) {   // (a 512-thread block: threads 256+ add zeros; red holds blockDim floats)
    const float* p = part + red_col[j];
    for (int r0 = rg; r0 < nprow; r0 += 16 * RG) {
      float x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u] = (r0 + RG * u < nprow) ? p[(size_t)(r0 + RG * u) * npart] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (r0 + RG * u < nprow) s += x[u];
    }
  }
  red[tid] = s;
  __syncthreads();
  if (tid < ITEM_IPB) {
    float o = red[tid];
#pragma unroll
    for (int g = 1; g < RG; ++g) o += red[g * ITEM_IPB + tid];
    out = o;
  }
  return tid < ITEM_IPB && j < nitems;
}
