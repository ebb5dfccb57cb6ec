// Value head on 32x32x16 MFMAs in the TRANSPOSED chain, ONE WAVE PER SIMD (SURVEY K5, K11;
// model.py:42-44 forward, train.py:109-112 GAE input, the value loss of train.py:154-157 /
// ppo.py:164 and its backward through fc3 and fc2 — the update of train.py:162-170 consumes the
// outputs).
//
// Every layer computes out^T = W . in^T:  A = a weight fragment (32 output features x 16 k, from
// the LDS ring, shared by all waves of the workgroup), B = the activations (16 k x 32 batch rows,
// in registers).  The 32x32 accumulator has the batch row on the lane and 16 output features in
// its registers (col = lane & 31, feature (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)), which is the
// NEXT layer's B operand up to one v_permlane32_swap per dword (t32.h b_operand): no LDS transpose
// anywhere in the chain, and one 32x16 fragment read from LDS feeds 32x32 outputs.
//
// Workgroup: 4 waves x 32 rows = 128 rows, one wave per SIMD and one workgroup per CU (<= 512
// registers per wave: the MFMA accumulators live in AGPRs — this file is built WITHOUT
// -amdgpu-mfma-vgpr-form, ops/_build.py).  Each wave holds ALL 512 fc1 features of its 32 rows
// (16 accumulator tiles, 256 registers) from fc1 to the end of the dgrad: no pair split of fc1 /
// fc2 (round 5's 8-wave form summed two fc2 partials through LDS and ran the dgrad in 4 pair
// passes at 254 VGPRs: 187 k cycles per workgroup, slower than the 16x16 kernel).
//
// Weights stream through an S-stage LDS ring of 32 KiB stages (8 LDS-DMA instructions of 1 KiB per
// wave and stage) straight from the packed FM images (csrc/common.h fm_index): a 32x16 A fragment
// is four 256-byte pieces of two 16x32 FM blocks, gathered by per-lane DMA source offsets,
// landing lane-linear.  Observation rows: a per-wave S-slot X ring (2 KiB per fc1 stage, 64-bit
// per-lane row addresses: any buffer size).  Counted vmcnt waits (every vector-memory instruction
// a wave issues — refills, X loads, operand stores — is counted, VmQ) + one raw s_barrier per
// stage; S - 1 stages of DMA stay in flight across it (cdna_hip_programming.md 'Pipelining
// across barriers').
//
// Stream (split-bf16 / bf16 stage counts): fc1 d_in/16 k-steps (24 / 12) | fc2 32 k-steps x 4
// tiles (8 / 4) | dgrad W2^T, 4 passes of 4 h1 tiles x 7 k-steps (8 / 4).
#include "t32.h"

namespace {

using namespace t32;

constexpr int VH_ROWS = 128;            // rows per workgroup
constexpr int VH_WAVES = 4;
constexpr int VH_SB = 32 * 1024;        // ring stage bytes
constexpr int VH_S = 4;                 // ring stages (3 in flight across each barrier)
constexpr int VH_GL = 8;                // ring DMA instructions per wave and stage
constexpr int VH_XB = 2048;             // X bytes per wave and fc1 stage
constexpr int VH_XS = VH_S;             // X slots per wave (issued with the weight batch of the same stage)

constexpr size_t vh_lds_bytes() { return (size_t)VH_S * VH_SB + (size_t)VH_WAVES * VH_XS * VH_XB; }
static_assert(vh_lds_bytes() <= 160 * 1024, "value head LDS");
// after fc1 the X rings hold: fc3 weights (129 floats), the dW_v partials [wave][half][64] and
// the loss partials
constexpr int VH_W3 = 128;
static_assert((VH_W3 + 4 + VH_WAVES * 2 * 64 + VH_WAVES) * 4 <= VH_WAVES * VH_XS * VH_XB, "scratch fits the X rings");

template <int DT>
constexpr int vh_ns2() { return 32 / (4 * VT<DT>::KPS); }   // fc2 stages: 4 (split) / 8 (bf16) k-steps x 4 tiles
template <int DT>
constexpr int vh_nsd() { return DT == DT_S3 ? 8 : 4; }      // dgrad stages: 4 passes x (2 / 1)

// Counted-wait bookkeeping of an S-stage ring: n counts every vector-memory instruction the wave
// issues; mk[i] the count right after the i-th oldest of the S - 1 pending ring batches.  The sync
// of the oldest pending stage waits with exactly the instructions issued after its batch still in
// flight (vmcnt retires in issue order); an op left uncounted only makes a wait longer.  In
// straight-line code every count folds to a constant.
template <int S>
struct VmQ {
  int n, mk[S - 1];
  // entering with S - 1 pending batches of `batch` instructions each, the newest ending now
  DEV explicit VmQ(int batch) : n(0) {
#pragma unroll
    for (int i = 0; i < S - 1; ++i) mk[i] = -(S - 2 - i) * batch;
  }
  DEV void add(int k) { n += k; }
  DEV int younger() const { return n - mk[0]; }
  // the oldest batch's sync is done; the refill of `k` instructions (0: none) becomes the newest
  DEV void advance(int k) {
    n += k;
#pragma unroll
    for (int i = 0; i + 1 < S - 1; ++i) mk[i] = mk[i + 1];
    mk[S - 2] = n;
  }
};

// t32.h half_sum32 with its per-lane selects as explicit v_cndmask (constant lane masks: the
// lanes with bit m set): written as `up ? v[i] : v[i + m]` the compiler folded the select of two
// array / vector elements into a lane-dependent INDEX and expanded every access as a 32-way compare
// / select chain (~3,700 SGPR spills); a level's 2 m shuffles issue back to back
DEV float vh_sel(float up_v, float lo_v, unsigned long long up_mask) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(lo_v), "v"(up_v), "s"(up_mask));
  return r;
}
DEV float vh_half_sum32(float (&v)[32], int lane) {
  (void)lane;
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) {
    const unsigned long long um = m == 16 ? 0xFFFF0000FFFF0000ull : m == 8 ? 0xFF00FF00FF00FF00ull
                                : m == 4 ? 0xF0F0F0F0F0F0F0F0ull : m == 2 ? 0xCCCCCCCCCCCCCCCCull
                                                                           : 0xAAAAAAAAAAAAAAAAull;
    float got[16];
#pragma unroll
    for (int i = 0; i < m; ++i) got[i] = __shfl_xor(vh_sel(v[i], v[i + m], um), m, 64);
#pragma unroll
    for (int i = 0; i < m; ++i) v[i] = vh_sel(v[i + m], v[i], um) + got[i];
  }
  return v[0];
}

// t32.h ring_mma with a hook after each group's MFMAs: the stage's ring refill (and X) DMAs are
// issued there, one or two per group, instead of as one burst right after the barrier — at one
// wave per SIMD an LDS-DMA instruction's issue (~60 cycles) stalls the wave, and in the burst the
// matrix pipe idles for all of them; between MFMAs each one overlaps the MFMA in flight.  The
// sched_barriers keep every DMA inside its group (the counted waits depend on the issue order).
template <int DT, int N, int G, typename SLOT, typename F, typename HOOK>
DEV void ring_mma_dma(const char* stg, int lane, SLOT&& slot, F&& f, HOOK&& hook) {
  using Frag = typename VT<DT>::Frag;
  constexpr int NG = N / G;
  static_assert(N % G == 0, "groups");
  Frag b[2][G];
  static_for_vh<0, G>([&](auto ic) __attribute__((always_inline)) {
    b[0][decltype(ic)::value] = VT<DT>::ring(stg, slot(decltype(ic)::value), lane);
  });
  static_for_vh<0, NG>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    if constexpr (g + 1 < NG) {
      static_for_vh<0, G>([&](auto ic) __attribute__((always_inline)) {
        b[(g + 1) & 1][decltype(ic)::value] = VT<DT>::ring(stg, slot((g + 1) * G + decltype(ic)::value), lane);
      });
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for_vh<0, G>([&](auto ic) __attribute__((always_inline)) {
      f(g * G + decltype(ic)::value, b[g & 1][decltype(ic)::value]);
    });
    hook(gc, std::integral_constant<int, NG>{});
    __builtin_amdgcn_sched_barrier(0);
  });
}

// phase timeline (diagnostics, scripts/head_timeline.py --vhead): lane 0 of each wave of every
// tstamp_every-th workgroup records the shader clock at the phase boundaries (a vector store no
// counted wait covers: an undercount, safe); real runs take STAMP = false
#define VH_STAMP(i)                                                                               \
  do {                                                                                            \
    if (STAMP && (blockIdx.x % a.tstamp_every) == 0 && lane == 0)                                 \
      a.tstamp[((size_t)(blockIdx.x / a.tstamp_every) * VH_WAVES + wave) * 16 + (i)] =            \
          __builtin_amdgcn_s_memtime();                                                           \
  } while (0)

// TRAIN: the value head's update chain (the loss, its backward through fc3 and fc2, the fused
// narrow-layer weight gradient dW_v; h1 / g1 / g2 stored row-major for the wgrad, csrc/wgrad.hip RM
// operands).  !TRAIN: V(x) into v_out (the GAE input).
template <int DT, bool TRAIN, bool STAMP>
__global__ __launch_bounds__(VH_WAVES * 64, 1) void vhead_kernel(MlpArgs a) {
  using V = VT<DT>;
  using Frag = typename V::Frag;
  constexpr int EB = V::EB, KPS = V::KPS, S = VH_S;
  constexpr bool S3 = DT == DT_S3;
  extern __shared__ __attribute__((aligned(16))) char smem[];   // the kernel's ONLY LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int m0 = blockIdx.x * VH_ROWS;
  const int d1 = a.d_in[3];
  const int ns1 = (d1 >> 4) / KPS;
  char* ring = smem;
  char* xr0 = smem + S * VH_SB;                 // X rings; after fc1 the scratch below
  char* xring = xr0 + wave * (VH_XS * VH_XB);
  float* w3s = reinterpret_cast<float*>(xr0);   // [129] fc3 weights + bias (after fc1)
  float* red = w3s + VH_W3 + 4;                 // [wave][half][64] dW_v partials | [wave] loss

  // the lane's row (rows past M re-read row m0: zero gradient) and, TRAIN, its loss inputs —
  // loaded before any DMA (the oldest vector-memory ops: they never hold up a counted wait)
  const int mr = m0 + 32 * wave + r;
  const bool valid = mr < a.M;
  const int rr = valid ? mr : m0;
  const int srow = a.idx ? a.idx[rr] : a.row0 + rr;
  const bool ref_loss = a.loss_kind != 0;
  float l_ret = 0.f, l_vold = 0.f;
  if constexpr (TRAIN) {
    l_ret = a.ret[srow];
    l_vold = ref_loss ? (a.first_step ? 0.f : a.v_prev[srow]) : a.v_old[srow];
  }
  // this thread's fc3 weight (fp32 from the packed image; zero past the real inputs, the bias at
  // [128]), staged into LDS after fc1
  float w3v = 0.f;
  {
    const int n2 = a.n_out[4], k = tid;
    if (k < n2) w3v = V::img(a.W, (size_t)a.off_w[5] + fm_index(0, k, a.d_in[5]));
    else if (k == VH_W3) w3v = V::img(a.W, (size_t)a.off_w[5] + fm_index(0, n2, a.d_in[5]));
  }

  // ---- DMA sources ----
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), (short)0, 0x7fffffff, 0x00020000);
  // per-lane byte offset of the lane's piece of a 32x16 A fragment in an FM image of c32 = d_in / 32
  // block columns (split: the DMA instruction d carries reader lanes 32 d .. 32 d + 31, its lanes
  // L >= 32 the lo halves)
  auto lane_off = [&](int c32, int d) __attribute__((always_inline)) -> unsigned {
    const int i = lane & 31;
    if constexpr (S3) return (unsigned)(((i >> 4) * c32 * 512 + ((i & 15) + 16 * d) * 8) * 4 + 16 * (lane >> 5));
    else return (unsigned)(((i >> 4) * c32 * 512 + ((i & 15) + 16 * (lane >> 5)) * 8) * 2);
  };
  const int c1 = d1 >> 5, c2 = a.d_in[4] >> 5, c3 = a.d_out[4] >> 5;
  const unsigned vo1[2] = {lane_off(c1, 0), lane_off(c1, 1)};
  const unsigned vo2[2] = {lane_off(c2, 0), lane_off(c2, 1)};
  const unsigned vo3[2] = {lane_off(c3, 0), lane_off(c3, 1)};
  // element offset of the (32-feature tile t, 16-deep k-step k16) fragment of an image (c32 columns)
  auto frag_u = [&](int t, int k16, int c32) __attribute__((always_inline)) {
    return t * 2 * c32 * 512 + (k16 >> 1) * 512 + (k16 & 1) * 256;
  };
  constexpr int NS2 = vh_ns2<DT>(), NSD = TRAIN ? vh_nsd<DT>() : 0, NREST = NS2 + NSD;
  // this wave's 8 ring DMA instructions (of the stage's 32) for stream step st into slot st % S.
  // Slot u of a stage (split: 2 instructions per fragment; bf16: 1):
  //  fc1 stage j (k-steps KPS j ..):  u = tile (split) | tile + 16 e (bf16, k-step KPS j + e)
  //  fc2 stage j (k-steps 4 KPS j ..): u = 4 kk + t (output tile t of the stage's k-step kk)
  //  dgrad stage j (pass p = j / (2 / KPS)): u = 4 kk + t4, h1 tile 4 p + t4 of W2^T k-step
  //    kk (+ 4 for a pass's second split stage)
  // fc1 stages take a runtime index (ns1 = d_in / 16 / KPS); the rest of the stream is unrolled, so
  // its stages are compile-time J = st - ns1 — every DMA's source offset folds to one add
  auto dma = [&](int st, int i, unsigned soff, unsigned voff) __attribute__((always_inline)) {
#ifdef VH_ABL_NODMA
    if (st >= S - 1) return;
#endif
    __attribute__((address_space(3))) char* dst =
        (__attribute__((address_space(3))) char*)(ring + (st % S) * VH_SB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, dst + (VH_GL * wave + i) * 1024, 16, voff, soff, 0, 0);
  };
  // DMA i (0 .. 7) of this wave's batch for fc1 stage st (runtime) / stage ns1 + J (J static)
  auto issue_fc1_i = [&](int st, int i) __attribute__((always_inline)) {
    const int I = VH_GL * wave + i;
    const int u = S3 ? I >> 1 : I, d = S3 ? (I & 1) : 0;
    const int t = S3 ? u : (u & 15), k16 = S3 ? st : 2 * st + (u >> 4);
    dma(st, i, (unsigned)(a.off_w[3] + frag_u(t, k16, c1)) * EB, vo1[d]);
  };
  auto issue_fc1 = [&](int st) __attribute__((always_inline)) {
    // (opaque here, after the sync's asm: the offsets are computed where they are issued instead
    // of being hoisted to the kernel start and held)
    asm volatile("" : "+s"(st));
#pragma unroll
    for (int i = 0; i < VH_GL; ++i) issue_fc1_i(st, i);
  };
  auto issue_rest_i = [&](auto jc, int st, int i) __attribute__((always_inline)) {
    constexpr int J = decltype(jc)::value;
    const int I = VH_GL * wave + i;
    const int u = S3 ? I >> 1 : I, d = S3 ? (I & 1) : 0;
    if constexpr (J < NS2) {
      const int kk = u >> 2, t = u & 3;
      dma(st, i, (unsigned)(a.off_w[4] + frag_u(t, 4 * KPS * J + kk, c2)) * EB, vo2[d]);
    } else {
      constexpr int j = J - NS2, pass = S3 ? j >> 1 : j;
      const int kk = u >> 2, t4 = u & 3, k16 = S3 ? 4 * (j & 1) + kk : kk;
      dma(st, i, (unsigned)(a.off_wt[4] + frag_u(4 * pass + t4, k16, c3)) * EB, vo3[d]);
    }
  };
  const char* xrow = reinterpret_cast<const char*>(a.x_buf) + (size_t)srow * (size_t)d1 * EB;
  // this wave's 2 X DMA instructions of fc1 stage st (split: hi, lo of the k-step; bf16: 2 k-steps)
  auto issue_x_e = [&](int st, int e) __attribute__((always_inline)) {
    char* dx = xring + (st % VH_XS) * VH_XB;
    if constexpr (S3) glds16(xrow + (size_t)(16 * st + 8 * h) * 4 + 16 * e, dx + e * 1024);
    else glds16(xrow + (size_t)(16 * (2 * st + e) + 8 * h) * 2, dx + e * 1024);
  };
  auto issue_x = [&](int st) __attribute__((always_inline)) {
    issue_x_e(st, 0);
    issue_x_e(st, 1);
  };
  auto x_frag = [&](int st, int e) __attribute__((always_inline)) -> Frag {
    const char* xs = xring + (st % VH_XS) * VH_XB;
    if constexpr (S3) {
      return Frag{*reinterpret_cast<const bf16x8*>(xs + 16 * lane), *reinterpret_cast<const bf16x8*>(xs + 1024 + 16 * lane)};
    } else {
      return *reinterpret_cast<const bf16x8*>(xs + e * 1024 + 16 * lane);
    }
  };

  // the loss inputs land before the stream starts (one load latency per workgroup): the asm
  // redefines them, so no compiler-inserted wait for them can fall inside the counted stream —
  // where it would also wait for every in-flight DMA and operand store
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(l_ret), "+v"(l_vold), "+v"(w3v)::"memory");
  // ---- prime: X and ring stages 0 .. S-2 (the launcher checks ns1 >= S) ----
  VH_STAMP(0);
#pragma unroll
  for (int s = 0; s < S - 1; ++s) {
    issue_x(s);
    issue_fc1(s);
  }

  f32x16 acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = f32x16{};

  // one stream step's sync: this wave's DMAs of ring stage st by count (`younger` = its vector
  // memory instructions issued after that stage's batch may stay in flight), then the barrier:
  // every wave's stage st landed, and everyone is done with stage st - 1
  auto sync = [&](int younger) __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    wait_vm_rt(younger);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  constexpr int XB = 2 + VH_GL;   // an fc1 batch: X + ring instructions
  constexpr int SP = S3 ? 2 : 1;  // store instructions per operand fragment
  // fc1 stage st's MFMAs; dma(k) issues DMA k of the batch spread over its groups (k < nd)
  auto fc1 = [&](const char* stg, int st, auto&& dmak, auto ndc) __attribute__((always_inline)) {
    constexpr int ND = decltype(ndc)::value;
    static_for_vh<0, KPS>([&](auto ec) __attribute__((always_inline)) {
      constexpr int e = decltype(ec)::value;
      const Frag xb = x_frag(st, e);
      ring_mma_dma<DT, 16, 2>(stg, lane, [&](int i) { return 16 * e + i; },
                              [&](int i, const Frag& w) __attribute__((always_inline)) { acc[i] = V::mma(acc[i], w, xb); },
                              [&](auto gc, auto ngc) __attribute__((always_inline)) {
                                constexpr int NGT = KPS * decltype(ngc)::value;
                                constexpr int g = e * decltype(ngc)::value + decltype(gc)::value;
                                static_for_vh<g * ND / NGT, (g + 1) * ND / NGT>([&](auto kc) __attribute__((always_inline)) {
                                  dmak(decltype(kc)::value);
                                });
                              });
    });
  };

  // ---- fc1: h1^T (all 512 features of the wave's 32 rows) += W1 . x^T ----
  // steps 0 .. ns1-S: refill fc1 stage st + S - 1 (+ its X); S - 2 batches stay younger
  for (int st = 0; st <= ns1 - S; ++st) {
    sync((S - 2) * XB);
    int sr = st + S - 1;
    asm volatile("" : "+s"(sr));   // (see issue_fc1)
    // the batch of stage st + S - 1: its 2 X DMAs first (older than its weights), then 8 weights
    fc1(ring + (st % S) * VH_SB, st,
        [&](int k) __attribute__((always_inline)) {
          if (k < 2) issue_x_e(sr, k);
          else issue_fc1_i(sr, k - 2);
        },
        std::integral_constant<int, XB>{});
  }
  // from the last S - 1 fc1 steps on, the stream is unrolled: stage ns1 + J (J compile-time,
  // from -(S - 1)) refills stage ns1 + J + S - 1 (no more X); counts by VmQ
  VmQ<S> vq(XB);
  // sync of stage ns1 + J; its refill (stage ns1 + J + S - 1, VH_GL DMAs) is counted here and
  // issued by refill(k) from the stage's MFMA hooks (ring_mma_dma), before any later memory op
  auto sync_late = [&](auto jc) __attribute__((always_inline)) {
    constexpr int J = decltype(jc)::value, JR = J + S - 1;
    sync(vq.younger());
    vq.advance(JR < NREST ? VH_GL : 0);
    return ring + ((ns1 + J) % S) * VH_SB;
  };
  auto refill = [&](auto jc) __attribute__((always_inline)) {
    constexpr int JR = decltype(jc)::value + S - 1;
    return [&, jc](int k) __attribute__((always_inline)) {
      if constexpr (JR < NREST) issue_rest_i(std::integral_constant<int, JR>{}, ns1 + JR, k);
    };
  };
  auto nref = [&](auto jc) __attribute__((always_inline)) {
    constexpr int JR = decltype(jc)::value + S - 1;
    return std::integral_constant<int, (JR < NREST ? VH_GL : 0)>{};
  };
  static_for_vh<1, S>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = S - decltype(ic)::value;     // S - 1 .. 1
    constexpr auto jc = std::integral_constant<int, -i>{};
    const char* stg = sync_late(jc);
    fc1(stg, ns1 - i, refill(jc), nref(jc));
  });
  VH_STAMP(1);
  // h1 = tanh; the bias column (feature n_out[3], in tile 15: vhead_shape_ok) = 1
  auto h1_tanh = [&](int t) __attribute__((always_inline)) {
    acc[t] = tanh16(acc[t]);
    if (t == 15) {
      const int rb = a.n_out[3] & 31, g = (rb & 3) + 4 * (rb >> 3);
      const bool mine = ((rb >> 2) & 1) == h;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = (mine && i == g) ? 1.f : acc[t][i];
    }
  };
#ifndef VH_TANH_SPREAD
#pragma unroll
  for (int t = 0; t < 16; ++t) h1_tanh(t);
#endif
  // the wgrad operands h1 / g1 / g2 in the k16-blocked row-major layout [features / 16][ldT][16]
  // (csrc/wgrad.hip rm < 0): k-step k16's 16 features of the wave's 32 rows are ONE contiguous
  // 1 KiB (bf16) / 2 KiB (split) piece, so a store instruction writes whole cache lines — plain
  // [ldT][512] rows made every 16-byte store instruction touch 32 lines, 32 bytes each, and the
  // stores cost 64 of the kernel's 179 us per call at bf16x3 (profiles/r6).  The lane's byte offset
  // in a block (its row mr, its 8-feature group 8 h; the launcher checks ldT * 512 * EB < 2^31) and
  // the block stride
  const __amdgpu_buffer_rsrc_t rs_h1 = __builtin_amdgcn_make_buffer_rsrc(a.h1vT, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_g1 = __builtin_amdgcn_make_buffer_rsrc(a.g1vT, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_g2 = __builtin_amdgcn_make_buffer_rsrc(a.g2vT, (short)0, 0x7fffffff, 0x00020000);
#ifdef VH_ABL_HOTSTORE
  const unsigned v512 = (unsigned)((32 * wave + r) * 16 + 8 * h) * EB, v128 = v512;
  const unsigned kblk = 0;
#else
  const unsigned v512 = (unsigned)(mr * 16 + 8 * h) * EB, v128 = v512;
  const unsigned kblk = (unsigned)a.ldT * 16u * EB;   // bytes per 16-feature block
#endif
  // an operand store, counted
  auto sto = [&](__amdgpu_buffer_rsrc_t rs, unsigned vrow, unsigned fsoff, const Frag& f) __attribute__((always_inline)) {
#ifndef VH_ABL_NOSTORE
    st_op<DT>(rs, vrow, fsoff, f);
    vq.add(SP);
#endif
  };

  // ---- fc2: h2^T += W2 . h1^T; stage j takes k-steps 4 KPS j .. (h1 tiles 2 KPS j ..); their B
  // operands — also the h1 operand stores — before the wait ----
  f32x16 acc2[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc2[t] = f32x16{};
  static_for_vh<0, NS2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    constexpr int NB = 4 * KPS;    // k-steps of the stage
#ifdef VH_TANH_SPREAD
    // (the tanh of stage j's tiles in the shadow of stage j - 1's MFMAs)
#pragma unroll
    for (int tt = 0; tt < NB / 2; ++tt) h1_tanh(NB / 2 * j + tt);
#endif
    Frag b[NB];
#pragma unroll
    for (int e = 0; e < NB; ++e) {
      const int k16 = NB * j + e;
      b[e] = b_operand<DT>(acc[k16 >> 1], k16 & 1);
#ifndef VH_LATE_STORE
      if constexpr (TRAIN) sto(rs_h1, v512, k16 * kblk, b[e]);
#endif
    }
    constexpr auto jc2 = std::integral_constant<int, j>{};
    const char* stg = sync_late(jc2);
    if constexpr (j == 0) {
      // the fc3 weights into the freed X rings: past this barrier every wave is done with fc1
      if (tid <= VH_W3) w3s[tid] = w3v;
    }
    constexpr int ND = decltype(nref(jc2))::value;
    auto rf = refill(jc2);
    ring_mma_dma<DT, 4 * NB, (S3 ? 2 : 4)>(stg, lane, [&](int i) { return i; },
                                          [&](int i, const Frag& w) __attribute__((always_inline)) {
                                            acc2[i & 3] = V::mma(acc2[i & 3], w, b[i >> 2]);
                                          },
                                          [&](auto gc, auto ngc) __attribute__((always_inline)) {
                                            constexpr int g = decltype(gc)::value, NG = decltype(ngc)::value;
                                            static_for_vh<g * ND / NG, (g + 1) * ND / NG>([&](auto kc) __attribute__((always_inline)) {
                                              rf(decltype(kc)::value);
                                            });
                                          });
#ifdef VH_LATE_STORE
#pragma unroll
    for (int e = 0; e < NB; ++e)
      if constexpr (TRAIN) sto(rs_h1, v512, (NB * j + e) * kblk, b[e]);
#endif
  });
  VH_STAMP(2);
  // ---- h2 = tanh (the bias column n_out[4] = 1), fc3 on the VALU (fp32): v = b3 + sum_k w3[k] h2[k] ----
  {
    // (n_out[4] in 97 .. 111: tile 3, vhead_shape_ok)
    const int rb = a.n_out[4] & 31, g = (rb & 3) + 4 * (rb >> 3);
    const bool mine = ((rb >> 2) & 1) == h;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc2[t] = tanh16(acc2[t]);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc2[3][i] = (mine && i == g) ? 1.f : acc2[3][i];
  }
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(w3s + 32 * t + 8 * g + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) part = __builtin_fmaf(w[i], acc2[t][4 * g + i], part);
    }
  }
  // (the bias column's weight is b3: h2[n2] = 1 carries it, w3s[n2] = 0 past the real inputs)
  const float v = w3s[VH_W3] + (part + __shfl_xor(part, 32, 64));
  if constexpr (!TRAIN) {
    if (h == 0 && valid) a.v_out[mr] = v;
    VH_STAMP(7);
    WAIT_VMCNT(0);   // (nothing of the ring in flight: the stream ended with fc2)
    return;
  } else {
    // ---- the value loss (ppo.py:164 mse | train.py:154-157 clipped, x 1/2) and dL/dv ----
    float lv, dv;
    {
      const float vold = ref_loss && a.first_step ? v : l_vold;
      if (a.value_loss == 0) {
        const float d = v - l_ret;
        lv = d * d;
        dv = 2.f * d;
      } else {
        const float d1v = v - l_ret, dd = v - vold;
        const float vc = vold + fminf(fmaxf(dd, -a.clip), a.clip);
        const float d2v = vc - l_ret;
        const float f1 = d1v * d1v, f2 = d2v * d2v;
        const float inr = (dd >= -a.clip && dd <= a.clip) ? 1.f : 0.f;
        lv = 0.5f * fmaxf(f1, f2);
        dv = f1 > f2 ? d1v : (f2 > f1 ? d2v * inr : 0.5f * d1v + 0.5f * d2v * inr);
      }
      if (ref_loss && valid && h == 0) a.v_prev[srow] = v;   // train.py:164 model_old <- model
      dv = valid ? dv : 0.f;
      lv = valid ? lv : 0.f;
    }
    // (the v_prev store is left out of the counts: an undercount only waits longer)
    // the fused v-layer weight gradient over the wave's 32 rows: dW_v[k] = sum_r dL/dv[r] h2b[r][k]
    // (h2b: h2 with the bias column n2 = 1, already set above), two half-wave butterflies of 32
    // values (tiles 0-1, 2-3); lane r of half h ends with value r of each
    {
#pragma unroll
      for (int hv = 0; hv < 2; ++hv) {
        float x[32];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int i = 0; i < 16; ++i) x[16 * tt + i] = dv * acc2[2 * hv + tt][i];
        red[(wave * 2 + h) * 64 + 32 * hv + r] = vh_half_sum32(x, lane);
      }
      float l = h == 0 ? lv : 0.f;
#pragma unroll
      for (int m = 1; m < 32; m <<= 1) l += __shfl_xor(l, m, 64);
      if (lane == 0) red[VH_WAVES * 2 * 64 + wave] = l;
    }
    // g2 = dL/dv w3 (1 - h2^2) (zero past n2: w3s is), its B operands (7 k-steps used by the dgrad;
    // the 8th — features 112-127, past n2 <= 111 — is zero) and the g2 operand stores
    Frag gb[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 g2;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(w3s + 32 * t + 8 * g + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float hv = acc2[t][4 * g + i];
          g2[4 * g + i] = dv * w[i] * __builtin_fmaf(-hv, hv, 1.f);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) gb[2 * t + s] = b_operand<DT>(g2, s);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) sto(rs_g2, v128, k * kblk, gb[k]);

    VH_STAMP(3);
    // ---- dgrad fc2: g1 = (W2^T g2) (1 - h1^2), 4 passes of 4 h1 tiles; each pass's g1 operand
    // stores ride along ----
    constexpr int SPP = S3 ? 2 : 1;   // ring stages per pass
    static_for_vh<0, 4>([&](auto pc) __attribute__((always_inline)) {
      constexpr int p = decltype(pc)::value;
      f32x16 ga[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) ga[t] = f32x16{};
      static_for_vh<0, SPP>([&](auto sc) __attribute__((always_inline)) {
        constexpr int sp = decltype(sc)::value;
        constexpr auto jcd = std::integral_constant<int, NS2 + SPP * p + sp>{};
        const char* stg = sync_late(jcd);
        constexpr int NK = S3 ? (sp == 0 ? 4 : 3) : 7;   // k-steps computed (the 8th is zero)
        constexpr int ND = decltype(nref(jcd))::value;
        auto rf = refill(jcd);
        ring_mma_dma<DT, 4 * NK, (S3 ? 2 : 4)>(stg, lane, [&](int i) { return i; },
                                              [&](int i, const Frag& w) __attribute__((always_inline)) {
                                                ga[i & 3] = V::mma(ga[i & 3], w, gb[4 * sp + (i >> 2)]);
                                              },
                                              [&](auto gc, auto ngc) __attribute__((always_inline)) {
                                                constexpr int g = decltype(gc)::value, NG = decltype(ngc)::value;
                                                static_for_vh<g * ND / NG, (g + 1) * ND / NG>([&](auto kc) __attribute__((always_inline)) {
                                                  rf(decltype(kc)::value);
                                                });
                                              });
      });
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4) {
        const int t = 4 * p + t4;
        f32x16 g1;
#pragma unroll
        for (int i = 0; i < 16; ++i) g1[i] = ga[t4][i] * __builtin_fmaf(-acc[t][i], acc[t][i], 1.f);
#pragma unroll
        for (int s = 0; s < 2; ++s) sto(rs_g1, v512, (2 * t + s) * kblk, b_operand<DT>(g1, s));
      }
      if constexpr (p == 1) VH_STAMP(4);
      if constexpr (p == 2) VH_STAMP(5);
    });
    VH_STAMP(6);
    // ---- per-workgroup partials (fixed order): the value loss (column 1) and dW_v ----
    // (no DMA is in flight: the last stage's sync waited for all of them; the operand stores may
    // drain after the waves end)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float* dst = a.part + (size_t)blockIdx.x * a.npart;
    if (tid < 128) {
      const int k = tid, t = k >> 5, rr2 = k & 31;
      const int hh = (rr2 >> 2) & 1, i = (rr2 & 3) + 4 * (rr2 >> 3);
      const int j = 16 * t + i;
      float sv = 0.f;
#pragma unroll
      for (int w = 0; w < VH_WAVES; ++w) sv += red[(w * 2 + hh) * 64 + j];
      dst[a.part_dw + k] = sv;
    } else if (tid == 128) {
      const float* lw = red + VH_WAVES * 2 * 64;
      dst[1] = ((lw[0] + lw[1]) + lw[2]) + lw[3];
    }
    VH_STAMP(7);
  }
}

int g_vhead = 1;

}  // namespace

// the shapes the kernel covers: the reference value head (500 -> 100 -> 1; observation widths
// 64 .. 384 that are a multiple of 32 with at least S fc1 stages)
extern "C" int vhead_shape_ok(const MlpArgs& a) {
  return a.d_in[3] % 32 == 0 && a.d_in[3] >= 128 && a.d_in[3] <= 384 && a.d_out[3] == 512 &&
         a.n_out[3] >= 481 && a.n_out[3] < 512 && a.d_in[4] == 512 && a.d_out[4] == 128 && a.n_out[4] <= 111 &&
         a.n_out[4] >= 97 && a.d_in[5] == 128 && (a.d_in[3] >> 4) % 2 == 0;
}

extern "C" int vhead_applies(const MlpArgs& a) { return g_vhead && vhead_shape_ok(a); }

extern "C" int vhead_rows() { return VH_ROWS; }

template <int DT, bool TRAIN>
void vhead_launch_t(const MlpArgs& a, hipStream_t s) {
  const int nblk = (a.M + VH_ROWS - 1) / VH_ROWS;
  if (a.tstamp != nullptr) {
    set_max_lds_once<vhead_kernel<DT, TRAIN, true>>(vh_lds_bytes());
    hipLaunchKernelGGL((vhead_kernel<DT, TRAIN, true>), dim3(nblk), dim3(VH_WAVES * 64), vh_lds_bytes(), s, a);
  } else {
    set_max_lds_once<vhead_kernel<DT, TRAIN, false>>(vh_lds_bytes());
    hipLaunchKernelGGL((vhead_kernel<DT, TRAIN, false>), dim3(nblk), dim3(VH_WAVES * 64), vh_lds_bytes(), s, a);
  }
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_vhead_fwd(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_S3) vhead_launch_t<DT_S3, false>(a, s);
  else vhead_launch_t<DT_BF16, false>(a, s);
}

// the update chain (a.part / part_dw / the row-major h1vT, g1vT, g2vT operands; csrc/kernels.h)
extern "C" void launch_vhead_train(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_S3) vhead_launch_t<DT_S3, true>(a, s);
  else vhead_launch_t<DT_BF16, true>(a, s);
}

extern "C" void set_vhead(int enable) { g_vhead = enable ? 1 : 0; }
