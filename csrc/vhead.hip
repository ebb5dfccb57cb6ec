// Value head on 32x32x16 MFMAs in the TRANSPOSED chain (model.py:42-44 forward,
// train.py:109-112 GAE input).
//
// Every layer computes out^T = W . in^T:  A = a weight fragment (32 output features x 16 k, from
// the LDS ring, shared by all waves of the workgroup), B = the activations (16 k x 32 batch rows,
// in registers).  The 32x32 accumulator has the batch row on the lane and 16 output features in
// its registers (col = lane & 31, feature (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)), which is
// already the NEXT layer's B operand up to one v_permlane32_swap per dword: no LDS transpose
// anywhere in the chain (csrc/mlp_head.hip stages every layer's activations through [16][36] LDS
// tiles).  Against the 16x16x32 row-stationary head kernel the 32x32 form also halves the LDS
// weight-fragment bytes per MAC (one 32x16 fragment feeds 32x32 outputs, not 16x16).
//
// Workgroup: 8 waves = 4 PAIRS x 32 rows (128 rows).  Wave w = (pair p = w & 3, half q = w >> 2)
// holds fc1 features 256 q .. 256 q + 255 of its pair's 32 rows (8 accumulator tiles = 128
// registers): the pair splits fc1's N, so each wave reads only its 8 of a stage's 16 fragments
// (half the LDS reads of one wave holding all 512 features), and splits fc2's K the same way —
// each wave's fc2 is a partial sum over its own h1 half, the pair adds the two partials through
// LDS in a fixed order (both get identical sums), then fc3 (1 output) runs on the VALU in fp32.
// Two waves per SIMD (waves w and w + 4 share one: a pair), <= 256 registers each.
//
// Weights stream through an S-stage LDS ring of 32 KiB stages (32 LDS-DMA instructions of 1 KiB,
// 4 per wave) straight from the packed FM images (csrc/common.h fm_index): a 32x16 A fragment is
// four 256-byte pieces of two 16x32 FM blocks, gathered by per-lane DMA source offsets, landing
// lane-linear.  Observation rows: per pair a 2 KiB X slot per stage, its two DMA instructions
// split between the pair's waves (64-bit per-lane row addresses: any buffer size).  Counted vmcnt
// waits + a raw s_barrier per stage (cdna_hip_programming.md 'Pipelining across barriers').
#include "t32.h"

namespace {

using namespace t32;

constexpr int VH_ROWS = 128;            // rows per workgroup
constexpr int VH_WAVES = 8;
constexpr int VH_SB = 32 * 1024;        // ring stage bytes
constexpr int VH_S = 3;                 // ring stages
constexpr int VH_XS = 3;                // X slots per pair (>= VH_S: X of stage k is older than its weight batch)
constexpr int VH_XB = 2048;             // X bytes per pair and stage
constexpr int VH_GL = 4;                // ring DMA instructions per wave and stage
constexpr int VH_W3 = 128;              // fc3 weights staged in LDS (fp32, zero past n_out[4])
constexpr int VH_SCR = 32 * 1024;       // X ring (fc1) / pair-sum scratch: 8 waves x one 4 KiB tile

constexpr size_t vh_lds_bytes() { return (size_t)VH_S * VH_SB + VH_SCR + (VH_W3 + 4) * sizeof(float); }
static_assert(vh_lds_bytes() <= 160 * 1024, "value head LDS");
static_assert(4 * VH_XS * VH_XB <= VH_SCR && VH_WAVES * 16 * 64 * 4 <= VH_SCR && (512 + 4) * 4 <= VH_SCR,
              "X ring / pair-sum tile / reductions fit the scratch");

// fc1 stages: d_in / 16 k-steps, KPS per stage; fc2: 512 / 16 = 32 k-steps, 4 tiles each,
// 4 (split) / 8 (bf16) k-steps per stage
template <int DT>
DEV int vh_ns1(int d_in) { return (d_in >> 4) / VT<DT>::KPS; }
template <int DT> constexpr int vh_nsd();
template <int DT>
constexpr int vh_ns2() { return 32 / (4 * VT<DT>::KPS); }
// dgrad fc2 stages: 4 passes of 2 h1 tiles per wave over the 8 W2^T k-steps (h2 features 0-127)
template <int DT>
constexpr int vh_nsd() { return DT == DT_S3 ? 8 : 4; }

// phase timeline (diagnostics, scripts/head_timeline.py --vhead): lane 0 of each wave of every
// tstamp_every-th workgroup records the shader clock at the phase boundaries (a vector store no
// counted wait covers: an undercount, safe); null in real runs
#define VH_STAMP(i)                                                                               \
  do {                                                                                            \
    if (STAMP && (blockIdx.x % a.tstamp_every) == 0 && lane == 0)                                 \
      a.tstamp[((size_t)(blockIdx.x / a.tstamp_every) * VH_WAVES + wave) * 16 + (i)] =            \
          __builtin_amdgcn_s_memtime();                                                           \
  } while (0)

// TRAIN: the value head's update chain (the loss of train.py:154-157 / ppo.py:164, its backward
// through fc3 and fc2; the fused narrow-layer weight gradient dW_v; h1 / g1 / g2 stored row-major
// for the wgrad, csrc/wgrad.hip RM operands).  !TRAIN: V(x) into v_out (the GAE input).
// STAMP: the diagnostic instantiation with the phase stamps (a.tstamp set); real runs take STAMP = false
template <int DT, bool TRAIN, bool STAMP>
__global__ __launch_bounds__(VH_WAVES * 64, 1) void vhead_kernel(MlpArgs a) {
  using V = VT<DT>;
  using Frag = typename V::Frag;
  constexpr int EB = V::EB, KPS = V::KPS;
  extern __shared__ __attribute__((aligned(16))) char smem[];   // the kernel's ONLY LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = wave & 3, q = wave >> 2;
  const int h = lane >> 5, r = lane & 31;
  const int m0 = blockIdx.x * VH_ROWS;
  const int d1 = a.d_in[3];
  const int ns1 = vh_ns1<DT>(d1);
  char* ring = smem;
  char* scr0 = smem + VH_S * VH_SB;   // X ring (fc1), then the pair-sum / reduction scratch
  char* xring = scr0 + p * (VH_XS * VH_XB);
  float* w3s = reinterpret_cast<float*>(smem + VH_S * VH_SB + VH_SCR);

  // the lane's row (rows past M re-read row m0: zero gradient) and, TRAIN, its loss inputs —
  // loaded before any DMA (the oldest vector-memory ops: they never hold up a counted wait)
  const int mr = m0 + 32 * p + r;
  const bool valid = mr < a.M;
  const int rr = valid ? mr : m0;
  const int srow = a.idx ? a.idx[rr] : a.row0 + rr;
  const bool ref_loss = a.loss_kind != 0;
  float l_ret = 0.f, l_vold = 0.f;
  if constexpr (TRAIN) {
    l_ret = a.ret[srow];
    l_vold = ref_loss ? (a.first_step ? 0.f : a.v_prev[srow]) : a.v_old[srow];
  }
  // fc3 weights (fp32 from the packed image; zero past the real inputs) + bias
  {
    const int n2 = a.n_out[4];
    for (int k = tid; k <= VH_W3; k += VH_WAVES * 64) {
      float w = 0.f;
      if (k < n2) w = V::img(a.W, (size_t)a.off_w[5] + fm_index(0, k, a.d_in[5]));
      else if (k == VH_W3) w = V::img(a.W, (size_t)a.off_w[5] + fm_index(0, n2, a.d_in[5]));
      w3s[k] = w;
    }
  }

  // ---- DMA sources ----
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), (short)0, 0x7fffffff, 0x00020000);
  // per-lane byte offset of the lane's piece of a 32x16 A fragment in an FM image of c32 = d_in / 32
  // block columns (split: the DMA instruction d carries reader lanes 32 d .. 32 d + 31, its lanes
  // L >= 32 the lo halves)
  auto lane_off = [&](int c32, int d) __attribute__((always_inline)) -> unsigned {
    const int i = lane & 31;
    if constexpr (DT == DT_S3) return (unsigned)(((i >> 4) * c32 * 512 + ((i & 15) + 16 * d) * 8) * 4 + 16 * (lane >> 5));
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
  // this wave's 4 ring DMA instructions (of the stage's 32) for stream step st, into ring slot st % S:
  //  fc1 stage j (k-steps KPS j ..): slot u = tile (split) | tile + 16 e (bf16, k-step e)
  //  fc2 stage j: slot u = 4 kk + t, output tile t of the stage's k-step kk; the stage takes 2 KPS
  //    k-steps from each h1 half (kk / (2 KPS) = the half), so both waves of a pair compute
  //  dgrad stage j (pass i = j / (2 / KPS)): slot u = 4 kk + t4, h1 tile (t4 >> 1) * 8 + 2 i + (t4 & 1)
  //    (wave q takes t4 = 2 q, 2 q + 1) of the W2^T k-step kk (+ 4 for the second split stage)
  auto issue = [&](int st) __attribute__((always_inline)) {
    __attribute__((address_space(3))) char* dst =
        (__attribute__((address_space(3))) char*)(ring + (st % VH_S) * VH_SB);
#pragma unroll
    for (int i = 0; i < VH_GL; ++i) {
      const int I = VH_GL * wave + i;   // 1 KiB DMA instruction of the stage
      const int u = DT == DT_S3 ? I >> 1 : I, d = DT == DT_S3 ? (I & 1) : 0;
      unsigned soff, voff;
      if (st < ns1) {
        const int t = DT == DT_S3 ? u : (u & 15), k16 = DT == DT_S3 ? st : 2 * st + (u >> 4);
        soff = (unsigned)(a.off_w[3] + frag_u(t, k16, c1)) * EB;
        voff = vo1[d];
      } else if (st < ns1 + vh_ns2<DT>()) {
        const int j = st - ns1, kk = u >> 2, t = u & 3;
        const int k16 = (kk / (2 * KPS)) * 16 + 2 * KPS * j + (kk % (2 * KPS));
        soff = (unsigned)(a.off_w[4] + frag_u(t, k16, c2)) * EB;
        voff = vo2[d];
      } else {
        const int j = st - ns1 - vh_ns2<DT>(), kk = u >> 2, t4 = u & 3;
        const int pass = DT == DT_S3 ? j >> 1 : j, k16 = DT == DT_S3 ? 4 * (j & 1) + kk : kk;
        const int tile = (t4 >> 1) * 8 + 2 * pass + (t4 & 1);
        soff = (unsigned)(a.off_wt[4] + frag_u(tile, k16, c3)) * EB;
        voff = vo3[d];
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, dst + I * 1024, 16, voff, soff, 0, 0);
    }
  };
  const char* xrow = reinterpret_cast<const char*>(a.x_buf) + (size_t)srow * (size_t)d1 * EB;
  // this wave's DMA instruction (q) of the pair's X slot of fc1 stage st
  auto issue_x = [&](int st) __attribute__((always_inline)) {
    char* d = xring + (st % VH_XS) * VH_XB + q * 1024;
    if constexpr (DT == DT_S3) glds16(xrow + (size_t)(16 * st + 8 * h) * 4 + 16 * q, d);
    else glds16(xrow + (size_t)(16 * (2 * st + q) + 8 * h) * 2, d);
  };
  auto x_frag = [&](int st, int e) __attribute__((always_inline)) -> Frag {
    const char* xs = xring + (st % VH_XS) * VH_XB;
    if constexpr (DT == DT_S3) {
      return Frag{*reinterpret_cast<const bf16x8*>(xs + 16 * lane), *reinterpret_cast<const bf16x8*>(xs + 1024 + 16 * lane)};
    } else {
      return *reinterpret_cast<const bf16x8*>(xs + e * 1024 + 16 * lane);
    }
  };

  constexpr int NS2 = vh_ns2<DT>(), NSD = TRAIN ? vh_nsd<DT>() : 0;
  const int ntot = ns1 + NS2 + NSD;
  // the loss inputs land before the stream starts (one load latency per workgroup): the asm
  // redefines them, so no compiler-inserted wait for them can fall inside the counted stream —
  // where it would also wait for every in-flight DMA and operand store
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(l_ret), "+v"(l_vold)::"memory");
  // ---- prime: X stages 0, 1 and ring stages 0, 1 (the launcher checks ns1 >= 3) ----
  static_assert(VH_S == 3 && VH_XS == 3, "the wait counts below are written for 3-stage rings");
  VH_STAMP(0);
  issue_x(0);
  issue_x(1);
  issue(0);
  issue(1);

  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  f32x16 acc2[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc2[t] = f32x16{};

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
  // from the last two fc1 steps on: the counts by VmTrack (entering with stage ns1 - 2's batch
  // X(ns1 - 1) + R(ns1 - 1) back)
  VmTrack vt(1 + VH_GL);
  constexpr int SP = DT == DT_S3 ? 2 : 1;   // store instructions per operand fragment
  auto sync_t = [&](int st) __attribute__((always_inline)) {
    sync(vt.younger());
    const bool refill = st + 2 < ntot;
    if (refill) issue(st + 2);
    vt.advance(refill ? VH_GL : 0);
  };
  auto sync_late = [&](int st) __attribute__((always_inline)) {
    sync_t(st);
    return ring + (st % VH_S) * VH_SB;
  };
  // an operand store, counted
  auto sto = [&](__amdgpu_buffer_rsrc_t rs, unsigned vrow, unsigned fsoff, const Frag& f) __attribute__((always_inline)) {
    st_op<DT>(rs, vrow, fsoff, f);
    vt.add(SP);
  };
  constexpr int G1 = DT == DT_S3 ? 2 : 4;   // fragments per LDS read group (<= 8 reads in flight)
  auto fc1 = [&](const char* stg, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < KPS; ++e) {
      const Frag xb = x_frag(st, e);
      ring_mma<DT, 8, G1>(stg, lane, [&](int i) { return 16 * e + 8 * q + i; },
                          [&](int i, const Frag& w) __attribute__((always_inline)) { acc[i] = V::mma(acc[i], w, xb); });
    }
  };

  // ---- fc1: h1^T (this wave's 256 features) += W1 . x^T ----
  // steps 0 .. ns1-3 issue X(st + 2) and fc1 stage st + 2; step 0 waits with R(1) younger
  for (int st = 0; st < ns1 - 2; ++st) {
    sync(st == 0 ? VH_GL : 1 + VH_GL);
    issue_x(st + 2);
    issue(st + 2);
    fc1(ring + (st % VH_S) * VH_SB, st);
  }
  // the last two fc1 steps refill with fc2 stages 0, 1 (no more X)
  sync_t(ns1 - 2);
  fc1(ring + ((ns1 - 2) % VH_S) * VH_SB, ns1 - 2);
  sync_t(ns1 - 1);
  fc1(ring + ((ns1 - 1) % VH_S) * VH_SB, ns1 - 1);
  VH_STAMP(1);
  {
    // h1 = tanh, the bias column (feature n_out[3]) = 1
    const int nb = a.n_out[3] - 256 * q, tb = nb >> 5, rb = nb & 31;
    const int g = (rb & 3) + 4 * (rb >> 3);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      acc[t] = tanh16(acc[t]);
      if (t == tb && ((rb >> 2) & 1) == h) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i == g) acc[t][i] = 1.f;
      }
    }
  }
  // row-major operand rows of this lane (the minibatch position mr is the wgrad's k; the launcher
  // checks ldT * 512 * EB < 2^31): its byte offset + its 8-feature group (8 h)
  const __amdgpu_buffer_rsrc_t rs_h1 = __builtin_amdgcn_make_buffer_rsrc(a.h1vT, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_g1 = __builtin_amdgcn_make_buffer_rsrc(a.g1vT, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_g2 = __builtin_amdgcn_make_buffer_rsrc(a.g2vT, (short)0, 0x7fffffff, 0x00020000);
  const unsigned v512 = (unsigned)(mr * 512 + 8 * h) * EB, v128 = (unsigned)(mr * 128 + 8 * h) * EB;
  // ---- fc2: this wave's partial h2^T over its h1 half (the k-steps e of a stage's share: h1 tile
  // KPS j + e / 2, half e & 1; their B operands — also the h1 operand stores — before the wait) ----
  static_for_vh<0, NS2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    Frag b[2 * KPS];
#pragma unroll
    for (int e = 0; e < 2 * KPS; ++e) {
      b[e] = b_operand<DT>(acc[KPS * j + (e >> 1)], e & 1);
      if constexpr (TRAIN) sto(rs_h1, v512, (256 * q + 32 * (KPS * j + (e >> 1)) + 16 * (e & 1)) * EB, b[e]);
    }
    const char* stg = sync_late(ns1 + j);
    // (fc2 holds h1 and the fc2 accumulators: one / two fragments per read group)
    ring_mma<DT, 8 * KPS, (DT == DT_S3 ? 1 : 2)>(stg, lane, [&](int i) { return 4 * (2 * KPS * q + (i >> 2)) + (i & 3); },
                              [&](int i, const Frag& w) __attribute__((always_inline)) {
                                acc2[i & 3] = V::mma(acc2[i & 3], w, b[i >> 2]);
                              });
  });

  VH_STAMP(2);
  // ---- the pair's two fc2 partials, summed in a fixed order (both waves get the same bits), one
  // tile per round through the scratch (the X ring is idle; raw barriers: the dgrad stream stays
  // in flight) ----
  f32x4* scr = reinterpret_cast<f32x4*>(scr0);
  auto bar = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      scr[(wave * 4 + g) * 64 + lane] = f32x4{acc2[t][4 * g], acc2[t][4 * g + 1], acc2[t][4 * g + 2], acc2[t][4 * g + 3]};
    bar();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 o = scr[((wave ^ 4) * 4 + g) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc2[t][4 * g + i] += o[i];
    }
    bar();
  }
  VH_STAMP(3);
  // ---- h2 = tanh, fc3 on the VALU (fp32): v = b3 + sum_k w3[k] h2[k] ----
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc2[t] = tanh16(acc2[t]);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(w3s + 32 * t + 8 * g + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) part = __builtin_fmaf(w[i], acc2[t][4 * g + i], part);
    }
  }
  const float v = w3s[VH_W3] + (part + __shfl_xor(part, 32, 64));
  if constexpr (!TRAIN) {
    if (q == 0 && h == 0 && valid) a.v_out[mr] = v;
    VH_STAMP(7);
    WAIT_VMCNT(0);   // (nothing in flight: the stream ended with fc2)
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
      if (ref_loss && valid && q == 0 && h == 0) a.v_prev[srow] = v;   // train.py:164 model_old <- model
      dv = valid ? dv : 0.f;
      lv = valid ? lv : 0.f;
    }
    // the fused v-layer weight gradient over the pair's 32 rows, this wave's tiles 2q, 2q+1:
    // dW_v[k] = sum_r dL/dv[r] h2b[r][k] (h2b: h2 with the bias column n2 = 1)
    const int n2 = a.n_out[4];
    float* red = reinterpret_cast<float*>(scr0);   // [pair][q][h][32] dW_v partials | [pair] loss
    {
      float x[32];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int f = 32 * (2 * q + tt) + (i & 3) + 8 * (i >> 2) + 4 * h;
          x[16 * tt + i] = f == n2 ? dv : dv * (q == 0 ? acc2[tt][i] : acc2[2 + tt][i]);
        }
      red[((p * 2 + q) * 2 + h) * 32 + r] = half_sum32(x, lane);
      float l = (q == 0 && h == 0) ? lv : 0.f;
#pragma unroll
      for (int m = 1; m < 32; m <<= 1) l += __shfl_xor(l, m, 64);
      if (q == 0 && lane == 0) red[512 + p] = l;
    }
    // g2 = dL/dv w3 (1 - h2^2) (zero past n2: w3s is), its B operands (7 k-steps used by dgrad;
    // the 8th is zero) and the g2 operand stores (wave q: k-steps 4q .. 4q + 3)
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
    // (unconditional stores of a selected fragment: the counted waits stay compile-time constants)
#pragma unroll
    for (int k = 0; k < 4; ++k) sto(rs_g2, v128, 16 * (4 * q + k) * EB, q ? gb[4 + k] : gb[k]);

    VH_STAMP(4);
    // ---- dgrad fc2: g1 = (W2^T g2) (1 - h1^2) over this wave's h1 tiles, two per pass ----
    constexpr int SPP = DT == DT_S3 ? 2 : 1;   // ring stages per pass
    constexpr int GD = DT == DT_S3 ? 1 : 2;    // fragments per read group (registers)
    static_for_vh<0, 4>([&](auto ic) __attribute__((always_inline)) {
      constexpr int ip = decltype(ic)::value;
      f32x16 ga[2] = {f32x16{}, f32x16{}};
      static_for_vh<0, SPP>([&](auto sc) __attribute__((always_inline)) {
        constexpr int sp = decltype(sc)::value;
        const char* stg = sync_late(ns1 + NS2 + SPP * ip + sp);
        constexpr int NK = DT == DT_S3 ? (sp == 0 ? 4 : 3) : 7;   // k-steps computed (the 8th is zero)
        ring_mma<DT, 2 * NK, GD>(stg, lane, [&](int i) { return 4 * (i >> 1) + 2 * q + (i & 1); },
                                 [&](int i, const Frag& w) __attribute__((always_inline)) {
                                   ga[i & 1] = V::mma(ga[i & 1], w, gb[4 * sp + (i >> 1)]);
                                 });
      });
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const f32x16 hv = acc[2 * ip + tt];
        f32x16 g1;
#pragma unroll
        for (int i = 0; i < 16; ++i) g1[i] = ga[tt][i] * __builtin_fmaf(-hv[i], hv[i], 1.f);
#pragma unroll
        for (int s = 0; s < 2; ++s)
          sto(rs_g1, v512, (256 * q + 32 * (2 * ip + tt) + 16 * s) * EB, b_operand<DT>(g1, s));
      }
      if constexpr (ip == 1) VH_STAMP(5);
    });
    VH_STAMP(6);
    // ---- per-workgroup partials (fixed order): the value loss (column 1) and dW_v ----
    // (no DMA is in flight: the last stage's sync waited for all of them; the operand stores may
    // drain after the waves end)
    float* dst = a.part + (size_t)blockIdx.x * a.npart;
    if (tid < 128) {
      const int k = tid, t = k >> 5, rr2 = k & 31;
      const int hh = (rr2 >> 2) & 1, i = (rr2 & 3) + 4 * (rr2 >> 3);
      float sv = 0.f;
#pragma unroll
      for (int pp = 0; pp < 4; ++pp) sv += red[((pp * 2 + (t >> 1)) * 2 + hh) * 32 + 16 * (t & 1) + i];
      dst[a.part_dw + k] = sv;
    } else if (tid == 128) {
      dst[1] = ((red[512] + red[513]) + red[514]) + red[515];
    }
    VH_STAMP(7);
  }
}

int g_vhead = 1;

}  // namespace

// the shapes the kernel covers: the reference value head (500 -> 100 -> 1; any observation width
// <= 384 that is a multiple of 32)
extern "C" int vhead_shape_ok(const MlpArgs& a) {
  return a.d_in[3] % 32 == 0 && a.d_in[3] >= 96 && a.d_in[3] <= 384 && a.d_out[3] == 512 &&
         a.n_out[3] >= 257 && a.n_out[3] < 512 && a.d_in[4] == 512 && a.d_out[4] == 128 && a.n_out[4] <= 127 &&
         a.d_in[5] == 128 && (a.d_in[3] >> 4) % 2 == 0;
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
