// Policy head update on 32x32x16 MFMAs in the TRANSPOSED chain (model.py:36-41
// forward, ppo.py:148-167 corrected loss, train.py:142-161 reference loss; the update of
// train.py:162-170 / ppo.py:168-175 consumes its outputs).
//
// The transposed chain (helpers in csrc/t32.h) on the narrow policy network
// (d0 -> 100 -> 100 -> A): every layer computes out^T = W . in^T with A = a 32x16 weight fragment
// from the LDS ring and B = the activations in registers (batch row on the lane); each wave owns
// 32 rows and ALL 128 (padded) features of both hidden layers (4 accumulator tiles each).
// Workgroup: 4 waves x 32 rows, two workgroups per CU (<= 80 KiB LDS, <= 256 registers), so one
// workgroup's loss / reduction phases overlap the other's MFMA stream.
//
// Weight stream (one 3-stage LDS ring of 8 KiB stages, 2 DMA instructions per wave per stage):
//   fc1 (d0 / 16 k-steps) | fc2 (7 / 4 stages) | mu (2 / 1) | dgrad mu: W3^T (2 / 1) |
//   dgrad fc2: W2^T, 2 passes of 2 h1 tiles (8 / 4)     (split-bf16 / bf16 stage counts)
// Observation rows: a per-wave 3-slot X ring (2 KiB per k-step stage).
//
// Outputs (TRAIN only — the rollout kernel computes the policy forward):
//   * the row-major wgrad operand g1 [ldT][128] (csrc/wgrad.hip RM reads) and, for a minibatch
//     (idx != null, !xT_ready), the observation rows [ldT][d0]
//     (full-batch calls: the wgrad reads x_buf itself — no x^T copy anywhere);
//   * per-workgroup partials: loss terms (columns 0, 2-7), dlog_std (8 + j), the mu layer's weight
//     gradient dW_mu [32][128] at part_dw (bias = column 100) and p_fc2's dW_p2 [128][128] right
//     after it (bias = column 100), each summed over the workgroup's 128 rows by MFMA with the
//     batch as K: the operands are staged row-major in LDS and read back transposed
//     (ds_read_b64_tr_b16).  So only p_fc1's operands (g1 and the observation rows) go through
//     HBM to the wgrad.
#include "t32.h"

namespace {

using namespace t32;

constexpr int PH_ROWS = 128;            // rows per workgroup
constexpr int PH_WAVES = 4;
constexpr int PH_SB = 8 * 1024;         // ring stage bytes
constexpr int PH_S = 3;                 // ring stages
constexpr int PH_GL = 2;                // ring DMA instructions per wave and stage
constexpr int PH_XS = 3, PH_XB = 2048;  // X ring slots per wave / bytes per slot
constexpr int PH_SCR = 48 * 1024;       // X rings (fc1) | dW_mu staging: h2 half [128][64] + dL/dmu [128][32], hi | lo
constexpr int PH_RED = 64;              // per wave: 8 loss terms | 32 dlog_std (floats)
constexpr int PH_HP = 128 * 64 * 2;     // one precision plane of the staged h2 half (bytes)
constexpr int PH_DP = 128 * 32 * 2;     // one precision plane of the staged dL/dmu

constexpr size_t ph_lds_bytes() {
  return (size_t)PH_S * PH_SB + PH_SCR + (PH_WAVES * PH_RED + 64) * sizeof(float);
}
static_assert(2 * ph_lds_bytes() <= 160 * 1024, "two policy workgroups per CU");
static_assert(PH_WAVES * PH_XS * PH_XB <= PH_SCR / 2 && PH_WAVES * 32 * 32 * 4 <= PH_SCR / 2 &&
              2 * PH_HP + 2 * PH_DP <= PH_SCR, "scratch: X rings | actions, then the dW staging");

// 16-byte chunk swizzle of the staged h2 rows (128-byte rows): rows r and r + 2 of a transposed
// read's 4-row group land in different 64-byte halves (conflict-free ds_read_b64_tr_b16)
DEV int ph_swz(int row) { return ((row >> 1) & 1) << 2; }

// 4 consecutive rows x 16 columns of a row-major bf16 plane, transposed: lane 4 q + p of each
// 16-lane group addresses row q, columns 4 p .. 4 p + 3; lane i receives column i (rows 0-3)
// (inline asm, no wait: with the builtin the compiler put an s_waitcnt vmcnt(0) — every in-flight
// DMA and operand store — in front of these reads; ph_settle waits for them instead)
typedef __attribute__((ext_vector_type(4))) short s16x4;
DEV s16x4 tr4(const char* p) {
  s16x4 v;
  const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
// the LDS reads of a group of fragments have landed (the asm redefines them: no use moves above)
template <int DT>
DEV void ph_settle(typename VT<DT>::Frag (&fa)[2], typename VT<DT>::Frag (&fb)[2]) {
  if constexpr (DT == DT_S3) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(fa[0].h), "+v"(fa[0].l), "+v"(fa[1].h), "+v"(fa[1].l), "+v"(fb[0].h), "+v"(fb[0].l),
                   "+v"(fb[1].h), "+v"(fb[1].l));
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[0]), "+v"(fa[1]), "+v"(fb[0]), "+v"(fb[1]));
  }
}
DEV bf16x8 cat8(s16x4 a0, s16x4 a1) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const s16x8 v{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
  return *reinterpret_cast<const bf16x8*>(&v);
}

// dimension of accumulator register i of a 32x32 tile on lane half h (t32.h layout)
DEV int ph_dim(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// P2: sum p_fc2's weight gradient in the kernel (dW_p2 partial blocks; h1 / g2 stay on chip) —
// the bf16x3 path (4.26 -> 4.15 ms per iteration, same box); at bf16 the operands' HBM round trip
// is half as many bytes and the kernel stores h1 / g2 row-major for the wgrad instead (2.27 vs
// 2.36 ms with P2; profiles/r5/ab_p2_by_dtype.log)
template <int DT, bool P2>
__global__ __launch_bounds__(PH_WAVES * 64, 2) void phead_kernel(MlpArgs a) {
  using V = VT<DT>;
  using Frag = typename V::Frag;
  constexpr bool S3 = DT == DT_S3;
  constexpr int EB = V::EB, KPS = V::KPS;
  // dgrad fc2 runs as two passes of 2 h1 tiles (g1 of a pass is finished and stored, and its h1
  // tiles die, before the next: the chain's register peak); split: 4 stages of 2 k-steps x 2
  // tiles per pass, bf16: 2 stages of 4 k-steps x 2 tiles
  constexpr int NS2 = S3 ? 7 : 4, NS3 = S3 ? 2 : 1, NG3 = S3 ? 2 : 1, NG2 = S3 ? 8 : 4;
  constexpr int KK2 = S3 ? 2 : 4;   // dgrad fc2 k-steps per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];   // the kernel's ONLY LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int m0 = blockIdx.x * PH_ROWS;
  const int d0 = a.d_in[0];
  const int ns1 = (d0 >> 4) / KPS;
  const int e2 = ns1 + NS2, e3 = e2 + NS3, eg3 = e3 + NG3, ntot = eg3 + NG2;
  const int A = a.A;
  char* ring = smem;
  char* scr = smem + PH_S * PH_SB;
  char* xring = scr + wave * (PH_XS * PH_XB);
  float* red = reinterpret_cast<float*>(scr + PH_SCR);   // [wave][PH_RED]
  float* lsd = red + PH_WAVES * PH_RED;                  // log_std [32] | log_std_old [32]

  // the lane's row (rows past M re-read row m0: zero gradient) and its loss inputs — loaded
  // before any DMA (the oldest vector-memory ops: they never hold up a counted wait)
  const int mr = m0 + 32 * wave + r;
  const bool valid = mr < a.M;
  const int rr = valid ? mr : m0;
  const int srow = a.idx ? a.idx[rr] : a.row0 + rr;
  const bool ref_loss = a.loss_kind != 0;
  // the actions of the wave's 32 rows into LDS ([dim][row] fp32, in the scratch half the X ring
  // leaves free until the dW staging) by dword DMAs: instruction k moves dims 2 k + h (no
  // registers held through fc1 / fc2).  The reference loss's mu_prev rows are read at the loss
  // (that mode's load waits for the stream's in-flight DMAs once)
  float* acts = reinterpret_cast<float*>(scr + PH_SCR / 2) + wave * 32 * 32;
  {
    const float* arow = a.actions + (size_t)srow * A;
    for (int k = 0; 2 * k < A; ++k) {
      const int d = min(2 * k + h, A - 1);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(arow + d),
                                       (__attribute__((address_space(3))) void*)(acts + 64 * k), 4, 0, 0);
    }
  }
  float l_adv = a.adv[srow];
  float l_lpo = ref_loss ? 0.f : a.logp_old[srow];
  if (tid < 64) {
    const int j = tid & 31;
    lsd[tid] = tid < 32 ? (j < A ? a.log_std[j] : 0.f) : ((ref_loss && j < A) ? a.log_std_old[j] : 0.f);
  }

  // ---- DMA sources ----
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), (short)0, 0x7fffffff, 0x00020000);
  // per-lane byte offset of the lane's piece of a 32x16 A fragment in an FM image of c32 block
  // columns: a 32x16 fragment is four 256-byte pieces of two 16x32 FM blocks (split: the DMA
  // instruction d carries reader lanes 32 d .. 32 d + 31, its lanes >= 32 the lo halves)
  auto lane_off = [&](int c32, int d) __attribute__((always_inline)) -> unsigned {
    const int i = lane & 31;
    if constexpr (S3) return (unsigned)(((i >> 4) * c32 * 512 + ((i & 15) + 16 * d) * 8) * 4 + 16 * (lane >> 5));
    else return (unsigned)(((i >> 4) * c32 * 512 + ((i & 15) + 16 * (lane >> 5)) * 8) * 2);
  };
  const int c1 = d0 >> 5;
  const unsigned vo1[2] = {lane_off(c1, 0), lane_off(c1, 1)};
  const unsigned vo4[2] = {lane_off(4, 0), lane_off(4, 1)};   // fc2, mu, W2^T: 128-wide images
  const unsigned vog[2] = {lane_off(1, 0), lane_off(1, 1)};   // W3^T: [128][32]
  auto frag_u = [&](int t, int k16, int c32) __attribute__((always_inline)) {
    return t * 2 * c32 * 512 + (k16 >> 1) * 512 + (k16 & 1) * 256;
  };
  // this wave's 2 ring DMA instructions (of the stage's 8) for stream step st into slot st % S.
  // Slot u of a stage: split (4 fragments): tile / k-step u; bf16 (8): tile u & 3, k-step u >> 2
  auto issue = [&](int st) __attribute__((always_inline)) {
    __attribute__((address_space(3))) char* dst =
        (__attribute__((address_space(3))) char*)(ring + (st % PH_S) * PH_SB);
#pragma unroll
    for (int i = 0; i < PH_GL; ++i) {
      const int I = PH_GL * wave + i;
      const int u = S3 ? I >> 1 : I, d = S3 ? (I & 1) : 0;
      const int tu = S3 ? u : (u & 3), ku = S3 ? 0 : (u >> 2);
      int off;
      unsigned voff;
      if (st < ns1) {
        off = a.off_w[0] + frag_u(tu, KPS * st + ku, c1);
        voff = vo1[d];
      } else if (st < e2) {
        off = a.off_w[1] + frag_u(tu, KPS * (st - ns1) + ku, 4);
        voff = vo4[d];
      } else if (st < e3) {   // mu: one output tile, the stage's fragments are k-steps
        off = a.off_w[2] + frag_u(0, S3 ? 4 * (st - e2) + u : u, 4);
        voff = vo4[d];
      } else if (st < eg3) {  // W3^T: h2 tiles x the dims' 2 k-steps (split stage j: tiles 2 j, 2 j + 1)
        off = a.off_wt[2] + (S3 ? frag_u(2 * (st - e3) + (u & 1), u >> 1, 1) : frag_u(tu, ku, 1));
        voff = vog[d];
      } else {                // W2^T: pass p's 2 h1 tiles x the h2 k-steps (slot u: tile 2 p + (u & 1))
        const int j = st - eg3, pass = j / (NG2 / 2), jj = j % (NG2 / 2);
        off = a.off_wt[1] + frag_u(2 * pass + (u & 1), KK2 * jj + (u >> 1), 4);
        voff = vo4[d];
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, dst + I * 1024, 16, voff, (unsigned)off * EB, 0, 0);
    }
  };
  const char* xrow = reinterpret_cast<const char*>(a.x_buf) + (size_t)srow * (size_t)d0 * EB;
  // the wave's 2 X DMA instructions of fc1 stage st (split: hi, lo of the k-step; bf16: 2 k-steps)
  auto issue_x = [&](int st) __attribute__((always_inline)) {
    char* dx = xring + (st % PH_XS) * PH_XB;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if constexpr (S3) glds16(xrow + (size_t)(16 * st + 8 * h) * 4 + 16 * e, dx + e * 1024);
      else glds16(xrow + (size_t)(16 * (2 * st + e) + 8 * h) * 2, dx + e * 1024);
    }
  };
  auto x_frag = [&](int st, int e) __attribute__((always_inline)) -> Frag {
    const char* xs = xring + (st % PH_XS) * PH_XB;
    if constexpr (S3) {
      return Frag{*reinterpret_cast<const bf16x8*>(xs + 16 * lane), *reinterpret_cast<const bf16x8*>(xs + 1024 + 16 * lane)};
    } else {
      return *reinterpret_cast<const bf16x8*>(xs + e * 1024 + 16 * lane);
    }
  };

  // row-major operand stores of this lane's row (the launcher checks ldT * max(d0, 128) * EB < 2^31)
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(a.xT, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_g1 = __builtin_amdgcn_make_buffer_rsrc(a.g1pT, (short)0, 0x7fffffff, 0x00020000);
  // (!P2: h1 and g2 row-major for the wgrad's p_fc2 tiles)
  const __amdgpu_buffer_rsrc_t rs_h1 =
      __builtin_amdgcn_make_buffer_rsrc(P2 ? a.g1pT : a.h1pT, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_g2 =
      __builtin_amdgcn_make_buffer_rsrc(P2 ? a.g1pT : a.g2pT, (short)0, 0x7fffffff, 0x00020000);
  const unsigned vx = (unsigned)(mr * d0 + 8 * h) * EB, v128 = (unsigned)(mr * 128 + 8 * h) * EB;
  const bool write_x = a.xT_ready == 0;
  const int xst = write_x ? 2 : 0;   // X operand stores per fc1 step

  // the loss inputs (and the action DMAs) land before the stream starts: the asm redefines the
  // registers, so no compiler-inserted wait for them falls inside the counted stream (where it
  // would also wait for every in-flight DMA and operand store)
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(l_adv), "+v"(l_lpo)::"memory");
  // ---- prime: X stages 0, 1 and ring stages 0, 1 (the launcher checks ns1 >= 3) ----
  static_assert(PH_S == 3 && PH_XS == 3, "the wait counts below are written for 3-stage rings");
  issue_x(0);
  issue_x(1);
  issue(0);
  issue(1);

  f32x16 acc1[4], acc2[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc1[t] = acc2[t] = f32x16{};

  // one stream step's sync: this wave's DMAs of ring stage st by count (`younger` = its vector
  // memory instructions issued after that stage's batch; an undercount only waits longer), then
  // the barrier: every wave's stage st landed, everyone is done with stage st - 1
  auto sync = [&](int younger) __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    wait_vm_rt(younger);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // from the last two fc1 steps on the counts come from VmTrack, entering with stage ns1 - 2's
  // batch followed by [its step's X stores,] X(ns1 - 1), R(ns1 - 1) and the previous step's X
  // stores (ns1 == 3: stage 1's batch is the prologue's, the first step's X stores only)
  VmTrack vt(ns1 == 3 ? 2 + PH_GL + xst : 2 + PH_GL + 2 * xst, xst);
  constexpr int SP = S3 ? 2 : 1;   // store instructions per operand fragment
  auto sync_t = [&](int st) __attribute__((always_inline)) {
    sync(vt.younger());
    const bool refill = st + 2 < ntot;
    if (refill) issue(st + 2);
    vt.advance(refill ? PH_GL : 0);
  };
  auto sync_late = [&](int st) __attribute__((always_inline)) {
    sync_t(st);
    return ring + (st % PH_S) * PH_SB;
  };
  // an operand store, counted
  auto sto = [&](__amdgpu_buffer_rsrc_t rs, unsigned vrow, unsigned fsoff, const Frag& f) __attribute__((always_inline)) {
    st_op<DT>(rs, vrow, fsoff, f);
    vt.add(SP);
  };
  auto fc1 = [&](const char* stg, int st) __attribute__((always_inline)) {
    Frag xb[KPS];
#pragma unroll
    for (int e = 0; e < KPS; ++e) {
      xb[e] = x_frag(st, e);
      if (write_x) st_op<DT>(rs_x, vx, 16 * (KPS * st + e) * EB, xb[e]);
    }
    ring_mma<DT, 4 * KPS, 2 * KPS>(stg, lane, [&](int i) { return i; },
                                   [&](int i, const Frag& w) __attribute__((always_inline)) {
                                     acc1[i & 3] = V::mma(acc1[i & 3], w, xb[i >> 2]);
                                   });
  };

  // ---- fc1: h1^T += W1 . x^T ----
  // steps 0 .. ns1-3 issue X(st + 2) and fc1 stage st + 2 (younger than R(st): X(st+1), R(st+1)
  // and the previous step's X operand stores; step 0: R(1) only)
  for (int st = 0; st < ns1 - 2; ++st) {
    sync(st == 0 ? PH_GL : (st == 1 ? 2 + PH_GL + xst : 2 + PH_GL + 2 * xst));
    issue_x(st + 2);
    issue(st + 2);
    fc1(ring + (st % PH_S) * PH_SB, st);
  }
  // the last two fc1 steps refill with fc2 stages 0, 1 (no more X)
  sync_t(ns1 - 2);
  fc1(ring + ((ns1 - 2) % PH_S) * PH_SB, ns1 - 2);
  vt.add(xst);
  sync_t(ns1 - 1);
  fc1(ring + ((ns1 - 1) % PH_S) * PH_SB, ns1 - 1);
  {
    // h1 = tanh, the bias column (feature n_out[0]) = 1
    const int nb = a.n_out[0], tb = nb >> 5, rb = nb & 31;
    const int g = (rb & 3) + 4 * (rb >> 3);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc1[t] = tanh16(acc1[t]);
      if (t == tb && ((rb >> 2) & 1) == h) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i == g) acc1[t][i] = 1.f;
      }
    }
  }

  // ---- fc2: h2^T += W2 . h1^T; stage j takes k-steps KPS j ..; their B operands double as the
  // h1 operand stores (split: the last stage also stores the zero k-step 7) ----
  vt.add(xst);
  static_for_vh<0, NS2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const char* stg = sync_late(ns1 + j);
    Frag b[KPS];
#pragma unroll
    for (int e = 0; e < KPS; ++e) {
      const int k16 = KPS * j + e;
      b[e] = b_operand<DT>(acc1[k16 >> 1], k16 & 1);
      if constexpr (!P2) sto(rs_h1, v128, 16 * k16 * EB, b[e]);
    }
    if constexpr (!P2 && S3 && j == NS2 - 1) {
      sto(rs_h1, v128, 16 * 7 * EB, b_operand<DT>(acc1[3], 1));
    }
    ring_mma<DT, 4 * KPS, (S3 ? 1 : 2)>(stg, lane, [&](int i) { return i; },
                                        [&](int i, const Frag& w) __attribute__((always_inline)) {
                                          acc2[i & 3] = V::mma(acc2[i & 3], w, b[i >> 2]);
                                        });
  });
  {
    // h2 = tanh, the bias column (feature n_out[1]) = 1
    const int nb = a.n_out[1], tb = nb >> 5, rb = nb & 31;
    const int g = (rb & 3) + 4 * (rb >> 3);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc2[t] = tanh16(acc2[t]);
      if (t == tb && ((rb >> 2) & 1) == h) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i == g) acc2[t][i] = 1.f;
      }
    }
  }

  // ---- mu^T = W3 . h2^T (one 32-dim tile; split: k-steps 4 j + u of stage j, bf16: u) ----
  f32x16 mu = f32x16{};
  static_for_vh<0, NS3>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const char* stg = sync_late(e2 + j);
    constexpr int NF = S3 ? 4 : 8;
    Frag b[NF];
#pragma unroll
    for (int u = 0; u < NF; ++u) {
      const int k16 = S3 ? 4 * j + u : u;
      b[u] = b_operand<DT>(acc2[k16 >> 1], k16 & 1);
    }
    ring_mma<DT, NF, (S3 ? 2 : 4)>(stg, lane, [&](int i) { return i; },
                                   [&](int i, const Frag& w) __attribute__((always_inline)) { mu = V::mma(mu, w, b[i]); });
  });

  // ---- the policy loss of this lane's row (dims ph_dim(i, h)) -> dL/dmu, dlog_std, loss terms ----
  f32x16 dmu;
  float dls[16];
  float lt[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  {
    const float cvar = a.std_var ? 0.5f : 1.f;
    const float vm = valid ? 1.f : 0.f;
    if (a.loss_kind == 0) {
      // corrected PPO (ppo.py:148-167): the row's log-prob over both lane halves
      float lp = 0.f, lent = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int d = ph_dim(i, h);
        if (d < A) {
          const float lsig = cvar * lsd[d];
          const float z = (acts[d * 32 + r] - mu[i]) * __expf(-lsig);
          lp += -0.5f * z * z - 0.5f * T32_LOG_2PI - lsig;
          lent += -a.ent_coeff * (0.5f + 0.5f * T32_LOG_2PI + lsig);
        }
      }
      const float logp = lp + __shfl_xor(lp, 32, 64);
      const float lrat = logp - l_lpo;
      const float ratio = __expf(lrat);
      const float s1 = ratio * l_adv;
      const float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * l_adv;
      const float dlogp = (s1 <= s2) ? -l_adv * ratio : 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int d = ph_dim(i, h);
        const float lsig = cvar * lsd[d & 31];
        const float isig = __expf(-lsig);
        const float z = (acts[(d < A ? d : 0) * 32 + r] - mu[i]) * isig;
        const bool on = valid && d < A;
        dmu[i] = on ? dlogp * z * isig : 0.f;
        dls[i] = on ? (dlogp * (z * z - 1.f) - a.ent_coeff) * cvar : 0.f;
      }
      if (h == 0) {
        lt[0] = -fminf(s1, s2) * vm;
        lt[3] = ((ratio - 1.f) - lrat) * vm;
        lt[4] = (fabsf(ratio - 1.f) > a.clip ? 1.f : 0.f) * vm;
        lt[5] = vm;
      }
      lt[2] = lent * vm;
    } else {
      // reference DPPO loss (train.py:142-161): per-dim pdf ratio, variance convention
      const float invA = 1.f / (float)A;
      const bool first = a.first_step != 0;
      float lclip = 0.f, lent = 0.f, cf = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int d = ph_dim(i, h);
        dmu[i] = 0.f;
        dls[i] = 0.f;
        if (d < A) {
          const float m = mu[i];
          const float var = __expf(lsd[d]);
          const float mu_o = first ? m : a.mu_prev[(size_t)srow * A + d];
          const float var_o = first ? var : __expf(lsd[32 + d]);
          const float x = acts[d * 32 + r];
          const float pd = __expf(-(x - m) * (x - m) / (2.f * var)) * rsqrtf(2.f * var * 3.14159265358979f);
          const float po = __expf(-(x - mu_o) * (x - mu_o) / (2.f * var_o)) * rsqrtf(2.f * var_o * 3.14159265358979f);
          const float ratio = pd / (1e-10f + po);
          const float s1 = ratio * l_adv;
          const float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * l_adv;
          lclip += -fminf(s1, s2) * invA;
          const float dratio = (s1 <= s2) ? -l_adv * invA : 0.f;
          float dp = dratio / (1e-10f + po);
          const float lgp = logf(pd + 1e-5f);
          lent += -a.ent_coeff * pd * lgp * invA;
          dp += -a.ent_coeff * invA * (lgp + pd / (pd + 1e-5f));
          dmu[i] = valid ? dp * pd * (x - m) / var : 0.f;
          dls[i] = valid ? dp * pd * ((x - m) * (x - m) / (2.f * var) - 0.5f) : 0.f;
          cf += (fabsf(ratio - 1.f) > a.clip) ? invA : 0.f;
          if (valid) a.mu_prev[(size_t)srow * A + d] = m;   // train.py:164 model_old <- model
        }
      }
      lt[0] = lclip * vm;
      lt[2] = lent * vm;
      lt[4] = cf * vm;
      if (h == 0) lt[5] = vm;
    }
  }
  // the wave's sums over its 32 rows (fixed order): loss terms over all 64 lanes, dlog_std per dim
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) lt[k] += __shfl_xor(lt[k], m, 64);
  {
    const float s = half_sum16(dls, lane);
    float* wr = red + wave * PH_RED;
    if (r < 16) wr[8 + ph_dim(r, h)] = s;
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) wr[k] = lt[k];
      wr[6] = wr[7] = 0.f;
    }
  }
  // dL/dmu as B operands (dims 0-15, 16-31) of the mu dgrad
  Frag db[2] = {b_operand<DT>(dmu, 0), b_operand<DT>(dmu, 1)};

  // ---- dW_mu^T [128 features][32 dims] = h2^T . dL/dmu over the workgroup's 128 rows: two
  // rounds of the h2 half [128][64] + dL/dmu [128][32] staged row-major (hi | lo planes); wave w
  // takes feature tile w in round w / 2 (K = all 128 rows: the whole workgroup sum, fixed order) ----
  const int row = 32 * wave + r;   // this lane's row of the workgroup's 128
  // row-major staging of 16-byte operand chunks (hi | lo planes) and the transposed fragment
  // (lane: column c0 + (l & 31), rows 16 kk + 8 (l >> 5) ..) of a staged plane
  auto put = [&](char* plane, int rowb, int chunk, const Frag& f, int pstride) __attribute__((always_inline)) {
    if constexpr (S3) {
      *reinterpret_cast<bf16x8*>(plane + rowb + 16 * chunk) = f.h;
      *reinterpret_cast<bf16x8*>(plane + pstride + rowb + 16 * chunk) = f.l;
    } else {
      *reinterpret_cast<bf16x8*>(plane + rowb + 16 * chunk) = f;
    }
  };
  auto get = [&](const char* plane, int pstride, int rowbytes, int c0, int kk, bool swz) __attribute__((always_inline)) -> Frag {
    const int li = lane & 15, g = lane >> 4;
    const int col = c0 + 16 * (g & 1) + 4 * (li & 3);
    auto rd = [&](const char* base, int sub) __attribute__((always_inline)) {
      const int rw2 = 16 * kk + 8 * (g >> 1) + 4 * sub + (li >> 2);
      const int ch = (col >> 3) ^ (swz ? ph_swz(rw2) : 0);
      return tr4(base + rw2 * rowbytes + 16 * ch + 2 * (col & 7));
    };
    if constexpr (S3) {
      return Frag{cat8(rd(plane, 0), rd(plane, 1)), cat8(rd(plane + pstride, 0), rd(plane + pstride, 1))};
    } else {
      return cat8(rd(plane, 0), rd(plane, 1));
    }
  };
  auto bar = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const __amdgpu_buffer_rsrc_t rs_part = __builtin_amdgcn_make_buffer_rsrc(a.part, (short)0, 0x7fffffff, 0x00020000);
  {
    char* Hp = scr;                     // [2 planes][128 rows][128 B]
    char* Dp = scr + 2 * PH_HP;         // [2 planes][128 rows][64 B]
    // every wave's loss has read its actions (acts, in the scratch the staging below overwrites:
    // Dp covers wave 2's, the split Hp lo plane waves 0 / 1's) before any wave stages
    bar();
#pragma unroll
    for (int s = 0; s < 2; ++s) put(Dp, row * 64, 2 * s + h, db[s], PH_DP);
#pragma unroll
    for (int round = 0; round < 2; ++round) {
      // the h2 tiles 2 round, 2 round + 1 of this wave's rows (pinned here: not converted early
      // and held across the barriers)
      asm volatile("" : "+v"(acc2[2 * round]), "+v"(acc2[2 * round + 1]));
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int chunk = (4 * tt + 2 * s + h) ^ ph_swz(row);
          put(Hp, row * 128, chunk, b_operand<DT>(acc2[2 * round + tt], s), PH_HP);
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if ((wave >> 1) == round) {
        const int tt = wave & 1;
        f32x16 dw = f32x16{};
        // (two k-steps' reads in flight per group: the h2 / dL/dmu tiles are live in registers)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) {
          Frag fa[2], fb[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            fa[q] = get(Hp, PH_HP, 128, 32 * tt, 2 * k2 + q, true);
            fb[q] = get(Dp, PH_DP, 64, 0, 2 * k2 + q, false);
          }
          ph_settle<DT>(fa, fb);
#pragma unroll
          for (int q = 0; q < 2; ++q) dw = V::mma(dw, fb[q], fa[q]);   // A = dL/dmu^T, B = h2: D[dim][feature]
          __builtin_amdgcn_sched_barrier(0);
        }
        // feature 32 w + (l & 31), dim ph_dim(i, h): dst[part_dw + dim * 128 + feature] (all 32
        // dims: those past A are zero — one store per register, a constant count)
        const unsigned base = (unsigned)((size_t)blockIdx.x * a.npart + a.part_dw + 32 * wave + r) * 4u;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int d = ph_dim(i, h);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dw[i]), rs_part, base + (unsigned)d * 512u, 0, 0);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    vt.add(16);   // this wave's dW_mu stores (in its round)
  }

  // ---- dgrad mu: g2 = (W3^T dL/dmu) (1 - h2^2) over the 4 h2 tiles ----
  // (split: stage j finishes h2 tiles 2 j, 2 j + 1 — their g2 operands are made and those h2
  // tiles die before the next stage; k-step 7 of g2 — h2 features 112-127, past n_out[1] — is
  // zero and not held)
  constexpr int NGB = S3 ? 7 : 8;
  Frag gb[NGB];
  auto g2_ops = [&](int t, const f32x16& gacc) __attribute__((always_inline)) {
    f32x16 g2;
#pragma unroll
    for (int i = 0; i < 16; ++i) g2[i] = gacc[i] * __builtin_fmaf(-acc2[t][i], acc2[t][i], 1.f);
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (2 * t + s < NGB) gb[2 * t + s] = b_operand<DT>(g2, s);
  };
  if constexpr (S3) {
    static_for_vh<0, NG3>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const char* stg = sync_late(e3 + j);
      f32x16 gq[2] = {f32x16{}, f32x16{}};
      ring_mma<DT, 4, 2>(stg, lane, [&](int i) { return i; },
                         [&](int i, const Frag& w) __attribute__((always_inline)) {
                           gq[i & 1] = V::mma(gq[i & 1], w, db[i >> 1]);
                         });
      g2_ops(2 * j, gq[0]);
      g2_ops(2 * j + 1, gq[1]);
    });
  } else {
    const char* stg = sync_late(e3);
    f32x16 ga[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) ga[t] = f32x16{};
    ring_mma<DT, 8, 4>(stg, lane, [&](int i) { return i; },
                       [&](int i, const Frag& w) __attribute__((always_inline)) {
                         ga[i & 3] = V::mma(ga[i & 3], w, db[i >> 2]);
                       });
#pragma unroll
    for (int t = 0; t < 4; ++t) g2_ops(t, ga[t]);
  }

  // ---- dgrad fc2: g1 = (W2^T g2) (1 - h1^2), two passes of 2 h1 tiles; the g2 operand stores
  // ride along (one k-step per split step / two per bf16 step) ----
  static_for_vh<0, 2>([&](auto pc) __attribute__((always_inline)) {
    constexpr int pass = decltype(pc)::value;
    f32x16 gp[2] = {f32x16{}, f32x16{}};
    static_for_vh<0, NG2 / 2>([&](auto jc) __attribute__((always_inline)) {
      constexpr int jj = decltype(jc)::value, j = pass * (NG2 / 2) + jj;
      const char* stg = sync_late(eg3 + j);
      if constexpr (!P2) {
        if constexpr (S3) {
          sto(rs_g2, v128, 16 * j * EB, j < NGB ? gb[j < NGB ? j : 0] : Frag{});
        } else {
#pragma unroll
          for (int e = 0; e < 2; ++e) sto(rs_g2, v128, 16 * (2 * j + e) * EB, gb[2 * j + e]);
        }
      }
      // (split: the last stage's k-step 7 is zero: its 2 fragments are not multiplied)
      constexpr int NF = (S3 && jj == NG2 / 2 - 1) ? 2 : 4 * KPS;
      ring_mma<DT, NF, (S3 ? 1 : 2)>(stg, lane, [&](int i) { return i; },
                                     [&](int i, const Frag& w) __attribute__((always_inline)) {
                                       gp[i & 1] = V::mma(gp[i & 1], w, gb[KK2 * jj + (i >> 1)]);
                                     });
    });
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * pass + tt;
      f32x16 g1;
#pragma unroll
      for (int i = 0; i < 16; ++i) g1[i] = gp[tt][i] * __builtin_fmaf(-acc1[t][i], acc1[t][i], 1.f);
#pragma unroll
      for (int s = 0; s < 2; ++s) sto(rs_g1, v128, (32 * t + 16 * s) * EB, b_operand<DT>(g1, s));
    }
  });

  // ---- dW_p2^T [out 128][in 128] = g2^T . h1b over the workgroup's 128 rows (h1b: h1 with its
  // bias column), fused like dW_mu (train.py:166's p_fc2 gradient without the g2 / h1 operand
  // round trip through HBM and the wgrad): four rounds of an out-half of g2 and an in-half of h1
  // staged row-major in the freed ring + scratch (2 x 32 KiB), wave w taking the round's tile
  // (out 64 go + 32 (w >> 1), in 64 ih + 32 (w & 1)) with K = all 128 rows (fixed order) ----
  if constexpr (P2) {
    static_assert(2 * 2 * PH_HP <= PH_S * PH_SB + PH_SCR, "two staged halves fit the ring + scratch");
    char* Gs = smem;                  // g2 out-half [2 planes][128 rows][128 B]
    char* Hs = smem + 2 * PH_HP;      // h1 in-half  [2 planes][128 rows][128 B]
    bar();   // every wave is done with the ring's last stage and the scratch
    auto stage_g = [&](int go) __attribute__((always_inline)) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k16 = 4 * go + kk;   // g2 features 16 k16 + 8 h ..: the half's chunk 2 kk + h
        put(Gs, row * 128, (2 * kk + h) ^ ph_swz(row), k16 < NGB ? gb[k16 < NGB ? k16 : 0] : Frag{}, PH_HP);
      }
    };
    auto stage_h = [&](int ih) __attribute__((always_inline)) {
      // (pinned here: the conversions are not hoisted above the barriers and held)
      asm volatile("" : "+v"(acc1[2 * ih]), "+v"(acc1[2 * ih + 1]));
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          put(Hs, row * 128, (4 * tt + 2 * s + h) ^ ph_swz(row), b_operand<DT>(acc1[2 * ih + tt], s), PH_HP);
    };
    const unsigned base = (unsigned)((size_t)blockIdx.x * a.npart + a.part_dw + 32 * 128 + 32 * (wave & 1) + r) * 4u;
    // rounds (go, ih) = (0, 0), (0, 1), (1, 1), (1, 0): one half restaged per round after the first
    static_for_vh<0, 4>([&](auto rc) __attribute__((always_inline)) {
      constexpr int rd = decltype(rc)::value;
      constexpr int go = rd >> 1, ih = (rd == 1 || rd == 2) ? 1 : 0;
      if constexpr (rd == 0) {
        stage_g(0);
        stage_h(0);
      } else if constexpr (rd == 2) {
        stage_g(1);
      } else {
        stage_h(ih);
      }
      bar();
      f32x16 dw = f32x16{};
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        Frag fa[2], fb[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          fa[q] = get(Gs, PH_HP, 128, 32 * (wave >> 1), 2 * k2 + q, true);
          fb[q] = get(Hs, PH_HP, 128, 32 * (wave & 1), 2 * k2 + q, true);
        }
        ph_settle<DT>(fa, fb);
#pragma unroll
        for (int q = 0; q < 2; ++q) dw = V::mma(dw, fa[q], fb[q]);   // A = g2^T (out), B = h1b (in)
        __builtin_amdgcn_sched_barrier(0);
      }
      // out feature 64 go + 32 (w >> 1) + ph_dim(i, h) (registers), in feature 64 ih + 32 (w & 1)
      // + (l & 31) (lanes): dst[part_dw + 4096 + out * 128 + in]; only the entries the gather
      // reads (out < n2, in <= n1: the bias column) — the kernel's tail is its stores (no vector
      // memory instruction follows them, so no counted wait sees the difference)
      const bool in_ok = 64 * ih + 32 * (wave & 1) + r <= a.n_out[0];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const unsigned o = (unsigned)(64 * go + 32 * (wave >> 1) + ph_dim(i, h));
        if (in_ok && o < (unsigned)a.n_out[1])
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dw[i]), rs_part, base + (o * 128u + 64u * ih) * 4u,
                                                0, 0);
      }
      bar();
    });
  }

  // ---- per-workgroup partials (fixed order over the waves): loss terms (not column 1: the
  // value head's) and dlog_std ----
  // (no DMA is in flight: the last stage's sync waited for all of them; the operand stores may
  // drain after the waves end)
  float* dst = a.part + (size_t)blockIdx.x * a.npart;
  if (tid < 8 + A && tid != 1) {
    dst[tid] = ((red[tid] + red[PH_RED + tid]) + red[2 * PH_RED + tid]) + red[3 * PH_RED + tid];
  }
}

int g_phead = 1;

}  // namespace

// the shapes the kernel covers: the reference policy (d0 -> 100 -> 100 -> A <= 32; observation
// widths 128, 256, 384: the wgrad reads the observation operand as row-major rows of the operand
// width, d0 rounded up to its 128-row tile, so x_buf's rows serve only when d0 is that width)
extern "C" int phead_shape_ok(const MlpArgs& a) {
  return a.d_in[0] % 128 == 0 && a.d_in[0] >= 128 && a.d_in[0] <= 384 && a.d_out[0] == 128 && a.n_out[0] < 128 &&
         a.n_out[0] >= 97 && a.d_in[1] == 128 && a.d_out[1] == 128 && a.n_out[1] < 128 && a.n_out[1] >= 97 &&
         a.d_in[2] == 128 && a.d_out[2] == 32 && a.A >= 1 && a.A <= 32 && a.n_out[2] <= 32;
}

extern "C" int phead_applies(const MlpArgs& a) { return g_phead && phead_shape_ok(a); }

extern "C" int phead_rows() { return PH_ROWS; }

template <int DT, bool P2>
void launch_ph(const MlpArgs& a, int nblk, hipStream_t s) {
  set_max_lds_once<phead_kernel<DT, P2>>(ph_lds_bytes());
  hipLaunchKernelGGL((phead_kernel<DT, P2>), dim3(nblk), dim3(PH_WAVES * 64), ph_lds_bytes(), s, a);
}

extern "C" void launch_phead_train(int dt, const MlpArgs& a, int p2, hipStream_t s) {
  const int nblk = (a.M + PH_ROWS - 1) / PH_ROWS;
  if (dt == DT_S3) {
    if (p2) launch_ph<DT_S3, true>(a, nblk, s);
    else launch_ph<DT_S3, false>(a, nblk, s);
  } else {
    if (p2) launch_ph<DT_BF16, true>(a, nblk, s);
    else launch_ph<DT_BF16, false>(a, nblk, s);
  }
  HIP_CHECK_LAUNCH();
}

extern "C" void set_phead(int enable) { g_phead = enable ? 1 : 0; }
