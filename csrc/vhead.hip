// Value head forward V(x) on 32x32x16 MFMAs in the TRANSPOSED chain, ONE WAVE PER SIMD (SURVEY K5;
// model.py:42-44 forward, train.py:109-112: the GAE input of every rollout row).
//
// Every layer computes out^T = W . in^T:  A = a weight fragment (32 output features x 16 k, from
// the LDS ring, shared by all waves of the workgroup), B = the activations (16 k x 32 batch rows,
// in registers).  The 32x32 accumulator has the batch row on the lane and 16 output features in
// its registers (col = lane & 31, feature (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)), which is the
// NEXT layer's B operand up to one v_permlane32_swap per dword (t32.h b_operand): no LDS transpose
// anywhere in the chain, and one 32x16 fragment read from LDS feeds 32x32 outputs.
//
// Workgroup: 4 waves x 32 rows = 128 rows, one wave per SIMD and one workgroup per CU (<= 512
// registers per wave: the 16 fc1 accumulator tiles — all 512 features of the wave's 32 rows, 256
// registers — live in AGPRs; this file is built WITHOUT -amdgpu-mfma-vgpr-form, ops/_build.py).
// fc3 (one output) runs on the VALU in fp32.
//
// Round 6 also built the value head's UPDATE on this scheme (the loss, the dgrad through fc2, the
// fused dW_v / dW_v2 and k16-blocked operand stores) and measured it slower than the 16x16
// two-waves-per-SIMD head kernel at every step (docs/ARCHITECTURE.md §13, profiles/r6): with one
// wave per SIMD the operand stores, the LDS-DMA issue and the VALU epilogues stall the matrix pipe
// with nothing to cover them.  The update stays on csrc/mlp_head.hip; this kernel is the forward
// only (at par with the 16x16 forward: ~111 us per 65,536 rows at bf16x3).
//
// Weights stream through an S-stage LDS ring of 32 KiB stages (8 LDS-DMA instructions of 1 KiB per
// wave and stage, interleaved with the MFMAs: ring_mma_dma) straight from the packed FM images
// (csrc/common.h fm_index): a 32x16 A fragment is four 256-byte pieces of two 16x32 FM blocks,
// gathered by per-lane DMA source offsets, landing lane-linear.  Observation rows: a per-wave S-slot
// X ring (2 KiB per fc1 stage, 64-bit per-lane row addresses: any buffer size).  Counted vmcnt
// waits (VmQ) + one raw s_barrier per stage; S - 1 stages of DMA stay in flight across it
// (cdna_hip_programming.md 'Pipelining across barriers').
//
// Stream (split-bf16 / bf16 stage counts): fc1 d_in/16 k-steps (24 / 12) | fc2 32 k-steps x 4
// tiles (8 / 4).
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
// after fc1 the X rings hold the fc3 weights (129 floats)
constexpr int VH_W3 = 128;
static_assert((VH_W3 + 4) * 4 <= VH_WAVES * VH_XS * VH_XB, "fc3 weights fit the X rings");

template <int DT>
constexpr int vh_ns2() { return 32 / (4 * VT<DT>::KPS); }   // fc2 stages: 4 (split) / 8 (bf16) k-steps x 4 tiles

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

// V(x) into v_out
template <int DT>
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
  char* xr0 = smem + S * VH_SB;                 // X rings; after fc1 the fc3 weights
  char* xring = xr0 + wave * (VH_XS * VH_XB);
  float* w3s = reinterpret_cast<float*>(xr0);   // [129] fc3 weights + bias (after fc1)

  // the lane's row (rows past M re-read row m0) — loaded before any DMA (the oldest vector-memory
  // ops: they never hold up a counted wait)
  const int mr = m0 + 32 * wave + r;
  const bool valid = mr < a.M;
  const int rr = valid ? mr : m0;
  const int srow = a.idx ? a.idx[rr] : a.row0 + rr;
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
  const int c1 = d1 >> 5, c2 = a.d_in[4] >> 5;
  const unsigned vo1[2] = {lane_off(c1, 0), lane_off(c1, 1)};
  const unsigned vo2[2] = {lane_off(c2, 0), lane_off(c2, 1)};
  // element offset of the (32-feature tile t, 16-deep k-step k16) fragment of an image (c32 columns)
  auto frag_u = [&](int t, int k16, int c32) __attribute__((always_inline)) {
    return t * 2 * c32 * 512 + (k16 >> 1) * 512 + (k16 & 1) * 256;
  };
  constexpr int NS2 = vh_ns2<DT>();
  // this wave's 8 ring DMA instructions (of the stage's 32) for stream step st into slot st % S.
  // Slot u of a stage (split: 2 instructions per fragment; bf16: 1):
  //  fc1 stage j (k-steps KPS j ..):  u = tile (split) | tile + 16 e (bf16, k-step KPS j + e)
  //  fc2 stage j (k-steps 4 KPS j ..): u = 4 kk + t (output tile t of the stage's k-step kk)
  // fc1 stages take a runtime index (ns1 = d_in / 16 / KPS); the rest of the stream is unrolled, so
  // its stages are compile-time J = st - ns1 — every DMA's source offset folds to one add
  auto dma = [&](int st, int i, unsigned soff, unsigned voff) __attribute__((always_inline)) {
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
    const int kk = u >> 2, t = u & 3;
    dma(st, i, (unsigned)(a.off_w[4] + frag_u(t, 4 * KPS * J + kk, c2)) * EB, vo2[d]);
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

  // the fc3 weight lands before the stream starts: the asm redefines it, so no compiler-inserted
  // wait for it can fall inside the counted stream, where it would also wait for every DMA
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(w3v)::"memory");
  // ---- prime: X and ring stages 0 .. S-2 (the launcher checks ns1 >= S) ----
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
    vq.advance(JR < NS2 ? VH_GL : 0);
    return ring + ((ns1 + J) % S) * VH_SB;
  };
  auto refill = [&](auto jc) __attribute__((always_inline)) {
    constexpr int JR = decltype(jc)::value + S - 1;
    return [&, jc](int k) __attribute__((always_inline)) {
      if constexpr (JR < NS2) issue_rest_i(std::integral_constant<int, JR>{}, ns1 + JR, k);
    };
  };
  auto nref = [&](auto jc) __attribute__((always_inline)) {
    constexpr int JR = decltype(jc)::value + S - 1;
    return std::integral_constant<int, (JR < NS2 ? VH_GL : 0)>{};
  };
  static_for_vh<1, S>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = S - decltype(ic)::value;     // S - 1 .. 1
    constexpr auto jc = std::integral_constant<int, -i>{};
    const char* stg = sync_late(jc);
    fc1(stg, ns1 - i, refill(jc), nref(jc));
  });
  // h1 = tanh; the bias column (feature n_out[3]) = 1
  {
    const int nb = a.n_out[3], tb = nb >> 5, rb = nb & 31;
    const int g = (rb & 3) + 4 * (rb >> 3);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      acc[t] = tanh16(acc[t]);
      if (t == tb && ((rb >> 2) & 1) == h) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i == g) acc[t][i] = 1.f;
      }
    }
  }

  // ---- fc2: h2^T += W2 . h1^T; stage j takes k-steps 4 KPS j .. (h1 tiles 2 KPS j ..), their B
  // operands built before the wait ----
  f32x16 acc2[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc2[t] = f32x16{};
  static_for_vh<0, NS2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    constexpr int NB = 4 * KPS;    // k-steps of the stage
    Frag b[NB];
#pragma unroll
    for (int e = 0; e < NB; ++e) {
      const int k16 = NB * j + e;
      b[e] = b_operand<DT>(acc[k16 >> 1], k16 & 1);
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
  });
  // ---- h2 = tanh (the bias column n_out[4] = 1), fc3 on the VALU (fp32): v = b3 + sum_k w3[k] h2[k] ----
  {
    const int nb = a.n_out[4], tb = nb >> 5, rb = nb & 31;
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
  if (h == 0 && valid) a.v_out[mr] = v;
  WAIT_VMCNT(0);   // (nothing of the ring in flight: the stream ended with fc2)
}

int g_vhead = 1;

}  // namespace

// the shapes the kernel covers: the reference value head (d_in -> 500 -> 100 -> 1; observation
// widths 128 .. 384 that are a multiple of 32 with at least S fc1 stages)
extern "C" int vhead_shape_ok(const MlpArgs& a) {
  return a.d_in[3] % 32 == 0 && a.d_in[3] >= 128 && a.d_in[3] <= 384 && a.d_out[3] == 512 &&
         a.n_out[3] >= 481 && a.n_out[3] < 512 && a.d_in[4] == 512 && a.d_out[4] == 128 && a.n_out[4] <= 111 &&
         a.n_out[4] >= 97 && a.d_in[5] == 128 && (a.d_in[3] >> 4) % 2 == 0;
}

extern "C" int vhead_applies(const MlpArgs& a) { return g_vhead && vhead_shape_ok(a); }

extern "C" int vhead_rows() { return VH_ROWS; }

template <int DT>
void vhead_launch_t(const MlpArgs& a, hipStream_t s) {
  const int nblk = (a.M + VH_ROWS - 1) / VH_ROWS;
  set_max_lds_once<vhead_kernel<DT>>(vh_lds_bytes());
  hipLaunchKernelGGL((vhead_kernel<DT>), dim3(nblk), dim3(VH_WAVES * 64), vh_lds_bytes(), s, a);
  HIP_CHECK_LAUNCH();
}

extern "C" void launch_vhead_fwd(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_S3) vhead_launch_t<DT_S3>(a, s);
  else vhead_launch_t<DT_BF16>(a, s);
}

extern "C" void set_vhead(int enable) { g_vhead = enable ? 1 : 0; }
