// Row-stationary, weight-streaming fused PPO update for split-bf16 operands (DT_S3, the
// fp32-accurate headline mode).  Same math and outputs as mlp_train_kernel (mlp.hip), which stays
// the generic path for every other precision and shape (the loss is
// the corrected ppo.py:148-167 or the reference DPPO loss train.py:142-161).
//
// Why a second kernel.  mlp_train_kernel keeps a 32-row tile's activations in LDS and lets each
// wave stream ITS weight columns from L2 into registers: at split-bf16 the 32-row tile already
// takes 134 of 160 KiB of LDS, so a weight fragment fetched from L2 feeds only 32 rows, and the
// kernel runs at the per-CU L2->CU rate (~80 GB/s per CU in v_fc1, MI355X_MICROARCH.md
// §Indexed rows: 66-73 GB/s for L2-resident rows) — 1.7 MB of hi|lo weights per 32 rows.
// Here the roles swap:
//  * a workgroup is 4 waves (one per SIMD, up to 512 VGPRs each) and owns 64 batch rows; wave w
//    owns rows 16w..16w+15 through the WHOLE chain (fc1 -> fc2 -> fc3 -> loss -> dgrad fc3 ->
//    dgrad fc2).  Activations never leave registers (MFMA C layout); the next layer's A operand
//    is rebuilt from them through a 2.3 KiB per-wave LDS transpose, so no layer waits on another
//    wave and no activation tile occupies LDS;
//  * the weights stream through an S-stage LDS ring filled by LDS-DMA (global_load_lds_dwordx4,
//    no VGPR holds in-flight data): a stage is 8 split-bf16 fragments (16 KiB), each wave DMAs 2,
//    all 4 read all 8 — one L2 read of a fragment feeds 64 rows, half the L2->CU bytes per row;
//  * the observation rows come through the same ring: one fragment per wave per fc1 k-step,
//    gathered by per-lane source addresses (rows of x_buf, or of idx[]), two k-steps ahead.
//    Counted vmcnt waits + a raw s_barrier keep S-1 stages in flight across every barrier
//    (cdna_hip_programming.md 'Pipelining across barriers'); past-the-end stages re-load the last
//    one, so every wave issues exactly GL DMAs per stage and the count is exact.
// Stream schedule of one tile (steps = ring stages):
//   0                      X[0] | X[1] of every wave
//   fc1, 6 per k-step      stage 0: 4 weight fragments + each wave's X[ks + 2]; stages 1-5: 8 weight
//                          fragments — 44 slots for the 7 policy + 32 value output tiles
//   fc2 policy / value     one per k-step: the 8 output tiles of that k-step
//   fc3                    mu: 2 tiles x 4 k-steps;  v: 1 tile x 4 k-steps
//   dgrad fc3              policy, value: the 8 output tiles (K = 32)
//   dgrad fc2              2 output tiles x 4 k-steps per stage (policy 4 stages, value 16)
#include <type_traits>

#include "kernels.h"
#include "mlp_core.h"

namespace {

using P = Prec<DT_S3>;
using T = P::T;
using Frag = P::Frag;

constexpr float RS_LOG_2PI = 1.8378770664093453f;
constexpr int RS_NPART = 8;           // fixed loss-term columns of a partial row (mlp.hip NPART_FIXED)
constexpr int NW = 4, ROWS = 64;      // waves, rows per workgroup (16 per wave)
constexpr int FB = 2048;              // bytes of one split-bf16 fragment (512 slots x 4 B)
constexpr int NSLOT = 16;             // fragments per ring stage (4 DMA'd by each wave)
constexpr int SPW = NSLOT / NW;       // slots per wave: wave w DMAs slots SPW*w .. SPW*w + SPW-1
constexpr int SB = NSLOT * FB;        // 32 KiB per stage
constexpr int GL = 2 * SPW;           // buffer_load ... lds per wave per stage (hi | lo per fragment)
constexpr int SST = 36;               // fp32 row stride of a [16][32] transpose tile (conflict-free)
constexpr int TILE_F = 16 * SST;
constexpr int P1 = 7, V1 = 32;        // fc1 output tiles held: policy <= 7 (hidden <= 112), value <= 32
constexpr int NACC1 = 8 + V1;         // acc1[t] policy tile t (t = 7 stays 0), acc1[8 + t] value tile t
constexpr int JMAX = 8;               // action dims per lane held in registers (A <= 4 * JMAX)
constexpr int TPR = 4;                // lanes per row in the loss (16 rows x 4 = 64 lanes)
// per-wave scratch (floats): the transpose tile (also mu [16][32] | v [16] in the loss), then a
// region holding the 2-slot observation ring during fc1 and, from the loss on, dL/dmu [16][SST]
// (dL/dv in its column 32) and the wave's partial sums [8 loss terms | 32 dlog_std]
constexpr int XR_F = 2 * FB / 4;
constexpr int WS_F = 2 * TILE_F + XR_F;
static_assert(TILE_F + 40 <= XR_F && 16 * 32 + 16 <= TILE_F, "scratch aliasing");

constexpr int MAX_STEPS = 64;         // stream steps of one tile (59 at Humanoid dims)

// default on: whole iteration 5.34 vs 5.51 ms for the 32-row tile kernel (scripts/ab_iter.py
// rs,tile, same box); set_s3_stream(False, ...) selects the tile kernel (A/B)
int g_rs_enable = 1;
int g_rs_stages = 3;
int g_rs_dense = 1;   // dense-DMA fragment layout (frag_lane_off)

template <int S>
constexpr size_t rs_lds_bytes() { return (size_t)S * SB + (size_t)NW * WS_F * sizeof(float); }

struct Plan {
  int ks1, k3p, k3v;                         // k-steps: fc1, fc3 p / v
  int np1, nv1, np2, nv2, nmu;               // output tiles: fc1 p / v (real), fc2 p / v, mu
  int nd3p, nd3v, nd2p, nd2v, kq2p, kq2v;    // dgrad: tiles of the transposed images, their k-steps
  int s_fc2, s_fc3, s_dg3, s_dg2, s_end;
};

// (the fc2 / dgrad-fc2 extents are the fixed ones mlp_rs_applies admits: 4 policy + 16 value
// k-steps, 4 policy + 16 value output-tile pairs)
DEV Plan make_plan(const MlpArgs& a) {
  Plan p;
  p.ks1 = a.d_in[0] >> 5;
  p.k3p = a.d_in[2] >> 5;
  p.k3v = a.d_in[5] >> 5;
  p.kq2p = a.d_out[1] >> 5;
  p.kq2v = a.d_out[4] >> 5;
  p.np1 = (a.n_out[0] + 15) >> 4;
  p.nv1 = (a.n_out[3] + 15) >> 4;
  p.np2 = a.d_out[1] >> 4;
  p.nv2 = a.d_out[4] >> 4;
  p.nmu = a.d_out[2] >> 4;
  p.nd3p = a.d_in[2] >> 4;
  p.nd3v = a.d_in[5] >> 4;
  p.nd2p = a.d_in[1] >> 4;
  p.nd2v = a.d_in[4] >> 4;
  p.s_fc2 = 3 * p.ks1;
  p.s_fc3 = p.s_fc2 + 10;
  p.s_dg3 = p.s_fc3 + 1;
  p.s_dg2 = p.s_dg3 + 1;
  p.s_end = p.s_dg2 + 10;
  return p;
}

// Ring slot q of stream step st: element offset of a weight fragment, or -1 for a slot no MFMA
// reads (output tiles that are pure padding at the shapes mlp_rs_applies admits: fc1 f >= 39,
// the 8th output tile of fc2 / dgrad fc3 / policy dgrad fc2, fc3 slots 12-15).
// fc1 k-step order is rotated per workgroup (rot = blockIdx % ks1).
// Schedule (16 slots per step; wave w DMAs slots 4w..4w+3):
//   fc1, 3/ks    fragment f = 16 sub + q (f < 7 policy tile f, else value tile f - 7, f >= 39 spare)
//   fc2, 10      step j: fc2 k-steps i = 2j (slots 0-7) and 2j + 1 (slots 8-15), the 8 output tiles
//                each (i < 4 policy k-step i, else value k-step i - 4)
//   fc3, 1       slots 0-7 mu (tile q / 4, k-step q % 4), 8-11 v (k-step q % 4)
//   dgrad fc3, 1 slots 0-7 policy, 8-15 value: the 8 output tiles (K = 32)
//   dgrad fc2,10 step j: output-tile pairs P = 2j (slots 0-7) and 2j + 1 (8-15), tile 2P' + (q / 4 % 2),
//                k-step q % 4 (P < 4 policy pair P' = P, else value pair P' = P - 4)
DEV int fc1_ks(const Plan& p, int ks, int rot) {
  const int k = ks + rot;
  return k >= p.ks1 ? k - p.ks1 : k;
}

DEV int step_src(const MlpArgs& a, const Plan& p, int st, int q, int rot) {
  if (st >= p.s_end) st = p.s_end - 1;
  if (st < p.s_fc2) {
    const int ks0 = st / 3, sub = st - 3 * ks0;
    const int ks = fc1_ks(p, ks0, rot);
    int f = 16 * sub + q;
    if (f >= P1 + V1) return -1;
    if (f < P1) return a.off_w[0] + (int)fm_frag(f < p.np1 ? f : 0, ks, a.d_in[0], 0);
    f -= P1;
    return a.off_w[3] + (int)fm_frag(f < p.nv1 ? f : 0, ks, a.d_in[3], 0);
  }
  if (st < p.s_fc3) {
    const int i = 2 * (st - p.s_fc2) + (q >> 3), t = q & 7;
    if (t == 7) return -1;   // output tile 7 (features 112-127) is padding
    if (i < 4) return a.off_w[1] + (int)fm_frag(t < p.np2 ? t : 0, i, a.d_in[1], 0);
    return a.off_w[4] + (int)fm_frag(t < p.nv2 ? t : 0, i - 4, a.d_in[4], 0);
  }
  if (st == p.s_fc3) {
    if (q < 8) {
      const int t = q >> 2, ks = q & 3;
      return a.off_w[2] + (int)fm_frag(t < p.nmu ? t : 0, ks < p.k3p ? ks : 0, a.d_in[2], 0);
    }
    if (q >= 12) return -1;
    const int ks = q & 3;
    return a.off_w[5] + (int)fm_frag(0, ks < p.k3v ? ks : 0, a.d_in[5], 0);
  }
  if (st == p.s_dg3) {
    if ((q & 7) == 7) return -1;
    if (q < 8) return a.off_wt[2] + (int)fm_frag(q < p.nd3p ? q : 0, 0, a.d_out[2], 0);
    return a.off_wt[5] + (int)fm_frag(q - 8 < p.nd3v ? q - 8 : 0, 0, a.d_out[5], 0);
  }
  const int P = 2 * (st - p.s_dg2) + (q >> 3);
  const bool pol = P < 4;
  const int t = 2 * (pol ? P : P - 4) + ((q >> 2) & 1), ks = q & 3;
  if (pol && t == 7) return -1;
  const int kq = pol ? p.kq2p : p.kq2v;
  const int nt = pol ? p.nd2p : p.nd2v;
  return (pol ? a.off_wt[1] : a.off_wt[4]) +
         (int)fm_frag(t < nt ? t : 0, ks < kq ? ks : 0, pol ? a.d_out[1] : a.d_out[4], 0);
}

// LDS image of one DMA'd 2 KiB fragment.  HS (dense): the first DMA instruction moves the
// fragment's first KiB (lanes 0-31, hi | lo each), the second the second KiB, both as fully used
// 64-byte segments, and each lands as [hi of its 32 lanes][lo of its 32 lanes]: lane l reads hi
// at (l / 32) KiB + 16 (l % 32) and lo 512 bytes on (any 16 consecutive lanes read 256
// contiguous bytes: conflict-free).  !HS: every lane's hi 16 B, then every lane's lo — each DMA
// instruction then touches 16 of every 32 bytes of the whole 2 KiB.
template <bool HS>
DEV int frag_lane_off(int lane) { return HS ? (lane >> 5) * 1024 + (lane & 31) * 16 : lane * 16; }
// per-lane byte offset into a fragment's global 2 KiB for the first of its two DMA instructions
// (the second adds HS ? 1024 : 16 in the SGPR offset; its lo half is at HS ? 512 : 1024 in LDS)
template <bool HS>
DEV unsigned dma_lane_src(int lane) { return HS ? (unsigned)((lane & 31) * 32 + (lane >> 5) * 16) : (unsigned)lane * 32u; }

typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

DEV Frag split8(const f32x8& x) {
  const bf16x8 h = __builtin_convertvector(x, bf16x8);
  const bf16x8 l = __builtin_convertvector(x - __builtin_convertvector(h, f32x8), bf16x8);
  return Frag{h, l};
}

DEV f32x8 join8(const Frag& f) {
  return __builtin_convertvector(f.h, f32x8) + __builtin_convertvector(f.l, f32x8);
}

// C-layout tiles of features c0..c0+15 (v0) and c0+16..c0+31 (v1) -> [16][SST] fp32 (row = lane's
// 4 rows 4*lg + i, column = lr): bank ((4lg + i) * 36 + lr) mod 64 is distinct over the wave
DEV void tp_put(float* tp, const f32x4& v0, const f32x4& v1, int lane) {
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    tp[(4 * lg + i) * SST + lr] = v0[i];
    tp[(4 * lg + i) * SST + 16 + lr] = v1[i];
  }
}

// A operand (row lr, k = 8 * lg .. 8 * lg + 7) of a [16][SST] tile, split to hi | lo.  The two
// reads and their lgkmcnt wait are ONE asm statement: as plain loads, hipcc's waitcnt pass makes
// every read of this per-wave tile wait vmcnt(0) for the ring's in-flight LDS-DMA (it cannot
// tell the two LDS regions apart), which would drain the ring at every chained layer step.  The
// tile is written by this wave's own ds_writes just before (LDS executes one wave's DS
// instructions in order).
DEV Frag tp_getA(const float* tp, int lane) {
  const float* r = tp + (lane & 15) * SST + 8 * (lane >> 4);
  const uint32_t addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)r;
  float4 x0, x1;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(x0), "=&v"(x1)
               : "v"(addr)
               : "memory");
  return split8(f32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w});
}

// the A operands of two [16][SST] tiles: four reads, one wait (one stall per fc2 step, not two)
DEV void tp_get2A(const float* ta, const float* tb, int lane, Frag& fa, Frag& fb) {
  const int o = (lane & 15) * SST + 8 * (lane >> 4);
  const uint32_t aa = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(ta + o);
  const uint32_t ab = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(tb + o);
  float4 x0, x1, y0, y1;
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %5\n\t"
      "ds_read_b128 %3, %5 offset:16\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(x0), "=&v"(x1), "=&v"(y0), "=&v"(y1)
      : "v"(aa), "v"(ab)
      : "memory");
  fa = split8(f32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w});
  fb = split8(f32x8{y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w});
}

// activation chained into the next layer: features >= nb are zero padding except the constant-1
// bias column nb (PackedLayout: the bias is column K of every weight image)
DEV f32x4 bias_col(const f32x4& v, int c, int nb) {
  const float o = c == nb ? 1.f : 0.f;
  return c < nb ? v : f32x4{o, o, o, o};
}

// 4 consecutive m (rows 4lg..4lg+3 of the wave) of feature 16 t + (lane & 15) -> the FM wgrad
// operand, from the lane's base pointer (its hi slot of feature lane & 15, row m) and the byte
// stride tsb of one 16-feature row block:
// fm_index(16 t + f, m, ld) = fm_index(f, m, ld) + t * (ld / 32) * 512
DEV void store_Tt(__bf16* lane_base, int t, size_t tsb, const f32x4& v) {
  const bf16x4v hv = __builtin_convertvector(v, bf16x4v);
  const bf16x4v lv = __builtin_convertvector(v - __builtin_convertvector(hv, f32x4), bf16x4v);
  char* p = reinterpret_cast<char*>(lane_base) + (size_t)t * tsb;
  opnd_store(*reinterpret_cast<const u32x2*>(&hv), reinterpret_cast<u32x2*>(p));
  opnd_store(*reinterpret_cast<const u32x2*>(&lv), reinterpret_cast<u32x2*>(p + 16));
}

// 8 consecutive m (rows 8h..8h+7) of column col of a [16][ld] fp32 tile -> one 32-byte FM group
// of feature `feat`
DEV void store_T8(void* outT, const float* tile, int ld, int col, int h, int feat, int m, int ldT) {
  f32x8 x;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = tile[(8 * h + j) * ld + col];
  const Frag s = split8(x);
  u32x4* o = reinterpret_cast<u32x4*>(P::hi_ptr(reinterpret_cast<T*>(outT), fm_index(feat, m, ldT)));
  opnd_store(*reinterpret_cast<const u32x4*>(&s.h), o);
  opnd_store(*reinterpret_cast<const u32x4*>(&s.l), o + 1);
}

// s_waitcnt vmcnt(BASE + extra): vector-memory operations retire in issue order (loads, stores
// and LDS-DMA together, MI355X_MICROARCH.md §Per-instruction cycle constants), so a wait for the
// DMA batch of step `cur` may leave outstanding every younger operation: the S-2 later batches
// (BASE) AND the `extra` stores / X loads issued since.  Undercounting `extra` is safe (the wait
// is longer), overcounting is not.
template <int BASE, int E = 0>
DEV void wait_vm(int extra) {
  if constexpr (E >= 20 || BASE + E >= 63) {
    WAIT_VMCNT(BASE + E);
  } else {
    if (extra <= E) WAIT_VMCNT(BASE + E);
    else wait_vm<BASE, E + 1>(extra);
  }
}

// phase timeline (diagnostics, scripts/phase_timeline.py): lane 0 of each wave of every
// tstamp_every-th workgroup records the shader clock at the phase boundaries
#define RS_STAMP(i)                                                                               \
  do {                                                                                            \
    if (a.tstamp != nullptr && (blockIdx.x % a.tstamp_every) == 0 && lane == 0)                   \
      a.tstamp[((size_t)(blockIdx.x / a.tstamp_every) * NW + wave) * 16 + (i)] =                  \
          __builtin_amdgcn_s_memtime();                                                           \
  } while (0)

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1 (register-array indices
// stay constants whatever the unroller decides for big bodies)
template <int B, int E, typename F>
DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// A stage's fragments q in [0, N) with bit q of MASK set, in two register halves: the second
// half's LDS reads are in flight while the first half's MFMAs run (left to itself hipcc reads each
// fragment right before its 3 MFMAs and, at one wave per SIMD, exposes the LDS latency once per
// fragment).  f(integral_constant<q>, fragment).
template <bool HS, unsigned MASK, int N, typename F>
DEV void for_stage(const char* stg, int lane, F&& f) {
  constexpr int H = N / 2;
  Frag b[N];
  // one lane address per stage; every fragment then is an immediate offset (q * FB < 64 KiB)
  const char* base = stg + frag_lane_off<HS>(lane);
  auto rd = [&](auto qc) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
    if constexpr ((MASK >> q) & 1u)
      b[q] = Frag{*reinterpret_cast<const bf16x8*>(base + q * FB),
                  *reinterpret_cast<const bf16x8*>(base + q * FB + (HS ? 512 : 1024))};
  };
  static_for<0, H>(rd);
  __builtin_amdgcn_sched_barrier(0);
  static_for<H, N>(rd);
  static_for<0, H>([&](auto qc) __attribute__((always_inline)) {
    if constexpr ((MASK >> decltype(qc)::value) & 1u) f(qc, b[decltype(qc)::value]);
  });
  __builtin_amdgcn_sched_barrier(0);
  static_for<H, N>([&](auto qc) __attribute__((always_inline)) {
    if constexpr ((MASK >> decltype(qc)::value) & 1u) f(qc, b[decltype(qc)::value]);
  });
}

// sum over the 16 lanes with the same lane & 3 (the wave's 16 rows in the loss layout), the same
// value in every one of them, fixed order: DPP row rotations by 4 and 8 inside each 16-lane row,
// then two cross-row exchanges
DEV float rowsum16(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x124, 0xf, 0xf, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x128, 0xf, 0xf, true));
  x += __shfl_xor(x, 16, 64);
  return x + __shfl_xor(x, 32, 64);
}

template <int G>
DEV float gsum(float x) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) x += __shfl_xor(x, o, 64);
  return x;
}

template <int S, bool HS>
__global__ __launch_bounds__(NW * 64, 1) void mlp_train_rs_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];   // the kernel's ONLY LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * ROWS;
  const int A = a.A;
  const Plan p = make_plan(a);
  char* ring = smem;
  float* scr = reinterpret_cast<float*>(smem + (size_t)S * SB) + wave * WS_F;
  float* tp = scr;
  float* tp2 = scr + TILE_F;      // second transpose tile (two operands per fc2 step)
  float* mus = tp;                // (loss only)
  float* vs = tp + 16 * 32;       // (loss only)
  float* dmu = scr + 2 * TILE_F;  // (after fc1: aliases the observation ring)
  float* wpart = dmu + TILE_F;

  // source row of tile row r (rows past M re-read row m0: finite data, zero gradient)
  auto src_of = [&](int r) __attribute__((always_inline)) {
    const int rr = (m0 + r < a.M) ? m0 + r : m0;
    return a.idx ? a.idx[rr] : a.row0 + rr;
  };
  const int mw = m0 + 16 * wave;   // first row (m) of this wave
  // the loss's row (TPR lanes per row): its source index is read before any DMA is in flight
  const int lrow = lane / TPR, lsub = lane % TPR;
  const bool lvalid = mw + lrow < a.M;
  const int lsrc = src_of(16 * wave + lrow);

  // DMA sources: raw buffer resources, so an issue is 2 buffer_load ... lds per slot with the
  // per-lane part of the address in a constant VGPR (weights: the lane's 32 bytes of a
  // fragment; X: the lane's row and k-group) and the step's offset in an SGPR
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x_buf), (short)0, 0x7fffffff, 0x00020000);
  const unsigned vw = dma_lane_src<HS>(lane);
  // X fragment lane fl = (row fl & 15, k-group fl >> 4): with HS the first instruction moves
  // fragment lanes 0-31 (k-groups 0, 1: 64 contiguous bytes of each of the 16 rows), the second
  // k-groups 2, 3 (+64 bytes)
  const unsigned vx =
      HS ? (unsigned)((size_t)src_of(16 * wave + lr) * a.d_in[0] * sizeof(T) + 32 * ((lane >> 4) & 1) + 16 * (lane >> 5))
         : (unsigned)(((size_t)src_of(16 * wave + lr) * a.d_in[0] + 8 * lg) * sizeof(T));

  // The stream's sources, computed once per workgroup and held in two VGPRs: lane l of cw0 packs
  // this wave's slot codes 4w, 4w+1 of step l, cw1 its slots 4w+2, 4w+3, 16 bits each — a weight
  // fragment index (element offset / 512), or 0x8000 | ks for this wave's X fragment of k-step
  // ks.  An issue reads its step with v_readlane: no LDS table read (which hipcc would make wait
  // for the ring's DMA) and none of step_src's scalar phase arithmetic per step (at one wave per
  // SIMD every issued instruction costs the MFMA pipe ~4 cycles).
  const int rot = (int)(blockIdx.x % (unsigned)p.ks1);
  auto code16 = [&](int st, int q) __attribute__((always_inline)) {
    // a slot no MFMA reads re-loads the step's slot 0 (every wave then issues the same number of
    // DMAs per step, so the vmcnt counts are compile-time; skipping them measured slower: 297.5
    // vs 277.9 us, the per-wave runtime wait counts and the uneven batches cost more than the
    // saved L2 reads)
    int c = step_src(a, p, min(st, p.s_end - 1), q, rot);
    if (c < 0) c = step_src(a, p, min(st, p.s_end - 1), 0, rot);
    return (uint32_t)(c >> 9);
  };
  const uint32_t cw0 = code16(lane, SPW * wave) | (code16(lane, SPW * wave + 1) << 16);
  const uint32_t cw1 = code16(lane, SPW * wave + 2) | (code16(lane, SPW * wave + 3) << 16);

  const bool abl_dma = (a.ablate & 2) != 0;   // diagnostics only (phase_timeline TIMELINE_ABLATE=2)
  const bool abl_x = (a.ablate & 8) != 0;     // diagnostics only: no observation DMA (stale X)
  auto issue = [&](int st, int stage) __attribute__((always_inline)) {
    if (abl_dma) return;
    const int l = min(st, MAX_STEPS - 1);
    const uint32_t w01 = __builtin_amdgcn_readlane(cw0, l);
    const uint32_t w23 = __builtin_amdgcn_readlane(cw1, l);
    __attribute__((address_space(3))) char* stg =
        (__attribute__((address_space(3))) char*)(ring + stage * SB) + SPW * wave * FB;
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const uint32_t code = ((u < 2 ? w01 : w23) >> (16 * (u & 1))) & 0xffffu;
      // (the instruction's immediate offset would move the LDS destination too: the hi | lo
      // 16-byte halves differ in the SGPR offset instead)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, stg + u * FB, 16, vw, code * 2048u, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, stg + u * FB + 1024, 16, vw, code * 2048u + (HS ? 1024u : 16u), 0, 0);
    }
  };
  // This wave's observation fragments (its 16 rows, 32 features of k-step ks) go to a private
  // 2-slot LDS ring, DMA'd two k-steps (6 stream steps) ahead of use: a gather from HBM / the
  // Infinity Cache outlasts the weight ring's lookahead.  The ring aliases the loss scratch
  // (dead until fc3).
  char* xring = reinterpret_cast<char*>(scr + 2 * TILE_F);
  auto issue_x = [&](int ks0) __attribute__((always_inline)) {
    if (abl_dma || abl_x) return;
    const uint32_t xo = (uint32_t)fc1_ks(p, min(ks0, p.ks1 - 1), rot) * 128u;
    __attribute__((address_space(3))) char* d = (__attribute__((address_space(3))) char*)(xring + (ks0 & 1) * FB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, d, 16, vx, xo, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, d + 1024, 16, vx, xo + (HS ? 64u : 16u), 0, 0);
  };
  // its fragment of k-step ks (the DMA landed: every vmcnt wait since covers it, in issue order);
  // read and waited in one asm statement (a plain LDS load would wait for the ring's DMA)
  auto read_x = [&](int ks0) __attribute__((always_inline)) {
    const uint32_t addr =
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(xring + (ks0 & 1) * FB) + frag_lane_off<HS>(lane);
    bf16x8 h, l;
    const uint32_t addr_lo = addr + (uint32_t)(HS ? 512 : 1024);
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(h), "=&v"(l)
                 : "v"(addr), "v"(addr_lo)
                 : "memory");
    return Frag{h, l};
  };
  int cur = 0, cst = 0, ist = 0;   // next step to consume, its stage, the stage refill() fills
  // Younger-than-the-waited-batch bookkeeping.  A step's stores precede its refill, so they are
  // younger than the batches of the next S-2 steps; the X loads follow the refill, so they are
  // younger than the next S-1 steps' batches (and every report made at a wait after the previous
  // step's refill stays younger for that many waits).
  constexpr int NH = S - 2 > 0 ? S - 2 : 1, NX = S - 1;
  int hist[NH], xhist[NX];
#pragma unroll
  for (int i = 0; i < NH; ++i) hist[i] = 0;
#pragma unroll
  for (int i = 0; i < NX; ++i) xhist[i] = 0;
  // Ring sync for step `cur`: this wave's DMAs of it by count (every younger vector-memory
  // operation may stay in flight), every wave's by the barrier, which also retires every wave's
  // reads of the stage refill() refills.  `stores` / `xs` = store / X-load instructions issued
  // during the previous step (undercounting is safe, overcounting is not).
  auto wait_step = [&](int stores, int xs = 0) __attribute__((always_inline)) -> const char* {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = NH - 1; i > 0; --i) hist[i] = hist[i - 1];
    hist[0] = stores;
#pragma unroll
    for (int i = NX - 1; i > 0; --i) xhist[i] = xhist[i - 1];
    xhist[0] = xs;
    int extra = 0;
    if constexpr (S > 2) {
#pragma unroll
      for (int i = 0; i < NH; ++i) extra += hist[i];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) extra += xhist[i];
    wait_vm<GL * (S - 2)>(extra);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* stg = ring + cst * SB;
    ist = cst == 0 ? S - 1 : cst - 1;
    cst = cst + 1 == S ? 0 : cst + 1;
    ++cur;
    return stg;
  };
  // last thing of every step (after its reads and stores): DMA step cur + S - 2 into the stage the
  // previous step used
  auto refill = [&]() __attribute__((always_inline)) { issue(cur + S - 2, ist); };
  RS_STAMP(0);
  issue_x(0);
  issue_x(1);
#pragma unroll
  for (int st = 0; st < S - 1; ++st) issue(st, st);

  // ---------------- fc1 (policy + value heads share X) ----------------
  f32x4 acc1[NACC1];
#pragma unroll
  for (int t = 0; t < NACC1; ++t) acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* stg;
  const bool want_xT = !a.xT_ready && (a.ablate & 1) == 0;
  Frag xa;
  // fc1 weight fragment f (of a k-step) -> accumulator
  auto mma1 = [&](auto fc, const Frag& b) __attribute__((always_inline)) {
    constexpr int f = decltype(fc)::value;
    if constexpr (f < P1 + V1) {
      constexpr int t = f < P1 ? f : f + 1;
      acc1[t] = P::mma(acc1[t], xa, b);
    }
  };
  for (int ks = 0; ks < p.ks1; ++ks) {
    // (sub 0 issues the X^T stores, if any, and — after its refill — the 2 X loads of ks + 2)
    static_for<0, 3>([&](auto sc) __attribute__((always_inline)) {
      constexpr int sub = decltype(sc)::value;
      // (sub 1 waits with sub 0's 2 X loads outstanding; sub 0's X^T stores, when the rollout did
      // not write X^T, are not counted — an undercount, so the wait also covers them — which
      // keeps every fc1 wait count a compile-time constant)
      stg = sub == 1 ? wait_step(0, 2) : wait_step(0);
      if constexpr (sub == 0) xa = read_x(ks);
      // (sub 2: fragments f = 32..38 only; f >= 39 are not DMA'd)
      constexpr unsigned M1 = sub == 2 ? ((1u << (P1 + V1 - 32)) - 1u) : 0xffffu;
      for_stage<HS, M1, 16>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
        mma1(std::integral_constant<int, 16 * sub + decltype(qc)::value>{}, b);
      });
      if constexpr (sub == 0) {
        if (want_xT) {
          // the rollout did not write this call's X^T: transpose the wave's 16 x 32 block here
          const f32x8 x = join8(xa);
          float4* w = reinterpret_cast<float4*>(tp + lr * SST + 8 * lg);
          w[0] = float4{x[0], x[1], x[2], x[3]};
          w[1] = float4{x[4], x[5], x[6], x[7]};
          store_T8(a.xT, tp, SST, lane >> 1, lane & 1, 32 * fc1_ks(p, ks, rot) + (lane >> 1),
                   mw + 8 * (lane & 1), a.ldT);
        }
        refill();
        issue_x(ks + 2);   // into the slot X[ks] just left
      } else {
        refill();
      }
    });
  }

  RS_STAMP(1);
  // ---------------- fc2: h1 = tanh(fc1) chained two tiles (one k-step) at a time ----------------
  // Software-pipelined: step j's MFMAs and step j+1's two operands (tanh, the h1^T stores, the
  // LDS transposes) share one scheduling region, so the VALU work fills the MFMA shadow.
  const int n1p = a.n_out[0], n1v = a.n_out[3], n2p = a.n_out[1], n2v = a.n_out[4];
  f32x4 acc2p[8], acc2v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc2p[t] = acc2v[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int mr = mw + 4 * lg;   // first of the lane's 4 rows (C layout)
  // per-lane base pointers of the wgrad operands this kernel writes (feature lane & 15, row mr)
  const size_t tsb = (size_t)a.ldT * 64;
  auto lane_base = [&](void* buf) __attribute__((always_inline)) {
    return P::hi_ptr(reinterpret_cast<T*>(buf), fm_index(lr, mr, a.ldT));
  };
  __bf16* const bh1p = lane_base(a.h1pT);
  __bf16* const bh1v = lane_base(a.h1vT);
  __bf16* const bh2p = lane_base(a.h2pT);
  __bf16* const bh2v = lane_base(a.h2vT);
  __bf16* const bg2p = lane_base(a.g2pT);
  __bf16* const bg2v = lane_base(a.g2vT);
  __bf16* const bg1p = lane_base(a.g1pT);
  __bf16* const bg1v = lane_base(a.g1vT);
  // operands of fc2 k-steps 2J and 2J + 1 (i < 4: policy k-step i, else value k-step i - 4):
  // tanh in place, the h1^T stores, both transposes, one LDS wait; returns the stores.  Only the
  // last k-step of a head holds features >= its width (the bias column and padding): the shapes
  // mlp_rs_applies admits make every other k-step's tiles all real.
  auto prep2 = [&](auto Jc, Frag& fa, Frag& fb) __attribute__((always_inline)) -> int {
    constexpr int J = decltype(Jc)::value;
    int nst = 0;
    static_for<0, 2>([&](auto uc) __attribute__((always_inline)) {
      constexpr int u = decltype(uc)::value;
      constexpr int i = 2 * J + u;
      constexpr bool pol = i < 4;
      constexpr int ks = pol ? i : i - 4;
      constexpr int t0 = pol ? 2 * ks : 8 + 2 * ks;
      constexpr bool last = pol ? ks == 3 : ks == 15;
      const int nr = pol ? n1p : n1v;
      const f32x4 h0 = act_tanh4<DT_S3>(acc1[t0]), h1 = act_tanh4<DT_S3>(acc1[t0 + 1]);
      acc1[t0] = h0;
      acc1[t0 + 1] = h1;
      const int c0 = 32 * ks + lr;
      __bf16* oT = pol ? bh1p : bh1v;
      float* tt = u == 0 ? tp : tp2;
      // (the last k-step's features >= nr are the bias column (1) and zero padding: stored
      // as such, rewriting the operand's constant bias row with its own value, so every lane
      // stores and the step's store count is a compile-time constant)
      const f32x4 s0 = last ? bias_col(h0, c0, nr) : h0, s1 = last ? bias_col(h1, c0 + 16, nr) : h1;
      store_Tt(oT, 2 * ks, tsb, s0);
      store_Tt(oT, 2 * ks + 1, tsb, s1);
      nst += 4;
      tp_put(tt, s0, s1, lane);
    });
    tp_get2A(tp, tp2, lane, fa, fb);
    return nst;
  };
  Frag ah0, ah1;
  int nst = prep2(std::integral_constant<int, 0>{}, ah0, ah1);
  static_for<0, 10>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    stg = wait_step(nst);
    for_stage<HS, 0x7f7fu, 16>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      constexpr int i = 2 * j + (q >> 3);
      if constexpr (i < 4) acc2p[q & 7] = P::mma(acc2p[q & 7], q < 8 ? ah0 : ah1, b);
      else acc2v[q & 7] = P::mma(acc2v[q & 7], q < 8 ? ah0 : ah1, b);
    });
    if constexpr (j + 1 < 10) {
      nst = prep2(std::integral_constant<int, j + 1>{}, ah0, ah1);
    } else {
      RS_STAMP(2);
      // h2 = tanh(fc2), kept for dgrad fc3; its stores belong to this step (before the refill)
      nst = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc2p[q] = act_tanh4<DT_S3>(acc2p[q]);
        acc2v[q] = act_tanh4<DT_S3>(acc2v[q]);
        const int c = 16 * q + lr;
        store_Tt(bh2p, q, tsb, bias_col(acc2p[q], c, n2p));   // (bias row 1, padding 0)
        store_Tt(bh2v, q, tsb, bias_col(acc2v[q], c, n2v));
        nst += 4;
      }
    }
    refill();
  });

  // loss inputs of this lane's row (TPR lanes per row): issued now, consumed after fc3
  // (every global value the loss reads is loaded here: with the ring's LDS-DMA in flight, hipcc
  // waits vmcnt(0) at the first use of an ordinary load, so they must all be in flight together)
  const bool ref_loss = a.loss_kind != 0;
  float actv[JMAX], lsv[JMAX], lsov[JMAX], mupv[JMAX];
#pragma unroll
  for (int q = 0; q < JMAX; ++q) {
    const int j = lsub + q * TPR;
    actv[q] = j < A ? a.actions[(size_t)lsrc * A + j] : 0.f;
    lsv[q] = j < A ? a.log_std[j] : 0.f;
    lsov[q] = (ref_loss && j < A) ? a.log_std_old[j] : 0.f;
    mupv[q] = (ref_loss && j < A) ? a.mu_prev[(size_t)lsrc * A + j] : 0.f;
  }
  const float l_adv = a.adv[lsrc], l_ret = a.ret[lsrc];
  const float l_lpo = !ref_loss ? a.logp_old[lsrc] : 0.f;
  const float l_vold = !ref_loss ? a.v_old[lsrc] : 0.f;
  const float l_vprev = ref_loss ? a.v_prev[lsrc] : 0.f;

  // ---------------- fc3 (mu, v) + loss: one step ----------------
  Frag am[4], av[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int c0 = 32 * ks + lr;
    tp_put(tp, bias_col(acc2p[2 * ks], c0, n2p), bias_col(acc2p[2 * ks + 1], c0 + 16, n2p), lane);
    am[ks] = tp_getA(tp, lane);
    tp_put(tp, bias_col(acc2v[2 * ks], c0, n2v), bias_col(acc2v[2 * ks + 1], c0 + 16, n2v), lane);
    av[ks] = tp_getA(tp, lane);
  }
  stg = wait_step(nst);
  f32x4 amu0 = f32x4{0.f, 0.f, 0.f, 0.f}, amu1 = amu0, av0 = amu0;
  for_stage<HS, 0x0fffu, 12>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
    if constexpr (q < 4) amu0 = P::mma(amu0, am[q], b);
    else if constexpr (q < 8) amu1 = P::mma(amu1, am[q - 4], b);
    else av0 = P::mma(av0, av[q - 8], b);
  });

  RS_STAMP(3);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * lg + i;
    if (lr < A) mus[r * 32 + lr] = amu0[i];
    if (16 + lr < A) mus[r * 32 + 16 + lr] = amu1[i];
    if (lr == 0) vs[r] = av0[i];
  }
  {
    // zero the dL/dmu tile (columns >= A are the padded K of dgrad fc3; column 32 takes dL/dv)
    float4* z0 = reinterpret_cast<float4*>(dmu + lr * SST + 8 * lg);
    z0[0] = z0[1] = float4{0.f, 0.f, 0.f, 0.f};
  }
  // per-lane dL/dlog_std (j = lsub + 4q) and, in the lsub == 0 lanes, the row's loss terms: summed
  // over the wave's 16 rows by a fixed xor tree after the loss (deterministic)
  float dlsv[JMAX], lt[6];
#pragma unroll
  for (int q = 0; q < JMAX; ++q) dlsv[q] = 0.f;
#pragma unroll
  for (int k = 0; k < 6; ++k) lt[k] = 0.f;
  {
    const int r = lrow, sub = lsub, src = lsrc;
    const bool valid = lvalid;
    // action dim j = sub + q * TPR < A <= TPR * JMAX: every loop over j is unrolled over q, so
    // actv[q] is a static register index
    const float advv = l_adv;
    const float v = vs[r];
    const float cvar = a.std_var ? 0.5f : 1.f;
    float lclip = 0.f, lent = 0.f, kl = 0.f, cf = 0.f, vold;
    if (a.loss_kind == 0) {
      // ---- corrected PPO (ppo.py:148-167) ----
      float logp = 0.f;
#pragma unroll
      for (int q = 0; q < JMAX; ++q) {
        const int j = sub + q * TPR;
        if (j >= A) break;
        const float lsig = cvar * lsv[q];
        const float z = (actv[q] - mus[r * 32 + j]) * __expf(-lsig);
        logp += -0.5f * z * z - 0.5f * RS_LOG_2PI - lsig;
      }
      logp = gsum<TPR>(logp);
      const float lrat = logp - l_lpo;
      const float ratio = __expf(lrat);
      const float s1 = ratio * advv;
      const float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * advv;
      lclip = -fminf(s1, s2);
      const float dlogp = (s1 <= s2) ? -advv * ratio : 0.f;
      kl = (ratio - 1.f) - lrat;
      cf = (fabsf(ratio - 1.f) > a.clip) ? 1.f : 0.f;
#pragma unroll
      for (int q = 0; q < JMAX; ++q) {
        const int j = sub + q * TPR;
        if (j >= A) break;
        const float lsig = cvar * lsv[q];
        const float isig = __expf(-lsig);
        const float z = (actv[q] - mus[r * 32 + j]) * isig;
        dmu[r * SST + j] = valid ? dlogp * z * isig : 0.f;
        // d/dlog_std: logp term + entropy bonus (-ent_coeff * sum_j log sigma_j)
        dlsv[q] = valid ? (dlogp * (z * z - 1.f) - a.ent_coeff) * cvar : 0.f;
        lent += -a.ent_coeff * (0.5f + 0.5f * RS_LOG_2PI + lsig);
      }
      lent = gsum<TPR>(lent);
      vold = l_vold;
    } else {
      // ---- reference DPPO loss (train.py:142-161): per-dim pdf ratio, variance convention ----
      const float invA = 1.f / (float)A;
      const bool first = a.first_step != 0;
#pragma unroll
      for (int q = 0; q < JMAX; ++q) {
        const int j = sub + q * TPR;
        if (j >= A) break;
        const float mu = mus[r * 32 + j];
        const float var = __expf(lsv[q]);
        const float mu_o = first ? mu : mupv[q];
        const float var_o = first ? var : __expf(lsov[q]);
        const float x = actv[q];
        const float pd = __expf(-(x - mu) * (x - mu) / (2.f * var)) * rsqrtf(2.f * var * 3.14159265358979f);
        const float po = __expf(-(x - mu_o) * (x - mu_o) / (2.f * var_o)) * rsqrtf(2.f * var_o * 3.14159265358979f);
        const float ratio = pd / (1e-10f + po);
        const float s1 = ratio * advv;
        const float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * advv;
        lclip += -fminf(s1, s2) * invA;
        const float dratio = (s1 <= s2) ? -advv * invA : 0.f;
        float dp = dratio / (1e-10f + po);
        const float lgp = logf(pd + 1e-5f);
        lent += -a.ent_coeff * pd * lgp * invA;
        dp += -a.ent_coeff * invA * (lgp + pd / (pd + 1e-5f));
        dmu[r * SST + j] = valid ? dp * pd * (x - mu) / var : 0.f;
        dlsv[q] = valid ? dp * pd * ((x - mu) * (x - mu) / (2.f * var) - 0.5f) : 0.f;
        cf += (fabsf(ratio - 1.f) > a.clip) ? invA : 0.f;
        if (valid) a.mu_prev[(size_t)src * A + j] = mu;   // train.py:164 model_old <- model
      }
      lclip = gsum<TPR>(lclip);
      lent = gsum<TPR>(lent);
      cf = gsum<TPR>(cf);
      vold = first ? v : l_vprev;
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
      dmu[r * SST + 32] = valid ? dv : 0.f;
      const float vm = valid ? 1.f : 0.f;
      lt[0] = lclip * vm; lt[1] = lv * vm; lt[2] = lent * vm; lt[3] = kl * vm; lt[4] = cf * vm; lt[5] = vm;
    }
  }
  // the wave's partial sums over its 16 rows (lanes lsub + 4r)
#pragma unroll
  for (int q = 0; q < JMAX; ++q) dlsv[q] = rowsum16(dlsv[q]);
#pragma unroll
  for (int k = 0; k < 6; ++k) lt[k] = rowsum16(lt[k]);
  if (lane < TPR) {
#pragma unroll
    for (int q = 0; q < JMAX; ++q)
      if (lane + TPR * q < A) wpart[RS_NPART + lane + TPR * q] = dlsv[q];
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) wpart[k] = lt[k];
      wpart[6] = wpart[7] = 0.f;
    }
  }
  // dY^T of the output layers: item = (feature, 8-row half) of this wave's 16 rows (dL/dv is
  // column 32 of the dL/dmu tile)
  for (int it = lane; it < 2 * A + 2; it += 64) {
    if (it < 2 * A) store_T8(a.g3pT, dmu, SST, it >> 1, it & 1, it >> 1, mw + 8 * (it & 1), a.ldT);
    else store_T8(a.g3vT, dmu, SST, 32, it - 2 * A, 0, mw + 8 * (it - 2 * A), a.ldT);
  }

  refill();   // (the loss's stores are not counted: the next S-2 waits also wait for them)

  RS_STAMP(4);
  // ---------------- dgrad fc3: dpre2 = (dY W3) * (1 - h2^2), both heads in one step ----------------
  Frag a2p[4], a2v[4];
  {
    // dL/dv as the A operand of the value head's dgrad: K = 32 with only k = 0 nonzero
    const Frag adp = tp_getA(dmu, lane);
    float dvv;
    {
      const uint32_t addr =
          (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(dmu + lr * SST + 32);
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(dvv) : "v"(addr) : "memory");
    }
    const Frag adv = split8(f32x8{lg == 0 ? dvv : 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f});
    stg = wait_step(0);
    f32x4 dp[8], dv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) dp[q] = dv[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    for_stage<HS, 0x7f7fu, 16>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      if constexpr (q < 8) dp[q] = P::mma(f32x4{0.f, 0.f, 0.f, 0.f}, adp, b);
      else dv[q - 8] = P::mma(f32x4{0.f, 0.f, 0.f, 0.f}, adv, b);
    });
    nst = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = 16 * q + lr;
      dp[q] = c < n2p ? dp[q] * (1.0f - acc2p[q] * acc2p[q]) : f32x4{0.f, 0.f, 0.f, 0.f};
      dv[q] = c < n2v ? dv[q] * (1.0f - acc2v[q] * acc2v[q]) : f32x4{0.f, 0.f, 0.f, 0.f};
      // (dY^T rows past the layer's width: zeros; wgrad's output rows there are never gathered)
      store_Tt(bg2p, q, tsb, dp[q]);
      store_Tt(bg2v, q, tsb, dv[q]);
      nst += 4;
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      tp_put(tp, dp[2 * ks], dp[2 * ks + 1], lane);
      a2p[ks] = tp_getA(tp, lane);
      tp_put(tp, dv[2 * ks], dv[2 * ks + 1], lane);
      a2v[ks] = tp_getA(tp, lane);
    }
    refill();
  }

  RS_STAMP(5);
  // ---------------- dgrad fc2: g1 = (dpre2 W2) * (1 - h1^2), only the wgrad operand ----------------
  // 10 steps of two output-tile pairs (4 policy + 16 value pairs); step j's epilogue (dtanh +
  // stores) runs in step j+1 beside its MFMAs
  f32x4 gq[4];   // previous step's 4 tiles: pair 2j' tiles 0,1 and pair 2j'+1 tiles 0,1
#pragma unroll
  for (int u = 0; u < 4; ++u) gq[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto epi_pair = [&](int P_, const f32x4& g0, const f32x4& g1) __attribute__((always_inline)) -> int {
    const bool pol = P_ < 4;
    const int jj = pol ? P_ : P_ - 4;
    const int t0 = pol ? 2 * jj : 8 + 2 * jj;
    __bf16* oT = pol ? bg1p : bg1v;
    // (rows past the width carry don't-care values: wgrad's output rows there are never gathered)
    store_Tt(oT, 2 * jj, tsb, g0 * (1.0f - acc1[t0] * acc1[t0]));
    store_Tt(oT, 2 * jj + 1, tsb, g1 * (1.0f - acc1[t0 + 1] * acc1[t0 + 1]));
    return 4;
  };
  static_for<0, 10>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    stg = wait_step(nst);
    f32x4 g[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) g[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr unsigned M2 = j == 1 ? 0x0fffu : 0xffffu;   // policy pair 3's tile 7 is padding
    for_stage<HS, M2, 16>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      constexpr int P_ = 2 * j + (q >> 3);
      const Frag& a2 = P_ < 4 ? a2p[q & 3] : a2v[q & 3];
      g[q >> 2] = P::mma(g[q >> 2], a2, b);
    });
    if constexpr (j > 0) {
      nst = epi_pair(2 * j - 2, gq[0], gq[1]);
      nst += epi_pair(2 * j - 1, gq[2], gq[3]);
    } else {
      nst = 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) gq[u] = g[u];
    refill();
    if constexpr (j == 1) RS_STAMP(6);
  });
  epi_pair(18, gq[0], gq[1]);
  epi_pair(19, gq[2], gq[3]);
  RS_STAMP(7);

  // ---------------- per-workgroup partials (deterministic fixed order) ----------------
  WAIT_VMCNT(0);   // no DMA may outlive the workgroup's LDS
  __syncthreads();
  const float* sc0 = reinterpret_cast<const float*>(smem + (size_t)S * SB);
  for (int q = tid; q < RS_NPART + A; q += NW * 64) {
    float s = 0.f;
    for (int w = 0; w < NW; ++w) s += sc0[w * WS_F + 3 * TILE_F + q];   // wpart of wave w
    a.part[(size_t)blockIdx.x * a.npart + q] = s;
  }
}

template <int S, bool HS>
void rs_launch(const MlpArgs& a, hipStream_t s) {
  const size_t lds = rs_lds_bytes<S>();
  set_max_lds_once<mlp_train_rs_kernel<S, HS>>(lds);
  const int nblk = (a.M + ROWS - 1) / ROWS;
  hipLaunchKernelGGL((mlp_train_rs_kernel<S, HS>), dim3(nblk), dim3(NW * 64), lds, s, a);
  HIP_CHECK_LAUNCH();
}

}  // namespace

// shapes the streaming kernel covers: its register tiles and unrolled step bodies are those of
// the reference network (policy 100-100, value 500-100; hidden widths 97-112 / 497-511 / 97-112
// give the same tile counts and padding tiles), any observation width <= 383 and action width <= 32; every other
// shape runs the 32-row tile kernel
extern "C" int mlp_rs_applies(const MlpArgs& a) {
  if (!g_rs_enable) return 0;
  // the observation gather uses a raw buffer resource with 32-bit per-lane byte offsets: an
  // x_buf of 2 GiB or more (e.g. > 1.4 M Humanoid rows at split-bf16) takes the tile kernel,
  // whose row loads use 64-bit addresses
  if (a.x_bytes >= ((int64_t)1 << 31)) return 0;
  return a.d_in[0] <= 384 && a.d_in[0] == a.d_in[3] && (a.n_out[0] + 15) / 16 == P1 &&
         (a.n_out[3] + 15) / 16 == V1 && a.d_in[1] == 128 && a.d_in[4] == 512 && a.d_in[2] == 128 &&
         a.d_in[5] == 128 && a.d_out[1] == 128 && a.d_out[4] == 128 && a.d_out[2] == 32 && a.d_out[5] == 32 &&
         a.n_out[1] > 96 && a.n_out[1] <= 112 && a.n_out[4] > 96 && a.n_out[4] <= 112 && a.A >= 1 && a.A <= 32;
}

// (a 4-stage ring measured no faster, 279 vs 274 us, and no longer fits beside two transpose
// tiles per wave)
extern "C" size_t mlp_rs_lds_bytes() { return g_rs_stages == 2 ? rs_lds_bytes<2>() : rs_lds_bytes<3>(); }
static_assert(rs_lds_bytes<3>() <= 160 * 1024, "3-stage ring must fit LDS");

extern "C" void launch_mlp_train_rs(const MlpArgs& a, hipStream_t s) {
  if (g_rs_dense) {
    if (g_rs_stages == 2) rs_launch<2, true>(a, s);
    else rs_launch<3, true>(a, s);
  } else {
    if (g_rs_stages == 2) rs_launch<2, false>(a, s);
    else rs_launch<3, false>(a, s);
  }
}

// 0 = off, else stages + 10 * dense-DMA layout
extern "C" int s3_stream_state() { return g_rs_enable ? g_rs_stages + 10 * g_rs_dense : 0; }

extern "C" void set_s3_stream(int enable, int stages, int dense) {
  g_rs_enable = enable ? 1 : 0;
  if (stages == 2 || stages == 3) g_rs_stages = stages;
  if (dense >= 0) g_rs_dense = dense ? 1 : 0;
}
