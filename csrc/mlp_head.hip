// Per-head, row-stationary, weight-streaming fused PPO update, in split-bf16 (bf16x3, the
// fp32-accurate headline precision) and bf16 (BASELINE config 2; config 5's fp8 mode runs the bf16
// kernels with e4m3 forward GEMMs — value fc1, policy fc1 + fc2 — and e4m3 wgrad operands).  SURVEY K4, K5, K8, K10, K11; loss = corrected ppo.py:148-167 or the reference
// DPPO loss train.py:142-161; the backward of model.py:35-45 through one head.
//
// The actor-critic's two heads share only their input rows: the policy loss (clip + entropy,
// log_std) reads p_fc1 -> p_fc2 -> mu, the value loss v_fc1 -> v_fc2 -> v.  So the update runs
// as TWO kernels, one per head, instead of one over the whole network:
//  * each head's whole gradient chain (kernel -> wgrad -> gather -> [all-reduce] -> Adam) is
//    independent of the other head's, so at world size > 1 one head's RCCL all-reduce overlaps
//    the other head's kernels (runtime/engine_hip.py), the reference's chief sum
//    (chief.py:13-20) off the critical path;
//  * a head alone needs half the registers of both, so one 128-row workgroup streams a head's
//    weights once for all its rows: every weight fragment a workgroup pulls from L2 into its LDS
//    ring feeds 128 rows instead of 64 — half the L2->CU weight bytes per row, the bound of the
//    round-2 64-row kernel (docs/ARCHITECTURE.md: ~20 B/clk per CU of LDS-DMA).
// The observation rows are read once per head (2 x 100 MB per epoch at the bench geometry).
//
// Structure per workgroup (HeadCfg: 8 waves, two per SIMD, 256 registers each; wave w owns rows
// 16w .. 16w+15 of the workgroup's 128 through the whole chain, activations in registers in the
// MFMA C layout):
//   fc1      X (gathered rows, per-wave LDS ring, LDS-DMA with 64-bit per-lane row addresses —
//            any buffer size) x W1: value 2 stages per k-step (32 output tiles), policy 2 k-steps
//            per stage (7 tiles each)
//   fc2      2 k-steps per stage; the next k-step's A operand (tanh, h1^T stores, LDS transpose)
//            is prepared between the two k-steps' MFMAs
//   fc3 + loss + dgrad fc3   one stage (fc3 slots 0-7, dgrad fc3 slots 8-14)
//   dgrad fc2  4 output tiles x 4 k-steps per stage; a stage's dtanh epilogue runs in the next
// Weights stream through an S-stage LDS ring (16 fragments per stage: 32 KiB split-bf16, 16 KiB
// bf16; wave w DMAs slots 2w, 2w+1 by buffer_load ... lds with the fragment codes of every step
// held in two VGPRs' lanes); counted vmcnt waits + a raw s_barrier per step (vector-memory
// operations retire in issue order).
#include <type_traits>

#include "kernels.h"
#include "mlp_core.h"

namespace {

constexpr float HD_LOG_2PI = 1.8378770664093453f;
constexpr int NPF = 8;                      // fixed loss-term columns of a partial row
constexpr int ROWS = 128;                   // rows per workgroup (both heads)
constexpr int NSLOT = 16;                   // fragments per ring stage
constexpr int SST = 36, TILE_F = 16 * SST;  // [16][SST] fp32 transpose tile (conflict-free)
constexpr int MAX_STEPS = 64;
// fc2: VALU instructions the scheduler may place after each MFMA (mma_mix).  Same-box A/B
// (profiles/r4/ab_fc2_vpm/): split-bf16 3 (4.118 ms) vs 2 (4.187) vs 6 (4.156); bf16 2 (2.239) vs 3
// (2.259) vs 6 (2.257) — the bf16 MFMA chain is a third as long, so fewer fillers per MFMA fit
constexpr int HD_VPM_S3 = 3, HD_VPM_BF16 = 2;
constexpr int HD_G4_BF16 = 4;   // bf16 dgrad fc2: fragments per LDS read group (groups of 2: no gain, r4)
// value fc1: fragments per LDS read group.  2: bf16 2.320 vs 2.345 ms, bf16x3 4.258 vs 4.264 ms per
// iteration against 4 (same box, profiles/r4/ab_value_fc1_g2/; split-bf16 groups of 4 put 16 reads in
// flight, past lgkmcnt's 15)
constexpr int HD_G1 = 2;

typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4h;

// Operand precision of the head kernels: how a 512-element fragment sits in global memory and in
// LDS, and how fp32 register values become MFMA operands / stored wgrad operands.
template <int DT> struct HT;
// split-bf16: 2 KiB fragments (lane l: 8 hi then 8 lo bf16), moved as two DMA instructions — the
// dense layout: instruction h moves lanes 32h .. 32h+31 and lands as [their hi][their lo], so lane
// l reads hi at (l / 32) KiB + 16 (l % 32), lo 512 bytes on (both conflict-free)
template <> struct HT<DT_S3> {
  using P = Prec<DT_S3>;
  using Frag = P::Frag;
  static constexpr int FB = 2048, NI = 2;   // fragment bytes, DMA instructions per fragment
  static constexpr int SPS = 2;             // opnd_store instructions per store4 / store8
  DEV static int lane_off(int lane) { return (lane >> 5) * 1024 + (lane & 31) * 16; }
  DEV static unsigned wsrc(int lane) { return (unsigned)((lane & 31) * 32 + (lane >> 5) * 16); }
  // observation row bytes of lane l's slot in DMA instruction 0 (k-groups 2h, 2h+1 per instruction)
  DEV static int xlane(int lane) { return 32 * ((lane >> 4) & 1) + 16 * (lane >> 5); }
  DEV static Frag lds(const char* p) {
    return Frag{*reinterpret_cast<const bf16x8*>(p), *reinterpret_cast<const bf16x8*>(p + 512)};
  }
  DEV static Frag from8(const f32x8& x) {
    const bf16x8 h = __builtin_convertvector(x, bf16x8);
    const bf16x8 l = __builtin_convertvector(ew_sub(x, __builtin_convertvector(h, f32x8)), bf16x8);
    return Frag{h, l};
  }
  DEV static f32x8 to8(const Frag& f) {
    return ew_add(__builtin_convertvector(f.h, f32x8), __builtin_convertvector(f.l, f32x8));
  }
  DEV static char* eptr(void* buf, size_t i) { return reinterpret_cast<char*>(P::hi_ptr(reinterpret_cast<P::T*>(buf), i)); }
  // 4 consecutive elements of an 8-group (hi at p, lo 16 bytes on)
  DEV static void store4(char* p, const f32x4& v) {
    const bf16x4v hv = __builtin_convertvector(v, bf16x4v);
    const bf16x4v lv = __builtin_convertvector(ew_sub(v, __builtin_convertvector(hv, f32x4)), bf16x4v);
    opnd_store(*reinterpret_cast<const u32x2*>(&hv), reinterpret_cast<u32x2*>(p));
    opnd_store(*reinterpret_cast<const u32x2*>(&lv), reinterpret_cast<u32x2*>(p + 16));
  }
  DEV static void store8(char* p, const f32x8& v) {
    const Frag f = from8(v);
    opnd_store(*reinterpret_cast<const u32x4h*>(&f.h), reinterpret_cast<u32x4h*>(p));
    opnd_store(*reinterpret_cast<const u32x4h*>(&f.l), reinterpret_cast<u32x4h*>(p + 16));
  }
};
// bf16: 1 KiB fragments, lane order, one DMA instruction
template <> struct HT<DT_BF16> {
  using P = Prec<DT_BF16>;
  using Frag = P::Frag;
  static constexpr int FB = 1024, NI = 1, SPS = 1;
  DEV static int lane_off(int lane) { return lane * 16; }
  DEV static unsigned wsrc(int lane) { return (unsigned)lane * 16u; }
  DEV static int xlane(int lane) { return 16 * (lane >> 4); }
  DEV static Frag lds(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }
  DEV static Frag from8(const f32x8& x) { return __builtin_convertvector(x, bf16x8); }
  DEV static f32x8 to8(const Frag& f) { return __builtin_convertvector(f, f32x8); }
  DEV static char* eptr(void* buf, size_t i) { return reinterpret_cast<char*>(reinterpret_cast<__bf16*>(buf) + i); }
  DEV static void store4(char* p, const f32x4& v) {
    const bf16x4v hv = __builtin_convertvector(v, bf16x4v);
    opnd_store(*reinterpret_cast<const u32x2*>(&hv), reinterpret_cast<u32x2*>(p));
  }
  DEV static void store8(char* p, const f32x8& v) {
    const bf16x8 h = __builtin_convertvector(v, bf16x8);
    opnd_store(*reinterpret_cast<const u32x4h*>(&h), reinterpret_cast<u32x4h*>(p));
  }
};

template <int HEAD> struct HeadCfg;
// NW waves of RB 16-row blocks each (NW * 16 * RB = 128 rows): 8 waves (two per SIMD, 256
// registers each) of 16 rows — the SIMD's two waves interleave one's VALU epilogues, loss and LDS
// transposes with the other's MFMAs (an in-order wave alone runs them back to back; measured on
// the value kernel: 181k -> 143k cycles per workgroup against 4 waves of 32 rows).
template <> struct HeadCfg<0> {   // policy: p_fc1 -> p_fc2 -> mu
  static constexpr int NW = 8, RB = 1;
  static constexpr int L1 = 0, L2 = 1, L3 = 2;
  static constexpr int N1 = 8, N1R = 7;     // fc1 tiles held / real (100 features + the bias column)
  static constexpr int K2 = 4;              // fc2 k-steps (fc1 output padded to 128)
  static constexpr int N3 = 2;              // fc3 output tiles (A <= 32)
  static constexpr int S3 = 2, SBF = 4;     // weight ring stages (split-bf16 / bf16: 64 KiB)
  static constexpr int NS4 = 2;             // dgrad fc2 stages (4 output tiles each)
  static constexpr int NEED = 1900;         // per-wave scratch floats: loss tile, partials, h2^T image
};
template <> struct HeadCfg<1> {   // value: v_fc1 -> v_fc2 -> v
  static constexpr int NW = 8, RB = 1;
  static constexpr int L1 = 3, L2 = 4, L3 = 5;
  static constexpr int N1 = 32, N1R = 32;   // 500 features + the bias column: 32 tiles
  static constexpr int K2 = 16;
  static constexpr int N3 = 1;
  static constexpr int S3 = 3, SBF = 6;     // (96 KiB; F8: 4 stages, 64 KiB)
  static constexpr int NS4 = 8;
  static constexpr int NEED = 744;          // loss tile, partials, dW_v partials
};

// F8 (fp8 mode, bf16 update): the forward GEMMs read the e4m3 weight image (the Adam step's shadow,
// csrc/adam_core.h f8_put; W / qscale[layer]).  A 1 KiB ring slot holds one tile's e4m3 fragments of
// two consecutive k-steps, so the stream and its LDS reads are half the bf16 bytes.
//  * value head: fc1 on v_mfma_f32_16x16x32_fp8_fp8 with e4m3-rounded observations x Q8_SX (2 stages
//    of 16 tiles per k-step pair);
//  * policy head: fc1 AND fc2 on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (twice the bf16
//    MFMA rate): a stage holds 4 k-steps of the 8 tiles (slots 2t, 2t + 1), the A operand is the
//    lane's 8 e4m3 bytes of each of the 4 k-steps (observations x Q8_SX, h1 x Q8_SH), the same k
//    order as the weight pieces, so the 128-term sum covers every k once (E8M0 scales 1; the epilogue
//    multiplies by qscale / the activation scale).  fc1: ks1 / 4 stages, fc2: ONE stage (K = 128).
template <int DT, int HEAD, bool F8 = false>
constexpr int head_stages() { return DT == DT_S3 ? HeadCfg<HEAD>::S3 : (F8 ? 4 : HeadCfg<HEAD>::SBF); }
// X ring slots (k-steps), a power of two.  An observation DMA must be OLDER than the weight batch
// whose counted wait precedes its read, so it is issued >= S stream steps ahead: X(k + XS) is
// issued when X(k) is read — policy 2 k-steps per step (XS / 2 >= S), value 2 steps per k-step
// (2 XS >= S; F8: 1 step per k-step, XS >= S).
template <int DT, int HEAD, bool F8 = false>
constexpr int head_xs() { return HEAD == 0 ? (DT == DT_S3 ? 4 : 8) : (DT == DT_S3 ? 2 : 4); }
template <int DT, int HEAD, bool F8 = false>
constexpr int x_lead_steps() {
  return HEAD == 0 ? head_xs<DT, HEAD, F8>() / 2 : (F8 ? 1 : 2) * head_xs<DT, HEAD, F8>();
}
template <int DT>
constexpr int stage_bytes() { return NSLOT * HT<DT>::FB; }
// per-wave scratch: the X ring (fc1), reused after fc1 for the loss tile and the partials
template <int DT, int HEAD, bool F8 = false>
constexpr int xr_floats() {
  constexpr int x = head_xs<DT, HEAD, F8>() * HeadCfg<HEAD>::RB * HT<DT>::FB / 4;
  return x > HeadCfg<HEAD>::NEED ? x : HeadCfg<HEAD>::NEED;
}
template <int DT, int HEAD, bool F8 = false>
constexpr int ws_floats() { return xr_floats<DT, HEAD, F8>() + HeadCfg<HEAD>::RB * TILE_F; }
// (+ Q8: the 2 x Q8_SUB sub-slot maxima of the head's gradient tensors the step's scales come from)
template <int DT, int HEAD, bool F8 = false>
constexpr size_t head_lds_bytes() {
  return (size_t)head_stages<DT, HEAD, F8>() * stage_bytes<DT>() +
         (size_t)HeadCfg<HEAD>::NW * ws_floats<DT, HEAD, F8>() * sizeof(float) + 2 * Q8_SUB * sizeof(float);
}
template <int HEAD>
constexpr int wrows() { return 16 * HeadCfg<HEAD>::RB; }
template <int DT, bool F8 = false>
constexpr bool head_lds_ok() {
  return head_lds_bytes<DT, 0>() <= 160 * 1024 && head_lds_bytes<DT, 1, F8>() <= 160 * 1024 &&
         // value: loss tile + partials + its 128 dW_v partials; policy: + the [64][20] h2^T image
         wrows<1>() * SST + NPF + 32 + 128 <= xr_floats<DT, 1, F8>() &&
         ((wrows<0>() * SST + NPF + 32 + 3) & ~3) + 64 * 20 <= xr_floats<DT, 0>() &&
         // the dW_mu tiles of 4 waves go through the policy ring
         4 * 32 * 128 * 4 <= head_stages<DT, 0>() * stage_bytes<DT>() &&
         // the observation DMAs lead the weight waits
         x_lead_steps<DT, 0>() >= head_stages<DT, 0>() && x_lead_steps<DT, 1, F8>() >= head_stages<DT, 1, F8>();
}
static_assert(head_lds_ok<DT_S3>() && head_lds_ok<DT_BF16>() && head_lds_ok<DT_BF16, true>(),
              "head kernel LDS carving / observation lead");
// the fp8 policy: LDS, the dW_mu reduction through its ring, and an X ring two 4-k-step stages deep
// (its waits retire every refill, so the observations need lead 2 >= 2, not >= S)
static_assert(head_lds_bytes<DT_BF16, 0, true>() <= 160 * 1024 &&
                  4 * 32 * 128 * 4 <= head_stages<DT_BF16, 0, true>() * stage_bytes<DT_BF16>() &&
                  head_xs<DT_BF16, 0, true>() / 4 >= 2 && head_stages<DT_BF16, 0, true>() >= 3,
              "fp8 policy head LDS carving / observation lead");
static_assert(HeadCfg<0>::NW * wrows<0>() == ROWS && HeadCfg<1>::NW * wrows<1>() == ROWS, "128 rows per workgroup");
// loss scratch (after fc1, in the X ring): dL/dmu | dL/dv [rows][SST], then the wave's partials
static_assert(wrows<0>() * 32 <= HeadCfg<0>::RB * TILE_F, "mu tile fits the transpose tiles");
static_assert(HeadCfg<0>::NW == 8 && HeadCfg<0>::RB == 1, "the fused dW_mu reduction assumes 8 waves of 16 rows");

template <int HEAD, bool F8 = false>
DEV int fc1_stages(int ks1) { return HEAD == 0 ? (F8 ? ks1 >> 2 : (ks1 + 1) >> 1) : (F8 ? ks1 : 2 * ks1); }
// fc2 stages: 2 k-steps each; the fp8 policy's e4m3 fc2 (K = 128) on the x128 MFMA in ONE.  (The value
// head's fc2 on e4m3 — 4 stages of 4 k-steps — was measured slower: 2.095 vs 1.983 ms per fp8
// iteration, the value kernel spilling 27 VGPRs; profiles/r4/fp8_heads.md)
template <int HEAD, bool F8 = false>
constexpr int fc2_stages() { return (F8 && HEAD == 0) ? HeadCfg<HEAD>::K2 / 4 : HeadCfg<HEAD>::K2 / 2; }
template <int HEAD, bool F8 = false>
constexpr bool f8_fc2() { return F8 && HEAD == 0; }

DEV int rot_ks(int ks, int rot, int ks1) {
  const int k = ks + rot;
  return k >= ks1 ? k - ks1 : k;
}

// Ring slot q of stream step st: element offset of a weight fragment, or -1 (a slot no MFMA
// reads; its DMA re-loads slot 0's fragment so every wave issues GL DMAs per step).  FWD (the
// value forward): the stream ends with the fc3 stage.
template <int HEAD, bool FWD, bool F8>
DEV int step_src(const MlpArgs& a, int st, int q, int rot, int ks1) {
  using C = HeadCfg<HEAD>;
  const int ns1 = fc1_stages<HEAD, F8>(ks1), ns2 = fc2_stages<HEAD, F8>();
  const int s_fc3 = ns1 + ns2, s_dg2 = s_fc3 + 1, s_end = FWD ? s_dg2 : s_dg2 + C::NS4;
  if (st >= s_end) st = s_end - 1;
  if (st < ns1) {
    int ks, t;
    if constexpr (HEAD == 0 && F8) {
      // slots 2t, 2t + 1: tile t's k-step pairs 4 st, 4 st + 2 (rot a multiple of 4, ks1 too)
      ks = 4 * st + 2 * (q & 1);
      t = q >> 1;
      if (t >= C::N1R) return -1;
    } else if constexpr (HEAD == 0) {
      ks = 2 * st + (q >> 3);
      t = q & 7;
      if (t >= C::N1R || ks >= ks1) return -1;
    } else {
      // (F8: the slot's first k-step of a pair 2j, 2j + 1 — contiguous in the e4m3 image; rot and
      // ks1 even keep the pair contiguous after the rotation)
      ks = F8 ? (st & ~1) : st >> 1;
      t = 16 * (st & 1) + q;
    }
    return a.off_w[C::L1] + (int)fm_frag(t, rot_ks(ks, rot, ks1), a.d_in[C::L1], 0);
  }
  if (f8_fc2<HEAD, F8>() && st < s_fc3) {   // the e4m3 fc2 stage(s): tile q >> 1, k-steps 4 (st - ns1) + 2 (q & 1) + {0, 1}
    const int t = q >> 1;
    if (t == 7) return -1;
    return a.off_w[C::L2] + (int)fm_frag(t, 4 * (st - ns1) + 2 * (q & 1), a.d_in[C::L2], 0);
  }
  if (st < s_fc3) {
    const int i = 2 * (st - ns1) + (q >> 3), t = q & 7;
    if (t == 7) return -1;   // output tile 7 (features 112-127) is padding
    return a.off_w[C::L2] + (int)fm_frag(t, i, a.d_in[C::L2], 0);
  }
  if (st == s_fc3) {
    if (q < 8) {
      if (q >= 4 * C::N3) return -1;
      return a.off_w[C::L3] + (int)fm_frag(q >> 2, q & 3, a.d_in[C::L3], 0);
    }
    if (q == 15) return -1;
    return a.off_wt[C::L3] + (int)fm_frag(q - 8, 0, a.d_out[C::L3], 0);
  }
  const int t = 4 * (st - s_dg2) + (q >> 2), ks = q & 3;
  if (t >= C::N1R) return -1;
  return a.off_wt[C::L2] + (int)fm_frag(t, ks, a.d_out[C::L2], 0);
}

// the head kernels' fragment product
template <int DT>
DEV f32x4 hmma(f32x4 c, const typename HT<DT>::Frag& a, const typename HT<DT>::Frag& b) {
  return HT<DT>::P::mma(c, a, b);
}

// C-layout tiles of features c0..c0+15 (v0) and c0+16..c0+31 (v1) -> [16][SST] fp32
DEV void tp_put(float* tp, const f32x4& v0, const f32x4& v1, int lane) {
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    tp[(4 * lg + i) * SST + lr] = v0[i];
    tp[(4 * lg + i) * SST + 16 + lr] = v1[i];
  }
}

// A operand (row lane & 15, k = 8 (lane >> 4) .. +7) of a [16][SST] tile; reads + wait in one asm
// statement (a plain LDS load would wait vmcnt(0) for the ring's LDS-DMA)
DEV f32x8 tp_get8(const float* tp, int lane) {
  const float* r = tp + (lane & 15) * SST + 8 * (lane >> 4);
  const uint32_t addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)r;
  float4 x0, x1;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(x0), "=&v"(x1)
               : "v"(addr)
               : "memory");
  return f32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
}
template <int DT>
DEV typename HT<DT>::Frag tp_getA(const float* tp, int lane) {
  return HT<DT>::from8(tp_get8(tp, lane));
}

DEV f32x4 bias_col(const f32x4& v, int c, int nb) {
  const float o = c == nb ? 1.f : 0.f;
  return c < nb ? v : f32x4{o, o, o, o};
}

// 4 consecutive m of feature 16 t + (lane & 15) -> the FM wgrad operand from the lane's base
template <int DT>
DEV void store_Tt(char* lane_base, int t, size_t tsb, const f32x4& v) {
  HT<DT>::store4(lane_base + (size_t)t * tsb, v);
}

// 8 consecutive m (rows 8h..8h+7) of column col of a [rows][ld] fp32 tile -> one FM group
template <int DT>
DEV void store_T8(void* outT, const float* tile, int ld, int col, int h, int feat, int m, int ldT) {
  f32x8 x;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = tile[(8 * h + j) * ld + col];
  HT<DT>::store8(HT<DT>::eptr(outT, fm_index(feat, m, ldT)), x);
}

// s_waitcnt vmcnt(BASE + extra) with a compile-time immediate (mlp_stream.hip wait_vm):
// undercounting `extra` is safe (the wait is longer), overcounting is not
template <int BASE, int E = 0>
DEV void wait_vm(int extra) {
  if constexpr (BASE + E >= 63) {
    WAIT_VMCNT(63);
  } else {
    if (extra <= E) WAIT_VMCNT(BASE + E);
    else wait_vm<BASE, E + 1>(extra);
  }
}

template <int B, int E, typename F>
DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Fragments q in [Q0, Q1) of a stage with bit q of MASK set, read in groups of G: group g + 1's
// LDS reads are in flight while group g's MFMAs run.  f(integral_constant<q>, fragment).
struct NoHook {
  DEV void operator()() const {}
};
// (pre(): called once the first group's LDS reads are issued — the stage's ring refill goes there,
// so its issue cost overlaps their latency instead of delaying them)
template <int DT, unsigned MASK, int Q0, int Q1, int G, typename F, typename PRE = NoHook>
DEV void for_slots(const char* stg, int lane, F&& f, PRE&& pre = PRE{}) {
  using H = HT<DT>;
  constexpr int NG = (Q1 - Q0 + G - 1) / G;
  typename H::Frag b[2][G];
  const char* base = stg + H::lane_off(lane);
  auto rd = [&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    static_for<0, G>([&](auto ic) __attribute__((always_inline)) {
      constexpr int q = Q0 + g * G + decltype(ic)::value;
      if constexpr (q < Q1 && ((MASK >> q) & 1u))
        b[g & 1][decltype(ic)::value] = H::lds(base + q * H::FB);
    });
  };
  rd(std::integral_constant<int, 0>{});
  pre();
  static_for<0, NG>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    if constexpr (g + 1 < NG) rd(std::integral_constant<int, g + 1>{});
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, G>([&](auto ic) __attribute__((always_inline)) {
      constexpr int q = Q0 + g * G + decltype(ic)::value;
      if constexpr (q < Q1 && ((MASK >> q) & 1u)) f(std::integral_constant<int, q>{}, b[g & 1][decltype(ic)::value]);
    });
  });
}

// One scheduling region of a stage's fragments q in [Q0, Q1) with bit q of MASK set: all their
// LDS reads first, then the MFMAs f(q, fragment) INTERLEAVED with other independent work v()
// (VALU epilogues / operand preparation of the next k-step, their stores and LDS writes): the
// sched_group_barrier pipeline asks the scheduler for 1 MFMA then up to VPM VALU instructions,
// NM times, so the VALU issues in the MFMAs' shadow instead of after them (at one wave per SIMD
// an in-order wave otherwise runs the MFMA block and the VALU block back to back).  v() must not
// contain inline asm (a scheduling boundary).
template <int DT, unsigned MASK, int Q0, int Q1, int NM, int VPM, typename F, typename V, typename PRE = NoHook>
DEV void mma_mix(const char* stg, int lane, F&& f, V&& v, PRE&& pre = PRE{}) {
  using H = HT<DT>;
  constexpr int N = Q1 - Q0;
  typename H::Frag b[N];
  const char* base = stg + H::lane_off(lane);
  static_for<0, N>([&](auto ic) __attribute__((always_inline)) {
    constexpr int q = Q0 + decltype(ic)::value;
    if constexpr ((MASK >> q) & 1u) b[decltype(ic)::value] = H::lds(base + q * H::FB);
  });
  pre();
  __builtin_amdgcn_sched_barrier(0);
  static_for<0, N>([&](auto ic) __attribute__((always_inline)) {
    constexpr int q = Q0 + decltype(ic)::value;
    if constexpr ((MASK >> q) & 1u) f(std::integral_constant<int, q>{}, b[decltype(ic)::value]);
  });
  v();
  static_for<0, NM>([&](auto) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // 1 MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);   // then VALU
  });
  __builtin_amdgcn_sched_barrier(0);
}

template <int G>
DEV float xsum(float x) {   // sum over the lanes that differ only in the bits of G (xor tree)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1)
    if (G & o) x += __shfl_xor(x, o, 64);
  return x;
}

// phase timeline (diagnostics, scripts/head_timeline.py): lane 0 of each wave of every
// tstamp_every-th workgroup records the shader clock at the phase boundaries (a vector store the
// wait bookkeeping does not count: an undercount, safe)
#define HD_STAMP(i)                                                                               \
  do {                                                                                            \
    if (a.tstamp != nullptr && (blockIdx.x % a.tstamp_every) == 0 && lane == 0)                   \
      a.tstamp[((size_t)(blockIdx.x / a.tstamp_every) * NW + wave) * 16 + (i)] =                  \
          __builtin_amdgcn_s_memtime();                                                           \
  } while (0)

// FWD (value head only): the forward alone, V(x) of rows [row0, row0 + M) into v_out — the GAE
// input pass (train.py:87,109-112) at the update kernel's 128 rows per weight stream instead of
// mlp.hip's 32-row value kernel
// Q8 (fp8 mode, bf16 update): the wgrad operands are stored as scaled e4m3 bytes (csrc/common.h Q8)
template <int DT, int HEAD, bool FWD = false, bool F8 = false, bool Q8 = false>
__global__ __launch_bounds__(HeadCfg<HEAD>::NW * 64, 1) void mlp_head_kernel(MlpArgs a) {
  static_assert(!FWD || HEAD == 1, "forward mode is the value head's");
  static_assert(!F8 || DT == DT_BF16, "the e4m3 forward GEMMs are the bf16 update's (fp8 mode)");
  static_assert(!Q8 || (DT == DT_BF16 && !FWD), "e4m3 wgrad operands: the fp8 mode's (bf16) update");
  using C = HeadCfg<HEAD>;
  using H = HT<DT>;
  using P = typename H::P;
  using T = typename P::T;
  using Frag = typename H::Frag;
  constexpr int FB = H::FB, SB = stage_bytes<DT>();
  constexpr int S = head_stages<DT, HEAD, F8>(), XS = head_xs<DT, HEAD, F8>();
  constexpr int NW = C::NW, RB = C::RB, WROWS = 16 * RB;
  constexpr int SPW = NSLOT / NW, GL = H::NI * SPW;   // ring slots / DMA instructions per wave per stage
  constexpr int XDMA = H::NI * RB;                    // DMA instructions of one wave's X fragments of a k-step
  constexpr int TPR = 64 / WROWS;                     // loss lanes per row
  constexpr int WS_F = ws_floats<DT, HEAD, F8>();
  constexpr int MPP = DT == DT_S3 ? 3 : 1;            // MFMAs per fragment product
  constexpr int VPM = DT == DT_S3 ? HD_VPM_S3 : HD_VPM_BF16;
  extern __shared__ __attribute__((aligned(16))) char smem[];   // the kernel's ONLY LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * ROWS;
  const int A = a.A;
  const int ks1 = a.d_in[0] >> 5;
  const int ns1 = fc1_stages<HEAD, F8>(ks1);
  char* ring = smem;
  float* scr = reinterpret_cast<float*>(smem + (size_t)S * SB) + wave * WS_F;
  char* xring = reinterpret_cast<char*>(scr);
  float* tpb = scr + xr_floats<DT, HEAD, F8>();   // RB transpose tiles [16][SST]
  float* dml = scr;                        // (after fc1) dL/dmu [32][SST] | dL/dv column 32
  float* wpart = scr + WROWS * SST;        // (after fc1) [8 loss terms | 32 dlog_std]
  float* mus = tpb;                        // (loss) mu [32][32] | v [32]

  auto src_of = [&](int r) __attribute__((always_inline)) {
    const int rr = (m0 + r < a.M) ? m0 + r : m0;   // rows past M re-read row m0 (zero gradient)
    return a.idx ? a.idx[rr] : a.row0 + rr;
  };
  const int mw = m0 + WROWS * wave;
  // the loss's row and sub-lane: policy 2 lanes per row (32 rows), value lanes 0-15 one row each
  const int lrow = HEAD == 0 ? lane / TPR : lane % WROWS;
  const int lsub = HEAD == 0 ? lane % TPR : lane / WROWS;
  const bool lvalid = mw + lrow < a.M;
  const int lsrc = src_of(WROWS * wave + lrow);

  // loss inputs of this lane's row, loaded before any DMA: older than every ring batch, they never
  // hold up a counted wait (policy: 4 x 16 registers, held through fc1 / fc2)
  const bool ref_loss = a.loss_kind != 0;
  constexpr int JM = HEAD == 0 ? 32 / TPR : 1;   // action dims per lane (policy: j = lsub + TPR q, A <= 32)
  float actv[JM], lsv[JM], lsov[JM], mupv[JM];
  float l_adv = 0.f, l_ret = 0.f, l_lpo = 0.f, l_vold = 0.f, l_vprev = 0.f;
  if constexpr (HEAD == 0) {
#pragma unroll
    for (int q = 0; q < JM; ++q) {
      const int j = lsub + TPR * q;
      actv[q] = j < A ? a.actions[(size_t)lsrc * A + j] : 0.f;
      lsv[q] = j < A ? a.log_std[j] : 0.f;
      lsov[q] = (ref_loss && j < A) ? a.log_std_old[j] : 0.f;
      mupv[q] = (ref_loss && j < A) ? a.mu_prev[(size_t)lsrc * A + j] : 0.f;
    }
    l_adv = a.adv[lsrc];
    l_lpo = !ref_loss ? a.logp_old[lsrc] : 0.f;
  } else if constexpr (!FWD) {
    l_ret = a.ret[lsrc];
    l_vold = !ref_loss ? a.v_old[lsrc] : 0.f;
    l_vprev = ref_loss ? a.v_prev[lsrc] : 0.f;
  }

  // ---- DMA sources ----
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), (short)0, 0x7fffffff, 0x00020000);
  const unsigned vw = H::wsrc(lane);
  // observation rows: 64-bit per-lane addresses (global_load_lds), so a buffer of any size works;
  // instruction h of a row block moves 64 contiguous bytes of each row (split-bf16: k-groups 2h,
  // 2h+1; bf16: the whole k-step)
  const char* xsrc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
    xsrc[rb] = reinterpret_cast<const char*>(a.x_buf) +
               (size_t)src_of(WROWS * wave + 16 * rb + lr) * (size_t)a.d_in[0] * sizeof(T) + H::xlane(lane);
  // (F8: an even rotation keeps each fc1 k-step pair contiguous; the launcher checks ks1 even — the
  // policy's: a multiple of 4, ks1 % 4 == 0)
  const int rot = (F8 && HEAD == 0) ? 4 * (int)(blockIdx.x % (unsigned)(ks1 >> 2))
                  : F8              ? 2 * (int)(blockIdx.x % (unsigned)(ks1 >> 1))
                                    : (int)(blockIdx.x % (unsigned)ks1);
  auto code16 = [&](int st, int q) __attribute__((always_inline)) {
    int c = step_src<HEAD, FWD, F8>(a, st, q, rot, ks1);
    if (c < 0) c = step_src<HEAD, FWD, F8>(a, st, 0, rot, ks1);
    if (c < 0) c = a.off_w[C::L1];
    return (uint32_t)(c >> 9);
  };
  const uint32_t cw0 = code16(lane, SPW * wave) | (code16(lane, SPW * wave + 1) << 16);
  const uint32_t cw1 = SPW > 2 ? code16(lane, SPW * wave + 2) | (code16(lane, SPW * wave + 3) << 16) : 0u;

  __amdgpu_buffer_rsrc_t rw8 = rw;
  if constexpr (F8) rw8 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W8), (short)0, 0x7fffffff, 0x00020000);
  auto issue = [&](int st, int stage) __attribute__((always_inline)) {
    const int l = min(st, MAX_STEPS - 1);
    const uint32_t w01 = __builtin_amdgcn_readlane(cw0, l);
    const uint32_t w23 = SPW > 2 ? __builtin_amdgcn_readlane(cw1, l) : 0u;
    __attribute__((address_space(3))) char* stg =
        (__attribute__((address_space(3))) char*)(ring + stage * SB) + SPW * wave * FB;
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const uint32_t code = ((u < 2 ? w01 : w23) >> (16 * (u & 1))) & 0xffffu;
      // the e4m3 stages (fc1; the policy's fc2): two e4m3 fragments (512 B each) of a tile per slot
      if (F8 && st < ns1 + (f8_fc2<HEAD, F8>() ? fc2_stages<HEAD, F8>() : 0)) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw8, stg + u * FB, 16, vw, code * 512u, 0, 0);
      } else {
#pragma unroll
        for (int h = 0; h < H::NI; ++h)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, stg + u * FB + 1024 * h, 16, vw, code * (unsigned)FB + 1024u * h,
                                                   0, 0);
      }
    }
  };
  // this wave's RB observation fragments of fc1 k-step ks into X ring slot ks % XS
  auto issue_x = [&](int ks) __attribute__((always_inline)) {
    const size_t xo = (size_t)rot_ks(min(ks, ks1 - 1), rot, ks1) * (32u * sizeof(T));
    char* d = xring + (ks & (XS - 1)) * (RB * FB);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int h = 0; h < H::NI; ++h) glds16(xsrc[rb] + xo + 64 * h, d + rb * FB + 1024 * h);
  };
  auto xaddr = [&](int ks, int rb) __attribute__((always_inline)) -> uint32_t {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(
               xring + (ks & (XS - 1)) * (RB * FB) + rb * FB) + H::lane_off(lane);
  };
  // the observation fragments of two k-steps (row block 0) behind ONE wait (the policy's fc1 stage)
  auto read_x2 = [&](int ka, int kb, Frag& fa, Frag& fb) __attribute__((always_inline)) {
    const uint32_t aa = xaddr(ka, 0), ab = xaddr(kb, 0);
    if constexpr (DT == DT_S3) {
      bf16x8 h0, l0, h1, l1;
      asm volatile(
          "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:512\n\tds_read_b128 %2, %5\n\t"
          "ds_read_b128 %3, %5 offset:512\n\ts_waitcnt lgkmcnt(0)"
          : "=&v"(h0), "=&v"(l0), "=&v"(h1), "=&v"(l1)
          : "v"(aa), "v"(ab)
          : "memory");
      fa = Frag{h0, l0};
      fb = Frag{h1, l1};
    } else {
      bf16x8 h0, h1;
      asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(h0), "=&v"(h1)
                   : "v"(aa), "v"(ab)
                   : "memory");
      fa = h0;
      fb = h1;
    }
  };
  auto read_x = [&](int ks, int rb) __attribute__((always_inline)) {
    const uint32_t addr = xaddr(ks, rb);
    if constexpr (DT == DT_S3) {
      bf16x8 h, l;
      asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:512\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(h), "=&v"(l)
                   : "v"(addr)
                   : "memory");
      return Frag{h, l};
    } else {
      bf16x8 h;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(h) : "v"(addr) : "memory");
      return h;
    }
  };

  // Ring bookkeeping.  Every step: wait for its stage (this wave's DMAs by count, every wave's by
  // the barrier, which also retires every wave's reads of the previous step's stage), then at
  // once refill that previous stage with step cur + S - 1, then compute.  Vector-memory
  // operations retire in issue order (loads, stores, LDS-DMA together), so the wait for step c's
  // batch — issued at the start of step c - S + 1 — may leave outstanding everything younger:
  // the S - 2 later refills and every store / X load issued since (`younger` = those of the
  // previous step; undercounting is safe, overcounting is not).
  int cst = 0, cur = 0;
  constexpr int NH = S - 1;
  int hist[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) hist[i] = 0;
  auto flush = NoHook{};   // (A/B in round 4: the refill issued after the first fragment reads: no gain)
  // LEAD > 0: the wait also retires the next LEAD stages' batches (the fp8 policy's fc1: every
  // refill, so an observation DMA issued two stages back is certified with them — its X ring leads
  // by 2 stages of 4 k-steps; a batch then has LEAD fewer stages of compute to land in)
  auto wait_step_l = [&](int younger, auto leadc) __attribute__((always_inline)) -> const char* {
    constexpr int LEAD = decltype(leadc)::value;
    static_assert(S - 2 - LEAD >= 0, "ring too shallow for the lead");
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = NH - 1; i > 0; --i) hist[i] = hist[i - 1];
    hist[0] = younger;
    // (the younger ops that may stay outstanding: those issued after the oldest refill allowed to)
    int extra = 0;
#pragma unroll
    for (int i = 0; i < NH - LEAD; ++i) extra += hist[i];
    wait_vm<GL * (S - 2 - LEAD)>(extra);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* stg = ring + cst * SB;
    issue(cur + S - 1, cst == 0 ? S - 1 : cst - 1);
    cst = cst + 1 == S ? 0 : cst + 1;
    ++cur;
    return stg;
  };
  auto wait_step = [&](int younger) __attribute__((always_inline)) -> const char* {
    return wait_step_l(younger, std::integral_constant<int, 0>{});
  };

  HD_STAMP(0);
  // Q8: wave 0 DMAs the previous step's sub-slot maxima of the head's two gradient tensors into
  // LDS — the oldest vector-memory ops of the wave (never behind a counted wait), read after many
  // barriers at dgrad fc3
  const uint32_t* q8l = reinterpret_cast<const uint32_t*>(smem + head_lds_bytes<DT, HEAD, F8>() - 2 * Q8_SUB * 4);
  if constexpr (Q8) {
    if (wave == 0) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(a.q8_rd + ((2 * HEAD + k) * Q8_SUB + lane) * Q8_LINE),
            (__attribute__((address_space(3))) void*)(q8l + k * Q8_SUB), 4, 0, 0);
    }
  }
  // ---- prime: the first X k-steps, then ring stages 0 .. S-2 ----
#pragma unroll
  for (int k = 0; k < XS; ++k) issue_x(k);
#pragma unroll
  for (int st = 0; st < S - 1; ++st) issue(st, st);

  // bytes of one 16-feature row block of an FM operand (Q8: one byte per element)
  const size_t tsb = (size_t)a.ldT * 16 * (Q8 ? 1 : sizeof(T));
  auto lane_base = [&](void* buf, int rb) __attribute__((always_inline)) {
    const size_t i = fm_index(lr, mw + 16 * rb + 4 * lg, a.ldT);
    return Q8 ? reinterpret_cast<char*>(buf) + i : H::eptr(buf, i);
  };
  // a wgrad operand group of 4 consecutive batch rows of one feature (Q8: x s, saturated for the
  // gradients; the activations' fixed scales keep them in range)
  auto opnd4 = [&](char* p, const f32x4& v, float s) __attribute__((always_inline)) {
    if constexpr (Q8) opnd_store(q8_pack4(v, s), reinterpret_cast<uint32_t*>(p));
    else HT<DT>::store4(p, v);
  };
  auto opnd4u = [&](char* p, const f32x4& v, float s) __attribute__((always_inline)) {
    if constexpr (Q8) opnd_store(q8_pack4u(v, s), reinterpret_cast<uint32_t*>(p));
    else HT<DT>::store4(p, v);
  };
  void* const h1T = HEAD == 0 ? a.h1pT : a.h1vT;
  void* const g2T = HEAD == 0 ? a.g2pT : a.g2vT;
  void* const g1T = HEAD == 0 ? a.g1pT : a.g1vT;

  // ---------------- fc1 ----------------
  f32x4 acc1[RB][C::N1];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < C::N1; ++t) acc1[rb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool want_xT = HEAD == 0 && !a.xT_ready;
  const char* stg;
  // (the policy kernel writes the x^T wgrad operand when the rollout did not: the wave's 16 x 32
  // block of k-step ks of row block rb, transposed through its tile)
  auto put_xT = [&](const Frag& x, int ks, int rb) __attribute__((always_inline)) {
    float* tp = tpb + rb * TILE_F;
    const f32x8 v = H::to8(x);
    float4* w = reinterpret_cast<float4*>(tp + lr * SST + 8 * lg);
    w[0] = float4{v[0], v[1], v[2], v[3]};
    w[1] = float4{v[4], v[5], v[6], v[7]};
    if constexpr (Q8) {
      const int col = lane >> 1, hh = lane & 1;
      f32x4 x0, x1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x0[j] = tp[(8 * hh + j) * SST + col];
        x1[j] = tp[(8 * hh + 4 + j) * SST + col];
      }
      const uint32_t w0 = q8_pack4u(x0, Q8_SX), w1 = q8_pack4u(x1, Q8_SX);
      opnd_store(u32x2{w0, w1}, reinterpret_cast<u32x2*>(reinterpret_cast<char*>(a.xT) +
                                                        fm_index(32 * rot_ks(ks, rot, ks1) + col,
                                                                 mw + 16 * rb + 8 * hh, a.ldT)));
    } else {
      store_T8<DT>(a.xT, tp, SST, lane >> 1, lane & 1, 32 * rot_ks(ks, rot, ks1) + (lane >> 1),
                   mw + 16 * rb + 8 * (lane & 1), a.ldT);
    }
  };
  // 8 fp32 -> 8 OCP e4m3 bytes (round to nearest even, saturating: v_cvt_pk_fp8_f32)
  auto f8x8 = [&](const f32x8& v) __attribute__((always_inline)) -> long {
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
    return (long)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
  };
  // observations x Q8_SX (|x| <= 5 after the clamp: <= 320, below e4m3's 448) so the small normalised
  // features stay out of e4m3's subnormal range; fc1's epilogue divides it out with the weight scale
  auto to_f8 = [&](const Frag& x) __attribute__((always_inline)) -> long { return f8x8(H::to8(x) * Q8_SX); };
  // the x128 B operand of tile t from a stage of the fp8 policy (slots 2t, 2t + 1: k-steps 4j .. 4j+3)
  auto b128 = [&](const char* sb, int t) __attribute__((always_inline)) -> i32x8 {
    const char* p = sb + 2 * t * FB + lane * 8;
    const long x0 = *reinterpret_cast<const long*>(p), x1 = *reinterpret_cast<const long*>(p + 512);
    const long x2 = *reinterpret_cast<const long*>(p + FB), x3 = *reinterpret_cast<const long*>(p + FB + 512);
    return i32x8{(int)x0, (int)(x0 >> 32), (int)x1, (int)(x1 >> 32), (int)x2, (int)(x2 >> 32), (int)x3, (int)(x3 >> 32)};
  };
  auto a128 = [&](long q0, long q1, long q2, long q3) __attribute__((always_inline)) -> i32x8 {
    return i32x8{(int)q0, (int)(q0 >> 32), (int)q1, (int)(q1 >> 32), (int)q2, (int)(q2 >> 32), (int)q3, (int)(q3 >> 32)};
  };
  if constexpr (F8 && HEAD == 0) {
    // e4m3 fc1 of the policy on the x128 MFMA: stage st = k-steps 4 st .. 4 st + 3 of the 7 tiles.
    // Every wait retires all refills (LEAD = S - 2): the observation k-steps a stage reads were
    // issued two stages back, before the previous stage's refill, so that wait certifies them.
    for (int st = 0; st < ns1; ++st) {
      stg = wait_step_l(st > 0 ? 4 * XDMA : 0, std::integral_constant<int, S - 2>{});
      Frag xf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xf[j] = read_x(4 * st + j, 0);
      const i32x8 xq = a128(to_f8(xf[0]), to_f8(xf[1]), to_f8(xf[2]), to_f8(xf[3]));
#pragma unroll
      for (int t = 0; t < C::N1R; ++t)
        acc1[0][t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(xq, b128(stg, t), acc1[0][t], 0, 0, 0, 127, 0, 127);
      if (want_xT) {
#pragma unroll
        for (int j = 0; j < 4; ++j) put_xT(xf[j], 4 * st + j, 0);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) issue_x(4 * st + j + XS);   // into the slots just read
      if (st == 0) HD_STAMP(8);
      if (st == 1) HD_STAMP(9);
    }
    const float s1 = a.qscale[C::L1] * (1.0f / Q8_SX);   // the e4m3 image holds W1 / qscale
#pragma unroll
    for (int t = 0; t < C::N1; ++t) acc1[0][t] *= s1;
  } else if constexpr (F8) {
    // e4m3 fc1: per k-step pair 2 stages (tiles 0-15, 16-31), each slot one tile's two fragments;
    // the observation fragments (bf16 in the X ring) rounded to e4m3 in registers
    long xq0 = 0, xq1 = 0;
    for (int j = 0; j < (ks1 >> 1); ++j) {
      static_for<0, 2>([&](auto sc) __attribute__((always_inline)) {
        constexpr int sub = decltype(sc)::value;
        stg = wait_step(sub == 1 ? 2 * XDMA : 0);
        flush();
        if constexpr (sub == 0) {
          xq0 = to_f8(read_x(2 * j, 0));
          xq1 = to_f8(read_x(2 * j + 1, 0));
        }
        const char* base = stg + 8 * lane;
        static_for<0, 16>([&](auto qc) __attribute__((always_inline)) {
          constexpr int q = decltype(qc)::value;
          const long w0 = *reinterpret_cast<const long*>(base + q * FB);
          const long w1 = *reinterpret_cast<const long*>(base + q * FB + 512);
          acc1[0][16 * sub + q] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(xq0, w0, acc1[0][16 * sub + q], 0, 0, 0);
          acc1[0][16 * sub + q] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(xq1, w1, acc1[0][16 * sub + q], 0, 0, 0);
        });
        if constexpr (sub == 0) {   // into the slots X[2j], X[2j + 1] just left
          issue_x(2 * j + XS);
          issue_x(2 * j + 1 + XS);
        }
      });
    }
    const float s1 = a.qscale[C::L1] * (1.0f / Q8_SX);   // the e4m3 image holds W1 / qscale
#pragma unroll
    for (int t = 0; t < C::N1; ++t) acc1[0][t] *= s1;
  } else if constexpr (HEAD == 1) {
    Frag xa[RB];
    for (int ks = 0; ks < ks1; ++ks) {
      static_for<0, 2>([&](auto sc) __attribute__((always_inline)) {
        constexpr int sub = decltype(sc)::value;
        stg = wait_step(sub == 1 ? XDMA : 0);
        if constexpr (sub == 0) {
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) xa[rb] = read_x(ks, rb);
        }
        for_slots<DT, 0xffffu, 0, 16, HD_G1>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
            constexpr int t = 16 * sub + decltype(qc)::value;
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) acc1[rb][t] = hmma<DT>(acc1[rb][t], xa[rb], b);
          }, flush);
        if constexpr (sub == 0) issue_x(ks + XS);   // into the slot X[ks] just left
      });
      if (ks == 1) HD_STAMP(8);
      if (ks == 5) HD_STAMP(9);
    }
  } else {
    for (int st = 0; st < ns1; ++st) {
      stg = wait_step(st > 0 ? 2 * XDMA : 0);
      const int ka = 2 * st, kb = 2 * st + 1;
      const bool two = kb < ks1;
      Frag xa[RB], xb[RB];
      read_x2(ka, kb, xa[0], xb[0]);   // (RB == 1: static_assert above)
      // an odd ks1's last stage: its second k-step is past the end — a zero operand instead of a
      // branch around those MFMAs (a branch splits the stage's read / MFMA schedule in two)
      if (!two) xb[0] = Frag{};
      // (split-bf16: read groups of 2 fragments = 4 ds_read_b128, so two groups in flight stay within
      // lgkmcnt's 15 and the compiler can wait for one group instead of lgkmcnt(0))
      for_slots<DT, 0x7f7fu, 0, 16, DT == DT_S3 ? 2 : 4>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        if constexpr (q < 8) {
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) acc1[rb][q] = hmma<DT>(acc1[rb][q], xa[rb], b);
        } else {
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) acc1[rb][q - 8] = hmma<DT>(acc1[rb][q - 8], xb[rb], b);
        }
      }, flush);
      if (want_xT) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          put_xT(xa[rb], ka, rb);
          if (two) put_xT(xb[rb], kb, rb);
        }
      }
      issue_x(ka + XS);   // into the slots X[ka], X[kb] just left
      issue_x(kb + XS);
      if (st == 0) HD_STAMP(8);
      if (st == 3) HD_STAMP(9);
    }
  }
  HD_STAMP(1);
  // ---------------- fc2: h1 = tanh(fc1), one k-step's A operand prepared at a time ----------------
  const int n1 = a.n_out[C::L1], n2 = a.n_out[C::L2];
  char* bh1[RB];
  char* bg2[RB];
  char* bg1[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    bh1[rb] = lane_base(h1T, rb);
    bg2[rb] = lane_base(g2T, rb);
    bg1[rb] = lane_base(g1T, rb);
  }
  // A operand of fc2 k-step I (h1 features 32 I .. 32 I + 31) for both row blocks: tanh in place,
  // the h1^T stores, the transposes; returns the number of stores
  constexpr int NSTA = FWD ? 0 : 2 * H::SPS * RB;   // h1^T store instructions of one prep_a
  auto prep_a = [&](auto Ic) __attribute__((always_inline)) {
    constexpr int I = decltype(Ic)::value;
    constexpr bool last = I == C::K2 - 1;
    const int c0 = 32 * I + lr;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const f32x4 h0 = act_tanh4<DT_S3>(acc1[rb][2 * I]), h1 = act_tanh4<DT_S3>(acc1[rb][2 * I + 1]);
      acc1[rb][2 * I] = h0;
      acc1[rb][2 * I + 1] = h1;
      // (the last k-step holds the bias column (1) and zero padding: stored as such)
      const f32x4 s0 = last ? bias_col(h0, c0, n1) : h0, s1 = last ? bias_col(h1, c0 + 16, n1) : h1;
      if constexpr (!FWD) {
        opnd4u(bh1[rb] + (size_t)(2 * I) * tsb, s0, Q8_SH);
        opnd4u(bh1[rb] + (size_t)(2 * I + 1) * tsb, s1, Q8_SH);
      }
      tp_put(tpb + rb * TILE_F, s0, s1, lane);
    }
  };
  auto prep_b = [&](Frag (&fa)[RB]) __attribute__((always_inline)) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) fa[rb] = tp_getA<DT>(tpb + rb * TILE_F, lane);
  };
  auto prep = [&](auto Ic, Frag (&fa)[RB]) __attribute__((always_inline)) -> int {
    prep_a(Ic);
    prep_b(fa);
    return NSTA;
  };
  f32x4 acc2[RB][8];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc2[rb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  int nst = 0;
  if constexpr (f8_fc2<HEAD, F8>()) {
    // e4m3 fc2 of the policy: h1 (4 k-steps per stage, e4m3 x Q8_SH) x the e4m3 W2 image on the x128
    // MFMA — K = 128 in ONE stage; the operand preparation (tanh, h1^T stores, transposes) precedes
    // the wait (+ the first wait: the last fc1 stage's past-the-end X re-loads)
    nst = 4 * XDMA;
    static_for<0, fc2_stages<HEAD, F8>()>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      __builtin_amdgcn_sched_barrier(0);
      i32x8 ha;
      static_for<0, 4>([&](auto Ic) __attribute__((always_inline)) {
        constexpr int I = decltype(Ic)::value;
        prep_a(std::integral_constant<int, 4 * j + I>{});
        const long q = f8x8(tp_get8(tpb, lane) * Q8_SH);
        ha[2 * I] = (int)q;
        ha[2 * I + 1] = (int)(q >> 32);
      });
      stg = wait_step(nst + 4 * NSTA);
      nst = 0;
      // (tile pairs between scheduling barriers: at most two tiles' 8-register B operands live —
      // the value head has no registers for all seven)
      static_for<0, 7>([&](auto tc) __attribute__((always_inline)) {
        constexpr int t = decltype(tc)::value;
        acc2[0][t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ha, b128(stg, t), acc2[0][t], 0, 0, 0, 127, 0, 127);
        if constexpr (t & 1) __builtin_amdgcn_sched_barrier(0);
      });
    });
    const float s2 = a.qscale[C::L2] * (1.0f / Q8_SH);
    // h2 = tanh(fc2), kept in registers for fc3, dgrad fc3 and the fused narrow-layer wgrad
#pragma unroll
    for (int t = 0; t < 8; ++t) acc2[0][t] = act_tanh4<DT_S3>(acc2[0][t] * s2);
  } else {
  Frag a0[RB], a1[RB];
  // (+ the X loads of the last fc1 step: policy past-the-end re-loads)
  nst = prep(std::integral_constant<int, 0>{}, a0) + (HEAD == 0 ? 2 * XDMA : 0);
  static_for<0, C::K2 / 2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    stg = wait_step(nst);
    // k-step 2j's MFMAs with k-step 2j+1's operand preparation in their shadow, then k-step
    // 2j+1's with 2j+2's
    mma_mix<DT, 0x7fu, 0, 8, 7 * RB * MPP, VPM>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
      constexpr int t = decltype(qc)::value;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc2[rb][t] = hmma<DT>(acc2[rb][t], a0[rb], b);
    }, [&]() __attribute__((always_inline)) { prep_a(std::integral_constant<int, 2 * j + 1>{}); }, flush);
    prep_b(a1);
    nst = NSTA;
    if constexpr (2 * j + 2 < C::K2) {
      mma_mix<DT, 0x7f00u, 8, 16, 7 * RB * MPP, VPM>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
        constexpr int t = decltype(qc)::value - 8;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc2[rb][t] = hmma<DT>(acc2[rb][t], a1[rb], b);
      }, [&]() __attribute__((always_inline)) { prep_a(std::integral_constant<int, 2 * j + 2>{}); }, flush);
      prep_b(a0);
      nst += NSTA;
    } else {
      for_slots<DT, 0x7f00u, 8, 16, 4>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
        constexpr int t = decltype(qc)::value - 8;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc2[rb][t] = hmma<DT>(acc2[rb][t], a1[rb], b);
      }, flush);
      // h2 = tanh(fc2), kept in registers for fc3, dgrad fc3 and the fused narrow-layer wgrad
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc2[rb][t] = act_tanh4<DT_S3>(acc2[rb][t]);
    }
  });
  }

  HD_STAMP(2);
  // ---------------- fc3 + loss + dgrad fc3: one stage ----------------
  stg = wait_step(nst);
  HD_STAMP(3);
  f32x4 a3[RB][C::N3];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < C::N3; ++t) a3[rb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fc3 k-step by k-step: the A operand (h2 features 32 ks .. +31, bias column, padding) and the
  // fragments of that k-step (slot 4 t + ks)
  static_for<0, 4>([&](auto kc) __attribute__((always_inline)) {
    constexpr int ks = decltype(kc)::value;
    const int c0 = 32 * ks + lr;
    Frag am[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      tp_put(tpb + rb * TILE_F, bias_col(acc2[rb][2 * ks], c0, n2), bias_col(acc2[rb][2 * ks + 1], c0 + 16, n2), lane);
      am[rb] = tp_getA<DT>(tpb + rb * TILE_F, lane);
    }
    constexpr unsigned M3 = C::N3 == 2 ? ((1u << ks) | (1u << (4 + ks))) : (1u << ks);
    for_slots<DT, M3, 0, 8, 8>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
      constexpr int t = decltype(qc)::value >> 2;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) a3[rb][t] = hmma<DT>(a3[rb][t], am[rb], b);
    }, flush);
  });
  HD_STAMP(12);
  if constexpr (FWD) {
    // V of the wave's rows: column 0 of the fc3 tile (lanes lr == 0 hold rows 4 lg .. 4 lg + 3)
    if (lr == 0) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mw + 16 * rb + 4 * lg + i;
          if (m < a.M) a.v_out[m] = a3[rb][0][i];
        }
    }
    WAIT_VMCNT(0);   // no DMA may outlive the workgroup's LDS
    return;
  } else {
  // (the transpose tiles hold mu / v from here: every wave's own)
  float dls[JM], lt[6];
#pragma unroll
  for (int q = 0; q < JM; ++q) dls[q] = 0.f;
#pragma unroll
  for (int k = 0; k < 6; ++k) lt[k] = 0.f;
  Frag ad[RB];   // the A operand of dgrad fc3: dL/dmu (policy) | dL/dv in column 0 (value)
  if constexpr (HEAD == 0) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * rb + 4 * lg + i;
        if (lr < A) mus[r * 32 + lr] = a3[rb][0][i];
        if (16 + lr < A) mus[r * 32 + 16 + lr] = a3[rb][1][i];
      }
    {
      // zero the wave's dL/dmu tile [16][32] (columns >= A are the padded K of dgrad fc3)
      float4* z = reinterpret_cast<float4*>(dml + (lane >> 2) * SST + 8 * (lane & 3));
      z[0] = z[1] = float4{0.f, 0.f, 0.f, 0.f};
    }
    const int r = lrow, sub = lsub;
    const bool valid = lvalid;
    const float cvar = a.std_var ? 0.5f : 1.f;
    float lclip = 0.f, lent = 0.f, kl = 0.f, cf = 0.f;
    if (a.loss_kind == 0) {
      // ---- corrected PPO (ppo.py:148-167) ----
      float logp = 0.f;
#pragma unroll
      for (int q = 0; q < JM; ++q) {
        const int j = sub + TPR * q;
        if (j >= A) break;
        const float lsig = cvar * lsv[q];
        const float z = (actv[q] - mus[r * 32 + j]) * __expf(-lsig);
        logp += -0.5f * z * z - 0.5f * HD_LOG_2PI - lsig;
      }
      logp = xsum<TPR - 1>(logp);
      const float lrat = logp - l_lpo;
      const float ratio = __expf(lrat);
      const float s1 = ratio * l_adv;
      const float s2 = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip) * l_adv;
      lclip = -fminf(s1, s2);
      const float dlogp = (s1 <= s2) ? -l_adv * ratio : 0.f;
      kl = (ratio - 1.f) - lrat;
      cf = (fabsf(ratio - 1.f) > a.clip) ? 1.f : 0.f;
#pragma unroll
      for (int q = 0; q < JM; ++q) {
        const int j = sub + TPR * q;
        if (j >= A) break;
        const float lsig = cvar * lsv[q];
        const float isig = __expf(-lsig);
        const float z = (actv[q] - mus[r * 32 + j]) * isig;
        dml[r * SST + j] = valid ? dlogp * z * isig : 0.f;
        dls[q] = valid ? (dlogp * (z * z - 1.f) - a.ent_coeff) * cvar : 0.f;
        lent += -a.ent_coeff * (0.5f + 0.5f * HD_LOG_2PI + lsig);
      }
      lent = xsum<TPR - 1>(lent);
    } else {
      // ---- reference DPPO loss (train.py:142-161): per-dim pdf ratio, variance convention ----
      const float invA = 1.f / (float)A;
      const bool first = a.first_step != 0;
#pragma unroll
      for (int q = 0; q < JM; ++q) {
        const int j = sub + TPR * q;
        if (j >= A) break;
        const float mu = mus[r * 32 + j];
        const float var = __expf(lsv[q]);
        const float mu_o = first ? mu : mupv[q];
        const float var_o = first ? var : __expf(lsov[q]);
        const float x = actv[q];
        const float pd = __expf(-(x - mu) * (x - mu) / (2.f * var)) * rsqrtf(2.f * var * 3.14159265358979f);
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
        dml[r * SST + j] = valid ? dp * pd * (x - mu) / var : 0.f;
        dls[q] = valid ? dp * pd * ((x - mu) * (x - mu) / (2.f * var) - 0.5f) : 0.f;
        cf += (fabsf(ratio - 1.f) > a.clip) ? invA : 0.f;
        if (valid) a.mu_prev[(size_t)lsrc * A + j] = mu;   // train.py:164 model_old <- model
      }
      lclip = xsum<TPR - 1>(lclip);
      lent = xsum<TPR - 1>(lent);
      cf = xsum<TPR - 1>(cf);
    }
    if (sub == 0) {
      const float vm = valid ? 1.f : 0.f;
      lt[0] = lclip * vm; lt[2] = lent * vm; lt[3] = kl * vm; lt[4] = cf * vm; lt[5] = vm;
    }
    // the wave's partial sums over its 32 rows (lanes of one sub-lane: xor over lane bits 1-5)
#pragma unroll
    for (int q = 0; q < JM; ++q) dls[q] = xsum<63 & ~(TPR - 1)>(dls[q]);
#pragma unroll
    for (int k = 0; k < 6; ++k) lt[k] = xsum<63 & ~(TPR - 1)>(lt[k]);
    if (lane < TPR) {
#pragma unroll
      for (int q = 0; q < JM; ++q)
        if (lane + TPR * q < A) wpart[NPF + lane + TPR * q] = dls[q];
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) wpart[k] = lt[k];
        wpart[6] = wpart[7] = 0.f;
      }
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) ad[rb] = tp_getA<DT>(dml + 16 * rb * SST, lane);
  } else {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (lr == 0) mus[16 * rb + 4 * lg + i] = a3[rb][0][i];
    float dv = 0.f;
    if (lsub == 0) {
      const float v = mus[lrow];
      const bool valid = lvalid;
      const bool first = a.first_step != 0;
      const float vold = ref_loss ? (first ? v : l_vprev) : l_vold;
      float lv;
      if (a.value_loss == 0) {
        const float d = v - l_ret;
        lv = d * d;
        dv = 2.f * d;
      } else {
        const float d1 = v - l_ret;
        const float dd = v - vold;
        const float vc = vold + fminf(fmaxf(dd, -a.clip), a.clip);
        const float d2 = vc - l_ret;
        const float f1 = d1 * d1, f2 = d2 * d2;
        const float inr = (dd >= -a.clip && dd <= a.clip) ? 1.f : 0.f;
        lv = 0.5f * fmaxf(f1, f2);
        if (f1 > f2) dv = d1;
        else if (f2 > f1) dv = d2 * inr;
        else dv = 0.5f * d1 + 0.5f * d2 * inr;
      }
      if (ref_loss && valid) a.v_prev[lsrc] = v;
      dv = valid ? dv : 0.f;
      const float vm = valid ? 1.f : 0.f;
      lt[1] = lv * vm;
      lt[5] = vm;
      dml[lrow] = dv;   // dL/dv of the wave's 32 rows
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) lt[k] = xsum<WROWS - 1>(lt[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) wpart[k] = lt[k];
      wpart[6] = wpart[7] = 0.f;
    }
    // the A operand of dgrad fc3 (K = 32, only k = 0 nonzero)
    float dvr[RB];
    {
      const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)dml;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        float d0;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(d0) : "v"(base + 4u * (16 * rb + lr)) : "memory");
        dvr[rb] = d0;
      }
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) ad[rb] = H::from8(f32x8{lg == 0 ? dvr[rb] : 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f});
    // the fused v-layer weight gradient over the wave's 32 rows: dW_v[k] = sum_r dL/dv[r] h2[r][k]
    // (h2 with the bias column 1: k = 100 is the bias gradient) -> the wave's 128 partials
    {
      const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)dml;
      f32x4 dq[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        float4 q0;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(q0) : "v"(base + 16u * (4 * rb + lg)) : "memory");
        dq[rb] = f32x4{q0.x, q0.y, q0.z, q0.w};
      }
      float* wdw = wpart + NPF + 32;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        float sacc = 0.f;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const f32x4 h = bias_col(acc2[rb][t], 16 * t + lr, n2);
#pragma unroll
          for (int i = 0; i < 4; ++i) sacc = fmaf(dq[rb][i], h[i], sacc);
        }
        sacc += __shfl_xor(sacc, 16, 64);
        sacc += __shfl_xor(sacc, 32, 64);
        if (lg == 0) wdw[16 * t + lr] = sacc;
      }
    }
  }

  HD_STAMP(4);
  // dgrad fc3: dpre2 = (dY W3) * (1 - h2^2) -> g2^T stores and the A operands of dgrad fc2
  f32x4 d2[RB][8];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < 8; ++t) d2[rb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for_slots<DT, 0x7f00u, 8, 16, 4>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
    constexpr int t = decltype(qc)::value - 8;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) d2[rb][t] = hmma<DT>(d2[rb][t], ad[rb], b);
  }, flush);
  nst = 0;
  // Q8: this step's store scales of the head's two gradient tensors (g1: 2 HEAD, g2: 2 HEAD + 1)
  // from the previous step's maxima (scalar loads); the running |g| maxima of this wave
  float sg1 = 1.f, sg2 = 1.f, am1 = 0.f, am2 = 0.f;
  if constexpr (Q8) {
    sg1 = q8_pow2(q8_exp(wave_umax(q8l[lane])));
    sg2 = q8_pow2(q8_exp(wave_umax(q8l[Q8_SUB + lane])));
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int c = 16 * t + lr;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      d2[rb][t] = c < n2 ? ew_dtanh(d2[rb][t], acc2[rb][t]) : f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (Q8) am2 = fmaxf(am2, absmax4(d2[rb][t]));
      opnd4(bg2[rb] + (size_t)t * tsb, d2[rb][t], sg2);
    }
  }
  nst += 8 * H::SPS * RB;
  Frag a2[4][RB];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      tp_put(tpb + rb * TILE_F, d2[rb][2 * ks], d2[rb][2 * ks + 1], lane);
      a2[ks][rb] = tp_getA<DT>(tpb + rb * TILE_F, lane);
    }
  // (the loss's dY^T stores are not counted: an undercount, the next waits cover them)

  HD_STAMP(5);
  // ---------------- dgrad fc2: g1 = (dpre2 W2) * (1 - h1^2), only the wgrad operand ----------------
  f32x4 gq[4][RB];
  auto epi = [&](auto sc) __attribute__((always_inline)) -> int {
    constexpr int s = decltype(sc)::value;
    int n = 0;
    static_for<0, 4>([&](auto uc) __attribute__((always_inline)) {
      constexpr int tt = 4 * s + decltype(uc)::value;
      if constexpr (tt < C::N1R) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const f32x4 h = acc1[rb][tt];
          const f32x4 gv = ew_dtanh(gq[decltype(uc)::value][rb], h);
          if constexpr (Q8) am1 = fmaxf(am1, absmax4(gv));
          opnd4(bg1[rb] + (size_t)tt * tsb, gv, sg1);
        }
        n += H::SPS * RB;
      }
    });
    return n;
  };
  static_for<0, C::NS4>([&](auto sc) __attribute__((always_inline)) {
    constexpr int s = decltype(sc)::value;
    stg = wait_step(nst);
    f32x4 g[4][RB];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) g[u][rb] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr unsigned M4 = (4 * s + 3 < C::N1R) ? 0xffffu : ((1u << (4 * ((C::N1R - 4 * s) & 3))) - 1u);
    // (fragment reads in groups of 2 where the registers are tight: split-bf16, and the value
    // head with the e4m3 operand stores' scales / maxima)
    constexpr int G4 = (DT == DT_S3 || (Q8 && HEAD == 1)) ? 2 : HD_G4_BF16;
    for_slots<DT, M4, 0, 16, G4>(stg, lane, [&](auto qc, const Frag& b) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) g[q >> 2][rb] = hmma<DT>(g[q >> 2][rb], a2[q & 3][rb], b);
    }, flush);
    if constexpr (s > 0) nst = epi(std::integral_constant<int, s - 1>{});
    else nst = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) gq[u][rb] = g[u][rb];
  });
  epi(std::integral_constant<int, C::NS4 - 1>{});
  HD_STAMP(6);

  // ---------------- policy: the fused mu-layer weight gradient over the wave's rows ----------------
  // dW_mu[j][k] = sum_r dL/dmu[r][j] h2[r][k] (h2 with the bias column 1: k = 100 is the bias
  // gradient) as MFMAs with the rows as K: A = dL/dmu^T (lane j, 8 rows) from the loss tile,
  // B = h2^T (lane k, 8 rows) through a [k][rows] LDS image, in two 64-feature halves
  f32x4 dwm[2][8];
  if constexpr (HEAD == 0) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int t = 0; t < 8; ++t) dwm[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // (the wave's 16 rows are k = 0-15 of the MFMA's 32: lane groups 2, 3 hold zeros)
    Frag am2[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      f32x8 x;
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = lg < 2 ? dml[(8 * lg + e) * SST + 16 * m + lr] : 0.f;
      am2[m] = H::from8(x);
    }
    constexpr int HLD = 20;                                    // [64 features][HLD] (16 rows + pad)
    float* h2t = dml + ((WROWS * SST + NPF + 32 + 3) & ~3);    // after the loss tile + partials
    static_for<0, 2>([&](auto hc) __attribute__((always_inline)) {
      constexpr int hh = decltype(hc)::value;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int t = 4 * hh + tt;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          // lane (feature 16 t + lr, rows 16 rb + 4 lg .. +3): one 16-byte store
          const f32x4 h = bias_col(acc2[rb][t], 16 * t + lr, n2);
          *reinterpret_cast<float4*>(h2t + (16 * tt + lr) * HLD + 16 * rb + 4 * lg) = float4{h[0], h[1], h[2], h[3]};
        }
      }
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const float* r = h2t + (16 * tt + lr) * HLD + 8 * (lg & 1);
        float4 x0 = *reinterpret_cast<const float4*>(r), x1 = *reinterpret_cast<const float4*>(r + 4);
        if (lg >= 2) x0 = x1 = float4{0.f, 0.f, 0.f, 0.f};
        const Frag bh = H::from8(f32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w});
#pragma unroll
        for (int m = 0; m < 2; ++m) dwm[m][4 * hh + tt] = hmma<DT>(dwm[m][4 * hh + tt], am2[m], bh);
      }
    });
  }

  HD_STAMP(10);
  if constexpr (Q8) {
    // this step's gradient maxima (max is order-independent: the atomics keep it deterministic)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      am1 = fmaxf(am1, __shfl_xor(am1, o, 64));
      am2 = fmaxf(am2, __shfl_xor(am2, o, 64));
    }
    const int sub = (blockIdx.x * NW + wave) & (Q8_SUB - 1);
    if (lane == 0) {
      atomicMax(a.q8_acc + ((2 * HEAD) * Q8_SUB + sub) * Q8_LINE, __float_as_uint(am1));
      atomicMax(a.q8_acc + ((2 * HEAD + 1) * Q8_SUB + sub) * Q8_LINE, __float_as_uint(am2));
    }
    if (blockIdx.x == 0 && tid < 2 * Q8_SUB) a.q8_clr[(2 * HEAD * Q8_SUB + tid) * Q8_LINE] = 0u;
  }
  // ---------------- per-workgroup partials (deterministic fixed order) ----------------
  WAIT_VMCNT(0);   // no DMA may outlive the workgroup's LDS
  HD_STAMP(11);
  __syncthreads();
  if constexpr (HEAD == 0) {
    // the 8 waves' dW_mu tiles [32][128] through the (now idle) 64 KiB ring in two rounds:
    // slot w = wave w + 4's tile, then + wave w's; the 4 slots summed in order (fixed order)
    float* red = reinterpret_cast<float*>(smem) + (wave & 3) * 32 * 128;
    if (wave >= 4) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[(16 * m + 4 * lg + i) * 128 + 16 * t + lr] = dwm[m][t][i];
    }
    __syncthreads();
    if (wave < 4) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[(16 * m + 4 * lg + i) * 128 + 16 * t + lr] += dwm[m][t][i];
    }
    __syncthreads();
    const float* r0 = reinterpret_cast<const float*>(smem);
    float* dst = a.part + (size_t)blockIdx.x * a.npart + a.part_dw;
    for (int e = tid; e < 32 * 128; e += NW * 64)
      dst[e] = ((r0[e] + r0[4096 + e]) + r0[2 * 4096 + e]) + r0[3 * 4096 + e];
  } else {
    const float* sc1 = reinterpret_cast<const float*>(smem + (size_t)S * SB);
    float* dst = a.part + (size_t)blockIdx.x * a.npart + a.part_dw;
    if (tid < 128) {
      float sv = 0.f;
      for (int w = 0; w < NW; ++w) sv += sc1[w * WS_F + WROWS * SST + NPF + 32 + tid];
      dst[tid] = sv;
    }
  }
  // (each head writes only its own columns — policy: loss terms 0, 2-7 and the A dlog_std;
  // value: the value-loss column 1 — so both kernels can share one partial buffer)
  const float* sc0 = reinterpret_cast<const float*>(smem + (size_t)S * SB);
  const int np = HEAD == 0 ? NPF + A : 1;
  for (int i = tid; i < np; i += NW * 64) {
    const int q = HEAD == 0 ? (i == 1 ? NPF + A : i) : 1;   // (policy: column 1 is the value's)
    if (q >= NPF + A) continue;
    float s = 0.f;
    for (int w = 0; w < NW; ++w) s += sc0[w * WS_F + WROWS * SST + q];
    a.part[(size_t)blockIdx.x * a.npart + q] = s;
  }
  HD_STAMP(7);
  }   // !FWD
}

template <int DT, int HEAD, bool FWD = false, bool F8 = false, bool Q8 = false>
void head_launch_t(const MlpArgs& a, hipStream_t s) {
  const size_t lds = head_lds_bytes<DT, HEAD, F8>();
  set_max_lds_once<mlp_head_kernel<DT, HEAD, FWD, F8, Q8>>(lds);
  const int nblk = (a.M + ROWS - 1) / ROWS;
  hipLaunchKernelGGL((mlp_head_kernel<DT, HEAD, FWD, F8, Q8>), dim3(nblk), dim3(HeadCfg<HEAD>::NW * 64), lds, s, a);
  HIP_CHECK_LAUNCH();
}

// the value head in fp8 mode (a.W8: the e4m3 image, a.qscale its per-layer scales) takes the
// e4m3 fc1 when the k-steps pair up (d_in a multiple of 64)
// (F8 needs the fc1 k-steps to group: pairs for the value head, quads for the policy's x128 MFMA)
template <int HEAD>
bool f8_applies(const MlpArgs& a) {
  const int ks1 = a.d_in[0] >> 5;
  return a.W8 != nullptr && a.qscale != nullptr && (HEAD == 0 ? (ks1 & 3) == 0 : (ks1 & 1) == 0);
}

template <int DT, int HEAD, bool FWD = false>
void head_launch(const MlpArgs& a, hipStream_t s) {
  if constexpr (DT == DT_BF16 && !FWD) {
    if (a.q8_rd != nullptr) {   // fp8 mode: e4m3 wgrad operands (+ the e4m3 forward GEMMs)
      if (f8_applies<HEAD>(a)) {
        head_launch_t<DT, HEAD, FWD, true, true>(a, s);
        return;
      }
      head_launch_t<DT, HEAD, FWD, false, true>(a, s);
      return;
    }
  }
  if constexpr (DT == DT_BF16 && (HEAD == 1 || !FWD)) {
    if (f8_applies<HEAD>(a)) {
      head_launch_t<DT, HEAD, FWD, true>(a, s);
      return;
    }
  }
  head_launch_t<DT, HEAD, FWD>(a, s);
}

int g_head_enable = 1;

}  // namespace

// shapes the per-head kernels cover (the reference network: policy 100-100, value 500-100; any
// observation width <= 383 and action width <= 32); anything else runs the generic kernels
extern "C" int mlp_head_applies(const MlpArgs& a) {
  if (!g_head_enable) return 0;
  return a.d_in[0] <= 384 && a.d_in[0] >= 32 && a.d_in[0] == a.d_in[3] && (a.n_out[0] + 15) / 16 == 7 &&
         (a.n_out[3] + 15) / 16 == 32 && a.d_in[1] == 128 && a.d_in[4] == 512 && a.d_in[2] == 128 &&
         a.d_in[5] == 128 && a.d_out[1] == 128 && a.d_out[4] == 128 && a.d_out[2] == 32 && a.d_out[5] == 32 &&
         a.n_out[1] > 96 && a.n_out[1] <= 112 && a.n_out[4] > 96 && a.n_out[4] <= 112 && a.A >= 1 && a.A <= 32;
}

extern "C" int mlp_head_rows() { return ROWS; }
extern "C" int mlp_head_waves(int head) { return head == 0 ? HeadCfg<0>::NW : HeadCfg<1>::NW; }

extern "C" void launch_mlp_head(int dt, int head, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_S3) {
    if (head == 0) head_launch<DT_S3, 0>(a, s);
    else head_launch<DT_S3, 1>(a, s);
  } else {
    if (head == 0) head_launch<DT_BF16, 0>(a, s);
    else head_launch<DT_BF16, 1>(a, s);
  }
}

// the value forward (GAE input) on the value head's streaming kernel (split-bf16)
extern "C" void launch_mlp_head_value(int dt, const MlpArgs& a, hipStream_t s) {
  if (dt == DT_S3) head_launch<DT_S3, 1, true>(a, s);
  else head_launch<DT_BF16, 1, true>(a, s);
}

extern "C" void set_head_kernels(int enable) { g_head_enable = enable ? 1 : 0; }
extern "C" int head_kernels_enabled() { return g_head_enable; }
