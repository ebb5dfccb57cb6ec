// Host-visible launcher prototypes + argument structs (no torch headers: the .hip files
// compile fast and only bindings.cpp pulls in torch).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct RolloutArgs {
  // env (state lives in global memory between launches, in LDS during the launch)
  int kind;            // 0 synthetic, 1 pendulum
  int E, O, A, S;      // envs, obs dims, act dims, state dims
  int T;               // steps in this launch
  int t_base;          // buffer time index of the first step
  int buf_E;           // env stride of the [T+1][E] buffers (== E)
  uint32_t t0;         // global step counter of the first step (RNG key)
  int limit;           // episode step limit
  uint32_t key_env, key_term, key_reset, key_action;
  float* state;        // [E][S]
  int* ep_len;         // [E]
  float* ep_ret;       // [E]
  // policy (packed weight image, storage precision)
  const void* W;
  int off_w1, off_w2, off_w3;
  int d1, d2, d3;      // padded input widths of the 3 layers (P32(K+1))
  int n1, n2, n3;      // real output widths (H1, H2, A)
  float s1, s2, s3;    // dequant scales (fp8; 1 otherwise)
  const float* qscale; // optional device array of the 6 per-layer dequant scales (overrides s*)
  const float* log_std;  // [A] fp32 master
  int std_var;         // 1: exp(log_std) is the variance (reference DPPO), 0: it is sigma
  // observation normalisation
  const float* mean;
  const float* inv_std;
  const float* shift;
  float reward_clip;   // <= 0: off
  // outputs
  void* x_out;         // [(T+1)*E][d1] storage precision (row-major, update input)
  float* actions;      // [T][E][A]
  float* logp;         // [T][E]
  float* rewards;      // [T][E] (clipped)
  float* dones;        // [T][E]
  void* xT_out;        // optional FM [rows][ldT] transposed copy of x rows t*E+e (wgrad operand)
  int ldT;             // its row length (== T*E of the whole buffer)
  float* mom;          // [nblk][2][O]  sum(x-shift), sum((x-shift)^2)
  float* epstat;       // [nblk][2]     finished-episode return sum, count
  unsigned long long* tstamp;  // DIAGNOSTIC ONLY (null in real runs): [nblk][NW][8] phase cycles
  // Per-step observation normalisation INSIDE the launch (obs_norm_update = "step", the reference's
  // filter that absorbs every observation before normalising it, model.py:68 / train.py:84-85);
  // sn_g1 == null: off (mean / inv_std above are fixed for the launch).  Step t, all workgroups
  // co-resident (cooperative launch): each publishes its batch moments about `shift` as 8-byte
  // {tag, fp32} granules (sn_g1, sn_g1_index); workgroup b sums the 4-feature units b, b + nblk, ... over all
  // workgroups in a fixed order (fp64), Chan-merges them into the fp64 running stats (sn_mean,
  // sn_m2: each feature owned by ONE workgroup for the whole launch) and publishes the new fp32
  // (mean, 1/std) as granules (sn_g2[2O]); every workgroup gathers those and normalises.  Tags
  // are sn_epoch0 + t (the host never reuses one: no memset), spins are bounded (sn_err).
  double* sn_mean;           // [O] running mean (fp64, in place)
  double* sn_m2;             // [O] running sum of squared deviations (fp64, in place)
  float* sn_mean_f32;        // [O] fp32 images after the last step (host-visible)
  float* sn_inv_std;         // [O]
  unsigned long long* sn_g1; // sn_g1_elems(nblk, O) partial-moment granules (sn_g1_index)
  unsigned long long* sn_g2; // [2O] stats granules
  unsigned* sn_err;          // nonzero: a spin timed out (the launch gave up; the host raises)
  double sn_n0;              // running count before step 0 (each step adds E)
  unsigned sn_epoch0;        // tag of step 0's granules (>= 1)
  double sn_var_floor;
};

// The per-step filter's partial-moment granules (RolloutArgs::sn_g1), line-blocked: a 128-byte
// line holds moment m of features 4 fu .. 4 fu + 3 of workgroups 4 wb .. 4 wb + 3 (granule
// 4 (w & 3) + (d & 3)); lines ordered [m][fu][wb].
inline __host__ __device__ size_t sn_g1_index(int m, int d, int w, int O, int nblk) {
  const int nfu = (O + 3) >> 2, nwb = (nblk + 3) >> 2;
  return ((size_t)(m * nfu + (d >> 2)) * nwb + (w >> 2)) * 16 + (size_t)(w & 3) * 4 + (d & 3);
}
inline __host__ __device__ size_t sn_g1_elems(int nblk, int O) {
  return (size_t)2 * ((O + 3) >> 2) * ((nblk + 3) >> 2) * 16;
}

// fp8 mode's gradient-amax ring (csrc/common.h Q8): [3 slots][4 tensors][Q8_SUB sub-slots][Q8_LINE]
constexpr int Q8_SUB = 64, Q8_LINE = 32;
constexpr int Q8_SLOT = 4 * Q8_SUB * Q8_LINE;   // dwords per ring slot

struct MlpArgs {
  // input rows: x_buf row-major [*][d1]; row m of this call reads x_buf[idx ? idx[m] : row0 + m]
  const void* x_buf;
  const int* idx;
  int row0;
  int M;               // rows in this call (multiple of ROWS handled by masking)
  // packed weights (storage precision) + offsets (elements) of Wp / Wpt per layer
  const void* W;
  const void* W8;        // fp8 mode: the e4m3 image (the value head's fc1, csrc/mlp_head.hip F8)
  int off_w[6];        // p1 p2 p3 v1 v2 v3 (forward images)
  int off_wt[6];       // transposed images (dgrad)
  int d_in[6];         // padded input width per layer
  int d_out[6];        // padded output width per layer
  int n_out[6];        // real output width per layer
  float scale[6];      // fp8 dequant scale per layer
  const float* qscale; // optional device array of the 6 per-layer scales (overrides scale[])
  int A;
  const float* log_std;  // [A]
  const float* log_std_old;  // [A] dppo_ref: log_std of the previous step
  // ---- training inputs (indexed by source row) ----
  const float* actions;   // [N][A]
  const float* logp_old;  // [N]
  const float* adv;       // [N]
  const float* ret;       // [N]
  const float* v_old;     // [N]
  float* mu_prev;         // [N][A] dppo_ref: params of the previous step (read, then overwritten)
  float* v_prev;          // [N]
  int loss_kind;          // 0 ppo, 1 dppo_ref
  int value_loss;         // 0 mse, 1 clipped_half
  int std_var;
  float clip, ent_coeff;
  int first_step;         // dppo_ref: 1 -> old == current
  // ---- outputs ----
  float* v_out;           // value-only mode: [M] (written at position m)
  // transposed (feature-major) operands for the wgrad GEMM, [rows][ldT] storage precision
  void* xT; void* h1pT; void* h2pT; void* h1vT; void* h2vT;
  void* g1pT; void* g2pT; void* g3pT; void* g1vT; void* g2vT; void* g3vT;
  int ldT;                // = M (row length of every transposed buffer)
  int xT_ready;           // 1: xT already holds this call's rows (full-batch: the rollout wrote it)
  int x_stream;           // 1: non-temporal observation-row loads (A/B knob; 0 default: cached)
  int64_t x_bytes;        // bytes of x_buf (kernels with 32-bit buffer offsets refuse >= 2 GiB)
  float* part;            // [nblk][NPART] per-workgroup partial sums (loss terms, dlog_std)
  int npart;
  int part_dw;            // per-head kernels: column of the fused narrow-layer weight gradient in a
                          // partial row (policy: dW_mu [32][128], value: dW_v [128]; bias = column 100)
  // fp8 mode's e4m3 wgrad operands (csrc/common.h Q8): null = the operands in the update's
  // precision.  Slots of the gradient-amax ring (4 tensors g1p, g2p, g1v, g2v x Q8_SUB sub-slots,
  // fp32 bits): the scales of this step come from q8_rd, its |g| maxima go to q8_acc, q8_clr is
  // zeroed
  const unsigned* q8_rd;
  unsigned* q8_acc;
  unsigned* q8_clr;
  // DIAGNOSTIC ONLY (scripts/phase_timeline.py; null in every real run): per-wave s_memtime
  // stamps at the phase boundaries of every tstamp_every-th workgroup, [blk][NW][16]
  unsigned long long* tstamp;
  int tstamp_every;
};

// per-head streaming update (csrc/mlp_head.hip): head 0 = policy, 1 = value; 128 rows per workgroup
extern "C" int mlp_head_applies(const MlpArgs& a);
extern "C" int mlp_head_rows();
extern "C" int mlp_head_waves(int head);
extern "C" void launch_mlp_head(int dt, int head, const MlpArgs& a, hipStream_t s);   // dt: bf16x3 or bf16
extern "C" void launch_mlp_head_value(int dt, const MlpArgs& a, hipStream_t s);   // V(x) on the value head kernel
extern "C" void set_head_kernels(int enable);
extern "C" int head_kernels_enabled();
// policy head update on 32x32x16 MFMAs, transposed chain (csrc/phead.hip): 128 rows per workgroup
extern "C" int phead_applies(const MlpArgs& a);   // set_phead flag and shapes
extern "C" int phead_shape_ok(const MlpArgs& a);
extern "C" int phead_rows();
// p2: p_fc2's weight gradient summed in the kernel (else h1p / g2p stored row-major for the wgrad)
extern "C" void launch_phead_train(int dt, const MlpArgs& a, int p2, hipStream_t s);
extern "C" void set_phead(int enable);

// fp8 mode: the Adam kernels also refresh the e4m3 image the update's fc1 reads (csrc/mlp_head.hip
// F8), element i as p / qs[lid[i]] with the iteration's per-layer scales; img == nullptr: off
struct F8Shadow {
  uint8_t* img;
  const int* lid;
  const float* qs;
};

#define DEV_HOST_INLINE __host__ __device__ inline

// The slab elements of a gather: up to 4 runs [lo, hi) of flat indices, every element with a slab
// source (src_meta != 0); start[r] = elements before run r (start[n..3] = INT_MAX), total = all.
// The gathers iterate over them without a data-dependent branch, so every per-element load of a
// thread issues in one round trip before its slab-chunk loads.
struct SlabRuns {
  int n, total;
  int lo[4], start[4];
  DEV_HOST_INLINE int flat(int j) const {
    int i = lo[0] + j;
#pragma unroll
    for (int r = 1; r < 4; ++r)
      if (j >= start[r]) i = lo[r] + (j - start[r]);
    return i;
  }
};

// reduce items per block of the gather kernels (common.h item_reduce)
constexpr int ITEM_IPB = 32;
inline __host__ __device__ int item_blocks(int nitems) { return (nitems + ITEM_IPB - 1) / ITEM_IPB; }

struct WgradTask {
  int layer;      // 0..5
  int n0, k0;     // output tile origin
  int m0, m1;     // reduction (batch) range
  int slab;       // slab offset (floats) of this task's [nq*64][kq*64] tile
  int nq, kq;     // tile extent in 64x64 quadrants (one per wave): nq*kq <= 8, nq + kq <= 6
};

struct WgradArgs {
  const void* gT[6];   // dY^T per layer  [rows >= n tile][ld]
  const void* xT[6];   // X^T per layer   [rows >= k tile][ld]
  int ld;
  const WgradTask* tasks;
  int ntasks;
  float* slab;
  // e4m3 operands (dt fp8, csrc/common.h Q8): the product tile of layer l is multiplied by
  // 1 / (2^q8_exp(max of tensor q8_t[l]'s sub-slots in q8_rd) * q8_xs[l]) — the gradient
  // tensor's delayed scale (the slot the update read) times the activation side's fixed scale
  const unsigned* q8_rd;
  int q8_t[6];
  float q8_xs[6];
  // row-major operands: the row length in elements of layer l's dY (g_rm) / X (x_rm) operand
  // ([ld rows][features]: csrc/phead.hip, x_buf), 0 = fragment-major
  int g_rm[6], x_rm[6];
  int wide;   // some task runs two quadrants per wave (wgrad_task_ok): the launch takes the wider LDS ring
};

extern "C" {
// first launch / attribute error recorded since the last call (0 = none), message into msg;
// resets the record (csrc/common.h dppo_note_error)
int dppo_take_error(char* msg, int cap);
void launch_debug_invalid(double* out, hipStream_t s);   // test hook: a launch the runtime refuses
void launch_rollout(int dt, const RolloutArgs& a, int rows, hipStream_t s);
void set_rollout_waves(int nw);                 // 4 or 8 waves per rollout workgroup (A/B)
int rollout_stepnorm_cap(int dt, const RolloutArgs& a, int rows);   // co-resident grid of the SN launch
void launch_mlp_value(int dt, const MlpArgs& a, hipStream_t s);
void launch_mlp_train(int dt, const MlpArgs& a, hipStream_t s);
size_t mlp_train_lds_bytes(int dt, const MlpArgs& a);
int mlp_train_rows(int dt, const MlpArgs& a);   // row tile the launcher will use (LDS-fit)
void set_mlp_rows_override(int rows);           // 0 auto; 16/32/64 force (A/B diagnostics)
void set_s3_train_waves(int nw);                // split-bf16 32-row tile: 4 or 8 waves (A/B)
void set_s3_value_waves(int nw);                // split-bf16 value forward: 4 or 8 waves (A/B)
int mlp_train_waves(int dt, const MlpArgs& a);  // workgroup waves the launcher will use
void launch_wgrad(int dt, const WgradArgs& a, hipStream_t s);
int wgrad_task_ok(int dt, int nq, int kq);   // the (nq, kq) quadrant tiles the wgrad kernel runs
// grad[i] for i in [i_lo, i_hi) from the slabs (src_off / src_meta: see grad_gather_kernel);
// with_partials: also log_std grads [0, A) and the 8 loss sums from the per-workgroup partials
void launch_grad_gather(const float* slab, const int* src_off, const int* src_meta, const float* part, int nblk,
                        int npart, const int* red_col, const int* red_dst, int nitems, float scale, float* grad,
                        const SlabRuns& runs, float* loss_out, hipStream_t s);
void launch_gae(const float* rewards, const float* values, const float* dones, float* adv, float* ret,
                int T, int E, float gamma, float lam, int mode, int seg, hipStream_t s);
void set_adam_fused(int on);
void launch_adam(float* p, const float* g, float* m, float* v, int n, float lr, float b1, float b2,
                 float eps, float max_norm, float* state, float* norm_part, int nblk,
                 void* wimg, const int* w_map, const int* wt_map, int dt, const float* img_scale, int host_step,
                 const F8Shadow& f8, hipStream_t s);
// grad_gather (with the partials pass, range [A, n)) + no-clip Adam fused: world size 1 only
// (no all-reduce between them); nblk = norm_part size, must exceed A + 8
void launch_gather_adam(const float* slab, const int* src_off, const int* src_meta, const float* part, int npblk,
                        int npart, const int* red_col, const int* red_dst, int nitems, const SlabRuns& runs,
                        float scale, float* loss_out, float* g, float* p, float* m, float* v,
                        int n, float lr, float b1, float b2, float eps, int step, float* state, float* norm_part,
                        int nblk, void* wimg, const int* w_map, const int* wt_map, int dt, const float* img_scale,
                        const F8Shadow& f8, hipStream_t s);
void launch_pack(const float* p, int n, void* wimg, const int* w_map, const int* wt_map, int dt,
                 const float* img_scale, hipStream_t s);
// fp8 forward image: qscale[6] = per-layer amax / 416 of p (lid: layer of each parameter, -1
// none; must be < 6), then the e4m3 image of p / qscale[lid] (two launches; part: 128 x 6
// floats of per-block maxima)
void launch_fp8_refresh(const float* p, const int* lid, int n, float* qscale, float* part, void* wimg,
                        const int* w_map, const int* wt_map, hipStream_t s);
// ep == nullptr: the moments only (epstat unread)
void launch_obs_reduce(const float* part, int nblk, int O, double* s12, const float* epstat, double* ep,
                       hipStream_t s);
// [E][O] observations -> [obs_moments_blocks(E)][2][O] fp32 partials about shift
int obs_moments_blocks(int E);
void launch_obs_moments(const float* obs, int E, int O, const float* shift, float* part, hipStream_t s);
void launch_obs_merge(const double* s12, int O, double count, double n_a, const float* shift, double* mean,
                      double* m2, float* mean_f32, float* inv_std, double var_floor, hipStream_t s);
// out f64[11] = [episode return sum, count | 8 loss sums | gradient L2 norm from the nblk
// per-block sums of squares the last Adam launch left in norm_part]
void launch_metrics_pack(const double* ep, const float* loss8, const float* norm_part, int nblk, double* out,
                         hipStream_t s);
// diagnostics: nblk workgroups of nthreads (lds bytes each) spinning `us` microseconds each
void launch_probe_spin(int nblk, int nthreads, int lds, double us, int* sink, hipStream_t s);
}

// operand buffers (feature-major) are padded to multiples of 128 rows
#define WGRAD_TILE 128
#define WGRAD_TASK_INTS 8
static_assert(sizeof(WgradTask) == WGRAD_TASK_INTS * sizeof(int), "WgradTask is an 8-int record");
