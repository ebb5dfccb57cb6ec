// PyTorch bindings for the DPPO HIP kernels.  Every entry point validates device, dtype,
// contiguity and the exact extents the kernel's grid/indexing assumes BEFORE launching, so
// a shape bug raises a Python exception instead of faulting the GPU.  Launches go to the
// current HIP stream (graph-capturable: no allocation, no sync in here).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <limits>
#include <vector>

#include "kernels.h"

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// Debug mode (DPPO_DEBUG_SYNC=1 / set_debug_sync, SURVEY §5.2 "HIP_LAUNCH_BLOCKING mode"): every
// binding synchronises its stream after its launch and raises on a launch or execution error,
// naming the binding — a kernel fault surfaces at the op that caused it, not at a later sync.
bool g_debug_sync = false;
void set_debug_sync(bool on) { g_debug_sync = on; }
// Always: a launch (or LDS attribute) error the launchers recorded raises here, naming the op.
void after_launch(const char* what) {
  char msg[192];
  const int code = dppo_take_error(msg, (int)sizeof(msg));
  TORCH_CHECK(code == 0, what, ": HIP launch failed: ", msg);
  if (!g_debug_sync) return;
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(cur_stream());
  TORCH_CHECK(e == hipSuccess, "debug-sync: ", what, " failed: ", hipGetErrorString(e));
}

// diagnostics only: per-phase cycle sums of the rollout kernel (scripts/phase_timeline.py)
unsigned long long* g_roll_tstamp = nullptr;
int64_t g_roll_tstamp_numel = 0;
void set_rollout_tstamp(torch::Tensor buf) {
  if (!buf.defined() || buf.numel() == 0) { g_roll_tstamp = nullptr; return; }
  TORCH_CHECK(buf.scalar_type() == at::kLong && buf.is_cuda() && buf.is_contiguous(), "int64 device buffer");
  g_roll_tstamp = reinterpret_cast<unsigned long long*>(buf.data_ptr<int64_t>());
  g_roll_tstamp_numel = buf.numel();
}
// diagnostics only: phase-timeline stamps of mlp_train (scripts/phase_timeline.py)
unsigned long long* g_tstamp = nullptr;
int g_tstamp_every = 1;
int64_t g_tstamp_numel = 0;
void set_train_tstamp(torch::Tensor buf, int64_t every) {
  if (!buf.defined() || buf.numel() == 0) { g_tstamp = nullptr; return; }
  g_tstamp_numel = buf.numel();
  TORCH_CHECK(buf.scalar_type() == at::kLong && buf.is_cuda() && buf.is_contiguous(), "int64 device buffer");
  TORCH_CHECK(every >= 1, "every");
  g_tstamp = reinterpret_cast<unsigned long long*>(buf.data_ptr<int64_t>());
  g_tstamp_every = (int)every;
}
int g_x_stream = 0;     // A/B: non-temporal observation-row loads in the value / update kernels
void set_x_stream(int64_t on) { g_x_stream = on ? 1 : 0; }

// dt 3 (split-bf16): one 4-byte slot per logical element (hi | lo bf16 pairs in 32-byte groups,
// csrc/common.h Prec<DT_S3>), held in int32 tensors so numel counts logical elements
at::ScalarType storage_type(int dt) {
  return dt == 0 ? at::kFloat : (dt == 1 ? at::kBFloat16 : (dt == 3 ? at::kInt : at::kByte));
}

void check(const torch::Tensor& t, const char* name, at::ScalarType st, int64_t min_numel) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
  TORCH_CHECK(t.numel() >= min_numel, name, " has ", t.numel(), " elements, kernel needs >= ", min_numel);
}

const float* opt_scales(const torch::Tensor& q) {
  if (!q.defined() || q.numel() == 0) return nullptr;
  check(q, "qscale", at::kFloat, 6);
  return q.data_ptr<float>();
}

struct Layout {
  int off_w[6], off_wt[6], d_in[6], d_out[6], n_out[6];
};

Layout parse_layout(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 30, "layout must have 30 ints");
  Layout L;
  for (int i = 0; i < 6; ++i) {
    L.off_w[i] = (int)v[i];
    L.off_wt[i] = (int)v[6 + i];
    L.d_in[i] = (int)v[12 + i];
    L.d_out[i] = (int)v[18 + i];
    L.n_out[i] = (int)v[24 + i];
    TORCH_CHECK(L.d_in[i] % 32 == 0 && L.d_out[i] % 32 == 0, "padded dims must be multiples of 32");
    TORCH_CHECK(L.n_out[i] < L.d_out[i], "n_out must leave a pad column");
  }
  return L;
}

int64_t wimg_extent(const Layout& L) {
  int64_t mx = 0;
  for (int i = 0; i < 6; ++i) {
    mx = std::max<int64_t>(mx, (int64_t)L.off_w[i] + (int64_t)L.d_out[i] * L.d_in[i]);
    mx = std::max<int64_t>(mx, (int64_t)L.off_wt[i] + (int64_t)L.d_in[i] * L.d_out[i]);
  }
  return mx;
}

// ------------------------------------------------------------------------------------------
RolloutArgs rollout_args(int64_t dt, int64_t rows, torch::Tensor state, torch::Tensor ep_len, torch::Tensor ep_ret,
                         torch::Tensor wimg, std::vector<int64_t> layout, std::vector<double> scales, torch::Tensor flat,
                         torch::Tensor mean, torch::Tensor inv_std, torch::Tensor shift, torch::Tensor x_out,
                         torch::Tensor actions, torch::Tensor logp, torch::Tensor rewards, torch::Tensor dones,
                         torch::Tensor mom, torch::Tensor epstat, std::vector<int64_t> ints, std::vector<int64_t> keys,
                         double reward_clip, torch::Tensor qscale, torch::Tensor xT_out, int64_t xT_rows) {
  TORCH_CHECK(ints.size() == 11, "ints: kind,E,O,A,S,T,t_base,buf_E,t0,limit,std_var");
  TORCH_CHECK(keys.size() == 4, "keys: env,term,reset,action");
  TORCH_CHECK(rows == 16 || rows == 32, "rows must be 16 or 32");
  Layout L = parse_layout(layout);
  RolloutArgs a{};
  a.kind = (int)ints[0]; a.E = (int)ints[1]; a.O = (int)ints[2]; a.A = (int)ints[3]; a.S = (int)ints[4];
  a.T = (int)ints[5]; a.t_base = (int)ints[6]; a.buf_E = (int)ints[7]; a.t0 = (uint32_t)ints[8];
  a.limit = (int)ints[9]; a.std_var = (int)ints[10];
  TORCH_CHECK(a.E > 0 && a.T >= 1 && a.buf_E == a.E, "bad E/T");
  TORCH_CHECK(a.kind == 0 || a.kind == 1, "kind");
  TORCH_CHECK(a.kind == 0 ? a.S == a.O : (a.S == 2 && a.O == 3), "state dims");
  TORCH_CHECK(L.n_out[2] == a.A && L.d_in[0] == ((a.O + 1 + 31) / 32) * 32, "layout/env mismatch");
  const int nblk = (a.E + (int)rows - 1) / (int)rows;
  check(state, "state", at::kFloat, (int64_t)a.E * a.S);
  check(ep_len, "ep_len", at::kInt, a.E);
  check(ep_ret, "ep_ret", at::kFloat, a.E);
  check(wimg, "wimg", storage_type((int)dt), wimg_extent(L));
  check(flat, "flat", at::kFloat, a.A);
  check(mean, "mean", at::kFloat, a.O);
  check(inv_std, "inv_std", at::kFloat, a.O);
  check(shift, "shift", at::kFloat, a.O);
  const int64_t rows_needed = (int64_t)(a.t_base + a.T + 1) * a.E;
  check(x_out, "x_out", storage_type(dt == 2 ? 1 : (int)dt), rows_needed * L.d_in[0]);
  check(actions, "actions", at::kFloat, (int64_t)(a.t_base + a.T) * a.E * a.A);
  check(logp, "logp", at::kFloat, (int64_t)(a.t_base + a.T) * a.E);
  check(rewards, "rewards", at::kFloat, (int64_t)(a.t_base + a.T) * a.E);
  check(dones, "dones", at::kFloat, (int64_t)(a.t_base + a.T) * a.E);
  check(mom, "mom", at::kFloat, (int64_t)nblk * 2 * a.O);
  check(epstat, "epstat", at::kFloat, (int64_t)nblk * 2);
  a.key_env = (uint32_t)keys[0]; a.key_term = (uint32_t)keys[1]; a.key_reset = (uint32_t)keys[2];
  a.key_action = (uint32_t)keys[3];
  a.state = state.data_ptr<float>();
  a.ep_len = ep_len.data_ptr<int>();
  a.ep_ret = ep_ret.data_ptr<float>();
  a.W = wimg.data_ptr();
  a.off_w1 = L.off_w[0]; a.off_w2 = L.off_w[1]; a.off_w3 = L.off_w[2];
  a.d1 = L.d_in[0]; a.d2 = L.d_in[1]; a.d3 = L.d_in[2];
  a.n1 = L.n_out[0]; a.n2 = L.n_out[1]; a.n3 = L.n_out[2];
  a.qscale = opt_scales(qscale);
  a.s1 = (float)scales.at(0); a.s2 = (float)scales.at(1); a.s3 = (float)scales.at(2);
  a.log_std = flat.data_ptr<float>();
  a.mean = mean.data_ptr<float>();
  a.inv_std = inv_std.data_ptr<float>();
  a.shift = shift.data_ptr<float>();
  a.reward_clip = (float)reward_clip;
  a.x_out = x_out.data_ptr();
  a.actions = actions.data_ptr<float>();
  a.logp = logp.data_ptr<float>();
  a.rewards = rewards.data_ptr<float>();
  a.dones = dones.data_ptr<float>();
  a.mom = mom.data_ptr<float>();
  a.xT_out = nullptr;
  a.ldT = 0;
  if (xT_out.defined() && xT_out.numel() > 0) {
    // FM transposed copy of the T*E training rows: the kernel writes 8-row groups per 16-env tile
    const int64_t ld = (int64_t)a.buf_E * (a.t_base + a.T);
    TORCH_CHECK(a.t_base == 0, "xT_out is written by a whole-rollout launch (t_base == 0)");
    TORCH_CHECK(a.E % 16 == 0 && ld % 32 == 0, "xT_out needs E % 16 == 0 and T*E % 32 == 0");
    TORCH_CHECK(xT_rows >= L.d_in[0] && xT_rows % 16 == 0, "xT_out rows must cover d_in and be a multiple of 16");
    check(xT_out, "xT_out", storage_type(dt == 2 ? 1 : (int)dt), xT_rows * ld);
    a.xT_out = xT_out.data_ptr();
    a.ldT = (int)ld;
  }
  a.epstat = epstat.data_ptr<float>();
  if (g_roll_tstamp != nullptr) {
    TORCH_CHECK(g_roll_tstamp_numel >= (int64_t)nblk * 8 * 16, "rollout tstamp buffer too small ([blk][8 waves][16])");
    a.tstamp = g_roll_tstamp;
  }
  return a;
}

void rollout(int64_t dt, int64_t rows, torch::Tensor state, torch::Tensor ep_len, torch::Tensor ep_ret,
             torch::Tensor wimg, std::vector<int64_t> layout, std::vector<double> scales, torch::Tensor flat,
             torch::Tensor mean, torch::Tensor inv_std, torch::Tensor shift, torch::Tensor x_out,
             torch::Tensor actions, torch::Tensor logp, torch::Tensor rewards, torch::Tensor dones,
             torch::Tensor mom, torch::Tensor epstat, std::vector<int64_t> ints, std::vector<int64_t> keys,
             double reward_clip, torch::Tensor qscale, torch::Tensor xT_out, int64_t xT_rows) {
  RolloutArgs a = rollout_args(dt, rows, state, ep_len, ep_ret, wimg, layout, scales, flat, mean, inv_std, shift,
                               x_out, actions, logp, rewards, dones, mom, epstat, ints, keys, reward_clip, qscale,
                               xT_out, xT_rows);
  launch_rollout((int)dt, a, (int)rows, cur_stream());
  after_launch(__func__);
}

// The per-step observation-normalisation rollout (obs_norm_update = "step") as ONE cooperative
// launch (csrc/rollout.hip sn_step): `sn` = [mean f64, m2 f64, mean_f32, inv_std] of the stats the
// steps absorb (updated in place), g1 / g2 the granule buffers (int64, zero-initialised once; tags
// never reused: epoch0 grows by T per launch), err an int32 timeout word.  The launch's own
// normalisation inputs (mean / inv_std) are ignored: every step takes the freshly merged stats.
void rollout_stepnorm(int64_t dt, int64_t rows, torch::Tensor state, torch::Tensor ep_len, torch::Tensor ep_ret,
                      torch::Tensor wimg, std::vector<int64_t> layout, std::vector<double> scales, torch::Tensor flat,
                      torch::Tensor shift, torch::Tensor x_out, torch::Tensor actions, torch::Tensor logp,
                      torch::Tensor rewards, torch::Tensor dones, torch::Tensor mom, torch::Tensor epstat,
                      std::vector<int64_t> ints, std::vector<int64_t> keys, double reward_clip, torch::Tensor qscale,
                      std::vector<torch::Tensor> sn, torch::Tensor g1, torch::Tensor g2, torch::Tensor err,
                      double n0, int64_t epoch0, double var_floor) {
  TORCH_CHECK(sn.size() == 4, "sn: mean f64, m2 f64, mean_f32, inv_std");
  RolloutArgs a = rollout_args(dt, rows, state, ep_len, ep_ret, wimg, layout, scales, flat, sn[2], sn[3], shift,
                               x_out, actions, logp, rewards, dones, mom, epstat, ints, keys, reward_clip, qscale,
                               torch::Tensor(), 0);
  TORCH_CHECK(a.t_base == 0, "the per-step normalisation launch covers the whole rollout");
  const int nblk = (a.E + (int)rows - 1) / (int)rows;
  check(sn[0], "sn mean", at::kDouble, a.O);
  check(sn[1], "sn m2", at::kDouble, a.O);
  TORCH_CHECK(sn[2].data_ptr() != shift.data_ptr(), "the shift must not alias the stats being merged into");
  check(g1, "g1", at::kLong, (int64_t)sn_g1_elems(nblk, a.O));
  check(g2, "g2", at::kLong, 2 * (int64_t)a.O);
  check(err, "err", at::kInt, 1);
  TORCH_CHECK(epoch0 >= 1 && epoch0 + a.T < (int64_t)UINT32_MAX, "epoch0");
  a.sn_mean = sn[0].data_ptr<double>();
  a.sn_m2 = sn[1].data_ptr<double>();
  a.sn_mean_f32 = sn[2].data_ptr<float>();
  a.sn_inv_std = sn[3].data_ptr<float>();
  a.sn_g1 = reinterpret_cast<unsigned long long*>(g1.data_ptr<int64_t>());
  a.sn_g2 = reinterpret_cast<unsigned long long*>(g2.data_ptr<int64_t>());
  a.sn_err = reinterpret_cast<unsigned*>(err.data_ptr<int>());
  a.sn_n0 = n0;
  a.sn_epoch0 = (unsigned)epoch0;
  a.sn_var_floor = var_floor;
  launch_rollout((int)dt, a, (int)rows, cur_stream());
  after_launch(__func__);
}

// the largest env-tile grid the per-step normalisation launch can run co-resident
int64_t rollout_stepnorm_cap_b(int64_t dt, int64_t rows, std::vector<int64_t> layout, int64_t O, int64_t A, int64_t S) {
  Layout L = parse_layout(layout);
  RolloutArgs a{};
  a.O = (int)O; a.A = (int)A; a.S = (int)S;
  a.d1 = L.d_in[0]; a.d2 = L.d_in[1]; a.d3 = L.d_in[2];
  a.sn_g1 = reinterpret_cast<unsigned long long*>(1);   // (only selects the LDS size of the SN kernel)
  return (int64_t)::rollout_stepnorm_cap((int)dt, a, (int)rows);
}

// idx_limit: exclusive upper bound every gathered row index must respect (rows of x_buf and of
// every per-row array).  check_idx=true range-checks the index VALUES on the device (one
// device->host read).  check_idx=false is only for callers that range-checked the indices on
// the host before uploading them (the hipGraph-captured update path, which cannot sync).
int64_t train_lds_bytes_impl(int dt, const Layout& L, int64_t A) {
  MlpArgs a{};
  for (int i = 0; i < 6; ++i) { a.d_in[i] = L.d_in[i]; a.d_out[i] = L.d_out[i]; a.n_out[i] = L.n_out[i]; }
  a.A = (int)A;
  return (int64_t)mlp_train_lds_bytes(dt, a);
}

MlpArgs base_mlp(int dt, const Layout& L, const std::vector<double>& scales, torch::Tensor x_buf,
                 torch::Tensor idx, int64_t row0, int64_t M, torch::Tensor wimg, torch::Tensor flat, int64_t A,
                 bool check_idx, int64_t idx_limit) {
  MlpArgs a{};
  check(wimg, "wimg", storage_type(dt), wimg_extent(L));
  check(flat, "flat", at::kFloat, A);
  TORCH_CHECK(M > 0, "M must be > 0");
  TORCH_CHECK(L.d_in[0] == L.d_in[3], "both heads share the input width");
  const int64_t nrows_x = x_buf.numel() / L.d_in[0];
  check(x_buf, "x_buf", storage_type(dt == 2 ? 1 : dt), 1);  // fp8 kernels read a bf16 buffer
  TORCH_CHECK(x_buf.numel() % L.d_in[0] == 0, "x_buf rows must have d_in[0] elements");
  const int64_t limit = std::min<int64_t>(idx_limit, nrows_x);
  if (idx.defined() && idx.numel() > 0) {
    check(idx, "idx", at::kInt, M);
    if (check_idx) {
      auto mm = torch::aminmax(idx.narrow(0, 0, M));
      const int mn = std::get<0>(mm).item<int>();
      const int mx = std::get<1>(mm).item<int>();
      TORCH_CHECK(mn >= 0 && mx < limit, "idx values out of range [0, ", limit, "): min ", mn, " max ", mx);
    }
    a.idx = idx.data_ptr<int>();
  } else {
    a.idx = nullptr;
    TORCH_CHECK(row0 >= 0 && row0 + M <= limit, "row range out of x_buf / per-row arrays");
  }
  a.x_buf = x_buf.data_ptr();
  a.x_bytes = (int64_t)x_buf.numel() * (int64_t)x_buf.element_size();
  a.row0 = (int)row0;
  a.M = (int)M;
  a.W = wimg.data_ptr();
  for (int i = 0; i < 6; ++i) {
    a.off_w[i] = L.off_w[i]; a.off_wt[i] = L.off_wt[i]; a.d_in[i] = L.d_in[i]; a.d_out[i] = L.d_out[i];
    a.n_out[i] = L.n_out[i]; a.scale[i] = (float)scales.at(i);
  }
  a.A = (int)A;
  a.log_std = flat.data_ptr<float>();
  a.x_stream = g_x_stream;
  return a;
}

// w8 (optional, fp8 mode with dt bf16): the e4m3 image the value head's fc1 reads with qscale
void set_w8(MlpArgs& a, torch::Tensor w8, torch::Tensor qscale, const Layout& L) {
  if (w8.defined() && w8.numel() > 0) {
    check(w8, "w8", at::kByte, wimg_extent(L));
    check(qscale, "qscale", at::kFloat, 6);
    a.W8 = w8.data_ptr();
    a.qscale = qscale.data_ptr<float>();
  }
}

void mlp_value(int64_t dt, torch::Tensor x_buf, torch::Tensor idx, int64_t row0, int64_t M, torch::Tensor wimg,
               std::vector<int64_t> layout, std::vector<double> scales, torch::Tensor flat, int64_t A,
               torch::Tensor v_out, bool check_idx, torch::Tensor qscale, torch::Tensor w8) {
  Layout L = parse_layout(layout);
  MlpArgs a = base_mlp((int)dt, L, scales, x_buf, idx, row0, M, wimg, flat, A, check_idx,
                       std::numeric_limits<int64_t>::max());
  check(v_out, "v_out", at::kFloat, M);
  a.v_out = v_out.data_ptr<float>();
  a.qscale = opt_scales(qscale);
  TORCH_CHECK(!(w8.defined() && w8.numel() > 0) || dt == 1, "w8: the fp8 mode's bf16 value forward only");
  set_w8(a, w8, qscale, L);
  launch_mlp_value((int)dt, a, cur_stream());
  after_launch(__func__);
}

void mlp_train(int64_t dt, torch::Tensor x_buf, torch::Tensor idx, int64_t row0, int64_t M, torch::Tensor wimg,
               std::vector<int64_t> layout, std::vector<double> scales, torch::Tensor flat, torch::Tensor log_std_old,
               int64_t A, torch::Tensor actions, torch::Tensor logp_old, torch::Tensor adv, torch::Tensor ret,
               torch::Tensor v_old, torch::Tensor mu_prev, torch::Tensor v_prev, std::vector<int64_t> opts,
               std::vector<double> fopts, std::vector<torch::Tensor> tbufs, int64_t ldT, torch::Tensor part,
               bool check_idx, bool xT_ready, torch::Tensor w8, torch::Tensor qscale, torch::Tensor q8_amax,
               int64_t q8_step) {
  TORCH_CHECK(dt != 2, "the fp8 mode's update runs in bf16 (its e4m3 parts: the value fc1 image w8 and the wgrad operands q8_amax)");
  Layout L = parse_layout(layout);
  TORCH_CHECK(A > 0, "A");
  check(actions, "actions", at::kFloat, A);
  const int64_t nrows = actions.numel() / A;
  MlpArgs a = base_mlp((int)dt, L, scales, x_buf, idx, row0, M, wimg, flat, A, check_idx, nrows);
  TORCH_CHECK(opts.size() == 5 || opts.size() == 7 || opts.size() == 8,
              "opts: loss_kind, value_loss, std_var, first_step, npart[, head, part_dw[, t32]]");
  // head >= 0: one head's per-head streaming kernel (csrc/mlp_head.hip; 0 policy, 1 value) with
  // its fused narrow-layer weight gradient at partial column part_dw (policy [32][128], value [128])
  const int head = opts.size() >= 7 ? (int)opts[5] : -1;
  const int part_dw = opts.size() >= 7 ? (int)opts[6] : 0;
  // t32: the policy head's transposed-chain 32x32 kernel (csrc/phead.hip): h1p / g1p / g2p and,
  // unless xT_ready, the observation rows into xT, ROW-MAJOR (the engine's wgrad reads them so: its
  // rm flags).  opts[7] == 1 also sums p_fc2's weight gradient in the kernel (no h1p / g2p), 2
  // stores h1p / g2p.  (The value head's update stays on the 16x16 kernel: docs/ARCHITECTURE.md §13.)
  const bool t32 = opts.size() == 8 && opts[7] != 0;
  const bool p2 = t32 && opts[7] == 1;
  TORCH_CHECK(head >= -1 && head <= 1, "head: -1 (both heads, one kernel), 0 policy, 1 value");
  TORCH_CHECK(fopts.size() == 2, "fopts: clip, ent_coeff");
  TORCH_CHECK(tbufs.size() == 11, "11 transposed buffers");
  check(logp_old, "logp_old", at::kFloat, nrows);
  check(adv, "adv", at::kFloat, nrows);
  check(ret, "ret", at::kFloat, nrows);
  check(v_old, "v_old", at::kFloat, nrows);
  check(mu_prev, "mu_prev", at::kFloat, nrows * A);
  check(v_prev, "v_prev", at::kFloat, nrows);
  check(log_std_old, "log_std_old", at::kFloat, A);
  if (head >= 0)
    TORCH_CHECK((dt == 3 || dt == 1) && mlp_head_applies(a), "the per-head kernels cover split-bf16 / bf16 and the reference network only");
  const int ROWS = head >= 0 ? mlp_head_rows() : mlp_train_rows((int)dt, a);
  TORCH_CHECK(head >= 0 || train_lds_bytes_impl((int)dt, L, A) <= 160 * 1024, "mlp_train tile does not fit LDS");
  const int64_t Mpad = ((M + ROWS - 1) / ROWS) * ROWS;
  TORCH_CHECK(ldT >= Mpad && ldT % 32 == 0, "ldT must cover M padded to the row tile and be a multiple of 32");
  // rows each transposed buffer must hold (writer side)
  const int64_t need[11] = {L.d_in[0], L.d_in[1], L.d_in[2], L.d_in[4], L.d_in[5],
                            L.n_out[0], L.n_out[1], L.n_out[2], L.n_out[3], L.n_out[4], L.n_out[5]};
  // q8_amax (fp8 mode, per-head bf16 update): the 3 x 4 slot ring of gradient maxima; the
  // operand buffers then hold e4m3 bytes (csrc/common.h Q8)
  const bool q8 = q8_amax.defined() && q8_amax.numel() > 0;
  if (q8) {
    TORCH_CHECK(dt == 1 && head >= 0, "e4m3 wgrad operands: the fp8 mode's per-head bf16 update only");
    check(q8_amax, "q8_amax", at::kInt, 3 * Q8_SLOT);
    unsigned* base = reinterpret_cast<unsigned*>(q8_amax.data_ptr<int>());
    const int64_t e = ((q8_step % 3) + 3) % 3;   // step -1: the calibration pass
    a.q8_acc = base + Q8_SLOT * e;
    a.q8_rd = base + Q8_SLOT * ((e + 2) % 3);
    a.q8_clr = base + Q8_SLOT * ((e + 1) % 3);
  }
  for (int i = 0; i < 11; ++i)
    check(tbufs[i], "transposed buffer", q8 ? at::kByte : storage_type((int)dt), need[i] * ldT);
  const int npart = (int)opts[4];
  TORCH_CHECK(npart >= 8 + A || (head == 1 && npart >= 8), "npart too small");
  if (head == 0) TORCH_CHECK(part_dw >= 8 + A && part_dw + 32 * 128 <= npart, "part_dw: policy dW_mu block");
  if (head == 1) TORCH_CHECK(part_dw >= 8 && part_dw + 128 <= npart, "part_dw: value dW_v block");
  a.part_dw = part_dw;
  const int nblk = (int)(Mpad / ROWS);
  check(part, "part", at::kFloat, (int64_t)nblk * npart);
  a.log_std_old = log_std_old.data_ptr<float>();
  a.actions = actions.data_ptr<float>();
  a.logp_old = logp_old.data_ptr<float>();
  a.adv = adv.data_ptr<float>();
  a.ret = ret.data_ptr<float>();
  a.v_old = v_old.data_ptr<float>();
  a.mu_prev = mu_prev.data_ptr<float>();
  a.v_prev = v_prev.data_ptr<float>();
  a.loss_kind = (int)opts[0];
  a.value_loss = (int)opts[1];
  a.std_var = (int)opts[2];
  a.first_step = (int)opts[3];
  a.npart = npart;
  a.clip = (float)fopts[0];
  a.ent_coeff = (float)fopts[1];
  void** dst[11] = {&a.xT, &a.h1pT, &a.h2pT, &a.h1vT, &a.h2vT, &a.g1pT, &a.g2pT, &a.g3pT, &a.g1vT, &a.g2vT, &a.g3vT};
  for (int i = 0; i < 11; ++i) *dst[i] = tbufs[i].data_ptr();
  a.ldT = (int)ldT;
  // a precomputed xT is only valid for the identity row order covering the whole buffer
  // (t32 policy: x_buf itself is the wgrad's X operand then, so only the row order matters)
  TORCH_CHECK(!xT_ready || (a.idx == nullptr && row0 == 0 && (ldT == M || (t32 && head == 0))),
              "xT_ready needs a full-batch call");
  a.xT_ready = xT_ready ? 1 : 0;
  if (g_tstamp != nullptr) {
    // (the 32x32 policy head takes no stamps)
    const int64_t nw = head >= 0 ? mlp_head_waves(head) : mlp_train_waves((int)dt, a);
    TORCH_CHECK(g_tstamp_numel >= ((nblk + g_tstamp_every - 1) / g_tstamp_every) * nw * 16, "tstamp buffer too small");
    a.tstamp = g_tstamp;
    a.tstamp_every = g_tstamp_every;
  }
  a.part = part.data_ptr<float>();
  TORCH_CHECK(!(w8.defined() && w8.numel() > 0) || (dt == 1 && head >= 0), "w8: the fp8 mode's per-head bf16 update only");
  set_w8(a, w8, qscale, L);
  if (t32) {   // the row-major operand rows the kernels write are whole padded widths
    const int64_t pn = !p2 ? 128 : 0;   // h1p / g2p
    const int64_t wid[11] = {!xT_ready ? L.d_in[0] : 0, pn, 0, 0, 0, 128, pn, 0, 0, 0, 0};
    for (int i = 0; i < 11; ++i)
      TORCH_CHECK(tbufs[i].numel() >= wid[i] * ldT, "t32 head: row-major operand buffer ", i, " too small");
  }
  if (t32) {
    TORCH_CHECK(head == 0 && !q8 && a.W8 == nullptr && phead_shape_ok(a), "phead: the policy head at bf16x3 / bf16");
    TORCH_CHECK(part_dw + 32 * 128 + (p2 ? 128 * 128 : 0) <= npart,
                "phead: the dW_mu (and dW_p2) blocks must fit the partial row");
    const int64_t eb = dt == 3 ? 4 : 2;
    TORCH_CHECK(ldT * std::max<int64_t>(L.d_in[0], 128) * eb < (int64_t(1) << 31), "phead: row-major operands beyond 2 GiB");
    TORCH_CHECK((int64_t)nblk * npart * 4 < (int64_t(1) << 31), "phead: partial buffer beyond 2 GiB");
    TORCH_CHECK(ldT % phead_rows() == 0 && Mpad <= ldT && (L.d_in[0] >> 4) / (dt == 3 ? 1 : 2) >= 3,
                "phead: ldT covers whole workgroups; fc1 has >= 3 stages");
    launch_phead_train((int)dt, a, p2 ? 1 : 0, cur_stream());
  } else if (head >= 0) {
    launch_mlp_head((int)dt, (int)head, a, cur_stream());
  } else {
    launch_mlp_train((int)dt, a, cur_stream());
  }
  after_launch(__func__);
}

// the transposed-chain policy head covers this (dtype, network, action width)
bool phead_train_applies(int64_t dt, std::vector<int64_t> layout, int64_t A) {
  const Layout L = parse_layout(layout);
  MlpArgs a{};
  for (int i = 0; i < 6; ++i) { a.d_in[i] = L.d_in[i]; a.d_out[i] = L.d_out[i]; a.n_out[i] = L.n_out[i]; }
  a.A = (int)A;
  return (dt == 3 || dt == 1) && phead_shape_ok(a) != 0 && (L.d_in[0] >> 4) / (dt == 3 ? 1 : 2) >= 3;
}

// the per-head kernels cover this (dtype, network); x_bytes is irrelevant to them (64-bit rows)
bool head_applies(int64_t dt, std::vector<int64_t> layout, int64_t A) {
  const Layout L = parse_layout(layout);
  MlpArgs a{};
  for (int i = 0; i < 6; ++i) { a.d_in[i] = L.d_in[i]; a.d_out[i] = L.d_out[i]; a.n_out[i] = L.n_out[i]; }
  a.A = (int)A;
  return (dt == 3 || dt == 1) && mlp_head_applies(a) != 0;
}

int64_t train_lds_bytes(int64_t dt, std::vector<int64_t> layout, int64_t A) {
  return train_lds_bytes_impl((int)dt, parse_layout(layout), A);
}

int64_t train_rows(int64_t dt, std::vector<int64_t> layout, int64_t A, int64_t x_bytes) {
  const Layout L = parse_layout(layout);
  MlpArgs a{};
  for (int i = 0; i < 6; ++i) { a.d_in[i] = L.d_in[i]; a.d_out[i] = L.d_out[i]; a.n_out[i] = L.n_out[i]; }
  a.A = (int)A;
  a.x_bytes = x_bytes;
  return mlp_train_rows((int)dt, a);
}

int64_t train_waves(int64_t dt, std::vector<int64_t> layout, int64_t A) {
  const Layout L = parse_layout(layout);
  MlpArgs a{};
  for (int i = 0; i < 6; ++i) { a.d_in[i] = L.d_in[i]; a.d_out[i] = L.d_out[i]; a.n_out[i] = L.n_out[i]; }
  a.A = (int)A;
  return mlp_train_waves((int)dt, a);
}

void set_mlp_rows(int64_t rows) {
  TORCH_CHECK(rows == 0 || rows == 16 || rows == 32 || rows == 64, "rows: 0 (auto), 16, 32 or 64");
  set_mlp_rows_override((int)rows);
}

// dt 2 (fp8 mode): e4m3 operands; q8_amax / q8_step name the slot the update read its gradient
// scales from, q8_t the gradient tensor of each layer (-1: none), q8_xs the activation scales
F8Shadow f8_shadow(torch::Tensor img, torch::Tensor lid, torch::Tensor qs, int64_t n);

WgradArgs wgrad_args(int64_t dt, std::vector<torch::Tensor> gT, std::vector<torch::Tensor> xT,
                     std::vector<int64_t> g_rows, std::vector<int64_t> x_rows, int64_t ld, torch::Tensor tasks,
                     torch::Tensor tasks_host, torch::Tensor slab, torch::Tensor q8_amax, int64_t q8_step,
                     std::vector<int64_t> q8_t, std::vector<double> q8_xs, std::vector<int64_t> rm) {
  TORCH_CHECK(gT.size() == 6 && xT.size() == 6 && g_rows.size() == 6 && x_rows.size() == 6, "6 layers");
  check(tasks, "tasks", at::kInt, WGRAD_TASK_INTS);
  TORCH_CHECK(tasks.numel() % WGRAD_TASK_INTS == 0, "tasks are 8-int records");
  TORCH_CHECK(!tasks_host.is_cuda() && tasks_host.numel() == tasks.numel(), "tasks_host must mirror tasks on CPU");
  const int ntasks = (int)(tasks.numel() / WGRAD_TASK_INTS);
  auto th = tasks_host.contiguous();
  const int* tp = th.data_ptr<int>();
  int64_t slab_need = 0;
  bool wide = false;
  for (int i = 0; i < ntasks; ++i) {
    const int* t = tp + WGRAD_TASK_INTS * i;
    TORCH_CHECK(t[0] >= 0 && t[0] < 6, "task layer");
    const int nq = t[6], kq = t[7];
    TORCH_CHECK(wgrad_task_ok((int)dt, nq, kq), "task quadrants beyond the workgroup (wgrad_task_ok)");
    wide = wide || nq * kq > 8;
    TORCH_CHECK(t[1] >= 0 && t[2] >= 0 && t[1] % 16 == 0 && t[2] % 16 == 0, "task tile origin");
    TORCH_CHECK(t[1] + 64 * nq <= g_rows[t[0]] && t[2] + 64 * kq <= x_rows[t[0]], "task tile beyond operand rows");
    // the kernel consumes 32-row k-steps in pairs (e4m3: in fours): every range is a positive
    // multiple of 64 (128) rows
    const int kq_rows = dt == 2 ? 128 : 64;
    TORCH_CHECK(t[3] >= 0 && t[4] <= ld && t[4] > t[3] && (t[4] - t[3]) % kq_rows == 0 && t[3] % 32 == 0,
                "task batch range (must be a positive multiple of 64 rows, 128 for e4m3)");
    TORCH_CHECK(t[5] >= 0, "task slab offset");
    slab_need = std::max<int64_t>(slab_need, (int64_t)t[5] + (int64_t)(64 * nq) * (64 * kq));
  }
  check(slab, "slab", at::kFloat, slab_need);
  WgradArgs a{};
  for (int i = 0; i < 6; ++i) {
    check(gT[i], "gT", storage_type((int)dt), g_rows[i] * ld);
    check(xT[i], "xT", storage_type((int)dt), x_rows[i] * ld);
    a.gT[i] = gT[i].data_ptr();
    a.xT[i] = xT[i].data_ptr();
  }
  a.ld = (int)ld;
  // rm: 12 flags (dY side of layers 0-5, then X side): 1 = row-major operands of row length g_rows /
  // x_rows (csrc/phead.hip, x_buf); split-bf16 / bf16 only, 64-feature quadrants inside the row
  TORCH_CHECK(rm.empty() || rm.size() == 12, "rm: 12 row-major flags");
  for (size_t i = 0; i < rm.size(); ++i) {
    if (!rm[i]) continue;
    TORCH_CHECK(dt == 1 || dt == 3, "row-major wgrad operands: split-bf16 / bf16 only");
    TORCH_CHECK(rm[i] == 1, "rm flag: 0 fragment-major, 1 row-major");
    const int64_t len = i < 6 ? g_rows[i] : x_rows[i - 6];
    TORCH_CHECK(len % 64 == 0 && ld * len * (dt == 3 ? 4 : 2) < (int64_t(1) << 40), "row-major operand rows");
    (i < 6 ? a.g_rm[i] : a.x_rm[i - 6]) = (int)len;
  }
  a.wide = wide ? 1 : 0;
  a.tasks = reinterpret_cast<const WgradTask*>(tasks.data_ptr<int>());
  a.ntasks = ntasks;
  a.slab = slab.data_ptr<float>();
  TORCH_CHECK(dt == 0 || dt == 1 || dt == 2 || dt == 3, "wgrad runs in fp32, bf16, e4m3 or bf16x3");
  if (dt == 2) {
    check(q8_amax, "q8_amax", at::kInt, 3 * Q8_SLOT);
    TORCH_CHECK(q8_t.size() == 6 && q8_xs.size() == 6, "q8_t / q8_xs: one per layer");
    const int64_t e = ((q8_step % 3) + 3) % 3;
    a.q8_rd = reinterpret_cast<const unsigned*>(q8_amax.data_ptr<int>()) + Q8_SLOT * ((e + 2) % 3);
    for (int i = 0; i < ntasks; ++i) {
      const int l = tp[WGRAD_TASK_INTS * i];
      TORCH_CHECK(q8_t[l] >= 0 && q8_t[l] < 4 && q8_xs[l] > 0, "e4m3 wgrad task on a layer without operand scales");
    }
    for (int i = 0; i < 6; ++i) { a.q8_t[i] = (int)q8_t[i]; a.q8_xs[i] = (float)q8_xs[i]; }
  }
  return a;
}

void wgrad(int64_t dt, std::vector<torch::Tensor> gT, std::vector<torch::Tensor> xT, std::vector<int64_t> g_rows,
           std::vector<int64_t> x_rows, int64_t ld, torch::Tensor tasks, torch::Tensor tasks_host, torch::Tensor slab,
           torch::Tensor q8_amax, int64_t q8_step, std::vector<int64_t> q8_t, std::vector<double> q8_xs,
           std::vector<int64_t> rm) {
  const WgradArgs a = wgrad_args(dt, gT, xT, g_rows, x_rows, ld, tasks, tasks_host, slab, q8_amax, q8_step, q8_t, q8_xs, rm);
  launch_wgrad((int)dt, a, cur_stream());
  after_launch(__func__);
}

// The gradient of one flat range: slab elements [i_lo, i_hi) (src_meta != 0) as split-K slab
// sums, and the reduce items (red_col / red_dst: the partial-row column of each, and its flat
// index in `grad` or -1 - q for loss_out[q]) as column sums of the per-workgroup partial rows.
// grad / src_off / src_meta may be one head's slice of the flat vectors; red_dst then indexes
// the slice.  The item tables are validated on the host when the engine builds them
// (HipEngine._reduce_items): no per-epoch device sync here.
// the slab runs of a gather: flattened [lo0, hi0, lo1, hi1, ...] (<= 4, ascending, disjoint, inside
// [0, n)); every element of a run must have a slab source (src_meta != 0: the engine asserts it
// when it builds the plan, runtime/engine_hip.py _slab_runs)
SlabRuns make_runs(const std::vector<int64_t>& v, int64_t n) {
  TORCH_CHECK(v.size() % 2 == 0 && v.size() / 2 >= 1 && v.size() / 2 <= 4, "slab runs: 1-4 [lo, hi) pairs");
  SlabRuns r{};
  r.n = (int)(v.size() / 2);
  int64_t total = 0, prev = 0;
  for (int k = 0; k < 4; ++k) {
    if (k < r.n) {
      const int64_t lo = v[2 * k], hi = v[2 * k + 1];
      TORCH_CHECK(prev <= lo && lo <= hi && hi <= n, "slab runs must be ascending, disjoint and inside [0, n)");
      r.lo[k] = (int)lo;
      r.start[k] = (int)total;
      total += hi - lo;
      prev = hi;
    } else {
      r.lo[k] = 0;
      r.start[k] = INT32_MAX;
    }
  }
  r.total = (int)total;
  return r;
}

void grad_gather(torch::Tensor slab, torch::Tensor src_off, torch::Tensor src_meta, torch::Tensor part,
                 int64_t nblk, int64_t npart, torch::Tensor red_col, torch::Tensor red_dst, double scale,
                 torch::Tensor grad, torch::Tensor loss_out, std::vector<int64_t> runs) {
  const int64_t n = grad.numel();
  const SlabRuns sr = make_runs(runs, n);
  check(grad, "grad", at::kFloat, n);
  check(src_off, "src_off", at::kInt, n);
  check(src_meta, "src_meta", at::kInt, n);
  check(slab, "slab", at::kFloat, 1);
  check(part, "part", at::kFloat, nblk * npart);
  check(loss_out, "loss_out", at::kFloat, 8);
  const int64_t nitems = red_col.numel();
  check(red_col, "red_col", at::kInt, nitems);
  check(red_dst, "red_dst", at::kInt, nitems);
  TORCH_CHECK(red_dst.numel() == nitems, "red_col / red_dst sizes");
  launch_grad_gather(slab.data_ptr<float>(), src_off.data_ptr<int>(), src_meta.data_ptr<int>(),
                     part.data_ptr<float>(), (int)nblk, (int)npart, red_col.data_ptr<int>(), red_dst.data_ptr<int>(),
                     (int)nitems, (float)scale, grad.data_ptr<float>(), sr, loss_out.data_ptr<float>(), cur_stream());
  after_launch(__func__);
}

void obs_reduce(torch::Tensor part, int64_t nblk, int64_t O, torch::Tensor s12, torch::Tensor epstat,
                torch::Tensor ep) {
  check(part, "part", at::kFloat, nblk * 2 * O);
  check(s12, "s12", at::kDouble, 2 * O);
  check(epstat, "epstat", at::kFloat, nblk * 2);
  check(ep, "ep", at::kDouble, 2);
  launch_obs_reduce(part.data_ptr<float>(), (int)nblk, (int)O, s12.data_ptr<double>(), epstat.data_ptr<float>(),
                    ep.data_ptr<double>(), cur_stream());
  after_launch(__func__);
}

// the per-step obs-norm mode's observe (model.py:68 over one step's E observations): moments about
// shift -> fixed-order fp64 reduce -> Chan merge into (mean, m2) and the fp32 images; three
// launches, no host sync (n_a: the stats' count before this batch, tracked on the host)
void obs_observe(torch::Tensor obs, torch::Tensor shift, torch::Tensor mean, torch::Tensor m2, torch::Tensor mean_f32,
                 torch::Tensor inv_std, double n_a, torch::Tensor part, torch::Tensor s12, double var_floor) {
  const int64_t O = mean.numel();
  TORCH_CHECK(obs.dim() == 2 && obs.size(1) == O && obs.size(0) > 0, "obs must be [E][O]");
  const int E = (int)obs.size(0);
  const int nblk = obs_moments_blocks(E);
  check(obs, "obs", at::kFloat, (int64_t)E * O);
  check(shift, "shift", at::kFloat, O);
  check(part, "part", at::kFloat, (int64_t)nblk * 2 * O);
  check(s12, "s12", at::kDouble, 2 * O);
  check(mean, "mean", at::kDouble, O);
  check(m2, "m2", at::kDouble, O);
  check(mean_f32, "mean_f32", at::kFloat, O);
  check(inv_std, "inv_std", at::kFloat, O);
  TORCH_CHECK(shift.data_ptr() != mean_f32.data_ptr(), "shift must be a snapshot, not the stats' own mean image");
  const hipStream_t s = cur_stream();
  launch_obs_moments(obs.data_ptr<float>(), E, (int)O, shift.data_ptr<float>(), part.data_ptr<float>(), s);
  launch_obs_reduce(part.data_ptr<float>(), nblk, (int)O, s12.data_ptr<double>(), nullptr, nullptr, s);
  launch_obs_merge(s12.data_ptr<double>(), (int)O, (double)E, n_a, shift.data_ptr<float>(), mean.data_ptr<double>(),
                   m2.data_ptr<double>(), mean_f32.data_ptr<float>(), inv_std.data_ptr<float>(), var_floor, s);
  after_launch(__func__);
}

int64_t obs_moments_nblk(int64_t E) { return obs_moments_blocks((int)E); }

void obs_merge(torch::Tensor s12, double count, double n_a, torch::Tensor shift, torch::Tensor mean, torch::Tensor m2,
               torch::Tensor mean_f32, torch::Tensor inv_std, double var_floor) {
  const int64_t O = mean.numel();
  TORCH_CHECK(count > 0, "count must be positive");
  check(s12, "s12", at::kDouble, 2 * O);
  check(shift, "shift", at::kFloat, O);
  check(mean, "mean", at::kDouble, O);
  check(m2, "m2", at::kDouble, O);
  check(mean_f32, "mean_f32", at::kFloat, O);
  check(inv_std, "inv_std", at::kFloat, O);
  launch_obs_merge(s12.data_ptr<double>(), (int)O, count, n_a, shift.data_ptr<float>(), mean.data_ptr<double>(),
                   m2.data_ptr<double>(), mean_f32.data_ptr<float>(), inv_std.data_ptr<float>(), var_floor,
                   cur_stream());
  after_launch(__func__);
}

void gae(torch::Tensor rewards, torch::Tensor values, torch::Tensor dones, torch::Tensor adv, torch::Tensor ret,
         double gamma, double lam, int64_t mode, int64_t seg) {
  TORCH_CHECK(seg >= 0, "segment length must be >= 0 (0: no segment cut)");
  TORCH_CHECK(rewards.dim() == 2, "rewards [T,E]");
  TORCH_CHECK(mode >= 0 && mode <= 2, "gae mode: 0 auto, 1 per-env lanes, 2 parallel-in-time scan");
  const int64_t T = rewards.size(0), E = rewards.size(1);
  check(rewards, "rewards", at::kFloat, T * E);
  check(values, "values", at::kFloat, (T + 1) * E);
  check(dones, "dones", at::kFloat, T * E);
  check(adv, "adv", at::kFloat, T * E);
  check(ret, "ret", at::kFloat, T * E);
  launch_gae(rewards.data_ptr<float>(), values.data_ptr<float>(), dones.data_ptr<float>(), adv.data_ptr<float>(),
             ret.data_ptr<float>(), (int)T, (int)E, (float)gamma, (float)lam, (int)mode, (int)seg, cur_stream());
  after_launch(__func__);
}

void metrics_pack(torch::Tensor ep, torch::Tensor loss8, torch::Tensor norm_part, torch::Tensor out) {
  check(ep, "ep", at::kDouble, 2);
  check(loss8, "loss8", at::kFloat, 8);
  check(norm_part, "norm_part", at::kFloat, 1);
  check(out, "out", at::kDouble, 11);
  launch_metrics_pack(ep.data_ptr<double>(), loss8.data_ptr<float>(), norm_part.data_ptr<float>(),
                      (int)norm_part.numel(), out.data_ptr<double>(), cur_stream());
  after_launch(__func__);
}

// diagnostics (scripts/probe_side_kernel.py): an RCCL-footprint stand-in on the current stream
void probe_spin(int64_t nblk, int64_t nthreads, int64_t lds, double us, torch::Tensor sink) {
  TORCH_CHECK(nblk >= 1 && nblk <= 4096 && nthreads >= 64 && nthreads <= 1024 && nthreads % 64 == 0 && lds >= 0 &&
                  lds <= 65536 && lds >= 4 * nthreads && us > 0 && us < 1e5,
              "probe_spin: 1-4096 blocks of 64-1024 threads, 4 * threads <= lds <= 64 KiB, 0 < us < 1e5");
  check(sink, "sink", at::kInt, nblk);
  launch_probe_spin((int)nblk, (int)nthreads, (int)lds, us, sink.data_ptr<int>(), cur_stream());
  after_launch(__func__);
}

// fp8 mode's shadow image (csrc/kernels.h F8Shadow): empty tensors = off
F8Shadow f8_shadow(torch::Tensor img, torch::Tensor lid, torch::Tensor qs, int64_t n) {
  F8Shadow f{nullptr, nullptr, nullptr};
  if (img.defined() && img.numel() > 0) {
    check(img, "f8_img", at::kByte, 1);
    check(lid, "f8_lid", at::kInt, n);
    check(qs, "f8_qscale", at::kFloat, 6);
    f.img = img.data_ptr<uint8_t>();
    f.lid = lid.data_ptr<int>();
    f.qs = qs.data_ptr<float>();
  }
  return f;
}

void adam(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, double lr, double b1, double b2,
          double eps, double max_norm, torch::Tensor state, torch::Tensor norm_part, torch::Tensor wimg,
          torch::Tensor w_map, torch::Tensor wt_map, int64_t dt, torch::Tensor qmul, int64_t host_step,
          torch::Tensor f8_img, torch::Tensor f8_lid, torch::Tensor f8_qs) {
  // host_step >= 1: the step number of this update (eager launch: one fused kernel when there is
  // no clipping); 0: read the device counter (graph replay)
  const int64_t n = p.numel();
  check(p, "p", at::kFloat, n);
  check(g, "g", at::kFloat, n);
  check(m, "m", at::kFloat, n);
  check(v, "v", at::kFloat, n);
  check(state, "state", at::kFloat, 4);
  check(w_map, "w_map", at::kInt, n);
  check(wt_map, "wt_map", at::kInt, n);
  check(wimg, "wimg", storage_type((int)dt), 1);
  const int nblk = (int)norm_part.numel();
  check(norm_part, "norm_part", at::kFloat, nblk);
  TORCH_CHECK(nblk >= 1 && nblk <= 4096, "norm_part size");
  const float* q = nullptr;
  if (qmul.defined() && qmul.numel() > 0) { check(qmul, "qmul", at::kFloat, n); q = qmul.data_ptr<float>(); }
  launch_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), (int)n, (float)lr,
              (float)b1, (float)b2, (float)eps, (float)max_norm, state.data_ptr<float>(), norm_part.data_ptr<float>(),
              nblk, wimg.data_ptr(), w_map.data_ptr<int>(), wt_map.data_ptr<int>(), (int)dt, q, (int)host_step,
              f8_shadow(f8_img, f8_lid, f8_qs, n), cur_stream());
  after_launch(__func__);
}

// grad_gather (reduce items + slab elements of [i_lo, n)) and the no-clip Adam step in one
// launch (world size 1: nothing runs between them).  Bit-identical parameters to grad_gather ->
// adam(host_step).  The flat tensors may be one head's slice (red_dst indexes the slice).
void gather_adam(torch::Tensor slab, torch::Tensor src_off, torch::Tensor src_meta, torch::Tensor part,
                 int64_t npblk, int64_t npart, torch::Tensor red_col, torch::Tensor red_dst, std::vector<int64_t> runs,
                 double scale, torch::Tensor loss_out, torch::Tensor g, torch::Tensor p, torch::Tensor m,
                 torch::Tensor v, double lr, double b1, double b2, double eps, int64_t step, torch::Tensor state,
                 torch::Tensor norm_part, torch::Tensor wimg, torch::Tensor w_map, torch::Tensor wt_map, int64_t dt,
                 torch::Tensor qmul, torch::Tensor f8_img, torch::Tensor f8_lid, torch::Tensor f8_qs) {
  const int64_t n = p.numel();
  check(p, "p", at::kFloat, n);
  check(g, "g", at::kFloat, n);
  check(m, "m", at::kFloat, n);
  check(v, "v", at::kFloat, n);
  check(src_off, "src_off", at::kInt, n);
  check(src_meta, "src_meta", at::kInt, n);
  check(slab, "slab", at::kFloat, 1);
  check(part, "part", at::kFloat, npblk * npart);
  check(loss_out, "loss_out", at::kFloat, 8);
  check(state, "state", at::kFloat, 4);
  check(w_map, "w_map", at::kInt, n);
  check(wt_map, "wt_map", at::kInt, n);
  check(wimg, "wimg", storage_type((int)dt), 1);
  const int64_t nitems = red_col.numel();
  check(red_col, "red_col", at::kInt, nitems);
  check(red_dst, "red_dst", at::kInt, nitems);
  TORCH_CHECK(red_dst.numel() == nitems, "red_col / red_dst");
  const SlabRuns sr = make_runs(runs, n);
  TORCH_CHECK(step >= 1, "gather_adam needs the host step number (eager launches only)");
  const int nblk = (int)norm_part.numel();
  check(norm_part, "norm_part", at::kFloat, nblk);
  TORCH_CHECK(nblk > item_blocks((int)nitems) && nblk <= 4096, "norm_part must hold more blocks than the reduce blocks");
  const float* q = nullptr;
  if (qmul.defined() && qmul.numel() > 0) { check(qmul, "qmul", at::kFloat, n); q = qmul.data_ptr<float>(); }
  launch_gather_adam(slab.data_ptr<float>(), src_off.data_ptr<int>(), src_meta.data_ptr<int>(),
                     part.data_ptr<float>(), (int)npblk, (int)npart, red_col.data_ptr<int>(), red_dst.data_ptr<int>(),
                     (int)nitems, sr, (float)scale, loss_out.data_ptr<float>(), g.data_ptr<float>(),
                     p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), (int)n, (float)lr, (float)b1,
                     (float)b2, (float)eps, (int)step, state.data_ptr<float>(), norm_part.data_ptr<float>(), nblk,
                     wimg.data_ptr(), w_map.data_ptr<int>(), wt_map.data_ptr<int>(), (int)dt, q,
                     f8_shadow(f8_img, f8_lid, f8_qs, n), cur_stream());
  after_launch(__func__);
}

void fp8_refresh(torch::Tensor p, torch::Tensor lid, torch::Tensor qscale, torch::Tensor part, torch::Tensor wimg,
                 torch::Tensor w_map, torch::Tensor wt_map) {
  check(part, "part", at::kFloat, 128 * 6);
  const int64_t n = p.numel();
  check(p, "p", at::kFloat, n);
  check(lid, "lid", at::kInt, n);
  check(qscale, "qscale", at::kFloat, 6);
  check(w_map, "w_map", at::kInt, n);
  check(wt_map, "wt_map", at::kInt, n);
  check(wimg, "wimg", at::kByte, 1);
  // lid must name a layer in [0, 6) for every parameter with an image entry (the kernel's scale
  // index): HipEngine validates the static map once at construction (no per-call device sync)
  launch_fp8_refresh(p.data_ptr<float>(), lid.data_ptr<int>(), (int)n, qscale.data_ptr<float>(), part.data_ptr<float>(),
                     wimg.data_ptr(), w_map.data_ptr<int>(), wt_map.data_ptr<int>(), cur_stream());
  after_launch(__func__);
}

void debug_invalid_launch() {
  launch_debug_invalid(nullptr, cur_stream());
  after_launch(__func__);
}

void pack(torch::Tensor p, torch::Tensor wimg, torch::Tensor w_map, torch::Tensor wt_map, int64_t dt, torch::Tensor qmul) {
  const int64_t n = p.numel();
  check(p, "p", at::kFloat, n);
  check(w_map, "w_map", at::kInt, n);
  check(wt_map, "wt_map", at::kInt, n);
  check(wimg, "wimg", storage_type((int)dt), 1);
  const float* q = nullptr;
  if (qmul.defined() && qmul.numel() > 0) { check(qmul, "qmul", at::kFloat, n); q = qmul.data_ptr<float>(); }
  launch_pack(p.data_ptr<float>(), (int)n, wimg.data_ptr(), w_map.data_ptr<int>(), wt_map.data_ptr<int>(), (int)dt, q,
              cur_stream());
  after_launch(__func__);
}

}  // namespace

void register_comm(pybind11::module& m);   // csrc/comm.cpp: native RCCL communicator

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native DPPO kernels (gfx950 HIP)";
  register_comm(m);
  m.def("rollout", &rollout);
  m.def("rollout_stepnorm", &rollout_stepnorm);
  m.def("rollout_stepnorm_cap", &rollout_stepnorm_cap_b);
  m.def("mlp_value", &mlp_value);
  m.def("mlp_train", &mlp_train);
  m.def("head_applies", &head_applies);
  m.def("phead_train_applies", &phead_train_applies);
  m.def("set_phead", [](int64_t on) { set_phead((int)on); });
  m.def("head_rows", []() { return (int64_t)mlp_head_rows(); });
  m.def("head_waves", [](int64_t h) { return (int64_t)mlp_head_waves((int)h); });
  m.def("set_head_kernels", [](bool on) { set_head_kernels(on ? 1 : 0); });
  m.def("head_kernels_enabled", []() { return head_kernels_enabled() != 0; });
  m.def("train_lds_bytes", &train_lds_bytes);
  m.def("train_rows", &train_rows);
  m.def("train_waves", &train_waves);
  m.def("set_mlp_rows", &set_mlp_rows);
  m.def("set_s3_value_waves", [](int64_t nw) {
    TORCH_CHECK(nw == 4 || nw == 8, "split-bf16 value waves: 4 or 8");
    set_s3_value_waves((int)nw);
  });
  m.def("set_s3_train_waves", [](int64_t nw) {
    TORCH_CHECK(nw == 4 || nw == 8, "split-bf16 train waves: 4 or 8");
    set_s3_train_waves((int)nw);
  });
  m.def("set_debug_sync", &set_debug_sync);
  m.def("set_rollout_waves", [](int64_t nw) {
    TORCH_CHECK(nw == 4 || nw == 8, "rollout waves: 4 or 8");
    set_rollout_waves((int)nw);
  });
  m.def("set_train_tstamp", &set_train_tstamp);
  m.def("set_rollout_tstamp", &set_rollout_tstamp);
  m.def("wgrad", &wgrad);
  m.def("wgrad_task_ok", [](int64_t dt, int64_t nq, int64_t kq) { return wgrad_task_ok((int)dt, (int)nq, (int)kq) != 0; });
  m.def("grad_gather", &grad_gather);
  m.def("gae", &gae);
  m.def("set_adam_fused", [](int64_t on) { set_adam_fused((int)on); });
  m.def("obs_reduce", &obs_reduce);
  m.def("obs_merge", &obs_merge);
  m.def("obs_observe", &obs_observe);
  m.def("obs_moments_nblk", &obs_moments_nblk);
  m.def("adam", &adam);
  m.def("gather_adam", &gather_adam);
  m.def("pack", &pack);
  m.def("debug_invalid_launch", &debug_invalid_launch);
  m.def("fp8_refresh", &fp8_refresh);
  m.def("set_x_stream", &set_x_stream);
  m.def("metrics_pack", &metrics_pack);
  m.def("probe_spin", &probe_spin);
  m.attr("arch") = "gfx950";
}
