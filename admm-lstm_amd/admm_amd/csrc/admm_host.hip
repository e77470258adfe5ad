// admm_host.hip -- context, step orchestration and the C ABI of libadmmlstm.so
// (include/admm_lstm.h).  Everything is enqueued on the caller's stream; no host sync
// except admm_get_stats.  Multi-GPU: one process per GPU, the batch sums of the step are
// all-reduced with RCCL (the only cross-sample couplings of the reference).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "admm_kernels.hpp"
#include "admm_lstm.h"

using namespace admm;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                             \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(ADMM_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define NCCL_TRY(expr)                                                                              \
  do {                                                                                              \
    ncclResult_t r_ = (expr);                                                                       \
    if (r_ != ncclSuccess) return fail(ADMM_ECOMM, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

// Sets the context's device for the duration of one C-ABI call and restores the caller's
// current device on return, so torch's current device is not moved by the library.
struct DeviceGuard {
  int prev = -1;
  hipError_t err;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = prev == dev ? hipSuccess : hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

#define DEVICE_GUARD(dev)                                                                          \
  DeviceGuard dg_(dev);                                                                            \
  if (dg_.err != hipSuccess) return fail(ADMM_EHIP, "hipSetDevice(%d) failed: %s", (int)(dev), hipGetErrorString(dg_.err))

template <typename T>
int dalloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e != hipSuccess) return fail(ADMM_ENOMEM, "hipMalloc(%zu bytes) failed: %s", n * sizeof(T), hipGetErrorString(e));
  return ADMM_OK;
}

}  // namespace

constexpr int kMaxSweepStreams = 4;

struct StepSig {   // admm_step's launch-sequence signature (see step_sig)
  uint32_t flags;
  AdmmBuffers buf;
  float* trace[4];
  void* comm;
};
constexpr int kMaxOutputs = 4096;

constexpr int kSweepFallbackLimit = 3;   // AdmmCtx::cs_off

struct AdmmCtx {
  Geom g{};
  Hyper hp{};
  int device = 0;
  AdmmBuffers buf{};
  bool bound = false;
  bool z_valid = false;
  bool force_generic = false;  // weight stages on the generic kernels (ADMM_GENERIC=1; tests)
  bool tgt_valid = false;  // tgt holds lam/rho + S of the current state (left by the persistent sweep)
  // the persistent sweep writes tgt for the next x stage, which then reads it instead of
  // recomputing it from the gate and dual planes (ADMM_TGT_SWEEP=0 disables)
  bool tgt_sweep = true;
  // ... and the next x stage's X^T R partials (k_sweep_rows GX, D <= 16), so that stage skips
  // k_resid_gx (ADMM_GX_SWEEP=0 disables)
  bool gx_sweep = true;
  // dual h before T: zero unless written from outside (the library ascends it only at T);
  // lamh_known says whether lamh_nz (device) describes the bound plane
  int* lamh_nz = nullptr;
  bool lamh_known = false;
  bool lamh_skip = true;   // ADMM_LAMH_SKIP=0: always load it
  bool gx_valid = false;
  float* gx_slab = nullptr;   // [sweep blocks][4][D][H]
  int gx_nblk = 0;
  int steps = 0;
  // workspace (all device)
  float *zc = nullptr, *tgt = nullptr, *R = nullptr, *Q = nullptr;  // [4][BT][H]
  // speculative x-stage z update (SpecX, H % 256 == 0 fast path; ADMM_SPEC_X=0 disables):
  // zx = zc + x dWx is written by pass 0 of the x trials for the predicted exponent
  bool spec_x = false;
  float* zx = nullptr;   // [4][BT][H], the h stage's z
  int* kpred = nullptr;
  float *G = nullptr, *dW = nullptr, *gslab = nullptr;
  double *tr_part = nullptr, *tr_sums = nullptr, *tr_poly = nullptr;
  int nblk_resid = 1, nblk_trial = 1, nblk_rx = 1;
  int* found = nullptr;
  int* pick = nullptr;
  int sweep_split = 2;     // sample parts of the per-t sweep, one stream each
  bool sweep_rows = false; // whole sweep as one persistent launch (k_sweep_rows; ADMM_SWEEP_ROWS=0 disables)
  float* swt = nullptr;    // its B-operand image of the weights
  // the image's zero padding (x rows D .. 16 XC) is written once by k_sweep_wt; after that the
  // weight selections keep every weight element's pieces current (SelectArgs::wt)
  bool wt_init = false;
  bool split3 = false;     // h-stage GEMMs on split bf16 MFMAs (admm_split3.hip; ADMM_SPLIT3=0 disables)
  // the h-side gradient G_h = rho Hprev^T R (k_atr3w) on split3's six products, f32-accurate
  // (tests/test_gpu_weight_phase.py: within the error of an fp32 GEMM of the same operands) ...
  // ... unless the operand ranges are known: the h-side gradient then runs on scaled fp16 two-way
  // splits (k_atr3w<2, true>: f32-accurate at the matrix work of two pieces; ADMM_ATR_F16=0: off).
  // range [8] (device): SweepT::range's maxima from the last persistent sweep ([0..4], valid when
  // range_valid) and max_row sum_d |x_d| ([5], valid when x1_valid)
  bool atr_f16 = true;
  bool atr_wide = true;    // ... and at H = 512 in 512 x 128 tiles (ADMM_ATR_WIDE=0: 256 x 256)
  float* range = nullptr;
  bool range_valid = false, x1_valid = false;
  // column-split sweep (strong-scaling ranks, sweep_rows_nc > 1): the h_t hand-off granules
  float* xbuf = nullptr;
  bool cs_poison = false;   // test hook (ADMM_SWEEP_SPLIT_COLS=2)
  // the column split is turned off for the context once kSweepFallbackLimit of its launches found
  // their grid not resident (each such step paid the entry wait, up to 2 ms, before the row-block
  // sweep ran): from then on the row-block sweep runs directly
  bool cs_off = false;
  // pass 0 of a gate whose last exponent was past the first window also sums the per-candidate
  // elements' polynomial, so the exponents past it are decided without pass 1 (ADMM_P16=0: off)
  bool p16 = true;
  float* gimg = nullptr;   // split image of G_h for k_qgemm3
  hipStream_t sx[kMaxSweepStreams - 1] = {};
  hipEvent_t ev_fork = nullptr, ev_join[kMaxSweepStreams - 1] = {};
  float *U = nullptr, *wy_slab = nullptr, *Gy = nullptr;
  bool gy_pending = false;   // G_y waits in gy_slot for the x stage's all-reduce (several processes)
  int wy_nsplit = 1;
  double *ht_part = nullptr, *ht_sums = nullptr;
  int ht_nblk = 1;
  unsigned* sel_count = nullptr;  // [4] per-gate arrival counts of the fused tail selection
  // U holds the wy residual of the bound state (written by the last step's k_ht_apply): the wy stage
  // skips k_wy_u.  Cleared whenever the caller may have changed h_T, a, wy or the dual y flag.
  bool u_valid = false;
  DevStats* stats = nullptr;
  // multi-GPU
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  // host-staged communicator (admm_set_comm_host): stream sync + D2H + callback + H2D
  admm_host_allreduce_fn host_ar = nullptr;
  void* host_ar_user = nullptr;
  std::vector<double> host_stage;
  // host-mapped mirror of DevStats {unresolved, nonfinite, handoff_fail, sweep_fallback}, written
  // by the step's last kernel and read without a sync by admm_poll_status / admm_poll_faults
  int* status_host = nullptr;
  int* status_dev = nullptr;
  // hand-off timeouts already reported (admm_step refuses to run on a state a timed-out hand-off
  // left invalid until the caller restores it and says so: admm_ack_fault, or admm_init_state)
  int handoff_ack = 0;
  // admm_debug_fault: one-shot fault injection (tests)
  bool fault_skip_publish = false, fault_capture = false;
  // optional live kernel timing (admm_profile): hipEvent pairs around launches of the
  // selected kernel classes, on the launch stream
  uint32_t prof_mask = 0;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_used;
  // admm_debug_trace: caller buffers receiving each stage's G (tests)
  float* trace_g[2] = {nullptr, nullptr};
  // admm_debug_trace_resid: caller buffers receiving each stage's residual R [4][BT][H] (tests)
  float* trace_r[2] = {nullptr, nullptr};
  // admm_debug_force: forced line-search decisions [8 exponents, h_T failing tests] (tests)
  int* force_dev = nullptr;
  bool force_on = false;
  // steady-state step graph (ADMM_GRAPH=1, admm_step)
  bool graph = false;
  hipStream_t gs = nullptr;
  hipEvent_t ev_gfork = nullptr, ev_gjoin = nullptr;
  hipGraphExec_t gexec = nullptr;
  StepSig gsig{}, last_sig{};
  bool have_last_sig = false;
  int64_t graph_replays = 0;
  int32_t graph_captures = 0;
  bool graph_disabled = false;   // a capture failed: steps run eagerly from then on
};

namespace {

hipEvent_t take_event(AdmmCtx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Records an event pair around the launches issued in its scope when the class is enabled.
struct ProfScope {
  AdmmCtx* c;
  int cls;
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(AdmmCtx* c_, int cls_, hipStream_t s_) : c(c_), cls(cls_), s(s_) {
    if (c->prof_mask & (1u << cls)) {
      a = take_event(c);
      b = take_event(c);
      (void)hipEventRecord(a, s);
    }
  }
  ~ProfScope() {
    if (a) {
      (void)hipEventRecord(b, s);
      c->ev_used.push_back({cls, {a, b}});
    }
  }
};

Weights weights_of(const AdmmCtx* c) {
  Weights w;
  for (int q = 0; q < 4; ++q) {
    w.wx[q] = c->buf.wx[q];
    w.wh[q] = c->buf.wh[q];
  }
  return w;
}

Planes6 planes(float* const p[6]) {
  Planes6 r;
  for (int i = 0; i < 6; ++i) r.p[i] = p[i];
  return r;
}

// Host-staged all-reduce (admm_set_comm_host): a test / fallback path, not the RCCL one.
int allreduce_host(AdmmCtx* c, void* p, size_t n, int dtype, hipStream_t s) {
  const size_t bytes = n * (dtype == 0 ? sizeof(float) : sizeof(double));
  if (c->host_stage.size() * sizeof(double) < bytes) c->host_stage.resize((bytes + 7) / 8);
  void* h = c->host_stage.data();
  HIP_TRY(hipMemcpyAsync(h, p, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const int rc = c->host_ar(h, (int64_t)n, dtype, c->host_ar_user);
  if (rc != 0) return fail(ADMM_ECOMM, "host all-reduce callback returned %d", rc);
  HIP_TRY(hipMemcpyAsync(p, h, bytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return ADMM_OK;
}

int allreduce_f32(AdmmCtx* c, float* p, size_t n, hipStream_t s) {
  if (c->host_ar) return allreduce_host(c, p, n, 0, s);
  if (!c->comm) return ADMM_OK;
  ProfScope ps(c, ADMM_PROF_COMM, s);
  NCCL_TRY(ncclAllReduce(p, p, n, ncclFloat32, ncclSum, c->comm, s));
  return ADMM_OK;
}

int allreduce_f64(AdmmCtx* c, double* p, size_t n, hipStream_t s) {
  if (c->host_ar) return allreduce_host(c, p, n, 1, s);
  if (!c->comm) return ADMM_OK;
  ProfScope ps(c, ADMM_PROF_COMM, s);
  NCCL_TRY(ncclAllReduce(p, p, n, ncclFloat64, ncclSum, c->comm, s));
  return ADMM_OK;
}

// G_y's slot after the x stage's G [4][D][H] (the G buffer holds 4 max(D, H) H + H O floats)
float* gy_slot(AdmmCtx* c) { return c->G + (size_t)4 * c->g.D * c->g.H; }

// wy update (admm.py:246-280; admm.no_dual_y.py:226-249)
int stage_wy(AdmmCtx* c, hipStream_t s) {
  const Geom& g = c->g;
  ProfScope ps(c, ADMM_PROF_SMALL, s);
  launch_wy_grad(g, c->hp, c->buf.gates[ADMM_H], c->buf.a, c->buf.dual_y, c->buf.wy, c->U, c->wy_slab,
                 c->wy_nsplit, s, c->u_valid);
  if (!c->comm && !c->host_ar) {   // one process: reduce and apply in one launch
    launch_wy_reduce(g, c->hp, c->wy_slab, c->wy_nsplit, c->Gy, c->buf.wy, s);
    return ADMM_OK;
  }
  // several processes: G_y is all-reduced together with the x stage's G (the x stage does not
  // read wy), in the slot right after it, and wy is updated once that all-reduce is done
  launch_wy_reduce(g, c->hp, c->wy_slab, c->wy_nsplit, gy_slot(c), nullptr, s);
  c->gy_pending = true;
  return ADMM_OK;
}

// One weight stage: the 4 gates' (side) weights, each a backtracking proximal-linearised
// update (admm.py:282-343).  side 0 = x2q (input weights), side 1 = h2q (recurrent).
int stage_weights(AdmmCtx* c, int side, hipStream_t s) {
  const Geom& g = c->g;
  const int Kd = side == 0 ? g.D : g.H;
  const bool fast = fast_path(g) && !c->force_generic;
  const Planes6 S = planes(c->buf.gates), L = planes(c->buf.duals);
  const bool spec = fast && c->spec_x;
  // z of the h-side searches uses the updated x2q (admm.py:298-300): zc += x dWx, or with
  // speculation zx (written by the x trials) fixed up for mispredicted gates
  if (fast && side == 1) {
    ProfScope ps(c, ADMM_PROF_RESID, s);
    if (spec) launch_apply_fix(g, c->buf.x, c->dW, c->zc, c->zx, c->kpred, c->stats, s);
    else launch_apply_dwx(g, c->buf.x, c->dW, c->zc, s);
  }
  float* const zh = spec ? c->zx : c->zc;   // z of this stage's h side
  int ns;
  // 1. G_q = rho_q sum_rows A^T R_q
  const float* gsrc = c->gslab;
  if (fast && side == 0 && c->gx_valid && c->tgt_valid && c->z_valid) {
    ns = c->gx_nblk;        // the sweep left the partials (and tgt) of this state
    gsrc = c->gx_slab;
  } else if (fast && side == 0) {
    ns = c->nblk_rx;
    ProfScope ps(c, ADMM_PROF_RESID, s);
    launch_resid_gx(g, c->hp, c->buf.x, S, L, c->zc, c->tgt, c->gslab, ns, c->tgt_valid && c->z_valid, s);
  } else if (fast && c->split3) {
    ns = atr3_splits(g);
    // scaled fp16 operands once a persistent sweep has left the operand ranges of this state
    const bool f16 = c->atr_f16 && c->range_valid;
    if (f16 && !c->x1_valid) {
      HIP_TRY(hipMemsetAsync(c->range + 5, 0, sizeof(float), s));
      launch_x_l1max(g, c->buf.x, c->range, s);
      c->x1_valid = true;
    }
    ProfScope ps(c, ADMM_PROF_ATR_H, s);
    launch_atr3(g, c->buf.gates[ADMM_H], zh, c->tgt, c->gslab, ns, s, f16 ? c->range : nullptr,
                f16 ? c->dW : nullptr, c->atr_wide);
  } else if (fast) {
    ns = atr_splits(g, 1);
    ProfScope ps(c, ADMM_PROF_ATR_H, s);
    launch_atr_fused(g, c->hp, c->buf.x, c->buf.gates[ADMM_H], zh, c->tgt, c->dW, c->gslab, ns, s);
  } else {
    ResidArgs ra{};
    ra.stage = side;
    ra.x = c->buf.x;
    ra.S = S;
    ra.L = L;
    ra.zc = c->zc;
    ra.tgt = c->tgt;
    ra.R = c->R;
    ra.dW = c->dW;
    ra.nblk = c->nblk_resid;
    {
      ProfScope ps(c, ADMM_PROF_RESID, s);
      launch_resid(g, c->hp, ra, s);
    }
    ns = atr_splits(g, side);
    ProfScope ps(c, side == 0 ? ADMM_PROF_ATR_X : ADMM_PROF_ATR_H, s);
    launch_atr(g, side, c->buf.x, c->buf.gates[ADMM_H], c->R, c->gslab, ns, s);
  }
  if (c->trace_r[side]) {   // the residual this stage's G was formed from, as that kernel formed it
    if (!fast) HIP_TRY(hipMemcpyAsync(c->trace_r[side], c->R, (size_t)4 * g.BT() * g.H * sizeof(float),
                                      hipMemcpyDeviceToDevice, s));
    else launch_debug_resid(g, side == 0 ? c->zc : zh, c->tgt, c->trace_r[side], s);
  }
  // one process, split3 Q GEMM: the h side's reduce also forms the split G image for k_qgemm3 (no
  // k_split_g launch); several processes split it after the all-reduce
  const bool gimg_fused = side == 1 && fast && c->split3 && !c->comm && !c->host_ar;
  if (gimg_fused)
    launch_reduce_gh_img(g, c->hp, gsrc, ns, c->G, c->found, c->stats, s, c->p16, c->range, c->gimg);
  else
    launch_reduce_g(g, side, c->hp, gsrc, ns, c->G, c->found, spec && side == 0 ? c->kpred : nullptr, c->stats, s,
                    c->p16, side == 1 ? c->range : nullptr);   // (the h side clears the ranges for the sweep)
  // (x stage with G_y pending: one all-reduce for both, then the wy update)
  const bool with_gy = side == 0 && c->gy_pending;
  int rc = allreduce_f32(c, c->G, (size_t)4 * Kd * g.H + (with_gy ? (size_t)g.H * g.O : 0), s);
  if (rc) return rc;
  if (with_gy) {
    ProfScope ps(c, ADMM_PROF_SMALL, s);
    launch_wy_apply(g, c->hp, gy_slot(c), c->buf.wy, s);
    c->gy_pending = false;
  }
  if (c->trace_g[side])
    HIP_TRY(hipMemcpyAsync(c->trace_g[side], c->G, (size_t)4 * Kd * g.H * sizeof(float), hipMemcpyDeviceToDevice, s));
  // 2. trial direction Q = A G (not needed on the fast x side: formed inside the trials)
  if (!(fast && side == 0)) {
    ProfScope ps(c, side == 0 ? ADMM_PROF_QGEMM_X : ADMM_PROF_QGEMM_H, s);
    if (side == 1 && c->split3) launch_qgemm3(g, c->buf.gates[ADMM_H], c->G, c->gimg, c->Q, s, gimg_fused);
    else launch_qgemm(g, side, c->buf.x, c->buf.gates[ADMM_H], c->G, c->Q, s);
  }
  // 3. line search: trial passes of kTrialJ exponents each until every gate has passed
  SelectArgs sa{};
  sa.side = side;
  sa.last_pass = kMaxPasses - 1;
  sa.sums = c->tr_sums;
  sa.poly = c->tr_poly;
  sa.G = c->G;
  for (int q = 0; q < 4; ++q) sa.W[q] = side == 0 ? c->buf.wx[q] : c->buf.wh[q];
  sa.dW = side == 0 ? c->dW : nullptr;
  const bool fused_reduce = !c->comm && !c->host_ar;   // one process: k_select reduces the partials
  sa.pick = c->pick;
  sa.stats = c->stats;
  sa.force = c->force_on ? c->force_dev : nullptr;
  sa.wt = c->sweep_rows ? c->swt : nullptr;   // the sweep's weight image of the updated weights
  sa.wt_rows16 = sweep_wt_rows16(g);
  sa.wt_xc = sweep_wt_xc(g);
  const int nblk = fast ? trial_fast_blocks(g, side) : c->nblk_trial;
  // the row-pair trial kernel (H % 256 == 0) writes one partial per (block, column block)
  const int nred = fast && side == 0 && trial_mx_ok(g) ? nblk * (g.H / 128)
                   : fast && trial_rows_ok(g) ? nblk * (g.H / 256) : nblk;
  if (nred > c->nblk_trial)   // the partial buffer holds nblk_trial per slot and window
    return fail(ADMM_ESTATE, "trial partials %d exceed the %d allocated", nred, c->nblk_trial);
  // pass 0, then the tail (windows 1 .. kMaxPasses - 1 in one launch, one selection, one
  // all-reduce) for the gates pass 0 left undecided -- with the polynomial past the window
  // (hint, k_reduce_g) that is rare, and the tail's workgroups exit at once
  for (int pass : {0, kTailPass}) {
    const int par = pass == 0 ? 0 : 1;   // parity of the found flags this pass reads
    sa.pass = pass;
    sa.found_in = c->found + 4 * par;
    sa.found_out = c->found + 4 * (par ^ 1);
    const int nwin = pass == 0 ? 1 : kMaxPasses - 1;
    if (fused_reduce) {   // k_select reduces the partials itself (no all-reduce in between)
      sa.part = c->tr_part;
      sa.nred = nred;
    } else {
      sa.part = nullptr;
    }
    // one process: the tail launch makes its own selection (its last workgroup per gate)
    const bool tail_fused = fused_reduce && fast && pass == kTailPass && tail_select_fused(g, side);
    {
      ProfScope ps(c, pass != 0 ? ADMM_PROF_TRIAL_EXTRA : side == 0 ? ADMM_PROF_TRIAL : ADMM_PROF_TRIAL_H, s);
      SpecX sx{};
      if (spec && side == 0 && pass == 0) {
        sx.kpred = c->kpred;
        for (int q = 0; q < 4; ++q) sx.W[q] = c->buf.wx[q];
        sx.zx = c->zx;
        sx.hp = c->hp;
      }
      if (fast)
        launch_trial_fast(g, side, pass, side == 1 ? zh : c->zc, c->tgt, side == 1 ? c->Q : nullptr, c->buf.x,
                          side == 0 ? c->G : c->dW, c->found + 4 * par, c->tr_part, nblk, s, sx.zx ? &sx : nullptr,
                          side == 1 && c->split3 ? q_layout(g) : 0, tail_fused ? &sa : nullptr,
                          tail_fused ? &c->hp : nullptr, tail_fused ? c->sel_count : nullptr);
      else
        launch_trial(g, pass, c->zc, c->tgt, c->Q, c->found + 4 * par, c->tr_part, nblk, s);
    }
    if (tail_fused) continue;
    if (!fused_reduce) {
      launch_trial_reduce(g, pass, c->tr_part, nred, sa.found_in, c->tr_sums, s);
      rc = allreduce_f64(c, c->tr_sums, (size_t)nwin * 4 * kTrialSlots, s);
      if (rc) return rc;
    }
    launch_select(g, c->hp, sa, s);
  }
  return ADMM_OK;
}

// Sequential sweep t = 1..T (admm.py:72-76) and the h_T / a / dual work at T.
int stage_sweep(AdmmCtx* c, hipStream_t s) {
  const Geom& g = c->g;
  const Weights w = weights_of(c);
  SweepT sa{};
  sa.x = c->buf.x;
  sa.S = planes(c->buf.gates);
  sa.L = planes(c->buf.duals);
  sa.zc = c->zc;
  if (c->sweep_rows) {
    ProfScope ps(c, ADMM_PROF_SWEEP, s);
    sa.r0 = 0;
    sa.r1 = g.B;
    sa.tgt = fast_path(g) && c->tgt_sweep ? c->tgt : nullptr;   // the fast x stage reads it next step
    sa.gx_slab = sa.tgt ? c->gx_slab : nullptr;
    if (g.H % 4 == 0 && g.T > 1 && !c->lamh_known) {
      HIP_TRY(hipMemsetAsync(c->lamh_nz, 0, sizeof(int), s));
      launch_check_lamh(g, c->buf.duals[ADMM_H], c->lamh_nz, s);
      c->lamh_known = true;
    }
    sa.lamh_nz = c->lamh_known && c->lamh_skip ? c->lamh_nz : nullptr;
    sa.range = c->range;   // zeroed by this step's h-stage k_reduce_g
    if (c->xbuf && !c->cs_off && ((const volatile int*)c->status_host)[3] >= kSweepFallbackLimit)
      c->cs_off = true;    // (the mirror: fallbacks as of the last completed step)
    sa.xbuf = c->cs_off ? nullptr : c->xbuf;   // zeroed by k_sweep_wt (column split only)
    sa.fail = &c->stats->handoff_fail;       // a hand-off that timed out makes the step's results invalid
    sa.fallback = &c->stats->sweep_fallback;  // the column split's grid was not resident: row-block sweep ran
    sa.skip_publish = c->fault_skip_publish ? 1 : 0;
    c->fault_skip_publish = false;
    // the weight image: once (its padding); later steps' selections wrote the new weights into it,
    // and the last step's k_ht_apply zeroed the hand-off buffer
    if (!c->wt_init) {
      launch_sweep_wt(g, w, c->swt, s, c->xbuf);
      c->wt_init = true;
    }
    if (c->cs_poison && sa.xbuf) sweep_poison_entry(g, c->xbuf, s);
    launch_sweep_rows(g, c->swt, c->hp, sa, s);
  } else {
    // Samples are independent across the sweep: two halves on two streams run their
    // per-t kernels concurrently, so one half's HBM-bound epilogue overlaps the other's
    // MFMA-bound GEMM on the same CUs (one kernel per t alone runs them back to back).
    ProfScope ps(c, ADMM_PROF_SWEEP, s);
    // part p of np: rows [p*chunk, (p+1)*chunk), chunk a multiple of the 128-row tile
    const int np = std::max(1, std::min<int>(c->sweep_split, (int)((g.B + 127) / 128)));
    const int64_t chunk = ((g.B + np - 1) / np + 127) / 128 * 128;
    const int nparts = (int)((g.B + chunk - 1) / chunk);
    hipStream_t st[kMaxSweepStreams];
    st[0] = s;
    for (int p = 1; p < nparts; ++p) st[p] = c->sx[p - 1];
    if (nparts > 1) {
      HIP_TRY(hipEventRecord(c->ev_fork, s));
      for (int p = 1; p < nparts; ++p) HIP_TRY(hipStreamWaitEvent(st[p], c->ev_fork, 0));
    }
    for (int t = 1; t <= g.T; ++t)
      for (int p = 0; p < nparts; ++p) {
        sa.r0 = p * chunk;
        sa.r1 = std::min<int64_t>(sa.r0 + chunk, g.B);
        launch_sweep_t(g, t, w, c->hp, sa, st[p]);
      }
    for (int p = 1; p < nparts; ++p) {
      HIP_TRY(hipEventRecord(c->ev_join[p - 1], st[p]));
      HIP_TRY(hipStreamWaitEvent(s, c->ev_join[p - 1], 0));
    }
  }
  ProfScope ps(c, ADMM_PROF_SMALL, s);
  launch_ht_partial(g, c->hp, sa.S, sa.L, c->buf.a, c->buf.dual_y, c->buf.wy, c->ht_part, c->ht_nblk, s);
  launch_ht_reduce(c->ht_part, c->ht_nblk, c->ht_sums, s);
  int rc = allreduce_f64(c, c->ht_sums, kHTSums, s);
  if (rc) return rc;
  // (also the next step's wy residual U: the wy stage then skips k_wy_u)
  launch_ht_apply(g, c->hp, sa.S, sa.L, c->buf.a, c->buf.dual_y, c->buf.y, c->buf.wy, c->ht_sums, c->stats,
                  c->status_dev, s, c->force_on ? c->force_dev : nullptr, c->U, c->xbuf);
  return ADMM_OK;
}

int check_dims(const AdmmDims* d) {
  if (!d) return fail(ADMM_EINVAL, "dims is NULL");
  if (d->batch <= 0 || d->seq_len <= 0 || d->input_size <= 0 || d->hidden_size <= 0 || d->output_size <= 0)
    return fail(ADMM_EINVAL, "all dims must be positive (B=%lld T=%d D=%d H=%d O=%d)", (long long)d->batch,
                d->seq_len, d->input_size, d->hidden_size, d->output_size);
  if (d->global_batch < d->batch) return fail(ADMM_EINVAL, "global_batch < batch");
  // the h_T kernels keep one LDS row of O floats per wave (4 waves per workgroup)
  if (d->output_size > kMaxOutputs)
    return fail(ADMM_EINVAL, "output_size %d > %d is not supported", d->output_size, kMaxOutputs);
  if (d->batch * (int64_t)d->seq_len >= (1ll << 31))
    return fail(ADMM_EINVAL, "batch*seq_len = %lld rows per device exceeds 2^31-1", (long long)(d->batch * (int64_t)d->seq_len));
  return ADMM_OK;
}

}  // namespace

extern "C" {

int32_t admm_abi_version(void) { return ADMM_LSTM_ABI_VERSION; }

#ifndef ADMM_SRC_STAMP
#define ADMM_SRC_STAMP "unstamped"
#endif
// "... src <stamp>": the Makefile's hash of the sources this library was built from
const char* admm_build_info(void) {
  return "libadmmlstm gfx950 (split bf16/fp16 and fp32 MFMA, RCCL), abi 3, src " ADMM_SRC_STAMP;
}

const char* admm_last_error(void) { return g_last_error.c_str(); }

int admm_create(const AdmmDims* dims, const AdmmParams* params, int device, AdmmCtx** out) {
  if (!out) return fail(ADMM_EINVAL, "out is NULL");
  *out = nullptr;
  int rc = check_dims(dims);
  if (rc) return rc;
  if (!params) return fail(ADMM_EINVAL, "params is NULL");
  if (params->variant != ADMM_VARIANT_ADMM && params->variant != ADMM_VARIANT_NO_DUAL_Y)
    return fail(ADMM_EINVAL, "unknown variant %d", params->variant);
  for (int i = 0; i < 7; ++i)
    if (!std::isfinite(params->rho[i])) return fail(ADMM_EINVAL, "rho[%d] is not finite", i);
  DEVICE_GUARD(device);
  AdmmCtx* c = new AdmmCtx();
  c->device = device;
  Geom& g = c->g;
  g.B = dims->batch;
  g.Bg = dims->global_batch;
  g.T = dims->seq_len;
  g.D = dims->input_size;
  g.H = dims->hidden_size;
  g.O = dims->output_size;
  g.set_T();
  // kernel-choice knobs live in the context's Geom (a per-context read: tests flip them
  // between contexts of one process)
  if (const char* e = std::getenv("ADMM_SWEEP_R16")) g.r16 = std::atoi(e) != 0;
  c->sweep_rows = sweep_rows_ok(g);
  if (const char* e = std::getenv("ADMM_SWEEP_ROWS")) c->sweep_rows = c->sweep_rows && std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_TGT_SWEEP")) c->tgt_sweep = std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_GX_SWEEP")) c->gx_sweep = std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_LAMH_SKIP")) c->lamh_skip = std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_GENERIC")) c->force_generic = std::atoi(e) != 0;
  c->split3 = fast_path(g) && split3_ok(g);
  c->spec_x = fast_path(g) && trial_rows_ok(g);
  if (const char* e = std::getenv("ADMM_SPEC_X")) c->spec_x = c->spec_x && std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_SPLIT3")) c->split3 = c->split3 && std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_P16")) c->p16 = std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_ATR_F16")) c->atr_f16 = std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_ATR_WIDE")) c->atr_wide = std::atoi(e) != 0;
  if (const char* e = std::getenv("ADMM_GRAPH")) c->graph = std::atoi(e) != 0;
  Hyper& h = c->hp;
  for (int i = 0; i < 7; ++i) h.rho[i] = params->rho[i];
  h.rinv_exact = 1;
  for (int i = 0; i < 4; ++i) {   // rho = 2^(e-1) with 2^(1-e) a normal float
    int e = 0;
    const float m = std::frexp(h.rho[i], &e);
    const bool p2 = m == 0.5f && 1 - e >= -126 && 1 - e <= 127;
    h.rinv_gate[i] = p2 ? std::ldexp(1.f, 1 - e) : 0.f;
    h.rinv_exact &= p2 ? 1 : 0;
  }
  if (const char* e = std::getenv("ADMM_RINV")) h.rinv_exact &= std::atoi(e) != 0 ? 1 : 0;
  for (int q = 0; q < 4; ++q) {
    h.beta_x[q] = params->beta_x[q];
    h.beta_h[q] = params->beta_h[q];
  }
  h.beta_y = params->beta_y;
  h.variant = params->variant;
  h.with_dual_y = params->with_dual_y;

  // the column-split sweep keeps all its workgroups resident at once: one per CU, kSweepCUs of them
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 0;
  {   // ADMM_SWEEP_SPLIT_COLS=0: row blocks only; =2: the column split's entry count poisoned before
      // every launch, so the gated row-block sweep does the work (test hooks); default on
    const char* e = std::getenv("ADMM_SWEEP_SPLIT_COLS");
    if (e && std::atoi(e) == 0) cus = 0;
    c->cs_poison = e && std::atoi(e) == 2;
  }
  const size_t plane = (size_t)g.BT() * g.H;
  // the sweep's x-stage partials: persistent sweep, fast path, D <= 16, targets from the sweep
  c->gx_nblk = c->sweep_rows && sweep_rows_gx_ok(g) && fast_path(g) && c->tgt_sweep && c->gx_sweep ? sweep_rows_blocks(g) : 0;
  const int Kmax = g.D > g.H ? g.D : g.H;
  c->nblk_resid = resid_blocks(g);
  c->nblk_trial = std::max(trial_blocks(g), stream_blocks(g) * (trial_mx_ok(g) ? g.H / 128 : trial_rows_ok(g) ? g.H / 256 : 1));
  c->nblk_rx = resid_gx_blocks(g);
  size_t slab = (size_t)atr_splits(g, 0) * 4 * g.D * g.H;
  slab = std::max(slab, (size_t)atr_splits(g, 1) * 4 * g.H * g.H);
  slab = std::max(slab, (size_t)c->nblk_rx * 4 * g.D * g.H);
  if (c->split3) slab = std::max(slab, (size_t)atr3_splits(g) * 4 * g.H * g.H);
  c->wy_nsplit = wy_splits(g);
  c->ht_nblk = ht_blocks(g);
  if ((rc = dalloc(&c->zc, 4 * plane)) || (rc = dalloc(&c->tgt, 4 * plane)) || (rc = dalloc(&c->R, fast_path(g) && !c->force_generic ? 1 : 4 * plane)) ||
      (rc = dalloc(&c->Q, 4 * plane)) || (rc = dalloc(&c->G, (size_t)4 * Kmax * g.H + (size_t)g.H * g.O)) ||
      (rc = dalloc(&c->dW, (size_t)4 * g.D * g.H)) ||
      (rc = dalloc(&c->gslab, slab)) ||
      (rc = dalloc(&c->tr_part, (size_t)(kMaxPasses - 1) * 4 * kTrialSlots * c->nblk_trial)) ||
      (rc = dalloc(&c->tr_sums, (size_t)(kMaxPasses - 1) * 4 * kTrialSlots)) || (rc = dalloc(&c->tr_poly, (size_t)4 * kPolyN)) ||
      (rc = dalloc(&c->found, 12)) || (rc = dalloc(&c->pick, 4)) ||
      (rc = dalloc(&c->U, (size_t)g.B * g.O)) || (rc = dalloc(&c->wy_slab, (size_t)c->wy_nsplit * g.H * g.O)) ||
      (rc = dalloc(&c->Gy, (size_t)g.H * g.O)) || (rc = dalloc(&c->ht_part, (size_t)c->ht_nblk * kHTSums)) ||
      (rc = dalloc(&c->ht_sums, kHTSums)) || (rc = dalloc(&c->sel_count, 4)) || (rc = dalloc(&c->stats, 1)) || (rc = dalloc(&c->lamh_nz, 1)) || (rc = dalloc(&c->force_dev, 9)) || (rc = dalloc(&c->range, 8)) ||
      (c->sweep_rows && (rc = dalloc(&c->swt, sweep_wt_floats(g)))) ||
      (c->sweep_rows && sweep_rows_nc(g) > 1 && cus >= kSweepCUs && (rc = dalloc(&c->xbuf, sweep_xbuf_bytes(g) / 4))) ||
      (c->split3 && (rc = dalloc(&c->gimg, split3_gimg_floats(g)))) ||
      (c->spec_x && ((rc = dalloc(&c->zx, 4 * plane)) || (rc = dalloc(&c->kpred, 4)))) ||
      (c->gx_nblk > 0 && (rc = dalloc(&c->gx_slab, (size_t)c->gx_nblk * 4 * g.D * g.H)))) {
    std::string msg = g_last_error;
    admm_destroy(c);
    return fail(rc, "%s", msg.c_str());
  }
  bool ok = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_gfork, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_gjoin, hipEventDisableTiming) == hipSuccess &&
            hipStreamCreateWithFlags(&c->gs, hipStreamNonBlocking) == hipSuccess;
  for (int p = 0; ok && p < kMaxSweepStreams - 1; ++p)
    ok = hipStreamCreateWithFlags(&c->sx[p], hipStreamNonBlocking) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_join[p], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    admm_destroy(c);
    return fail(ADMM_EHIP, "stream/event creation failed");
  }
  if (hipMemset(c->stats, 0, sizeof(DevStats)) != hipSuccess || hipMemset(c->range, 0, 8 * sizeof(float)) != hipSuccess ||
      hipMemset(c->sel_count, 0, 4 * sizeof(unsigned)) != hipSuccess) {
    admm_destroy(c);
    return fail(ADMM_EHIP, "hipMemset(stats) failed");
  }
  if (hipHostMalloc((void**)&c->status_host, 4 * sizeof(int), hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&c->status_dev, c->status_host, 0) != hipSuccess) {
    admm_destroy(c);
    return fail(ADMM_EHIP, "mapped status mirror allocation failed");
  }
  for (int i = 0; i < 4; ++i) c->status_host[i] = 0;
  *out = c;
  return ADMM_OK;
}

int admm_destroy(AdmmCtx* c) {
  if (!c) return ADMM_OK;
  DeviceGuard dg_(c->device);
  void* ptrs[] = {c->zc, c->tgt, c->R, c->Q, c->G, c->dW, c->gslab, c->tr_part, c->tr_sums, c->tr_poly, c->found, c->pick,
                  c->U, c->wy_slab, c->Gy, c->ht_part, c->ht_sums, c->sel_count, c->stats, c->swt, c->gimg, c->zx, c->kpred, c->gx_slab, c->lamh_nz, c->force_dev, c->range, c->xbuf};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->status_host) (void)hipHostFree(c->status_host);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
  if (c->ev_gfork) (void)hipEventDestroy(c->ev_gfork);
  if (c->ev_gjoin) (void)hipEventDestroy(c->ev_gjoin);
  if (c->gs) (void)hipStreamDestroy(c->gs);
  for (int p = 0; p < kMaxSweepStreams - 1; ++p) {
    if (c->ev_join[p]) (void)hipEventDestroy(c->ev_join[p]);
    if (c->sx[p]) (void)hipStreamDestroy(c->sx[p]);
  }
  for (auto& u : c->ev_used) {
    (void)hipEventDestroy(u.second.first);
    (void)hipEventDestroy(u.second.second);
  }
  delete c;
  return ADMM_OK;
}

int admm_bind(AdmmCtx* c, const AdmmBuffers* b) {
  if (!c || !b) return fail(ADMM_EINVAL, "NULL argument");
  const void* req[] = {b->x, b->y, b->wy, b->a, b->dual_y};
  for (const void* p : req)
    if (!p) return fail(ADMM_EINVAL, "admm_bind: a required buffer is NULL");
  for (int q = 0; q < 4; ++q)
    if (!b->wx[q] || !b->wh[q]) return fail(ADMM_EINVAL, "admm_bind: weight %d is NULL", q);
  for (int q = 0; q < 6; ++q)
    if (!b->gates[q] || !b->duals[q]) return fail(ADMM_EINVAL, "admm_bind: gate/dual %d is NULL", q);
  c->buf = *b;
  c->bound = true;
  c->u_valid = false;
  c->z_valid = false;
  c->tgt_valid = false;
  c->gx_valid = false;
  c->lamh_known = false;
  c->range_valid = c->x1_valid = false;
  return ADMM_OK;
}

int admm_set_with_dual_y(AdmmCtx* c, int32_t flag) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  if ((flag ? 1 : 0) != c->hp.with_dual_y) c->u_valid = false;   // U's dual-y shift changes
  c->hp.with_dual_y = flag ? 1 : 0;
  return ADMM_OK;
}

int admm_invalidate_cache(AdmmCtx* c) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  c->u_valid = false;
  c->z_valid = false;
  c->tgt_valid = false;
  c->gx_valid = false;
  c->lamh_known = false;
  c->range_valid = c->x1_valid = false;
  return ADMM_OK;
}

int admm_ack_fault(AdmmCtx* c) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  c->handoff_ack = c->status_host[2];   // the caller restored the state: the timed-out hand-offs are behind it
  return admm_invalidate_cache(c);
}

int admm_init_state(AdmmCtx* c, void* stream) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  if (!c->bound) return fail(ADMM_ESTATE, "admm_init_state before admm_bind");
  c->handoff_ack = c->status_host[2];
  c->u_valid = false;
  hipStream_t s = (hipStream_t)stream;
  const Geom& g = c->g;
  DEVICE_GUARD(c->device);
  const size_t pbytes = (size_t)g.B * g.TP() * g.H * sizeof(float);
  for (int q = 0; q < 6; ++q) {
    HIP_TRY(hipMemsetAsync(c->buf.gates[q], 0, pbytes, s));
    HIP_TRY(hipMemsetAsync(c->buf.duals[q], 0, pbytes, s));
  }
  HIP_TRY(hipMemsetAsync(c->buf.dual_y, 0, (size_t)g.B * g.O * sizeof(float), s));
  const Weights w = weights_of(c);
  const int64_t rs = (int64_t)g.TP() * g.H;
  for (int t = 1; t <= g.T; ++t) {
    ForwardT fa{};
    fa.x = c->buf.x;
    fa.hprev = c->buf.gates[ADMM_H] + (int64_t)(t - 1) * g.H;
    fa.hprev_stride = rs;
    fa.cprev = c->buf.gates[ADMM_C] + (int64_t)(t - 1) * g.H;
    fa.cprev_stride = rs;
    fa.hout = c->buf.gates[ADMM_H] + (int64_t)t * g.H;
    fa.hout_stride = rs;
    fa.cout = c->buf.gates[ADMM_C] + (int64_t)t * g.H;
    fa.cout_stride = rs;
    for (int q = 0; q < 4; ++q) fa.gout[q] = c->buf.gates[q] + (int64_t)t * g.H;
    fa.gout_stride = rs;
    fa.zc = c->zc;
    launch_forward_t(g, t, w, fa, s);
  }
  launch_rowdot(g.B, g.H, g.O, c->buf.gates[ADMM_H] + (int64_t)g.T * g.H, rs, c->buf.wy, c->buf.a, s);
  HIP_TRY(hipGetLastError());
  c->z_valid = true;
  c->tgt_valid = false;   // recomputed from the new state by the first x stage
  c->gx_valid = false;
  c->range_valid = false;   // the first h stage takes split3 (no sweep has bounded its operands)
  HIP_TRY(hipMemsetAsync(c->lamh_nz, 0, sizeof(int), s));   // the duals were just zeroed
  c->lamh_known = true;
  return ADMM_OK;
}

namespace {

// Everything the launch sequence of one step depends on besides the device data: two steps with
// equal signatures enqueue the same kernels with the same arguments (the steady state).
StepSig step_sig(const AdmmCtx* c) {
  StepSig g{};
  g.flags = (c->z_valid ? 1u : 0u) | (c->tgt_valid ? 2u : 0u) | (c->gx_valid ? 4u : 0u) | (c->range_valid ? 8u : 0u) |
            (c->x1_valid ? 16u : 0u) | (c->lamh_known ? 32u : 0u) | (c->hp.with_dual_y ? 64u : 0u) |
            (c->force_on ? 128u : 0u) | (c->prof_mask ? 256u : 0u) | (c->host_ar ? 512u : 0u) | (c->u_valid ? 1024u : 0u) |
            (c->wt_init ? 2048u : 0u) | (c->cs_off ? 4096u : 0u);
  g.buf = c->buf;
  g.trace[0] = c->trace_g[0]; g.trace[1] = c->trace_g[1]; g.trace[2] = c->trace_r[0]; g.trace[3] = c->trace_r[1];
  g.comm = c->comm;
  return g;
}

bool sig_eq(const StepSig& a, const StepSig& b) { return std::memcmp(&a, &b, sizeof a) == 0; }

int run_step(AdmmCtx* c, hipStream_t s) {
  int rc;
  if (!c->z_valid) {
    ProfScope ps(c, ADMM_PROF_ZGEMM, s);
    launch_zgemm(c->g, weights_of(c), c->buf.x, c->buf.gates[ADMM_H], c->zc, s);
  }
  if ((rc = stage_wy(c, s))) return rc;
  if ((rc = stage_weights(c, 0, s))) return rc;
  if ((rc = stage_weights(c, 1, s))) return rc;
  if ((rc = stage_sweep(c, s))) return rc;
  HIP_TRY(hipGetLastError());
  c->z_valid = true;  // the sweep left x_t Wx + h_{t-1} Wh of the final state in the cache
  c->tgt_valid = c->sweep_rows && fast_path(c->g) && c->tgt_sweep;
  c->gx_valid = c->tgt_valid && c->gx_slab != nullptr;
  c->range_valid = c->sweep_rows;   // the persistent sweep tracked the next weight phase's operand ranges
  c->u_valid = true;                // k_ht_apply left the next wy stage's residual
  return ADMM_OK;
}

void drop_graph(AdmmCtx* c) {
  if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
  c->gexec = nullptr;
}

}  // namespace

// Steady-state steps replay one HIP graph (ADMM_GRAPH=1): once two consecutive steps start from the
// same signature (step_sig), the next one is captured on the context's own stream (the caller's may
// be the legacy default stream, which cannot be captured), instantiated, and replayed from then on
// while the signature holds, forked from and joined back to the caller's stream by events.  Any
// change (re-binding, invalidation, profiling, a debug hook, with_dual_y) runs the step eagerly.
// The host-staged communicator synchronises inside the step and is never captured.
int admm_step(AdmmCtx* c, void* stream) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  if (!c->bound) return fail(ADMM_ESTATE, "admm_step before admm_bind");
  {   // a column-split hand-off timed out in an earlier step (as of the last completed step): its
      // A image held stale h, so every state since is invalid -- refuse until the caller rewrites it
    const int hf = ((const volatile int*)c->status_host)[2];
    if (hf > c->handoff_ack)
      return fail(ADMM_EFAULT, "column-split sweep: %d hand-off wait(s) timed out in an earlier step; the state "
                  "is invalid (restore it and call admm_ack_fault, or admm_init_state)", hf - c->handoff_ack);
  }
  hipStream_t s = (hipStream_t)stream;
  DEVICE_GUARD(c->device);
  int rc;
  // the column split's switch-off (stage_sweep) is decided here too: a replayed graph skips
  // stage_sweep, and the flag is part of the signature, so the switch drops the graph at once
  if (c->xbuf && !c->cs_off && ((const volatile int*)c->status_host)[3] >= kSweepFallbackLimit) c->cs_off = true;
  const StepSig sig = step_sig(c);
  const bool capturable = c->graph && !c->graph_disabled && !c->prof_mask && !c->host_ar;
  if (capturable && c->gexec && sig_eq(sig, c->gsig)) {
    HIP_TRY(hipEventRecord(c->ev_gfork, s));
    HIP_TRY(hipStreamWaitEvent(c->gs, c->ev_gfork, 0));
    HIP_TRY(hipGraphLaunch(c->gexec, c->gs));
    HIP_TRY(hipEventRecord(c->ev_gjoin, c->gs));
    HIP_TRY(hipStreamWaitEvent(s, c->ev_gjoin, 0));
    c->steps++;
    c->graph_replays++;
    return ADMM_OK;
  }
  if (capturable && c->have_last_sig && sig_eq(sig, c->last_sig)) {
    drop_graph(c);
    hipGraph_t graph = nullptr;
    HIP_TRY(hipEventRecord(c->ev_gfork, s));
    HIP_TRY(hipStreamWaitEvent(c->gs, c->ev_gfork, 0));
    HIP_TRY(hipStreamBeginCapture(c->gs, hipStreamCaptureModeRelaxed));
    rc = run_step(c, c->gs);
    hipError_t e = hipStreamEndCapture(c->gs, &graph);
    if (e == hipSuccess && c->fault_capture) e = hipErrorUnknown;   // admm_debug_fault(2)
    c->fault_capture = false;
    if (rc == 0 && e == hipSuccess) e = hipGraphInstantiate(&c->gexec, graph, nullptr, nullptr, 0);
    if (graph) (void)hipGraphDestroy(graph);
    if (rc == 0 && e == hipSuccess) {
      c->gsig = step_sig(c);   // == sig: the steady step leaves the flags as it found them
      c->graph_captures++;
      HIP_TRY(hipGraphLaunch(c->gexec, c->gs));
      HIP_TRY(hipEventRecord(c->ev_gjoin, c->gs));
      HIP_TRY(hipStreamWaitEvent(s, c->ev_gjoin, 0));
      c->steps++;
      return ADMM_OK;
    }
    // Nothing captured ran.  The steady step leaves the host flags as it found them (sig), so the
    // step can run eagerly; graphs stay off for this context rather than failing every later step.
    c->gexec = nullptr;
    c->graph_disabled = true;
    (void)hipGetLastError();
    if (rc) return rc;   // the step itself failed (e.g. a collective): report that
  }
  if ((rc = run_step(c, s))) return rc;
  c->last_sig = sig;
  c->have_last_sig = true;
  c->steps++;
  return ADMM_OK;
}

int admm_comm_unique_id(void* out, int64_t out_bytes) {
  if (!out || out_bytes < (int64_t)sizeof(ncclUniqueId)) return fail(ADMM_EINVAL, "unique id buffer too small");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof id);
  return ADMM_OK;
}

int admm_set_comm(AdmmCtx* c, const void* uid, int64_t id_bytes, int rank, int world) {
  if (!c || !uid || id_bytes < (int64_t)sizeof(ncclUniqueId)) return fail(ADMM_EINVAL, "bad arguments");
  if (world < 1 || rank < 0 || rank >= world) return fail(ADMM_EINVAL, "bad rank %d / world %d", rank, world);
  DEVICE_GUARD(c->device);
  if (c->comm) {
    ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  c->host_ar = nullptr;
  c->rank = rank;
  c->world = world;
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof id);
  NCCL_TRY(ncclCommInitRank(&c->comm, world, id, rank));
  return ADMM_OK;
}

int admm_set_comm_host(AdmmCtx* c, admm_host_allreduce_fn fn, void* user, int rank, int world) {
  if (!c || !fn) return fail(ADMM_EINVAL, "admm_set_comm_host: NULL argument");
  if (world < 1 || rank < 0 || rank >= world) return fail(ADMM_EINVAL, "bad rank %d / world %d", rank, world);
  DEVICE_GUARD(c->device);
  if (c->comm) {
    ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  c->host_ar = fn;
  c->host_ar_user = user;
  c->rank = rank;
  c->world = world;
  return ADMM_OK;
}

int admm_poll_status(AdmmCtx* c, int32_t* unresolved, int32_t* nonfinite) {
  if (!c || !unresolved || !nonfinite) return fail(ADMM_EINVAL, "admm_poll_status: NULL argument");
  const volatile int* m = c->status_host;
  *unresolved = m[0];
  *nonfinite = m[1];
  if (m[2] > c->handoff_ack)
    return fail(ADMM_EFAULT, "column-split sweep: %d hand-off wait(s) timed out; the state is invalid", m[2] - c->handoff_ack);
  return ADMM_OK;
}

int admm_poll_faults(AdmmCtx* c, int32_t* handoff_fail, int32_t* sweep_fallbacks) {
  if (!c || !handoff_fail || !sweep_fallbacks) return fail(ADMM_EINVAL, "admm_poll_faults: NULL argument");
  const volatile int* m = c->status_host;
  *handoff_fail = m[2];
  *sweep_fallbacks = m[3];
  return ADMM_OK;
}

int admm_debug_fault(AdmmCtx* c, int32_t kind) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  switch (kind) {
    case 0: c->fault_skip_publish = c->fault_capture = false; return ADMM_OK;
    case 1:
      if (!c->xbuf) return fail(ADMM_ESTATE, "admm_debug_fault(1): this context has no column-split sweep");
      c->fault_skip_publish = true;
      return ADMM_OK;
    case 2: c->fault_capture = true; return ADMM_OK;
    default: return fail(ADMM_EINVAL, "admm_debug_fault: unknown kind %d", kind);
  }
}

int admm_profile(AdmmCtx* c, uint32_t class_mask) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  c->prof_mask = class_mask;
  return ADMM_OK;
}

int admm_profile_read(AdmmCtx* c, double* ms, int32_t* count) {
  if (!c || !ms || !count) return fail(ADMM_EINVAL, "NULL argument");
  DEVICE_GUARD(c->device);
  for (int i = 0; i < ADMM_PROF_CLASSES; ++i) {
    ms[i] = 0.0;
    count[i] = 0;
  }
  for (auto& u : c->ev_used) {
    HIP_TRY(hipEventSynchronize(u.second.second));
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, u.second.first, u.second.second));
    ms[u.first] += t;
    count[u.first] += 1;
    c->ev_pool.push_back(u.second.first);
    c->ev_pool.push_back(u.second.second);
  }
  c->ev_used.clear();
  return ADMM_OK;
}

int admm_get_stats(AdmmCtx* c, AdmmStats* out) {
  if (!c || !out) return fail(ADMM_EINVAL, "NULL argument");
  DEVICE_GUARD(c->device);
  DevStats d;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(&d, c->stats, sizeof d, hipMemcpyDeviceToHost));
  std::memset(out, 0, sizeof *out);
  out->steps = c->steps;
  for (int i = 0; i < 8; ++i) {
    out->k[i] = d.k[i];
    out->f_w[i] = d.f_w[i];
    out->grad_sq[i] = d.grad_sq[i];
    out->direct_frac[i] = d.direct_frac[i];
  }
  out->passes[0] = d.passes[0];
  out->passes[1] = d.passes[1];
  out->theta_h = d.theta_h;
  out->unresolved = d.unresolved;
  out->nonfinite = d.nonfinite;
  out->handoff_fail = d.handoff_fail;
  out->sweep_fallbacks = d.sweep_fallback;
  out->graph_captures = c->graph_captures;
  out->graph_disabled = c->graph_disabled ? 1 : 0;
  out->graph_replays = c->graph_replays;
  out->sweep_split_off = c->cs_off ? 1 : 0;
  return ADMM_OK;
}

int admm_debug_workspace(AdmmCtx* c, int32_t which, void* dst, int64_t bytes, void* stream) {
  if (!c || !dst) return fail(ADMM_EINVAL, "admm_debug_workspace: NULL argument");
  const int64_t need = (int64_t)4 * c->g.BT() * c->g.H * (int64_t)sizeof(float);
  if (bytes < need) return fail(ADMM_EINVAL, "admm_debug_workspace: %lld bytes < %lld", (long long)bytes, (long long)need);
  const float* src = which == 0 ? c->zc : which == 1 ? c->tgt : which == 2 ? c->Q : nullptr;
  if (!src) return fail(ADMM_EINVAL, "admm_debug_workspace: unknown array %d", which);
  DEVICE_GUARD(c->device);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(dst, src, need, hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (which == 2) return 1;
  return which == 0 ? (c->z_valid ? 1 : 0) : (c->tgt_valid && c->z_valid ? 1 : 0);
}

int admm_debug_trace(AdmmCtx* c, float* gx, float* gh) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  c->trace_g[0] = gx;
  c->trace_g[1] = gh;
  return ADMM_OK;
}

int admm_debug_trace_resid(AdmmCtx* c, float* rx, float* rh) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  c->trace_r[0] = rx;
  c->trace_r[1] = rh;
  return ADMM_OK;
}

int admm_debug_force(AdmmCtx* c, const int32_t* k8, int32_t ht_fails) {
  if (!c) return fail(ADMM_EINVAL, "NULL ctx");
  if (!k8) {
    c->force_on = false;
    return ADMM_OK;
  }
  int h[9];
  for (int i = 0; i < 8; ++i) {
    if (k8[i] < 0 || k8[i] >= kMaxK) return fail(ADMM_EINVAL, "admm_debug_force: k[%d] = %d out of [0, %d)", i, k8[i], kMaxK);
    h[i] = k8[i];
  }
  if (ht_fails < 0 || ht_fails > kHTCand) return fail(ADMM_EINVAL, "admm_debug_force: ht_fails = %d", ht_fails);
  h[8] = ht_fails;
  DEVICE_GUARD(c->device);
  HIP_TRY(hipDeviceSynchronize());   // the previous step may still read the old values
  HIP_TRY(hipMemcpy(c->force_dev, h, sizeof h, hipMemcpyHostToDevice));
  c->force_on = true;
  return ADMM_OK;
}

int admm_debug_own(AdmmCtx* c, int32_t* k8, float* theta_h) {
  if (!c || !k8 || !theta_h) return fail(ADMM_EINVAL, "admm_debug_own: NULL argument");
  DEVICE_GUARD(c->device);
  DevStats d;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(&d, c->stats, sizeof d, hipMemcpyDeviceToHost));
  for (int i = 0; i < 8; ++i) k8[i] = d.k_own[i];
  *theta_h = d.theta_h_own;
  return ADMM_OK;
}

int admm_debug_trial(const float* z, const float* tgt, const float* q, int64_t n, int32_t tanh_gate, int32_t kbase,
                     double* out, void* stream) {
  if (!z || !tgt || !q || !out || n <= 0) return fail(ADMM_EINVAL, "admm_debug_trial: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const int nblk = 64;
  double* part = nullptr;
  int rc = dalloc(&part, (size_t)nblk * kTrialJ);
  if (rc) return rc;
  launch_trial_debug(n, tanh_gate, kbase, z, tgt, q, part, nblk, s);
  std::vector<double> h((size_t)nblk * kTrialJ);
  hipError_t e = hipMemcpyAsync(h.data(), part, h.size() * sizeof(double), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(part);
  if (e != hipSuccess) return fail(ADMM_EHIP, "admm_debug_trial: %s", hipGetErrorString(e));
  for (int k = 0; k < kTrialJ; ++k) {
    double acc = 0.0;
    for (int b = 0; b < nblk; ++b) acc += h[(size_t)b * kTrialJ + k];
    out[k] = acc;
  }
  return ADMM_OK;
}

int admm_forward(const float* x, int64_t batch, int32_t seq_len, int32_t input_size, int32_t hidden_size,
                 int32_t output_size, const float* const wx[4], const float* const wh[4], const float* wy,
                 float* const gates_out[6], float* h_scratch, float* c_scratch, float* z_out, float* out_a,
                 void* stream) {
  AdmmDims d{batch, batch, seq_len, input_size, hidden_size, output_size};
  int rc = check_dims(&d);
  if (rc) return rc;
  if (!x || !wy || !out_a) return fail(ADMM_EINVAL, "admm_forward: NULL buffer");
  if (!gates_out && (!h_scratch || !c_scratch)) return fail(ADMM_EINVAL, "admm_forward: need gates_out or scratch");
  hipStream_t s = (hipStream_t)stream;
  Geom g{batch, batch, seq_len, input_size, hidden_size, output_size};
  g.set_T();
  Weights w;
  for (int q = 0; q < 4; ++q) {
    if (!wx[q] || !wh[q]) return fail(ADMM_EINVAL, "admm_forward: NULL weight");
    w.wx[q] = wx[q];
    w.wh[q] = wh[q];
  }
  const int64_t BH = batch * (int64_t)hidden_size;
  if (!gates_out) {  // gates_out: time-0 slices are the caller's initial c/h (blocks/lstm.py:69-72)
    HIP_TRY(hipMemsetAsync(h_scratch, 0, (size_t)BH * sizeof(float), s));
    HIP_TRY(hipMemsetAsync(c_scratch, 0, (size_t)BH * sizeof(float), s));
  }
  const int64_t rs = (int64_t)(seq_len + 1) * hidden_size;
  for (int t = 1; t <= seq_len; ++t) {
    ForwardT fa{};
    fa.x = x;
    if (gates_out) {
      fa.hprev = gates_out[ADMM_H] + (int64_t)(t - 1) * hidden_size;
      fa.cprev = gates_out[ADMM_C] + (int64_t)(t - 1) * hidden_size;
      fa.hout = gates_out[ADMM_H] + (int64_t)t * hidden_size;
      fa.cout = gates_out[ADMM_C] + (int64_t)t * hidden_size;
      fa.hprev_stride = fa.cprev_stride = fa.hout_stride = fa.cout_stride = rs;
      for (int q = 0; q < 4; ++q) fa.gout[q] = gates_out[q] + (int64_t)t * hidden_size;
      fa.gout_stride = rs;
    } else {
      fa.hprev = h_scratch + ((t - 1) & 1) * BH;
      fa.cprev = c_scratch + ((t - 1) & 1) * BH;
      fa.hout = h_scratch + (t & 1) * BH;
      fa.cout = c_scratch + (t & 1) * BH;
      fa.hprev_stride = fa.cprev_stride = fa.hout_stride = fa.cout_stride = hidden_size;
    }
    fa.zc = z_out;
    launch_forward_t(g, t, w, fa, s);
  }
  if (gates_out)
    launch_rowdot(batch, hidden_size, output_size, gates_out[ADMM_H] + (int64_t)seq_len * hidden_size, rs, wy, out_a,
                  s);
  else
    launch_rowdot(batch, hidden_size, output_size, h_scratch + (seq_len & 1) * BH, hidden_size, wy, out_a, s);
  HIP_TRY(hipGetLastError());
  return ADMM_OK;
}

}  // extern "C"
