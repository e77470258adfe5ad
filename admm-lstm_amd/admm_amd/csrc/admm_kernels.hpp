// admm_kernels.hpp -- launch interface between the host orchestration (admm_host.hip)
// and the gfx950 kernels (admm_kernels.hip).  Plain pointers only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace admm {

constexpr int kTrialJ = 16;      // line-search candidates evaluated per trial pass
// per-gate sums of a trial pass: [J candidates][10 polynomial coefficients][sum d0^2][#per-candidate elements]
constexpr int kPolyN = 10;
// |q| bound of the polynomial (5-term Taylor) regime, 2^-KPOLYQ_LOG2 (admm_kernels.hip "Trial pass")
#ifndef KPOLYQ_LOG2
#define KPOLYQ_LOG2 4
#endif
constexpr float kPolyQ = 1.0f / (float)(1 << KPOLYQ_LOG2);
// + pass 0's second polynomial (kPolyHiN coefficients of s^2..s^10 over the per-candidate
// elements, valid for k >= kTrialJ) and the count of elements it cannot cover
constexpr int kPolyHiN = 9;
constexpr int kTrialSlots = kTrialJ + kPolyN + 2 + kPolyHiN + 1;
constexpr int kMaxK = 96;        // exponents decided from the polynomial alone go up to this
constexpr int kMaxPasses = 4;    // => exponents k in [0, 64)
constexpr int kTailPass = -1;    // trial / select "pass" covering windows 1 .. kMaxPasses - 1 in one launch
constexpr int kFastD = 16;       // fused weight-stage path for input_size <= 16
constexpr int kHTCand = 4;       // theta = 0.1, 0.2, 0.4, 0.8 (admm.py:447-480)
constexpr int kHTSums = 1 + 3 * kHTCand;

// n / d for 0 <= n < 2^31 by multiply-high (Granlund-Montgomery): no integer division in
// the GEMM operand loaders.  make() runs on the host.
struct DivU32 {
  uint32_t m = 1;
  int s = 0;
  static DivU32 make(uint32_t d) {
    DivU32 r;
    int l = 0;
    while ((1ull << l) < d) ++l;
    r.s = l;
    r.m = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
    return r;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(m, n) + n) >> s; }
};

struct Geom {
  int64_t B;    // local rows
  int64_t Bg;   // global rows (a-update constant)
  int T, D, H, O;
  DivU32 dT{};  // by T; set with set_T() (B*T < 2^31 is checked at create)
  // test hook read from the environment once per context (admm_create): ADMM_SWEEP_R16=0 runs
  // 256 < H <= 512 on the per-t sweep (the path of the other widths) to compare the two
  bool r16 = true;
  __host__ __device__ int64_t BT() const { return B * (int64_t)T; }
  __host__ __device__ int TP() const { return T + 1; }
  void set_T() { dT = DivU32::make((uint32_t)T); }
  // row (b, t) of the [B][T] grid -> row of the h plane [B][T+1] holding h_{t-1}: b*(T+1) + t
  __device__ __forceinline__ int64_t hrow(int64_t row) const { return row + dT.div((uint32_t)row); }
};

struct Weights {            // model parameters, read in place (no packing)
  const float* wx[4];
  const float* wh[4];
};

struct Planes6 { float* p[6]; };

struct Hyper {
  float rho[7];             // i f g o c h y
  float beta_x[4], beta_h[4], beta_y;
  int variant;              // 0 admm, 1 no_dual_y
  int with_dual_y;
  // 1/rho of gates i, f, g, o when all four rho are powers of two (then lam * (1/rho) is
  // exact and equals the IEEE quotient lam / rho bit for bit), else 0: tgt_quot's fast form
  float rinv_gate[4];
  int rinv_exact;
};

// Device-side diagnostics, copied out by admm_get_stats.
struct DevStats {
  int k[8];
  int passes[2];
  int unresolved;
  int nonfinite;
  float theta_h;
  int handoff_fail;         // column-split sweep: hand-off waits that timed out (the step's state is invalid)
  double f_w[8];
  double grad_sq[8];
  double direct_frac[8];
  // admm_debug_force: the exponents (and h_T theta) the step would have taken itself
  int k_own[8];
  float theta_h_own;
  int sweep_fallback;       // column-split sweep launches whose grid was not resident (the row-block sweep ran)
};

// ---- time step (one t): GEMM [x_t | h_{t-1}] @ [Wx; Wh] for the 4 gates + fused epilogue
struct ForwardT {
  const float* x;           // [B,T,D]
  const float* hprev; int64_t hprev_stride;   // row b of h_{t-1} at hprev + b*stride
  const float* cprev; int64_t cprev_stride;
  float* hout; int64_t hout_stride;
  float* cout; int64_t cout_stride;
  float* gout[4]; int64_t gout_stride;        // i,f,g,o at t (nullable)
  float* zc;                                  // [4][B*T][H] (nullable)
};
void launch_forward_t(const Geom& g, int t, const Weights& w, const ForwardT& a, hipStream_t s);

struct SweepT {
  const float* x;
  Planes6 S, L;             // [B,T+1,H] each
  float* zc;                // [4][B*T][H]: z cache for the next step's first weight stage
  float* tgt;               // [4][B*T][H]: lam/rho + S of the updated state (k_sweep_rows; nullable)
  float* gx_slab;           // [blocks][4][D][H]: next x stage's X^T R partials (k_sweep_rows, D <= 16; nullable)
  const int* lamh_nz;       // k_sweep_rows: device flag, 0 = dual h is zero at every t < T (nullable: unknown)
  // k_sweep_rows (nullable): running maxima, as float bits under atomicMax (zeroed beforehand), of
  // the next step's weight-phase operands: [q] = max |phi(z) - tgt| of gate q (the x stage's
  // residual before phi'), [4] = max |h_{t-1}| over t = 1..T (the h stage's H_prev).  They bound
  // the h-side residual so k_atr3w can scale its fp16 operands (admm_split3.hip, kRange*)
  float* range;
  // column-split sweep (sweep_rows_nc > 1): the h_t granules of every padded row block
  // (sweep_xbuf_bytes), zeroed by launch_sweep_wt; fail (nullable) counts hand-off waits that timed
  // out (DevStats::handoff_fail: the step's results are invalid and the host raises), fallback
  // (nullable) the launches whose grid was not all resident (DevStats::sweep_fallback)
  void* xbuf;
  int* fail;
  int* fallback;
  // test hook (admm_debug_fault): row block 0's column group 1 skips its publish of h_1, so that
  // the other groups' hand-off waits time out
  int skip_publish;
  // the row-block sweep launched after a column-split one (launch_sweep_rows): runs only if that
  // launch found its workgroups not all resident and left without touching the state (nullable)
  const unsigned* gate;
  int64_t r0, r1;           // sample rows [r0, r1) of this launch
};
void launch_sweep_t(const Geom& g, int t, const Weights& w, const Hyper& hp, const SweepT& a, hipStream_t s);
// Whole sweep in one persistent launch (k_sweep_rows): eligible when sweep_rows_ok(g).
// wt: sweep_wt_floats(g) floats, filled by launch_sweep_wt from the current weights.
bool sweep_rows_ok(const Geom& g);
bool sweep_rows_gx_ok(const Geom& g);   // ... and it can form the x stage's G_x partials (32-row tiles with D <= 16, 16-row tiles with D == 1)
int sweep_rows_blocks(const Geom& g);   // its workgroups = its G_x slabs
size_t sweep_wt_floats(const Geom& g);
// column groups of the 32-row persistent sweep (1: row blocks only), its padded row blocks and its
// hand-off buffer (SweepT::xbuf); the column split needs every one of its workgroups resident at
// once: kSweepCUs (one 140-KB-LDS workgroup per CU) bounds the grid, and the host checks the device
constexpr int kSweepCUs = 256;
int sweep_rows_nc(const Geom& g);
// test hook: poison the column split's entry count in xbuf (after launch_sweep_wt zeroed it), so
// that its launch leaves at once and the gated row-block sweep runs
void sweep_poison_entry(const Geom& g, void* xbuf, hipStream_t s);
int sweep_row_blocks_padded(const Geom& g);
size_t sweep_xbuf_bytes(const Geom& g);
// xbuf (nullable): zeroed in the same launch (before a column-split sweep)
void launch_sweep_wt(const Geom& g, const Weights& w, float* wt, hipStream_t s, void* xbuf = nullptr);
int sweep_wt_rows16(const Geom& g);   // the image layout of launch_sweep_wt: 1 = 16-row tiles
int sweep_wt_xc(const Geom& g);       // its x chunks
void launch_sweep_rows(const Geom& g, const float* wt, const Hyper& hp, const SweepT& a, hipStream_t s);
// flag |= 1 if lh[b][t][j] != 0 for some t in [1, T) (H % 4 == 0; flag zeroed by the caller)
void launch_check_lamh(const Geom& g, const float* lh, int* flag, hipStream_t s);


// out[b][o] = h_row(b) . wy[:, o]
void launch_rowdot(int64_t B, int H, int O, const float* h, int64_t h_stride, const float* wy, float* out,
                   hipStream_t s);

// ---- weight stage (4 gates at once)
// z cache recompute over all rows: zc[q] = X Wx_q + Hprev Wh_q
void launch_zgemm(const Geom& g, const Weights& w, const float* x, const float* Sh, float* zc, hipStream_t s);

struct ResidArgs {
  int stage;                // 0 = x side, 1 = h side
  const float* x;
  Planes6 S, L;
  float* zc;                // read (stage 0) / read-modify-write (stage 1: += X dWx)
  float* tgt;               // written (stage 0) / read (stage 1); [4][BT][H] = L/rho + S
  float* R;                 // [4][BT][H] residual (phi(z) - tgt) * phi'(z)
  const float* dW;          // [4][D][H] (stage 1)
  int nblk;
};
int resid_blocks(const Geom& g);
void launch_resid(const Geom& g, const Hyper& hp, const ResidArgs& a, hipStream_t s);

// Gslab[split][q][m][j] = sum_{rows in split} A[row][m] * R[q][row][j], A = X (side 0) or Hprev (side 1)
int atr_splits(const Geom& g, int side);
void launch_atr(const Geom& g, int side, const float* x, const float* Sh, const float* R, float* Gslab,
                int nsplit, hipStream_t s);
// G[q][m][j] = rho_q * sum_split Gslab; also clears found[0..3] for the stage's line searches
// kpred (nullable, side 0): receives the previous step's x-side exponents from stats (SpecX)
void launch_reduce_g(const Geom& g, int side, const Hyper& hp, const float* Gslab, int nsplit, float* G, int* found,
                     int* kpred, const DevStats* stats,
                     hipStream_t s,
                     bool p16 = true, float* range_reset = nullptr);   // range_reset: zero range[0..4] (SweepT::range)
// h side, one process, split3 Q GEMM: launch_reduce_g's G (bitwise the same) and, in the same launch,
// the split G image that launch_qgemm3 would form (gimg: split3_gimg_floats(g); H % 32 == 0)
void launch_reduce_gh_img(const Geom& g, const Hyper& hp, const float* slab, int nsplit, float* G, int* found,
                          const DevStats* stats, hipStream_t s, bool p16, float* range_reset, float* gimg);
// Q[q][row][j] = sum_m A[row][m] * G[q][m][j]
void launch_qgemm(const Geom& g, int side, const float* x, const float* Sh, const float* G, float* Q,
                  hipStream_t s);

// trial pass: part[q][jj][blk] = sum over elements of inc(k = pass*J + jj)
int trial_blocks(const Geom& g);
void launch_trial(const Geom& g, int pass, const float* zc, const float* tgt, const float* Q, const int* found,
                  double* part, int nblk, hipStream_t s);
// test hook: part[blk][J] for caller-provided z, tgt, q of one gate
void launch_trial_debug(int64_t n, int tanh_gate, int kbase, const float* z, const float* tgt, const float* q,
                        double* part, int nblk, hipStream_t s);
// test hook: R[4][BT][H] = (phi(z) - tgt) phi'(z) with the activation every stage forms it with (phi_acc)
void launch_debug_resid(const Geom& g, const float* z, const float* tgt, float* R, hipStream_t s);
// sums[q][0..J) = sum_blk part[q][k] ; sums[q][J] = sum d0^2 (= 2 f(W)/rho)
void launch_trial_reduce(const Geom& g, int pass, const double* part, int nblk, const int* found, double* sums,
                         hipStream_t s);

// ---- fast weight-stage path (D <= 16, H % 4 == 0): fused residual/gradient kernels
bool fast_path(const Geom& g);
int resid_gx_blocks(const Geom& g);
// x stage: tgt = lam/rho + S (stored) and slab[blk][q][d][j] = sum_rows x[row][d] R_q[row][j]
// tgt_ready: tgt already holds lam/rho + S of this state (written by the persistent sweep):
// read instead of S and L, and not rewritten
void launch_resid_gx(const Geom& g, const Hyper& hp, const float* x, const Planes6& S, const Planes6& L,
                     const float* zc, float* tgt, float* slab, int nblk, bool tgt_ready, hipStream_t s);
// trial pass without a materialised Q (side 0: q = x.G_x) or z (side 1: z = zc + x.dWx)
// Speculative Gauss-Seidel z update of the x stage (H % 256 == 0): pass 0 of the x-side trials
// also writes zx = zc + x dWx(kpred) for the exponent the gate took in the previous step
// (kpred, copied from the stats by k_reduce_g), with dWx formed exactly as k_select forms it;
// k_apply_fix recomputes zx only for the gates whose decided exponent differs.
struct SpecX {
  const int* kpred;         // [4] predicted x-side exponent per gate
  const float* W[4];        // x2q before the update
  float* zx;                // [4][BT][H] z of the h stage (zc + x dWx)
  Hyper hp;
};
// fsel, fhp, fcount (one process, pass == kTailPass, tail_select_fused): the tail launch also makes
// the tail's selection (k_select's work, by the last workgroup of each gate; fcount: [4] zeroed
// counters the kernel re-arms), so no launch_select follows it
struct SelectArgs;
void launch_trial_fast(const Geom& g, int side, int pass, const float* zc, const float* tgt, const float* Q,
                       const float* x, const float* Wsrc, const int* found, double* part, int nblk, hipStream_t s,
                       const SpecX* spec = nullptr, int qpair = 0, const SelectArgs* fsel = nullptr,
                       const Hyper* fhp = nullptr, unsigned* fcount = nullptr);
bool tail_select_fused(const Geom& g, int side);
// after the x decision: zx = zc + X dWx for the gates whose exponent was mispredicted
void launch_apply_fix(const Geom& g, const float* x, const float* dW, const float* zc, float* zx, const int* kpred,
                      const DevStats* stats, hipStream_t s);
int stream_blocks(const Geom& g);   // grid (per gate) of the fast streaming passes
// H % 256 == 0: the fast trial passes run as row-pair workgroups over H/256 column blocks, and
// write stream_blocks(g) * H/256 partials per slot (the reduce's nblk)
bool trial_rows_ok(const Geom& g);
// H % 256 == 0, D <= 16: the x-side trial passes run on the matrix cores (k_trial_mx) over
// H/128 column groups, writing stream_blocks(g) * H/128 partials per slot
bool trial_mx_ok(const Geom& g);
int trial_fast_blocks(const Geom& g, int side);   // the fast trial passes' workgroups per gate (nblk)

// after the x stage (fast path): zc += X dWx
void launch_apply_dwx(const Geom& g, const float* x, const float* dW, float* zc, hipStream_t s);
// h stage A^T R with R computed on the fly from zc (already updated) and tgt (side 1, fast path)
void launch_atr_fused(const Geom& g, const Hyper& hp, const float* x, const float* Sh, const float* zc,
                      const float* tgt, const float* dW, float* slab, int nsplit, hipStream_t s);
// h stage on bf16 matrix cores with three-way split f32 operands (admm_split3.hip), H % 256 == 0:
// slab[sp][q][m][j] = sum_rows Hprev[row][m] R_q[row][j] (R from zc, tgt), and Q = Hprev G
// (gimg: split3_gimg_floats(g) floats of workspace for the split G image)
bool split3_ok(const Geom& g);
size_t split3_gimg_floats(const Geom& g);
int atr3_splits(const Geom& g);
// range, dW non-null: k_atr3w on scaled-fp16 two-way splits, with the operand ranges the persistent
// sweep left (SweepT::range, plus [5] = max_row sum_d |x_d|) and the x stage's decided update dW
// [4][D][H]; else on split3 (both f32-accurate).  wide_ok: the fp16 path at H = 512 takes 512 x 128
// tiles instead of 256 x 256 (bit-identical slabs)
void launch_atr3(const Geom& g, const float* Sh, const float* zc, const float* tgt, float* slab, int nsplit,
                 hipStream_t s, const float* range = nullptr, const float* dW = nullptr, bool wide_ok = true);
// range[5] = max over rows of sum_d |x[row][d]| (atomicMax into a zeroed slot)
void launch_x_l1max(const Geom& g, const float* x, float* range, hipStream_t s);
// Q = Hprev G, the h-side trial direction: Hprev in two bf16 pieces, G rounded to bf16 (it enters
// only the line-search remainder, DESIGN.md "trial direction precision").  Layout: bf16 row quads
// [q][row / 4][j][row % 4] when qpair_ok (BT % 4 == 0), else row-major f32 -- launch_trial_fast's
// qpair argument is q_layout(g).  H = 256 (qres_ok): k_qgemm_res, the G image resident in LDS;
// otherwise the staged k_qgemm3<1, layout>.
bool qpair_ok(const Geom& g);
bool qres_ok(const Geom& g);
int q_layout(const Geom& g);   // 2 (bf16 row quads) or 0 (row-major f32)
// gimg_ready: the image was already formed (launch_reduce_gh_img)
void launch_qgemm3(const Geom& g, const float* Sh, const float* G, float* gimg, float* Q, hipStream_t s,
                   bool gimg_ready = false);
// decide the first passing k in this pass's window; on success update the weights
struct SelectArgs {
  int side;                 // 0 x, 1 h
  int pass, last_pass;
  const double* part;       // [4][kTrialSlots][nred] per-block partials of this pass (single process), or
  int nred;
  const double* sums;       // [4][kTrialSlots] all-reduced sums of this pass (part == nullptr)
  double* poly;             // [4][kPolyN] polynomial coefficients kept from pass 0
  const float* G;           // [4][K][H]
  float* W[4];              // weights being updated (in place)
  float* dW;                // [4][K][H] W_new - W_old (side 0), nullable
  const int* found_in;      // [4] decided before this pass (found + 4 (pass & 1))
  int* found_out;           // [4] decided after it (found + 4 ((pass + 1) & 1))
  int* pick;                // [4] exponent chosen in this pass, -1 if none
  DevStats* stats;
  const int* force;         // [8] forced exponents per (gate, side) (admm_debug_force; nullable)
  // the persistent sweep's weight image (launch_sweep_wt's layout; nullable): every updated weight
  // element's three split pieces are written there too, so the image of the new weights is ready for
  // the sweep without a k_sweep_wt launch (every element of every gate weight is updated each step)
  void* wt;
  int wt_rows16;            // its layout: 16-row (H > 256) or 32-row tiles
  int wt_xc;                // x chunks of the image (sweep_xc)
};
void launch_select(const Geom& g, const Hyper& hp, const SelectArgs& a, hipStream_t s);

// ---- output weight wy (admm.py:246-280; admm.no_dual_y.py:226-249)
int wy_splits(const Geom& g);
// u_ready: U already holds this state's residual (k_ht_apply of the previous step wrote it)
void launch_wy_grad(const Geom& g, const Hyper& hp, const float* Sh, const float* a, const float* Ly,
                    const float* wy, float* U, float* slab, int nsplit, hipStream_t s, bool u_ready = false);
// wy_apply non-null: also wy <- update(wy, G_y) in the same launch (no all-reduce of G_y needed)
void launch_wy_reduce(const Geom& g, const Hyper& hp, const float* slab, int nsplit, float* Gy, float* wy_apply,
                      hipStream_t s);
void launch_wy_apply(const Geom& g, const Hyper& hp, const float* Gy, float* wy, hipStream_t s);

// ---- h_T search (admm.py:459-487; admm.no_dual_y.py:426-449), a update, duals at T
int ht_blocks(const Geom& g);
void launch_ht_partial(const Geom& g, const Hyper& hp, const Planes6& S, const Planes6& L, const float* a,
                       const float* Ly, const float* wy, double* part, int nblk, hipStream_t s);
void launch_ht_reduce(const double* part, int nblk, double* sums, hipStream_t s);
// U: also the next wy stage's residual; xbuf (nullable): also zero the column-split sweep's hand-off
// buffer (sweep_xbuf_bytes) for the next step's sweep
void launch_ht_apply(const Geom& g, const Hyper& hp, const Planes6& S, const Planes6& L, float* a, float* Ly,
                     const float* y, const float* wy, const double* sums, DevStats* stats, int* status, hipStream_t s,
                     const int* force = nullptr, float* U = nullptr, void* xbuf = nullptr);

}  // namespace admm
