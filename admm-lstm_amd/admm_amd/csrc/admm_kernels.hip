// admm_kernels.hip -- gfx950 kernels of the ADMM-LSTM update step.
//
// Reference semantics (Frederick2309/ADMM-LSTM):
//   time step / LSTM forward ........ blocks/lstm.py:65-88, admm.py:345-386, 388-457, 504-539
//   weight-stage residual + gradient  admm.py:302-314
//   line-search trials / selection .. admm.py:316-343
//   output weight wy ................ admm.py:246-280, admm.no_dual_y.py:226-249
//   h_T search, a, duals at T ....... admm.py:459-502, 532-546, admm.no_dual_y.py:414-456
// Layouts: gates/duals [B][T+1][H] (the reference's), caches [4][B*T][H] (row = b*T + t-1).
#include <cstdio>
#include <cstdlib>

#include "admm_dev.hpp"
#include "admm_kernels.hpp"
#include <type_traits>

namespace admm {

namespace {

inline int cdiv64(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Calls f(integral_constant<DP>, integral_constant<XV>) for the padded input width of g.
template <class F>
void with_dp(const Geom& g, F&& f) {
  using std::integral_constant;
  const bool xv = (g.D % 4) == 0;
  switch ((g.D + 3) / 4) {
    case 1: xv ? f(integral_constant<int, 4>{}, std::true_type{}) : f(integral_constant<int, 4>{}, std::false_type{}); break;
    case 2: xv ? f(integral_constant<int, 8>{}, std::true_type{}) : f(integral_constant<int, 8>{}, std::false_type{}); break;
    case 3: xv ? f(integral_constant<int, 12>{}, std::true_type{}) : f(integral_constant<int, 12>{}, std::false_type{}); break;
    default: xv ? f(integral_constant<int, 16>{}, std::true_type{}) : f(integral_constant<int, 16>{}, std::false_type{}); break;
  }
}


// ============================================================================ time step
// Tile: 128 rows (samples) x 128 columns = 4 gates x 32 hidden units; each wave owns 32
// rows x all 4 gates, so gate q's pre-activation of (b, j) sits in the same lane for every
// q and the element-wise ADMM updates run straight out of the accumulators.
constexpr int TS_BM = 128, TS_BN = 128, TS_WM = 32, TS_WN = 128, TS_KC = 32;
using TSTile = Tile<TS_BM, TS_BN, TS_WM, TS_WN, TS_KC, true>;

__device__ __forceinline__ const float* pick4(const float* const (&p)[4], int q) {
  return q == 0 ? p[0] : (q == 1 ? p[1] : (q == 2 ? p[2] : p[3]));
}

// B operand of every "z" GEMM: [Wx_q; Wh_q] of the 4 gates, column n = 32*q + (j - j0).
template <bool VEC>
__device__ __forceinline__ float4 weights4(const Weights& w, int D, int H, int j0, int64_t k, int64_t n) {
  const int q = (int)(n >> 5), j = j0 + (int)(n & 31);
  const int K = D + H;
  if (VEC) {
    if (k >= K || j >= H) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* base = k < D ? pick4(w.wx, q) + k * H : pick4(w.wh, q) + (k - D) * H;
    return *reinterpret_cast<const float4*>(base + j);
  }
  float v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int jj = j + u;
    v[u] = (k < K && jj < H && (jj - j0) < 32 * (q + 1))
               ? (k < D ? pick4(w.wx, q)[k * H + jj] : pick4(w.wh, q)[(k - D) * H + jj])
               : 0.f;
  }
  return make_float4(v[0], v[1], v[2], v[3]);
}

template <bool VEC>
struct StepSrc {  // A = [x_t | h_{t-1}] rows (row-major, K = D + H)
  const float* x; int64_t x_stride;
  const float* h; int64_t h_stride;
  int64_t B; int D, H;
  Weights w; int j0;
  static constexpr bool A_ROW_MAJOR = true;
  __device__ float4 a4(int64_t m, int64_t k) const {
    const int K = D + H;
    if (VEC) {
      if (m >= B || k >= K) return make_float4(0.f, 0.f, 0.f, 0.f);
      const float* src = k < D ? x + m * x_stride + k : h + m * h_stride + (k - D);
      return *reinterpret_cast<const float4*>(src);
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t kk = k + u;
      v[u] = (m < B && kk < K) ? (kk < D ? x[m * x_stride + kk] : h[m * h_stride + (kk - D)]) : 0.f;
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ float4 b4(int64_t k, int64_t n) const { return weights4<VEC>(w, D, H, j0, k, n); }
};

template <bool VEC>
__device__ __forceinline__ void step_gemm(const Geom& g, int t, const Weights& w, const float* hprev, int64_t hstride,
                                          const float* x, f32x16 (&acc)[1][4], float* smem, int64_t m0, int j0,
                                          int64_t rend) {
  StepSrc<VEC> src{x + (int64_t)(t - 1) * g.D, (int64_t)g.T * g.D, hprev, hstride, rend, g.D, g.H, w, j0};
  Engine<TS_BM, TS_BN, TS_WM, TS_WN, TS_KC, StepSrc<VEC>> eng;
  eng.run(src, m0, 0, 0, g.D + g.H, acc, smem);
}

template <bool VEC>
__global__ __launch_bounds__(kThreads) void k_forward_t(Geom g, int t, Weights w, ForwardT a) {
  __shared__ float smem[TSTile::LDS_FLOATS];
  const int nj = (g.H + 31) / 32;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)(lid / nj) * TS_BM;
  const int j0 = (lid % nj) * 32;
  f32x16 acc[1][4];
  zero_acc(acc);
  step_gemm<VEC>(g, t, w, a.hprev, a.hprev_stride, a.x, acc, smem, m0, j0, g.B);
  const int lane = threadIdx.x & 63, wm0 = (threadIdx.x >> 6) * TS_WM;
  const int j = j0 + (lane & 31);
  if (j >= g.H) return;
  const int64_t BT = g.BT();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t b = m0 + wm0 + acc_row(r, lane);
    if (b >= g.B) continue;
    const float zi = acc[0][0][r], zf = acc[0][1][r], zg = acc[0][2][r], zo = acc[0][3][r];
    const float gi = sigm(zi), gf = sigm(zf), gg = tanhf(zg), go = sigm(zo);
    const float cp = a.cprev[b * a.cprev_stride + j];
    const float c = gf * cp + gi * gg;
    const float h = go * tanhf(c);
    a.cout[b * a.cout_stride + j] = c;
    a.hout[b * a.hout_stride + j] = h;
    if (a.gout[0]) {
      a.gout[0][b * a.gout_stride + j] = gi;
      a.gout[1][b * a.gout_stride + j] = gf;
      a.gout[2][b * a.gout_stride + j] = gg;
      a.gout[3][b * a.gout_stride + j] = go;
    }
    if (a.zc) {
      const int64_t e = (b * g.T + (t - 1)) * g.H + j;
      a.zc[e] = zi; a.zc[BT * g.H + e] = zf; a.zc[2 * BT * g.H + e] = zg; a.zc[3 * BT * g.H + e] = zo;
    }
  }
}

// The line-search target tgt = lam / rho + S of a gate (the lam/rho + S term of the residual,
// admm.py:302-312), written by k_resid_gx or by the persistent sweep: one expression (IEEE
// division, as the reference) so that either source gives equal bits.
__device__ __forceinline__ f32x4 tgt_quot(f32x4 lam, float rho, f32x4 s) { return lam / rho + s; }
// The same value when rho is a power of two (Hyper::rinv_exact): lam * 2^-k is exact, so it
// equals the correctly rounded quotient; __fmul_rn keeps the product out of an fma with s.
__device__ __forceinline__ f32x4 tgt_mulq(f32x4 lam, float rinv, f32x4 s) {
  f32x4 q;
#pragma unroll
  for (int u = 0; u < 4; ++u) q[u] = __fmul_rn(lam[u], rinv);
  return q + s;
}

// ---- one (b, j) point of the time sweep: i, f, g, o (admm.py:353-386), c (388-436),
// h for t < T (455-457), duals of i, f, g, o, c (504-530).  Operand grouping follows the
// reference expression by expression (fp32).
struct SweepIn {
  float zi, zf, zg, zo;       // pre-activations x_t Wx_q + h_{t-1} Wh_q
  float f0, g0, c0, h0, cp;   // old f, g, c, h at t; new c at t-1
  float li, lf, lg, lo, lc, lh;
};
struct SweepRes {
  float i1, f1, g1, o1, c1, h1;
  float li, lf, lg, lo, lc;
  // phi'(z) of the four pre-activations (the next x stage's residual, k_sweep_rows GX)
  float di, df, dg, dO;
  float ai, af, ag, ao;    // phi(z)
};

__device__ __forceinline__ SweepRes sweep_point(const Hyper& hp, const SweepIn& v, bool last) {
  const float ri = hp.rho[0], rf = hp.rho[1], rg = hp.rho[2], ro = hp.rho[3], rc = hp.rho[4], rh = hp.rho[5];
  const SigPair pi = sig_pair(v.zi), pf = sig_pair(v.zf), po = sig_pair(v.zo);
  const float ai = pi.s, af = pf.s, ag = tanhf(v.zg), ao = po.s;
  const float f0 = v.f0, g0 = v.g0, c0 = v.c0, h0 = v.h0, cp = v.cp;
  const float li = v.li, lf = v.lf, lg = v.lg, lo = v.lo, lc = v.lc, lh = v.lh;
  SweepRes o;
  // admm.py:384-386 with (p1,p2,p3) of :360-375 and (var2, rho2, lam2) of :376-383
  o.i1 = div_fast(-((li - ri * ai) + (rc * (f0 * cp - c0) - lc) * g0), ri + rc * g0 * g0);
  o.f1 = div_fast(-((lf - rf * af) + (rc * (g0 * o.i1 - c0) - lc) * cp), rf + rc * cp * cp);
  o.g1 = div_fast(-((lg - rg * ag) + (rc * (o.f1 * cp - c0) - lc) * o.i1), rg + rc * o.i1 * o.i1);
  const float tc0 = tanhf(c0);
  o.o1 = div_fast(-((lo - ro * ao) + (rh * (0.f - h0) - lh) * tc0), ro + rh * tc0 * tc0);
  // admm.py:388-436: autograd gradient of .5||tanh(c) o - (h + lam_h/rho_h)||^2, theta* = 0.5
  const float div_h = div_fast(lh, rh), div_c = div_fast(lc, rc);
  const float vv = tc0 * o.o1 - (h0 + div_h);
  const float gc = (vv * o.o1) * (1.f - tc0 * tc0);
  const float A = (div_c - o.f1 * cp) - o.i1 * o.g1;
  o.c1 = div_fast(0.5f * c0 - gc - rc * A, rc + 0.5f);
  o.h1 = last ? h0 : div_fast(rh * o.o1 * tanhf(o.c1) - lh, rh);  // admm.py:455-457
  // admm.py:512-530
  o.li = li + ri * (o.i1 - ai);
  o.lf = lf + rf * (o.f1 - af);
  o.lg = lg + rg * (o.g1 - ag);
  o.lo = lo + ro * (o.o1 - ao);
  o.lc = lc + rc * (o.c1 - (o.f1 * cp + o.i1 * o.g1));
  o.ai = ai; o.af = af; o.ag = ag; o.ao = ao;
  o.di = pi.s * pi.sc; o.df = pf.s * pf.sc; o.dg = 1.f - ag * ag; o.dO = po.s * po.sc;
  return o;
}

// c_t and h_t are read back at t+1 (c_{t-1} of the update, h_{t-1} of the next GEMM): cached
// stores; everything else is streamed.
__device__ __forceinline__ void sweep_store(const SweepT& a, const SweepRes& o, int64_t ot, bool last) {
  st_nt(a.S.p[0] + ot, o.i1); st_nt(a.S.p[1] + ot, o.f1); st_nt(a.S.p[2] + ot, o.g1); st_nt(a.S.p[3] + ot, o.o1);
  a.S.p[4][ot] = o.c1;
  if (!last) a.S.p[5][ot] = o.h1;
  st_nt(a.L.p[0] + ot, o.li); st_nt(a.L.p[1] + ot, o.lf); st_nt(a.L.p[2] + ot, o.lg); st_nt(a.L.p[3] + ot, o.lo);
  st_nt(a.L.p[4] + ot, o.lc);
}

// One ADMM time step t (admm.py:72-76): i, f, g, o (admm.py:353-386), c (388-436),
// h for t < T (455-457), dual ascent for i, f, g, o, c (504-530).  h_T, a and the
// duals of h at T are finished by the h_T kernels below.
#ifndef SWEEP_AHEAD
#define SWEEP_AHEAD 1   // points whose operands are in flight while one is computed
#endif
template <bool VEC>
__global__ __launch_bounds__(kThreads) void k_sweep_t(Geom g, int t, Weights w, Hyper hp, SweepT a) {
  __shared__ float smem[TSTile::LDS_FLOATS];
  const int nj = (g.H + 31) / 32;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t m0 = a.r0 + (int64_t)(lid / nj) * TS_BM;
  const int j0 = (lid % nj) * 32;
  const int64_t rs = (int64_t)g.TP() * g.H;  // row stride of a [B,T+1,H] plane
  f32x16 acc[1][4];
  zero_acc(acc);
  step_gemm<VEC>(g, t, w, a.S.p[5] + (int64_t)(t - 1) * g.H, rs, a.x, acc, smem, m0, j0, a.r1);
  const int lane = threadIdx.x & 63, wm0 = (threadIdx.x >> 6) * TS_WM;
  const int j = j0 + (lane & 31);
  if (j >= g.H) return;
  const int64_t BT = g.BT();
  const bool last = (t == g.T);
  // The operands of point r+1 are loaded before point r's results are stored: vmcnt counts
  // loads and stores in order, so a load issued after the stores would wait for them too
  // (one full memory round trip per point).
  // Rows past r1 load row r1-1 (branch-free, so the prefetched registers need no phi copies).
  auto load_pt = [&](int r, SweepIn& v) {
    const int64_t b = min(m0 + wm0 + acc_row(r, lane), a.r1 - 1);
    const int64_t ot = b * rs + (int64_t)t * g.H + j;
    v.f0 = ld_nt(a.S.p[1] + ot, 0); v.g0 = ld_nt(a.S.p[2] + ot, 0); v.c0 = ld_nt(a.S.p[4] + ot, 0);
    v.h0 = ld_nt(a.S.p[5] + ot, 0);
    v.cp = a.S.p[4][ot - g.H];   // written at t-1 by this sweep: keep it cacheable
    v.li = ld_nt(a.L.p[0] + ot, 0); v.lf = ld_nt(a.L.p[1] + ot, 0); v.lg = ld_nt(a.L.p[2] + ot, 0);
    v.lo = ld_nt(a.L.p[3] + ot, 0); v.lc = ld_nt(a.L.p[4] + ot, 0); v.lh = ld_nt(a.L.p[5] + ot, 0);
  };
  constexpr int kAhead = SWEEP_AHEAD;
  SweepIn ring[kAhead + 1];
#pragma unroll
  for (int r = 0; r < kAhead; ++r) load_pt(r, ring[r]);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (r + kAhead < 16) load_pt(r + kAhead, ring[(r + kAhead) % (kAhead + 1)]);
    SweepIn v = ring[r % (kAhead + 1)];
    const int64_t b = m0 + wm0 + acc_row(r, lane);
    const int64_t ot = b * rs + (int64_t)t * g.H + j;
    v.zi = acc[0][0][r]; v.zf = acc[0][1][r]; v.zg = acc[0][2][r]; v.zo = acc[0][3][r];
    const SweepRes o = sweep_point(hp, v, last);
    if (b >= a.r1) continue;
    sweep_store(a, o, ot, last);
    const int64_t e = (b * g.T + (t - 1)) * g.H + j;
    st_nt(a.zc + e, v.zi); st_nt(a.zc + BT * g.H + e, v.zf); st_nt(a.zc + 2 * BT * g.H + e, v.zg);
    st_nt(a.zc + 3 * BT * g.H + e, v.zo);
  }
}

// ---- the whole sweep in one persistent launch (H % 32 == 0, H <= 256, D <= 32) ----
// Samples are independent across t, so a workgroup owns 32 rows for all of t = 1..T and no
// grid-wide step is needed.  [x_t | h_{t-1}] of its rows lives in LDS (two buffers by t
// parity, already split into three bf16 pieces): h never makes an HBM round trip inside the
// sweep.  Eight waves, two roles, one tile (4 gates x 32 hidden units) per step:
//   waves 0-3 (producer, wave q = gate q): z tile of step s over K = 16*XC + H in 16-deep
//              chunks, each chunk 6 bf16 MFMAs of the split operands (split3: f32-accurate),
//              written to the LDS tile buffer s&1;
//   waves 4-7 (consumer): the element-wise ADMM update of tile s-1 (sweep_point), its HBM
//              loads issued one tile ahead, h_t split into the other LDS A-buffer.
// The producer's matrix pipe and the consumer's memory stream overlap on every SIMD.  At a
// t boundary the producer's tile (t+1, 0) needs h_t of the tile the consumer is finishing:
// it runs K up to that tile's 32 columns, meets the consumer at a mid-step barrier, then
// finishes the last two chunks.
// max over the wave of a non-negative v, folded into *dst (float bits, atomicMax: for values >= 0
// the integer order of the bits is the float order) by lane 0 -- a vector atomic
__device__ __forceinline__ void range_max(float* dst, float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned*>(dst), __float_as_uint(v));
}

#ifdef SR_CS_TIMING   // tools/kbench: per-t phase timestamps of the column-split sweep's workgroup 0
__device__ unsigned long long g_cs_t[64][12];
#define CS_STAMP(t, e) do { if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (t) < 64) g_cs_t[t][e] = wall_clock64(); } while (0)
#else
#define CS_STAMP(t, e) do { } while (0)
#endif

constexpr int SR_ROWS = 32, SR_THREADS = 512;
#ifndef SR_CS_ORDER
#define SR_CS_ORDER 1   // 0: the column split's producer ring as before round 6's fix (A/B builds)
#endif
#ifndef SR16_PRO_ORDER
#define SR16_PRO_ORDER 1   // 0: the 16-row producer's B-ring prologue in the scheduler's order (A/B builds)
#endif
#ifdef SR_TIMING
__device__ unsigned long long g_sr_wait[2048][2];   // per workgroup: cycles the producer / consumer wave 0 waited at barriers
#define SR_SYNC() do { const unsigned long long t0_ = clock64(); __syncthreads(); \
    if ((threadIdx.x & 63) == 0) sr_wait += clock64() - t0_; } while (0)
#else
#define SR_SYNC() __syncthreads()
#endif

// ROWS = 32: tiles of 32 rows x 32 columns, v_mfma_f32_32x32x16_bf16 over 16-deep chunks
//            (H <= 256: the two split A buffers of 32 rows fit the LDS).
// ROWS = 16: tiles of 16 rows x 64 columns, v_mfma_f32_16x16x32_bf16 over 32-deep chunks
//            (256 < H <= 512, the C5 shape; a gate's tile is four 16x16 products).
template <int NT, int XC, int ROWS = 32>
struct SrGeom {
  static constexpr int TW = ROWS == 32 ? 32 : 64;   // tile width (columns)
  static constexpr int KD = ROWS == 32 ? 16 : 32;   // chunk depth
  static constexpr int H = TW * NT, XK = KD * XC, K2 = XK + H;
  static constexpr int KC2 = K2 / KD;          // chunks per tile
  static constexpr int AST = K2 + 8;           // A row stride (bf16): 16-B reads conflict-free over 16 rows
  static constexpr int APIECE = ROWS * AST;    // one split piece of one A buffer
  static constexpr int GT = NT * KC2;          // chunks per t
  static constexpr int U = ROWS == 16 ? (GT % 2 == 0 ? 2 : 1)   // 12 bf16x8 per chunk: a 2-deep ring
                         : GT % 8 == 0 ? 8 : GT % 4 == 0 ? 4 : GT % 3 == 0 ? 3 : GT % 2 == 0 ? 2 : 1;
};

// B operand image: for gate q, tile n, chunk c, piece p and lane (h, c32) the 8 bf16
// pieces of W[16c + 8h + j][32n + c32], j = 0..7, W = [Wx_q zero-padded to 16*XC rows; Wh_q].
// ROWS = 16 image: for gate q, tile n, chunk c, column block jq, piece p and lane (kq, r16) the 8
// bf16 pieces of W[32c + 8kq + j][64n + 16jq + r16] (the v_mfma_f32_16x16x32_bf16 B fragment).
__global__ __launch_bounds__(kThreads) void k_sweep_wt16(int D, int H, int XC, Weights w, bf16x8* __restrict__ wt) {
  const int NT = H / 64, KC2 = XC + H / 32, XK = 32 * XC;
  const int total = 4 * NT * KC2 * 4 * 64;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < total; i += gridDim.x * kThreads) {
    const int lane = i & 63, jq = (i >> 6) & 3, c = (i >> 8) % KC2, n = (i / (256 * KC2)) % NT,
              q = i / (256 * KC2 * NT);
    const int jj = 64 * n + 16 * jq + (lane & 15), kb = 32 * c + 8 * (lane >> 4);
    bf16x8 p0, p1, p2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kb + j;
      const float v = k < XK ? (k < D ? w.wx[q][(int64_t)k * H + jj] : 0.f) : w.wh[q][(int64_t)(k - XK) * H + jj];
      __bf16 a0, a1, a2;
      split3(v, a0, a1, a2);
      p0[j] = a0; p1[j] = a1; p2[j] = a2;
    }
    const int base = ((((q * NT + n) * KC2 + c) * 4 + jq) * 3) * 64 + lane;
    wt[base] = p0; wt[base + 64] = p1; wt[base + 128] = p2;
  }
}

__global__ __launch_bounds__(kThreads) void k_sweep_wt(int D, int H, int XC, Weights w, bf16x8* __restrict__ wt,
                                                         uint4* __restrict__ xbuf, int nx) {
  const int NT = H / 32, KC2 = XC + 2 * NT, XK = 16 * XC;
  const int total = 4 * NT * KC2 * 64;
  // the column-split sweep's h_t granules start every launch with tag 0 (this kernel runs right
  // before it on the stream)
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < nx; i += gridDim.x * kThreads) xbuf[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < total; i += gridDim.x * kThreads) {
    const int lane = i & 63, c = (i >> 6) % KC2, n = (i / (64 * KC2)) % NT, q = i / (64 * KC2 * NT);
    const int jj = 32 * n + (lane & 31), h = lane >> 5;
    bf16x8 p0, p1, p2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * c + 8 * h + j;
      const float v = k < XK ? (k < D ? w.wx[q][(int64_t)k * H + jj] : 0.f) : w.wh[q][(int64_t)(k - XK) * H + jj];
      __bf16 a0, a1, a2;
      split3(v, a0, a1, a2);
      p0[j] = a0; p1[j] = a1; p2[j] = a2;
    }
    const int base = (((q * NT + n) * KC2 + c) * 3) * 64 + lane;
    wt[base] = p0; wt[base + 64] = p1; wt[base + 128] = p2;
  }
}

// GX (D <= 16): the sweep also forms the next step's x-stage gradient partials
// slab[blk][q][d][j] = sum_{its rows, t} x_t[row][d] R_q[row][j], R_q = (phi(z) - tgt) phi'(z) of
// the new state (admm.py:302-312, x side), so that x stage needs no residual pass.  The consumer
// leaves R of its tile in the z tile's LDS slot; two steps later the gate's producer wave folds
// it in with 16 v_mfma_f32_16x16x4_f32 (K = the tile's 32 rows, M = d, N = 32 columns) into a
// register ring of NT column tiles that turns once per tile.
// ROWS = 16 (D == 1): the producer has no registers to spare for that ring, and a one-column x
// makes the 16x16x4 fold mostly padding, so the consumer forms the partials: each lane takes
// x_t R_q of its four points for the four gates, a reduce-scatter over the wave's four rows (two
// xor shuffles) leaves lane (row r, column group) the four-row sum of gate r, which goes to an
// LDS slot of the tile (by step parity).  One step later, past the barrier, thread (wave q, lane
// j) adds the four waves' sums of gate q, column j of that tile in wave order into a register
// ring of the NT column tiles, and writes its slab entries at the end: a fixed summation order,
// 8 KB of LDS and NT registers.
// NC > 1 (ROWS = 32, the strong-scaling path: few rows per GPU): the column-split sweep.  Workgroup
// (rb, cg) owns the 32 rows of row block rb and the NTC = NT / NC column tiles cg NTC .. of every t,
// so that B = 1024 rows fill 32 x 8 = 256 CUs instead of 32.  [x_t | h_{t-1}] still lives whole in
// each workgroup's LDS; the NC workgroups of a row block exchange h_t through memory once per t as
// 8-byte granules {h value, tag t} (cdna_hip_programming.md Guideline 16, R2: the data is the flag):
// each consumer thread publishes its four h values with two 16-byte write-through (sc1) stores as
// soon as they are computed, and before the producer may start the h chunks of t + 1 the consumer
// waves re-read the other groups' granules (sc1 loads) until every tag is t, then split them into
// the A image.  No drain, counter or fence.  The granule buffer (a.xbuf) is zeroed by k_sweep_wt
// before every launch; all workgroups must be resident at once (the host checks the grid against
// the CUs), and every spin is bounded.
// Column-split entry consensus: the hand-off needs every workgroup of the grid resident at once.
// Each workgroup counts itself in and waits (bounded by the wall clock) for the whole grid; one
// that gives up poisons the count with a CAS against the value it last saw, so either the count
// reaches the grid size (all run) or it is poisoned first (every workgroup, late ones included,
// leaves before touching the state, and the row-block sweep launched next does the work instead).
constexpr unsigned kSweepPoison = 0x40000000u;
constexpr uint64_t kSweepArriveTicks = 200000;   // 2 ms of the 100 MHz wall clock
// A hand-off wait (exchange) that sees no tag t for this long gives up: 50 ms of the wall clock,
// against ~3 us per t in a healthy sweep.  The step is then invalid and counted (SweepT::fail).
// Only time this wave was running counts: a gap between two polls longer than kHandoffGapTicks
// (one poll takes ~1 us) means the dispatch was preempted or time-sliced -- the publishers were
// paused too -- so the gap is not charged; and the wait must also have polled kHandoffMinSpins
// times, so a few long gaps just under the bound cannot add up to a failure either.
constexpr uint64_t kHandoffTicks = 5000000;
constexpr uint64_t kHandoffGapTicks = 10000;     // 100 us
constexpr unsigned kHandoffMinSpins = 20000;
__device__ __forceinline__ bool sweep_arrive(unsigned* ctl, unsigned n) {
  unsigned v = __hip_atomic_fetch_add(ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    if (v >= kSweepPoison) return false;
    if (v == n) return true;
    if (wall_clock64() - t0 > kSweepArriveTicks) {
      const unsigned old = atomicCAS(ctl, v, v | kSweepPoison);
      if (old == v) return false;
      v = old;
      continue;
    }
    __builtin_amdgcn_s_sleep(4);
    v = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int NT, int XC, bool GX, int ROWS = 32, int NC = 1>
__global__ __launch_bounds__(SR_THREADS) void k_sweep_rows(Geom g, const bf16x8* __restrict__ wt, Hyper hp,
                                                            SweepT a) {
  using SG = SrGeom<NT, XC, ROWS>;
  static_assert(NC == 1 || (ROWS == 32 && NT % NC == 0), "column split: 32-row tiles, whole tiles per group");
  constexpr int NTC = NT / NC;   // column tiles of this workgroup per t
  constexpr bool GXP = GX && ROWS == 32;   // G_x partials folded by the producer (MFMA)
  constexpr bool GXC = GX && ROWS == 16;   // ... accumulated by the consumer (D == 1)
  constexpr int H = SG::H, XK = SG::XK, K2 = SG::K2, KC2 = SG::KC2, AST = SG::AST, AP = SG::APIECE;
  constexpr int TW = SG::TW, ZG = ROWS * TW;   // tile width; one gate's z tile (floats)
  __shared__ __attribute__((aligned(16))) __bf16 Ab[2][3 * AP];
  __shared__ __attribute__((aligned(16))) float Zb[2][4 * ZG];
  // GXC: per step parity, consumer wave and gate, the four-row sums of the tile's TW columns
  __shared__ __attribute__((aligned(16))) float Px[GXC ? 2 : 1][GXC ? 4 : 1][GXC ? 4 : 1][GXC ? TW : 1];
  __shared__ float Rg[GXC ? 5 * 256 : 1];   // GXC: the consumer threads' running range maxima
  // the workgroup's five range maxima (float bits under LDS atomicMax): one global atomicMax per slot
  // and workgroup at the end (sweep_done) -- with one per wave and slot, 256 workgroups queued ~5 000
  // atomics on one cache line behind the sweep
  __shared__ unsigned Rmax[5];
  const int T = g.T, D = g.D;
  if constexpr (NC > 1) {
    __shared__ int go_s;
    if (threadIdx.x == 0) {
      const size_t xset = (size_t)(gridDim.x / NC) * 32 * H * 8;   // the two granule sets, then the count
      go_s = sweep_arrive(reinterpret_cast<unsigned*>(static_cast<char*>(a.xbuf) + 2 * xset), gridDim.x);
    }
    __syncthreads();
    if (!go_s) return;
  } else {
    if (a.gate) {
      if (*a.gate < kSweepPoison) return;   // the column split ran
      // this launch does the sweep because the column split's grid was not resident: counted once
      if (blockIdx.x == 0 && threadIdx.x == 0 && a.fallback) atomicAdd(a.fallback, 1);
    }
  }
  // NC > 1: block b -> (row block rb, column group cg); the NC groups of a row block are blocks
  // b = x + 8 (NC i + cg), one XCD's under the observed round-robin placement (speed only)
  const int rb = NC == 1 ? (int)blockIdx.x : (int)(blockIdx.x % 8) + 8 * (int)(blockIdx.x / (8 * NC));
  const int cg = NC == 1 ? 0 : (int)((blockIdx.x / 8) % NC);
  const int n0 = cg * NTC;        // first column tile of this workgroup
  const int64_t m0 = a.r0 + (int64_t)rb * ROWS;
  if (NC > 1 && m0 >= a.r1) return;   // a padding row block: its whole group exits
  const int64_t rs = (int64_t)(T + 1) * H;
  const int64_t BTH = g.BT() * H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#ifdef SR_TIMING
  unsigned long long sr_wait = 0, sr_t0 = clock64(), sr_comp = 0, sr_store = 0, sr_lw = 0;
#endif
  auto put_a = [&](int buf, int row, int k, float v) {
    __bf16 p0, p1, p2;
    split3(v, p0, p1, p2);
    __bf16* d = &Ab[buf][row * AST + k];
    d[0] = p0; d[AP] = p1; d[2 * AP] = p2;
  };

  if (threadIdx.x < 5) Rmax[threadIdx.x] = 0u;
  auto lds_max = [&](unsigned* dst, float v) {   // wave max, one LDS atomic per wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    if ((threadIdx.x & 63) == 0) atomicMax(dst, __float_as_uint(v));
  };
  auto sweep_done = [&]() {   // every wave, once, at its end
    __syncthreads();
    if (a.range && threadIdx.x < 5) atomicMax(reinterpret_cast<unsigned*>(a.range) + threadIdx.x, Rmax[threadIdx.x]);
  };
  // A image for t = 1: [x_1 | h_0]
  float mh0 = 0.f;   // max |h_0| of the block's rows (range[4])
  for (int i = threadIdx.x; i < ROWS * K2; i += SR_THREADS) {
    const int row = i / K2, k = i % K2;
    const int64_t b = min(m0 + row, a.r1 - 1);
    const float v = k < XK ? (k < D ? a.x[b * T * D + k] : 0.f) : a.S.p[5][b * rs + (k - XK)];
    if (k >= XK) mh0 = fmaxf(mh0, fabsf(v));
    put_a(1, row, k, v);
  }
  __syncthreads();
  if (a.range) lds_max(&Rmax[4], mh0);

  if (ROWS == 16 && wave < 4) {
    // ------------------------------------------------------------------ producer, 16-row tiles
    // As below with the 16x16x32 shape: per 32-deep chunk one A fragment set (row lane % 16,
    // k 8 (lane / 16) ..) and four column blocks of B, 4 x 6 MFMAs; a 2-deep ring of B chunks.
    constexpr int GT = SG::GT, U = SG::U;
    const int q = wave, r16 = lane & 15, kq = lane >> 4;
    const bf16x8* wq = wt + (size_t)q * GT * 12 * 64 + lane;
    bf16x8 bq[U][4][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int p = 0; p < 3; ++p) bq[u][j][p] = wq[(u * 12 + j * 3 + p) * 64];
      // in slot order, as the loop refills them: the loop's vmcnt waits are merged over its entry
      // and its back edge, and a prologue scheduled slot 1 before slot 0 made every slot-0 chunk
      // wait for all loads in flight (vmcnt(0)), i.e. the ring one chunk deep instead of U
      if (SR16_PRO_ORDER) __builtin_amdgcn_sched_barrier(0);
    }
    f32x4 acc[4] = {};
    for (int t = 1; t <= T; ++t) {
      const __bf16* A = &Ab[t & 1][r16 * AST + 8 * kq];
#pragma unroll 1
      for (int G0 = 0; G0 < GT; G0 += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int G = G0 + u, n = G / KC2, cc = G - n * KC2;
          if (n == 0 && cc == KC2 - 2) SR_SYNC();   // mid-step: h_{t-1} of tile NT-1 is in
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(A + 32 * cc);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(A + AP + 32 * cc);
          const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(A + 2 * AP + 32 * cc);
#pragma unroll
          for (int j = 0; j < 4; ++j) {   // smallest terms first
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bq[u][j][0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bq[u][j][1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bq[u][j][2], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bq[u][j][0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bq[u][j][1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bq[u][j][0], acc[j], 0, 0, 0);
          }
          const int Gn = G + U < GT ? G + U : G + U - GT;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p) bq[u][j][p] = wq[(Gn * 12 + j * 3 + p) * 64];
          if (cc == KC2 - 1) {   // C map: row 4 (lane / 16) + v, column 16 j + lane % 16
            float* Z = &Zb[((t - 1) * NT + n) & 1][q * ZG + 4 * kq * TW + r16];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int v = 0; v < 4; ++v) Z[v * TW + 16 * j] = acc[j][v];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = f32x4{};
            SR_SYNC();   // end of step
          }
        }
      }
    }
    __syncthreads();         // final step: the consumer drains the last tile
    sweep_done();
    return;
  }
  if (NC > 1 && wave < 4) {
    // ------------------------------------------------------------------ producer, column split
    // As the row producer below over this group's NTC tiles only, the chunk sequence flattened
    // over t with a U-deep ring (GTC = NTC KC2 chunks per t need not divide by U).  The mid-step
    // barrier comes before the first h chunk of every t (h_{t-1} of the other groups arrives then);
    // the end-of-step barrier right at each tile's end, and the G_x fold (GX) after it.
    constexpr int U = 4, GTC = NTC * KC2;
    static_assert(GTC >= U, "ring deeper than the chunk cycle");
    const int q = wave, c = lane & 31, kh = lane >> 5;
    const bf16x8* wq = wt + ((size_t)q * SG::GT + (size_t)n0 * KC2) * 3 * 64 + lane;   // [q][n][c]: contiguous
    bf16x8 bq[NTC == 1 ? 1 : U][3];
    if constexpr (NTC > 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int p = 0; p < 3; ++p) bq[u][p] = wq[(u * 3 + p) * 64];
        if (SR_CS_ORDER) __builtin_amdgcn_sched_barrier(0);   // in slot order (see the 16-row producer)
      }
    }
    f32x16 acc = {};
    f32x4 gx[NTC][2];
    float xcur[8], xnext[NTC == 1 ? 1 : 8];
    int gxs = 0;
    auto load_gx_x = [&](int tn, float (&xv)[8]) {
      // from an opaque copy of the lane index, so that the eight row addresses are formed per call:
      // hoisted as loop invariants they were spilled (64-bit each) and reloaded one wait at a time
      int ln = lane;
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int64_t b = min(m0 + 4 * ks + (ln >> 4), a.r1 - 1);
        const int d = ln & 15;
        xv[ks] = a.x[(b * T + (tn - 1)) * D + (d < D ? d : D - 1)];   // masked at use (gx_x)
      }
    };
    const auto gx_x = [&](float v) { return (lane & 15) < D ? v : 0.f; };   // x operand lanes d < D
    auto gx_fold = [&](int buf) {
      if constexpr (NTC == 1) {
        load_gx_x(gxs + 1, xcur);   // off the critical path: the producer then waits at mid-step
      } else if ((gxs % NTC) == 0) {
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) xcur[ks] = xnext[ks];
        const int tn = gxs / NTC + 2;
        if (tn <= T) load_gx_x(tn, xnext);
      }
      const float* Rq = &Zb[buf][q * ZG + (lane >> 4) * 32 + (lane & 15)];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          gx[0][h] = __builtin_amdgcn_mfma_f32_16x16x4f32(gx_x(xcur[ks]), Rq[4 * ks * 32 + 16 * h], gx[0][h], 0, 0, 0);
      const f32x4 r0 = gx[0][0], r1 = gx[0][1];
#pragma unroll
      for (int k = 0; k + 1 < NTC; ++k) {
        gx[k][0] = gx[k + 1][0];
        gx[k][1] = gx[k + 1][1];
      }
      gx[NTC - 1][0] = r0;
      gx[NTC - 1][1] = r1;
      ++gxs;
    };
    if constexpr (GX) {
#pragma unroll
      for (int k = 0; k < NTC; ++k) gx[k][0] = gx[k][1] = f32x4{};
      if constexpr (NTC > 1) load_gx_x(1, xnext);
    }
    if constexpr (NTC == 1) {
      // One column tile per group (NC = NT): the tile's whole B image, KC2 chunks x 3 pieces (204
      // VGPRs at H = 256), stays in registers for the sweep -- the weights do not change during it, and
      // streaming it from L2 per t kept the h chunks waiting on loads (4.5 us per t against 1.4 of
      // MFMAs, kbench SR_CS_TIMING).  The x chunks (before the mid-step wait) are loaded per t.
      constexpr int KH = KC2 - XC;
      bf16x8 bres[KH][3], bx[XC][3];
#pragma unroll
      for (int cc = 0; cc < KH; ++cc)
#pragma unroll
        for (int p = 0; p < 3; ++p) bres[cc][p] = wq[((XC + cc) * 3 + p) * 64];
#pragma unroll 1
      for (int t = 1; t <= T; ++t) {
        const __bf16* A = &Ab[t & 1][c * AST + 8 * kh];
        if (q == 0) CS_STAMP(t, 8);
#pragma unroll
        for (int cc = 0; cc < XC; ++cc)
#pragma unroll
          for (int p = 0; p < 3; ++p) bx[cc][p] = wq[(cc * 3 + p) * 64];
#pragma unroll
        for (int cc = 0; cc < KC2; ++cc) {
          if (cc == XC) {
            SR_SYNC();   // mid-step: all of h_{t-1} is in this A buffer
            if (q == 0) CS_STAMP(t, 9);
          }
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(A + 16 * cc);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(A + AP + 16 * cc);
          const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(A + 2 * AP + 16 * cc);
          const bf16x8* b = cc < XC ? bx[cc < XC ? cc : 0] : bres[cc < XC ? 0 : cc - XC];
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[0], acc, 0, 0, 0);
        }
        const int st = t - 1;   // step index
        float* Z = &Zb[st & 1][q * ZG + c];
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) Z[acc_row(rr, lane) * 32] = acc[rr];
        acc = f32x16{};
        if (q == 0) CS_STAMP(t, 10);
        SR_SYNC();   // end of step
        if constexpr (GX)
          if (st >= 1) gx_fold((st - 1) & 1);
      }
    } else {
    const int total = T * GTC;
    // chunk G through ring slot u.  The loop runs whole groups of U chunks with no per-chunk guard
    // (SR_CS_ORDER): with one, the path on which slot u - 1 was skipped reaches slot u's waits, and
    // the loop's vmcnt waits merged over it drained every load in flight (vmcnt(0)) in every slot
    auto chunk = [&](auto uc, const int G) {
      constexpr int u = decltype(uc)::value;
      {
        {
          const int t = G / GTC + 1, r = G - (t - 1) * GTC, nl = r / KC2, cc = r - nl * KC2;
          if (nl == 0 && cc == 0 && q == 0) CS_STAMP(t, 8);
          if (nl == 0 && cc == XC) SR_SYNC();   // mid-step: all of h_{t-1} is in this A buffer
          if (nl == 0 && cc == XC && q == 0) CS_STAMP(t, 9);
          const __bf16* A = &Ab[t & 1][c * AST + 8 * kh];
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(A + 16 * cc);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(A + AP + 16 * cc);
          const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(A + 2 * AP + 16 * cc);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, bq[u][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq[u][1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[u][2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq[u][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[u][1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[u][0], acc, 0, 0, 0);
          const int rn = r + U < GTC ? r + U : r + U - GTC;
#pragma unroll
          for (int p = 0; p < 3; ++p) bq[u][p] = wq[(rn * 3 + p) * 64];
          if (cc == KC2 - 1) {
            const int st = (t - 1) * NTC + nl;   // step index
            float* Z = &Zb[st & 1][q * ZG + c];
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) Z[acc_row(rr, lane) * 32] = acc[rr];
            acc = f32x16{};
            if (q == 0) CS_STAMP(t, 10);
            SR_SYNC();   // end of step
            if constexpr (GX)
              if (st >= 1) gx_fold((st - 1) & 1);
          }
        }
      }
    };
    int G0 = 0;
    if (SR_CS_ORDER) {
#pragma unroll 1
      for (; G0 + U <= total; G0 += U) {
        chunk(std::integral_constant<int, 0>{}, G0);
        chunk(std::integral_constant<int, 1>{}, G0 + 1);
        chunk(std::integral_constant<int, 2>{}, G0 + 2);
        chunk(std::integral_constant<int, 3>{}, G0 + 3);
      }
    }
#pragma unroll 1
    for (; G0 < total; G0 += U) {
      chunk(std::integral_constant<int, 0>{}, G0);
      if (G0 + 1 < total) chunk(std::integral_constant<int, 1>{}, G0 + 1);
      if (G0 + 2 < total) chunk(std::integral_constant<int, 2>{}, G0 + 2);
      if (G0 + 3 < total) chunk(std::integral_constant<int, 3>{}, G0 + 3);
    }
    static_assert(U == 4, "the chunk calls above spell out four ring slots");
    }   // NTC > 1
    __syncthreads();         // final step: the consumer drains the last tile
    if constexpr (GX) {
      gx_fold((T * NTC - 1) & 1);
      float* out = a.gx_slab + ((int64_t)rb * 4 + q) * D * H;
#pragma unroll
      for (int k = 0; k < NTC; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int d = 4 * (lane >> 4) + v;
            if (d < D) out[(int64_t)d * H + 32 * (n0 + k) + 16 * h + (lane & 15)] = gx[k][h][v];
          }
    }
    sweep_done();
    return;
  }
  if (ROWS == 32 && NC == 1 && wave < 4) {
    // ------------------------------------------------------------------ producer (gate q)
    // The B stream of a wave is the cyclic sequence of its GT chunks per t (3 x 16 B per lane
    // each).  The loop walks it U chunks at a time with a U-deep register ring: slot u holds
    // chunk G+u and is refilled with chunk G+u+U right after its 6 MFMAs.
    constexpr int GT = SG::GT, U = SG::U;
    const int q = wave, c = lane & 31, kh = lane >> 5;
    const bf16x8* wq = wt + (size_t)q * GT * 3 * 64 + lane;
    bf16x8 bq[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int p = 0; p < 3; ++p) bq[u][p] = wq[(u * 3 + p) * 64];
    f32x16 acc = {};
    // GX: ring of the gate's G_x partials, slot 0 = the column tile folded next
    f32x4 gx[NT][2];
    float xcur[8], xnext[8];
    int gxs = 0;   // tiles folded so far
    auto load_gx_x = [&](int tn, float (&xv)[8]) {   // A operand: x_tn[row 4ks + lane/16][d = lane%16]
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        // unmasked (d clamped): a select here would wait for the load; gx_x masks it at its use
        const int64_t b = min(m0 + 4 * ks + (lane >> 4), a.r1 - 1);
        const int d = lane & 15;
        xv[ks] = a.x[(b * T + (tn - 1)) * D + (d < D ? d : D - 1)];
      }
    };
    const auto gx_x = [&](float v) { return (lane & 15) < D ? v : 0.f; };   // x operand lanes d < D
    auto gx_fold = [&](int buf) {   // R of the tile folded next, from Zb[buf]
      if ((gxs % NT) == 0) {
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) xcur[ks] = xnext[ks];
        const int tn = gxs / NT + 2;
        if (tn <= T) load_gx_x(tn, xnext);
      }
      const float* Rq = &Zb[buf][q * ZG + (lane >> 4) * 32 + (lane & 15)];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          gx[0][h] = __builtin_amdgcn_mfma_f32_16x16x4f32(gx_x(xcur[ks]), Rq[4 * ks * 32 + 16 * h], gx[0][h], 0, 0, 0);
      const f32x4 r0 = gx[0][0], r1 = gx[0][1];
#pragma unroll
      for (int k = 0; k + 1 < NT; ++k) {
        gx[k][0] = gx[k + 1][0];
        gx[k][1] = gx[k + 1][1];
      }
      gx[NT - 1][0] = r0;
      gx[NT - 1][1] = r1;
      ++gxs;
    };
    if constexpr (GX) {
#pragma unroll
      for (int k = 0; k < NT; ++k) gx[k][0] = gx[k][1] = f32x4{};
      load_gx_x(1, xnext);
    }
    for (int t = 1; t <= T; ++t) {
      const __bf16* A = &Ab[t & 1][c * AST + 8 * kh];
#pragma unroll 1
      for (int G0 = 0; G0 < GT; G0 += U) {
        int ended = -1;   // GX: the tile step that ended in this group (at most one: KC2 > U)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int G = G0 + u, n = G / KC2, cc = G - n * KC2;
          if (n == 0 && cc == KC2 - 2) SR_SYNC();   // mid-step: h_{t-1} of tile NT-1 is in
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(A + 16 * cc);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(A + AP + 16 * cc);
          const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(A + 2 * AP + 16 * cc);
          // smallest terms first
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, bq[u][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq[u][1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[u][2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq[u][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[u][1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[u][0], acc, 0, 0, 0);
          const int Gn = G + U < GT ? G + U : G + U - GT;
#pragma unroll
          for (int p = 0; p < 3; ++p) bq[u][p] = wq[(Gn * 3 + p) * 64];
          if (cc == KC2 - 1) {
            float* Z = &Zb[((t - 1) * NT + n) & 1][q * ZG + c];
#pragma unroll
            for (int r = 0; r < 16; ++r) Z[acc_row(r, lane) * 32] = acc[r];
            acc = f32x16{};
            if constexpr (GX) ended = (t - 1) * NT + n;
            else SR_SYNC();   // end of step
          }
        }
        // GX: the end-of-step barrier moves to the group's end (the next tile's chunks of this
        // group read only A and B), so that the fold below exists once, not in every unrolled
        // slot.  Past the barrier of step s the consumer's R of tile s - 1 is in its slot, which
        // the z of tile s + 1 overwrites only at that tile's end.
        if constexpr (GX)
          if (ended >= 0) {
            SR_SYNC();   // end of step
            if (ended >= 1) gx_fold((ended - 1) & 1);
          }
      }
    }
    const int slast = T * NT - 1;
    __syncthreads();         // final step: the consumer drains the last tile
    if constexpr (GX) {
      gx_fold(slast & 1);
      // slot k = column tile k; C map of 16x16x4: row d = 4 (lane / 16) + v, column lane % 16
      float* out = a.gx_slab + ((int64_t)blockIdx.x * 4 + q) * D * H;
#pragma unroll
      for (int k = 0; k < NT; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int d = 4 * (lane >> 4) + v;
            if (d < D) out[(int64_t)d * H + 32 * k + 16 * h + (lane & 15)] = gx[k][h][v];
          }
    }
#ifdef SR_TIMING
    if (threadIdx.x == 0) { g_sr_wait[blockIdx.x][0] = sr_wait; g_sr_wait[blockIdx.x][1] = clock64() - sr_t0; }
#endif
    sweep_done();
    return;
  }

  // -------------------------------------------------------------------- consumer
  // Thread ct owns row ct/8 and hidden units 4(ct%8) .. +3 of every tile: each plane access is
  // one 16-byte buffer op per lane (a wave: 8 rows x 128 B), so a tile costs a lane 11 loads
  // and 15 stores -- with one load per point it was 100 memory ops, past the 63 a wave can have
  // outstanding, and every tile waited out full memory round trips.  Plane accesses go through
  // buffer descriptors: one 32-bit byte offset per thread serves every plane, and the record
  // count (rows < r1) turns loads past the last row into zeros and drops their stores.
  const int ct = threadIdx.x - 4 * 64;      // 0..255
  constexpr int TPR = TW / 4;               // threads per tile row (8 or 16)
  const int row = ct / TPR, j4 = (ct % TPR) * 4;
  const uint32_t pbytes = (uint32_t)(a.r1 * rs * 4), zbytes = (uint32_t)(a.r1 * T * H * 4);
  __amdgpu_buffer_rsrc_t rS[6], rL[6];
#pragma unroll
  for (int p = 0; p < 6; ++p) {
    rS[p] = __builtin_amdgcn_make_buffer_rsrc(a.S.p[p], 0, pbytes, kBufWord3);
    rL[p] = __builtin_amdgcn_make_buffer_rsrc(a.L.p[p], 0, pbytes, kBufWord3);
  }
  // z cache and lam/rho + S of the updated i, f, g, o (the next step's x-stage targets): one
  // descriptor per [4][B*T][H] array, the gate plane selected by soffset
  const uint32_t zpl = (uint32_t)(BTH * 4), zrec = 3 * zpl + zbytes;   // plane stride, records
  const __amdgpu_buffer_rsrc_t rZ = __builtin_amdgcn_make_buffer_rsrc(a.zc, 0, zrec, kBufWord3);
  const bool wtgt = a.tgt != nullptr;
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc(wtgt ? a.tgt : a.zc, 0, wtgt ? zrec : 0, kBufWord3);
  const bool rok = m0 + row < a.r1;
  const uint32_t pofs = (uint32_t)(((m0 + row) * rs + j4) * 4);       // t = 0, tile 0
  const uint32_t zofs = (uint32_t)(((m0 + row) * T * H + j4) * 4);    // t = 1, tile 0

  // The dual of h is zero before T (admm.py:504-539 ascends it only at t = T) unless the caller
  // wrote it: a.lamh_nz, set by k_check_lamh after every external change, says which.
  const bool lh_zero = a.lamh_nz != nullptr && *a.lamh_nz == 0;
  struct St4 { f32x4 f0, g0, c0, h0, cp, li, lf, lg, lo, lc, lh; };
  auto load_tile = [&](int t, int n, St4& v) {
    const uint32_t o = pofs + (uint32_t)(t * H + TW * n) * 4;
    v.f0 = buf_ld4(rS[1], o); v.g0 = buf_ld4(rS[2], o); v.c0 = buf_ld4(rS[4], o); v.h0 = buf_ld4(rS[5], o);
    // c_{t-1}: from the state plane only at t = 1 (the initial c); later this thread's own
    // update of the previous t, kept in registers (cring)
    if (t == 1) v.cp = buf_ld4(rS[4], o - H * 4);
    v.li = buf_ld4(rL[0], o); v.lf = buf_ld4(rL[1], o); v.lg = buf_ld4(rL[2], o);
    v.lo = buf_ld4(rL[3], o); v.lc = buf_ld4(rL[4], o);
    v.lh = lh_zero && t < T ? f32x4{} : buf_ld4(rL[5], o);
  };
  // x_{tn} into A-buffer tn&1 (ROWS rows x XK)
  auto load_x = [&](int tn) {
    if (tn > T) return;
#pragma unroll
    for (int u = 0; u < ROWS * XK / 256; ++u) {
      const int i = ct + 256 * u, xr = i / XK, k = i % XK;
      const int64_t b = min(m0 + xr, a.r1 - 1);
      put_a(tn & 1, xr, k, k < D ? a.x[(b * T + (tn - 1)) * D + k] : 0.f);
    }
  };

  // NC > 1: the h_t granules (see the kernel's comment).  rX spans the padded row blocks' granules.
  // Two granule sets by the parity of t: a group overwrites the set of h_t only when it publishes
  // h_{t+2}, after its exchange of h_{t+1}, which every other group published after reading all of
  // h_t -- so no reader can miss a tag (with one set, a reader slowed past a group's h_{t+1} publish,
  // e.g. behind its own plane stores, would spin on a tag that had already been overwritten).
  const uint32_t xset = (uint32_t)(gridDim.x / NC) * 32 * H * 8;   // bytes per set
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      NC > 1 ? a.xbuf : a.zc, 0, NC > 1 ? 2 * xset : 0u, kBufWord3);
  // publish: this thread's four h_t values of tile n as two 16-byte granule pairs
  auto publish = [&](int t, int n, f32x4 h) {
    const float tg = __uint_as_float((unsigned)t);
    const uint32_t go = (t & 1) * xset + (uint32_t)(((rb * 32 + row) * H + TW * n + j4) * 8);
    buf_st4<16>(rX, go, f32x4{h[0], tg, h[1], tg});
    buf_st4<16>(rX, go + 16, f32x4{h[2], tg, h[3], tg});
  };
  // read the other groups' columns of h_t once every granule carries tag t, into the A image of t + 1
  auto exchange = [&](int t) {
    constexpr int OC = H - TW * NTC;               // other groups' columns
    constexpr int NP = ROWS * OC / 2 / 256;        // 16-byte granule pairs per consumer thread
    f32x4 gv[NP > 0 ? NP : 1];
    // the granule addresses are formed here each t from an opaque copy of the thread index: hoisted
    // out of the sweep's loop as loop invariants they took 2 NP registers for the whole kernel, which
    // the GX variants spilled to scratch and reloaded one wait at a time every t
    // (one constant division per exchange; granule pair i = ct + 256 i steps it by constants)
    unsigned cto = (unsigned)ct;
    if constexpr (NC < 8) asm volatile("" : "+v"(cto));
    constexpr unsigned OC2 = OC > 0 ? OC / 2 : 1;   // (NC == 1 instantiates this with OC = 0, never called)
    const unsigned q0 = cto / OC2, r0 = cto % OC2;
    const uint32_t xo = (t & 1) * xset + (uint32_t)(rb * 32 * H * 8);
    auto addr = [&](int i, int& hr, int& col) {
      unsigned r = r0 + (256u * i) % OC2, q = q0 + (256u * i) / OC2;
      if (r >= OC2) { r -= OC2; ++q; }
      hr = (int)q;
      const int oc = 2 * (int)r;
      col = oc < TW * n0 ? oc : oc + TW * NTC;
      return xo + (uint32_t)((hr * H + col) * 8);
    };
    const unsigned want = (unsigned)t;
    uint64_t prev = 0, waited = 0;
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        int hr, col;
        gv[i] = buf_ld4<kAuxL2>(rX, addr(i, hr, col));
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) ok &= __float_as_uint(gv[i][1]) == want && __float_as_uint(gv[i][3]) == want;
      if (__all(ok)) break;
      // bounded by the wall clock this wave ran (the clock is read only once a wait is not
      // immediately served; gaps from preemption are not charged, kHandoffGapTicks)
      const uint64_t now = wall_clock64();
      if (spins > 0 && now - prev < kHandoffGapTicks) waited += now - prev;
      prev = now;
      if (waited > kHandoffTicks && spins >= kHandoffMinSpins) {
        // a group did not publish h_t: the A image would hold stale h.  Counted per wave
        // (DevStats::handoff_fail); the host turns it into an error (admm_step / admm_get_stats)
        if (lane == 0 && a.fail) atomicAdd(a.fail, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (ct == 0) CS_STAMP(t, 4);
#pragma unroll
    for (int i = 0; i < NP; ++i) {   // two adjacent columns per granule pair: 4-byte LDS writes
      int hr, col;
      (void)addr(i, hr, col);
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      bf16x2 p0, p1, p2;
      split3(f32x2{gv[i][0], gv[i][2]}, p0, p1, p2);
      __bf16* d = &Ab[(t + 1) & 1][hr * AST + XK + col];
      *reinterpret_cast<bf16x2*>(d) = p0;
      *reinterpret_cast<bf16x2*>(d + AP) = p1;
      *reinterpret_cast<bf16x2*>(d + 2 * AP) = p2;
    }
    if (ct == 0) CS_STAMP(t, 5);
  };
  // Tile operands are loaded one tile early (loading two tiles ahead measured no faster).
  // cring[0] is c_{t-1} of the tile being updated: popped at every tile, c_t pushed at the back.
  static_assert(NT > 1, "the mid-step barrier protocol needs two or more column tiles");
  f32x4 cring[NTC];
#pragma unroll
  for (int k = 0; k < NTC; ++k) cring[k] = f32x4{};
  // GXC: this thread's slab entries (gate = its consumer wave, column = its lane) of each column
  // tile, a ring turned once per step like cring
  float gxr[GXC ? NT : 1];   // slot 0 = the tile summed next (turned once per step)
#pragma unroll
  for (int k = 0; k < (GXC ? NT : 1); ++k) gxr[k] = 0.f;
  const int cq = ct >> 6;     // GXC: the gate this thread sums (its consumer wave)
  // the slot read at step 0 holds no tile: zeros (the ring turns for it like for any step)
  if (GXC) *reinterpret_cast<f32x4*>(&Px[GXC ? 1 : 0][0][0][0] + 4 * ct) = f32x4{};
  const int64_t bx = min(m0 + row, a.r1 - 1);
  // range (a.range): max |phi(z) - tgt| per gate and max |h_t|, t < T, over this thread's points.
  // GXC (16-row tiles, D == 1): the consumer is at the register limit, so the five running maxima
  // live in the thread's LDS slots (Rg) instead of registers
  float rq0 = 0.f, rq1 = 0.f, rq2 = 0.f, rq3 = 0.f, rh = 0.f;
  if constexpr (GXC) {
#pragma unroll
    for (int k = 0; k < 5; ++k) Rg[k * 256 + ct] = 0.f;
  }
  St4 nxt;
  load_tile(1, n0, nxt);
  load_x(2);                 // step 0: the producer computes tile (1, 0)
  __syncthreads();           // its mid-step barrier
  __syncthreads();           // end of step 0
  for (int t = 1; t <= T; ++t) {
    const bool last = (t == T);
    __bf16* An = &Ab[(t + 1) & 1][row * AST + XK + j4];
#pragma unroll 1
    for (int nl = 0; nl < NTC; ++nl) {
      const int n = n0 + nl;   // column tile (NC == 1: n0 = 0)
#ifdef SR_TIMING
      const unsigned long long ta_ = clock64();
#endif
      const St4 cur = nxt;
      if (NC > 1 && ct == 0) CS_STAMP(t, 0);
      float xm = 0.f;   // GXC (D == 1): x_t of this row (its address formed per tile: as a hoisted
      if constexpr (GXC) {   // 64-bit invariant it was spilled)
        int64_t bxo = bx;
        asm volatile("" : "+v"(bxo));
        xm = rok ? a.x[bxo * T + (t - 1)] : 0.f;
      }
#ifdef SR_TIMING
      asm volatile("" :: "v"(cur.f0), "v"(cur.g0), "v"(cur.c0), "v"(cur.h0), "v"(cur.li), "v"(cur.lf), "v"(cur.lg),
                   "v"(cur.lo), "v"(cur.lc), "v"(cur.lh), "v"(cur.cp));
      const unsigned long long tw_ = clock64();
      if ((threadIdx.x & 63) == 0) sr_lw += tw_ - ta_;
#endif
      if (nl + 1 < NTC) load_tile(t, n + 1, nxt);
      else if (!last) load_tile(t + 1, n0, nxt);
      f32x4* Z = reinterpret_cast<f32x4*>(&Zb[((t - 1) * NTC + nl) & 1][row * TW + j4]);
      constexpr int ZG4 = ZG / 4;   // one gate's tile in f32x4
      const f32x4 zi = Z[0], zf = Z[ZG4], zg = Z[2 * ZG4], zo = Z[3 * ZG4];
      f32x4 i1, f1, g1, o1, c1, h1, li, lf, lg, lo, lc;
      f32x4 ai, af, ag, ao, di, df, dg, dO;   // phi(z), phi'(z) (GX)
      const f32x4 cpv = t == 1 ? cur.cp : cring[0];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        SweepIn v;
        v.zi = zi[u]; v.zf = zf[u]; v.zg = zg[u]; v.zo = zo[u];
        v.f0 = cur.f0[u]; v.g0 = cur.g0[u]; v.c0 = cur.c0[u]; v.h0 = cur.h0[u]; v.cp = cpv[u];
        v.li = cur.li[u]; v.lf = cur.lf[u]; v.lg = cur.lg[u]; v.lo = cur.lo[u]; v.lc = cur.lc[u]; v.lh = cur.lh[u];
        const SweepRes o = sweep_point(hp, v, last);
        i1[u] = o.i1; f1[u] = o.f1; g1[u] = o.g1; o1[u] = o.o1; c1[u] = o.c1; h1[u] = o.h1;
        li[u] = o.li; lf[u] = o.lf; lg[u] = o.lg; lo[u] = o.lo; lc[u] = o.lc;
        ai[u] = o.ai; af[u] = o.af; ag[u] = o.ag; ao[u] = o.ao;
        di[u] = o.di; df[u] = o.df; dg[u] = o.dg; dO[u] = o.dO;
      }
#pragma unroll
      for (int k = 0; k + 1 < NTC; ++k) cring[k] = cring[k + 1];
      cring[NTC - 1] = c1;
      // h_t first: the other groups (NC > 1) and the producer wait for it; the targets, maxima and
      // residuals below are off that path
      if constexpr (NC > 1)
        if (!last && !(a.skip_publish && t == 1 && rb == 0 && cg == 1)) publish(t, n, h1);
      if (!last) {
        bf16x4 p0, p1, p2;
        split3(h1, p0, p1, p2);
        __bf16* d = An + TW * n;
        *reinterpret_cast<bf16x4*>(d) = p0;
        *reinterpret_cast<bf16x4*>(d + AP) = p1;
        *reinterpret_cast<bf16x4*>(d + 2 * AP) = p2;
      }
      if (NC > 1 && ct == 0) CS_STAMP(t, 3);
      // lam/rho + S of the updated i, f, g, o: the next x stage's targets (tgt_quot, as k_resid_gx)
      f32x4 ti, tf, tg, to;
      if (hp.rinv_exact) {   // workgroup-uniform: 16 IEEE divisions per tile and thread saved
        ti = tgt_mulq(li, hp.rinv_gate[0], i1); tf = tgt_mulq(lf, hp.rinv_gate[1], f1);
        tg = tgt_mulq(lg, hp.rinv_gate[2], g1); to = tgt_mulq(lo, hp.rinv_gate[3], o1);
      } else {
        ti = tgt_quot(li, hp.rho[0], i1); tf = tgt_quot(lf, hp.rho[1], f1);
        tg = tgt_quot(lg, hp.rho[2], g1); to = tgt_quot(lo, hp.rho[3], o1);
      }
      if (a.range && rok) {
        if constexpr (GXC) {   // one LDS slot at a time (the consumer is at the register limit)
          auto upd = [&](int k, f32x4 a_, f32x4 t_) {
            float m = Rg[k * 256 + ct];
#pragma unroll
            for (int u = 0; u < 4; ++u) m = fmaxf(m, fabsf(a_[u] - t_[u]));
            Rg[k * 256 + ct] = m;
          };
          upd(0, ai, ti); upd(1, af, tf); upd(2, ag, tg); upd(3, ao, to);
          if (!last) upd(4, h1, f32x4{});
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            rq0 = fmaxf(rq0, fabsf(ai[u] - ti[u]));
            rq1 = fmaxf(rq1, fabsf(af[u] - tf[u]));
            rq2 = fmaxf(rq2, fabsf(ag[u] - tg[u]));
            rq3 = fmaxf(rq3, fabsf(ao[u] - to[u]));
            if (!last) rh = fmaxf(rh, fabsf(h1[u]));
          }
        }
      }
      if constexpr (GXP) {   // R = (phi(z) - tgt) phi'(z) into the z slot (0 past the last row)
        const float m = rok ? 1.f : 0.f;
        Z[0] = (ai - ti) * di * m;
        Z[ZG4] = (af - tf) * df * m;
        Z[2 * ZG4] = (ag - tg) * dg * m;
        Z[3 * ZG4] = (ao - to) * dO * m;
      }
      if constexpr (GXC) {   // x_t R_q of the four points (0 past the last row: xm = 0)
        const int sp = ((t - 1) * NT + n) & 1;
        const bool b1 = (lane >> 5) & 1, b0 = (lane >> 4) & 1;   // the row's bits within the wave
        // rows r and r ^ 2 (lanes 32 apart): keep gates 2 b1, 2 b1 + 1; then rows r, r ^ 1: keep r.
        // One gate pair at a time (registers).
        auto pair = [&](f32x4 va, f32x4 vb) {   // gates q, q + 2 -> the kept one, summed over r, r ^ 2
          f32x4 k = b1 ? vb : va;
          const f32x4 sx = b1 ? va : vb;
#pragma unroll
          for (int u = 0; u < 4; ++u) k[u] += __shfl_xor(sx[u], 32, 64);
          return k;
        };
        const f32x4 k0 = pair((ai - ti) * di * xm, (ag - tg) * dg * xm);
        const f32x4 k1 = pair((af - tf) * df * xm, (ao - to) * dO * xm);
        f32x4 kk = b0 ? k1 : k0;
        const f32x4 sk = b0 ? k0 : k1;
#pragma unroll
        for (int u = 0; u < 4; ++u) kk[u] += __shfl_xor(sk[u], 16, 64);
        *reinterpret_cast<f32x4*>(&Px[sp][cq][lane >> 4][j4]) = kk;
        // the previous step's tile: gate cq, column lane, summed over the four waves in order
        const float* pp = &Px[sp ^ 1][0][cq][lane];
        const float tot = ((pp[0] + pp[4 * TW]) + pp[8 * TW]) + pp[12 * TW];
        const float h0 = gxr[0] + tot;
#pragma unroll
        for (int k = 0; k + 1 < NT; ++k) gxr[k] = gxr[k + 1];
        gxr[NT - 1] = h0;
      }
#ifdef SR_TIMING
      asm volatile("" :: "v"(i1), "v"(f1), "v"(g1), "v"(o1), "v"(c1), "v"(h1), "v"(li), "v"(lf), "v"(lg), "v"(lo), "v"(lc));
      const unsigned long long tb_ = clock64();
#endif
      if (NC > 1 && ct == 0) CS_STAMP(t, 1);
      const uint32_t po = pofs + (uint32_t)(t * H + TW * n) * 4, zo4 = zofs + (uint32_t)((t - 1) * H + TW * n) * 4;
      buf_st4(rS[0], po, i1); buf_st4(rS[1], po, f1); buf_st4(rS[2], po, g1); buf_st4(rS[3], po, o1);
      buf_st4<0>(rS[4], po, c1);             // c_t: read by the next step's kernels
      if (!last) buf_st4<0>(rS[5], po, h1);
      buf_st4(rL[0], po, li); buf_st4(rL[1], po, lf); buf_st4(rL[2], po, lg); buf_st4(rL[3], po, lo);
      buf_st4(rL[4], po, lc);
      // one descriptor spans the 4 planes, so its record count cannot drop the stores of rows
      // past r1 (a ragged last block): they would land in the next plane -- predicate them
      if (rok) {
        buf_st4s(rZ, zo4, 0, zi); buf_st4s(rZ, zo4, zpl, zf); buf_st4s(rZ, zo4, 2 * zpl, zg);
        buf_st4s(rZ, zo4, 3 * zpl, zo);
      }
      if (wtgt && rok) {   // same expression as k_resid_gx (tgt_quot), so either source gives equal bits
        buf_st4s(rT, zo4, 0, ti); buf_st4s(rT, zo4, zpl, tf);
        buf_st4s(rT, zo4, 2 * zpl, tg); buf_st4s(rT, zo4, 3 * zpl, to);
      }
#ifdef SR_TIMING
      const unsigned long long tc_ = clock64();
      if ((threadIdx.x & 63) == 0) { sr_comp += tb_ - ta_; sr_store += tc_ - tb_; }
#endif
      if (NC > 1 && ct == 0) CS_STAMP(t, 2);
      // (NC > 1: the hand-off comes after this tile's plane stores, although its poll loads then
      // return behind them.  Issued after the poll but before the mid-step barrier, the stores delay
      // the barrier (round 4); issued past it, they slow the producer's h chunks of t + 1 more than
      // the earlier poll gains: 9.5 against 9.1 us per t at c3s, profiles/r05e_c3s_cs_phase_timing.txt)
      if (nl == NTC - 1 && !last) {
        if constexpr (NC > 1) exchange(t);   // the other groups' columns of h_t into this A buffer
        SR_SYNC();           // the producer's mid-step barrier: h_t is complete
        if (NC > 1 && ct == 0) CS_STAMP(t, 6);
      }
      // x_{t+2} into the A buffer of t+2 (the producer's z_t is done with it): needed only past the end
      // of this step, so its loads -- each waited for by its LDS write -- stay off the mid-step path
      if (nl == NTC - 1 && !last) load_x(t + 2);
      SR_SYNC();             // end of step
    }
  }
  if (a.range) {
    if constexpr (GXC) {
      rq0 = Rg[ct]; rq1 = Rg[256 + ct]; rq2 = Rg[512 + ct]; rq3 = Rg[768 + ct]; rh = Rg[1024 + ct];
    }
    lds_max(&Rmax[0], rq0);
    lds_max(&Rmax[1], rq1);
    lds_max(&Rmax[2], rq2);
    lds_max(&Rmax[3], rq3);
    lds_max(&Rmax[4], rh);
  }
  if constexpr (GXC) {   // past the last step's barrier: its tile, then the slab (D == 1)
    const float* pp = &Px[((T - 1) * NT + NT - 1) & 1][0][cq][lane];
    const float tot = ((pp[0] + pp[4 * TW]) + pp[8 * TW]) + pp[12 * TW];
    const float h0 = gxr[0] + tot;
#pragma unroll
    for (int k = 0; k + 1 < NT; ++k) gxr[k] = gxr[k + 1];
    gxr[NT - 1] = h0;
    float* out = a.gx_slab + ((int64_t)blockIdx.x * 4 + cq) * H + lane;
#pragma unroll
    for (int k = 0; k < NT; ++k) out[TW * k] = gxr[k];   // slot k = column tile k after T NT + 1 turns
  }
  sweep_done();
#ifdef SR_TIMING
  if (threadIdx.x == 256) {
    g_sr_wait[1024 + blockIdx.x][0] = sr_wait;
    g_sr_wait[1024 + blockIdx.x][1] = sr_comp;
    g_sr_wait[1536 + blockIdx.x][0] = sr_store;
    g_sr_wait[1536 + blockIdx.x][1] = sr_lw;
  }
#endif
}

__global__ __launch_bounds__(kThreads) void k_rowdot(int64_t B, int H, int O, const float* h, int64_t hs,
                                                       const float* wy, float* out) {
  const int lane = threadIdx.x & 63;
  for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += (int64_t)gridDim.x * 4) {
    for (int o = 0; o < O; ++o) {
      float s = 0.f;
      for (int j = lane; j < H; j += kWave) s += h[b * hs + j] * wy[(int64_t)j * O + o];
      s = wave_sum(s);
      if (lane == 0) out[b * O + o] = s;
    }
  }
}

// ============================================================================ weight stage
// Row index of the weight phase: row = b*T + (t-1), t = 1..T (admm.py:304-311).
// X row = x + row*D;  Hprev row (S[h] at t-1) = Sh + (row + b)*H  since b*(T+1) + t-1 = row + b.

template <bool VEC>
struct AllRowSrc {  // z cache recompute: A = [X | Hprev] over all rows (K = D+H), B = [Wx; Wh]
  const float* x; const float* Sh; int64_t BT; DivU32 dT; int D, H; Weights w; int j0;
  static constexpr bool A_ROW_MAJOR = true;
  __device__ float4 a4(int64_t m, int64_t k) const {
    const int K = D + H;
    if (VEC) {
      if (m >= BT || k >= K) return make_float4(0.f, 0.f, 0.f, 0.f);
      const float* src = k < D ? x + m * D + k : Sh + (m + dT.div((uint32_t)m)) * H + (k - D);
      return *reinterpret_cast<const float4*>(src);
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t kk = k + u;
      v[u] = (m < BT && kk < K) ? (kk < D ? x[m * D + kk] : Sh[(m + dT.div((uint32_t)m)) * H + (kk - D)]) : 0.f;
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ float4 b4(int64_t k, int64_t n) const { return weights4<VEC>(w, D, H, j0, k, n); }
};

template <bool VEC>
__device__ __forceinline__ void zgemm_body(const Geom& g, const Weights& w, const float* x, const float* Sh, float* zc,
                                           float* smem) {
  const int nj = (g.H + 31) / 32;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)(lid / nj) * TS_BM;
  const int j0 = (lid % nj) * 32;
  const int64_t BT = g.BT();
  AllRowSrc<VEC> src{x, Sh, BT, g.dT, g.D, g.H, w, j0};
  f32x16 acc[1][4];
  zero_acc(acc);
  Engine<TS_BM, TS_BN, TS_WM, TS_WN, TS_KC, AllRowSrc<VEC>> eng;
  eng.run(src, m0, 0, 0, g.D + g.H, acc, smem);
  const int lane = threadIdx.x & 63, wm0 = (threadIdx.x >> 6) * TS_WM;
  const int j = j0 + (lane & 31);
  if (j >= g.H) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = m0 + wm0 + acc_row(r, lane);
    if (row >= BT) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) zc[((int64_t)q * BT + row) * g.H + j] = acc[0][q][r];
  }
}

template <bool VEC>
__global__ __launch_bounds__(kThreads) void k_zgemm(Geom g, Weights w, const float* x, const float* Sh, float* zc) {
  __shared__ float smem[TSTile::LDS_FLOATS];
  zgemm_body<VEC>(g, w, x, Sh, zc, smem);
}

// Element loop helper over (row, j) of a [BT][H] plane with cheap index math.
struct RowJ {
  int hchunk, rpb, rr, jj;
  __device__ RowJ(int H) {
    hchunk = H < kThreads ? H : kThreads;
    rpb = kThreads / hchunk;
    rr = threadIdx.x / hchunk;
    jj = threadIdx.x - rr * hchunk;
  }
};

// Generic path (any D, H): admm.py:302-314 residual for the 4 gates, materialised; also
// tgt = lam/rho + S (reused by the trials) and, on the h side, z += X dWx written back.
__global__ __launch_bounds__(kThreads) void k_resid(Geom g, Hyper hp, ResidArgs a) {
  const int q = blockIdx.y;
  const bool th = (q == 2);
  const float rho = hp.rho[q];
  const int64_t BT = g.BT(), n = BT * g.H;
  float* zq = a.zc + (int64_t)q * n;
  float* tq = a.tgt + (int64_t)q * n;
  float* Rq = a.R + (int64_t)q * n;
  const float* Sq = a.S.p[q];
  const float* Lq = a.L.p[q];
  const float* dWq = a.dW ? a.dW + (int64_t)q * g.D * g.H : nullptr;
  RowJ ix(g.H);
  if (ix.rr < ix.rpb) {
    for (int64_t row = (int64_t)blockIdx.x * ix.rpb + ix.rr; row < BT; row += (int64_t)gridDim.x * ix.rpb) {
      const int64_t b = g.dT.div((uint32_t)row);
      const int t = (int)(row - b * g.T) + 1;
      const int64_t so = (b * g.TP() + t) * g.H;
      for (int j = ix.jj; j < g.H; j += ix.hchunk) {
        const int64_t e = row * g.H + j;
        float z = zq[e], tg;
        if (a.stage == 0) {
          tg = Lq[so + j] / rho + Sq[so + j];
          tq[e] = tg;
        } else {
          float dz = 0.f;
          for (int d = 0; d < g.D; ++d) dz += a.x[row * g.D + d] * dWq[d * g.H + j];
          z = z + dz;
          zq[e] = z;
          tg = tq[e];
        }
        float phi, dphi;
        if (th) {
          phi = tanhf(z);
          dphi = 1.f - phi * phi;
        } else {
          const SigPair sp = sig_pair(z);
          phi = sp.s;
          dphi = sp.s * sp.sc;
        }
        Rq[e] = (phi - tg) * dphi;
      }
    }
  }
}

// G_q = A^T R_q split over rows.  Side 1 (A = Hprev, Kd = H): 128 x 128 tiles, 2x2 waves
// of 64x64; side 0 (A = X, Kd = D small): 32 x 128 tiles.
template <bool VEC, int SIDE>
struct AtRSrc {  // A^T: A stored [row][m] (m contiguous); B = R[q] [row][j]
  const float* x; const float* Sh; const float* Rq; DivU32 dT; int D, H, Kd; int64_t rend;
  static constexpr bool A_ROW_MAJOR = false;
  __device__ float4 a4(int64_t m, int64_t row) const {
    if (row >= rend) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* base = SIDE == 0 ? x + row * D : Sh + (row + dT.div((uint32_t)row)) * H;
    if (VEC) {
      if (m >= Kd) return make_float4(0.f, 0.f, 0.f, 0.f);
      return *reinterpret_cast<const float4*>(base + m);
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (m + u < Kd) ? base[m + u] : 0.f;
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ float4 b4(int64_t row, int64_t j) const {
    if (row >= rend) return make_float4(0.f, 0.f, 0.f, 0.f);
    if (VEC) {
      if (j >= H) return make_float4(0.f, 0.f, 0.f, 0.f);
      return *reinterpret_cast<const float4*>(Rq + row * H + j);
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (j + u < H) ? Rq[row * H + j + u] : 0.f;
    return make_float4(v[0], v[1], v[2], v[3]);
  }
};

template <int BM, int WM, bool VEC, int SIDE>
__device__ __forceinline__ void atr_body(const Geom& g, const float* x, const float* Sh, const float* R,
                                         float* slab, int nsplit, float* smem) {
  constexpr int BN = 128, WN = (BM == 128) ? 64 : 32, KC = 32;
  using S = Tile<BM, BN, WM, WN, KC, false>;
  const int Kd = SIDE == 0 ? g.D : g.H;
  const int nm = (Kd + BM - 1) / BM, nn = (g.H + BN - 1) / BN;
  int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int mt = lid % nm; lid /= nm;
  const int nt = lid % nn; lid /= nn;
  const int q = lid % 4, sp = lid / 4;
  const int64_t BT = g.BT();
  const int64_t per = ((BT + nsplit - 1) / nsplit + KC - 1) / KC * KC;
  const int64_t r0 = sp * per, r1 = (r0 + per < BT) ? r0 + per : BT;
  const int m0 = mt * BM, n0 = nt * BN;
  AtRSrc<VEC, SIDE> src{x, Sh, R + (int64_t)q * BT * g.H, g.dT, g.D, g.H, Kd, r1};
  f32x16 acc[S::MT][S::NT];
  zero_acc(acc);
  Engine<BM, BN, WM, WN, KC, AtRSrc<VEC, SIDE>> eng;
  if (r0 < r1) eng.run(src, m0, n0, r0, r1, acc, smem);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm0 = (wave / S::WAVES_N) * WM, wn0 = (wave % S::WAVES_N) * WN;
  float* out = slab + ((int64_t)sp * 4 + q) * Kd * g.H;
#pragma unroll
  for (int mi = 0; mi < S::MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < S::NT; ++ni) {
      const int j = n0 + wn0 + ni * 32 + (lane & 31);
      if (j >= g.H) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + mi * 32 + acc_row(r, lane);
        if (m < Kd) out[(int64_t)m * g.H + j] = acc[mi][ni][r];
      }
    }
}

template <int BM, int WM, bool VEC, int SIDE>
__global__ __launch_bounds__(kThreads) void k_atr(Geom g, const float* x, const float* Sh,
                                                    const float* R, float* slab, int nsplit) {
  __shared__ float smem[Tile<BM, 128, WM, (BM == 128) ? 64 : 32, 32, false>::LDS_FLOATS];
  atr_body<BM, WM, VEC, SIDE>(g, x, Sh, R, slab, nsplit, smem);
}

// h-stage A^T R with the residual formed in the B-operand loader (admm.py:302-312, h side):
// z (the cached pre-activation with X dWx already applied by k_apply_dwx) and the target
// are loaded ahead of the MFMAs; R = (phi(z) - tgt) phi'(z) is formed at LDS-store time.
// R is never materialised.
template <bool TANH>
struct AtRFusedSrc {
  const float* Sh; const float* zq; const float* tq;
  DivU32 dT; int H; int64_t rend;
  static constexpr bool A_ROW_MAJOR = false;
  struct BRaw { float4 z, t; };
  __device__ float4 a4(int64_t m, int64_t row) const {
    if (row >= rend || m >= H) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *reinterpret_cast<const float4*>(Sh + (row + dT.div((uint32_t)row)) * H + m);
  }
  __device__ BRaw braw(int64_t row, int64_t j) const {
    // out of range: z = 0 with tgt = phi(0) (0.5 / 0, both exact) gives R = 0
    const float t0 = TANH ? 0.f : 0.5f;
    if (row >= rend || j >= H) return BRaw{make_float4(0.f, 0.f, 0.f, 0.f), make_float4(t0, t0, t0, t0)};
    const int64_t e = row * H + j;
    return BRaw{ld_nt(zq + e), ld_nt(tq + e)};
  }
  __device__ float4 bfin(const BRaw& v) const {
    const float zz[4] = {v.z.x, v.z.y, v.z.z, v.z.w}, tt[4] = {v.t.x, v.t.y, v.t.z, v.t.w};
    float r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float phi, dphi;
      phi_acc<TANH>(zz[u], phi, dphi);
      r[u] = (phi - tt[u]) * dphi;
    }
    return make_float4(r[0], r[1], r[2], r[3]);
  }
};

template <int BM, int WM, int KC, bool TANH>
__device__ __forceinline__ void atr_fused_body(const Geom& g, const float* x, const float* Sh, const float* zc,
                                               const float* tgt, const float* dW, float* slab, int nsplit,
                                               float* smem) {
  constexpr int BN = 128, WN = 64;
  using S = Tile<BM, BN, WM, WN, KC, false>;
  const int nm = (g.H + BM - 1) / BM, nn = (g.H + BN - 1) / BN;
  int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int mt = lid % nm; lid /= nm;
  const int nt = lid % nn; lid /= nn;
  const int q = lid % 4, sp = lid / 4;
  const int64_t BT = g.BT(), n = BT * g.H;
  const int64_t per = ((BT + nsplit - 1) / nsplit + KC - 1) / KC * KC;
  const int64_t r0 = sp * per, r1 = (r0 + per < BT) ? r0 + per : BT;
  const int m0 = mt * BM, n0 = nt * BN;
  AtRFusedSrc<TANH> src{Sh, zc + (int64_t)q * n, tgt + (int64_t)q * n, g.dT, g.H, r1};
  f32x16 acc[S::MT][S::NT];
  zero_acc(acc);
  Engine<BM, BN, WM, WN, KC, AtRFusedSrc<TANH>> eng;
  if (r0 < r1) eng.run(src, m0, n0, r0, r1, acc, smem);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm0 = (wave / S::WAVES_N) * WM, wn0 = (wave % S::WAVES_N) * WN;
  float* out = slab + ((int64_t)sp * 4 + q) * g.H * g.H;
#pragma unroll
  for (int mi = 0; mi < S::MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < S::NT; ++ni) {
      const int j = n0 + wn0 + ni * 32 + (lane & 31);
      if (j >= g.H) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + mi * 32 + acc_row(r, lane);
        if (m < g.H) out[(int64_t)m * g.H + j] = acc[mi][ni][r];
      }
    }
}

// Tiles: BM = 128 (2 x 2 waves of 64 x 64, KC = 32) or BM = 256 (the whole hidden dim of the
// A^T side for H = 256: z and tgt are then streamed once; 2 x 2 waves of 128 x 64, KC = 16).
template <int BM, int WM, int KC>
__global__ __launch_bounds__(kThreads) void k_atr_fused(Geom g, const float* x, const float* Sh, const float* zc,
                                                          const float* tgt, const float* dW, float* slab, int nsplit) {
  __shared__ float smem[Tile<BM, 128, WM, 64, KC, false>::LDS_FLOATS];
  const int nm = (g.H + BM - 1) / BM, nn = (g.H + 127) / 128;
  if ((xcd_swizzle(blockIdx.x, gridDim.x) / (nm * nn)) % 4 == 2)
    atr_fused_body<BM, WM, KC, true>(g, x, Sh, zc, tgt, dW, slab, nsplit, smem);
  else
    atr_fused_body<BM, WM, KC, false>(g, x, Sh, zc, tgt, dW, slab, nsplit, smem);
}

__global__ __launch_bounds__(kThreads) void k_reduce_g(int Kd, int H, int side, int p16, Hyper hp, const float* slab,
                                                         int nsplit, float* G, int* found, int* kpred,
                                                         const DevStats* stats, float* range_reset) {
  const int64_t per_q = (int64_t)Kd * H;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  // the h stage's k_atr3w has read the ranges: clear them for the sweep that follows (SweepT::range)
  if (range_reset && i < 5) range_reset[i] = 0.f;
  if (i < 4) {
    found[i] = 0;   // this stage's line searches start undecided (no memset launch)
    if (kpred) kpred[i] = stats->k[2 * i];   // last step's x-side exponent (SpecX)
    // hint: the gate's last exponent on this side was past pass 0's window, so pass 0 also forms
    // the per-candidate elements' polynomial for k >= kTrialJ (dq_hint, k_select)
    found[8 + i] = p16 && stats->k[2 * i + side] >= kTrialJ ? 1 : 0;
  }
  if (i >= 4 * per_q) return;
  const int q = (int)(i / per_q);
  // sequential fp64 sum over the splits (fixed order: deterministic), loads issued 8 at a time
  const float* p = slab + i;
  const int64_t st = 4 * per_q;
  double s = 0.0;
  int sp = 0;
  // 32 loads in flight while there are that many splits (the x side reduces the sweep's 256
  // per-workgroup slabs with only 64 workgroups), then 8; the summation order is the same
  for (; sp + 32 <= nsplit; sp += 32) {
    float v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = p[(int64_t)(sp + u) * st];
#pragma unroll
    for (int u = 0; u < 32; ++u) s += (double)v[u];
  }
  for (; sp + 8 <= nsplit; sp += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(sp + u) * st];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (double)v[u];
  }
  for (; sp < nsplit; ++sp) s += (double)p[(int64_t)sp * st];
  G[i] = (float)s * hp.rho[q];  // (sum_t A_t^T R_t) * rho (admm.py:312)
}

// The h stage's reduce (one process, split3 Q GEMM): k_reduce_g's G_q = rho_q sum_sp slab (the same
// sequential fp64 sum over the splits, so the same bits) for the eight rows of one k_qgemm3 B
// fragment per thread, which it also writes to the split G image (k_split_g's layout and split), so
// k_split_g's launch is not needed.  gi[(((q * NK + c) * NTT + n) * 3 + p) * 64 + lane] = piece p of
// G_q[16c + 8(lane>>5) + e][32n + (lane&31)], e = 0..7.
__global__ __launch_bounds__(kThreads) void k_reduce_gh_img(int H, int p16, Hyper hp, const float* __restrict__ slab,
                                                              int nsplit, float* __restrict__ G, int* found,
                                                              const DevStats* stats, float* range_reset,
                                                              bf16x8* __restrict__ gi) {
  const int NK = H / 16, NTT = H / 32;
  const int64_t per_q = (int64_t)H * H;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (range_reset && i < 5) range_reset[i] = 0.f;
  if (i < 4) {
    found[i] = 0;
    found[8 + i] = p16 && stats->k[2 * i + 1] >= kTrialJ ? 1 : 0;
  }
  if (i >= 4 * NK * NTT * 64) return;
  const int lane = i & 63, n = (i >> 6) % NTT, c = (i / (64 * NTT)) % NK, q = i / (64 * NTT * NK);
  const int j = 32 * n + (lane & 31), k0 = 16 * c + 8 * (lane >> 5);
  const float* p = slab + (int64_t)q * per_q + (int64_t)k0 * H + j;
  const int64_t st = 4 * per_q;
  double s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.0;
  int sp = 0;
  for (; sp + 4 <= nsplit; sp += 4) {   // 32 loads in flight; each element's sum in split order
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[u][e] = p[(int64_t)(sp + u) * st + (int64_t)e * H];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += (double)v[u][e];
  }
  for (; sp < nsplit; ++sp)
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += (double)p[(int64_t)sp * st + (int64_t)e * H];
  float __attribute__((ext_vector_type(8))) gv;
  float* Gq = G + (int64_t)q * per_q + (int64_t)k0 * H + j;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    gv[e] = (float)s[e] * hp.rho[q];   // as k_reduce_g (admm.py:312)
    Gq[(int64_t)e * H] = gv[e];
  }
  bf16x8 p0, p1, p2;
  split3(gv, p0, p1, p2);
  const int base = (((q * NK + c) * NTT + n) * 3) * 64 + lane;
  gi[base] = p0;
  gi[base + 64] = p1;
  gi[base + 128] = p2;
}

template <bool VEC, int SIDE>
struct QSrc {  // A = X or Hprev rows (row-major, K = Kd); B = G_q [Kd][H]
  const float* x; const float* Sh; const float* G; int64_t BT; DivU32 dT; int D, H, Kd, j0;
  static constexpr bool A_ROW_MAJOR = true;
  __device__ float4 a4(int64_t row, int64_t k) const {
    if (row >= BT) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* base = SIDE == 0 ? x + row * D : Sh + (row + dT.div((uint32_t)row)) * H;
    if (VEC) {
      if (k >= Kd) return make_float4(0.f, 0.f, 0.f, 0.f);
      return *reinterpret_cast<const float4*>(base + k);
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (k + u < Kd) ? base[k + u] : 0.f;
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ float4 b4(int64_t k, int64_t n) const {
    const int q = (int)(n >> 5), j = j0 + (int)(n & 31);
    if (VEC) {
      if (k >= Kd || j >= H) return make_float4(0.f, 0.f, 0.f, 0.f);
      return *reinterpret_cast<const float4*>(G + ((int64_t)q * Kd + k) * H + j);
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = (k < Kd && j + u < H && (j + u - j0) < 32 * (q + 1)) ? G[((int64_t)q * Kd + k) * H + j + u] : 0.f;
    return make_float4(v[0], v[1], v[2], v[3]);
  }
};

// Q_q = A G_q: the trial direction, so that z(W + G/theta) = z(W) + Q / theta exactly.
template <bool VEC, int SIDE>
__device__ __forceinline__ void qgemm_body(const Geom& g, const float* x, const float* Sh, const float* G,
                                           float* Q, float* smem) {
  const int Kd = SIDE == 0 ? g.D : g.H;
  const int nj = (g.H + 31) / 32;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)(lid / nj) * TS_BM;
  const int j0 = (lid % nj) * 32;
  const int64_t BT = g.BT();
  QSrc<VEC, SIDE> src{x, Sh, G, BT, g.dT, g.D, g.H, Kd, j0};
  f32x16 acc[1][4];
  zero_acc(acc);
  Engine<TS_BM, TS_BN, TS_WM, TS_WN, TS_KC, QSrc<VEC, SIDE>> eng;
  eng.run(src, m0, 0, 0, Kd, acc, smem);
  const int lane = threadIdx.x & 63, wm0 = (threadIdx.x >> 6) * TS_WM;
  const int j = j0 + (lane & 31);
  if (j >= g.H) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = m0 + wm0 + acc_row(r, lane);
    if (row >= BT) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) st_nt(Q + ((int64_t)q * BT + row) * g.H + j, acc[0][q][r]);
  }
}

template <bool VEC, int SIDE>
__global__ __launch_bounds__(kThreads) void k_qgemm(Geom g, const float* x, const float* Sh,
                                                      const float* G, float* Q) {
  __shared__ float smem[TSTile::LDS_FLOATS];
  qgemm_body<VEC, SIDE>(g, x, Sh, G, Q, smem);
}

// Trial pass.  For the line search (admm.py:316-336) each gate needs, for k = 0, 1, ...,
//   f(W + G/2^k) - f(W) = 0.5 rho sum_e [ (d0 + D_k)^2 - d0^2 ],  D_k = phi(z + q 2^-k) - phi(z),
// evaluated without cancellation (DESIGN.md "line-search numerics").  Two regimes per element:
//  * |q| <= kPolyQ = 2^-4 (the common case): D_k = sum_{n<=5} a_n s^n with s = 2^-k and a_n = c_n q^n
//    (5-term Taylor: truncation |c6/c1| (qs)^5, about 1e-7 of D for tanh at qs = 2^-4 and 2^-5 times
//    less per exponent beyond; round 3's bound 2^-5 gave 3e-9 but left most of the g gate's elements
//    to the per-candidate loop), so the increment is a degree-10 polynomial in s whose
//    10 coefficients are summed once (pass 0) and cover every exponent;
//  * otherwise: D_k per candidate of the pass window k in [pass*J, pass*J + J), branch-free
//    (see trial_direct).
// Slot layout per gate: kSlots = [J candidates][6 poly][sum d0^2][#per-candidate elements].
constexpr int kSlots = kTrialSlots;
constexpr int kSlotPoly = kTrialJ, kSlotFw = kTrialJ + kPolyN, kSlotNne = kTrialJ + kPolyN + 1;
constexpr int kSlotP16 = kSlotNne + 1, kSlotN16 = kSlotP16 + kPolyHiN;

// Per-wave queue of the elements in the per-candidate regime.  Which elements need the
// 16-candidate loop is data dependent (on C3, 0-95 % per gate), so evaluating it in place
// would run the loop for the whole wave whenever any lane needs it.  Instead each element's
// five inputs are appended (ballot + prefix count) to an LDS ring of this wave, and the
// loop runs once 64 entries are pending, with every lane busy.  All lanes of a wave must
// make the same sequence of dq_push / dq_run calls (loops below are wave-uniform).
constexpr int kDQ = 256;   // ring capacity: pending <= 63 before up to two pushes of <= 64 (trial_pair)
struct DirectQ {
  // the pushes (ds_write) and the run's reads (ds_read) of other lanes' entries address the same
  // array, so they stay in program order, and a wave's LDS operations execute in order: no
  // memory fence (a fence would also order, and so de-scalarise, the caller's global loads)
  float* buf;              // this wave's [3][kDQ] in LDS
  int head, tail;          // wave-uniform counters
  // pass 0 with the gate's hint set (its previous exponent was past the first window): the
  // per-candidate elements also accumulate their Taylor polynomial, valid for k >= kTrialJ, into
  // p16 ([kPolyHiN + 1][64] per wave in LDS, lane-indexed) so that k_select can decide
  // exponents past the window without another pass
  float* p16 = nullptr;
  bool hi = false;
};
constexpr int kDQLds = 3 * kDQ + (kPolyHiN + 1) * 64;   // floats of one wave's queue + p16

// enable the p16 polynomial for this block (pass 0, gate hint set: found[8 + q], k_reduce_g)
__device__ __forceinline__ void dq_hint(DirectQ& dq, int pass, const int* found, int q) {
  dq.p16 = dq.buf + 3 * kDQ;
  dq.hi = pass == 0 && found[8 + q] != 0;
  if (dq.hi) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int m = 0; m <= kPolyHiN; ++m) dq.p16[m * 64 + lane] = 0.f;
  }
}

// sw = f2 sg w (the pushed entry): w = |z| (sigmoid) or 2|z| (tanh) with the sign of z; E and
// r = sigma(w) are re-formed here exactly as trial_point / trial_pair formed them
#ifndef DC_ABL
#define DC_ABL 0   // timing ablations for tools/kbench (wrong sums): 1 no candidate loop, 2 four candidates,
                   // 4 no queue (profiles/r05k_trial_gate_imbalance.txt)
#endif
template <bool TANH>
__device__ __forceinline__ void direct_candidates(float sw, float e, float d2, float (&acc)[kSlots], const DirectQ& dq) {
  const float w = fabsf(sw);
  const float E = __expf(-w);
  const float r = __builtin_amdgcn_rcpf(1.f + E);
  const float F = sw >= 0.f ? (TANH ? 2.f : 1.f) : (TANH ? -2.f : -1.f);   // D = F (sigma(w + eps) - sigma(w))
  const float cr = -F * r;
  if (dq.hi) {
    // the element's Taylor polynomial in s for k >= kTrialJ: D = sum_n a_n s^n, a_n = F c_n(w) E0^n,
    // E0 = e 2^(J-1) = F q (pass 0), valid while |E0| s <= kPolyQ; remainder coefficients of s^2..s^10
    const int lane = threadIdx.x & 63;
    const float E0 = e * (float)(1 << (kTrialJ - 1));
    if (fabsf(E0) <= kPolyQ * (float)(1 << kTrialJ)) {
      const float sc = E * r;                       // 1 - sigma(w)
      const float p = r * sc, h = sc - r;           // sigma', 1 - 2 sigma
      const float e2 = E0 * E0;
      const float a1 = F * p * E0, a2 = F * (0.5f * p * h) * e2, a3 = F * (p * (1.f - 6.f * p) * (1.f / 6.f)) * e2 * E0;
      const float a4 = F * (p * h * (1.f - 12.f * p) * (1.f / 24.f)) * e2 * e2;
      const float a5 = F * (p * (1.f - 30.f * p + 120.f * p * p) * (1.f / 120.f)) * e2 * e2 * E0;
      const float t = d2;
      float* P = dq.p16 + lane;
      P[0 * 64] += fmaf(t, a2, a1 * a1);
      P[1 * 64] += fmaf(t, a3, 2.f * a1 * a2);
      P[2 * 64] += fmaf(t, a4, fmaf(2.f * a1, a3, a2 * a2));
      P[3 * 64] += fmaf(t, a5, 2.f * fmaf(a1, a4, a2 * a3));
      P[4 * 64] += fmaf(2.f * a1, a5, fmaf(2.f * a2, a4, a3 * a3));
      P[5 * 64] += 2.f * fmaf(a2, a5, a3 * a4);
      P[6 * 64] += fmaf(2.f * a3, a5, a4 * a4);
      P[7 * 64] += 2.f * a4 * a5;
      P[8 * 64] += a5 * a5;
    } else {
      dq.p16[kPolyHiN * 64 + lane] += 1.f;
    }
  }
  constexpr float kCap = 1e30f;
  float m = fminf(expm1_acc(-e), kCap);
  const float one_e = 1.f + E;
  // the element's first-order term: D is linear in y = E expm1(-e) ~ -E e to first order, so
  // D_lin = cr (-E e) r at the smallest candidate, doubling with e.  k_select compares the
  // remainder past it, so its share 2 d0 D_lin / s goes into the s^1 polynomial coefficient
  // (used from pass 0 only; the scale is pass 0's smallest candidate 2^-(J-1))
  acc[kSlotPoly + 0] -= d2 * ((cr * (-E * e)) * r) * (float)(1 << (kTrialJ - 1));
  if (DC_ABL & 1) return;
  constexpr int kLo = (DC_ABL & 2) ? kTrialJ - 4 : 0;
  if (fabsf(e) * (float)(1 << (kTrialJ - 1)) <= 20.f) {   // |e| <= 20 on every candidate: no exp
    // two candidates at a time on packed f32 operations (v_pk_mul / v_pk_add), the same operations
    // per candidate as the scalar loop below, so the same bits
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int k = kTrialJ - 1; k >= kLo + 1; k -= 2) {
      const float m1 = m * (m + 2.f);   // candidate k - 1
      const f2 y = E * f2{m, m1};
      const f2 den = one_e + y;
      const f2 D = (cr * y) * f2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
      const f2 dd = d2 + D;
      acc[k] = fmaf(D.x, dd.x, acc[k]);
      acc[k - 1] = fmaf(D.y, dd.y, acc[k - 1]);
      m = m1 * (m1 + 2.f);
    }
    return;
  }
#pragma unroll
  for (int k = kTrialJ - 1; k >= kLo; --k) {
    const float yb = fminf(__expf(-e - w), kCap);
    const float y = -e > 20.f ? yb : E * m;
    const float D = (cr * y) * __builtin_amdgcn_rcpf(one_e + y);
    acc[k] = fmaf(D, d2 + D, acc[k]);
    m = fminf(m * (m + 2.f), kCap);
    e *= 2.f;
  }
}

// An entry is (sw, e, d2): sw = the signed w (E, r and the sign are re-formed from it when the
// entry runs, one v_exp and one v_rcp per 64 entries instead of two more LDS words per push).
__device__ __forceinline__ void dq_push(DirectQ& dq, bool p, float sw, float e, float d2) {
  if (DC_ABL & 4) p = false;
  const unsigned long long m = __builtin_amdgcn_ballot_w64(p);
  if (p) {
    // this lane's rank among the pushing lanes: v_mbcnt_lo / v_mbcnt_hi on the ballot
    const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    const int slot = (dq.tail + rank) & (kDQ - 1);
    dq.buf[slot] = sw;
    dq.buf[kDQ + slot] = e;
    dq.buf[2 * kDQ + slot] = d2;
  }
  dq.tail += __popcll(m);
}

// final: also counts the wave's per-candidate elements (every push, in lane 0's slot) -- the
// number of elements the pass could not cover with the polynomial (k_select's poly_only test)
template <bool TANH>
__device__ __forceinline__ void dq_run(DirectQ& dq, float (&acc)[kSlots], bool final) {
  if (final && (threadIdx.x & 63) == 0) acc[kSlotNne] += (float)dq.tail;
  while (dq.tail - dq.head >= 64 || (final && dq.tail > dq.head)) {
    __builtin_amdgcn_wave_barrier();
    const int lane = threadIdx.x & 63;
    const int n = dq.tail - dq.head < 64 ? dq.tail - dq.head : 64;
    if (lane < n) {
      const int slot = (dq.head + lane) & (kDQ - 1);
      direct_candidates<TANH>(dq.buf[slot], dq.buf[kDQ + slot], dq.buf[2 * kDQ + slot], acc, dq);
    }
    dq.head += n;
  }
  if (final && dq.hi) {   // the lane's p16 sums into the block's slots
    __builtin_amdgcn_wave_barrier();
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int m = 0; m <= kPolyHiN; ++m) acc[kSlotP16 + m] += dq.p16[m * 64 + lane];
  }
}

// One element of a trial pass: f(W) and polynomial terms in place; per-candidate elements
// (|q| > kPolyQ) go to the wave's queue.  valid = false: no contribution (still pushes).
//
// Per-candidate form.  With w = |z| (sigmoid) and sg = sign z,
// sigma(z + d) - sigma(z) = sg [sigma(w + e) - sigma(w)], e = sg d, and with E = exp(-w),
// m = expm1(-e), y = E m:
//   sigma(w + e) - sigma(w) = -sigma(w) y / (1 + E + y)
// (no cancellation: m carries the difference).  tanh x = 2 sigma(2x) - 1 gives the tanh gate
// with w = 2|z|, e = 2 sg d and a factor 2.  Along the window d halves, so
// m_k = m_{k+1} (m_{k+1} + 2): one expm1 for the smallest d, then a multiply per candidate
// (relative error grows < 1 ulp per step).  Where -e > 20, m = exp(-e) to 2e-9 and
// y = exp(-e - w) is taken directly instead (E may underflow while y does not); y is capped
// at 1e30, where y / (1 + E + y) = 1 (the saturated limit D = -sg sigma(w)).
template <bool TANH>
__device__ __forceinline__ void trial_point(bool valid, float z, float tg, float qv, int pass, float (&acc)[kSlots],
                                            DirectQ& dq) {
  bool direct = false;
  float e = 0.f, E = 0.f, w = 0.f, d2 = 0.f;
  if (valid) {
    // E = exp(-w), r = sigma(w), sc = 1 - sigma(w) on w = |z| (sigmoid) or 2|z| (tanh)
    w = TANH ? 2.f * fabsf(z) : fabsf(z);
    E = __expf(-w);
    const float r = __builtin_amdgcn_rcpf(1.f + E);
    const float sc = E * r;
    // Taylor coefficients c_n = phi^(n)(z) / n!, n = 1..5, from phi and phi' (no cancellation)
    float d0, c1, c2, c3, c4, c5;
    if (TANH) {
      const float mz = 2.f * sc;                    // 1 - |tanh z|
      const float u = copysignf(1.f - mz, z);
      const float v = mz * (2.f - mz);              // 1 - u^2
      const float u2 = u * u;
      c1 = v;
      c2 = -u * v;
      c3 = v * (u2 - (1.f / 3.f));
      c4 = u * v * (2.f - 3.f * u2) * (1.f / 3.f);
      c5 = v * (2.f - 15.f * u2 * v) * (1.f / 15.f);
      d0 = copysignf(-expm1_acc(-w) * r, z) - tg;  // tanh z = sg (1 - E) / (1 + E)
    } else {
      const float s = z >= 0.f ? r : sc, s_c = z >= 0.f ? sc : r;   // = sig_pair(z)
      const float p = s * s_c, h = s_c - s;        // sigma', 1 - 2 sigma
      c1 = p;
      c2 = 0.5f * p * h;
      c3 = p * (1.f - 6.f * p) * (1.f / 6.f);
      c4 = p * h * (1.f - 12.f * p) * (1.f / 24.f);
      c5 = p * (1.f - 30.f * p + 120.f * p * p) * (1.f / 120.f);
      d0 = s - tg;
    }
    acc[kSlotFw] += d0 * d0;
    if (fabsf(qv) <= kPolyQ) {
      if (pass == 0) {
        // D(s) = sum_n a_n s^n, a_n = c_n q^n; increment D (2 d0 + D) = sum_j P_j s^j, j = 1..10
        const float q2 = qv * qv;
        const float a1 = c1 * qv, a2 = c2 * q2, a3 = c3 * q2 * qv, a4 = c4 * q2 * q2, a5 = c5 * q2 * q2 * qv;
        const float t = 2.f * d0;
        // (the first-order term t a1 is left out: the search compares the remainder past it,
        // see k_select)
        acc[kSlotPoly + 1] += fmaf(t, a2, a1 * a1);
        acc[kSlotPoly + 2] += fmaf(t, a3, 2.f * a1 * a2);
        acc[kSlotPoly + 3] += fmaf(t, a4, fmaf(2.f * a1, a3, a2 * a2));
        acc[kSlotPoly + 4] += fmaf(t, a5, 2.f * fmaf(a1, a4, a2 * a3));
        acc[kSlotPoly + 5] += fmaf(2.f * a1, a5, fmaf(2.f * a2, a4, a3 * a3));
        acc[kSlotPoly + 6] += 2.f * fmaf(a2, a5, a3 * a4);
        acc[kSlotPoly + 7] += fmaf(2.f * a3, a5, a4 * a4);
        acc[kSlotPoly + 8] += 2.f * a4 * a5;
        acc[kSlotPoly + 9] += a5 * a5;
      }
    } else {
      direct = true;
      const float sg = z >= 0.f ? 1.f : -1.f;
      const float f2 = TANH ? 2.f : 1.f;
      e = (f2 * sg) * qv * ldexpf(1.f, -(pass * kTrialJ + kTrialJ - 1));   // smallest candidate
      d2 = 2.f * d0;
    }
  }
  dq_push(dq, direct, z >= 0.f ? w : -w, e, d2);
}

// Two elements of a trial pass at once (the fast path's float4 halves), in packed f32
// (v_pk_fma_f32 / v_pk_mul_f32): same arithmetic as trial_point, branch-free.  Elements past
// the polynomial bound contribute q = 0 to the polynomial sums and go to the wave's queue.
// acc2 holds the f(W) sum (slot 0) and the kPolyN polynomial sums (slots 1..kPolyN) per lane
// pair; they are folded into acc at the end of the pass.
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kPair = kPolyN + 1;
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) {   // v_pk_fma_f32
  return f32x2{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)};
}

template <bool TANH>
__device__ __forceinline__ void trial_pair(bool ok, f32x2 z, f32x2 tg, f32x2 qv, int pass, float (&acc)[kSlots],
                                           f32x2 (&acc2)[kPair], DirectQ& dq, bool ok_y = true) {
  const f32x2 az = f32x2{fabsf(z.x), fabsf(z.y)};
  const f32x2 w = TANH ? 2.f * az : az;
  const f32x2 E = f32x2{__expf(-w.x), __expf(-w.y)};
  const f32x2 r = f32x2{__builtin_amdgcn_rcpf(1.f + E.x), __builtin_amdgcn_rcpf(1.f + E.y)};
  const f32x2 sc = E * r;
  // Taylor coefficients c_n = phi^(n)(z) / n! in factored form: with the trial direction q,
  // a_n = c_n q^n is a1 = c1 q, a2 = a1 (g2 q), a3 = a1 q^2 k3, a4 = a1 q^2 (g2 q) k4,
  // a5 = a1 q^4 k5 (trial_point has the c_n themselves)
  f32x2 d0, c1, g2, k3, k4, k5;
  if (TANH) {
    const f32x2 mz = 2.f * sc;                    // 1 - |tanh z|
    const f32x2 um = 1.f - mz;
    const f32x2 u = f32x2{copysignf(um.x, z.x), copysignf(um.y, z.y)};
    const f32x2 v = mz * (2.f - mz);              // 1 - u^2
    const f32x2 u2 = u * u;
    c1 = v;                                       // c2 = -u v, c3 = v (u^2 - 1/3),
    g2 = -u;                                      // c4 = u v (2 - 3 u^2) / 3,
    k3 = u2 - (1.f / 3.f);                        // c5 = v (2 - 15 u^2 v) / 15
    k4 = u2 - (2.f / 3.f);
    k5 = fma2(-u2, v, f32x2{2.f / 15.f, 2.f / 15.f});
    // |tanh z| = -expm1(-w) r: degree-8 Taylor of expm1 on |w| < 1/2, else exp - 1
    const f32x2 xm = -w;
    f32x2 pe = 1.f / 40320.f;
    pe = pe * xm + 1.f / 5040.f; pe = pe * xm + 1.f / 720.f; pe = pe * xm + 1.f / 120.f;
    pe = pe * xm + 1.f / 24.f; pe = pe * xm + 1.f / 6.f; pe = pe * xm + 0.5f; pe = pe * xm + 1.f;
    pe = pe * xm;
    const f32x2 em = f32x2{w.x < 0.5f ? pe.x : E.x - 1.f, w.y < 0.5f ? pe.y : E.y - 1.f};
    const f32x2 th = -em * r;
    d0 = f32x2{copysignf(th.x, z.x), copysignf(th.y, z.y)} - tg;
  } else {
    const f32x2 sg = f32x2{z.x >= 0.f ? r.x : sc.x, z.y >= 0.f ? r.y : sc.y};   // sigma(z)
    const f32x2 sgc = f32x2{z.x >= 0.f ? sc.x : r.x, z.y >= 0.f ? sc.y : r.y};  // 1 - sigma(z)
    const f32x2 p = sg * sgc, h = sgc - sg;
    c1 = p;                                       // c2 = p h / 2, c3 = p (1 - 6p) / 6,
    g2 = 0.5f * h;                                // c4 = p h (1 - 12p) / 24,
    k3 = (1.f / 6.f) - p;                         // c5 = p (1 - 30p + 120p^2) / 120
    k4 = (1.f / 12.f) - p;
    k5 = fma2(p, p - 0.25f, f32x2{1.f / 120.f, 1.f / 120.f});
    d0 = sg - tg;
  }
  const f32x2 okm = f32x2{ok ? 1.f : 0.f, ok && ok_y ? 1.f : 0.f};
  d0 = d0 * okm;
  acc2[0] += d0 * d0;
  const bool px = fabsf(qv.x) <= kPolyQ, py = fabsf(qv.y) <= kPolyQ;
  if (pass == 0) {
    // the same ten sums as fma chains into the accumulators, with b_n = 2 a_n (24 instead of
    // ~30 packed operations per pair; the rounding of each sum's terms differs in the last bit)
    const f32x2 qp = f32x2{px ? qv.x : 0.f, py ? qv.y : 0.f};
    const f32x2 q2 = qp * qp, gq = g2 * qp;
    const f32x2 a1 = c1 * qp, a2 = a1 * gq, w3 = a1 * q2;
    const f32x2 a3 = w3 * k3, a4 = (w3 * gq) * k4, a5 = (w3 * q2) * k5;
    const f32x2 t = 2.f * d0, b1 = 2.f * a1, b2 = 2.f * a2, b3 = 2.f * a3, b4 = 2.f * a4;
    // s^1 (acc2[1]): the first-order term t a1 is left out -- the search compares the remainder
    // past it (k_select); the per-candidate elements subtract theirs in direct_candidates
    acc2[2] = fma2(a1, a1, fma2(t, a2, acc2[2]));
    acc2[3] = fma2(b1, a2, fma2(t, a3, acc2[3]));
    acc2[4] = fma2(a2, a2, fma2(b1, a3, fma2(t, a4, acc2[4])));
    acc2[5] = fma2(b2, a3, fma2(b1, a4, fma2(t, a5, acc2[5])));
    acc2[6] = fma2(a3, a3, fma2(b2, a4, fma2(b1, a5, acc2[6])));
    acc2[7] = fma2(b3, a4, fma2(b2, a5, acc2[7]));
    acc2[8] = fma2(a4, a4, fma2(b3, a5, acc2[8]));
    acc2[9] = fma2(b4, a5, acc2[9]);
    acc2[10] = fma2(a5, a5, acc2[10]);
  }
  // per-candidate elements: sigma(w + e) - sigma(w) form (see trial_point)
  const f32x2 f2sg = f32x2{(TANH ? 2.f : 1.f) * (z.x >= 0.f ? 1.f : -1.f), (TANH ? 2.f : 1.f) * (z.y >= 0.f ? 1.f : -1.f)};
  const float s0 = ldexpf(1.f, -(pass * kTrialJ + kTrialJ - 1));   // smallest candidate
  const bool dx = ok && !px, dy = ok && ok_y && !py;
  dq_push(dq, dx, z.x >= 0.f ? w.x : -w.x, f2sg.x * qv.x * s0, 2.f * d0.x);
  dq_push(dq, dy, z.y >= 0.f ? w.y : -w.y, f2sg.y * qv.y * s0, 2.f * d0.y);
}

__device__ __forceinline__ void trial_pair_fold(float (&acc)[kSlots], const f32x2 (&acc2)[kPair]) {
  acc[kSlotFw] += acc2[0].x + acc2[0].y;
#pragma unroll
  for (int n = 0; n < kPolyN; ++n) acc[kSlotPoly + n] += acc2[n + 1].x + acc2[n + 1].y;
}

// Trial kernels take pass >= 0 (one window) or pass = kTailPass: the tail, windows 1 ..
// kMaxPasses - 1 one after the other in the same launch (their partials at part + (p - 1) times
// 4 kSlots nred), for the gates pass 0 left undecided.  One launch, one selection and (multi-
// process) one all-reduce replace three passes that almost never have work to do.
__device__ __forceinline__ int pass_lo(int pass) { return pass == kTailPass ? 1 : pass; }
__device__ __forceinline__ int pass_hi(int pass) { return pass == kTailPass ? kMaxPasses : pass + 1; }

// Per-slot wave sums of v[0 .. N) (N <= 64): lane s ends with slot s's sum over the wave's 64 lanes,
// bitwise equal to wave_sum(v[s]) -- the same pairs of partial sums, lanes 32 apart first, and IEEE
// addition commutes -- in 63 shuffles instead of 6 N: at each butterfly stage a lane keeps the half
// of its slots that its lane bit selects and sends the other half to its partner.  (k_select's 38
// slots through wave_sum took 13 of its 18-19 us, tools/kbench "sel"; every trial workgroup's
// epilogue reduces the same 38 slots.)
template <typename T, int N>
__device__ __forceinline__ T wave_sum_slots(T (&v)[N]) {   // in place: v is consumed
  static_assert(N <= 64, "one slot per lane");
  const int lane = threadIdx.x & 63;
  {
    const bool up = lane & 32;
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      const T lo = s < N ? v[s] : T(0), hi = s + 32 < N ? v[s + 32] : T(0);
      if (s < N) v[s] = (up ? hi : lo) + __shfl_xor(up ? lo : hi, 32, kWave);
    }
  }
#pragma unroll
  for (int wdt = 16; wdt >= 1; wdt /= 2) {
    const bool b = lane & wdt;
#pragma unroll
    for (int s = 0; s < wdt; ++s)
      if (s < N) {
        const T lo = v[s], hi = s + wdt < N ? v[s + wdt] : T(0);
        v[s] = (b ? hi : lo) + __shfl_xor(b ? lo : hi, wdt, kWave);
      }
  }
  return v[0];
}

// WT: agent-scope stores for a reader in another workgroup of the same launch (the fused tail
// selection, tail_select_last, which releases them)
template <bool WT = false>
__device__ __forceinline__ void trial_block_store(float (&acc)[kSlots], double* part, int q, int blk, int nblk) {
  __shared__ double red[4][kSlots];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float s = wave_sum_slots(acc);   // lane k: slot k (wave_sum's bits)
  if (lane < kSlots) red[w][lane] = (double)s;
  __syncthreads();
  if (threadIdx.x < kSlots) {
    const int k = threadIdx.x;
    const double v = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
    if constexpr (WT) {
      // (released to agent scope by the same wave's fence in tail_select_last: all storing threads are wave 0)
      __hip_atomic_store(&part[((int64_t)q * kSlots + k) * nblk + blk], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      part[((int64_t)q * kSlots + k) * nblk + blk] = v;
    }
  }
}

// Generic trial pass: materialised z (zc) and Q.  The loop is wave-uniform (see DirectQ).
template <bool TANH, int VEC>
__device__ __forceinline__ void trial_loop(int64_t n, const float* zq, const float* tq, const float* Qq, int pass,
                                           int blk, int nblk, float (&acc)[kSlots], DirectQ& dq) {
  const int64_t nv = n / VEC;
  const int64_t stride = (int64_t)nblk * kThreads;
  for (int64_t base = (int64_t)blk * kThreads; base < nv; base += stride) {
    const int64_t v = base + threadIdx.x;
    const bool ok = v < nv;
    if (VEC == 4) {
      float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f), t4 = z4, q4 = z4;
      if (ok) {
        z4 = reinterpret_cast<const float4*>(zq)[v];
        t4 = reinterpret_cast<const float4*>(tq)[v];
        q4 = reinterpret_cast<const float4*>(Qq)[v];
      }
#pragma unroll 1
      for (int u = 0; u < 4; ++u) {
        const float zu = u == 0 ? z4.x : (u == 1 ? z4.y : (u == 2 ? z4.z : z4.w));
        const float tu = u == 0 ? t4.x : (u == 1 ? t4.y : (u == 2 ? t4.z : t4.w));
        const float qu = u == 0 ? q4.x : (u == 1 ? q4.y : (u == 2 ? q4.z : q4.w));
        trial_point<TANH>(ok, zu, tu, qu, pass, acc, dq);
        dq_run<TANH>(dq, acc, false);
      }
    } else {
      trial_point<TANH>(ok, ok ? zq[v] : 0.f, ok ? tq[v] : 0.f, ok ? Qq[v] : 0.f, pass, acc, dq);
      dq_run<TANH>(dq, acc, false);
    }
  }
  dq_run<TANH>(dq, acc, true);
}

template <bool TAIL>
__global__ __launch_bounds__(kThreads) void k_trial(Geom g, int pass, const float* zc, const float* tgt,
                                                      const float* Q, const int* found, double* part, int nblk) {
  const int q = blockIdx.y, blk = blockIdx.x;  // gate-major: one code path per CU at a time (I-cache)
  if (found[q]) return;
  const int64_t n = g.BT() * g.H;
  const float* zq = zc + (int64_t)q * n;
  const float* tq = tgt + (int64_t)q * n;
  const float* Qq = Q + (int64_t)q * n;
  __shared__ float dqbuf[kThreads / 64][kDQLds];
  const bool vec = (g.H % 4) == 0;
  for (int ps = TAIL ? 1 : pass; ps < (TAIL ? kMaxPasses : pass + 1); ++ps) {
    float acc[kSlots];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) acc[k] = 0.f;
    DirectQ dq{dqbuf[threadIdx.x >> 6], 0, 0};
    dq_hint(dq, ps, found, q);
    if (q == 2) {
      if (vec) trial_loop<true, 4>(n, zq, tq, Qq, ps, blk, nblk, acc, dq);
      else trial_loop<true, 1>(n, zq, tq, Qq, ps, blk, nblk, acc, dq);
    } else {
      if (vec) trial_loop<false, 4>(n, zq, tq, Qq, ps, blk, nblk, acc, dq);
      else trial_loop<false, 1>(n, zq, tq, Qq, ps, blk, nblk, acc, dq);
    }
    trial_block_store(acc, part + (int64_t)(ps - (TAIL ? 1 : pass)) * 4 * kSlots * nblk, q, blk, nblk);
    __syncthreads();
  }
}

// Fast trial pass (D <= kFastD, H % 4 == 0): rows x float4 columns.  Side 0 forms the trial
// direction on the fly, q = x_row . G_x[:, j] (no Q buffer); side 1 applies the x-side
// update to the cached pre-activations on the fly, z = zc + x_row . dWx[:, j].

// W <- (0.5 rho T theta* W - G) / (beta + 0.5 rho theta* T), theta* = 2^k / 2 (admm.py:338-343):
// one definition for k_select and the speculative x-stage z update (SpecX), which must
// reproduce its dWx bit for bit.
struct WUpd {
  float c1, den;
  __device__ static WUpd make(float rho, float beta, int T, int pick) {
    const float theta = ldexpf(1.f, pick - 1);
    WUpd u;
    u.c1 = ((0.5f * rho) * (float)T) * theta;
    u.den = beta + ((0.5f * rho) * theta) * (float)T;
    return u;
  }
  __device__ float apply(float w0, float G) const { return fmaf(c1, w0, -G) / den; }
};

struct RowCols {  // thread -> (row offset, float4 column) of a rows x (H/4) grid
  int tpr, rpb, rr, c4;
  __device__ RowCols(int H) {
    const int cols4 = H / 4;
    tpr = cols4 < kThreads ? cols4 : kThreads;
    rpb = kThreads / tpr;
    rr = threadIdx.x / tpr;
    c4 = threadIdx.x - rr * tpr;
  }
};

// Fast-path input width: D is padded to DP in {4, 8, 12, 16} (the LDS weight rows d >= D
// are zero, so the per-row x . W loops have compile-time trip counts).  XV: D == DP, the
// x row is read with float4 loads; otherwise element loads masked by d < D.
template <int DP, bool XV>
__device__ __forceinline__ void load_xrow(const float* __restrict__ x, int64_t row, int D, float (&xr)[DP]) {
  if (XV) {
    const float4* p = reinterpret_cast<const float4*>(x + row * DP);
#pragma unroll
    for (int d4 = 0; d4 < DP / 4; ++d4) {
      const float4 v = p[d4];
      xr[4 * d4] = v.x; xr[4 * d4 + 1] = v.y; xr[4 * d4 + 2] = v.z; xr[4 * d4 + 3] = v.w;
    }
  } else {
    const float* p = x + row * D;
#pragma unroll
    for (int d = 0; d < DP; ++d) xr[d] = d < D ? p[d] : 0.f;
  }
}

// [DP][H] weight block of gate q into LDS, rows d >= D zeroed
template <int DP>
__device__ __forceinline__ void stage_wlds(const Geom& g, const float* __restrict__ src, float* wl) {
  const int nW = g.D * g.H;
  for (int i = threadIdx.x; i < DP * g.H; i += kThreads) wl[i] = i < nW ? src[i] : 0.f;
  __syncthreads();
}

// dz = x_row . W[:, j..j+3] with W in LDS as [DP][H/4] float4
template <int DP>
__device__ __forceinline__ float4 xw_row(const float (&xr)[DP], const float4* __restrict__ wl4, int H4, int c4) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int d = 0; d < DP; ++d) {   // explicit fmas: the speculative update (SpecX) uses the same order
    const float4 wv = wl4[d * H4 + c4];
    acc.x = fmaf(xr[d], wv.x, acc.x); acc.y = fmaf(xr[d], wv.y, acc.y);
    acc.z = fmaf(xr[d], wv.z, acc.z); acc.w = fmaf(xr[d], wv.w, acc.w);
  }
  return acc;
}

// Trial pass of the fast path over rows x float4 columns, two rows per thread per
// iteration (all loads issued before any use; restrict pointers so they are not serialised
// behind stores).  Side 0 forms the trial direction q = x_row . G_x[:, j] on the fly
// (Wlds = G_x of this gate in LDS); side 1 reads Q.
constexpr int kRPI = 2;

template <bool TANH, int SIDE, int DP, bool XV, bool UR>
__device__ __forceinline__ void trial_fast_body(const Geom& g, int q, int pass, const float* __restrict__ zc,
                                                const float* __restrict__ tgt, const float* __restrict__ Q,
                                                const float* __restrict__ x, const float* Wlds, int blk, int nblk,
                                                float (&acc)[kSlots], DirectQ& dq) {
  const int64_t BT = g.BT(), n = BT * g.H;
  const float* __restrict__ zq = zc + (int64_t)q * n;
  const float* __restrict__ tq = tgt + (int64_t)q * n;
  const float* __restrict__ Qq = Q ? Q + (int64_t)q * n : nullptr;
  const float4* __restrict__ wl4 = reinterpret_cast<const float4*>(Wlds);
  RowCols rc(g.H);
  const bool lane_ok = rc.rr < rc.rpb;     // idle lanes stay in the (wave-uniform) loop
  const int j = 4 * rc.c4, H4 = g.H / 4;   // fast path: H/4 <= 256, one float4 column per thread
  const int64_t stride = (int64_t)nblk * rc.rpb;
  // one row per thread per iteration, the next row's operands loaded while this one is
  // evaluated (branch-free: rows past the end are loaded clamped and masked by ok)
  struct In { float4 z, t, q; float xr[DP]; };
  auto load = [&](int64_t row, In& v) {
    const int64_t rr = row < BT ? row : BT - 1;
    v.z = ld_nt(zq + rr * g.H + j);
    v.t = ld_nt(tq + rr * g.H + j);
    // UR: one row per wave (H/4 a multiple of 64), so the x row is wave-uniform: scalar loads
    // into SGPRs instead of 16 VGPRs per row in flight
    if (SIDE == 0) load_xrow<DP, XV>(x, UR ? (int64_t)__builtin_amdgcn_readfirstlane((int)rr) : rr, g.D, v.xr);
    else v.q = ld_nt(Qq + rr * g.H + j);
  };
#ifndef TF_ABL
#define TF_ABL 0   // trial ablations for tools/kbench (bitmask, 0 = full kernel)
#endif
  int64_t base = (int64_t)blk * rc.rpb;
  f32x2 acc2[kPair];
#pragma unroll
  for (int k = 0; k < kPair; ++k) acc2[k] = f32x2{0.f, 0.f};
  In cur, nxt;
  load(base + rc.rr, cur);
  for (; base < BT; base += stride) {
    const bool ok = lane_ok && base + rc.rr < BT;
    load(base + stride + rc.rr, nxt);
    float4 q4 = cur.q;
    if (SIDE == 0) {
      q4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!(TF_ABL & 1)) {   // q = x_row . G_x; G_x reads in groups of 4 issued back to back
        const float4* wrow = wl4 + rc.c4;
#pragma unroll
        for (int d0 = 0; d0 < DP; d0 += 4) {
          float4 wv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) wv[i] = wrow[(d0 + i) * H4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float xv = cur.xr[d0 + i];
            q4.x = fmaf(xv, wv[i].x, q4.x); q4.y = fmaf(xv, wv[i].y, q4.y);
            q4.z = fmaf(xv, wv[i].z, q4.z); q4.w = fmaf(xv, wv[i].w, q4.w);
          }
        }
      }
    }
    if (TF_ABL & 2) {
      acc[0] += cur.z.x * cur.t.x + q4.x + cur.z.y * cur.t.y + q4.y;
      acc[1] += cur.z.z * cur.t.z + q4.z + cur.z.w * cur.t.w + q4.w;
    } else {
      trial_pair<TANH>(ok, f32x2{cur.z.x, cur.z.y}, f32x2{cur.t.x, cur.t.y}, f32x2{q4.x, q4.y}, pass, acc, acc2, dq);
      if (!(TF_ABL & 4)) dq_run<TANH>(dq, acc, false);
      trial_pair<TANH>(ok, f32x2{cur.z.z, cur.z.w}, f32x2{cur.t.z, cur.t.w}, f32x2{q4.z, q4.w}, pass, acc, acc2, dq);
      if (!(TF_ABL & 4)) dq_run<TANH>(dq, acc, false);
    }
    cur = nxt;
  }
  trial_pair_fold(acc, acc2);
  dq_run<TANH>(dq, acc, true);
}

// Wsrc: side 0 -> G_x [4][D][H]; side 1 -> unused (Q holds the h-side direction)
#ifndef TF_MINB
#define TF_MINB 1   // workgroups per CU the register allocation must allow (occupancy for the streams)
#endif
template <int SIDE, int DP, bool XV, bool UR, bool TAIL = false>
__global__ __launch_bounds__(kThreads, TF_MINB) void k_trial_fast(Geom g, int pass, const float* zc, const float* tgt,
                                                           const float* Q, const float* x, const float* Wsrc,
                                                           const int* found, double* part, int nblk) {
  extern __shared__ float wlds[];  // [DP][H] (side 0 only)
  const int q = blockIdx.y, blk = blockIdx.x;  // gate-major: one code path per CU at a time (I-cache)
  if (found[q]) return;
  if (SIDE == 0) stage_wlds<DP>(g, Wsrc + (int64_t)q * g.D * g.H, wlds);
  __shared__ float dqbuf[kThreads / 64][kDQLds];
  auto one = [&](int ps, double* pp) {
    float acc[kSlots];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) acc[k] = 0.f;
    DirectQ dq{dqbuf[threadIdx.x >> 6], 0, 0};
    dq_hint(dq, ps, found, q);
    if (q == 2) trial_fast_body<true, SIDE, DP, XV, UR>(g, q, ps, zc, tgt, Q, x, wlds, blk, nblk, acc, dq);
    else trial_fast_body<false, SIDE, DP, XV, UR>(g, q, ps, zc, tgt, Q, x, wlds, blk, nblk, acc, dq);
    trial_block_store(acc, pp, q, blk, nblk);
  };
  if constexpr (TAIL) {
    for (int ps = 1; ps < kMaxPasses; ++ps) {
      one(ps, part + (int64_t)(ps - 1) * 4 * kSlots * nblk);
      __syncthreads();
    }
  } else {
    one(pass, part);
  }
}

// Trial pass for H % 256 == 0 (the C3/C4/C5 shapes): a workgroup owns 256 columns j, one per
// thread, and walks row pairs.  The row pair is the same for the whole workgroup, so the x rows
// are wave-uniform (scalar loads, SGPR operands) and the thread's column of G_x stays in 16
// VGPRs for the whole pass: q = x_row . G_x costs 16 FMAs and no LDS.  The two rows are the two
// halves of trial_pair's packed arithmetic; the next pair's operands are loaded while this one
// is evaluated.  Side 1 reads q from Q instead and walks row quads (QP: Q in k_qgemm3's
// row-quad layout [row / 4][j][row % 4], one float4 per quad).
template <bool TANH, int SIDE, int DP, bool XV, bool SPEC, int QP = 0>
__device__ __forceinline__ void trial_rows_body(const Geom& g, int q, int pass, const float* __restrict__ zc,
                                                const float* __restrict__ tgt, const float* __restrict__ Q,
                                                const float* __restrict__ x, const float* __restrict__ Gx, int blk,
                                                int nblk, float (&acc)[kSlots], DirectQ& dq, const SpecX& sp,
                                                float4* dwl) {
  const int64_t BT = g.BT(), n = BT * g.H;
  const int j = blockIdx.z * 256 + threadIdx.x;
  const float* __restrict__ zq = zc + (int64_t)q * n + j;
  const float* __restrict__ tq = tgt + (int64_t)q * n + j;
  const float* __restrict__ Qq = Q ? Q + (int64_t)q * n + (QP ? 4 * j : j) : nullptr;
  float gw[DP];
#pragma unroll
  for (int d = 0; d < DP; ++d) gw[d] = (SIDE == 0 && d < g.D) ? Gx[((int64_t)q * g.D + d) * g.H + j] : 0.f;
  // SPEC: this column of dWx for the predicted exponent, as k_select will form it, parked in
  // LDS as [DP/4][256] float4 (each thread reads back only its own column: no barrier) so the
  // kernel keeps its 4 waves per SIMD
  float* __restrict__ zxq = SPEC ? sp.zx + (int64_t)q * n + j : nullptr;
  if constexpr (SPEC) {
    const WUpd u = WUpd::make(sp.hp.rho[q], sp.hp.beta_x[q], g.T, sp.kpred[q]);
#pragma unroll
    for (int d4 = 0; d4 < DP / 4; ++d4) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int d = 4 * d4 + e;
        const float w0 = d < g.D ? sp.W[q][(int64_t)d * g.H + j] : 0.f;
        v[e] = d < g.D ? u.apply(w0, gw[d]) - w0 : 0.f;
      }
      dwl[d4 * 256 + threadIdx.x] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  f32x2 acc2[kPair];
#pragma unroll
  for (int k = 0; k < kPair; ++k) acc2[k] = f32x2{0.f, 0.f};
  if constexpr (SIDE == 1) {
    // h side: row quads (two row pairs per iteration), so that one Q load in the row-quad
    // layout (QP) covers the iteration; the row-major path walks the same quads (same sums)
    struct In4 { f32x2 z[2], t[2], q[2]; };
    auto load4 = [&](int64_t ra, In4& v) {   // rows ra .. ra + 3 (clamped); ra % 4 == 0
      int64_t r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = __builtin_amdgcn_readfirstlane((int)(ra + i < BT ? ra + i : BT - 1));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        v.z[h] = f32x2{__builtin_nontemporal_load(zq + r[2 * h] * g.H), __builtin_nontemporal_load(zq + r[2 * h + 1] * g.H)};
        v.t[h] = f32x2{__builtin_nontemporal_load(tq + r[2 * h] * g.H), __builtin_nontemporal_load(tq + r[2 * h + 1] * g.H)};
      }
      if constexpr (QP == 2) {   // bf16 quads: 8 B per row quad and column
        const int64_t pr = __builtin_amdgcn_readfirstlane((int)((ra < BT ? ra : BT - 4) >> 2));
        const __bf16* Qb = reinterpret_cast<const __bf16*>(Q) + (int64_t)q * n + 4 * j;
        const f32x4 qq = __builtin_convertvector(
            __builtin_nontemporal_load(reinterpret_cast<const bf16x4*>(Qb + pr * 4 * g.H)), f32x4);
        v.q[0] = f32x2{qq[0], qq[1]};
        v.q[1] = f32x2{qq[2], qq[3]};
      } else {   // row-major f32 (BT % 4 != 0)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          v.q[h] = f32x2{__builtin_nontemporal_load(Qq + r[2 * h] * g.H), __builtin_nontemporal_load(Qq + r[2 * h + 1] * g.H)};
      }
    };
    const int64_t stride = 4 * (int64_t)nblk;
    int64_t base = 4 * (int64_t)blk;
    In4 cur, nxt;
    load4(base, cur);
    for (; base < BT; base += stride) {
      load4(base + stride, nxt);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // rows past the end (BT % 4 != 0): a pair entirely past it is skipped (uniform), the
        // second row of a pair is masked through its q and d0 (ok covers the pair)
        if (h == 1 && base + 2 >= BT) break;
        const bool ok1 = base + 2 * h + 1 < BT;
        trial_pair<TANH>(true, cur.z[h], ok1 ? cur.t[h] : f32x2{cur.t[h].x, 0.f},
                         ok1 ? cur.q[h] : f32x2{cur.q[h].x, 0.f}, pass, acc, acc2, dq, ok1);
        dq_run<TANH>(dq, acc, false);
      }
      cur = nxt;
    }
    trial_pair_fold(acc, acc2);
    dq_run<TANH>(dq, acc, true);
    return;
  }
  struct In { f32x2 z, t, q; float xa[DP], xb[DP]; };
  auto load = [&](int64_t ra, In& v) {   // rows ra, ra + 1 (clamped)
    const int64_t r0 = __builtin_amdgcn_readfirstlane((int)(ra < BT ? ra : BT - 1));
    const int64_t r1 = __builtin_amdgcn_readfirstlane((int)(ra + 1 < BT ? ra + 1 : BT - 1));
    v.z = f32x2{__builtin_nontemporal_load(zq + r0 * g.H), __builtin_nontemporal_load(zq + r1 * g.H)};
    v.t = f32x2{__builtin_nontemporal_load(tq + r0 * g.H), __builtin_nontemporal_load(tq + r1 * g.H)};
    if (SIDE == 0) {
      load_xrow<DP, XV>(x, r0, g.D, v.xa);
      load_xrow<DP, XV>(x, r1, g.D, v.xb);
    } else {
      v.q = f32x2{__builtin_nontemporal_load(Qq + r0 * g.H), __builtin_nontemporal_load(Qq + r1 * g.H)};
    }
  };
  const int64_t stride = 2 * (int64_t)nblk;
  int64_t base = 2 * (int64_t)blk;
  In cur, nxt;
  load(base, cur);
  for (; base < BT; base += stride) {
    load(base + stride, nxt);
    f32x2 qv = cur.q;
    if (SIDE == 0) {
      float qa = 0.f, qb = 0.f;   // scalar FMAs with the (uniform, SGPR) x values as operands
#pragma unroll
      for (int d = 0; d < DP; ++d) {
        qa = fmaf(cur.xa[d], gw[d], qa);
        qb = fmaf(cur.xb[d], gw[d], qb);
      }
      qv = f32x2{qa, qb};
      if constexpr (SPEC) {   // z + x dWx in k_apply_dwx's order (xw_row)
        // an opaque zero offset keeps the LDS reads inside the loop (hoisted, they would take
        // 16 VGPRs for the whole pass)
        int zo;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zo));
        const float4* dl = dwl + zo + threadIdx.x;
        float da = 0.f, db = 0.f;
#pragma unroll
        for (int d4 = 0; d4 < DP / 4; ++d4) {
          const float4 w = dl[d4 * 256];
          const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            da = fmaf(cur.xa[4 * d4 + e], wv[e], da);
            db = fmaf(cur.xb[4 * d4 + e], wv[e], db);
          }
        }
        const int64_t r0 = __builtin_amdgcn_readfirstlane((int)base);
        __builtin_nontemporal_store(cur.z.x + da, zxq + r0 * g.H);
        if (base + 1 < BT) __builtin_nontemporal_store(cur.z.y + db, zxq + (r0 + 1) * g.H);
      }
    }
    // row base + 1 may be past the end (odd BT): masked through its q and d0 (ok covers the pair)
    const bool ok1 = base + 1 < BT;
    trial_pair<TANH>(true, cur.z, ok1 ? cur.t : f32x2{cur.t.x, 0.f},
                     ok1 ? qv : f32x2{qv.x, 0.f}, pass, acc, acc2, dq, ok1);
    dq_run<TANH>(dq, acc, false);
    cur = nxt;
  }
  trial_pair_fold(acc, acc2);
  dq_run<TANH>(dq, acc, true);
}

#ifndef TR_MINB
#define TR_MINB 1   // workgroups per CU the register allocation must allow
#endif
// The three split pieces of updated weight elements k0 .. k0 + 7 (rows of x2q or h2q, k0 % 8 == 0) of
// column jj, as the three bf16x8 the sweep image holds them in (one 16-byte store per piece; rows past
// Kd are the image's zero padding and are given zeros)
__device__ __forceinline__ void sweep_wt_put8(const SelectArgs& a, const Geom& g, int q, int k0, int jj,
                                              const float (&w)[8]) {
  const int H = g.H;
  int64_t base;
  if (a.wt_rows16) {   // k_sweep_wt16: chunk 32 deep, 64-column tiles of 4 column blocks
    const int kk = (a.side == 0 ? 0 : 32 * a.wt_xc) + k0;
    const int NT = H / 64, KC2 = a.wt_xc + H / 32;
    const int c = kk >> 5, kq = (kk & 31) >> 3, n = jj >> 6, jq = (jj & 63) >> 4;
    const int lane = (jj & 15) + 16 * kq;
    base = ((((int64_t)(q * NT + n) * KC2 + c) * 4 + jq) * 3) * 64 + lane;
  } else {             // k_sweep_wt: chunk 16 deep, 32-column tiles
    const int kk = (a.side == 0 ? 0 : 16 * a.wt_xc) + k0;
    const int NT = H / 32, KC2 = a.wt_xc + 2 * NT;
    const int c = kk >> 4, h = (kk & 15) >> 3, n = jj >> 5;
    const int lane = (jj & 31) + 32 * h;
    base = (((int64_t)(q * NT + n) * KC2 + c) * 3) * 64 + lane;
  }
  bf16x8 p0, p1, p2;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    __bf16 b0, b1, b2;
    split3(w[e], b0, b1, b2);
    p0[e] = b0; p1[e] = b1; p2[e] = b2;
  }
  bf16x8* wt = static_cast<bf16x8*>(a.wt);
  wt[base] = p0;
  wt[base + 64] = p1;
  wt[base + 128] = p2;
}

// k_select's work for gate q by block mb of nmb (the weight update is split over the nmb blocks).
// LIGHT (one block of a fused tail trial launch, whose partials were handed off write-through): the
// partials are read with sc1 loads, a few slots at a time, and ||G||^2 with fewer loads in flight --
// the same sums in the same order, in a register budget the trial kernel can spare.
template <bool LIGHT>
__device__ __forceinline__ void select_gate(const Geom& g, const Hyper& hp, const SelectArgs& a, int q, int mb, int nmb) {
  __shared__ double red[4][kSlots];
  __shared__ double sums[kSlots];
  __shared__ double gred[4];
  __shared__ int pick_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (a.found_in[q]) {   // decided in an earlier pass
    if (mb == 0 && tid == 0) {
      a.found_out[q] = 1;
      a.pick[q] = -1;
    }
    return;
  }
  // 2. ||G||^2 (k_decide's order: float4 loads 8 at a time)
  const int Kd = a.side == 0 ? g.D : g.H;
  const int64_t nW = (int64_t)Kd * g.H;
  const float* Gq = a.G + (int64_t)q * nW;
  double gs = 0.0;
  if ((nW & 3) == 0) {
    const float4* G4 = reinterpret_cast<const float4*>(Gq);
    const int64_t n4 = nW / 4;
    int64_t i = tid;
    // two groups of 8 loads in flight; the sum order is the 8-at-a-time loop's
    for (; !LIGHT && i + 15 * kThreads < n4; i += 16 * kThreads) {
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = G4[i + u * kThreads];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        gs += ((double)v[u].x * v[u].x + (double)v[u].y * v[u].y) + ((double)v[u].z * v[u].z + (double)v[u].w * v[u].w);
    }
    for (; i + 7 * kThreads < n4; i += 8 * kThreads) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = G4[i + u * kThreads];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        gs += ((double)v[u].x * v[u].x + (double)v[u].y * v[u].y) + ((double)v[u].z * v[u].z + (double)v[u].w * v[u].w);
    }
    for (; i < n4; i += kThreads) {
      const float4 v = G4[i];
      gs += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
    }
  } else {
    for (int64_t i = tid; i < nW; i += kThreads) gs += (double)Gq[i] * (double)Gq[i];
  }
  const double gsq = block_sum(gs, gred);
  const float rho = hp.rho[q];
  // per window (one, or the tail's windows 1 .. kMaxPasses - 1 in order until one decides)
  for (int ps = pass_lo(a.pass); ps < pass_hi(a.pass); ++ps) {
  const int64_t wofs = (int64_t)(ps - pass_lo(a.pass)) * 4 * kSlots;
  // 1. the window's sums of this gate
  if (a.part && LIGHT) {
    // per slot: thread t adds partials t, t + 256, ... (k_select's order), then wave_sum (the bits of
    // wave_sum_slots) and the same cross-wave tree
    const double* p = a.part + wofs * a.nred + (int64_t)q * kSlots * a.nred;
    for (int k0 = 0; k0 < kSlots; k0 += 8) {
      double acc8[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc8[k] = 0.0;
      for (int i = tid; i < a.nred; i += kThreads) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          v[k] = k0 + k < kSlots ? __hip_atomic_load(&p[(int64_t)(k0 + k) * a.nred + i], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) : 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc8[k] += v[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double vv = wave_sum(acc8[k]);
        if (lane == 0 && k0 + k < kSlots) red[w][k0 + k] = vv;
      }
    }
    __syncthreads();
    if (tid < kSlots) sums[tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
  } else if (a.part) {
    double acc[kSlots];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) acc[k] = 0.0;
    const double* p = a.part + wofs * a.nred + (int64_t)q * kSlots * a.nred;
    int i = tid;
    for (; i + kThreads < a.nred; i += 2 * kThreads) {   // two partials' loads in flight, same sum order
      double v0[kSlots], v1[kSlots];
#pragma unroll
      for (int k = 0; k < kSlots; ++k) {
        v0[k] = p[(int64_t)k * a.nred + i];
        v1[k] = p[(int64_t)k * a.nred + i + kThreads];
      }
#pragma unroll
      for (int k = 0; k < kSlots; ++k) acc[k] = (acc[k] + v0[k]) + v1[k];
    }
    if (i < a.nred) {
#pragma unroll
      for (int k = 0; k < kSlots; ++k) acc[k] += p[(int64_t)k * a.nred + i];
    }
    const double v = wave_sum_slots(acc);
    if (lane < kSlots) red[w][lane] = v;
    __syncthreads();
    if (tid < kSlots) sums[tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
  } else if (tid < kSlots) {
    sums[tid] = a.sums[wofs + q * kSlots + tid];
  }
  __syncthreads();
  // 3. the decision
  if (tid == 0) {
    const double* sm = sums;
    double* pq = a.poly + q * kPolyN;
    double pl[kPolyN];
    for (int n = 0; n < kPolyN; ++n) pl[n] = ps == 0 ? sm[kSlotPoly + n] : pq[n];
    if (ps == 0 && mb == 0)
      for (int n = 0; n < kPolyN; ++n) pq[n] = pl[n];
    const bool poly_only = sm[kSlotNne] == 0.0;
    const int k_lo = poly_only ? 0 : ps * kTrialJ;
    const int k_hi = poly_only ? kMaxK : k_lo + kTrialJ;
    int pick = -1;
    for (int kk = k_lo; kk < k_hi; ++kk) {
      const double sk = ldexp(1.0, -kk);
      double poly = 0.0;
      for (int n = kPolyN - 1; n >= 0; --n) poly = (poly + pl[n]) * sk;
      const double cand = poly_only ? 0.0 : sm[kk - k_lo];
      const double lhs = 0.5 * (double)rho * (cand + poly);
      const double rhs = 0.5 * g.T * gsq * sk;
      if (!isfinite(lhs) && mb == 0) atomicAdd(&a.stats->nonfinite, 1);
      if (lhs > rhs) continue;
      pick = kk;
      break;
    }
    // pass 0, no exponent in the window, hint set and every per-candidate element covered by its
    // polynomial past the window (dq_hint): decide k in [kTrialJ, kMaxK) from both polynomials
    // (the s^1 slot only holds the per-candidate elements' linearisation, which the candidate sums
    // needed: left out here, as the remainder has no s^1 term)
    if (pick < 0 && ps == 0 && !poly_only && a.found_in[8 + q] && sm[kSlotN16] == 0.0) {
      for (int kk = kTrialJ; kk < kMaxK; ++kk) {
        const double sk = ldexp(1.0, -kk);
        double poly = 0.0;
        for (int n = kPolyN - 1; n >= 1; --n) poly = (poly + pl[n] + sm[kSlotP16 + n - 1]) * sk;
        poly *= sk;
        const double lhs = 0.5 * (double)rho * poly;
        const double rhs = 0.5 * g.T * gsq * sk;
        if (!isfinite(lhs) && mb == 0) atomicAdd(&a.stats->nonfinite, 1);
        if (lhs > rhs) continue;
        pick = kk;
        break;
      }
    }
    const int own = pick;   // -1: not decided within this pass's window
    if (a.force) {          // test hook: take the given exponent (the search above still ran)
      pick = a.force[2 * q + a.side];
    } else if (pick < 0 && (poly_only || ps == kMaxPasses - 1)) {
      pick = k_hi;
      if (mb == 0) atomicAdd(&a.stats->unresolved, 1);
    }
    if (mb == 0) {
      if (pick >= 0) {
        const int slot = 2 * q + a.side;
        a.stats->k[slot] = pick;
        if (a.force) a.stats->k_own[slot] = own;
        a.stats->f_w[slot] = 0.5 * (double)rho * sm[kSlotFw];
        a.stats->grad_sq[slot] = gsq;
        a.stats->direct_frac[slot] = sm[kSlotNne] / ((double)g.Bg * g.T * g.H);
        a.stats->passes[a.side] = ps + 1;
      }
      a.found_out[q] = pick >= 0 ? 1 : 0;
      a.pick[q] = pick;
    }
    pick_s = pick;
  }
  __syncthreads();
  if (pick_s >= 0) break;
  }
  __syncthreads();
  const int pick = pick_s;
  if (pick < 0) return;
  // 4. this block's slice of the weight update
  const float beta = a.side == 0 ? hp.beta_x[q] : hp.beta_h[q];
  const WUpd u = WUpd::make(rho, beta, g.T, pick);
  float* W = a.W[q];
  const int64_t gstride = (int64_t)nmb * kThreads;
  if (a.wt) {
    // with the sweep image: 8-row groups of one column per thread (the W / G loads of a row stay
    // coalesced across the block's threads; the image takes three 16-byte stores per group)
    const int64_t ng = (int64_t)((Kd + 7) / 8) * g.H;
    for (int64_t gi = (int64_t)mb * kThreads + tid; gi < ng; gi += gstride) {
      const int kg = (int)(gi / g.H), jj = (int)(gi - (int64_t)kg * g.H);
      float w0[8], gv[8], w1[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int64_t i = (int64_t)(8 * kg + r) * g.H + jj;
        const bool in = 8 * kg + r < Kd;
        w0[r] = in ? W[i] : 0.f;
        gv[r] = in ? Gq[i] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int64_t i = (int64_t)(8 * kg + r) * g.H + jj;
        if (8 * kg + r < Kd) {
          w1[r] = u.apply(w0[r], gv[r]);
          W[i] = w1[r];
          if (a.dW) a.dW[(int64_t)q * nW + i] = w1[r] - w0[r];
        } else {
          w1[r] = 0.f;
        }
      }
      sweep_wt_put8(a, g, q, 8 * kg, jj, w1);
    }
    return;
  }
  int64_t i = (int64_t)mb * kThreads + tid;
  for (; !LIGHT && i + 3 * gstride < nW; i += 4 * gstride) {   // four elements' loads in flight
    float w0[4], gv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) { w0[e] = W[i + e * gstride]; gv[e] = Gq[i + e * gstride]; }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float w1 = u.apply(w0[e], gv[e]);
      W[i + e * gstride] = w1;
      if (a.dW) a.dW[(int64_t)q * nW + i + e * gstride] = w1 - w0[e];
    }
  }
  for (; i < nW; i += gstride) {
    const float w0 = W[i];
    const float w1 = u.apply(w0, Gq[i]);
    W[i] = w1;
    if (a.dW) a.dW[(int64_t)q * nW + i] = w1 - w0;
  }
}

// The tail pass's selection inside its trial launch (one process): the workgroup of gate q that
// stores its partials last (an agent-scope count per gate; the partials went write-through, row 1
// of MI355X_MICROARCH.md's hand-off table) runs k_select's work for q alone and re-arms the count.
// Gates pass 0 decided: one workgroup sets their flags as k_select would (found_out 1, pick -1).
struct TailSel {
  SelectArgs a;
  Hyper hp;
  unsigned* count;   // [4], zero between launches; nullptr: not fused (a separate k_select follows)
};
__device__ __forceinline__ void tail_select_done(const TailSel& ts, int q) {
  if (ts.count && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) {
    ts.a.found_out[q] = 1;
    ts.a.pick[q] = -1;
  }
}
__device__ __forceinline__ void tail_select_last(const Geom& g, const TailSel& ts, int q, unsigned nblocks) {
  __shared__ int last_s;
  __syncthreads();
  if (threadIdx.x == 0) {
    // release: this workgroup's partials (stored by this wave, trial_block_store<true>) are visible at
    // agent scope before its arrival counts; the last arriver acquires everyone's before reading them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last_s = __hip_atomic_fetch_add(&ts.count[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1;
  }
  __syncthreads();
  if (!last_s) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  select_gate<true>(g, ts.hp, ts.a, q, 0, 1);
  if (threadIdx.x == 0) __hip_atomic_store(&ts.count[q], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int SIDE, int DP, bool XV, bool SPEC, int QP = 0, bool TAIL = false>
__global__ __launch_bounds__(kThreads, TR_MINB) void k_trial_rows(Geom g, int pass, const float* __restrict__ zc,
                                                         const float* __restrict__ tgt, const float* __restrict__ Q,
                                                         const float* __restrict__ x, const float* __restrict__ Gx,
                                                         const int* __restrict__ found, double* __restrict__ part,
                                                         int nblk, SpecX sp, TailSel ts) {
  const int q = blockIdx.y, blk = blockIdx.x;
  if (found[q]) {
    if constexpr (TAIL) tail_select_done(ts, q);
    return;
  }
  __shared__ float dqbuf[kThreads / 64][kDQLds];
  __shared__ float4 dwl[SPEC ? DP / 4 * 256 : 1];
  // the column blocks of one (blk, q) add into the same part slot row: blk index widened by z
  const int nred = nblk * gridDim.z;
  auto one = [&](int ps, double* pp) {
    float acc[kSlots];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) acc[k] = 0.f;
    DirectQ dq{dqbuf[threadIdx.x >> 6], 0, 0};
    dq_hint(dq, ps, found, q);
    if (q == 2) trial_rows_body<true, SIDE, DP, XV, SPEC, QP>(g, q, ps, zc, tgt, Q, x, Gx, blk, nblk, acc, dq, sp, dwl);
    else trial_rows_body<false, SIDE, DP, XV, SPEC, QP>(g, q, ps, zc, tgt, Q, x, Gx, blk, nblk, acc, dq, sp, dwl);
    if (TAIL && ts.count) trial_block_store<true>(acc, pp, q, blockIdx.z * nblk + blk, nred);
    else trial_block_store(acc, pp, q, blockIdx.z * nblk + blk, nred);
  };
  if constexpr (TAIL) {
    for (int ps = 1; ps < kMaxPasses; ++ps) {
      one(ps, part + (int64_t)(ps - 1) * 4 * kSlots * nred);
      __syncthreads();
    }
    if (ts.count) tail_select_last(g, ts, q, (unsigned)nred);
  } else {
    one(pass, part);
  }
}

// x-side trial pass on the matrix cores (H % 128 == 0, D <= 16): each wave owns a 32-column
// block of one gate and walks 16-row tiles.  The trial direction q = X G_x (and with SPEC the
// z update X dWx(kpred)) of a tile comes from v_mfma_f32_16x16x4_f32 chains over K = 16 (x
// rows as the A operand, zero-padded past D; G_x / dWx columns as B, resident in VGPRs), and
// the trial arithmetic (trial_pair) runs on the accumulator layout.  The wave's two 16x16
// products take the even and the odd columns, so lane l holds columns 2 (l % 16) + {0, 1} of
// rows 4 (l / 16) + v, v = 0..3: every z / tgt / zx access is a float2 per lane, 128 B per row,
// and the two columns are trial_pair's packed halves.  This frees the VALU of the 32 FMAs per
// element the row-pair kernel (k_trial_rows) spends on q and the z update.
template <bool TANH, bool SPEC>
__device__ __forceinline__ void trial_mx_body(const Geom& g, int q, int pass, const float* __restrict__ zc,
                                              const float* __restrict__ tgt, const float* __restrict__ x,
                                              const float* __restrict__ Gx, int blk, int nblk, float (&acc)[kSlots],
                                              DirectQ& dq, const SpecX& sp) {
  const int64_t BT = g.BT(), n = BT * g.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col0 = (blockIdx.z * 4 + wave) * 32 + 2 * (lane & 15);   // this lane's column pair
  // 32-bit buffer offsets into one gate plane (trial_mx_ok: a plane is < 2 GB); rows past BT
  // are past the descriptor's range, so they load 0 and their stores are dropped (and the
  // trial arithmetic masks them with ok below)
  const __amdgpu_buffer_rsrc_t rZ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(zc + (int64_t)q * n), 0, (int)(n * 4), kBufWord3);
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(tgt + (int64_t)q * n), 0, (int)(n * 4), kBufWord3);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, (int)(BT * g.D * 4), kBufWord3);
  const __amdgpu_buffer_rsrc_t rZX = SPEC ? __builtin_amdgcn_make_buffer_rsrc(sp.zx + (int64_t)q * n, 0, (int)(n * 4), kBufWord3)
                                          : rZ;
  const uint32_t rowb = (uint32_t)g.H * 4;   // bytes per row of a plane
  // this lane's byte offset within a tile: row 4 (lane / 16), columns col0, col0 + 1
  const uint32_t lofs = (uint32_t)(4 * (lane >> 4)) * rowb + (uint32_t)col0 * 4;
  // B operands: row 4 s + lane/16 of G_x (and dWx) at column col0 + h (product h)
  float gb[2][4], db[2][4];
  const WUpd u = SPEC ? WUpd::make(sp.hp.rho[q], sp.hp.beta_x[q], g.T, sp.kpred[q]) : WUpd{};
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    const int d = 4 * s4 + (lane >> 4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      gb[h][s4] = d < g.D ? Gx[((int64_t)q * g.D + d) * g.H + col0 + h] : 0.f;
      if constexpr (SPEC) {
        const float w0 = d < g.D ? sp.W[q][(int64_t)d * g.H + col0 + h] : 0.f;
        db[h][s4] = d < g.D ? u.apply(w0, gb[h][s4]) - w0 : 0.f;
      }
    }
  }
  f32x2 acc2[kPair];
#pragma unroll
  for (int k = 0; k < kPair; ++k) acc2[k] = f32x2{0.f, 0.f};
  const int64_t ntile = (BT + 15) / 16;
  // operands of one tile (rows past BT load 0 through the descriptor and are masked by ok below)
  struct In { float xa[4]; f32x2 zv[4], tv[4]; };
  auto load = [&](int64_t tile, In& v) {
    const uint32_t row0 = (uint32_t)tile * 16;
    // A operand: x[row0 + lane % 16][4 s + lane / 16]
    const uint32_t xo = ((row0 + (lane & 15)) * g.D + (lane >> 4)) * 4;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int d = 4 * s4 + (lane >> 4);
      v.xa[s4] = d < g.D ? buf_ld<0>(rX, xo + 16 * s4) : 0.f;
    }
    const uint32_t o = row0 * rowb + lofs;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v.zv[r] = buf_ld2(rZ, o + r * rowb);
      v.tv[r] = buf_ld2(rT, o + r * rowb);
    }
  };
#ifndef TMX_ROLL
#define TMX_ROLL 1
#endif
  // TMX_ROLL: a rolling prefetch in the registers of the tile being evaluated -- the next tile's
  // x operand is loaded once this tile's MFMAs have read theirs, and its row v once trial_pair
  // has consumed this tile's row v (a tile of latency cover for no extra registers)
  In cur;
  const auto load_x = [&](int64_t tile) {
    const uint32_t xo = (((uint32_t)tile * 16 + (lane & 15)) * g.D + (lane >> 4)) * 4;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int d = 4 * s4 + (lane >> 4);
      cur.xa[s4] = d < g.D ? buf_ld<0>(rX, xo + 16 * s4) : 0.f;
    }
  };
  if (TMX_ROLL) load(blk, cur);
  for (int64_t tile = blk; tile < ntile; tile += nblk) {
    const int64_t row0 = tile * 16;
    const int64_t tn = tile + nblk < ntile ? tile + nblk : tile;
    if (!TMX_ROLL) load(tile, cur);
    const float (&xa)[4] = cur.xa;
    f32x2 (&zv)[4] = cur.zv;
    f32x2 (&tv)[4] = cur.tv;
    f32x4 qa[2] = {}, da[2] = {};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int h = 0; h < 2; ++h) qa[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s4], gb[h][s4], qa[h], 0, 0, 0);
    if constexpr (SPEC) {
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int h = 0; h < 2; ++h) da[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s4], db[h][s4], da[h], 0, 0, 0);
      const uint32_t o = (uint32_t)row0 * rowb + lofs;
#pragma unroll
      for (int v = 0; v < 4; ++v) buf_st2(rZX, o + v * rowb, zv[v] + f32x2{da[0][v], da[1][v]});
    }
    if (TMX_ROLL) load_x(tn);
    const uint32_t on = (uint32_t)tn * 16 * rowb + lofs;
#pragma unroll
    for (int v = 0; v < 4; ++v) {   // the two columns of row 4 (lane / 16) + v
      const bool ok = (int)row0 + 4 * (lane >> 4) + v < (int)BT;   // 32-bit: trial_mx_ok bounds BT H
      trial_pair<TANH>(ok, zv[v], tv[v], f32x2{qa[0][v], qa[1][v]}, pass, acc, acc2, dq, ok);
      if (TMX_ROLL) {
        zv[v] = buf_ld2(rZ, on + v * rowb);
        tv[v] = buf_ld2(rT, on + v * rowb);
      }
      dq_run<TANH>(dq, acc, false);
    }
  }
  trial_pair_fold(acc, acc2);
  dq_run<TANH>(dq, acc, true);
}

#ifndef TMX_MINB
#define TMX_MINB 4   // 4 waves/SIMD (128 VGPRs), the next tile prefetched in place (TMX_ROLL)
#endif
template <bool SPEC, bool TAIL = false>
__global__ __launch_bounds__(kThreads, TMX_MINB) void k_trial_mx(Geom g, int pass, const float* __restrict__ zc,
                                                       const float* __restrict__ tgt, const float* __restrict__ x,
                                                       const float* __restrict__ Gx, const int* __restrict__ found,
                                                       double* __restrict__ part, int nblk, SpecX sp, TailSel ts) {
  const int q = blockIdx.y, blk = blockIdx.x;
  if (found[q]) {
    if constexpr (TAIL) tail_select_done(ts, q);
    return;
  }
  __shared__ float dqbuf[kThreads / 64][kDQLds];
  const int nred = nblk * gridDim.z;
  auto one = [&](int ps, double* pp) {
    float acc[kSlots];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) acc[k] = 0.f;
    DirectQ dq{dqbuf[threadIdx.x >> 6], 0, 0};
    dq_hint(dq, ps, found, q);
    if (q == 2) trial_mx_body<true, SPEC>(g, q, ps, zc, tgt, x, Gx, blk, nblk, acc, dq, sp);
    else trial_mx_body<false, SPEC>(g, q, ps, zc, tgt, x, Gx, blk, nblk, acc, dq, sp);
    if (TAIL && ts.count) trial_block_store<true>(acc, pp, q, blockIdx.z * nblk + blk, nred);
    else trial_block_store(acc, pp, q, blockIdx.z * nblk + blk, nred);
  };
  if constexpr (TAIL) {
    for (int ps = 1; ps < kMaxPasses; ++ps) {
      one(ps, part + (int64_t)(ps - 1) * 4 * kSlots * nred);
      __syncthreads();
    }
    if (ts.count) tail_select_last(g, ts, q, (unsigned)nred);
  } else {
    one(pass, part);
  }
}

// After the x stage: zc += X dWx, so the h stage sees z = X Wx_new + Hprev Wh
// (admm.py:298-300: the h-side search uses the already-updated x2q).
// k_apply_fix (kpred != nullptr): zx = zc + X dWx, only for the gates whose decided x-side
// exponent differs from the one pass 0 of the trials assumed (SpecX).
template <int DP, bool XV>
__global__ __launch_bounds__(kThreads) void k_apply_dwx(Geom g, const float* __restrict__ x,
                                                          const float* __restrict__ dW, const float* zsrc,
                                                          float* zdst, const int* __restrict__ kpred,
                                                          const DevStats* __restrict__ stats) {
  extern __shared__ float wl[];  // [DP][H] of gate q
  const int q = blockIdx.y;
  if (kpred && stats->k[2 * q] == kpred[q]) return;
  stage_wlds<DP>(g, dW + (int64_t)q * g.D * g.H, wl);
  const float4* __restrict__ wl4 = reinterpret_cast<const float4*>(wl);
  const int64_t BT = g.BT();
  const float* zq = zsrc + (int64_t)q * BT * g.H;
  float* zo = zdst + (int64_t)q * BT * g.H;
  RowCols rc(g.H);
  if (rc.rr >= rc.rpb) return;
  const int j = 4 * rc.c4, H4 = g.H / 4;
  const int64_t stride = (int64_t)gridDim.x * rc.rpb;
  for (int64_t row0 = (int64_t)blockIdx.x * rc.rpb + rc.rr; row0 < BT; row0 += kRPI * stride) {
    float4 z4[kRPI];
    float xr[kRPI][DP];
#pragma unroll
    for (int r = 0; r < kRPI; ++r) {
      const int64_t row = row0 + r * stride;
      if (row < BT) {
        z4[r] = ld_nt(zq + row * g.H + j);
        load_xrow<DP, XV>(x, row, g.D, xr[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < kRPI; ++r) {
      const int64_t row = row0 + r * stride;
      if (row >= BT) break;
      const float4 dz = xw_row<DP>(xr[r], wl4, H4, rc.c4);
      float4 zn;
      zn.x = z4[r].x + dz.x; zn.y = z4[r].y + dz.y; zn.z = z4[r].z + dz.z; zn.w = z4[r].w + dz.w;
      st_nt(zo + row * g.H + j, zn);
    }
  }
}

// x-stage residual fused with G_x = X^T R (admm.py:302-312, x side): per element
// tgt = lam/rho + S (stored for the trials and the h stage), R = (phi(z) - tgt) phi'(z),
// and per block the partial sums X^T R into a [D][H] slab (R never reaches HBM).
template <int DP, bool XV>
__global__ __launch_bounds__(kThreads) void k_resid_gx(Geom g, Hyper hp, const float* x, Planes6 S, Planes6 L,
                                                         const float* zc, float* tgt, float* slab, bool tgt_ready) {
  extern __shared__ float gl[];  // [D][H] block accumulator
  const int q = blockIdx.y;
  const bool th = (q == 2);
  const float rho = hp.rho[q];
  const int64_t BT = g.BT(), n = BT * g.H;
  const float* zq = zc + (int64_t)q * n;
  float* tq = tgt + (int64_t)q * n;
  const float* Sq = S.p[q];
  const float* Lq = L.p[q];
  RowCols rc(g.H);                 // fast path: H/4 <= 256, one float4 column per thread
  const int j = 4 * rc.c4;
  float acc[DP][4];
#pragma unroll
  for (int d = 0; d < DP; ++d) acc[d][0] = acc[d][1] = acc[d][2] = acc[d][3] = 0.f;
  const int64_t per_blk = (BT + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per_blk, r1 = r0 + per_blk < BT ? r0 + per_blk : BT;
  if (rc.rr < rc.rpb) {
    for (int64_t row = r0 + rc.rr; row < r1; row += rc.rpb) {
      const int64_t b = g.dT.div((uint32_t)row);
      const int64_t so = (row + b + 1) * g.H;  // (b*(T+1) + t) * H with t = row - b*T + 1
      float xr[DP];
      load_xrow<DP, XV>(x, row, g.D, xr);
      const float4 z4 = ld_nt(zq + row * g.H + j);
      float4 t4;
      if (tgt_ready) {
        t4 = ld_nt(tq + row * g.H + j);
      } else {
        const float4 l4 = ld_nt(Lq + so + j);
        const float4 s4 = ld_nt(Sq + so + j);
        const f32x4 tv = tgt_quot(f32x4{l4.x, l4.y, l4.z, l4.w}, rho, f32x4{s4.x, s4.y, s4.z, s4.w});
        t4 = make_float4(tv.x, tv.y, tv.z, tv.w);
        st_nt(tq + row * g.H + j, t4);
      }
      const float zz[4] = {z4.x, z4.y, z4.z, z4.w}, tt[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        // the activation of the stored gates (sig_pair / tanhf, as k_forward_t and k_resid): at
        // step 1 S = phi(z) bit for bit, so R and G_x are exactly zero as in the reference
        // (admm.py:302-312) and the x-side searches take k = 0, not a decision on rounding noise
        float phi, dphi;
        if (th) {
          phi = tanhf(zz[u]);
          dphi = 1.f - phi * phi;
        } else {
          const SigPair sp = sig_pair(zz[u]);
          phi = sp.s;
          dphi = sp.s * sp.sc;
        }
        const float R = (phi - tt[u]) * dphi;
#pragma unroll
        for (int d = 0; d < DP; ++d) acc[d][u] += xr[d] * R;
      }
    }
  }
  // deterministic in-block combine of the row groups, then one slab per block
  for (int i = threadIdx.x; i < g.D * g.H; i += kThreads) gl[i] = 0.f;
  __syncthreads();
  for (int grp = 0; grp < rc.rpb; ++grp) {
    if (rc.rr == grp) {
#pragma unroll
      for (int d = 0; d < DP; ++d) {
        if (d < g.D) {
          float* dst = gl + d * g.H + j;
          dst[0] += acc[d][0]; dst[1] += acc[d][1]; dst[2] += acc[d][2]; dst[3] += acc[d][3];
        }
      }
    }
    __syncthreads();
  }
  float* out = slab + ((int64_t)blockIdx.x * 4 + q) * g.D * g.H;
  for (int i = threadIdx.x; i < g.D * g.H; i += kThreads) out[i] = gl[i];
}

// the fast kernels' arithmetic (trial_pair: polynomial regime and per-candidate queue) over
// element pairs
template <bool TANH>
__device__ __forceinline__ void trial_pair_loop(int64_t n, const float* z, const float* tgt, const float* qv, int pass,
                                                int blk, int nblk, float (&acc)[kSlots], DirectQ& dq) {
  f32x2 acc2[kPair];
#pragma unroll
  for (int k = 0; k < kPair; ++k) acc2[k] = f32x2{0.f, 0.f};
  const int64_t np = (n + 1) / 2;
  for (int64_t base = (int64_t)blk * kThreads; base < np; base += (int64_t)nblk * kThreads) {   // wave-uniform
    const int64_t v = base + threadIdx.x;
    const bool ok = v < np, oky = 2 * v + 1 < n;
    const f32x2 zz = f32x2{ok ? z[2 * v] : 0.f, oky ? z[2 * v + 1] : 0.f};
    const f32x2 tt = f32x2{ok ? tgt[2 * v] : 0.f, oky ? tgt[2 * v + 1] : 0.f};
    const f32x2 qq = f32x2{ok ? qv[2 * v] : 0.f, oky ? qv[2 * v + 1] : 0.f};
    trial_pair<TANH>(ok, zz, tt, qq, pass, acc, acc2, dq, oky);
    dq_run<TANH>(dq, acc, false);
  }
  trial_pair_fold(acc, acc2);
  dq_run<TANH>(dq, acc, true);
}

// Test hook: the same per-element arithmetic on caller data (one gate), kbase = pass*J:
// per block the J candidate sums of that window, with the polynomial part already evaluated at
// s = 2^-(kbase+k), so part[blk][k] is the full increment sum.  mode bit 0: tanh gate; bit 1:
// the fast kernels' pair arithmetic (trial_pair) instead of the generic trial_point.
__global__ __launch_bounds__(kThreads) void k_trial_debug(int64_t n, int mode, int kbase, const float* z,
                                                            const float* tgt, const float* qv, double* part) {
  __shared__ double red[4][kSlots];
  float acc[kSlots];
#pragma unroll
  for (int k = 0; k < kSlots; ++k) acc[k] = 0.f;
  const int pass = kbase / kTrialJ;
  const bool tanh_gate = mode & 1, pair = mode & 2;
  // the polynomial slots are only filled on pass 0: run pass 0 for them, then this pass
  __shared__ float dqbuf[kThreads / 64][kDQLds];
  DirectQ dq{dqbuf[threadIdx.x >> 6], 0, 0};
  auto run = [&](int ps, float (&a)[kSlots]) {
    if (pair) {
      if (tanh_gate) trial_pair_loop<true>(n, z, tgt, qv, ps, blockIdx.x, gridDim.x, a, dq);
      else trial_pair_loop<false>(n, z, tgt, qv, ps, blockIdx.x, gridDim.x, a, dq);
    } else {
      if (tanh_gate) trial_loop<true, 1>(n, z, tgt, qv, ps, blockIdx.x, gridDim.x, a, dq);
      else trial_loop<false, 1>(n, z, tgt, qv, ps, blockIdx.x, gridDim.x, a, dq);
    }
  };
  run(0, acc);
  if (pass > 0) {
    float acc2[kSlots];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) acc2[k] = 0.f;
    run(pass, acc2);
#pragma unroll
    for (int k = 0; k < kTrialJ; ++k) acc[k] = acc2[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kSlots; ++k) {
    const float s = wave_sum(acc[k]);
    if (lane == 0) red[w][k] = (double)s;
  }
  __syncthreads();
  if (threadIdx.x < kTrialJ) {
    const int k = threadIdx.x;
    double tot[kSlots];
    for (int i = 0; i < kSlots; ++i) tot[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    const double sk = ldexp(1.0, -(kbase + k));
    double poly = 0.0;
    for (int n2 = kPolyN - 1; n2 >= 0; --n2) poly = (poly + tot[kSlotPoly + n2]) * sk;
    part[(int64_t)blockIdx.x * kTrialJ + k] = tot[k] + poly;
  }
}

__global__ __launch_bounds__(kThreads) void k_trial_reduce(int pass, const double* part, int nblk, const int* found,
                                                             double* sums) {
  __shared__ double red[4];
  const int k = blockIdx.x, q = blockIdx.y;      // one block per (slot, gate[, tail window z])
  if (found[q]) return;
  part += (int64_t)blockIdx.z * 4 * kSlots * nblk;
  sums += (int64_t)blockIdx.z * 4 * kSlots;
  double s = 0.0;
  const double* p = part + ((int64_t)q * kSlots + k) * nblk;
  for (int i = threadIdx.x; i < nblk; i += kThreads) s += p[i];
  const double tot = block_sum(s, red);
  if (threadIdx.x == 0) sums[q * kSlots + k] = tot;
}

// One trial pass's selection in one launch, grid (kSelBlocks, 4): every block of gate q
//  1. reduces the pass's per-block partials (a.part, a.nred per slot; or reads the all-reduced
//     a.sums when a.part is null, the multi-process path) in k_trial_reduce's order -- thread t
//     sums partials t, t + 256, ..., then the fixed wave / cross-wave tree of block_sum -- so
//     every block holds bit-identical sums;
//  2. computes ||G||^2 in the same fixed order;
//  3. takes the first k with f(W + G/2^k) - f(W) <= (1 + T/2) ||G||^2 2^-k (admm.py:331-338),
//     evaluated as the remainder past the first-order term: since G = grad f(W) (admm.py:302-312),
//     f(W + s G) - f(W) = s <grad f, G> + r(s) with <grad f, G> = ||G||^2, and the test reads
//     r(s) <= (T/2) ||G||^2 s.  The trial sums hold r directly (the per-element first-order terms
//     2 d0 phi'(z) q s are left out of the polynomial and subtracted from the candidate sums), so
//     the decision does not hinge on the rounding of d0 = phi(z) - tgt, which at C3 and C1 leaves
//     O(1) relative noise in G and in s <grad f, G> alike.
//     lhs_k = 0.5 rho (per-candidate sum of this window + polynomial part at s = 2^-k), in fp64;
//  4. updates its slice of W <- (0.5 rho T theta* W - G) / (beta + 0.5 rho theta* T),
//     theta* = 2^k / 2 (admm.py:338-343), and dW.
// Block 0 of the gate writes the stats and the flags.  The found flags are double-buffered by
// pass parity (a.found_in read, a.found_out written): a block that starts after block 0 has
// decided must still see the gate as undecided.
constexpr int kSelBlocks = 16;

__global__ __launch_bounds__(kThreads) void k_select(Geom g, Hyper hp, SelectArgs a) {
  select_gate<false>(g, hp, a, blockIdx.y, blockIdx.x, gridDim.x);
}

// ============================================================================ wy
// U[b][o] = rho_y (h_T . wy[:,o] - a[b][o] - s[b][o]),  s = lam_y / rho_y when with_dual_y.
__global__ __launch_bounds__(kThreads) void k_wy_u(Geom g, Hyper hp, const float* Sh, const float* a,
                                                     const float* Ly, const float* wy, float* U) {
  const int lane = threadIdx.x & 63;
  const float ry = hp.rho[6];
  const bool shift = hp.variant == 0 && hp.with_dual_y;
  const int64_t rs = (int64_t)g.TP() * g.H;
  for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < g.B; b += (int64_t)gridDim.x * 4) {
    const float* h = Sh + b * rs + (int64_t)g.T * g.H;
    for (int o = 0; o < g.O; ++o) {
      float s = 0.f;
      for (int j = lane; j < g.H; j += kWave) s += h[j] * wy[(int64_t)j * g.O + o];
      s = wave_sum(s);
      if (lane == 0) {
        float u = s - a[b * g.O + o];
        if (shift) u = u - Ly[b * g.O + o] / ry;
        U[b * g.O + o] = ry * u;
      }
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_wy_slab(Geom g, const float* Sh, const float* U, float* slab,
                                                        int nsplit) {
  const int64_t nHO = (int64_t)g.H * g.O;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nHO) return;
  const int j = (int)(i / g.O), o = (int)(i % g.O);
  const int64_t per = (g.B + nsplit - 1) / nsplit;
  const int64_t b0 = blockIdx.y * per, b1 = (b0 + per < g.B) ? b0 + per : g.B;
  const int64_t rs = (int64_t)g.TP() * g.H;
  // sequential sum over the rows (fixed order), the h_T and U loads issued 8 rows at a time
  const float* hp = Sh + (int64_t)g.T * g.H + j;
  const float* up = U + o;
  float s = 0.f;
  int64_t b = b0;
  for (; b + 8 <= b1; b += 8) {
    float hv[8], uv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { hv[u] = hp[(b + u) * rs]; uv[u] = up[(b + u) * g.O]; }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += hv[u] * uv[u];
  }
  for (; b < b1; ++b) s += hp[b * rs] * up[b * g.O];
  slab[blockIdx.y * nHO + i] = s;
}

// wy <- (theta* wy - G_y) / (theta* + beta'): admm theta = 1, dead search (admm.py:262-277) ->
// theta* = 1/2, beta' = beta_y; no_dual_y theta* = 0.005, beta' = 2 beta_y (admm.no_dual_y.py:231-249)
__device__ __forceinline__ float wy_new(const Hyper& hp, float w, float G) {
  if (hp.variant == 0) {
    const float th = 0.5f;
    return (th * w - G) / (th + hp.beta_y);
  }
  const float th = 0.005f;
  return (th * w - G) / (th + 2.f * hp.beta_y);
}

// G_y = sum of the slabs; with wy non-null (one process: no all-reduce in between) the same
// thread also applies the update, one launch instead of two
__global__ __launch_bounds__(kThreads) void k_wy_reduce(int64_t nHO, const float* slab, int nsplit, float* Gy,
                                                          Hyper hp, float* wy) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nHO) return;
  double s = 0.0;
  int sp = 0;
  for (; sp + 32 <= nsplit; sp += 32) {   // one workgroup at O = 1: 32 loads in flight, same order
    float v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = slab[(int64_t)(sp + u) * nHO + i];
#pragma unroll
    for (int u = 0; u < 32; ++u) s += (double)v[u];
  }
  for (; sp + 8 <= nsplit; sp += 8) {   // loads issued 8 at a time, the same summation order
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = slab[(int64_t)(sp + u) * nHO + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (double)v[u];
  }
  for (; sp < nsplit; ++sp) s += (double)slab[(int64_t)sp * nHO + i];
  const float G = (float)s;
  Gy[i] = G;
  if (wy) wy[i] = wy_new(hp, wy[i], G);
}

__global__ __launch_bounds__(kThreads) void k_wy_apply(int64_t nHO, Hyper hp, const float* Gy, float* wy) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nHO) return;
  wy[i] = wy_new(hp, wy[i], Gy[i]);
}

// ============================================================================ h_T
// Per row: u = h wy - a - s,  g = gamma u wy^T (admm: gamma = rho_y via autograd; no_dual_y:
// gamma = rho_h), candidates beta(theta) for theta = 0.1 * 2^c.
// Output columns per pass of the generic (runtime O) h_T kernels: their per-candidate
// accumulators stay in registers and any O is covered by ceil(O / kOChunk) passes over the row.
constexpr int kOChunk = 8;

// u = h wy - a - s of one row: in registers for a compile-time O (the O = 1 hot path), else in
// a per-wave LDS row of O floats (every lane writes the same value it holds after wave_sum)
template <int OC>
struct HTRow {
  float reg[OC > 0 ? OC : 1];
  float* lds;
  __device__ __forceinline__ float get(int o) const {
    if constexpr (OC > 0) return reg[o];
    else return lds[o];
  }
  __device__ __forceinline__ void set(int o, float v) {
    if constexpr (OC > 0) reg[o] = v;
    else lds[o] = v;
  }
};

template <int OC>
__device__ __forceinline__ void ht_row_u(const Geom& g, const float* h, const float* a_row, const float* ly_row,
                                         float ry, const float* wy, HTRow<OC>& r) {
  const int NO = OC > 0 ? OC : g.O;
  const int lane = threadIdx.x & 63;
  for (int o = 0; o < NO; ++o) {
    float s = 0.f;
    for (int j = lane; j < g.H; j += kWave) s += h[j] * wy[(int64_t)j * NO + o];
    s = wave_sum(s);
    float u = s - a_row[o];
    if (ly_row) u = u - ly_row[o] / ry;
    r.set(o, u);
  }
}

template <int OC>
__device__ __forceinline__ float ht_grad(const Geom& g, const Hyper& hp, const HTRow<OC>& r, const float* wy, int j) {
  const int NO = OC > 0 ? OC : g.O;
  float s = 0.f;
  if (hp.variant == 0) {
    const float ry = hp.rho[6];
    for (int o = 0; o < NO; ++o) s += (ry * r.get(o)) * wy[(int64_t)j * NO + o];
    return s;
  }
  for (int o = 0; o < NO; ++o) s += r.get(o) * wy[(int64_t)j * NO + o];
  return hp.rho[5] * s;
}

// The h_T search's kHTSums sums of nblk per-block partials: thread t adds partials t, t + 256, ...
// per sum, then the fixed wave / cross-wave tree.  (Folding this into k_ht_partial's last-arriving
// workgroup -- write-through partials, an arrival count -- measured slower than the launch: 18.0 against
// 10.6 + 4.7 us at c3s, profiles/r05f_c3s_step_timeline.txt.)
__device__ __forceinline__ void ht_reduce_block(const double* part, int nblk, double* sums) {
  __shared__ double red[4][kHTSums];
  double s[kHTSums];
#pragma unroll
  for (int i = 0; i < kHTSums; ++i) s[i] = 0.0;
  for (int b = threadIdx.x; b < nblk; b += kThreads) {
#pragma unroll
    for (int i = 0; i < kHTSums; ++i)
      s[i] += part[(int64_t)b * kHTSums + i];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < kHTSums; ++i) {
    const double v = wave_sum(s[i]);
    if (lane == 0) red[w][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < kHTSums) {
    const int i = threadIdx.x;
    sums[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// OC > 0: compile-time output count; OC == 0: runtime g.O, 4 * g.O floats of dynamic LDS
template <int OC>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_ht_partial(Geom g, Hyper hp, Planes6 S, Planes6 L, const float* a,
                                                           const float* Ly, const float* wy, double* part,
                                                           bool gcache) {
  constexpr int CW = OC > 0 ? OC : kOChunk;
  const int NO = OC > 0 ? OC : g.O;
  extern __shared__ float ht_u[];
  __shared__ double accs[4][kHTSums];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float ry = hp.rho[6], rh = hp.rho[5];
  const bool nd = hp.variant == 1;
  const bool shift = !nd && hp.with_dual_y;
  const int64_t rs = (int64_t)g.TP() * g.H, tofs = (int64_t)g.T * g.H;
  // the wave's running sums live in LDS (lane 0 adds, same order as registers would): 26 VGPRs
  // fewer, so all C3 rows' waves are resident at once
  double* acc = accs[w];
  if (lane == 0)
    for (int i = 0; i < kHTSums; ++i) acc[i] = 0.0;
  for (int64_t b = (int64_t)blockIdx.x * 4 + w; b < g.B; b += (int64_t)gridDim.x * 4) {
    const float* h = S.p[5] + b * rs + tofs;
    const float* o_ = S.p[3] + b * rs + tofs;
    const float* c_ = S.p[4] + b * rs + tofs;
    const float* lh = L.p[5] + b * rs + tofs;
    const float* ly = shift ? Ly + b * NO : nullptr;
    HTRow<OC> r;
    r.lds = ht_u + w * NO;
    ht_row_u<OC>(g, h, a + b * NO, ly, ry, wy, r);
    float fh = 0.f;
    for (int o = 0; o < NO; ++o) fh += r.get(o) * r.get(o);
    float ip[kHTCand], nq[kHTCand], fb[kHTCand];
    for (int c = 0; c < kHTCand; ++c) ip[c] = nq[c] = fb[c] = 0.f;
    // runtime O (several output chunks): the gradient g_j, an O-long dot product per j, is formed
    // once per row into the wave's LDS row (gcache) instead of once per chunk
    float* gc = OC == 0 && gcache ? ht_u + 4 * NO + w * g.H : nullptr;
    if (gc)
      for (int j = lane; j < g.H; j += kWave) gc[j] = ht_grad<OC>(g, hp, r, wy, j);
    for (int o0 = 0; o0 < NO; o0 += CW) {
      const int nw = NO - o0 < CW ? NO - o0 : CW;
      float v[kHTCand][CW];
      for (int c = 0; c < kHTCand; ++c)
        for (int oo = 0; oo < CW; ++oo) v[c][oo] = 0.f;
      for (int j = lane; j < g.H; j += kWave) {
        const float gj = gc ? gc[j] : ht_grad<OC>(g, hp, r, wy, j);   // (each lane reads its own j)
        const float hj = h[j], pj = rh * o_[j] * tanhf(c_[j]) - lh[j];
        for (int c = 0; c < kHTCand; ++c) {
          const float th = ldexpf(0.1f, c);
          const float bj = nd ? gj / th : (th * hj + pj - gj) / (th + rh);
          const float dj = bj - hj;
          if (o0 == 0) {
            ip[c] += gj * dj;
            nq[c] += dj * dj;
          }
          for (int oo = 0; oo < nw; ++oo) v[c][oo] += bj * wy[(int64_t)j * NO + o0 + oo];
        }
      }
      for (int c = 0; c < kHTCand; ++c)
        for (int oo = 0; oo < nw; ++oo) {
          float vv = wave_sum(v[c][oo]) - a[b * NO + o0 + oo];
          if (shift) vv = vv - ly[o0 + oo] / ry;
          fb[c] += vv * vv;
        }
    }
    // wave-reduce and accumulate (lane 0 holds the row's values)
    if (lane == 0) acc[0] += (double)fh;  // identical on every lane
    for (int c = 0; c < kHTCand; ++c) {
      const float sip = wave_sum(ip[c]), snq = wave_sum(nq[c]);
      if (lane == 0) {
        acc[1 + 3 * c] += (double)fb[c];
        acc[2 + 3 * c] += (double)sip;
        acc[3 + 3 * c] += (double)snq;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < kHTSums) {
    const int i = threadIdx.x;
    part[(int64_t)blockIdx.x * kHTSums + i] = (accs[0][i] + accs[1][i]) + (accs[2][i] + accs[3][i]);
  }
}

// all kHTSums sums in one pass over the partials (per sum: thread t adds partials t, t + 256, ...,
// then block_sum's fixed tree -- the order of a per-sum loop, one barrier instead of 2 kHTSums)
__global__ __launch_bounds__(kThreads) void k_ht_reduce(const double* part, int nblk, double* sums) {
  ht_reduce_block(part, nblk, sums);
}

__device__ __forceinline__ float ht_theta_star(const Hyper& hp, const double* sums) {
  const double ry = hp.rho[6];
  const double fh = 0.5 * ry * sums[0];
  float th = 0.1f;
  for (int c = 0; c < kHTCand; ++c) {  // admm.py:474-482
    const double fb = 0.5 * ry * sums[1 + 3 * c];
    const double est = fh + sums[2 + 3 * c] + 0.5 * (double)th * sums[3 + 3 * c];
    if (!(fb > est)) break;
    th *= 2.f;
    if (th >= 1.f) break;
  }
  return th / 2.f;
}

// h_T update with theta* (admm.py:482-487), a update (489-502), dual h at T (532-539),
// dual y (541-546, admm variant with with_dual_y).  OC as k_ht_partial.
template <int OC>
__global__ __launch_bounds__(kThreads) void k_ht_apply(Geom g, Hyper hp, Planes6 S, Planes6 L, float* a, float* Ly,
                                                         const float* y, const float* wy, const double* sums,
                                                         DevStats* stats, int* status, const int* force, float* U,
                                                         uint4* __restrict__ xbuf, int nx) {
  // the next step's column-split sweep starts from zeroed hand-off granules and entry count
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < nx; i += gridDim.x * kThreads) xbuf[i] = make_uint4(0u, 0u, 0u, 0u);
  constexpr int CW = OC > 0 ? OC : kOChunk;
  const int NO = OC > 0 ? OC : g.O;
  extern __shared__ float ht_u[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float ry = hp.rho[6], rh = hp.rho[5];
  const bool nd = hp.variant == 1;
  const bool shift = !nd && hp.with_dual_y;
  const float th_own = ht_theta_star(hp, sums);
  // admm_debug_force: force[8] = the number of failing comparisons of the reference's search
  // (theta = 0.1 doubled that many times, then halved: admm.py:474-482)
  const float th = force ? ldexpf(0.1f, force[8]) / 2.f : th_own;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stats->theta_h = th;
    stats->theta_h_own = th_own;
    if (status) {   // host-mapped mirror for admm_poll_status (the decide kernels and the sweep ran earlier on this stream)
      const int* src[4] = {&stats->unresolved, &stats->nonfinite, &stats->handoff_fail, &stats->sweep_fallback};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __hip_atomic_store(&status[i], __hip_atomic_load(src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  const int64_t rs = (int64_t)g.TP() * g.H, tofs = (int64_t)g.T * g.H;
  const float Bry = (float)g.Bg * ry;
  for (int64_t b = (int64_t)blockIdx.x * 4 + w; b < g.B; b += (int64_t)gridDim.x * 4) {
    float* h = S.p[5] + b * rs + tofs;
    const float* o_ = S.p[3] + b * rs + tofs;
    const float* c_ = S.p[4] + b * rs + tofs;
    float* lh = L.p[5] + b * rs + tofs;
    HTRow<OC> r;
    r.lds = ht_u + w * NO;
    ht_row_u<OC>(g, h, a + b * NO, shift ? Ly + b * NO : nullptr, ry, wy, r);
    // the first pass writes the new h_T (and its dual); later passes re-read the lane's own h_T
    for (int o0 = 0; o0 < NO; o0 += CW) {
      const int nw = NO - o0 < CW ? NO - o0 : CW;
      float hw[CW];
      for (int oo = 0; oo < CW; ++oo) hw[oo] = 0.f;
      for (int j = lane; j < g.H; j += kWave) {
        float hn;
        if (o0 == 0) {
          const float gj = ht_grad<OC>(g, hp, r, wy, j);
          const float tc = tanhf(c_[j]);
          hn = (th * h[j] + rh * o_[j] * tc - lh[j] - gj) / (th + rh);
          h[j] = hn;
          lh[j] = lh[j] + rh * (hn - o_[j] * tc);
        } else {
          hn = h[j];
        }
        for (int oo = 0; oo < nw; ++oo) hw[oo] += hn * wy[(int64_t)j * NO + o0 + oo];
      }
      for (int oo = 0; oo < nw; ++oo) {
        const float hwo = wave_sum(hw[oo]);
        if (lane == 0) {
          const int64_t i = b * NO + o0 + oo;
          float an;
          if (!nd) {
            const float corr = shift ? (float)g.Bg * Ly[i] : 0.f;
            an = (2.f * y[i] + Bry * hwo - corr) / (2.f + Bry);
          } else {
            an = (Bry * hwo + 2.f * y[i]) / (2.f + Bry);
          }
          a[i] = an;
          float ly_new = 0.f;
          if (shift) Ly[i] = ly_new = Ly[i] + ry * (an - hwo);
          // U (nullable): the next step's wy residual rho_y (h_T wy - a - s) of this row, which k_wy_u
          // would form from the same h_T, wy, a and dual y (hwo is its h_T . wy, same order)
          if (U) {
            float u = hwo - an;
            if (shift) u = u - ly_new / ry;
            U[i] = ry * u;
          }
        }
      }
    }
  }
}

}  // namespace

// flag <- 1 if the dual of h has a nonzero entry at some t in [1, T) (k_sweep_rows lh_zero)
__global__ __launch_bounds__(kThreads) void k_check_lamh(Geom g, const float* __restrict__ lh, int* flag) {
  const int64_t H4 = g.H / 4, per_b = (int64_t)(g.T - 1) * H4, n = g.B * per_b;
  bool nz = false;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const int64_t b = i / per_b, r = i - b * per_b;
    const float4 v = ld_nt(lh + b * g.TP() * g.H + g.H + 4 * r);
    nz |= (v.x != 0.f) | (v.y != 0.f) | (v.z != 0.f) | (v.w != 0.f);
  }
  if (__any(nz) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// range[5] = max over rows of sum_d |x[row][d]| (bounds |x dWx| for k_atr3w's fp16 scale)
__global__ __launch_bounds__(kThreads) void k_x_l1max(int64_t rows, int D, const float* __restrict__ x,
                                                        float* range) {
  float m = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < rows; r += (int64_t)gridDim.x * kThreads) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += fabsf(x[r * D + d]);
    m = fmaxf(m, s);
  }
  range_max(range + 5, m);
}

// ============================================================================ launchers

void launch_x_l1max(const Geom& g, const float* x, float* range, hipStream_t s) {
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(g.BT(), kThreads), 1024));
  k_x_l1max<<<nb, kThreads, 0, s>>>(g.BT(), g.D, x, range);
}

void launch_check_lamh(const Geom& g, const float* lh, int* flag, hipStream_t s) {
  const int64_t n = g.B * (int64_t)(g.T - 1) * (g.H / 4);
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, kThreads), 2048));
  k_check_lamh<<<nb, kThreads, 0, s>>>(g, lh, flag);
}

// float4 staging needs 16-byte aligned rows of x and of the [.., H] planes
inline int vec_ok(const Geom& g) { return (g.D % 4 == 0 && g.H % 4 == 0) ? 1 : 0; }

void launch_forward_t(const Geom& g, int t, const Weights& w, const ForwardT& a, hipStream_t s) {
  dim3 grid(cdiv64(g.B, TS_BM) * cdiv64(g.H, 32));
  if (vec_ok(g) && (a.hprev_stride % 4 == 0)) k_forward_t<true><<<grid, kThreads, 0, s>>>(g, t, w, a);
  else k_forward_t<false><<<grid, kThreads, 0, s>>>(g, t, w, a);
}

void launch_sweep_t(const Geom& g, int t, const Weights& w, const Hyper& hp, const SweepT& a, hipStream_t s) {
  dim3 grid(cdiv64(a.r1 - a.r0, TS_BM) * cdiv64(g.H, 32));
  if (vec_ok(g)) k_sweep_t<true><<<grid, kThreads, 0, s>>>(g, t, w, hp, a);
  else k_sweep_t<false><<<grid, kThreads, 0, s>>>(g, t, w, hp, a);
}

// 16-row tiles for 256 < H <= 512 (ADMM_SWEEP_R16=0: those shapes take the per-t sweep)
static bool sweep_r16(const Geom& g) { return g.r16 && g.H > 256 && g.H <= 512 && g.H % 64 == 0; }  // (r16: test hook)

bool sweep_rows_ok(const Geom& g) {
  // 32-bit buffer offsets: a [B][T+1][H] plane and a [B*T][H] z-cache plane in bytes
  // NT >= 2 column tiles (the mid-step barrier protocol)
  const bool shape = (g.H % 32 == 0 && g.H >= 64 && g.H <= 256) || sweep_r16(g);
  return shape && g.D <= 32 && g.B * (int64_t)g.TP() * g.H * 4 < (int64_t)UINT32_MAX &&
         4 * g.BT() * g.H * 4 < (int64_t)UINT32_MAX;   // the 4-plane z cache / target descriptors
}

bool sweep_rows_gx_ok(const Geom& g) { return sweep_rows_ok(g) && (sweep_r16(g) ? g.D == 1 : g.D <= 16); }
int sweep_rows_blocks(const Geom& g) { return (int)((g.B + (sweep_r16(g) ? 15 : 31)) / (sweep_r16(g) ? 16 : 32)); }

// Column groups of the persistent sweep (k_sweep_rows NC): 1 while the 32-row blocks alone give a
// workgroup to at least half of the 256 CUs; else the largest of 8, 4, 2 whose padded grid
// (row blocks rounded up to 8, times the groups) still has one workgroup per CU.  H = 256 only.
int sweep_rows_nc(const Geom& g) {
  if (sweep_r16(g) || g.H != 256 || !sweep_rows_ok(g)) return 1;
  const int64_t nrb = (g.B + 31) / 32, pad = (nrb + 7) / 8 * 8;
  // (at 4096 rows, 128 row blocks, two groups still pay: 1.07 against 1.39 ms for the row-block sweep;
  // 2048 rows, four groups: 0.63 against 1.31 ms; tools/kbench, profiles/r04r_sweep_nc_kbench.txt)
  if (nrb > 128) return 1;
  for (int nc : {8, 4, 2})
    if (pad * nc <= kSweepCUs) return nc;
  return 1;
}

int sweep_row_blocks_padded(const Geom& g) { return (int)(((g.B + 31) / 32 + 7) / 8 * 8); }

// one 8-byte granule {h value, tag t} per (row, column) of every padded row block (k_sweep_rows NC > 1)
void sweep_poison_entry(const Geom& g, void* xbuf, hipStream_t s) {
  (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(static_cast<char*>(xbuf) + sweep_xbuf_bytes(g) - 256),
                          (int)kSweepPoison, 1, s);
}
// two granule sets, then the entry count (k_sweep_rows' sweep_arrive)
size_t sweep_xbuf_bytes(const Geom& g) { return (size_t)sweep_row_blocks_padded(g) * 32 * g.H * 8 * 2 + 256; }

static int sweep_xc(const Geom& g) { return sweep_r16(g) ? (g.D + 31) / 32 : (g.D + 15) / 16; }
int sweep_wt_rows16(const Geom& g) { return sweep_r16(g) ? 1 : 0; }
int sweep_wt_xc(const Geom& g) { return sweep_xc(g); }

size_t sweep_wt_floats(const Geom& g) {   // bf16x8 image, in float units
  if (sweep_r16(g)) return (size_t)4 * (g.H / 64) * (sweep_xc(g) + g.H / 32) * 4 * 3 * 64 * 4;
  return (size_t)4 * (g.H / 32) * (sweep_xc(g) + 2 * (g.H / 32)) * 3 * 64 * 4;
}

void launch_sweep_wt(const Geom& g, const Weights& w, float* wt, hipStream_t s, void* xbuf) {
  const int xc = sweep_xc(g);
  if (sweep_r16(g)) {
    const int total = 4 * (g.H / 64) * (xc + g.H / 32) * 4 * 64;
    k_sweep_wt16<<<cdiv64(total, kThreads), kThreads, 0, s>>>(g.D, g.H, xc, w, reinterpret_cast<bf16x8*>(wt));
    return;
  }
  const int NT = g.H / 32;
  const int total = 4 * NT * (xc + 2 * NT) * 64;
  k_sweep_wt<<<cdiv64(total, kThreads), kThreads, 0, s>>>(g.D, g.H, xc, w, reinterpret_cast<bf16x8*>(wt),
                                                         reinterpret_cast<uint4*>(xbuf),
                                                         xbuf ? (int)(sweep_xbuf_bytes(g) / 16) : 0);
}

template <int XC>
static void launch_sweep_rows_xc(const Geom& g, const bf16x8* wt, const Hyper& hp, const SweepT& a, hipStream_t s) {
  if (sweep_r16(g)) {
    dim3 grid(cdiv64(a.r1 - a.r0, 16));
    switch (g.H / 64) {
#define SR16_CASE(N) case N: \
  if (XC == 1 && g.D == 1 && a.gx_slab) k_sweep_rows<N, XC, true, 16><<<grid, SR_THREADS, 0, s>>>(g, wt, hp, a); \
  else k_sweep_rows<N, XC, false, 16><<<grid, SR_THREADS, 0, s>>>(g, wt, hp, a); \
  break;
      SR16_CASE(5) SR16_CASE(6) SR16_CASE(7) SR16_CASE(8)
#undef SR16_CASE
      default: break;
    }
    return;
  }
  const int nc = a.xbuf ? sweep_rows_nc(g) : 1;
  if (nc > 1 && g.H == 256) {   // column split (strong-scaling ranks): padded row blocks x nc groups
    dim3 grid((unsigned)(sweep_row_blocks_padded(g) * nc));
    auto go = [&](auto ncv) {
      constexpr int NCV = decltype(ncv)::value;
      if (XC == 1 && a.gx_slab) k_sweep_rows<8, XC, true, 32, NCV><<<grid, SR_THREADS, 0, s>>>(g, wt, hp, a);
      else k_sweep_rows<8, XC, false, 32, NCV><<<grid, SR_THREADS, 0, s>>>(g, wt, hp, a);
    };
    if (nc == 8) go(std::integral_constant<int, 8>{});
    else if (nc == 4) go(std::integral_constant<int, 4>{});
    else go(std::integral_constant<int, 2>{});
    // the row-block sweep, in case the column split could not have its whole grid resident (its
    // workgroups leave at once otherwise: one empty launch per step)
    SweepT ar = a;
    ar.gate = reinterpret_cast<const unsigned*>(static_cast<const char*>(a.xbuf) + sweep_xbuf_bytes(g) - 256);
    ar.xbuf = nullptr;
    dim3 rgrid(cdiv64(a.r1 - a.r0, SR_ROWS));
    if (XC == 1 && a.gx_slab) k_sweep_rows<8, XC, true><<<rgrid, SR_THREADS, 0, s>>>(g, wt, hp, ar);
    else k_sweep_rows<8, XC, false><<<rgrid, SR_THREADS, 0, s>>>(g, wt, hp, ar);
    return;
  }
  dim3 grid(cdiv64(a.r1 - a.r0, SR_ROWS));
  switch (g.H / 32) {
#define SR_CASE(N) case N: \
  if (XC == 1 && a.gx_slab) k_sweep_rows<N, XC, true><<<grid, SR_THREADS, 0, s>>>(g, wt, hp, a); \
  else k_sweep_rows<N, XC, false><<<grid, SR_THREADS, 0, s>>>(g, wt, hp, a); \
  break;
    SR_CASE(2) SR_CASE(3) SR_CASE(4) SR_CASE(5) SR_CASE(6) SR_CASE(7) SR_CASE(8)
#undef SR_CASE
    default: break;
  }
}

void launch_sweep_rows(const Geom& g, const float* wt, const Hyper& hp, const SweepT& a, hipStream_t s) {
  const bf16x8* w = reinterpret_cast<const bf16x8*>(wt);
  if (sweep_xc(g) == 1) launch_sweep_rows_xc<1>(g, w, hp, a, s);
  else launch_sweep_rows_xc<2>(g, w, hp, a, s);
}

void launch_rowdot(int64_t B, int H, int O, const float* h, int64_t hs, const float* wy, float* out, hipStream_t s) {
  int nb = cdiv64(B, 4);
  if (nb > 2048) nb = 2048;
  k_rowdot<<<nb, kThreads, 0, s>>>(B, H, O, h, hs, wy, out);
}

void launch_zgemm(const Geom& g, const Weights& w, const float* x, const float* Sh, float* zc, hipStream_t s) {
  dim3 grid(cdiv64(g.BT(), TS_BM) * cdiv64(g.H, 32));
  if (vec_ok(g)) k_zgemm<true><<<grid, kThreads, 0, s>>>(g, w, x, Sh, zc);
  else k_zgemm<false><<<grid, kThreads, 0, s>>>(g, w, x, Sh, zc);
}

int resid_blocks(const Geom& g) {
  const int hchunk = g.H < kThreads ? g.H : kThreads;
  const int rpb = kThreads / hchunk;
  int nb = cdiv64(g.BT(), rpb);
  return nb > 1024 ? 1024 : nb;
}

void launch_resid(const Geom& g, const Hyper& hp, const ResidArgs& a, hipStream_t s) {
  dim3 grid(a.nblk, 4);
  k_resid<<<grid, kThreads, 0, s>>>(g, hp, a);
}

bool atr_wide(const Geom& g) { return g.H % 256 == 0; }

int atr_splits(const Geom& g, int side) {
  const int Kd = side == 0 ? g.D : g.H;
  const int tiles = cdiv64(Kd, side == 1 ? 128 : 32) * cdiv64(g.H, 128) * 4;
  int ns = 1024 / tiles;
  const int64_t max_by_rows = g.BT() / 256;  // keep >= 256 rows per split
  if (ns > max_by_rows) ns = (int)max_by_rows;
  if (ns > 256) ns = 256;
  return ns < 1 ? 1 : ns;
}

void launch_atr(const Geom& g, int side, const float* x, const float* Sh, const float* R, float* slab, int nsplit,
                hipStream_t s) {
  const int Kd = side == 0 ? g.D : g.H;
  dim3 grid(cdiv64(Kd, side == 1 ? 128 : 32) * cdiv64(g.H, 128) * 4 * nsplit);
  if (side == 1) {
    if (vec_ok(g)) k_atr<128, 64, true, 1><<<grid, kThreads, 0, s>>>(g, x, Sh, R, slab, nsplit);
    else k_atr<128, 64, false, 1><<<grid, kThreads, 0, s>>>(g, x, Sh, R, slab, nsplit);
  } else {
    if (vec_ok(g)) k_atr<32, 32, true, 0><<<grid, kThreads, 0, s>>>(g, x, Sh, R, slab, nsplit);
    else k_atr<32, 32, false, 0><<<grid, kThreads, 0, s>>>(g, x, Sh, R, slab, nsplit);
  }
}

void launch_reduce_g(const Geom& g, int side, const Hyper& hp, const float* slab, int nsplit, float* G, int* found,
                     int* kpred, const DevStats* stats, hipStream_t s, bool p16, float* range_reset) {
  const int Kd = side == 0 ? g.D : g.H;
  const int64_t n = 4LL * Kd * g.H;
  k_reduce_g<<<cdiv64(n, kThreads), kThreads, 0, s>>>(Kd, g.H, side, p16 ? 1 : 0, hp, slab, nsplit, G, found, kpred,
                                                       stats, range_reset);
}

void launch_reduce_gh_img(const Geom& g, const Hyper& hp, const float* slab, int nsplit, float* G, int* found,
                          const DevStats* stats, hipStream_t s, bool p16, float* range_reset, float* gimg) {
  const int total = 4 * (g.H / 16) * (g.H / 32) * 64;
  k_reduce_gh_img<<<cdiv64(total, kThreads), kThreads, 0, s>>>(g.H, p16 ? 1 : 0, hp, slab, nsplit, G, found, stats,
                                                               range_reset, reinterpret_cast<bf16x8*>(gimg));
}

void launch_qgemm(const Geom& g, int side, const float* x, const float* Sh, const float* G, float* Q,
                  hipStream_t s) {
  dim3 grid(cdiv64(g.BT(), TS_BM) * cdiv64(g.H, 32));
  if (side == 0) {
    if (vec_ok(g)) k_qgemm<true, 0><<<grid, kThreads, 0, s>>>(g, x, Sh, G, Q);
    else k_qgemm<false, 0><<<grid, kThreads, 0, s>>>(g, x, Sh, G, Q);
  } else {
    if (vec_ok(g)) k_qgemm<true, 1><<<grid, kThreads, 0, s>>>(g, x, Sh, G, Q);
    else k_qgemm<false, 1><<<grid, kThreads, 0, s>>>(g, x, Sh, G, Q);
  }
}

int trial_blocks(const Geom& g) {
  int nb = cdiv64(g.BT() * g.H, kThreads * 8);
  return nb > 2048 ? 2048 : (nb < 1 ? 1 : nb);
}

void launch_trial(const Geom& g, int pass, const float* zc, const float* tgt, const float* Q, const int* found,
                  double* part, int nblk, hipStream_t s) {
  dim3 grid(nblk, 4);
  if (pass == kTailPass) k_trial<true><<<grid, kThreads, 0, s>>>(g, pass, zc, tgt, Q, found, part, nblk);
  else k_trial<false><<<grid, kThreads, 0, s>>>(g, pass, zc, tgt, Q, found, part, nblk);
}

void launch_trial_debug(int64_t n, int tanh_gate, int kbase, const float* z, const float* tgt, const float* q,
                        double* part, int nblk, hipStream_t s) {
  k_trial_debug<<<nblk, kThreads, 0, s>>>(n, tanh_gate, kbase, z, tgt, q, part);
}

// Test hook (admm_debug_trace_resid): the residual R_q = (phi(z) - tgt) phi'(z) of one weight
// stage, element by element with the activation every stage forms it with (sig_pair / tanhf: the
// sweep's x-stage G_x partials, k_resid_gx, and the h stage's k_atr3w / k_atr_fused staging; the
// admm.py:302-312 residual), so a test can recompute G = rho A^T R on identical operands.
__global__ __launch_bounds__(kThreads) void k_debug_resid(int64_t n, const float* __restrict__ z,
                                                           const float* __restrict__ tgt, float* __restrict__ R) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < 4 * n; i += (int64_t)gridDim.x * kThreads) {
    const float zz = z[i], tt = tgt[i];
    float phi, dphi;
    if (i / n == 2) phi_acc<true>(zz, phi, dphi);
    else phi_acc<false>(zz, phi, dphi);
    R[i] = (phi - tt) * dphi;
  }
}

void launch_debug_resid(const Geom& g, const float* z, const float* tgt, float* R, hipStream_t s) {
  const int64_t n = g.BT() * g.H;
  const int nb = (int)std::min<int64_t>((4 * n + kThreads - 1) / kThreads, 8192);
  k_debug_resid<<<nb, kThreads, 0, s>>>(n, z, tgt, R);
}

void launch_trial_reduce(const Geom& g, int pass, const double* part, int nblk, const int* found, double* sums,
                         hipStream_t s) {
  (void)g;
  k_trial_reduce<<<dim3(kSlots, 4, pass == kTailPass ? kMaxPasses - 1 : 1), kThreads, 0, s>>>(pass, part, nblk, found, sums);
}

bool fast_path(const Geom& g) {
  return g.D <= kFastD && g.H % 4 == 0 && g.H / 4 <= kThreads && (int64_t)kFastD * g.H * 4 <= 64 * 1024;
}

int resid_gx_blocks(const Geom& g) {
  int nb = cdiv64(g.BT(), 256);
  return nb > 256 ? 256 : (nb < 1 ? 1 : nb);
}

size_t fast_lds(const Geom& g) { return (size_t)((g.D + 3) / 4) * 4 * g.H * sizeof(float); }

void launch_resid_gx(const Geom& g, const Hyper& hp, const float* x, const Planes6& S, const Planes6& L,
                     const float* zc, float* tgt, float* slab, int nblk, bool tgt_ready, hipStream_t s) {
  dim3 grid(nblk, 4);
  with_dp(g, [&](auto dp, auto xv) {
    k_resid_gx<decltype(dp)::value, decltype(xv)::value>
        <<<grid, kThreads, (size_t)g.D * g.H * sizeof(float), s>>>(g, hp, x, S, L, zc, tgt, slab, tgt_ready);
  });
}

void launch_atr_fused(const Geom& g, const Hyper& hp, const float* x, const float* Sh, const float* zc,
                      const float* tgt, const float* dW, float* slab, int nsplit, hipStream_t s) {
  (void)hp;
  if (atr_wide(g)) {
    dim3 grid(cdiv64(g.H, 256) * cdiv64(g.H, 128) * 4 * nsplit);
    k_atr_fused<256, 128, 16><<<grid, kThreads, 0, s>>>(g, x, Sh, zc, tgt, dW, slab, nsplit);
  } else {
    dim3 grid(cdiv64(g.H, 128) * cdiv64(g.H, 128) * 4 * nsplit);
    k_atr_fused<128, 64, 32><<<grid, kThreads, 0, s>>>(g, x, Sh, zc, tgt, dW, slab, nsplit);
  }
}

int stream_blocks(const Geom& g) {   // streaming passes: ~2 rows in flight per thread
  const int hchunk = g.H / 4 < kThreads ? g.H / 4 : kThreads;
  const int rpb = kThreads / (hchunk > 0 ? hchunk : 1);
  int nb = cdiv64(g.BT(), (int64_t)rpb * kRPI * 4);
  return nb > 512 ? 512 : (nb < 1 ? 1 : nb);
}

void launch_apply_dwx(const Geom& g, const float* x, const float* dW, float* zc, hipStream_t s) {
  dim3 grid(stream_blocks(g), 4);
  with_dp(g, [&](auto dp, auto xv) {
    k_apply_dwx<decltype(dp)::value, decltype(xv)::value>
        <<<grid, kThreads, fast_lds(g), s>>>(g, x, dW, zc, zc, nullptr, nullptr);
  });
}

void launch_apply_fix(const Geom& g, const float* x, const float* dW, const float* zc, float* zx, const int* kpred,
                      const DevStats* stats, hipStream_t s) {
  dim3 grid(stream_blocks(g), 4);
  with_dp(g, [&](auto dp, auto xv) {
    k_apply_dwx<decltype(dp)::value, decltype(xv)::value>
        <<<grid, kThreads, fast_lds(g), s>>>(g, x, dW, zc, zx, kpred, stats);
  });
}

bool trial_rows_ok(const Geom& g) { return g.H % 256 == 0; }

// workgroups per gate (and column block) of the fast trial passes.  Each walks the rows with a
// stride of that many tiles, so few rows per GPU leave each workgroup few tiles to amortise its
// setup and its epilogue (the 38-slot block reduction) over: at B = 1024 the x trials (k_trial_mx)
// take 111 / 99 / 92 us with 512 / 256 / 128 workgroups when every gate is in the polynomial regime
// (tools/kbench "tr", KB_NB).  But the step's g gate is mostly in the per-candidate regime, which
// costs its workgroups 2-3x the others', and with a single round of workgroups the CUs of the other
// gates then idle: with that mix (kbench "trg") 128 / 256 / 512 workgroups take 151 / 109 / 113 us
// (profiles/r05n_trial_grid_scan.txt).  So at least 8 tiles per workgroup (256 at B = 1024); at
// B = 8192 and for the h trials the streaming count stays.  Never more than stream_blocks(g): the
// partial buffer is sized for it.
int trial_fast_blocks(const Geom& g, int side) {
  const int sb = stream_blocks(g);
  if (side == 0 && trial_mx_ok(g)) {
    const int64_t nb = (g.BT() + 15) / 16 / 8;   // >= 8 tiles per workgroup
    return (int)std::min<int64_t>(sb, std::max<int64_t>(64, nb));
  }
  return sb;
}

bool tail_select_fused(const Geom& g, int side) {
  return side == 1 ? trial_rows_ok(g) : trial_mx_ok(g);
}

bool trial_mx_ok(const Geom& g) {   // else (a gate plane past 2 GB) the x side runs on k_trial_rows (VALU q)
  // 32-bit buffer offsets within one gate plane
  return g.H % 256 == 0 && g.D <= 16 && g.BT() * g.H * 4 < (int64_t)INT32_MAX;
}

void launch_trial_fast(const Geom& g, int side, int pass, const float* zc, const float* tgt, const float* Q,
                       const float* x, const float* Wsrc, const int* found, double* part, int nblk, hipStream_t s,
                       const SpecX* spec, int qpair, const SelectArgs* fsel, const Hyper* fhp, unsigned* fcount) {
  dim3 grid(nblk, 4);
  const SpecX sp = spec ? *spec : SpecX{};
  TailSel ts{};
  if (pass == kTailPass && fsel && fhp && fcount && tail_select_fused(g, side)) {
    ts.a = *fsel;
    ts.hp = *fhp;
    ts.count = fcount;
  }
  // TAIL: the windows 1 .. kMaxPasses - 1 in one launch (pass == kTailPass); only pass 0 speculates
  auto go = [&](auto tail) {
    constexpr bool TL = decltype(tail)::value;
    if (side == 1 && trial_rows_ok(g)) {
      dim3 gr(nblk, 4, g.H / 256);
      if (qpair == 2 && qpair_ok(g))
        k_trial_rows<1, 4, false, false, 2, TL><<<gr, kThreads, 0, s>>>(g, pass, zc, tgt, Q, x, Wsrc, found, part, nblk, sp, ts);
      else
        k_trial_rows<1, 4, false, false, 0, TL><<<gr, kThreads, 0, s>>>(g, pass, zc, tgt, Q, x, Wsrc, found, part, nblk, sp, ts);
      return;
    }
    if (side == 1) {  // no x . W product on this side: one instantiation
      k_trial_fast<1, 4, false, false, TL><<<grid, kThreads, 0, s>>>(g, pass, zc, tgt, Q, x, Wsrc, found, part, nblk);
      return;
    }
    if (trial_mx_ok(g)) {   // side 0 on the matrix cores
      dim3 gr(nblk, 4, g.H / 128);
      if (spec && !TL) k_trial_mx<true, false><<<gr, kThreads, 0, s>>>(g, pass, zc, tgt, x, Wsrc, found, part, nblk, sp, ts);
      else k_trial_mx<false, TL><<<gr, kThreads, 0, s>>>(g, pass, zc, tgt, x, Wsrc, found, part, nblk, sp, ts);
      return;
    }
    if (trial_rows_ok(g)) {
      dim3 gr(nblk, 4, g.H / 256);
      with_dp(g, [&](auto dp, auto xv) {
        if (spec && !TL)
          k_trial_rows<0, decltype(dp)::value, decltype(xv)::value, true, 0, false>
              <<<gr, kThreads, 0, s>>>(g, pass, zc, tgt, Q, x, Wsrc, found, part, nblk, sp, TailSel{});
        else
          k_trial_rows<0, decltype(dp)::value, decltype(xv)::value, false, 0, TL>
              <<<gr, kThreads, 0, s>>>(g, pass, zc, tgt, Q, x, Wsrc, found, part, nblk, sp, TailSel{});
      });
      return;
    }
    const bool ur = (g.H / 4) % 64 == 0;   // one row per wave
    with_dp(g, [&](auto dp, auto xv) {
      if (ur)
        k_trial_fast<0, decltype(dp)::value, decltype(xv)::value, true, TL>
            <<<grid, kThreads, fast_lds(g), s>>>(g, pass, zc, tgt, Q, x, Wsrc, found, part, nblk);
      else
        k_trial_fast<0, decltype(dp)::value, decltype(xv)::value, false, TL>
            <<<grid, kThreads, fast_lds(g), s>>>(g, pass, zc, tgt, Q, x, Wsrc, found, part, nblk);
    });
  };
  if (pass == kTailPass) go(std::integral_constant<bool, true>{});
  else go(std::integral_constant<bool, false>{});
}

void launch_select(const Geom& g, const Hyper& hp, const SelectArgs& a, hipStream_t s) {
  k_select<<<dim3(kSelBlocks, 4), kThreads, 0, s>>>(g, hp, a);
}

int wy_splits(const Geom& g) {   // 64 rows per split: the strided h_T loads are latency-bound
  int ns = cdiv64(g.B, 64);
  return ns > 512 ? 512 : (ns < 1 ? 1 : ns);
}

void launch_wy_grad(const Geom& g, const Hyper& hp, const float* Sh, const float* a, const float* Ly,
                    const float* wy, float* U, float* slab, int nsplit, hipStream_t s, bool u_ready) {
  int nb = cdiv64(g.B, 4);
  if (nb > 2048) nb = 2048;
  if (!u_ready) k_wy_u<<<nb, kThreads, 0, s>>>(g, hp, Sh, a, Ly, wy, U);
  const int64_t nHO = (int64_t)g.H * g.O;
  dim3 grid(cdiv64(nHO, kThreads), nsplit);
  k_wy_slab<<<grid, kThreads, 0, s>>>(g, Sh, U, slab, nsplit);
}

void launch_wy_reduce(const Geom& g, const Hyper& hp, const float* slab, int nsplit, float* Gy, float* wy_apply,
                      hipStream_t s) {
  const int64_t nHO = (int64_t)g.H * g.O;
  k_wy_reduce<<<cdiv64(nHO, kThreads), kThreads, 0, s>>>(nHO, slab, nsplit, Gy, hp, wy_apply);
}

void launch_wy_apply(const Geom& g, const Hyper& hp, const float* Gy, float* wy, hipStream_t s) {
  const int64_t nHO = (int64_t)g.H * g.O;
  k_wy_apply<<<cdiv64(nHO, kThreads), kThreads, 0, s>>>(nHO, hp, Gy, wy);
}

int ht_blocks(const Geom& g) {   // one row per wave up to B = 8192 (each row is a latency chain)
  int nb = cdiv64(g.B, 4);
  return nb > 2048 ? 2048 : nb;
}

void launch_ht_partial(const Geom& g, const Hyper& hp, const Planes6& S, const Planes6& L, const float* a,
                       const float* Ly, const float* wy, double* part, int nblk, hipStream_t s) {
  if (g.O == 1) {
    k_ht_partial<1><<<nblk, kThreads, 0, s>>>(g, hp, S, L, a, Ly, wy, part, false);
    return;
  }
  // more than one output chunk: cache g_j per wave in LDS while that fits 64 KB
  const size_t lds = 4 * (size_t)g.O * sizeof(float), lds_g = lds + 4 * (size_t)g.H * sizeof(float);
  const bool gc = g.O > kOChunk && lds_g <= 64 * 1024;
  k_ht_partial<0><<<nblk, kThreads, gc ? lds_g : lds, s>>>(g, hp, S, L, a, Ly, wy, part, gc);
}

void launch_ht_reduce(const double* part, int nblk, double* sums, hipStream_t s) {
  k_ht_reduce<<<1, kThreads, 0, s>>>(part, nblk, sums);
}

void launch_ht_apply(const Geom& g, const Hyper& hp, const Planes6& S, const Planes6& L, float* a, float* Ly,
                     const float* y, const float* wy, const double* sums, DevStats* stats, int* status, hipStream_t s,
                     const int* force, float* U, void* xbuf) {
  const int nx = xbuf ? (int)(sweep_xbuf_bytes(g) / 16) : 0;
  uint4* xb = static_cast<uint4*>(xbuf);
  if (g.O == 1) k_ht_apply<1><<<ht_blocks(g), kThreads, 0, s>>>(g, hp, S, L, a, Ly, y, wy, sums, stats, status, force, U, xb, nx);
  else k_ht_apply<0><<<ht_blocks(g), kThreads, 4 * g.O * sizeof(float), s>>>(g, hp, S, L, a, Ly, y, wy, sums, stats,
                                                                            status, force, U, xb, nx);
}

#ifdef SR_CS_TIMING
extern "C" void cs_timing_dump(int T) {
  unsigned long long h[64][12];
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cs_t), sizeof h);
  // wall_clock64: 100 MHz; per t: phase deltas in us, relative to the consumer's tile start
  double acc[12] = {};
  int n = 0;
  for (int t = 2; t < T && t < 64; ++t, ++n)
    for (int e = 1; e < 11; ++e) acc[e] += (double)(long long)(h[t][e] - h[t][0]) / 100.0;
  printf("column-split sweep, workgroup 0, mean over t (us from the consumer's tile start): "
         "published %.2f computed %.2f stored %.2f polled %.2f exchanged %.2f mid %.2f | producer z start %.2f after mid %.2f tile end %.2f\n",
         acc[3] / n, acc[1] / n, acc[2] / n, acc[4] / n, acc[5] / n, acc[6] / n, acc[8] / n, acc[9] / n, acc[10] / n);
  double per_t = 0;
  for (int t = 2; t < T - 1 && t < 63; ++t) per_t += (double)(long long)(h[t + 1][0] - h[t][0]) / 100.0;
  printf("  consumer tile start to next tile start: %.2f us per t\n", per_t / (T - 3));
}
#endif

}  // namespace admm

#ifdef SR_TIMING
extern "C" void sr_timing_dump(int nblk) {
  unsigned long long h[2048][2];
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(admm::g_sr_wait), sizeof(h));
  double pw = 0, cw = 0, tot = 0, cc = 0, cs = 0, lw = 0;
  for (int b = 0; b < nblk; ++b) {
    pw += h[b][0]; tot += h[b][1]; cw += h[1024 + b][0]; cc += h[1024 + b][1]; cs += h[1536 + b][0]; lw += h[1536 + b][1];
  }
  printf("sweep rows timing: total %.0f cyc/WG, producer waits %.1f%%, consumer waits %.1f%%, "
         "consumer load+compute %.1f%% (load wait %.1f%%), consumer store issue %.1f%%\n", tot / nblk,
         100.0 * pw / tot, 100.0 * cw / tot, 100.0 * cc / tot, 100.0 * lw / tot, 100.0 * cs / tot);
}
#endif
