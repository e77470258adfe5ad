// admm_kernels.hip -- gfx950 kernels of the ADMM-LSTM update step.
//
// Reference semantics (Frederick2309/ADMM-LSTM):
//   time step / LSTM forward ........ blocks/lstm.py:65-88, admm.py:345-386, 388-457, 504-539
//   weight-stage residual + gradient  admm.py:302-314
//   line-search trials / selection .. admm.py:316-343
//   output weight wy ................ admm.py:246-280, admm.no_dual_y.py:226-249
//   h_T search, a, duals at T ....... admm.py:459-502, 532-546, admm.no_dual_y.py:414-456
// Layouts: gates/duals [B][T+1][H] (the reference's), caches [4][B*T][H] (row = b*T + t-1).
#include "admm_dev.hpp"
#include "admm_kernels.hpp"

namespace admm {

namespace {

inline int cdiv64(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// ============================================================================ time step
// Tile: 128 rows (samples) x 128 columns = 4 gates x 32 hidden units; each wave owns 32
// rows x all 4 gates, so gate q's pre-activation of (b, j) sits in the same lane for every
// q and the element-wise ADMM updates run straight out of the accumulators.
constexpr int TS_BM = 128, TS_BN = 128, TS_WM = 32, TS_WN = 128;
using TSShape = TileShape<TS_BM, TS_BN, TS_WM, TS_WN>;

struct StepSrc {
  const float* x; int64_t x_stride;  // x_t rows
  const float* h; int64_t h_stride;  // h_{t-1} rows
  int64_t B; int D, H;
  Weights w; int j0;
  static constexpr bool A_M_FAST = false;
  __device__ float a(int64_t m, int64_t k) const {
    if (m >= B) return 0.f;
    return k < D ? x[m * x_stride + k] : h[m * h_stride + (k - D)];
  }
  __device__ float b(int64_t k, int64_t n) const {
    const int q = (int)(n >> 5), j = j0 + (int)(n & 31);
    if (j >= H) return 0.f;
    return k < D ? w.wx[q][k * H + j] : w.wh[q][(k - D) * H + j];
  }
};

__global__ __launch_bounds__(kThreads) void k_forward_t(Geom g, int t, Weights w, ForwardT a) {
  __shared__ float smem[TSShape::LDS_FLOATS];
  const int64_t m0 = (int64_t)blockIdx.x * TS_BM;
  const int j0 = blockIdx.y * 32;
  StepSrc src{a.x + (int64_t)(t - 1) * g.D, (int64_t)g.T * g.D, a.hprev, a.hprev_stride, g.B, g.D, g.H, w, j0};
  f32x16 acc[1][4];
  zero_acc(acc);
  gemm_tile<TS_BM, TS_BN, TS_WM, TS_WN>(src, m0, 0, 0, g.D + g.H, acc, smem);
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

// One ADMM time step t (admm.py:72-76): i, f, g, o (admm.py:353-386), c (388-436),
// h for t < T (455-457), dual ascent for i, f, g, o, c (504-530).  h_T, a and the
// duals of h at T are finished by the h_T kernels below.
__global__ __launch_bounds__(kThreads) void k_sweep_t(Geom g, int t, Weights w, Hyper hp, SweepT a) {
  __shared__ float smem[TSShape::LDS_FLOATS];
  const int64_t m0 = (int64_t)blockIdx.x * TS_BM;
  const int j0 = blockIdx.y * 32;
  const int64_t rs = (int64_t)g.TP() * g.H;  // row stride of a [B,T+1,H] plane
  StepSrc src{a.x + (int64_t)(t - 1) * g.D, (int64_t)g.T * g.D, a.S.p[5] + (int64_t)(t - 1) * g.H, rs,
              g.B, g.D, g.H, w, j0};
  f32x16 acc[1][4];
  zero_acc(acc);
  gemm_tile<TS_BM, TS_BN, TS_WM, TS_WN>(src, m0, 0, 0, g.D + g.H, acc, smem);
  const int lane = threadIdx.x & 63, wm0 = (threadIdx.x >> 6) * TS_WM;
  const int j = j0 + (lane & 31);
  if (j >= g.H) return;
  const int64_t BT = g.BT();
  const float ri = hp.rho[0], rf = hp.rho[1], rg = hp.rho[2], ro = hp.rho[3], rc = hp.rho[4], rh = hp.rho[5];
  const bool last = (t == g.T);
  float *Si = a.S.p[0], *Sf = a.S.p[1], *Sg = a.S.p[2], *So = a.S.p[3], *Sc = a.S.p[4], *Sh = a.S.p[5];
  float *Li = a.L.p[0], *Lf = a.L.p[1], *Lg = a.L.p[2], *Lo = a.L.p[3], *Lc = a.L.p[4], *Lh = a.L.p[5];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t b = m0 + wm0 + acc_row(r, lane);
    if (b >= g.B) continue;
    const int64_t ot = b * rs + (int64_t)t * g.H + j;
    const int64_t op = ot - g.H;
    const float zi = acc[0][0][r], zf = acc[0][1][r], zg = acc[0][2][r], zo = acc[0][3][r];
    const float ai = sigm(zi), af = sigm(zf), ag = tanhf(zg), ao = sigm(zo);
    const float f0 = Sf[ot], g0 = Sg[ot], c0 = Sc[ot], h0 = Sh[ot];
    const float cp = Sc[op];
    const float li = Li[ot], lf = Lf[ot], lg = Lg[ot], lo = Lo[ot], lc = Lc[ot], lh = Lh[ot];
    // admm.py:384-386 with (p1,p2,p3) of :360-375 and (var2, rho2, lam2) of :376-383
    const float i1 = -((li - ri * ai) + (rc * (f0 * cp - c0) - lc) * g0) / (ri + rc * g0 * g0);
    const float f1 = -((lf - rf * af) + (rc * (g0 * i1 - c0) - lc) * cp) / (rf + rc * cp * cp);
    const float g1 = -((lg - rg * ag) + (rc * (f1 * cp - c0) - lc) * i1) / (rg + rc * i1 * i1);
    const float tc0 = tanhf(c0);
    const float o1 = -((lo - ro * ao) + (rh * (0.f - h0) - lh) * tc0) / (ro + rh * tc0 * tc0);
    // admm.py:388-436: autograd gradient of .5||tanh(c) o - (h + lam_h/rho_h)||^2, theta* = 0.5
    const float div_h = lh / rh, div_c = lc / rc;
    const float v = tc0 * o1 - (h0 + div_h);
    const float gc = (v * o1) * (1.f - tc0 * tc0);
    const float A = (div_c - f1 * cp) - i1 * g1;
    const float c1 = (0.5f * c0 - gc - rc * A) / (rc + 0.5f);
    Si[ot] = i1; Sf[ot] = f1; Sg[ot] = g1; So[ot] = o1; Sc[ot] = c1;
    if (!last) Sh[ot] = (rh * o1 * tanhf(c1) - lh) / rh;  // admm.py:455-457
    // admm.py:512-530
    Li[ot] = li + ri * (i1 - ai);
    Lf[ot] = lf + rf * (f1 - af);
    Lg[ot] = lg + rg * (g1 - ag);
    Lo[ot] = lo + ro * (o1 - ao);
    Lc[ot] = lc + rc * (c1 - (f1 * cp + i1 * g1));
    const int64_t e = (b * g.T + (t - 1)) * g.H + j;
    a.zc[e] = zi; a.zc[BT * g.H + e] = zf; a.zc[2 * BT * g.H + e] = zg; a.zc[3 * BT * g.H + e] = zo;
  }
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

struct AllRowSrc {  // z cache recompute: A = [X | Hprev] (K = D+H), B = [Wx; Wh]
  const float* x; const float* Sh; int64_t BT; int T, D, H; Weights w; int j0;
  static constexpr bool A_M_FAST = false;
  __device__ float a(int64_t m, int64_t k) const {
    if (m >= BT) return 0.f;
    return k < D ? x[m * D + k] : Sh[(m + m / T) * H + (k - D)];
  }
  __device__ float b(int64_t k, int64_t n) const {
    const int q = (int)(n >> 5), j = j0 + (int)(n & 31);
    if (j >= H) return 0.f;
    return k < D ? w.wx[q][k * H + j] : w.wh[q][(k - D) * H + j];
  }
};

__global__ __launch_bounds__(kThreads) void k_zgemm(Geom g, Weights w, const float* x, const float* Sh,
                                                      float* zc) {
  __shared__ float smem[TSShape::LDS_FLOATS];
  const int64_t m0 = (int64_t)blockIdx.x * TS_BM;
  const int j0 = blockIdx.y * 32;
  const int64_t BT = g.BT();
  AllRowSrc src{x, Sh, BT, g.T, g.D, g.H, w, j0};
  f32x16 acc[1][4];
  zero_acc(acc);
  gemm_tile<TS_BM, TS_BN, TS_WM, TS_WN>(src, m0, 0, 0, g.D + g.H, acc, smem);
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

// admm.py:302-314 (residual part) for the 4 gates; also tgt = lam/rho + S (reused by the
// trials) and f(W) partial sums (admm.py:316-325 at beta = W).
__global__ __launch_bounds__(kThreads) void k_resid(Geom g, Hyper hp, ResidArgs a) {
  __shared__ double red[4];
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
  float fw = 0.f;
  if (ix.rr < ix.rpb) {
    for (int64_t row = (int64_t)blockIdx.x * ix.rpb + ix.rr; row < BT; row += (int64_t)gridDim.x * ix.rpb) {
      const int64_t b = row / g.T;
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
        const float d = phi - tg;
        Rq[e] = d * dphi;
        fw += d * d;
      }
    }
  }
  const double tot = block_sum((double)fw, red);
  if (threadIdx.x == 0) a.fw_part[(int64_t)q * a.nblk + blockIdx.x] = tot;
}

// G_q = A^T R_q split over rows: 64 (weight rows) x 128 (hidden units) tiles per gate.
constexpr int AT_BM = 64, AT_BN = 128, AT_WM = 32, AT_WN = 64;
using ATShape = TileShape<AT_BM, AT_BN, AT_WM, AT_WN>;

struct AtRSrc {
  const float* x; const float* Sh; const float* Rq; int side; int T, D, H, Kd;
  static constexpr bool A_M_FAST = true;
  __device__ float a(int64_t m, int64_t row) const {  // A^T[m][row]
    if (m >= Kd) return 0.f;
    return side == 0 ? x[row * D + m] : Sh[(row + row / T) * H + m];
  }
  __device__ float b(int64_t row, int64_t j) const { return j < H ? Rq[row * H + j] : 0.f; }
};

__global__ __launch_bounds__(kThreads) void k_atr(Geom g, int side, const float* x, const float* Sh,
                                                    const float* R, float* slab, int nsplit) {
  __shared__ float smem[ATShape::LDS_FLOATS];
  const int Kd = side == 0 ? g.D : g.H;
  const int q = blockIdx.z / nsplit, sp = blockIdx.z % nsplit;
  const int64_t BT = g.BT();
  const int64_t per = (BT + nsplit - 1) / nsplit;
  const int64_t r0 = sp * per, r1 = (r0 + per < BT) ? r0 + per : BT;
  const int m0 = blockIdx.x * AT_BM, n0 = blockIdx.y * AT_BN;
  AtRSrc src{x, Sh, R + (int64_t)q * BT * g.H, side, g.T, g.D, g.H, Kd};
  f32x16 acc[1][2];
  zero_acc(acc);
  if (r0 < r1) gemm_tile<AT_BM, AT_BN, AT_WM, AT_WN>(src, m0, n0, r0, r1, acc, smem);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm0 = (wave / ATShape::WAVES_N) * AT_WM, wn0 = (wave % ATShape::WAVES_N) * AT_WN;
  float* out = slab + ((int64_t)sp * 4 + q) * Kd * g.H;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int j = n0 + wn0 + ni * 32 + (lane & 31);
    if (j >= g.H) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm0 + acc_row(r, lane);
      if (m < Kd) out[(int64_t)m * g.H + j] = acc[0][ni][r];
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_reduce_g(int Kd, int H, Hyper hp, const float* slab, int nsplit,
                                                         float* G) {
  const int64_t per_q = (int64_t)Kd * H;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= 4 * per_q) return;
  const int q = (int)(i / per_q);
  double s = 0.0;
  for (int sp = 0; sp < nsplit; ++sp) s += (double)slab[(int64_t)sp * 4 * per_q + i];
  G[i] = (float)s * hp.rho[q];  // (sum_t A_t^T R_t) * rho (admm.py:312)
}

struct QSrc {
  const float* x; const float* Sh; const float* G; int64_t BT; int side, T, D, H, Kd, j0;
  static constexpr bool A_M_FAST = false;
  __device__ float a(int64_t row, int64_t k) const {
    if (row >= BT || k >= Kd) return 0.f;
    return side == 0 ? x[row * D + k] : Sh[(row + row / T) * H + k];
  }
  __device__ float b(int64_t k, int64_t n) const {
    const int q = (int)(n >> 5), j = j0 + (int)(n & 31);
    if (j >= H || k >= Kd) return 0.f;
    return G[((int64_t)q * Kd + k) * H + j];
  }
};

// Q_q = A G_q: the trial direction, so that z(W + G/theta) = z(W) + Q / theta exactly.
__global__ __launch_bounds__(kThreads) void k_qgemm(Geom g, int side, const float* x, const float* Sh,
                                                      const float* G, float* Q) {
  __shared__ float smem[TSShape::LDS_FLOATS];
  const int Kd = side == 0 ? g.D : g.H;
  const int64_t m0 = (int64_t)blockIdx.x * TS_BM;
  const int j0 = blockIdx.y * 32;
  const int64_t BT = g.BT();
  QSrc src{x, Sh, G, BT, side, g.T, g.D, g.H, Kd, j0};
  f32x16 acc[1][4];
  zero_acc(acc);
  gemm_tile<TS_BM, TS_BN, TS_WM, TS_WN>(src, m0, 0, 0, Kd, acc, smem);
  const int lane = threadIdx.x & 63, wm0 = (threadIdx.x >> 6) * TS_WM;
  const int j = j0 + (lane & 31);
  if (j >= g.H) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = m0 + wm0 + acc_row(r, lane);
    if (row >= BT) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) Q[((int64_t)q * BT + row) * g.H + j] = acc[0][q][r];
  }
}

// Trial pass: for k in [pass*J, pass*J + J) accumulate
//   f(W + G/2^k) - f(W) = 0.5 rho sum_e [ (d0 + D)^2 - d0^2 ],  D = phi(z + Q 2^-k) - phi(z),
// with D evaluated without cancellation (admm_dev.hpp, trial_delta).  The reference
// evaluates f(beta) and f(W) separately in fp32 and compares them (admm.py:327-334); see
// DESIGN.md.  Elements are streamed as float4 when H % 4 == 0.
template <bool TANH>
__device__ __forceinline__ void trial_accumulate(float z, float tg, float qv, float scale0, float (&acc)[kTrialJ]) {
  const TrialElem e = TANH ? trial_elem_tanh(z, tg) : trial_elem_sigmoid(z, tg);
  float sc = scale0;
#pragma unroll
  for (int k = 0; k < kTrialJ; ++k) {
    const float D = trial_delta<TANH>(e, qv * sc);   // sc = 2^-(kbase+k): exact scaling
    acc[k] += D * (2.f * e.d0 + D);
    sc *= 0.5f;
  }
}

template <bool TANH, int VEC>
__device__ __forceinline__ void trial_loop(int64_t n, const float* zq, const float* tq, const float* Qq, float scale0,
                                           float (&acc)[kTrialJ]) {
  const int64_t nv = n / VEC;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t v = (int64_t)blockIdx.x * kThreads + threadIdx.x; v < nv; v += stride) {
    if (VEC == 4) {
      const float4 z4 = reinterpret_cast<const float4*>(zq)[v];
      const float4 t4 = reinterpret_cast<const float4*>(tq)[v];
      const float4 q4 = reinterpret_cast<const float4*>(Qq)[v];
      trial_accumulate<TANH>(z4.x, t4.x, q4.x, scale0, acc);
      trial_accumulate<TANH>(z4.y, t4.y, q4.y, scale0, acc);
      trial_accumulate<TANH>(z4.z, t4.z, q4.z, scale0, acc);
      trial_accumulate<TANH>(z4.w, t4.w, q4.w, scale0, acc);
    } else {
      trial_accumulate<TANH>(zq[v], tq[v], Qq[v], scale0, acc);
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_trial(Geom g, int pass, const float* zc, const float* tgt,
                                                      const float* Q, const int* found, double* part, int nblk) {
  __shared__ double red[4][kTrialJ];
  const int q = blockIdx.y;
  if (found[q]) return;
  const int64_t n = g.BT() * g.H;
  const float* zq = zc + (int64_t)q * n;
  const float* tq = tgt + (int64_t)q * n;
  const float* Qq = Q + (int64_t)q * n;
  float acc[kTrialJ];
#pragma unroll
  for (int k = 0; k < kTrialJ; ++k) acc[k] = 0.f;
  const float scale0 = ldexpf(1.f, -pass * kTrialJ);
  const bool vec = (g.H % 4) == 0;
  if (q == 2) {
    if (vec) trial_loop<true, 4>(n, zq, tq, Qq, scale0, acc);
    else trial_loop<true, 1>(n, zq, tq, Qq, scale0, acc);
  } else {
    if (vec) trial_loop<false, 4>(n, zq, tq, Qq, scale0, acc);
    else trial_loop<false, 1>(n, zq, tq, Qq, scale0, acc);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kTrialJ; ++k) {
    const float s = wave_sum(acc[k]);
    if (lane == 0) red[w][k] = (double)s;
  }
  __syncthreads();
  if (threadIdx.x < kTrialJ) {
    const int k = threadIdx.x;
    part[((int64_t)q * kTrialJ + k) * nblk + blockIdx.x] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
  }
}

// Test hook: the same per-element arithmetic on caller data (one gate), partial sums per block.
__global__ __launch_bounds__(kThreads) void k_trial_debug(int64_t n, int tanh_gate, int kbase, const float* z,
                                                            const float* tgt, const float* qv, double* part) {
  __shared__ double red[4][kTrialJ];
  float acc[kTrialJ];
#pragma unroll
  for (int k = 0; k < kTrialJ; ++k) acc[k] = 0.f;
  const float scale0 = ldexpf(1.f, -kbase);
  if (tanh_gate) trial_loop<true, 1>(n, z, tgt, qv, scale0, acc);
  else trial_loop<false, 1>(n, z, tgt, qv, scale0, acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kTrialJ; ++k) {
    const float s = wave_sum(acc[k]);
    if (lane == 0) red[w][k] = (double)s;
  }
  __syncthreads();
  if (threadIdx.x < kTrialJ) {
    const int k = threadIdx.x;
    part[(int64_t)blockIdx.x * kTrialJ + k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
  }
}

__global__ __launch_bounds__(kThreads) void k_trial_reduce(int pass, const double* part, int nblk,
                                                             const double* fw_part, int fw_nblk, const int* found,
                                                             double* sums) {
  __shared__ double red[4];
  const int q = blockIdx.x;
  if (found[q]) return;
  for (int k = 0; k <= kTrialJ; ++k) {
    double s = 0.0;
    if (k < kTrialJ) {
      const double* p = part + ((int64_t)q * kTrialJ + k) * nblk;
      for (int i = threadIdx.x; i < nblk; i += kThreads) s += p[i];
    } else {
      const double* p = fw_part + (int64_t)q * fw_nblk;
      for (int i = threadIdx.x; i < fw_nblk; i += kThreads) s += p[i];
    }
    const double tot = block_sum(s, red);
    if (threadIdx.x == 0) sums[q * (kTrialJ + 1) + k] = tot;
  }
}

// First k of this window with f(W + G/2^k) <= est_k (admm.py:331-336); then
// W <- (0.5 rho T theta* W - G) / (beta + 0.5 rho theta* T), theta* = 2^k / 2 (admm.py:338-343).
__global__ __launch_bounds__(kThreads) void k_select(Geom g, Hyper hp, SelectArgs a) {
  __shared__ double red[4];
  __shared__ int pick_s;
  const int q = blockIdx.x;
  if (a.found[q]) return;
  const int Kd = a.side == 0 ? g.D : g.H;
  const int64_t nW = (int64_t)Kd * g.H;
  const float* Gq = a.G + (int64_t)q * nW;
  double gs = 0.0;
  for (int64_t i = threadIdx.x; i < nW; i += kThreads) gs += (double)Gq[i] * (double)Gq[i];
  const double gsq = block_sum(gs, red);
  const float rho = hp.rho[q];
  if (threadIdx.x == 0) {
    const double* sm = a.sums + q * (kTrialJ + 1);
    int pick = -1;
    for (int k = 0; k < kTrialJ; ++k) {
      const int kk = a.pass * kTrialJ + k;
      const double lhs = 0.5 * (double)rho * sm[k];
      const double rhs = (1.0 + 0.5 * g.T) * gsq * ldexp(1.0, -kk);
      if (!isfinite(lhs)) atomicAdd(&a.stats->nonfinite, 1);
      if (lhs > rhs) continue;
      pick = kk;
      break;
    }
    if (pick < 0 && a.pass == a.last_pass) {
      pick = (a.last_pass + 1) * kTrialJ;
      atomicAdd(&a.stats->unresolved, 1);
    }
    if (pick >= 0) {
      const int slot = 2 * q + a.side;
      a.stats->k[slot] = pick;
      a.stats->f_w[slot] = 0.5 * (double)rho * sm[kTrialJ];
      a.stats->grad_sq[slot] = gsq;
      a.stats->passes[a.side] = a.pass + 1;
      a.found[q] = 1;
    }
    pick_s = pick;
  }
  __syncthreads();
  const int pick = pick_s;
  if (pick < 0) return;
  const float theta = ldexpf(1.f, pick - 1);
  const float beta = a.side == 0 ? hp.beta_x[q] : hp.beta_h[q];
  const float c1 = ((0.5f * rho) * (float)g.T) * theta;
  const float den = beta + ((0.5f * rho) * theta) * (float)g.T;
  float* W = a.W[q];
  for (int64_t i = threadIdx.x; i < nW; i += kThreads) {
    const float w0 = W[i];
    const float w1 = (c1 * w0 - Gq[i]) / den;
    W[i] = w1;
    if (a.dW) a.dW[(int64_t)q * nW + i] = w1 - w0;
  }
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
  float s = 0.f;
  for (int64_t b = b0; b < b1; ++b) s += Sh[b * rs + (int64_t)g.T * g.H + j] * U[b * g.O + o];
  slab[blockIdx.y * nHO + i] = s;
}

__global__ __launch_bounds__(kThreads) void k_wy_reduce(int64_t nHO, const float* slab, int nsplit, float* Gy) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nHO) return;
  double s = 0.0;
  for (int sp = 0; sp < nsplit; ++sp) s += (double)slab[(int64_t)sp * nHO + i];
  Gy[i] = (float)s;
}

__global__ __launch_bounds__(kThreads) void k_wy_apply(int64_t nHO, Hyper hp, const float* Gy, float* wy) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nHO) return;
  if (hp.variant == 0) {
    const float th = 0.5f;  // theta = 1, dead search (admm.py:262-277) -> 1/2
    wy[i] = (th * wy[i] - Gy[i]) / (th + hp.beta_y);
  } else {
    const float th = 0.005f;  // theta = 0.01 -> 0.005 (admm.no_dual_y.py:231-249)
    wy[i] = (th * wy[i] - Gy[i]) / (th + 2.f * hp.beta_y);
  }
}

// ============================================================================ h_T
// Per row: u = h wy - a - s,  g = gamma u wy^T (admm: gamma = rho_y via autograd; no_dual_y:
// gamma = rho_h), candidates beta(theta) for theta = 0.1 * 2^c.
constexpr int kMaxO = 8;

struct HTRow {
  float u[kMaxO];
};

__device__ __forceinline__ void ht_row_u(const Geom& g, const float* h, const float* a_row, const float* s_row,
                                         const float* wy, HTRow& r) {
  const int lane = threadIdx.x & 63;
  for (int o = 0; o < g.O; ++o) {
    float s = 0.f;
    for (int j = lane; j < g.H; j += kWave) s += h[j] * wy[(int64_t)j * g.O + o];
    s = wave_sum(s);
    float u = s - a_row[o];
    if (s_row) u = u - s_row[o];
    r.u[o] = u;
  }
}

__device__ __forceinline__ float ht_grad(const Geom& g, const Hyper& hp, const HTRow& r, const float* wy, int j) {
  float s = 0.f;
  if (hp.variant == 0) {
    const float ry = hp.rho[6];
    for (int o = 0; o < g.O; ++o) s += (ry * r.u[o]) * wy[(int64_t)j * g.O + o];
    return s;
  }
  for (int o = 0; o < g.O; ++o) s += r.u[o] * wy[(int64_t)j * g.O + o];
  return hp.rho[5] * s;
}

__global__ __launch_bounds__(kThreads) void k_ht_partial(Geom g, Hyper hp, Planes6 S, Planes6 L, const float* a,
                                                           const float* Ly, const float* wy, double* part) {
  __shared__ double red[4];
  __shared__ double accs[4][kHTSums];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float ry = hp.rho[6], rh = hp.rho[5];
  const bool nd = hp.variant == 1;
  const bool shift = !nd && hp.with_dual_y;
  const int64_t rs = (int64_t)g.TP() * g.H, tofs = (int64_t)g.T * g.H;
  double acc[kHTSums];
  for (int i = 0; i < kHTSums; ++i) acc[i] = 0.0;
  float sbuf[kMaxO];
  for (int64_t b = (int64_t)blockIdx.x * 4 + w; b < g.B; b += (int64_t)gridDim.x * 4) {
    const float* h = S.p[5] + b * rs + tofs;
    const float* o_ = S.p[3] + b * rs + tofs;
    const float* c_ = S.p[4] + b * rs + tofs;
    const float* lh = L.p[5] + b * rs + tofs;
    if (shift)
      for (int o = 0; o < g.O; ++o) sbuf[o] = Ly[b * g.O + o] / ry;
    HTRow r;
    ht_row_u(g, h, a + b * g.O, shift ? sbuf : nullptr, wy, r);
    float fh = 0.f;
    for (int o = 0; o < g.O; ++o) fh += r.u[o] * r.u[o];
    float v[kHTCand][kMaxO], ip[kHTCand], nq[kHTCand];
    for (int c = 0; c < kHTCand; ++c) {
      ip[c] = 0.f; nq[c] = 0.f;
      for (int o = 0; o < g.O; ++o) v[c][o] = 0.f;
    }
    for (int j = lane; j < g.H; j += kWave) {
      const float gj = ht_grad(g, hp, r, wy, j);
      const float hj = h[j], pj = rh * o_[j] * tanhf(c_[j]) - lh[j];
      for (int c = 0; c < kHTCand; ++c) {
        const float th = ldexpf(0.1f, c);
        const float bj = nd ? gj / th : (th * hj + pj - gj) / (th + rh);
        const float dj = bj - hj;
        ip[c] += gj * dj;
        nq[c] += dj * dj;
        for (int o = 0; o < g.O; ++o) v[c][o] += bj * wy[(int64_t)j * g.O + o];
      }
    }
    // wave-reduce and accumulate (lane 0 holds the row's values)
    acc[0] += (double)fh;  // identical on every lane
    for (int c = 0; c < kHTCand; ++c) {
      float fb = 0.f;
      for (int o = 0; o < g.O; ++o) {
        float vv = wave_sum(v[c][o]) - a[b * g.O + o];
        if (shift) vv = vv - sbuf[o];
        fb += vv * vv;
      }
      acc[1 + 3 * c] += (double)fb;
      acc[2 + 3 * c] += (double)wave_sum(ip[c]);
      acc[3 + 3 * c] += (double)wave_sum(nq[c]);
    }
  }
  if (lane == 0)
    for (int i = 0; i < kHTSums; ++i) accs[w][i] = acc[i];
  __syncthreads();
  if (threadIdx.x < kHTSums) {
    const int i = threadIdx.x;
    part[(int64_t)blockIdx.x * kHTSums + i] = (accs[0][i] + accs[1][i]) + (accs[2][i] + accs[3][i]);
  }
  (void)red;
}

__global__ __launch_bounds__(kThreads) void k_ht_reduce(const double* part, int nblk, double* sums) {
  __shared__ double red[4];
  for (int i = 0; i < kHTSums; ++i) {
    double s = 0.0;
    for (int b = threadIdx.x; b < nblk; b += kThreads) s += part[(int64_t)b * kHTSums + i];
    const double tot = block_sum(s, red);
    if (threadIdx.x == 0) sums[i] = tot;
  }
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
// dual y (541-546, admm variant with with_dual_y).
__global__ __launch_bounds__(kThreads) void k_ht_apply(Geom g, Hyper hp, Planes6 S, Planes6 L, float* a, float* Ly,
                                                         const float* y, const float* wy, const double* sums,
                                                         DevStats* stats) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float ry = hp.rho[6], rh = hp.rho[5];
  const bool nd = hp.variant == 1;
  const bool shift = !nd && hp.with_dual_y;
  const float th = ht_theta_star(hp, sums);
  if (blockIdx.x == 0 && threadIdx.x == 0) stats->theta_h = th;
  const int64_t rs = (int64_t)g.TP() * g.H, tofs = (int64_t)g.T * g.H;
  const float Bry = (float)g.Bg * ry;
  float sbuf[kMaxO];
  for (int64_t b = (int64_t)blockIdx.x * 4 + w; b < g.B; b += (int64_t)gridDim.x * 4) {
    float* h = S.p[5] + b * rs + tofs;
    const float* o_ = S.p[3] + b * rs + tofs;
    const float* c_ = S.p[4] + b * rs + tofs;
    float* lh = L.p[5] + b * rs + tofs;
    if (shift)
      for (int o = 0; o < g.O; ++o) sbuf[o] = Ly[b * g.O + o] / ry;
    HTRow r;
    ht_row_u(g, h, a + b * g.O, shift ? sbuf : nullptr, wy, r);
    float hw[kMaxO];
    for (int o = 0; o < g.O; ++o) hw[o] = 0.f;
    for (int j = lane; j < g.H; j += kWave) {
      const float gj = ht_grad(g, hp, r, wy, j);
      const float tc = tanhf(c_[j]);
      const float hn = (th * h[j] + rh * o_[j] * tc - lh[j] - gj) / (th + rh);
      h[j] = hn;
      lh[j] = lh[j] + rh * (hn - o_[j] * tc);
      for (int o = 0; o < g.O; ++o) hw[o] += hn * wy[(int64_t)j * g.O + o];
    }
    for (int o = 0; o < g.O; ++o) {
      const float hwo = wave_sum(hw[o]);
      if (lane == 0) {
        const int64_t i = b * g.O + o;
        float an;
        if (!nd) {
          const float corr = shift ? (float)g.Bg * Ly[i] : 0.f;
          an = (2.f * y[i] + Bry * hwo - corr) / (2.f + Bry);
        } else {
          an = (Bry * hwo + 2.f * y[i]) / (2.f + Bry);
        }
        a[i] = an;
        if (shift) Ly[i] = Ly[i] + ry * (an - hwo);
      }
    }
  }
}

}  // namespace

// ============================================================================ launchers

void launch_forward_t(const Geom& g, int t, const Weights& w, const ForwardT& a, hipStream_t s) {
  dim3 grid(cdiv64(g.B, TS_BM), cdiv64(g.H, 32));
  k_forward_t<<<grid, kThreads, 0, s>>>(g, t, w, a);
}

void launch_sweep_t(const Geom& g, int t, const Weights& w, const Hyper& hp, const SweepT& a, hipStream_t s) {
  dim3 grid(cdiv64(g.B, TS_BM), cdiv64(g.H, 32));
  k_sweep_t<<<grid, kThreads, 0, s>>>(g, t, w, hp, a);
}

void launch_rowdot(int64_t B, int H, int O, const float* h, int64_t hs, const float* wy, float* out, hipStream_t s) {
  int nb = cdiv64(B, 4);
  if (nb > 2048) nb = 2048;
  k_rowdot<<<nb, kThreads, 0, s>>>(B, H, O, h, hs, wy, out);
}

void launch_zgemm(const Geom& g, const Weights& w, const float* x, const float* Sh, float* zc, hipStream_t s) {
  dim3 grid(cdiv64(g.BT(), TS_BM), cdiv64(g.H, 32));
  k_zgemm<<<grid, kThreads, 0, s>>>(g, w, x, Sh, zc);
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

int atr_splits(const Geom& g, int side) {
  const int Kd = side == 0 ? g.D : g.H;
  const int tiles = cdiv64(Kd, AT_BM) * cdiv64(g.H, AT_BN) * 4;
  int ns = 1024 / tiles;
  const int64_t max_by_rows = g.BT() / 256;  // keep >= 256 rows per split
  if (ns > max_by_rows) ns = (int)max_by_rows;
  if (ns > 256) ns = 256;
  return ns < 1 ? 1 : ns;
}

void launch_atr(const Geom& g, int side, const float* x, const float* Sh, const float* R, float* slab, int nsplit,
                hipStream_t s) {
  const int Kd = side == 0 ? g.D : g.H;
  dim3 grid(cdiv64(Kd, AT_BM), cdiv64(g.H, AT_BN), 4 * nsplit);
  k_atr<<<grid, kThreads, 0, s>>>(g, side, x, Sh, R, slab, nsplit);
}

void launch_reduce_g(const Geom& g, int side, const Hyper& hp, const float* slab, int nsplit, float* G,
                     hipStream_t s) {
  const int Kd = side == 0 ? g.D : g.H;
  const int64_t n = 4LL * Kd * g.H;
  k_reduce_g<<<cdiv64(n, kThreads), kThreads, 0, s>>>(Kd, g.H, hp, slab, nsplit, G);
}

void launch_qgemm(const Geom& g, int side, const float* x, const float* Sh, const float* G, float* Q,
                  hipStream_t s) {
  dim3 grid(cdiv64(g.BT(), TS_BM), cdiv64(g.H, 32));
  k_qgemm<<<grid, kThreads, 0, s>>>(g, side, x, Sh, G, Q);
}

int trial_blocks(const Geom& g) {
  int nb = cdiv64(g.BT() * g.H, kThreads * 8);
  return nb > 2048 ? 2048 : (nb < 1 ? 1 : nb);
}

void launch_trial(const Geom& g, int pass, const float* zc, const float* tgt, const float* Q, const int* found,
                  double* part, int nblk, hipStream_t s) {
  dim3 grid(nblk, 4);
  k_trial<<<grid, kThreads, 0, s>>>(g, pass, zc, tgt, Q, found, part, nblk);
}

void launch_trial_debug(int64_t n, int tanh_gate, int kbase, const float* z, const float* tgt, const float* q,
                        double* part, int nblk, hipStream_t s) {
  k_trial_debug<<<nblk, kThreads, 0, s>>>(n, tanh_gate, kbase, z, tgt, q, part);
}

void launch_trial_reduce(const Geom& g, int pass, const double* part, int nblk, const double* fw_part, int fw_nblk,
                         const int* found, double* sums, hipStream_t s) {
  (void)g;
  k_trial_reduce<<<4, kThreads, 0, s>>>(pass, part, nblk, fw_part, fw_nblk, found, sums);
}

void launch_select(const Geom& g, const Hyper& hp, const SelectArgs& a, hipStream_t s) {
  k_select<<<4, kThreads, 0, s>>>(g, hp, a);
}

int wy_splits(const Geom& g) {
  int ns = cdiv64(g.B, 256);
  return ns > 256 ? 256 : (ns < 1 ? 1 : ns);
}

void launch_wy_grad(const Geom& g, const Hyper& hp, const float* Sh, const float* a, const float* Ly,
                    const float* wy, float* U, float* slab, int nsplit, hipStream_t s) {
  int nb = cdiv64(g.B, 4);
  if (nb > 2048) nb = 2048;
  k_wy_u<<<nb, kThreads, 0, s>>>(g, hp, Sh, a, Ly, wy, U);
  const int64_t nHO = (int64_t)g.H * g.O;
  dim3 grid(cdiv64(nHO, kThreads), nsplit);
  k_wy_slab<<<grid, kThreads, 0, s>>>(g, Sh, U, slab, nsplit);
}

void launch_wy_reduce(const Geom& g, const float* slab, int nsplit, float* Gy, hipStream_t s) {
  const int64_t nHO = (int64_t)g.H * g.O;
  k_wy_reduce<<<cdiv64(nHO, kThreads), kThreads, 0, s>>>(nHO, slab, nsplit, Gy);
}

void launch_wy_apply(const Geom& g, const Hyper& hp, const float* Gy, float* wy, hipStream_t s) {
  const int64_t nHO = (int64_t)g.H * g.O;
  k_wy_apply<<<cdiv64(nHO, kThreads), kThreads, 0, s>>>(nHO, hp, Gy, wy);
}

int ht_blocks(const Geom& g) {
  int nb = cdiv64(g.B, 4);
  return nb > 1024 ? 1024 : nb;
}

void launch_ht_partial(const Geom& g, const Hyper& hp, const Planes6& S, const Planes6& L, const float* a,
                       const float* Ly, const float* wy, double* part, int nblk, hipStream_t s) {
  k_ht_partial<<<nblk, kThreads, 0, s>>>(g, hp, S, L, a, Ly, wy, part);
}

void launch_ht_reduce(const double* part, int nblk, double* sums, hipStream_t s) {
  k_ht_reduce<<<1, kThreads, 0, s>>>(part, nblk, sums);
}

void launch_ht_apply(const Geom& g, const Hyper& hp, const Planes6& S, const Planes6& L, float* a, float* Ly,
                     const float* y, const float* wy, const double* sums, DevStats* stats, hipStream_t s) {
  k_ht_apply<<<ht_blocks(g), kThreads, 0, s>>>(g, hp, S, L, a, Ly, y, wy, sums, stats);
}

}  // namespace admm
