// admm_split3.hip -- the h-stage GEMMs of the weight update on bf16 matrix cores with
// f32-accurate three-way split operands (admm_dev.hpp split3).
//
//   k_atr3w  slab[sp][q][m][j] = sum_{rows of split sp} Hprev[row][m] * R_q[row][j]
//            the gradient G_q = rho_q Hprev^T R_q of the h side (admm.py:302-312), with the
//            residual R_q = (phi(z) - tgt) phi'(z) formed from the z cache and the target while
//            the tile is staged (R is never materialised);
//   k_qgemm3 Q_q = Hprev G_q, the trial direction of the h-side line search (admm.py:316-336:
//            z(W + G/theta) = z(W) + Q/theta).
//
// fp32 MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate.  Each f32 operand is split
// into three bf16 pieces a = a0 + a1 + a2 (exact to ~2^-27 relative) and the product is the sum
// of the six piece products with i + j <= 2, each exact in the MFMA's f32 accumulator: six
// v_mfma_f32_32x32x16_bf16 (192 cycles) per 16-deep step instead of eight f32 MFMAs (512).
// Operands are split once per workgroup, when they are staged into LDS, and read back as MFMA
// fragments with ds_read_b128.
//
// LDS images: [rows][16 x bf16] per piece, 32 B per row; the two 16-B halves of row r are
// swapped when ((r >> 2) ^ (r >> 3)) & 1.  Fragment reads (32 consecutive rows per half-wave, one
// half) and staging writes (8 consecutive lanes on 8 consecutive rows, one half; or 4 rows x 2
// halves) are then conflict-free under the gfx950 bank rules (MI355X_MICROARCH.md §LDS).
#include <cstdlib>
#include "admm_split3.hpp"

#include <type_traits>

namespace admm {
namespace {

// ------------------------------------------------------------------ G image for k_qgemm3
// gi[(((q * NK + c) * NTT + n) * 3 + p) * 64 + lane] = piece p of G_q[16c + 8(lane>>5) + e][32n + (lane&31)],
// e = 0..7 (the MFMA B fragment), NK = H/16 chunks, NTT = H/32 column tiles.
__global__ __launch_bounds__(kThreads) void k_split_g(int H, const float* __restrict__ G, bf16x8* __restrict__ gi) {
  const int NK = H / 16, NTT = H / 32;
  const int total = 4 * NK * NTT * 64;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < total; i += gridDim.x * kThreads) {
    const int lane = i & 63, n = (i >> 6) % NTT, c = (i / (64 * NTT)) % NK, q = i / (64 * NTT * NK);
    const int j = 32 * n + (lane & 31), k0 = 16 * c + 8 * (lane >> 5);
    f32x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = G[((int64_t)q * H + k0 + e) * H + j];
    bf16x8 p0, p1, p2;
    split3(v, p0, p1, p2);
    const int base = (((q * NK + c) * NTT + n) * 3) * 64 + lane;
    gi[base] = p0;
    gi[base + 64] = p1;
    gi[base + 128] = p2;
  }
}

// ------------------------------------------------------------------ Q = Hprev G
// One 128 x 256 tile of one gate per workgroup (qgemm3_tile).  found != nullptr: gates whose
// line search has already decided are skipped (the later trial passes, when pass 0 ran fused
// in k_qtrial3 and Q was never formed).
// QP = 2: Q is written in the row-quad layout Q[q][row / 4][j][row % 4] of bf16 (BT % 4 == 0):
// registers 4i .. 4i + 3 of a 32x32 accumulator hold four consecutive rows of one column, so each
// lane stores 8 B per quad and column -- a quarter of the store instructions of the row-major layout
// (the epilogue is store-issue bound), and Q only enters the line-search remainder, where its ~2^-9
// relative rounding moves the decision quantity by ~2^-8 (DESIGN.md "trial direction precision").
// QP = 0: row-major f32 (the fallback for BT % 4 != 0).
template <int NP, int QP, int BM>
__global__ __launch_bounds__(2 * BM) void k_qgemm3(Geom g, const float* __restrict__ Sh,
                                                    const bf16x8* __restrict__ gi, float* __restrict__ Q,
                                                    const int* __restrict__ found) {
  __shared__ __attribute__((aligned(16))) char lds[Q3Lds<BM>()];
  const int H = g.H, ncb = H / Q3_BN;
  int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int cb = lid % ncb;
  lid /= ncb;
  const int q = lid % 4;
  if (found && found[q]) return;
  const int64_t m0 = (int64_t)(lid / 4) * BM, BT = g.BT();
  f32x16 acc[2][4];
  qgemm3_tile<NP, BM>(g, Sh, gi, q, cb, m0, lds, acc);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wr = wave >> 1, wc = wave & 1, c32 = lane & 31;
  float* Qq = Q + (int64_t)q * BT * H + Q3_BN * cb + wc * 128 + c32;
  if constexpr (QP == 2) {
    bf16x4* Qp = reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(Q) + (int64_t)q * BT * H) + Q3_BN * cb + wc * 128 + c32;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; r += 4) {
        const int64_t row = m0 + wr * 64 + mi * 32 + acc_row(r, lane);   // a multiple of 4
        if (row >= BT) continue;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const f32x4 v = f32x4{acc[mi][ni][r], acc[mi][ni][r + 1], acc[mi][ni][r + 2], acc[mi][ni][r + 3]};
          __builtin_nontemporal_store(__builtin_convertvector(v, bf16x4), Qp + (row >> 2) * H + ni * 32);
        }
      }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = m0 + wr * 64 + mi * 32 + acc_row(r, lane);
      if (row >= BT) continue;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        if (!(S3_ABL & 16) || acc[mi][ni][r] == 12345.f) st_nt(Qq + row * H + ni * 32, acc[mi][ni][r]);
    }
}

// ------------------------------------------------------------------ Q = Hprev G, G resident in LDS
// H = 256 with a one-piece G and bf16 row quads (NP = 1, QP = 2, the default trial direction).
// k_qgemm3 stages a 128-row tile of Hprev and the whole B image of its gate through LDS for every
// 16-deep step and waits at two barriers per step pair; its MFMAs ran about a third of the time.
// Here one workgroup per CU (8 waves, two per SIMD) loads the gate's bf16 G image (piece 0 of
// k_split_g's image, 128 KB) into LDS once and keeps it for the launch.  Each wave then owns
// 32-row tiles end to end (32 rows x all 256 columns, eight 32 x 32 accumulators): Hprev goes
// straight from memory into the A fragment registers (row lane % 32, k = 16c + 8(lane / 32) ..
// +7), QR_AHEAD steps ahead across tile boundaries, and is split into its two bf16 pieces in
// registers, so no wave waits on another after the image is in.  The per-accumulator product
// order (a1 b0, a0 b0 per step, steps in order) is k_qgemm3<1>'s: Q is bit-identical to it.
// Grid: 32 workgroups per XCD, as 8 row groups x the 4 gates, so the four workgroups that read
// the same Hprev rows share one L2.
#ifndef QR_ABL
#define QR_ABL 0   // timing ablations for tools/kbench (1: no Q stores, 2: no Hprev loads, 4: no MFMAs)
#endif
#ifndef QR_AHEAD_SEL
#define QR_AHEAD_SEL 4
#endif
constexpr int QR_WAVES = 8, QR_AHEAD = QR_AHEAD_SEL;
__global__ __launch_bounds__(64 * QR_WAVES, 1) void k_qgemm_res(Geom g, const float* __restrict__ Sh,
                                                                 const bf16x8* __restrict__ gi,
                                                                 float* __restrict__ Q,
                                                                 const int* __restrict__ found) {
  constexpr int H = 256, NK = H / 16, NTT = H / 32;
  __shared__ bf16x8 Gs[NK * NTT * 64];   // [c][n][lane]: the B fragment of rows 16c.., columns 32n..
  const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8, q = slot % 4;
  if (found && found[q]) return;
  const int ng = gridDim.x / 4, grp = xcd * (gridDim.x / 32) + slot / 4;
  const bf16x8* gq = gi + (size_t)q * NK * NTT * 192;
  {   // all 16 units of a thread in flight at once (a load-store loop waits out one L2 trip each)
    constexpr int NU = NK * NTT * 64 / (64 * QR_WAVES);
    bf16x8 u[NU];
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      const int i = threadIdx.x + k * 64 * QR_WAVES;
      u[k] = gq[(i >> 6) * 192 + (i & 63)];
    }
#pragma unroll
    for (int k = 0; k < NU; ++k) Gs[threadIdx.x + k * 64 * QR_WAVES] = u[k];
  }
  __syncthreads();
  const int64_t BT = g.BT(), ntile = (BT + 31) / 32;
  const int64_t t1 = ntile * (grp + 1) / ng;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c32 = lane & 31, kh = lane >> 5;
  int64_t tile = ntile * grp / ng + wave;
  if (tile >= t1) return;
  auto rowptr = [&](int64_t tl) {
    const int64_t r = tl * 32 + c32 < BT ? tl * 32 + c32 : BT - 1;   // rows past BT: computed, not stored
    return Sh + g.hrow(r) * H + 8 * kh;
  };
  const float* ap = rowptr(tile);
  f32x4 ring[QR_AHEAD][2];
#pragma unroll
  for (int s = 0; s < QR_AHEAD; ++s) {
    ring[s][0] = *reinterpret_cast<const f32x4*>(ap + 16 * s);
    ring[s][1] = *reinterpret_cast<const f32x4*>(ap + 16 * s + 4);
    // in slot order: the loop's waits count from the last load of its own order, and a reordered
    // prologue would make the tile's first step wait for every load and store in flight
    __builtin_amdgcn_sched_barrier(0);
  }
  f32x16 acc[NTT];
  const __amdgpu_buffer_rsrc_t rQ =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<__bf16*>(Q) + (int64_t)q * BT * H, 0, (uint32_t)(BT * H * 2), kBufWord3);
  // the 16 steps of tile `tile` (its rows at ap); the last QR_AHEAD steps load the first rows of
  // the next tile (at apn)
  auto steps = [&](const float* apn) {
#pragma unroll
    for (int n = 0; n < NTT; ++n) acc[n] = f32x16{};
#pragma unroll
    for (int c = 0; c < NK; ++c) {
      const int sl = c % QR_AHEAD;
      const f32x8 v = {ring[sl][0].x, ring[sl][0].y, ring[sl][0].z, ring[sl][0].w,
                       ring[sl][1].x, ring[sl][1].y, ring[sl][1].z, ring[sl][1].w};
      const float* src = c + QR_AHEAD < NK ? ap + 16 * (c + QR_AHEAD) : apn + 16 * (c + QR_AHEAD - NK);
      if (QR_ABL & 2) {
        ring[sl][0] = v.lo + 1.f; ring[sl][1] = v.hi;
      } else {
        ring[sl][0] = *reinterpret_cast<const f32x4*>(src);
        ring[sl][1] = *reinterpret_cast<const f32x4*>(src + 4);
      }
      bf16x8 a0, a1;
      split2(v, a0, a1);
#pragma unroll
      for (int n = 0; n < NTT; ++n) {
        const bf16x8 b0 = Gs[(c * NTT + n) * 64 + lane];
        if (QR_ABL & 4) {
          acc[n][0] += (float)a0[0] * (float)b0[0] + (float)a1[1];
        } else {
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[n], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep each step's loads where they are (hoisted, they spill)
    }
  };
  // Q of tile `tile` as bf16 row quads.  Quads past BT fall outside the descriptor (qres_ok:
  // BT % 4 == 0), so their stores are dropped without a branch.
  auto store = [&]() {
    const uint32_t qo = (uint32_t)((tile * 8 + (lane >> 5)) * H + c32) * 8;   // quad of row acc_row(0, lane)
#pragma unroll
    for (int r = 0; r < 16; r += 4)
#pragma unroll
      for (int n = 0; n < NTT; ++n) {
        const f32x4 v = f32x4{acc[n][r], acc[n][r + 1], acc[n][r + 2], acc[n][r + 3]};
        if (!(QR_ABL & 1) || v[0] == 12345.f)
        buf_st2(rQ, qo + (uint32_t)((r >> 2) * 2 * H + 32 * n) * 8,
                __builtin_bit_cast(f32x2, __builtin_convertvector(v, bf16x4)));
      }
  };
  // Rotated loop: the steps of the first tile run before it, so the loop is entered in the state
  // its back edge leaves (the next tile's first loads in flight behind the stores) and the
  // compiler's waits at the top of the steps count the stores instead of draining them.
  const float* apn = tile + QR_WAVES < t1 ? rowptr(tile + QR_WAVES) : ap;
  steps(apn);
  while (true) {
    store();
    if (tile + QR_WAVES >= t1) break;
    tile += QR_WAVES;
    ap = apn;
    apn = tile + QR_WAVES < t1 ? rowptr(tile + QR_WAVES) : ap;
    steps(apn);
  }
}

// ------------------------------------------------------------------ slab = Hprev^T R
// Tile: 256 hidden units m x 256 columns j of one gate (H % 256 == 0) over the rows of one split, in
// 16-row steps.  Both MFMA operands are k(= row)-strided in memory.  Staging keeps rows as they are
// (a wave-instruction = one 1-KB row) and stores the split pieces row-major; the fragments come back
// transposed through ds_read_b64_tr_b16 (two per piece: rows k..k+3 and k+4..k+7 of 16 columns per
// lane group).  Images: [piece][128-column block][16 rows][128 x 16 bit], 256-B rows whose 16-B
// chunks are XOR-permuted by the row (cdna_hip_programming.md T10 image (b)): the row-major staging
// writes and the transposed reads are both conflict-free.
constexpr int A3_BM = 256, A3_BN = 256, A3_KS = 16;
constexpr int A3_SUB = A3_KS * 128;          // bf16 of one 128-column block (16 rows x 128 columns)

template <int BN>
struct A3 {
  static constexpr int PA = (A3_BM / 128) * A3_SUB;   // one split piece of the Hprev operand
  static constexpr int PR = (BN / 128) * A3_SUB;      // one split piece of the R operand
};

__device__ __forceinline__ int a3_off(int row, int col) {   // bf16 offset of (row, col), col % 4 == 0
  const int sub = col >> 7, cw = col & 127, ch = cw >> 3;
  return sub * A3_SUB + row * 128 + 8 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) + (cw & 4);
}

// k_atr3w: 8 waves as 2 (m) x 4 (j) of 128 x 64 (4 x 2 in the 512 x 128 tile of H = 512): 128
// accumulators per lane, so two waves share each
// SIMD and one wave's staging VALU (phi, phi', the split of R and Hprev) and waits issue while the
// other's MFMAs run (at one wave per SIMD with 256 accumulators -- round 2's k_atr3 -- the staging
// and the MFMAs of a wave serialised: 0.85 against 0.80 ms at C3).  Each wave stages two rows of
// each operand per step (one 1-KB row per wave-instruction), two steps ahead through a two-slot
// register ring.
constexpr int A3W_THREADS = 512;

#ifndef A3W_ABL
#define A3W_ABL 0   // timing ablations for tools/build_lib_variant.sh: 1 no loads, 2 no MFMAs
#endif
// One step's operand loads of a wave: BM = 256, two rows of 256 H_prev and 256 z / tgt columns
// (one 1-KB row per wave-instruction); BM = 512, two rows of all 512 H_prev columns (four
// instructions) and two rows of 128 z / tgt columns (one instruction: a half-wave per row).
template <int BM>
struct Atr3wRing {
  static constexpr int NA = BM / 128, NZ = BM == 512 ? 1 : 2;
  float4 a[NA], z[NZ], t[NZ];
};

// Tile shapes (BM x BN, 128 accumulators per lane either way):
//  BM = 256: (mb, nb) is the 256 x 256 block of G_q (H_prev columns 256 mb.., R columns 256 nb..);
//  BM = 512 (H = 512): mb = 0, the 512 x 128 block of all H_prev columns and R columns 128 nb.., so
//  that every R element is formed (phi, phi', the fp16 split) by one workgroup instead of two, and
//  z / tgt are read once from HBM.  The per-output product sequence is the same: G is bit-identical.
// NP = 3: split3 operands, six products (f32-accurate); the first h stage after the state is bound
// or invalidated (no sweep has bounded the operands yet).
// NP = 2, F16: two fp16 pieces instead (bf16 two-way splits, ~2^-16 per product, measured 1.3-3.7x
// the error of a torch fp32 GEMM of the same operands and were dropped in round 4) (hi = rn(a), lo = rn(a - hi): 22 bits,
// ~2^-22 relative per piece pair, 2^-20.4 per product at worst -- f32-accurate once summed with the
// f32 accumulation of thousands of rows), on the same matrix rate (v_mfma_f32_32x32x16_f16).  fp16
// has 5 exponent bits, so both operands are first scaled by exact powers of two that put their
// largest possible magnitude at 2^14 (< 65504): sH from max |H_prev| and sR from a bound on |R|
// (atr_scales), undone on the slab (exact).  Values 2^17 below the bound lose relative precision in
// the lo piece (fp16 subnormals), i.e. absolute errors below 2^-39 of the bound.
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split2h(f32x4 a, bf16x4& p0, bf16x4& p1) {
  const f16x4 h0 = __builtin_convertvector(a, f16x4);
  const f16x4 h1 = __builtin_convertvector(a - __builtin_convertvector(h0, f32x4), f16x4);
  p0 = __builtin_bit_cast(bf16x4, h0);
  p1 = __builtin_bit_cast(bf16x4, h1);
}
// the three products of fp16 two-way splits (pieces carried as 16-bit patterns in bf16 vectors)
__device__ __forceinline__ f32x16 mfma_split2h(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 acc) {
  const f16x8 a0 = __builtin_bit_cast(f16x8, a[0]), a1 = __builtin_bit_cast(f16x8, a[1]);
  const f16x8 b0 = __builtin_bit_cast(f16x8, b[0]), b1 = __builtin_bit_cast(f16x8, b[1]);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc, 0, 0, 0);
  return acc;
}

// The scales of gate q's fp16 operands, from the ranges the last persistent sweep left (range[q] =
// max |phi(z) - tgt| over the x stage's z, range[4] = max |H_prev|, range[5] = max_row sum_d |x_d|)
// and the x stage's decided update dWx (the h stage's z is z + x dWx): |R| = |phi(z') - tgt| phi'(z')
// <= max|phi(z) - tgt| + |x dWx| (phi 1-Lipschitz, phi' <= 1).  The bound carries a factor 2 and an
// absolute 2^-16 for the rounding of z' and the ulps between the kernels' activation codes.
// Computed identically by every workgroup (512 threads); returns {sH, sR}.
__device__ __forceinline__ float2 atr_scales(const Geom& g, int q, const float* __restrict__ range,
                                             const float* __restrict__ dW, float* red /* LDS, >= 8 */) {
  const int n = g.D * g.H;
  const float* dq = dW + (int64_t)q * n;
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += A3W_THREADS) m = fmaxf(m, fabsf(dq[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float dwm = 0.f;
#pragma unroll
  for (int w = 0; w < A3W_THREADS / 64; ++w) dwm = fmaxf(dwm, red[w]);
  __syncthreads();   // red is reused
  const float rb = 2.f * (range[q] + range[5] * dwm + 0x1p-16f);
  const float hb = 2.f * range[4] + 0x1p-30f;
  auto scale = [](float b) {   // 2^(13 - floor(log2 b)): b * scale <= 2^14
    const int e = 13 - ilogbf(b);
    return ldexpf(1.f, e < -60 ? -60 : e > 60 ? 60 : e);
  };
  return make_float2(scale(hb), scale(rb));
}

template <int BM>
struct A3T {
  static constexpr int BN = BM == 512 ? 128 : 256;
  static constexpr int PA = (BM / 128) * A3_SUB;   // one split piece of the Hprev operand
  static constexpr int PR = (BN / 128) * A3_SUB;   // one split piece of the R operand
  static constexpr int WM = BM / 128;              // waves along m (128 rows each); 8 / WM along j
};

template <bool TANH, int NP, bool F16 = false, int BM = 256>
__device__ __forceinline__ void atr3w_body(const Geom& g, int q, int sp, int nsplit, int mb, int nb,
                                           const float* __restrict__ Sh, const float* __restrict__ zq,
                                           const float* __restrict__ tq, float* __restrict__ slab, __bf16* img,
                                           float2 scl = make_float2(1.f, 1.f)) {
  static_assert(!F16 || NP == 2, "fp16 operands come in two pieces");
  static_assert(BM == 256 || BM == 512, "tile rows");
  using P = A3T<BM>;
  using Ring = Atr3wRing<BM>;
  constexpr bool WIDE = BM == 512;
  const int H = g.H;
  const int64_t BT = g.BT();
  const int64_t per = ((BT + nsplit - 1) / nsplit + A3_KS - 1) / A3_KS * A3_KS;
  const int64_t r0 = sp * per, r1 = r0 + per < BT ? r0 + per : BT;
  constexpr int64_t ks = A3_KS;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rg = __builtin_amdgcn_readfirstlane(wave);   // rows 2 rg, 2 rg + 1 of each step
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Sh), 0,
                                                                      (int)(g.B * g.TP() * H * 4), kBufWord3);
  const __amdgpu_buffer_rsrc_t rZ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(zq), 0, (int)(BT * H * 4), kBufWord3);
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(tq), 0, (int)(BT * H * 4), kBufWord3);
  const int vo = 16 * lane;   // float4 column 4 lane of a 256-float row
  const int va = vo + 1024 * mb, vz = vo + 1024 * nb;   // + the block's first column
  // WIDE: z / tgt rows 2 rg (lanes 0-31) and 2 rg + 1 (lanes 32-63), 128 columns from 128 nb
  const int vzw = 16 * (lane & 31) + 512 * nb;
  auto gload = [&](Ring& R, int64_t k0) {   // rows past r1 clamped; they meet R = 0 in put()
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t r = k0 + 2 * rg + i, row = r < r1 ? r : r1 - 1;
      if (A3W_ABL & 1) {   // timing ablation (tools only): no operand loads
        const float4 f = make_float4((float)row, 0.5f, 0.25f, 0.125f);
#pragma unroll
        for (int h = 0; h < Ring::NA / 2; ++h) R.a[i * Ring::NA / 2 + h] = f;
        if (i < Ring::NZ) { R.z[i] = f; R.t[i] = f; }
        continue;
      }
      if constexpr (WIDE) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
          R.a[2 * i + h] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rA, vo + 1024 * h,
                                                                                            (int)(g.hrow(row) * H * 4), 0));
      } else {
        R.a[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rA, va, (int)(g.hrow(row) * H * 4), 0));
        R.z[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rZ, vz, (int)(row * H * 4), 2));
        R.t[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rT, vz, (int)(row * H * 4), 2));
      }
    }
    if constexpr (WIDE) {
      if (A3W_ABL & 1) return;
      const int64_t r = k0 + 2 * rg, row = r < r1 ? r : r1 - 1;   // the first row (uniform)
      const int vzr = vzw + ((lane >> 5) && r + 1 < r1 ? H * 4 : 0);   // the second: a row further
      R.z[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rZ, vzr, (int)(row * H * 4), 2));
      R.t[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rT, vzr, (int)(row * H * 4), 2));
    }
  };
  constexpr int STAGE = NP * (P::PA + P::PR);
  auto put = [&](int st, const Ring& R, int64_t k0) {
    __bf16* A = img + st * STAGE;
    __bf16* B = A + NP * P::PA;
    bf16x4 p0, p1, p2;
    auto pieces = [&](f32x4 v) {
      if constexpr (F16) split2h(v, p0, p1);
      else split3(v, p0, p1, p2);
    };
    auto put_a = [&](int o, const float4& a) {
      if constexpr (F16) pieces(f32x4{a.x, a.y, a.z, a.w} * scl.x);
      else pieces(f32x4{a.x, a.y, a.z, a.w});
      *reinterpret_cast<bf16x4*>(A + o) = p0;
      *reinterpret_cast<bf16x4*>(A + P::PA + o) = p1;
      if constexpr (NP == 3) *reinterpret_cast<bf16x4*>(A + 2 * P::PA + o) = p2;
    };
    auto put_r = [&](int o, bool ok, const float4& z, const float4& t) {
      const float zz[4] = {z.x, z.y, z.z, z.w};
      const float tt[4] = {t.x, t.y, t.z, t.w};
      f32x4 rv;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float phi, dphi;
        phi_acc<TANH>(zz[u], phi, dphi);
        rv[u] = ok ? (phi - tt[u]) * dphi : 0.f;
      }
      if constexpr (F16) pieces(rv * scl.y);
      else pieces(rv);
      *reinterpret_cast<bf16x4*>(B + o) = p0;
      *reinterpret_cast<bf16x4*>(B + P::PR + o) = p1;
      if constexpr (NP == 3) *reinterpret_cast<bf16x4*>(B + 2 * P::PR + o) = p2;
    };
    if constexpr (WIDE) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) put_a(a3_off(2 * rg + i, 256 * h + 4 * lane), R.a[2 * i + h]);
      const int rr = 2 * rg + (lane >> 5);
      put_r(a3_off(rr, 4 * (lane & 31)), k0 + rr < r1, R.z[0], R.t[0]);
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int rr = 2 * rg + i;
        const int o = a3_off(rr, 4 * lane);
        put_a(o, R.a[i]);
        put_r(o, k0 + rr < r1, R.z[i], R.t[i]);
      }
    }
  };
  // transposed fragment reads: lane group gi = lane >> 4 takes columns +16 (gi & 1) and rows
  // 8 (gi >> 1) .. +7; lane 4qq + pp of a group addresses row qq (+4 for the second read), columns 4pp..4pp+3
  const int gi = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int frow = 8 * (gi >> 1) + qq, fcol = 16 * (gi & 1) + 4 * pp;
  auto frag = [&](const __bf16* O, int piece, int cbase, bf16x8 (&f)[3]) {
    const int o0 = a3_off(frow, cbase + fcol), o1 = a3_off(frow + 4, cbase + fcol);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(O + p * piece + o0));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(O + p * piece + o1));
      f[p] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  const int wr = wave % P::WM, wc = wave / P::WM;   // 128-row m block, 64-column j block
  f32x16 acc[4][2];
  zero_acc(acc);
  auto compute = [&](int st) {
    const __bf16* A = img + st * STAGE;
    const __bf16* B = A + NP * P::PA;
    bf16x8 b[2][3];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) frag(B, P::PR, wc * 64 + ni * 32, b[ni]);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      bf16x8 a[3];
      frag(A, P::PA, wr * 128 + mi * 32, a);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        if (A3W_ABL & 2) acc[mi][ni][0] += (float)a[0][0] * (float)b[ni][0][0];   // ablation: no MFMAs
        else if constexpr (F16) acc[mi][ni] = mfma_split2h(a, b[ni], acc[mi][ni]);
        else acc[mi][ni] = mfma_split3(a, b[ni], acc[mi][ni]);
      }
    }
  };
  // Measured alternatives (C3, no gain or slower): sched_group_barrier interleaves of the staging
  // VALU into the MFMA stream (1 MFMA : 3-5 VALU : 1 DS), and the upper four waves staging before
  // multiplying (opposite phase to their SIMD partner: 0.84 against 0.76 ms, no spills in the loop).
  if (r0 < r1) {
    Ring R0, R1;
    gload(R0, r0);
    gload(R1, r0 + ks);
    put(0, R0, r0);
    __syncthreads();
    for (int64_t k0 = r0; k0 < r1; k0 += 2 * ks) {   // steps in pairs (an odd count ends masked)
      gload(R0, k0 + 2 * ks);
      compute(0);
      put(1, R1, k0 + ks);
      __syncthreads();
      gload(R1, k0 + 3 * ks);
      compute(1);
      put(0, R0, k0 + 2 * ks);
      __syncthreads();
    }
  }
  float* out = slab + ((int64_t)sp * 4 + q) * H * H + (int64_t)(BM * mb) * H + P::BN * nb + wc * 64 + (lane & 31);
  const float inv = F16 ? 1.f / (scl.x * scl.y) : 1.f;   // a power of two: exact
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = wr * 128 + mi * 32 + acc_row(r, lane);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) out[(int64_t)m * H + ni * 32] = F16 ? acc[mi][ni][r] * inv : acc[mi][ni][r];
    }
}

template <int NP, bool F16 = false, int BM = 256>
__global__ __launch_bounds__(A3W_THREADS, 1) void k_atr3w(Geom g, const float* __restrict__ Sh,
                                                         const float* __restrict__ zc, const float* __restrict__ tgt,
                                                         float* __restrict__ slab, int nsplit,
                                                         const float* __restrict__ range, const float* __restrict__ dW) {
  using P = A3T<BM>;
  __shared__ __attribute__((aligned(16))) __bf16 img[2 * NP * (P::PA + P::PR)];
  int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int q = lid % 4;          // the 4 gates of one split share the Hprev rows: same XCD
  lid /= 4;
  const int nmb = g.H / BM, nnb = g.H / P::BN, tl = lid % (nmb * nnb), sp = lid / (nmb * nnb);
  const int64_t n = g.BT() * g.H;
  float2 scl = make_float2(1.f, 1.f);
  if constexpr (F16) scl = atr_scales(g, q, range, dW, reinterpret_cast<float*>(img));
  if (q == 2)
    atr3w_body<true, NP, F16, BM>(g, q, sp, nsplit, tl / nnb, tl % nnb, Sh, zc + q * n, tgt + q * n, slab, img, scl);
  else
    atr3w_body<false, NP, F16, BM>(g, q, sp, nsplit, tl / nnb, tl % nnb, Sh, zc + q * n, tgt + q * n, slab, img, scl);
}

}  // namespace

bool split3_ok(const Geom& g) {   // 32-bit buffer offsets into the h plane and a z-cache plane
  return g.H % 256 == 0 && g.BT() >= 256 && g.B * (int64_t)g.TP() * g.H * 4 < (int64_t)INT32_MAX;
}

size_t split3_gimg_floats(const Geom& g) { return (size_t)4 * g.H * g.H * 3 / 2; }

// Rows accumulated in f32 (MFMA accumulators) per slab: at most atr_split_rows(g).  Each slab is
// then summed in fp64 by k_reduce_g.  Relative error of the h-side G against fp64 on identical
// operands (tests/test_gpu_weight_phase.py; profiles/r05b_c5_gradient_rows.txt), with the
// reference's own form (one fp32 GEMM per t, summed in fp32) for comparison:
//   C5 per GPU (H = 512): 16 384 rows 3.4-4.5e-6, 4 096 rows 0.7-0.9e-6 (split3 the same: it is the
//   accumulation, not the fp16 pieces), 1 024 rows 0.5-1.4e-7; reference form 1.8-2.3e-7.
//   C3 (H = 256): 4 096 rows 1.1-1.2e-7; reference form 1.7-2.2e-7.
// So 4 096 rows at H = 256 and 1 024 beyond (C5: 256 slabs, +1.6 GB of slab traffic per step).
static int64_t atr_split_rows(const Geom& g) {
  static const long env = [] {   // ADMM_ATR_ROWS: experiment hook (tools)
    const char* e = std::getenv("ADMM_ATR_ROWS");
    return e ? std::atol(e) : 0L;
  }();
  if (env >= 256) return env;
  return g.H <= 256 ? 4096 : 1024;
}
int atr3_splits(const Geom& g) {
  const int tiles = (g.H / A3_BM) * (g.H / A3_BN) * 4;
  int64_t ns = 256 / tiles;   // one resident wave of workgroups (one per CU) ...
  const int64_t by_acc = (g.BT() + atr_split_rows(g) - 1) / atr_split_rows(g);
  if (ns < by_acc) ns = by_acc;   // ... or more, so that no slab sums more than kAtrSplitRows rows
  const int64_t max_by_rows = g.BT() / 256;
  if (ns > max_by_rows) ns = max_by_rows;
  return ns < 1 ? 1 : (int)ns;
}

void launch_atr3(const Geom& g, const float* Sh, const float* zc, const float* tgt, float* slab, int nsplit,
                 hipStream_t s, const float* range, const float* dW, bool wide_ok) {
  // 256 x 256 blocks of each gate's G (H % 256 == 0, split3_ok), nsplit row ranges; at H = 512 the
  // fp16 path takes 512 x 128 blocks instead (the same count, every R element staged once)
  const int nt = g.H / 256, nb = 4 * nt * nt * nsplit;
  const bool wide = wide_ok && g.H == 512;
  if (range && dW) {   // scaled fp16 two-way splits: f32-accurate at two pieces' matrix work
    if (wide) k_atr3w<2, true, 512><<<nb, A3W_THREADS, 0, s>>>(g, Sh, zc, tgt, slab, nsplit, range, dW);
    else k_atr3w<2, true><<<nb, A3W_THREADS, 0, s>>>(g, Sh, zc, tgt, slab, nsplit, range, dW);
  } else {   // (once per bound state; the 512 x 128 tile spills here with three pieces)
    k_atr3w<3><<<nb, A3W_THREADS, 0, s>>>(g, Sh, zc, tgt, slab, nsplit, nullptr, nullptr);
  }
}

void launch_split_g(const Geom& g, const float* G, float* gimg, hipStream_t s) {
  const int total = 4 * (g.H / 16) * (g.H / 32) * 64;
  k_split_g<<<(total + kThreads - 1) / kThreads, kThreads, 0, s>>>(g.H, G, reinterpret_cast<bf16x8*>(gimg));
}

bool qpair_ok(const Geom& g) { return g.BT() % 4 == 0; }

bool qres_ok(const Geom& g) { return g.H == 256 && qpair_ok(g) && g.BT() * 256 * 2 < (int64_t)INT32_MAX; }

int q_layout(const Geom& g) { return qpair_ok(g) ? 2 : 0; }

void launch_qgemm3(const Geom& g, const float* Sh, const float* G, float* gimg, float* Q, hipStream_t s,
                   bool gimg_ready) {
  if (!gimg_ready) launch_split_g(g, G, gimg, s);
  const bf16x8* gb = reinterpret_cast<const bf16x8*>(gimg);
  if (qres_ok(g)) {   // G resident in LDS: one workgroup per CU
    k_qgemm_res<<<256, 64 * QR_WAVES, 0, s>>>(g, Sh, gb, Q, nullptr);
    return;
  }
  // 128-row tiles, two workgroups per CU
  dim3 grid((unsigned)((g.BT() + 127) / 128 * 4 * (g.H / Q3_BN)));
  if (q_layout(g) == 2) k_qgemm3<1, 2, 128><<<grid, 256, 0, s>>>(g, Sh, gb, Q, nullptr);
  else k_qgemm3<1, 0, 128><<<grid, 256, 0, s>>>(g, Sh, gb, Q, nullptr);
}

}  // namespace admm
