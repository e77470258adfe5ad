// admm_split3.hip -- the h-stage GEMMs of the weight update on bf16 matrix cores with
// f32-accurate three-way split operands (admm_dev.hpp split3).
//
//   k_atr3   slab[sp][q][m][j] = sum_{rows of split sp} Hprev[row][m] * R_q[row][j]
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
#include "admm_dev.hpp"
#include "admm_kernels.hpp"

namespace admm {
namespace {

typedef float f32x8 __attribute__((ext_vector_type(8)));

#ifndef S3_ABL
#define S3_ABL 0   // kernel ablations for tools/kbench (bitmask, 0 = full kernels)
#endif

__device__ __forceinline__ int sw_off(int r, int h) {   // bf16 offset of half h of row r
  return r * 16 + 8 * (h ^ (((r >> 2) ^ (r >> 3)) & 1));
}

// the six piece products, smallest first: (a2 b0, a1 b1, a0 b2, a1 b0, a0 b1, a0 b0)
__device__ __forceinline__ f32x16 mfma_split3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void frag3(const __bf16* img, int piece_stride, int off, bf16x8 (&f)[3]) {
#pragma unroll
  for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const bf16x8*>(img + p * piece_stride + off);
}

__device__ __forceinline__ void put3(__bf16* img, int piece_stride, int off, f32x8 v) {
  bf16x8 p0, p1, p2;
  split3(v, p0, p1, p2);
  *reinterpret_cast<bf16x8*>(img + off) = p0;
  *reinterpret_cast<bf16x8*>(img + piece_stride + off) = p1;
  *reinterpret_cast<bf16x8*>(img + 2 * piece_stride + off) = p2;
}

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
// Workgroup: 128 rows x 256 columns of one gate (H % 256 == 0), 4 waves as 2 (rows) x 2
// (columns) of 64 x 128; K = H in 16-deep steps through double-buffered LDS, the global loads
// of step c+1 in flight during the MFMAs of step c.
constexpr int Q3_BM = 128, Q3_BN = 256;

__global__ __launch_bounds__(kThreads) void k_qgemm3(Geom g, const float* __restrict__ Sh,
                                                      const bf16x8* __restrict__ gi, float* __restrict__ Q) {
  constexpr int AP = Q3_BM * 16;            // one piece of the A image (bf16)
  constexpr int BU = (Q3_BN / 32) * 3 * 64; // bf16x8 units of one B step image
  __shared__ __attribute__((aligned(16))) __bf16 As[2][3 * AP];
  __shared__ bf16x8 Bs[2][BU];
  const int H = g.H, NK = H / 16, NTT = H / 32, ncb = H / Q3_BN;
  int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int cb = lid % ncb;
  lid /= ncb;
  const int q = lid % 4;
  const int64_t m0 = (int64_t)(lid / 4) * Q3_BM, BT = g.BT();
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // staging: thread = (row sr, k-half sh) of A; 6 units of the B image
  const int sr = tid >> 1, sh = tid & 1;
  const int64_t arow = m0 + sr < BT ? m0 + sr : BT - 1;   // rows past BT: computed, not stored
  const float* ap = Sh + g.hrow(arow) * H + 8 * sh;
  const bf16x8* bp = gi + ((size_t)q * NK * NTT + (size_t)(Q3_BN / 32) * cb) * 192 + tid;
  const size_t bstep = (size_t)NTT * 192;
  float4 ra0, ra1;
  bf16x8 rb[BU / kThreads];
  auto gload = [&](int c) {
    if (S3_ABL & 32) {
      ra0 = make_float4(c, 1.f, 2.f, 3.f); ra1 = ra0;
    } else {
      ra0 = *reinterpret_cast<const float4*>(ap + 16 * c);
      ra1 = *reinterpret_cast<const float4*>(ap + 16 * c + 4);
    }
#pragma unroll
    for (int u = 0; u < BU / kThreads; ++u) rb[u] = bp[c * bstep + u * kThreads];
  };
  auto lstore = [&](int st) {
    put3(As[st], AP, sw_off(sr, sh), f32x8{ra0.x, ra0.y, ra0.z, ra0.w, ra1.x, ra1.y, ra1.z, ra1.w});
#pragma unroll
    for (int u = 0; u < BU / kThreads; ++u) Bs[st][tid + u * kThreads] = rb[u];
  };
  const int wr = wave >> 1, wc = wave & 1, c32 = lane & 31, kh = lane >> 5;
  f32x16 acc[2][4];
  zero_acc(acc);
  gload(0);
  lstore(0);
  __syncthreads();
  for (int c = 0; c < NK; ++c) {
    const int st = c & 1;
    if (c + 1 < NK) gload(c + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      bf16x8 a[3];
      frag3(As[st], AP, sw_off(wr * 64 + mi * 32 + c32, kh), a);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const bf16x8* bb = &Bs[st][(wc * 4 + ni) * 192 + lane];
        const bf16x8 b[3] = {bb[0], bb[64], bb[128]};
        if (S3_ABL & 64) acc[mi][ni][0] += (float)a[0][0] * (float)b[0][0];
        else acc[mi][ni] = mfma_split3(a, b, acc[mi][ni]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 < NK) lstore(st ^ 1);
    __syncthreads();
  }
  float* Qq = Q + (int64_t)q * BT * H + Q3_BN * cb + wc * 128 + c32;
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

// ------------------------------------------------------------------ slab = Hprev^T R
// Workgroup: 256 hidden units m x 256 columns j of one gate (H % 256 == 0) over the rows of one
// split, in 16-row steps; 4 waves as 2 (m) x 2 (j) of 128 x 128 (256 accumulators per lane),
// one wave per SIMD.  Both MFMA operands are k(= row)-strided in memory.  Staging keeps rows as
// they are: a thread loads 4 rows x 4 columns (float4, a wave-instruction = one 1-KB row) and
// stores the split pieces row-major; the fragments come back transposed through
// ds_read_b64_tr_b16 (two per piece: rows k..k+3 and k+4..k+7 of 16 columns per lane group).
// Images: [piece][half of the columns][16 rows][128 bf16], 256-B rows whose 16-B chunks are
// XOR-permuted by the row (cdna_hip_programming.md T10 image (b)): the row-major staging writes
// and the transposed reads are both conflict-free.  The loads run two steps ahead through a
// two-slot register ring.
constexpr int A3_BM = 256, A3_BN = 256, A3_KS = 16;
constexpr int A3_SUB = A3_KS * 128;          // bf16 of one half-image (16 rows x 128 columns)
constexpr int A3_PIECE = 2 * A3_SUB;         // one split piece of one operand
constexpr int A3_OPER = 3 * A3_PIECE;        // one operand (A or R) of one stage
constexpr int A3_STAGE = 2 * A3_OPER;

__device__ __forceinline__ int a3_off(int row, int col) {   // bf16 offset of (row, col), col % 4 == 0
  const int sub = col >> 7, cw = col & 127, ch = cw >> 3;
  return sub * A3_SUB + row * 128 + 8 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) + (cw & 4);
}

struct Atr3Ring { float4 a[4], z[4], t[4]; };

template <bool TANH>
__device__ __forceinline__ void atr3_body(const Geom& g, int mb, int nb, int q, int sp, int nsplit,
                                          const float* __restrict__ Sh, const float* __restrict__ zq,
                                          const float* __restrict__ tq, float* __restrict__ slab, __bf16* img) {
  const int H = g.H;
  const int64_t BT = g.BT();
  const int64_t per = ((BT + nsplit - 1) / nsplit + A3_KS - 1) / A3_KS * A3_KS;
  const int64_t r0 = sp * per, r1 = r0 + per < BT ? r0 + per : BT;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // staging: columns 4cg..4cg+3, rows 4rg..4rg+3 of a step; rg (the wave) made provably uniform
  // so the row offsets stay in SGPRs (no waterfall loops around the buffer loads, guide T20)
  const int cg = lane, rg = __builtin_amdgcn_readfirstlane(wave);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Sh), 0,
                                                                      (int)(g.B * g.TP() * H * 4), kBufWord3);
  const __amdgpu_buffer_rsrc_t rZ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(zq), 0, (int)(BT * H * 4), kBufWord3);
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(tq), 0, (int)(BT * H * 4), kBufWord3);
  const int va = (mb * A3_BM + 4 * cg) * 4, vz = (nb * A3_BN + 4 * cg) * 4;
  // rows past r1 are loaded clamped (branch-free) and meet R = 0 in put()
  auto gload = [&](Atr3Ring& R, int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t r = k0 + 4 * rg + i, row = r < r1 ? r : r1 - 1;
      const int sa = (int)(g.hrow(row) * H * 4), sz = (int)(row * H * 4);
      R.a[i] = (S3_ABL & 1) ? make_float4(i, 1, 2, 3)
                            : __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rA, va, sa, 0));
      R.z[i] = (S3_ABL & 2) ? make_float4(0.1f, 0.2f, 0.3f, 0.4f)
                            : __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rZ, vz, sz, 2));
      R.t[i] = (S3_ABL & 2) ? make_float4(0.5f, 0.5f, 0.5f, 0.5f)
                            : __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rT, vz, sz, 2));
    }
  };
  // split row i of a ring slot (4 columns of Hprev and of R) into the images of stage st
  auto put_row = [&](int st, const Atr3Ring& R, int64_t k0, int i) {
    __bf16* A = img + st * A3_STAGE;
    __bf16* B = A + A3_OPER;
    const int o = a3_off(4 * rg + i, 4 * cg);
    const bool ok = k0 + 4 * rg + i < r1;
    const float zz[4] = {R.z[i].x, R.z[i].y, R.z[i].z, R.z[i].w};
    const float tt[4] = {R.t[i].x, R.t[i].y, R.t[i].z, R.t[i].w};
    f32x4 rv;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float phi, dphi;
      phi_fast<TANH>(zz[u], phi, dphi);
      rv[u] = ok ? (phi - tt[u]) * dphi : 0.f;
    }
    bf16x4 p0, p1, p2;
    split3(f32x4{R.a[i].x, R.a[i].y, R.a[i].z, R.a[i].w}, p0, p1, p2);
    *reinterpret_cast<bf16x4*>(A + o) = p0;
    *reinterpret_cast<bf16x4*>(A + A3_PIECE + o) = p1;
    *reinterpret_cast<bf16x4*>(A + 2 * A3_PIECE + o) = p2;
    split3(rv, p0, p1, p2);
    *reinterpret_cast<bf16x4*>(B + o) = p0;
    *reinterpret_cast<bf16x4*>(B + A3_PIECE + o) = p1;
    *reinterpret_cast<bf16x4*>(B + 2 * A3_PIECE + o) = p2;
  };
  auto put = [&](int st, const Atr3Ring& R, int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) put_row(st, R, k0, i);
  };
  // transposed fragment reads: lane group gi = lane >> 4 takes columns +16 (gi & 1) and rows
  // 8 (gi >> 1) .. +7; lane 4qq + pp of a group addresses row qq (+4 for the second read),
  // columns 4pp..4pp+3
  const int gi = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int frow = 8 * (gi >> 1) + qq, fcol = 16 * (gi & 1) + 4 * pp;
  auto frag = [&](const __bf16* O, int cbase, bf16x8 (&f)[3]) {
    const int o0 = a3_off(frow, cbase + fcol), o1 = a3_off(frow + 4, cbase + fcol);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(O + p * A3_PIECE + o0));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(O + p * A3_PIECE + o1));
      f[p] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  const int wr = wave >> 1, wc = wave & 1;
  f32x16 acc[4][4];
  zero_acc(acc);
  auto compute = [&](int st) {
    const __bf16* A = img + st * A3_STAGE;
    const __bf16* B = A + A3_OPER;
    bf16x8 b[4][3];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) frag(B, wc * 128 + ni * 32, b[ni]);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      bf16x8 a[3];
      frag(A, wr * 128 + mi * 32, a);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        if (S3_ABL & 4) acc[mi][ni][0] += (float)a[0][0] * (float)b[ni][0][0];
        else acc[mi][ni] = mfma_split3(a, b[ni], acc[mi][ni]);
      }
    }
  };
  if (r0 < r1) {
    Atr3Ring R0, R1;
    gload(R0, r0);
    gload(R1, r0 + A3_KS);
    put(0, R0, r0);
    __syncthreads();
    // iteration of step s: issue step s+2 into the free slot, MFMAs of step s, split step s+1
    // into the other image.  Steps in pairs; an odd count runs one all-masked step (R = 0).
    for (int64_t k0 = r0; k0 < r1; k0 += 2 * A3_KS) {
      gload(R0, k0 + 2 * A3_KS);
      compute(0);
      put(1, R1, k0 + A3_KS);
      __syncthreads();
      gload(R1, k0 + 3 * A3_KS);
      compute(1);
      put(0, R0, k0 + 2 * A3_KS);
      __syncthreads();
    }
  }
  float* out = slab + ((int64_t)sp * 4 + q) * H * H + nb * A3_BN + wc * 128 + (lane & 31);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mb * A3_BM + wr * 128 + mi * 32 + acc_row(r, lane);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) out[(int64_t)m * H + ni * 32] = acc[mi][ni][r];
    }
}

__global__ __launch_bounds__(kThreads) void k_atr3(Geom g, const float* __restrict__ Sh, const float* __restrict__ zc,
                                                    const float* __restrict__ tgt, float* __restrict__ slab, int nsplit) {
  __shared__ __attribute__((aligned(16))) __bf16 img[2 * A3_STAGE];
  const int nmb = g.H / A3_BM, nnb = g.H / A3_BN;
  int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int q = lid % 4;          // the 4 gates of one split share the Hprev rows: same XCD
  lid /= 4;
  const int mb = lid % nmb;
  lid /= nmb;
  const int nb = lid % nnb, sp = lid / nnb;
  const int64_t n = g.BT() * g.H;
  if (q == 2)
    atr3_body<true>(g, mb, nb, q, sp, nsplit, Sh, zc + q * n, tgt + q * n, slab, img);
  else
    atr3_body<false>(g, mb, nb, q, sp, nsplit, Sh, zc + q * n, tgt + q * n, slab, img);
}

}  // namespace

bool split3_ok(const Geom& g) {   // 32-bit buffer offsets into the h plane and a z-cache plane
  return g.H % 256 == 0 && g.BT() >= 256 && g.B * (int64_t)g.TP() * g.H * 4 < (int64_t)INT32_MAX;
}

size_t split3_gimg_floats(const Geom& g) { return (size_t)4 * g.H * g.H * 3 / 2; }

int atr3_splits(const Geom& g) {
  const int tiles = (g.H / A3_BM) * (g.H / A3_BN) * 4;
  int ns = 256 / tiles;                     // one resident wave of workgroups (1 per CU)
  const int64_t max_by_rows = g.BT() / 256;
  if (ns > max_by_rows) ns = (int)max_by_rows;
  return ns < 1 ? 1 : ns;
}

void launch_atr3(const Geom& g, const float* Sh, const float* zc, const float* tgt, float* slab, int nsplit,
                 hipStream_t s) {
  dim3 grid((g.H / A3_BM) * (g.H / A3_BN) * 4 * nsplit);
  k_atr3<<<grid, kThreads, 0, s>>>(g, Sh, zc, tgt, slab, nsplit);
}

void launch_qgemm3(const Geom& g, const float* Sh, const float* G, float* gimg, float* Q, hipStream_t s) {
  const int total = 4 * (g.H / 16) * (g.H / 32) * 64;
  bf16x8* gi = reinterpret_cast<bf16x8*>(gimg);
  k_split_g<<<(total + kThreads - 1) / kThreads, kThreads, 0, s>>>(g.H, G, gi);
  const int64_t nrt = (g.BT() + Q3_BM - 1) / Q3_BM;
  dim3 grid((unsigned)(nrt * 4 * (g.H / Q3_BN)));
  k_qgemm3<<<grid, kThreads, 0, s>>>(g, Sh, gi, Q);
}

}  // namespace admm
