// admm_split3.hpp -- split-bf16 MFMA pieces shared by admm_split3.hip (k_qgemm3) and
// admm_kernels.hip (k_qtrial3, the h-side trial pass fused with Q = Hprev G).  See the header
// comment of admm_split3.hip for the three-way split and the LDS images.
#pragma once
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

// the three products of two-way splits (a = a0 + a1, b = b0 + b1 to ~2^-17): a0 b0 + a0 b1 + a1 b0,
// ~2^-16 relative -- for the trial direction Q only (see k_qgemm3)
__device__ __forceinline__ f32x16 mfma_split2(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void frag3(const __bf16* img, int piece_stride, int off, bf16x8 (&f)[3]) {
#pragma unroll
  for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const bf16x8*>(img + p * piece_stride + off);
}

template <int NP = 3>
__device__ __forceinline__ void put3(__bf16* img, int piece_stride, int off, f32x8 v) {
  bf16x8 p0, p1, p2;
  split3(v, p0, p1, p2);
  *reinterpret_cast<bf16x8*>(img + off) = p0;
  *reinterpret_cast<bf16x8*>(img + piece_stride + off) = p1;
  if (NP == 3) *reinterpret_cast<bf16x8*>(img + 2 * piece_stride + off) = p2;
}

// ------------------------------------------------------------------ Q tile = Hprev G
// Tile: BM rows x 256 columns of one gate (H % 256 == 0), BM / 32 waves as BM / 64 (rows) x 2
// (columns) of 64 x 128; K = H in 16-deep steps through double-buffered LDS, the global loads of
// step c+2 in flight during the MFMAs of step c.  G comes as the split image of k_split_g:
// gi[(((q * NK + c) * NTT + n) * 3 + p) * 64 + lane] = piece p of the MFMA B fragment of
// rows 16c.., columns 32n.. (NK = H/16, NTT = H/32).  Every workgroup reads the G image of its
// gate (32 KB per step from L2), so BM = 256 halves that traffic per Q row against BM = 128.
// Ends with a __syncthreads(): the LDS (Q3Lds<BM>() bytes from `lds`) is free for the caller's
// epilogue.
constexpr int Q3_BN = 256;
constexpr int kQ3BU = (Q3_BN / 32) * 3 * 64;    // bf16x8 units of one B step image
template <int BM>
constexpr int Q3Lds() { return 2 * 3 * (BM * 16) * 2 + 2 * kQ3BU * 16; }

// NP = 3: the six split3 products (f32-accurate); NP = 2: mfma_split2 (half the matrix work);
// NP = 1: Hprev in two pieces, G in one (a0 b0 + a1 b0: G rounded to bf16, ~2^-9 relative per
// element -- the trial direction only; a third of the B image and of the matrix work of NP = 3)
template <int NP, int BM>
__device__ __forceinline__ void qgemm3_tile(const Geom& g, const float* __restrict__ Sh,
                                            const bf16x8* __restrict__ gi, int q, int cb, int64_t m0,
                                            char* lds, f32x16 (&acc)[2][4]) {
  // B image per step: NP = 3 all three pieces of each 32-column tile (192 units), NP = 2 only
  // pieces 0 and 1 (128 units): the third piece is never multiplied there
  constexpr int NT = 2 * BM;   // threads
  constexpr int AP = BM * 16, PSTR = NP == 3 ? 192 : NP == 2 ? 128 : 64, BU = (Q3_BN / 32) * PSTR;
  static_assert(BU % NT == 0, "B image units per thread");
  __bf16* As = reinterpret_cast<__bf16*>(lds);                       // [2][3 * AP]
  bf16x8* Bs = reinterpret_cast<bf16x8*>(lds + 2 * 3 * AP * 2);       // [2][BU]
  const int H = g.H, NK = H / 16, NTT = H / 32;
  const int64_t BT = g.BT();
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // staging: thread = (row sr, k-half sh) of A; 6 units of the B image
  const int sr = tid >> 1, sh = tid & 1;
  const int64_t arow = m0 + sr < BT ? m0 + sr : BT - 1;   // rows past BT: computed, not used
  const float* ap = Sh + g.hrow(arow) * H + 8 * sh;
  const bf16x8* bp = gi + ((size_t)q * NK * NTT + (size_t)(Q3_BN / 32) * cb) * 192 + tid;
  const size_t bstep = (size_t)NTT * 192;
  // two-slot register ring: the loads of step c + 2 are issued at step c (one step of MFMAs does
  // not cover the L2/HBM latency of the next operands); NK is even (H % 256 == 0)
  struct Slot { float4 a0, a1; bf16x8 b[BU / NT]; };
  auto gload = [&](Slot& r, int c) {
    // past the last step: step NK - 1 again, unused.  Skipping the loads instead (a branch) left the
    // compiler's count of loads in flight unknown after it, and every step then waited for all of them
    c = c < NK ? c : NK - 1;
    if (S3_ABL & 32) {
      r.a0 = make_float4(c, 1.f, 2.f, 3.f); r.a1 = r.a0;
    } else {
      r.a0 = *reinterpret_cast<const float4*>(ap + 16 * c);
      r.a1 = *reinterpret_cast<const float4*>(ap + 16 * c + 4);
    }
#pragma unroll
    for (int u = 0; u < BU / NT; ++u) {
      const int i = tid + u * NT;   // image unit -> G-image unit (skipping piece 2 for NP = 2)
      const int src = NP == 3 ? i : NP == 2 ? (i >> 7) * 192 + (i & 127) : (i >> 6) * 192 + (i & 63);
      r.b[u] = bp[c * bstep + src - tid];
    }
  };
  auto lstore = [&](int st, const Slot& r) {
    put3<NP == 1 ? 2 : NP>(As + st * 3 * AP, AP, sw_off(sr, sh), f32x8{r.a0.x, r.a0.y, r.a0.z, r.a0.w, r.a1.x, r.a1.y, r.a1.z, r.a1.w});
#pragma unroll
    for (int u = 0; u < BU / NT; ++u) Bs[st * BU + tid + u * NT] = r.b[u];
  };
  const int wr = wave >> 1, wc = wave & 1, c32 = lane & 31, kh = lane >> 5;
  auto compute = [&](int st) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      bf16x8 a[3];
      if (NP == 3) {
        frag3(As + st * 3 * AP, AP, sw_off(wr * 64 + mi * 32 + c32, kh), a);
      } else {
        const int o = sw_off(wr * 64 + mi * 32 + c32, kh);
        a[0] = *reinterpret_cast<const bf16x8*>(As + st * 3 * AP + o);
        a[1] = *reinterpret_cast<const bf16x8*>(As + st * 3 * AP + AP + o);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const bf16x8* bb = &Bs[st * BU + (wc * 4 + ni) * PSTR + lane];
        if constexpr (NP == 1) {
          const bf16x8 b0 = bb[0];
          if (S3_ABL & 64) acc[mi][ni][0] += (float)a[0][0] * (float)b0[0];
          else {
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b0, acc[mi][ni], 0, 0, 0);
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b0, acc[mi][ni], 0, 0, 0);
          }
          continue;
        } else {
        const bf16x8 b[3] = {bb[0], bb[64], NP == 3 ? bb[128] : bb[0]};
        if (S3_ABL & 64) acc[mi][ni][0] += (float)a[0][0] * (float)b[0][0];
        else if (NP == 3) acc[mi][ni] = mfma_split3(a, b, acc[mi][ni]);
        else acc[mi][ni] = mfma_split2(a, b, acc[mi][ni]);
        }
      }
    }
  };
  zero_acc(acc);
  Slot R0, R1;
  gload(R0, 0);
  gload(R1, 1);
  lstore(0, R0);
  __syncthreads();
  for (int c = 0; c < NK; c += 2) {
    gload(R0, c + 2);
    __builtin_amdgcn_sched_barrier(0);
    compute(0);
    __builtin_amdgcn_sched_barrier(0);
    lstore(1, R1);
    __syncthreads();
    gload(R1, c + 3);
    __builtin_amdgcn_sched_barrier(0);
    compute(1);
    __builtin_amdgcn_sched_barrier(0);
    // unconditional (the last one stores step NK - 1 again, never read): under `if (c + 2 < NK)`
    // the compiler sank R0's loads into that branch, just before this store, and they lost their
    // step of lead
    lstore(0, R0);
    __syncthreads();
  }
}

}  // namespace
}  // namespace admm
