// admm_dev.hpp -- device-side building blocks for the gfx950 ADMM-LSTM step.
//
//  * activation numerics shared by every kernel (so that a gate stored as phi(z) and a
//    residual recomputed from the same z agree bit-for-bit: step 1 of the reference has
//    exactly zero weight gradients, admm.py:302-312 with gates == phi(z));
//  * accurate increments phi(z+d) - phi(z) for the line-search trials (no cancellation
//    at tiny d, see DESIGN.md "line-search numerics");
//  * an fp32 MFMA tile engine (v_mfma_f32_32x32x2_f32, exact f32 products/sums) with
//    LDS staging, used by the time-step GEMM, the Q = A*G GEMM and the A^T*R reduction.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

namespace admm {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Streaming (non-temporal) accesses for data touched once per pass: the ADMM state planes,
// the z cache and the line-search targets.  Calibrated on the box (tools/streambench.hip):
// +7 % read, +10 % copy bandwidth over plain loads/stores.
__device__ __forceinline__ float4 ld_nt(const float* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(float* p, const float4& v) {
  __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(p));
}
__device__ __forceinline__ float ld_nt(const float* p, int) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_nt(float* p, float v) { __builtin_nontemporal_store(v, p); }

constexpr int kWave = 64;
constexpr int kThreads = 256;  // every kernel: 4 waves per workgroup

// ----------------------------------------------------------------------------- numerics

struct SigPair {
  float s;   // sigma(z)
  float sc;  // 1 - sigma(z), computed without cancellation
};

__device__ __forceinline__ float div_fast(float a, float b);
// sigma(z) and 1 - sigma(z) without cancellation: accurate expf, then 1 / (1 + e) by v_rcp and one Newton
// step (div_fast), which equals the IEEE quotient 1.f / (1 + e) for every float 1 + e in [1, 2]: the pair
// is bit-identical to the expf + IEEE-division form over all finite z (tools/sigcheck.hip, exhaustive on
// an MI355X: profiles/r06f_sigcheck.txt) at half its VALU
__device__ __forceinline__ SigPair sig_pair(float z) {
  const float e = expf(-fabsf(z));
  const float r = div_fast(1.f, 1.f + e);
  const float er = e * r;
  return z >= 0.f ? SigPair{r, er} : SigPair{er, r};
}

__device__ __forceinline__ float sigm(float z) { return sig_pair(z).s; }

__device__ __forceinline__ float act(bool is_tanh, float z) { return is_tanh ? tanhf(z) : sigm(z); }

// expm1(x) to ~1 ulp: degree-8 Taylor on |x| < 1/2 (truncation < 2^-26 relative), else exp - 1.
// Branch-free (both forms, then a select): a per-lane branch here costs more than the 9 FMAs.
__device__ __forceinline__ float expm1_acc(float x) {
  float p = 1.f / 40320.f;
  p = fmaf(p, x, 1.f / 5040.f);
  p = fmaf(p, x, 1.f / 720.f);
  p = fmaf(p, x, 1.f / 120.f);
  p = fmaf(p, x, 1.f / 24.f);
  p = fmaf(p, x, 1.f / 6.f);
  p = fmaf(p, x, 0.5f);
  p = fmaf(p, x, 1.f);
  const float e = __expf(x) - 1.f;
  return fabsf(x) < 0.5f ? p * x : e;
}

// Three-way bf16 split of f32 values: a = p0 + p1 + p2 to ~2^-27 relative (each remainder is
// exact in f32).  Products of two split operands summed over the six terms with i + j <= 2
// (p_i q_j exact in the MFMA's f32 accumulation) reproduce an f32 product to ~2^-26 relative,
// at the bf16 matrix rate: 6 x v_mfma_f32_32x32x16_bf16 (192 cycles) per 16-deep step against
// 8 x v_mfma_f32_32x32x2_f32 (512 cycles, and those hold the SIMD's VALU issue).
// The f32 value of each rounded piece is read back from the packed dword of its pair (low half
// << 16, high half & 0xffff0000): one v_cvt_pk_bf16_f32 per pair and piece, where converting the
// bf16 vector back costs a second, single-lane v_cvt_pk per element.  Same pieces, bit for bit.
template <class V, class B>
__device__ __forceinline__ V bf16_widen(B p) {
  constexpr int N = sizeof(V) / 4;
  typedef unsigned U __attribute__((ext_vector_type(N / 2)));
  const U w = __builtin_bit_cast(U, p);
  V f;
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    f[2 * i] = __builtin_bit_cast(float, w[i] << 16);
    f[2 * i + 1] = __builtin_bit_cast(float, w[i] & 0xffff0000u);
  }
  return f;
}
template <class V, class B>
__device__ __forceinline__ void split3(V a, B& p0, B& p1, B& p2) {
  p0 = __builtin_convertvector(a, B);
  const V r1 = a - bf16_widen<V>(p0);
  p1 = __builtin_convertvector(r1, B);
  const V r2 = r1 - bf16_widen<V>(p1);
  p2 = __builtin_convertvector(r2, B);
}
// two-way split a = p0 + p1 (to ~2^-17 relative): the first two pieces of split3
template <class V, class B>
__device__ __forceinline__ void split2(V a, B& p0, B& p1) {
  p0 = __builtin_convertvector(a, B);
  p1 = __builtin_convertvector(a - bf16_widen<V>(p0), B);
}
__device__ __forceinline__ void split3(float a, __bf16& p0, __bf16& p1, __bf16& p2) {
  p0 = (__bf16)a;
  const float r1 = a - (float)p0;
  p1 = (__bf16)r1;
  p2 = (__bf16)(r1 - (float)p1);
}

// a / b: v_rcp and one Newton step on the quotient (about 1 ulp; IEEE division costs 3x the
// VALU issue, which the sweep's consumer waves share with the MFMA waves of their SIMD)
__device__ __forceinline__ float div_fast(float a, float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  const float q = a * r;
  return fmaf(fmaf(-b, q, a), r, q);
}

// phi(z) and phi'(z) of the h-side gradient's residual R = (phi(z) - tgt) phi'(z) (admm.py:302-312): the
// stored gates' activation (sig_pair / tanhf, as k_forward_t and k_resid_gx; ~1 ulp).  phi(z) - tgt is a
// difference of O(1) numbers that agree to ~1e-7 at C3, so phi's rounding is most of G (DESIGN.md
// section 2): with phi_fast's few ulps here the weights of the bench's 25 forced steps drifted 7x
// further from the fp64 trajectory than the reference's own (round 6); and where
// the stored h-side state is phi(z) itself (step 1) this activation gives R = 0 exactly, as the reference
template <bool TANH>
__device__ __forceinline__ void phi_acc(float z, float& phi, float& dphi) {
  if (TANH) {
    phi = tanhf(z);
    dphi = 1.f - phi * phi;
  } else {
    const SigPair sp = sig_pair(z);
    phi = sp.s;
    dphi = sp.s * sp.sc;
  }
}

// phi(z) and phi'(z) for the line-search paths (decisions only), from one v_exp and one
// v_rcp (a few ulp; these feed sums, not the stored state).  With w = |z| (sigmoid) or 2|z|
// (tanh), E = exp(-w), r = 1/(1+E):  sigma: phi = r or E r, phi' = E r^2;  tanh: |phi| =
// -expm1(-w) r (no cancellation near 0), phi' = 4 E r^2.
template <bool TANH>
__device__ __forceinline__ void phi_fast(float z, float& phi, float& dphi) {
  const float w = TANH ? 2.f * fabsf(z) : fabsf(z);
  const float E = __expf(-w);
  const float r = __builtin_amdgcn_rcpf(1.f + E);
  if (TANH) {
    phi = copysignf(-expm1_acc(-w) * r, z);
    dphi = 4.f * E * r * r;
  } else {
    phi = z >= 0.f ? r : E * r;
    dphi = E * r * r;
  }
}

// ----------------------------------------------------------------------------- reductions

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Deterministic block sum of one value per thread (fixed tree), result valid in thread 0.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red /* >= 4 entries of LDS */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  T r = 0;
  if (threadIdx.x == 0) r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// ----------------------------------------------------------------------------- MFMA tile engine
//
// C[BM x BN] += A[BM x K] * B[K x BN] over K in chunks of KC, fp32 in / fp32 accumulate
// (v_mfma_f32_32x32x2_f32: exact f32 products, k-ordered fma chain).
// Fragment maps (gfx950): A: lane l holds A[i = l&31][k = l>>5]; B: B[k = l>>5][j = l&31];
// C/D register r: row = (r&3) + 8*(r>>2) + 4*(l>>5), col = l&31.
//
// LDS images are k-major, As[k][m] and Bs[k][n], so every fragment read is a
// ds_read_b32 of 32 consecutive dwords per half-wave (conflict-free).  Global -> LDS
// staging is float4 and software-pipelined through registers: the loads of chunk c+1
// are issued before the MFMAs of chunk c and written to LDS after them.
//
// Operand source P supplies, per chunk, float4 loads of A and B:
//   P::A_ROW_MAJOR  true : A is [m][k] in memory -> float4 = 4 consecutive k of row m
//                   false: A is [k][m] in memory -> float4 = 4 consecutive m of row k
//   a4(m, k), b4(k, n): float4 at (m, k) / (k, n); zero outside the problem.
//   B is always [k][n] -> float4 = 4 consecutive n.

template <int BM, int BN, int WM, int WN, int KC, bool A_ROW = false>
struct Tile {
  static constexpr int MT = WM / 32, NT = WN / 32;
  static constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per workgroup");
  static_assert(KC % 8 == 0 && BM % 4 == 0 && BN % 4 == 0, "float4 staging");
  // A image: A_ROW -> As[m][KC+4] (rows 16-byte aligned; ds_read_b128 of 4 consecutive k is
  // conflict-free since (KC+4)/4 is odd); else As[k][BM+4].  B image: Bs[k][BN+4].
  static constexpr int AS = A_ROW ? KC + 4 : BM + 4, BS = BN + 4;
  static constexpr int A_FLOATS = A_ROW ? BM * AS : KC * AS;
  static constexpr int STAGE_FLOATS = A_FLOATS + KC * BS;
  static constexpr int LDS_FLOATS = 2 * STAGE_FLOATS;  // double-buffered
  static constexpr int A4 = BM * KC / 4, B4 = BN * KC / 4;
  static constexpr int A_PER = (A4 + kThreads - 1) / kThreads, B_PER = (B4 + kThreads - 1) / kThreads;
};

// XCD-aware block order (cdna_hip_programming.md T1): blocks are dealt round-robin over the
// 8 XCDs, so hand each XCD a contiguous range of logical tiles -- tiles that share operand
// rows then run on one L2.  Bijective for any grid size.
__device__ __forceinline__ int xcd_swizzle(int bid, int nb) {
  constexpr int NX = 8;
  const int q = nb / NX, r = nb % NX;
  const int x = bid % NX, i = bid / NX;
  // XCD x owns q (+1 if x < r) consecutive logical ids
  return x * q + (x < r ? x : r) + i;
}

// Raw buffer access (gfx9 descriptor word 3; aux 2 = nt).  Out-of-range offsets (>= the
// descriptor's byte count) load 0 and drop stores.
constexpr int kBufWord3 = 0x00020000;
constexpr int kAuxL2 = 1 | 16;   // buffer cache policy sc0 | sc1 (gfx940+): coherent at device scope, misses the L1
template <int AUX = 2>
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, AUX));
}
template <int AUX = 2>
__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX));
}
template <int AUX = 2>
__device__ __forceinline__ f32x2 buf_ld2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, AUX));
}
template <int AUX = 2>
__device__ __forceinline__ void buf_st2(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int, v), r,
                                        (int)off, 0, AUX);
}
template <int AUX = 2>
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r,
                                         (int)off, 0, AUX);
}
// store at off + soff (one descriptor serving several planes).  The plane offset goes into the
// VGPR offset, never the SGPR soffset field: LLVM assumes a >64-bit MUBUF store that names an
// soffset register has no store-data hazard and lets the next VALU overwrite the data VGPRs
// immediately, but on gfx950 such stores wrote clobbered data (the first ones of a back-to-back
// group, lane-dependent; DESIGN.md, "tgt from the sweep").  With soffset 0 the compiler inserts
// the wait states.
template <int AUX = 2>
__device__ __forceinline__ void buf_st4s(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r,
                                         (int)(off + soff), 0, AUX);
}
template <int AUX = 2>
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)off, 0, AUX);
}

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Two-phase B operand: a source with a BRaw type splits b4 into braw (the global loads,
// issued ahead of the MFMAs) and bfin (the element-wise transform, run at LDS-store time,
// after this chunk's MFMAs have been issued, so its VALU work overlaps the matrix pipe).
template <class P, class = void>
struct BRawOf {
  using type = float4;
  static constexpr bool two_phase = false;
};
template <class P>
struct BRawOf<P, std::void_t<typename P::BRaw>> {
  using type = typename P::BRaw;
  static constexpr bool two_phase = true;
};

template <int BM, int BN, int WM, int WN, int KC, class P>
struct Engine {
  using S = Tile<BM, BN, WM, WN, KC, P::A_ROW_MAJOR>;
  using BR = BRawOf<P>;
  float4 ra[S::A_PER];
  typename BR::type rb[S::B_PER];

  __device__ __forceinline__ void load(const P& p, int64_t m0, int64_t n0, int64_t kb) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < S::A_PER; ++i) {
      const int f = tid + i * kThreads;
      if (f < S::A4) {
        if (P::A_ROW_MAJOR) ra[i] = p.a4(m0 + f / (KC / 4), kb + 4 * (f % (KC / 4)));
        else ra[i] = p.a4(m0 + 4 * (f % (BM / 4)), kb + f / (BM / 4));
      }
    }
#pragma unroll
    for (int i = 0; i < S::B_PER; ++i) {
      const int f = tid + i * kThreads;
      if (f < S::B4) {
        if constexpr (BR::two_phase) rb[i] = p.braw(kb + f / (BN / 4), n0 + 4 * (f % (BN / 4)));
        else rb[i] = p.b4(kb + f / (BN / 4), n0 + 4 * (f % (BN / 4)));
      }
    }
  }

  __device__ __forceinline__ void store(const P& p, float* As, float* Bs) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < S::A_PER; ++i) {
      const int f = tid + i * kThreads;
      if (f < S::A4) {
        if (P::A_ROW_MAJOR)
          *reinterpret_cast<float4*>(&As[(f / (KC / 4)) * S::AS + 4 * (f % (KC / 4))]) = ra[i];
        else
          *reinterpret_cast<float4*>(&As[(f / (BM / 4)) * S::AS + 4 * (f % (BM / 4))]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < S::B_PER; ++i) {
      const int f = tid + i * kThreads;
      if (f < S::B4) {
        float4 v;
        if constexpr (BR::two_phase) v = p.bfin(rb[i]);
        else v = rb[i];
        *reinterpret_cast<float4*>(&Bs[(f / (BN / 4)) * S::BS + 4 * (f % (BN / 4))]) = v;
      }
    }
  }

  __device__ __forceinline__ static void compute(const float* As, const float* Bs,
                                                 f32x16 (&acc)[S::MT][S::NT]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm0 = (wave / S::WAVES_N) * WM, wn0 = (wave % S::WAVES_N) * WN;
    const int kh = lane >> 5, c = lane & 31;
    if (P::A_ROW_MAJOR) {
      // k-permuted: within each 8-k block, MFMA j uses k = {j (lanes 0-31), 4 + j (lanes 32-63)},
      // so one ds_read_b128 of A[m][8b + 4kh .. +3] feeds 4 MFMAs; B rows follow the same map.
#pragma unroll
      for (int kb = 0; kb < KC; kb += 8) {
        float4 a4[S::MT];
#pragma unroll
        for (int mi = 0; mi < S::MT; ++mi)
          a4[mi] = *reinterpret_cast<const float4*>(&As[(wm0 + mi * 32 + c) * S::AS + kb + 4 * kh]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float bv[S::NT];
#pragma unroll
          for (int ni = 0; ni < S::NT; ++ni) bv[ni] = Bs[(kb + 4 * kh + j) * S::BS + wn0 + ni * 32 + c];
#pragma unroll
          for (int mi = 0; mi < S::MT; ++mi) {
            const float av = j == 0 ? a4[mi].x : (j == 1 ? a4[mi].y : (j == 2 ? a4[mi].z : a4[mi].w));
#pragma unroll
            for (int ni = 0; ni < S::NT; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[ni], acc[mi][ni], 0, 0, 0);
          }
        }
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KC; kk += 2) {
        float av[S::MT], bv[S::NT];
#pragma unroll
        for (int mi = 0; mi < S::MT; ++mi) av[mi] = As[(kk + kh) * S::AS + wm0 + mi * 32 + c];
#pragma unroll
        for (int ni = 0; ni < S::NT; ++ni) bv[ni] = Bs[(kk + kh) * S::BS + wn0 + ni * 32 + c];
#pragma unroll
        for (int mi = 0; mi < S::MT; ++mi)
#pragma unroll
          for (int ni = 0; ni < S::NT; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
      }
    }
  }

  // Whole K loop: [k0, k1) in chunks of KC.  Two LDS stages: while the MFMAs consume
  // stage c%2, the global loads of chunk c+1 are in flight and then written to the other
  // stage; one barrier per chunk (the stage written at chunk c was last read at c-1).
  __device__ __forceinline__ void run(const P& p, int64_t m0, int64_t n0, int64_t k0, int64_t k1,
                                      f32x16 (&acc)[S::MT][S::NT], float* smem) {
    if (k0 >= k1) return;
    load(p, m0, n0, k0);
    store(p, smem, smem + S::A_FLOATS);
    __syncthreads();
    int stage = 0;
    for (int64_t kb = k0; kb < k1; kb += KC) {
      const bool more = kb + KC < k1;
      if (more) load(p, m0, n0, kb + KC);
      float* cur = smem + stage * S::STAGE_FLOATS;
      compute(cur, cur + S::A_FLOATS, acc);
      if (more) {
        float* nxt = smem + (stage ^ 1) * S::STAGE_FLOATS;
        store(p, nxt, nxt + S::A_FLOATS);
      }
      __syncthreads();
      stage ^= 1;
    }
  }
};

template <int MT, int NT>
__device__ __forceinline__ void zero_acc(f32x16 (&acc)[MT][NT]) {
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
}

}  // namespace admm
