// Memory-pattern study of the persistent sweep's consumer (no MFMA, trivial math): per
// (t, tile) every thread loads 11 state/dual planes ([B][T+1][H]) and stores 11 of them plus
// 8 [4][B*T][H] z / tgt planes, 16 B per access, one workgroup-wide barrier per tile, loads
// AHEAD tiles early -- the byte mix of k_sweep_rows (8.05 GB at C3).  The tile shape
// (ROWS x COLS, ROWS * COLS = 1024) decides how long the contiguous run of one row is per
// wave-instruction (COLS * 4 bytes).  Reports GB/s for each variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int B = 8192, T = 32, H = 256;
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ldnt(const float* p) { return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p)); }
__device__ __forceinline__ void stnt(float* p, f4 v) { __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p)); }

struct Planes {
  float* S[6];
  float* L[6];
  float* Z[4];
  float* G[4];
};

// ZI: the eight library planes (z cache, tgt) interleaved as one [B*T][8][H] buffer (P.Z[0]),
// so that the 8 stores of one point land in one 8-KB row instead of 8 planes
template <int ROWS, int AHEAD, bool ZI = false>
__global__ __launch_bounds__(256) void k_pat(Planes P) {
  constexpr int COLS = 1024 / ROWS, NT = H / COLS, TPR = COLS / 4;
  const int ct = threadIdx.x, row = ct / TPR, c4 = (ct % TPR) * 4;
  const int64_t b = (int64_t)blockIdx.x * ROWS + row;
  const int64_t rs = (int64_t)(T + 1) * H;
  struct Ld { f4 v[11]; };
  auto load = [&](int t, int n, Ld& l) {
    const int64_t o = b * rs + (int64_t)t * H + n * COLS + c4;
    l.v[0] = ldnt(P.S[1] + o); l.v[1] = ldnt(P.S[2] + o); l.v[2] = ldnt(P.S[4] + o); l.v[3] = ldnt(P.S[5] + o);
    l.v[4] = *reinterpret_cast<const f4*>(P.S[4] + o - H);
    for (int k = 0; k < 6; ++k) l.v[5 + k] = ldnt(P.L[k] + o);
  };
  Ld ring[AHEAD + 1];
  int tt = 1, nn = 0;
  for (int a = 0; a < AHEAD; ++a) {
    load(tt, nn, ring[a]);
    if (++nn == NT) { nn = 0; ++tt; }
  }
  int s = 0;
  for (int t = 1; t <= T; ++t)
    for (int n = 0; n < NT; ++n, ++s) {
      if (tt <= T) {
        load(tt, nn, ring[(s + AHEAD) % (AHEAD + 1)]);
        if (++nn == NT) { nn = 0; ++tt; }
      }
      const Ld& l = ring[s % (AHEAD + 1)];
      f4 acc = l.v[0];
#pragma unroll
      for (int k = 1; k < 11; ++k) acc = acc * 0.5f + l.v[k];
      const int64_t o = b * rs + (int64_t)t * H + n * COLS + c4;
      const int64_t e = (b * T + (t - 1)) * H + n * COLS + c4;
      for (int k = 0; k < 4; ++k) stnt(P.S[k] + o, acc + (float)k);
      *reinterpret_cast<f4*>(P.S[4] + o) = acc;
      *reinterpret_cast<f4*>(P.S[5] + o) = acc;
      for (int k = 0; k < 5; ++k) stnt(P.L[k] + o, acc - (float)k);
      if (ZI) {
        const int64_t ei = (b * T + (t - 1)) * 8 * H + n * COLS + c4;
        for (int k = 0; k < 4; ++k) stnt(P.Z[0] + ei + (2 * k) * H, acc * (float)k);
        for (int k = 0; k < 4; ++k) stnt(P.Z[0] + ei + (2 * k + 1) * H, acc * (float)(k + 2));
      } else {
        for (int k = 0; k < 4; ++k) stnt(P.Z[k] + e, acc * (float)k);
        for (int k = 0; k < 4; ++k) stnt(P.G[k] + e, acc * (float)(k + 2));
      }
      __syncthreads();
    }
}

// Pure streaming reference with the same byte mix (11 reads : 19 writes), fully sequential.
__global__ __launch_bounds__(256) void k_seq(Planes P, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t o = 4 * i;
    f4 acc = ldnt(P.S[1] + o);
    acc = acc + ldnt(P.S[2] + o) + ldnt(P.S[4] + o) + ldnt(P.S[5] + o) + ldnt(P.S[0] + o);
    for (int k = 0; k < 6; ++k) acc = acc * 0.5f + ldnt(P.L[k] + o);
    for (int k = 0; k < 6; ++k) stnt(P.S[k] + o, acc + (float)k);
    for (int k = 0; k < 5; ++k) stnt(P.L[k] + o, acc - (float)k);
    for (int k = 0; k < 4; ++k) stnt(P.Z[k] + o, acc * (float)k);
    for (int k = 0; k < 4; ++k) stnt(P.G[k] + o, acc * (float)(k + 2));
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  Planes P;
#define ATTR(RR, AA) CK(hipFuncSetAttribute((const void*)k_pat<RR, AA>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024))
  ATTR(32, 1); ATTR(32, 2); ATTR(16, 1); ATTR(16, 2); ATTR(8, 1); ATTR(8, 2); ATTR(4, 1); ATTR(4, 2);
  CK(hipFuncSetAttribute((const void*)k_pat<32, 1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
  CK(hipFuncSetAttribute((const void*)k_pat<16, 1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
  const size_t plane = (size_t)B * (T + 1) * H, zpl = (size_t)B * T * H;
  for (int k = 0; k < 6; ++k) {
    CK(hipMalloc(&P.S[k], plane * 4));
    CK(hipMalloc(&P.L[k], plane * 4));
    CK(hipMemset(P.S[k], 0, plane * 4));
    CK(hipMemset(P.L[k], 0, plane * 4));
  }
  for (int k = 0; k < 4; ++k) {
    CK(hipMalloc(&P.Z[k], (k == 0 ? 8 : 1) * zpl * 4));   // Z[0] also holds the interleaved image (ZI)
    CK(hipMalloc(&P.G[k], zpl * 4));
  }
  const double bytes = 30.0 * zpl * 4;   // 11 loads + 19 stores per point
  const int reps = 5;
  auto report = [&](const char* name, float ms) { printf("%-28s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6); };
  report("seq (1 pass, grid 4096)", timeit([&] { k_seq<<<4096, 256>>>(P, (int64_t)zpl / 4); }, reps));
  report("seq (1 pass, grid 1024)", timeit([&] { k_seq<<<1024, 256>>>(P, (int64_t)zpl / 4); }, reps));
  // dynamic LDS only limits residency: 100 KB -> 1 workgroup (4 waves) per CU, 60 KB -> 2
  // separate vs interleaved library planes, alternating rounds
  for (int round = 0; round < 3; ++round)
    for (int R : {32, 16})
      for (int zi : {0, 1})
        for (int lds : {100 * 1024, 60 * 1024, 0}) {
          char name[96];
          snprintf(name, sizeof name, "r%d tile %2d rows, %s, %s", round, R, zi ? "z/tgt interleaved" : "z/tgt planes",
                   lds > 80000 ? "1 WG/CU" : lds ? "2 WG/CU" : "max WG/CU");
          auto go = [&] {
            if (R == 32 && zi) k_pat<32, 1, true><<<B / 32, 256, lds>>>(P);
            if (R == 32 && !zi) k_pat<32, 1><<<B / 32, 256, lds>>>(P);
            if (R == 16 && zi) k_pat<16, 1, true><<<B / 16, 256, lds>>>(P);
            if (R == 16 && !zi) k_pat<16, 1><<<B / 16, 256, lds>>>(P);
          };
          report(name, timeit(go, reps));
        }
  for (int R : {32, 16, 8, 4})
    for (int A : {1, 2})
      for (int lds : {100 * 1024, 60 * 1024, 0}) {
        char name[96];
        snprintf(name, sizeof name, "tile %2d rows, ahead %d, %s", R, A, lds > 80000 ? "1 WG/CU" : lds ? "2 WG/CU" : "max WG/CU");
        auto go = [&] {
#define L(RR, AA) if (R == RR && A == AA) k_pat<RR, AA><<<B / RR, 256, lds>>>(P)
          L(32, 1); L(32, 2); L(16, 1); L(16, 2); L(8, 1); L(8, 2); L(4, 1); L(4, 2);
        };
        report(name, timeit(go, reps));
      }
  CK(hipDeviceSynchronize());
  return 0;
}
