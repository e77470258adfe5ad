// Exhaustive check (GPU box, one-off): is the library's sigmoid (sig_pair: expf, then 1/(1+e) by div_fast =
// v_rcp + one Newton step) bit-identical to the expf + IEEE-quotient form (sig_ieee below) for every finite
// float z?  Both pieces (sigma, 1 - sigma) are compared; also div_fast(1, d) against 1.f / d for every
// float d in [1, 2] (the denominators 1 + e take).  Prints the mismatch counts (profiles/r06f_sigcheck.txt).
//   hipcc -O3 --offload-arch=gfx950 -I../include -Iadmm-lstm_amd/admm_amd/csrc tools/sigcheck.hip -o tools/sigcheck
#include <hip/hip_runtime.h>
#include <cstdio>
#include "admm_dev.hpp"

using namespace admm;

__device__ __forceinline__ SigPair sig_ieee(float z) {
  const float e = expf(-fabsf(z));
  const float r = 1.0f / (1.0f + e);
  const float er = e * r;
  return z >= 0.f ? SigPair{r, er} : SigPair{er, r};
}

__global__ void k_sig(unsigned long long* bad, unsigned long long* first) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long nb = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
    const float z = __uint_as_float((unsigned)i);
    if (!isfinite(z)) continue;
    const SigPair a = sig_ieee(z), b = sig_pair(z);
    if (__float_as_uint(a.s) != __float_as_uint(b.s) || __float_as_uint(a.sc) != __float_as_uint(b.sc)) {
      ++nb;
      atomicMin(first, (unsigned long long)i);
    }
  }
  atomicAdd(bad, nb);
}

__global__ void k_div(unsigned long long* bad) {
  const unsigned lo = __float_as_uint(1.f), hi = __float_as_uint(2.f);
  unsigned long long nb = 0;
  for (unsigned u = lo + blockIdx.x * blockDim.x + threadIdx.x; u <= hi; u += gridDim.x * blockDim.x) {
    const float d = __uint_as_float(u);
    if (__float_as_uint(div_fast(1.f, d)) != __float_as_uint(1.f / d)) ++nb;
  }
  atomicAdd(bad, nb);
}

int main() {
  unsigned long long* d;
  if (hipMalloc(&d, 3 * sizeof(unsigned long long)) != hipSuccess) return 1;
  unsigned long long init[3] = {0, ~0ull, 0};
  (void)hipMemcpy(d, init, sizeof init, hipMemcpyHostToDevice);
  k_sig<<<8192, 256>>>(d, d + 1);
  k_div<<<1024, 256>>>(d + 2);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  unsigned long long h[3];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  printf("sig_ieee vs sig_pair (div_fast) over all finite floats: %llu mismatches (first at bits 0x%llx)\n", h[0],
         h[0] ? h[1] : 0ull);
  printf("div_fast(1, d) vs 1.f / d over all floats d in [1, 2]: %llu mismatches\n", h[2]);
  return 0;
}
