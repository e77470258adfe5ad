// ds_read_b64_tr_b16 lane map check (gfx950): LDS [4 rows][16 cols] bf16, value = 16*row + col.
// Lane 4q+p of each 16-lane group supplies the address of row q, cols 4p..4p+3; expect lane i of
// the group to receive column i of rows 0..3.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out) {
  __shared__ __attribute__((aligned(16))) __bf16 s[64];
  const int l = threadIdx.x;
  if (l < 64) s[l] = (__bf16)(float)(16 * (l / 16) + (l % 16));
  __syncthreads();
  const int g = l & 15, q = g >> 2, p = g & 3;
  bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(s + 16 * q + 4 * p));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (float)v[e];
}
int main() {
  float* d; hipMalloc(&d, 64 * 4 * 4);
  k<<<1, 64>>>(d);
  float h[256]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int e = 0; e < 4; ++e) if (h[l * 4 + e] != 16 * e + (l & 15)) ++bad;
  printf("trcheck: %s (lane 5: %g %g %g %g)\n", bad ? "MISMATCH" : "ok", h[20], h[21], h[22], h[23]);
  return bad != 0;
}
