// Streaming-pattern calibration on gfx950: z[q][row][j] += x[row][:] . W[q][:][j]  (H=256, D=16)
// variants: rows per thread-iteration (1, 2, 4), grid size.  Reports GB/s of (read z + write z).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int H = 256, D = 16;

template <int RPI>
__global__ __launch_bounds__(256) void k_apply(int64_t BT, const float* __restrict__ x, const float* __restrict__ W,
                                               float* __restrict__ z) {
  __shared__ float wl[D * H];
  const int q = blockIdx.y;
  for (int i = threadIdx.x; i < D * H; i += 256) wl[i] = W[q * D * H + i];
  __syncthreads();
  float* zq = z + (int64_t)q * BT * H;
  const int rr = threadIdx.x / 64, c4 = threadIdx.x % 64, j = 4 * c4;
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t row0 = (int64_t)blockIdx.x * 4 + rr; row0 < BT; row0 += stride * RPI) {
    float4 zv[RPI];
    float4 xv[RPI][D / 4];
#pragma unroll
    for (int r = 0; r < RPI; ++r) {
      const int64_t row = row0 + r * stride;
      if (row < BT) {
        zv[r] = *reinterpret_cast<const float4*>(zq + row * H + j);
#pragma unroll
        for (int d4 = 0; d4 < D / 4; ++d4) xv[r][d4] = *reinterpret_cast<const float4*>(x + row * D + 4 * d4);
      }
    }
#pragma unroll
    for (int r = 0; r < RPI; ++r) {
      const int64_t row = row0 + r * stride;
      if (row >= BT) break;
      float xr[D] = {xv[r][0].x, xv[r][0].y, xv[r][0].z, xv[r][0].w, xv[r][1].x, xv[r][1].y, xv[r][1].z, xv[r][1].w,
                     xv[r][2].x, xv[r][2].y, xv[r][2].z, xv[r][2].w, xv[r][3].x, xv[r][3].y, xv[r][3].z, xv[r][3].w};
      float4 a = zv[r];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float4 w = *reinterpret_cast<const float4*>(wl + d * H + j);
        a.x += xr[d] * w.x; a.y += xr[d] * w.y; a.z += xr[d] * w.z; a.w += xr[d] * w.w;
      }
      *reinterpret_cast<float4*>(zq + row * H + j) = a;
    }
  }
}

__global__ void k_copy(int64_t n4, const float4* __restrict__ a, float4* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

// read-only stream with a reduction (trial-like): sum of 3 planes
template <bool NT>
__global__ __launch_bounds__(256) void k_read3(int64_t n4, const float4* __restrict__ a, const float4* __restrict__ b,
                                               const float4* __restrict__ c, float* out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 x, y, z;
    if (NT) {
      typedef float v4 __attribute__((ext_vector_type(4)));
      const v4 xa = __builtin_nontemporal_load(reinterpret_cast<const v4*>(a) + i);
      const v4 ya = __builtin_nontemporal_load(reinterpret_cast<const v4*>(b) + i);
      const v4 za = __builtin_nontemporal_load(reinterpret_cast<const v4*>(c) + i);
      x = make_float4(xa.x, xa.y, xa.z, xa.w); y = make_float4(ya.x, ya.y, ya.z, ya.w); z = make_float4(za.x, za.y, za.z, za.w);
    } else {
      x = a[i]; y = b[i]; z = c[i];
    }
    s += (x.x + y.y) * z.z + (x.w - y.x) * z.w + x.y * y.z + z.x;
  }
  if (s == 123.456f) out[0] = s;
}

template <bool NT>
__global__ void k_copy2(int64_t n4, const float4* __restrict__ a, float4* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const v4*>(a) + i), reinterpret_cast<v4*>(b) + i);
    else b[i] = a[i];
  }
}

int main() {
  const int64_t BT = 8192 * 32;
  float *x, *W, *z, *z2;
  hipMalloc(&x, BT * D * 4);
  hipMalloc(&W, 4 * D * H * 4);
  hipMalloc(&z, 4 * BT * H * 4);
  hipMalloc(&z2, 4 * BT * H * 4);
  hipMemset(x, 0, BT * D * 4); hipMemset(W, 0, 4 * D * H * 4); hipMemset(z, 0, 4 * BT * H * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = 2.0 * 4 * BT * H * 4;
  auto timeit = [&](auto launch, const char* name) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    const int R = 10;
    for (int i = 0; i < R; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.3f ms  %7.0f GB/s\n", name, ms / R, bytes / (ms / R * 1e-3) / 1e9);
  };
  timeit([&] { k_copy<<<8192, 256>>>(4 * BT * H / 4, (const float4*)z, (float4*)z2); }, "copy (ref)");
  {
    const int64_t n4 = BT * H / 4;   // one plane = 268 MB; 3 planes read = 805 MB (bytes scaled below)
    float* o; hipMalloc(&o, 16);
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
      char nm[64];
      auto t3 = [&](bool nt) {
        hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) {
          if (nt) k_read3<true><<<grid, 256>>>(n4, (const float4*)z, (const float4*)(z + BT * H), (const float4*)(z + 2 * BT * H), o);
          else k_read3<false><<<grid, 256>>>(n4, (const float4*)z, (const float4*)(z + BT * H), (const float4*)(z + 2 * BT * H), o);
        }
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("read3 %s grid=%-6d %8.3f ms  %7.0f GB/s\n", nt ? "nt " : "   ", grid, ms / 10, 3.0 * n4 * 16 / (ms / 10 * 1e-3) / 1e9);
      };
      t3(false); t3(true);
      (void)nm;
    }
    for (int grid : {2048, 8192, 32768}) {
      for (int nt = 0; nt < 2; ++nt) {
        hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) {
          if (nt) k_copy2<true><<<grid, 256>>>(4 * BT * H / 4, (const float4*)z, (float4*)z2);
          else k_copy2<false><<<grid, 256>>>(4 * BT * H / 4, (const float4*)z, (float4*)z2);
        }
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("copy %s grid=%-6d %8.3f ms  %7.0f GB/s\n", nt ? "nt" : "  ", grid, ms / 10, bytes / (ms / 10 * 1e-3) / 1e9);
      }
    }
  }
  for (int grid : {512, 1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, 64, "apply RPI=1 grid=%d", grid);
    timeit([&] { k_apply<1><<<dim3(grid, 4), 256>>>(BT, x, W, z); }, nm);
    snprintf(nm, 64, "apply RPI=2 grid=%d", grid);
    timeit([&] { k_apply<2><<<dim3(grid, 4), 256>>>(BT, x, W, z); }, nm);
    snprintf(nm, 64, "apply RPI=4 grid=%d", grid);
    timeit([&] { k_apply<4><<<dim3(grid, 4), 256>>>(BT, x, W, z); }, nm);
  }
  return 0;
}
