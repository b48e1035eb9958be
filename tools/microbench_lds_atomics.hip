// Microbenchmark: LDS atomic throughput on gfx950 (random bins, histogram-like pattern).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_lds_atomics.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int PLANE = 257, NPL = 32;

template <int MODE>
__global__ __launch_bounds__(512) void k(const uint8_t* bins, int nrows, float* out, int* iout) {
  __shared__ float hf[NPL * PLANE * 2];
  __shared__ int hi_[NPL * PLANE * 2];
  for (int i = threadIdx.x; i < NPL * PLANE * 2; i += 512) { hf[i] = 0.f; hi_[i] = 0; }
  __syncthreads();
  const int half = threadIdx.x & 1;
  for (int r = blockIdx.x * 256 + (threadIdx.x >> 1); r < nrows; r += gridDim.x * 256) {
    const uint4 v = *(const uint4*)(bins + (size_t)r * 64 + half * 16);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t b = (w[j >> 2] >> ((j & 3) * 8)) & 0xff;
      const int off = (half * 16 + j) * PLANE + b;
      if constexpr (MODE == 0) { atomicAdd(&hf[off], 1.0f); atomicAdd(&hf[off + NPL * PLANE], 0.5f); }
      if constexpr (MODE == 1) { atomicAdd(&hi_[off], 1); atomicAdd(&hi_[off + NPL * PLANE], 3); }
      if constexpr (MODE == 2) { atomicAdd((unsigned long long*)&hi_[(off & ~1)], 1ull); }
      if constexpr (MODE == 3) { hf[off] += 1.0f; }   // racy plain RMW (upper bound)
      if constexpr (MODE == 4) { __hip_atomic_fetch_add(&hf[off], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                 __hip_atomic_fetch_add(&hf[off + NPL * PLANE], 0.5f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NPL * PLANE; i += 512) { out[blockIdx.x * NPL * PLANE + i] = hf[i]; iout[blockIdx.x * NPL * PLANE + i] = hi_[i]; }
}

int main() {
  const int nrows = 8 << 20;
  uint8_t* bins; float* out; int* iout;
  hipMalloc(&bins, (size_t)nrows * 64);
  hipMalloc(&out, 4096 * NPL * PLANE * 4);
  hipMalloc(&iout, 4096 * NPL * PLANE * 4);
  // random bytes
  uint8_t* h = (uint8_t*)malloc((size_t)nrows * 64);
  uint32_t s = 12345;
  for (size_t i = 0; i < (size_t)nrows * 64; ++i) { s = s * 1664525u + 1013904223u; h[i] = s >> 24; }
  hipMemcpy(bins, h, (size_t)nrows * 64, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const char* names[] = {"ds_add_f32 x2", "ds_add_u32 x2", "ds_add_u64 x1", "plain rmw", "hip_atomic_fetch_add wg-scope x2"};
  for (int grid : {512, 1024, 2048}) {
    for (int mode = 0; mode < 5; ++mode) {
      float best = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        switch (mode) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(512), 0, 0, bins, nrows, out, iout); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(512), 0, 0, bins, nrows, out, iout); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(512), 0, 0, bins, nrows, out, iout); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(512), 0, 0, bins, nrows, out, iout); break;
          case 4: hipLaunchKernelGGL(k<4>, dim3(grid), dim3(512), 0, 0, bins, nrows, out, iout); break;
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      const double upd = (double)nrows * 32;   // (row, feature) updates
      printf("grid %5d %-34s %8.3f ms  %8.2f G row-feature updates/s\n", grid, names[mode], best, upd / best / 1e6);
    }
  }
  return 0;
}
