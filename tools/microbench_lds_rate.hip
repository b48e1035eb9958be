// LDS atomic / store issue-rate ceiling on gfx950: conflict-free ds_add_u32 / ds_add_u64 /
// ds_write_b64 from 8-wave blocks with a 64 KiB LDS footprint (2 blocks per CU, as the GBDT
// histogram kernels), no global memory traffic inside the loop.  Prints lane-operations per clock
// per CU at the measured shader clock (s_memtime delta of one block / wall time).
//
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_lds_rate.hip -o /tmp/lds_rate && /tmp/lds_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int T = 512, ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(T) void lds_rate(unsigned long long* sink, long long* clk) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long h64[];
  uint32_t* h32 = (uint32_t*)h64;
  for (int i = threadIdx.x; i < 8192; i += T) h64[i] = 0;
  __syncthreads();
  const long long t0 = clock64();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = threadIdx.x * 2654435761u;
  for (int it = 0; it < ITERS; ++it) {
    x = x * 1664525u + 1013904223u;
    const uint32_t b = x >> 24;                          // random bin, lane-distinct bank
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (OP == 0) atomicAdd(&h32[(((b + j) & 255) << 6) | lane], 1u);
      else if constexpr (OP == 1) atomicAdd(&h64[(((b + j) & 127) << 6) | (lane ^ (w & 1))], 1ull);
      else h64[(((b + j) & 127) << 6) | lane] = x + j;
    }
  }
  __syncthreads();
  const long long t1 = clock64();
  if (threadIdx.x == 0) { sink[blockIdx.x] = h64[x & 8191]; if (blockIdx.x == 0) *clk = t1 - t0; }
}

int main() {
  int dev = 0, cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = cus * 2 * 8;
  unsigned long long* sink;
  long long* clk;
  hipMalloc(&sink, grid * 8);
  hipMalloc(&clk, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"ds_add_u32", "ds_add_u64", "ds_write_b64"};
  for (int op = 0; op < 3; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (op == 0) hipLaunchKernelGGL(lds_rate<0>, dim3(grid), dim3(T), 65536, 0, sink, clk);
      if (op == 1) hipLaunchKernelGGL(lds_rate<1>, dim3(grid), dim3(T), 65536, 0, sink, clk);
      if (op == 2) hipLaunchKernelGGL(lds_rate<2>, dim3(grid), dim3(T), 65536, 0, sink, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      long long c = 0;
      hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
      const double ops = (double)grid * T * ITERS * 16;
      const double per_cu_s = ops / cus / (ms * 1e-3);
      if (rep == 1)
        printf("%-14s %8.3f ms  %8.2f T lane-ops/s chip  %6.2f G/s per CU  block clocks %lld\n", names[op], ms,
               ops / (ms * 1e-3) / 1e12, per_cu_s / 1e9, c);
    }
  }
  return 0;
}
