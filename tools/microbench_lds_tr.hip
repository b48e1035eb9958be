// LDS read throughput: ds_read_b128 vs ds_read_b64_tr_b16 (gfx950), conflict-free addresses.
// hipcc --offload-arch=gfx950 -O3 tools/microbench_lds_tr.hip -o /tmp/mb_lds && /tmp/mb_lds
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int MODE>
__global__ __launch_bounds__(512) void k(unsigned* out, int iters) {
  __shared__ __attribute__((aligned(16))) char smem[65536];
  for (int i = threadIdx.x; i < 65536 / 4; i += 512) ((unsigned*)smem)[i] = i * 2654435761u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned acc = 0;
  // b128: lane reads 16 B at (wid*1024 + lane*16) (+ rotating base): 64 lanes x 16 B = 1 KiB, conflict-free
  // tr_b64: lane reads 8 B at (wid*512 + lane*8): 64 lanes x 8 B = 512 B
  for (int it = 0; it < iters; ++it) {
    const int base = (it * 4096) & 32767;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (MODE == 0) {
        u32x4 v = *(const u32x4*)(smem + ((base + u * 8192 + wid * 1024 + lane * 16) & 65535));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      } else if constexpr (MODE == 1) {
        s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + ((base + u * 4096 + wid * 512 + lane * 8) & 65535)));
        acc ^= (unsigned)v[0] ^ (unsigned)v[1] ^ (unsigned)v[2] ^ (unsigned)v[3];
      } else {
        unsigned long long v = *(const unsigned long long*)(smem + ((base + u * 4096 + wid * 512 + lane * 8) & 65535));
        acc ^= (unsigned)v ^ (unsigned)(v >> 32);
      }
    }
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main() {
  unsigned* d;
  const int blocks = 256 * 2, iters = 4096;
  hipMalloc(&d, blocks * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[3] = {"ds_read_b128", "ds_read_b64_tr_b16", "ds_read_b64"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 3; ++m) {
      hipEventRecord(e0);
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(512), 0, 0, d, iters);
      else if (m == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(512), 0, 0, d, iters);
      else hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(512), 0, 0, d, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double bytes = (double)blocks * 8 * iters * 8 * (m == 0 ? 1024 : 512);
      const double insts = (double)blocks * 8 * iters * 8;
      printf("%-20s %8.3f ms  %8.1f TB/s LDS  %6.1f B/clk/CU @2.4GHz  %.2f G wave-inst/s\n", names[m], ms,
             bytes / ms / 1e9, bytes / (ms * 1e-3) / 256 / 2.4e9, insts / ms / 1e6);
    }
  return 0;
}
