// K16: stable LSD radix sort of (64-bit key, int32 row) pairs on MI355X (gfx950).
//
// Replaces the sort behind the reference's eval ORDER BY (P/Eval.pig:38-39) and the ordered walk
// of ConfusionMatrix.bufferedComputeConfusionMatrixAndPerformance (J/core/ConfusionMatrix.java:
// 276-507): every rank orders its scores (descending, stable = row order on ties) before the
// k-way merge of the EvalScore runs and before the cumulative confusion sweep.
//
// MI355X design:
//   * keys: fp64 scores mapped to order-preserving uint64 (descending: complemented), 8-bit
//     digits, one upfront pass builds all 8 digit histograms so passes whose digit is constant
//     (the high exponent bytes of scores in [0, 1000]) are skipped;
//   * a pass = count (per-tile digit counts, digit-major [256][tiles]) -> exclusive scan of the
//     counts (reduce / scan-partials / scan, all in this file) -> scatter;
//   * stable tile ranking without atomics: a 4096-key tile is 4 waves x 16 slots x 64 lanes in key
//     order; per slot a wave finds the lanes with its digit by 8 ballots (match-any), ranks by
//     popcount below the lane, and the group's highest lane bumps the wave's private LDS digit
//     counter; waves then prefix their per-digit totals.  Tile order = (wave, slot, lane) = key
//     order, so equal keys keep their input order.
#include "common.h"

namespace {

constexpr int RT = 256;                 // threads per tile block (4 waves)
constexpr int SLOTS = 16;               // 64-key slots per wave
constexpr int TILE = RT * SLOTS;        // 4096 keys per tile
constexpr int NDIG = 256;

__device__ __forceinline__ uint64_t desc_key(double x) {
  uint64_t u = __double_as_longlong(x);
  // NaN scores sort with -inf (last): an integer test (a float x != x may be folded away)
  if ((u & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) u = 0xfff0000000000000ull;
  if (u == 0x8000000000000000ull) u = 0;               // -0.0 ties with +0.0 (stable row order)
  u = (u >> 63) ? ~u : (u | 0x8000000000000000ull);   // ascending order of x
  return ~u;                                           // descending
}

__global__ __launch_bounds__(RT) void key_init_kernel(const double* x, long n, uint64_t* keys, int* vals,
                                                      unsigned int* ghist) {
  __shared__ unsigned int h[8][NDIG];
  for (int i = threadIdx.x; i < 8 * NDIG; i += RT) (&h[0][0])[i] = 0;
  __syncthreads();
  const long base = (long)blockIdx.x * TILE;
  for (int s = 0; s < SLOTS; ++s) {
    const long i = base + (long)s * RT + threadIdx.x;
    if (i < n) {
      const uint64_t k = desc_key(x[i]);
      keys[i] = k;
      vals[i] = (int)i;
#pragma unroll
      for (int b = 0; b < 8; ++b) atomicAdd(&h[b][(k >> (8 * b)) & 0xff], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 8 * NDIG; i += RT) {
    const unsigned int c = (&h[0][0])[i];
    if (c) atomicAdd(ghist + i, c);
  }
}

// per-tile digit counts of byte `shift` -> cnt[d * ntiles + tile]
__global__ __launch_bounds__(RT) void count_kernel(const uint64_t* keys, long n, int shift, int ntiles,
                                                   unsigned int* cnt) {
  __shared__ unsigned int h[NDIG];
  h[threadIdx.x] = 0;
  __syncthreads();
  const long base = (long)blockIdx.x * TILE;
  for (int s = 0; s < SLOTS; ++s) {
    const long i = base + (long)s * RT + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xff], 1u);
  }
  __syncthreads();
  cnt[(long)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of m uint32 counts in three launches: block sums, scan of the sums, block scans
constexpr int ST = 256, SPT = 16, SBLK = ST * SPT;   // 4096 entries per scan block

__device__ __forceinline__ unsigned int block_excl_scan(unsigned int v, unsigned int* sh, unsigned int& total) {
  // v: this thread's value; returns the exclusive prefix over threads
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  unsigned int wo = 0;
  for (int k = 0; k < w; ++k) wo += sh[k];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return wo + x - v;
}

__global__ __launch_bounds__(ST) void scan_reduce_kernel(const unsigned int* in, long m, unsigned int* part) {
  __shared__ unsigned int sh[4];
  const long base = (long)blockIdx.x * SBLK;
  unsigned int s = 0;
  for (int k = 0; k < SPT; ++k) {
    const long i = base + (long)threadIdx.x * SPT + k;
    if (i < m) s += in[i];
  }
  unsigned int tot;
  block_excl_scan(s, sh, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(ST) void scan_partials_kernel(unsigned int* part, int nb) {
  __shared__ unsigned int sh[4];
  unsigned int carry = 0;
  for (int b0 = 0; b0 < nb; b0 += ST) {
    const int i = b0 + threadIdx.x;
    const unsigned int v = i < nb ? part[i] : 0u;
    unsigned int tot;
    const unsigned int ex = block_excl_scan(v, sh, tot);
    if (i < nb) part[i] = carry + ex;
    carry += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(ST) void scan_final_kernel(const unsigned int* in, long m, const unsigned int* part,
                                                        unsigned int* out) {
  __shared__ unsigned int sh[4];
  const long base = (long)blockIdx.x * SBLK;
  unsigned int v[SPT], s = 0;
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const long i = base + (long)threadIdx.x * SPT + k;
    v[k] = i < m ? in[i] : 0u;
    s += v[k];
  }
  unsigned int tot;
  unsigned int run = part[blockIdx.x] + block_excl_scan(s, sh, tot);
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const long i = base + (long)threadIdx.x * SPT + k;
    if (i < m) out[i] = run;
    run += v[k];
  }
}

// stable scatter of one 4096-key tile by digit `shift` (see the header)
template <bool VAL>
__global__ __launch_bounds__(RT) void scatter_kernel(const uint64_t* keys, const int* vals, long n, int shift,
                                                     int ntiles, const unsigned int* off, uint64_t* okeys,
                                                     int* ovals) {
  __shared__ unsigned int wc[4][NDIG];        // per-wave running digit counts
  __shared__ unsigned int tile_off[NDIG];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * NDIG; i += RT) (&wc[0][0])[i] = 0;
  tile_off[threadIdx.x] = off[(long)threadIdx.x * ntiles + blockIdx.x];
  __syncthreads();
  const long base = (long)blockIdx.x * TILE + (long)w * (SLOTS * 64);
  const uint64_t lt = (1ull << lane) - 1;
  uint64_t k[SLOTS];
  int v[SLOTS];
  unsigned int r[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const long i = base + s * 64 + lane;
    const bool ok = i < n;
    k[s] = ok ? keys[i] : ~0ull;
    if constexpr (VAL) v[s] = ok ? vals[i] : 0;
    const unsigned int d = (unsigned int)((k[s] >> shift) & 0xff);
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    const unsigned int below = __popcll(peers & lt);
    r[s] = wc[w][d] + below;                          // the group's count before this slot
    // the group's highest lane publishes the new count (one writer per digit and wave)
    if (ok && (peers >> lane) == 1ull) wc[w][d] += below + 1;
    __builtin_amdgcn_s_waitcnt(0xc07f);               // lgkmcnt(0): the wave sees its own LDS update
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // per digit: prefix of the wave totals (thread = digit)
  {
    const int d = threadIdx.x;
    unsigned int acc = tile_off[d];
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const unsigned int c = wc[ww][d];
      wc[ww][d] = acc;
      acc += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const long i = base + s * 64 + lane;
    if (i < n) {
      const unsigned int d = (unsigned int)((k[s] >> shift) & 0xff);
      const unsigned int p = wc[w][d] + r[s];
      okeys[p] = k[s];
      if constexpr (VAL) ovals[p] = v[s];
    }
  }
}

}  // namespace

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

SHIFU_API long shifu_sort_ws(long n) {
  // bytes of scratch: 2 key buffers + 2 value buffers + counts + offsets + partials + 8x256 hist
  const long nt = (n + TILE - 1) / TILE, m = nt * NDIG, nb = (m + SBLK - 1) / SBLK;
  return 2 * n * 8 + 2 * n * 4 + 2 * m * 4 + nb * 4 + 8 * NDIG * 4 + 256;
}

// Stable descending sort of x (fp64, n <= 2^31 - 1): order[i] = row of the i-th largest score,
// skeys[i] (nullable) = the sorted keys' scores order.  ws: shifu_sort_ws(n) bytes of device
// scratch; hist_host (nullable, 8 x 256 uint32): the upfront digit histograms are copied there.
SHIFU_API int shifu_sort_desc(const double* x, long n, int* order, void* ws, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > 0x7fffffffL) return -1;
  const long nt = (n + TILE - 1) / TILE, m = nt * NDIG, nb = (m + SBLK - 1) / SBLK;
  char* p = (char*)ws;
  uint64_t* k0 = (uint64_t*)p; p += n * 8;
  uint64_t* k1 = (uint64_t*)p; p += n * 8;
  int* v0 = (int*)p; p += n * 4;
  int* v1 = (int*)p; p += n * 4;
  unsigned int* cnt = (unsigned int*)p; p += m * 4;
  unsigned int* off = (unsigned int*)p; p += m * 4;
  unsigned int* part = (unsigned int*)p; p += nb * 4;
  unsigned int* gh = (unsigned int*)p;
  CHECK_HIP(hipMemsetAsync(gh, 0, 8 * NDIG * 4, stream));
  hipLaunchKernelGGL(key_init_kernel, dim3((unsigned)nt), dim3(RT), 0, stream, x, n, k0, v0, gh);
  CHECK_HIP(hipGetLastError());
  unsigned int h[8 * NDIG];
  CHECK_HIP(hipMemcpyAsync(h, gh, sizeof h, hipMemcpyDeviceToHost, stream));
  CHECK_HIP(hipStreamSynchronize(stream));
  for (int b = 0; b < 8; ++b) {
    bool constant = false;
    for (int d = 0; d < NDIG; ++d)
      if (h[b * NDIG + d] == (unsigned int)n) constant = true;
    if (constant) continue;                              // every key has the same digit: skip the pass
    const int shift = 8 * b;
    hipLaunchKernelGGL(count_kernel, dim3((unsigned)nt), dim3(RT), 0, stream, k0, n, shift, (int)nt, cnt);
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(ST), 0, stream, cnt, m, part);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(ST), 0, stream, part, (int)nb);
    hipLaunchKernelGGL(scan_final_kernel, dim3((unsigned)nb), dim3(ST), 0, stream, cnt, m, part, off);
    hipLaunchKernelGGL((scatter_kernel<true>), dim3((unsigned)nt), dim3(RT), 0, stream, k0, v0, n, shift, (int)nt,
                       off, k1, v1);
    CHECK_HIP(hipGetLastError());
    uint64_t* tk = k0; k0 = k1; k1 = tk;
    int* tv = v0; v0 = v1; v1 = tv;
  }
  CHECK_HIP(hipMemcpyAsync(order, v0, n * 4, hipMemcpyDeviceToDevice, stream));
  return 0;
}
