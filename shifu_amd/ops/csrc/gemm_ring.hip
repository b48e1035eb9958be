// Ring-pipelined MFMA GEMM engine for the MLP weight gradient (gfx950 / CDNA4).
//
//   G[n][k] += sum_m D[m][n] X[m][k]        (TN: both operands are row-major [rows][cols] and the
//                                            reduction runs over rows; SubGradient.java:224-311 sums
//                                            the same per-record products one record at a time)
//
// Why a new engine (profiles/r1d/pmc_wgrad_128_vs_8ph.txt, profiles/r2/): the row slabs of D and X
// stream from HBM, and at ~1.3 PF a 256 x 256 tile needs ~40 GB/s per CU of operand fetch.  By
// Little's law that needs ~100 KB in flight per CU at the ~1.1 us loaded HBM latency; the
// two-buffer 8-phase schedule keeps 32-48 KB in flight (SQ_WAIT_ANY 6.6x the 128^2 kernel's) and
// the 128^2 two-barrier kernel is capped by its structure (~700 TF).  Here:
//   * block = 512 threads (8 waves, 2 per SIMD), output tile 256 (n) x 256 (k); wave tile
//     128 x 64 (waves 0-3: n rows 0-127, waves 4-7: 128-255);
//   * the reduction axis is cut into 32-row k-steps; LDS holds a ring of 5 slots (32 KiB each:
//     D image [32 rows][256 n] + X image [32 rows][256 k], 160 KiB), filled by LDS-DMA
//     (global_load_lds_dwordx4) FOUR k-steps ahead, so ~3.5 slots (~112 KB) are in flight;
//   * every k-step is one LD segment (DMA issue 4 steps ahead + 24 ds_read_b64_tr_b16 fragment
//     reads + counted waits) and one MMA segment (32 x mfma_f32_16x16x32_bf16), separated by
//     raw s_barriers; waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave's
//     MFMAs overlap its partner's reads and DMA issue (cdna_hip_programming.md §5 8-phase idea);
//   * image rows are 512 B; 16-B chunk c of row r sits at c ^ f(r), f(r) = ((r & 3) << 2) |
//     (((r >> 3) & 1) << 1): the 8 rows one 32-lane half of a transposed read touches land on 8
//     distinct 32-B bank slots (conflict-free).  The DMA applies the swizzle on the SOURCE address
//     (lane-linear LDS destination);
//   * output: per-split fp32 partial slabs + a fixed-order reduction kernel -> the gradient is
//     bitwise reproducible run to run (no float atomics), unlike the split-K atomics of the
//     128^2 kernel.
//
// Schedule (per wave; "lag" = waves 4-7, which execute one extra barrier up front):
//   prologue: DMA k-steps 0..3; vmcnt(12) (own step-0 DMAs landed); BAR; [lag: BAR]
//   step t:   LD:  DMA step t+4 into ring slot (t+4)%5 (= the slot of step t-1); read the
//                  fragments of step t; vmcnt(12) (own DMAs of step t+1 landed: the 3 younger
//                  steps t+2..t+4 stay in flight); lgkmcnt(0); BAR
//             MMA: 32 MFMAs; BAR
//   epilogue: [lead: BAR]; vmcnt(0)
// RAW: step t+1's DMAs are waited for by EVERY wave before the barrier that precedes any read of
// them (lead: before the MMA(t) barrier pair ends, lag: in its LD(t)).  WAR: slot (t-1)%5 is
// refilled in LD(t); every wave's reads of step t-1 completed (lgkmcnt(0)) before the barrier
// that ends its LD(t-1), which precedes every wave's LD(t).
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int RG_T = 512;
constexpr int RG_NSLOT = 5;
constexpr int RG_IMG = 32 * 256 * 2;          // 16 KiB: [32 rows][256 cols] bf16
constexpr int RG_SLOT = 2 * RG_IMG;           // D image + X image
constexpr int RG_LDS = RG_NSLOT * RG_SLOT;    // 160 KiB

__device__ __forceinline__ int rg_xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ds_read_b64_tr_b16 as inline asm: through the builtin, hipcc treats the read as aliasing every
// in-flight LDS-DMA and emits s_waitcnt vmcnt(0) in front of it, draining the whole ring every
// k-step (the cause of the r1 8-phase TN kernel's waits).  The asm form is invisible to the
// waitcnt pass, so the kernel counts lgkmcnt itself (lgkmcnt(0) before every barrier) and the
// sched_barrier after each wait keeps the MFMAs behind it (cdna_hip_programming.md §5.4 rule 18).
__device__ __forceinline__ s16x4 rg_tr_read(uint32_t lds_addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr));
  return v;
}

__device__ __forceinline__ int rg_f(int r) { return ((r & 3) << 2) | (((r >> 3) & 1) << 1); }
// byte offset of the 8-byte quad holding columns col..col+3 (col % 4 == 0) of image row r
__device__ __forceinline__ int rg_off(int r, int col) {
  return r * 512 + (((col >> 3) ^ rg_f(r)) << 4) + ((col & 4) << 1);
}

struct RingTNArgs {
  const bf16_t* D; long ldd;   // [M, ldd] deltas (columns >= Nv are ignored)
  const bf16_t* X; long ldx;   // [M, ldx] layer inputs
  float* slab;                 // [S][NT * 256][KT * 256] fp32 partial sums
  int nsteps, S, NT, KT;       // nsteps = whole 32-row k-steps; split s takes steps s, s+S, ...
};

__global__ __launch_bounds__(RG_T, 2) void ring_tn_kernel(RingTNArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntiles = p.NT * p.KT;
  const int wg = rg_xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, tile = wg % ntiles;
  const int n0 = (tile / p.KT) * 256, k0 = (tile % p.KT) * 256;
  const int T = (p.nsteps - split + p.S - 1) / p.S;      // host guarantees S <= nsteps -> T >= 1
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 2, wk = wid & 3;
  const bool lag = wid >= 4;

  // ---- LDS-DMA sources: thread instr i (0/1) per image fills LDS bytes (i*8 + wid)*1024 + lane*16
  const bf16_t* srcD[2];
  const bf16_t* srcX[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int P = (i * 8 + wid) * 1024 + lane * 16;
    const int row = P >> 9, lc = ((P >> 4) & 31) ^ rg_f(row);
    const long r = (long)split * 32 + row;
    srcD[i] = p.D + r * p.ldd + min(n0 + lc * 8, (int)p.ldd - 8);
    srcX[i] = p.X + r * p.ldx + min(k0 + lc * 8, (int)p.ldx - 8);   // clamped columns: outputs dropped
  }
  const long stepD = (long)p.S * 32 * p.ldd, stepX = (long)p.S * 32 * p.ldx;
  auto dma = [&](int t, int slot) {
    const long tc = min(t, T - 1);             // steps past the end re-read the last one (never read)
    char* base = smem + slot * RG_SLOT + wid * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcD[i] + tc * stepD), (lds_ptr_t)(base + i * 8192), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcX[i] + tc * stepX), (lds_ptr_t)(base + RG_IMG + i * 8192), 16, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads (T10): group g = lane >> 4 supplies rows 8g + tq (+4), lane 4tq+tp
  // the quad at columns cb + 4tp; lane receives column cb + (lane & 15) of those rows
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int r_lo = 8 * g + tq, r_hi = r_lo + 4;
  bf16x8 af[8], bfr[4];
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  auto frag = [&](uint32_t img, int cb) {
    const s16x4 lo = rg_tr_read(img + rg_off(r_lo, cb + 4 * tp));
    const s16x4 hi = rg_tr_read(img + rg_off(r_hi, cb + 4 * tp));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

#define RG_BAR() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); \
                      __builtin_amdgcn_sched_barrier(0); } while (0)

  dma(0, 0); dma(1, 1); dma(2, 2); dma(3, 3);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  RG_BAR();
  if (lag) RG_BAR();

  int slot = 0, dslot = 4;
  for (int t = 0; t < T; ++t) {
    // ---- LD segment
    dma(t + 4, dslot);
    const uint32_t Dimg = lds0 + slot * RG_SLOT;
    const uint32_t Ximg = Dimg + RG_IMG;
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = frag(Ximg, wk * 64 + j * 16);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag(Dimg, wn * 128 + i * 16);
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    RG_BAR();
    // ---- MMA segment
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    RG_BAR();
    slot = slot == RG_NSLOT - 1 ? 0 : slot + 1;
    dslot = dslot == RG_NSLOT - 1 ? 0 : dslot + 1;
  }
  if (!lag) RG_BAR();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef RG_BAR

  // ---- epilogue: this split's partial tile -> slab (acc[i][j][r]: n = 16i + 4(lane>>4) + r,
  //      k = 16j + (lane & 15) within the wave tile)
  const long lds = (long)p.KT * 256;
  float* out = p.slab + (size_t)split * ((size_t)p.NT * 256) * lds;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wn * 128 + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + wk * 64 + j * 16 + (lane & 15);
        out[(size_t)n * lds + k] = acc[i][j][r];
      }
    }
}

// G[n][k] += sum_s slab[s][n][k] in fixed split order (n < Nv, k < Kx; Kx % 8 == 0)
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, int S, long sstride,
                                                          long lds, float* __restrict__ G, long ldg, int Nv, int Kx) {
  const long nq = (long)Nv * (Kx / 4);
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < nq; q += (long)gridDim.x * 256) {
    const int n = (int)(q / (Kx / 4)), k = (int)(q % (Kx / 4)) * 4;
    float4 a = *(const float4*)(G + (size_t)n * ldg + k);
    const float* s = slab + (size_t)n * lds + k;
    for (int i = 0; i < S; ++i) {
      const float4 v = *(const float4*)(s + (size_t)i * sstride);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    *(float4*)(G + (size_t)n * ldg + k) = a;
  }
}

// tail rows (< 32) that do not fill a ring k-step: one thread per (n, k), fixed row order
__global__ __launch_bounds__(256) void tail_tn_kernel(const bf16_t* __restrict__ D, long ldd,
                                                      const bf16_t* __restrict__ X, long ldx, int rows,
                                                      float* __restrict__ G, long ldg, int Nv, int Kx) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= (long)Nv * Kx) return;
  const int n = (int)(q / Kx), k = (int)(q % Kx);
  float a = 0.f;
  for (int m = 0; m < rows; ++m) a += bf2f(D[(size_t)m * ldd + n]) * bf2f(X[(size_t)m * ldx + k]);
  G[(size_t)n * ldg + k] += a;
}

}  // namespace

static int rg_splits(int nsteps, int ntiles) {
  int S = 256 / ntiles;                      // one 160-KiB block per CU on the 256 CUs
  if (S < 1) S = 1;
  if (S > nsteps) S = nsteps;
  return S;
}

// Workspace (bytes) shifu_wgrad_ring needs for these shapes (0: the shape takes the fallback).
SHIFU_API long shifu_wgrad_ring_ws(int M, int Nv, int Kx) {
  if (Kx % 8 || M < 32 || Nv <= 0) return 0;
  const int NT = (Nv + 255) / 256, KT = (Kx + 255) / 256;
  const int S = rg_splits(M / 32, NT * KT);
  return (long)S * NT * 256 * (long)KT * 256 * 4;
}

// G[n][k] += sum_m D[m][n] X[m][k] for n < Nv, k < Kx: whole 32-row steps through the ring engine,
// the M % 32 tail rows through tail_tn_kernel (same fixed order: reproducible).  ws: >= shifu_wgrad_ring_ws bytes (fp32 slabs).
SHIFU_API int shifu_wgrad_ring(const void* D, long ldd, const void* X, long ldx, float* G, long ldg,
                               int M, int Nv, int Kx, void* ws, long ws_bytes, hipStream_t stream) {
  if (Kx % 8 || ldd % 8 || ldx % 8 || ldg % 4 || M < 32 || Nv <= 0 || ldd < 8 || ldx < Kx) return -1;
  const int NT = (Nv + 255) / 256, KT = (Kx + 255) / 256;
  const int nsteps = M / 32;
  const int S = rg_splits(nsteps, NT * KT);
  const long need = (long)S * NT * 256 * (long)KT * 256 * 4;
  if (ws == nullptr || ws_bytes < need || ((uintptr_t)ws & 15) || ((uintptr_t)G & 15)) return -1;
  RingTNArgs p{(const bf16_t*)D, ldd, (const bf16_t*)X, ldx, (float*)ws, nsteps, S, NT, KT};
  hipLaunchKernelGGL(ring_tn_kernel, dim3(S * NT * KT), dim3(RG_T), RG_LDS, stream, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const long sstride = (long)NT * 256 * KT * 256;
  const long nq = (long)Nv * (Kx / 4);
  const int rgrid = (int)((nq + 255) / 256 < 2048 ? (nq + 255) / 256 : 2048);
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(rgrid), dim3(256), 0, stream, (const float*)ws, S, sstride,
                     (long)KT * 256, G, ldg, Nv, Kx);
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int tail = M - nsteps * 32;
  if (tail > 0) {
    const long nt = (long)Nv * Kx;
    hipLaunchKernelGGL(tail_tn_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream,
                       (const bf16_t*)D + (size_t)nsteps * 32 * ldd, ldd, (const bf16_t*)X + (size_t)nsteps * 32 * ldx,
                       ldx, tail, G, ldg, Nv, Kx);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
