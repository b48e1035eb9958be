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
typedef __attribute__((ext_vector_type(16))) float f32x16;    // MFMA 32x32 accumulator fragment

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

template <int OFF>
__device__ __forceinline__ s16x4 rg_tr_read_o(uint32_t lds_addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(lds_addr), "n"(OFF));
  return v;
}
__device__ __forceinline__ bf16x8 rg_read_b128(uint32_t lds_addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr));
  return v;
}
template <int OFF>
__device__ __forceinline__ bf16x8 rg_read_b128_o(uint32_t lds_addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(lds_addr), "n"(OFF));
  return v;
}
// 8-byte global store as inline asm: always exactly one instruction per call (the vmcnt counts
// of the NT ring assume a fixed number of stores per tile)
__device__ __forceinline__ void rg_store_b64(void* gaddr, uint2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(gaddr), "v"(v) : "memory");
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
  unsigned long long* dbg;     // STAMP builds only: per-wave segment cycle sums
};

// STAMP (diagnostic build, never the shipped path): s_memtime around every segment, per-wave sums
// [dma issue, fragment read issue, waits, LD barrier, MFMA issue, MMA barrier] written at the end
template <int MF, bool STAMP, bool DMA_IN_MMA>
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

  // ---- LDS-DMA: thread instr i (0/1) per image fills LDS bytes (i*8 + wid)*1024 + lane*16;
  // wave-uniform step base + per-lane 32-bit byte offsets (saddr form, no 64-bit math per step)
  uint32_t offD[2], offX[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int P = (i * 8 + wid) * 1024 + lane * 16;
    const int row = P >> 9, lc = ((P >> 4) & 31) ^ rg_f(row);
    offD[i] = (uint32_t)(row * p.ldd + min(n0 + lc * 8, (int)p.ldd - 8)) * 2u;
    offX[i] = (uint32_t)(row * p.ldx + min(k0 + lc * 8, (int)p.ldx - 8)) * 2u;   // clamped columns: outputs dropped
  }
  const size_t stepD = (size_t)p.S * 32 * p.ldd * 2, stepX = (size_t)p.S * 32 * p.ldx * 2;
  const char* dD = (const char*)(p.D + (size_t)split * 32 * p.ldd);
  const char* dX = (const char*)(p.X + (size_t)split * 32 * p.ldx);
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  int d_left = T - 1;                          // steps the DMA cursor may still advance
  auto dma = [&](int slot) {
    char* base = smem + slot * RG_SLOT + wid_u * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(dD + offD[i]), (lds_ptr_t)(base + i * 8192), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(dX + offX[i]), (lds_ptr_t)(base + RG_IMG + i * 8192), 16, 0, 0);
    if (d_left > 0) { dD += stepD; dX += stepX; --d_left; }   // past the end: re-read the last step
  };
  // one of the 4 LDS-DMA instructions of a step (q = 0, 1: D halves; 2, 3: X halves); q == 3 advances
  auto dma_piece = [&](int slot, int q) {
    char* base = smem + slot * RG_SLOT + wid_u * 1024 + (q >> 1) * RG_IMG + (q & 1) * 8192;
    if (q < 2) __builtin_amdgcn_global_load_lds((const void*)(dD + offD[q & 1]), (lds_ptr_t)base, 16, 0, 0);
    else __builtin_amdgcn_global_load_lds((const void*)(dX + offX[q & 1]), (lds_ptr_t)base, 16, 0, 0);
    if (q == 3 && d_left > 0) { dD += stepD; dX += stepX; --d_left; }
  };

  // accumulators: MF 16: acc16[i][j] (16 x 16 tiles, n block i, k block j); MF 32: acc32[b][c]
  f32x4 acc16[MF == 16 ? 8 : 1][MF == 16 ? 4 : 1];
  f32x16 acc32[MF == 32 ? 4 : 1][MF == 32 ? 2 : 1];
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc32[b][c][e] = 0.f;
  }

  // transposed fragment reads (T10): a 16-lane group supplies 4 rows x 16 columns (lane 4tq+tp the
  // quad at columns cb + 4tp of row tq) and lane t of the group receives column cb + t of the rows.
  //   MF 16: group g = lane >> 4 -> rows 8g + tq (+4): lane holds A[n = lane & 15][m = 8g + 0..7]
  //   MF 32: group G -> columns +16 (G & 1), rows 8 (G >> 1) + tq (+4) of k16 step s (+16 s):
  //          lane holds A[n = lane & 31][m = 16 s + 8 (lane >> 5) + 0..7]
  // Offsets are loop-invariant per lane (the XOR swizzle makes them non-additive in the fragment
  // index); +2048 B = the 4 high rows, +8192 B = the second k16 step (swizzle unchanged by both).
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int r_lo = MF == 16 ? 8 * g + tq : 8 * (g >> 1) + tq;
  const int cg = MF == 16 ? 0 : 16 * (g & 1);
  constexpr int NA = MF == 16 ? 8 : 4, NB = MF == 16 ? 4 : 2, CW = MF == 16 ? 16 : 32;
  uint32_t oD[NA], oX[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) oD[i] = rg_off(r_lo, wn * 128 + i * CW + cg + 4 * tp);
#pragma unroll
  for (int j = 0; j < NB; ++j) oX[j] = RG_IMG + rg_off(r_lo, wk * 64 + j * CW + cg + 4 * tp);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  auto frag0 = [&](uint32_t a) {
    const s16x4 lo = rg_tr_read_o<0>(a);
    const s16x4 hi = rg_tr_read_o<2048>(a);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto frag1 = [&](uint32_t a) {
    const s16x4 lo = rg_tr_read_o<8192>(a);
    const s16x4 hi = rg_tr_read_o<8192 + 2048>(a);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  bf16x8 af[2][NA], bfr[2][NB];      // [k16 step] (MF 16 uses step 0 only: one K = 32 MFMA)

#define RG_BAR() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); \
                      __builtin_amdgcn_sched_barrier(0); } while (0)

  dma(0); dma(1); dma(2); dma(3);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  RG_BAR();
  if (lag) RG_BAR();

  unsigned long long st_sum[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  auto stamp = [&](int k) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (k >= 0) st_sum[k] += now - st_prev;
      st_prev = now;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int slot = 0, dslot = 4;
  for (int t = 0; t < T; ++t) {
    // ---- LD segment
    stamp(-1);
    if constexpr (!DMA_IN_MMA) dma(dslot);
    stamp(0);
    const uint32_t sb = lds0 + slot * RG_SLOT;
#pragma unroll
    for (int j = 0; j < NB; ++j) bfr[0][j] = frag0(sb + oX[j]);
#pragma unroll
    for (int i = 0; i < NA; ++i) af[0][i] = frag0(sb + oD[i]);
    if constexpr (MF == 32) {
#pragma unroll
      for (int j = 0; j < NB; ++j) bfr[1][j] = frag1(sb + oX[j]);
#pragma unroll
      for (int i = 0; i < NA; ++i) af[1][i] = frag1(sb + oD[i]);
    }
    stamp(1);
    if constexpr (DMA_IN_MMA) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(2);
    RG_BAR();
    stamp(3);
    // ---- MMA segment
    __builtin_amdgcn_s_setprio(1);
    if constexpr (MF == 16) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j], acc16[i][j], 0, 0, 0);
        if constexpr (DMA_IN_MMA) {
          // the refill of slot (t+4)%5 = step t-1's slot: every wave finished its reads of step t-1
          // before the barrier that ended its LD(t-1), which precedes this segment
          if (i == 1 || i == 3 || i == 5 || i == 7) {
            __builtin_amdgcn_sched_barrier(0);
            dma_piece(dslot, i >> 1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
#pragma unroll
          for (int c = 0; c < 2; ++c)
            acc32[b][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s2][b], bfr[s2][c], acc32[b][c], 0, 0, 0);
          if constexpr (DMA_IN_MMA) {
            if (b == 1 || b == 3) {
              __builtin_amdgcn_sched_barrier(0);
              dma_piece(dslot, s2 * 2 + (b >> 1));
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
    }
    __builtin_amdgcn_s_setprio(0);
    stamp(4);
    RG_BAR();
    stamp(5);
    slot = slot == RG_NSLOT - 1 ? 0 : slot + 1;
    dslot = dslot == RG_NSLOT - 1 ? 0 : dslot + 1;
  }
  if (!lag) RG_BAR();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef RG_BAR
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* d = p.dbg + ((size_t)blockIdx.x * 8 + wid) * 8;
      for (int k = 0; k < 6; ++k) d[k] = st_sum[k];
      d[6] = T;
      d[7] = wg;
    }
  }

  // ---- epilogue: this split's partial tile -> slab
  const long lds = (long)p.KT * 256;
  float* out = p.slab + (size_t)split * ((size_t)p.NT * 256) * lds;
  if constexpr (MF == 16) {
    // acc16[i][j][r]: n = 16i + 4(lane>>4) + r, k = 16j + (lane & 15) within the wave tile
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 128 + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + wk * 64 + j * 16 + (lane & 15);
          out[(size_t)n * lds + k] = acc16[i][j][r];
        }
      }
  } else {
    // acc32[b][c][e]: n = 32b + (e & 3) + 8(e >> 2) + 4(lane >> 5), k = 32c + (lane & 31):
    // every store is two 128-B row segments
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + wn * 128 + b * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int k = k0 + wk * 64 + c * 32 + (lane & 31);
          out[(size_t)n * lds + k] = acc32[b][c][e];
        }
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

static unsigned long long* g_rg_stamp = nullptr;    // diagnostic: STAMP build of the TN ring
// Diagnostic switch: a device buffer of >= blocks * 8 * 8 u64 enables the STAMP build (nullptr: off).
SHIFU_API int shifu_ring_set_stamp(void* buf) { g_rg_stamp = (unsigned long long*)buf; return 0; }
static int g_rg_mf = 16;                            // MFMA shape of the TN ring (A/B switch: 16 or 32)
static int g_rg_dmamma = 1;                         // TN ring: LDS-DMA issued inside the MMA segment
SHIFU_API int shifu_ring_set_mf(int mf) { g_rg_mf = mf == 32 ? 32 : 16; return 0; }
SHIFU_API int shifu_ring_set_dmamma(int v) { g_rg_dmamma = v; return 0; }

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
  RingTNArgs p{(const bf16_t*)D, ldd, (const bf16_t*)X, ldx, (float*)ws, nsteps, S, NT, KT, g_rg_stamp};
  const dim3 grid(S * NT * KT);
  if (g_rg_mf == 16) {
    if (g_rg_dmamma) {
      if (g_rg_stamp) hipLaunchKernelGGL((ring_tn_kernel<16, true, true>), grid, dim3(RG_T), RG_LDS, stream, p);
      else hipLaunchKernelGGL((ring_tn_kernel<16, false, true>), grid, dim3(RG_T), RG_LDS, stream, p);
    } else {
      if (g_rg_stamp) hipLaunchKernelGGL((ring_tn_kernel<16, true, false>), grid, dim3(RG_T), RG_LDS, stream, p);
      else hipLaunchKernelGGL((ring_tn_kernel<16, false, false>), grid, dim3(RG_T), RG_LDS, stream, p);
    }
  } else {
    if (g_rg_dmamma) {
      if (g_rg_stamp) hipLaunchKernelGGL((ring_tn_kernel<32, true, true>), grid, dim3(RG_T), RG_LDS, stream, p);
      else hipLaunchKernelGGL((ring_tn_kernel<32, false, true>), grid, dim3(RG_T), RG_LDS, stream, p);
    } else {
      if (g_rg_stamp) hipLaunchKernelGGL((ring_tn_kernel<32, true, false>), grid, dim3(RG_T), RG_LDS, stream, p);
      else hipLaunchKernelGGL((ring_tn_kernel<32, false, false>), grid, dim3(RG_T), RG_LDS, stream, p);
    }
  }
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
