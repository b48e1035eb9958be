// MFMA GEMM kernels for the MLP (gfx950 / CDNA4): fused forward/dgrad NT GEMM and TN wgrad.
//
// Replaces the reference's per-row Java scalar loops
//   forward  FloatFlatNetwork.compute/computeLayer  (J/core/dtrain/dataset/FloatFlatNetwork.java:69-223)
//   backward SubGradient.process/processLevel         (J/core/dtrain/nn/SubGradient.java:224-311)
//   update   Weight.calculateWeights + nn/update/*    (J/core/dtrain/Weight.java:194-343)
// with row-tiled MFMA GEMMs.  Layout decisions (MI355X-first, not a translation):
//   * Every layer is a pure GEMM: the Encog bias neuron is a real input column (value 1.0)
//     stored right after the last feature, and K is zero-padded to a multiple of 64.  So
//     W_l is [out_l, in_pad_l] with column in_l = bias (exactly Encog's flat layout per block).
//   * Activations are bf16 row-major [rows, in_pad]; the forward epilogue writes act(z),
//     the bias column (1.0) and zero padding in one pass.
//   * dgrad is an NT GEMM against a per-step transposed bf16 copy of W, with the
//     activation derivative (+ Encog flat spot) fused into the epilogue.
//   * wgrad is a TN GEMM over the row axis (split-K over rows) using the gfx950
//     ds_read_b64_tr_b16 transposed LDS read for both operands; fp32 atomics into the
//     flat gradient buffer.
//   * the output layer (n_out <= 8) + loss + output delta + last-hidden dgrad + output
//     wgrad are one row kernel (memory-bound, one wave per row strip).
#include "common.h"
#include <type_traits>

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int TILE_BYTES = BM * BK * 2;   // 16 KiB per operand tile

// XCD-aware bijective block remap: consecutive logical ids land on the same XCD
// (blocks b, b+8, ... share an XCD under round-robin dispatch; speed only).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// [128 rows][64 bf16] tile, 128-B rows, 16-B chunk XOR swizzle: rows 0..15 of a fragment
// read land on 16 distinct 16-B slots of the 256-B bank row (conflict-free ds_read_b128).
__device__ __forceinline__ int swz_nt(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// 256-B-row LDS images read with ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group):
// quad XOR swizzle so that the 8 rows read by one 32-lane half hit 8 distinct bank groups.
__device__ __forceinline__ int tr_h(int m) { return (m & 3) | (((m >> 3) & 1) << 2); }
// byte offset of 8-byte quad q (4 bf16: cols 4q..4q+3) of row m
__device__ __forceinline__ int swz_tn_quad(int m, int q) { return m * 256 + ((q ^ (tr_h(m) << 2)) << 3); }

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
// gfx950 ds_read_b64_tr_b16 (compiler builtin: hipcc counts its lgkmcnt itself)
__device__ __forceinline__ s16x4 ds_read_tr16_b64(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
}

enum Epi : int { EPI_ACT = 0, EPI_DACT = 1, EPI_STORE = 2,
                 EPI_F32 = 3 };   // fp32 output tile (split-bf16 fp32-accurate products: algos/varsel.py)

struct GemmArgs {
  const bf16_t* A; long lda;   // [M, K] row-major
  const bf16_t* B; long ldb;   // [NB, K] row-major (rows >= NB read as 0)
  bf16_t* C; long ldc;         // [M, N] output
  bf16_t* C2; long ldc2;       // EPI_ACT optional: f'(z)+flat (activations not derivable from output)
  const bf16_t* H; long ldh;   // EPI_DACT: layer input activations (derivative from output)
  const bf16_t* Hd; long ldhd; // EPI_DACT: stored derivative (when !act_deriv_from_output)
  int M, N, K, NB, n_valid, act, bias_col;
  float flat;
  int dbg;                     // lab ablations (shifu_gemm_set_tune(9, v)); 0 in production
  // segmented K (corr_i8_kernel): k-tiles [q * seg_nk, (q + 1) * seg_nk) read A rows from
  // A + segA[q] * seg_stride and B rows from B + segB[q] * seg_stride (plane pairs summed in one
  // pipeline).  Held as wave-uniform values and picked with a select chain: a load (or a dynamic
  // index into a private array) inside the pipeline would be a vector-memory op that breaks the
  // counted vmcnt waits.
  int segA[7], segB[7]; long seg_stride; int seg_shift;   // seg_nk = 1 << seg_shift
};

// STAGES = LDS buffers.  1: single 32 KiB buffer + register prefetch (two barriers per k-step,
// up to 5 blocks = 5 waves/SIMD per CU -> the HBM/L2 latency of the next tile is hidden by the
// other resident blocks); 2: classic LDS double buffer (64 KiB, 2 blocks per CU).
template <int EPI, int ACT, int STAGES>
__global__ __launch_bounds__(NTHR) void gemm_nt_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntn = (p.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / ntn) * BM, n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  uint4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 3, ch = idx & 7;
      const int gm = m0 + row, gn = n0 + row;
      ra[i] = gm < p.M ? *(const uint4*)(p.A + (size_t)gm * p.lda + k0 + ch * 8) : make_uint4(0, 0, 0, 0);
      rb[i] = gn < p.NB ? *(const uint4*)(p.B + (size_t)gn * p.ldb + k0 + ch * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto swrite = [&](int buf) {
    char* As = smem + buf * 2 * TILE_BYTES;
    char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 3, ch = idx & 7;
      *(uint4*)(As + swz_nt(row, ch)) = ra[i];
      *(uint4*)(Bs + swz_nt(row, ch)) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};


  const int nk = p.K / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = STAGES == 2 ? (kt & 1) : 0;
    if (kt + 1 < nk) gload((kt + 1) * BK);        // issue next tile's HBM loads early
    const char* As = smem + buf * 2 * TILE_BYTES;
    const char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) af[j] = *(const bf16x8*)(As + swz_nt(wr * 64 + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i) bfr[i] = *(const bf16x8*)(Bs + swz_nt(wc * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[i], af[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (STAGES == 1) __syncthreads();     // every wave is done reading the buffer
    if (kt + 1 < nk) swrite(STAGES == 2 ? (buf ^ 1) : 0);
    __syncthreads();
  }

  // Epilogue.  acc[i][j] holds D[n][m]: m = lane&15 (+16j), n = 4*(lane>>4) + r (+16i):
  // each lane owns 4 consecutive output columns of one row.
  constexpr bool dfo = act_deriv_from_output(ACT);
  if constexpr ((EPI == EPI_ACT || EPI == EPI_DACT) && dfo || EPI == EPI_STORE) {
    // Staged epilogue: phase 1 packs the tile (bf16) into LDS with a 16-B chunk XOR swizzle,
    // phase 2 writes whole 256-B row segments with 16-B stores (and, for dgrad, reads the
    // matching H row segment coalesced) instead of 16 rows x 32 B per wave instruction.
    char* Cs = smem;                       // [128][256 B]; loop's last barrier freed the tiles
    const int c = tid & 15;
    // dgrad: issue all 8 H row-segment loads of this thread up front, so they are in flight while
    // the tile is staged through LDS (8 x 16 B per lane instead of one load per pass); rows clamped
    // to M - 1 and columns to ldh - 8 keep every load in bounds without a branch around it
    uint4 hreg[8];
    if constexpr (EPI == EPI_DACT) {
      const int nh = min(n0 + c * 8, (int)p.ldh - 8);
#pragma unroll
      for (int pass = 0; pass < 8; ++pass) {
        const int mh = min(m0 + pass * 16 + (tid >> 4), p.M - 1);
        hreg[pass] = *(const uint4*)(p.H + (size_t)mh * p.ldh + nh);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nl = wc * 64 + i * 16 + (lane >> 4) * 4;       // local column (multiple of 4)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = wr * 64 + j * 16 + (lane & 15);
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = acc[i][j][r];
          if constexpr (EPI == EPI_ACT) {
            const int n = n0 + nl + r;
            o[r] = n < p.n_valid ? act_fwd(ACT, z) : ((n == p.n_valid && p.bias_col) ? 1.f : 0.f);
          } else {
            o[r] = z;
          }
        }
        uint2 w;
        w.x = pack_bf16x2(o[0], o[1]);
        w.y = pack_bf16x2(o[2], o[3]);
        const int c = nl >> 3, half = (nl >> 2) & 1;
        *(uint2*)(Cs + ml * 256 + ((c ^ (ml & 15)) << 4) + half * 8) = w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      const int ml = pass * 16 + (tid >> 4);
      const int m = m0 + ml, n = n0 + c * 8;
      if (m >= p.M || n >= p.N) continue;
      uint4 v = *(const uint4*)(Cs + ml * 256 + ((c ^ (ml & 15)) << 4));
      if constexpr (EPI == EPI_DACT) {
        const uint4 h = hreg[pass];
        const uint32_t hv[4] = {h.x, h.y, h.z, h.w};
        uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float a0 = bf2f(vv[q] & 0xffff), a1 = bf2f(vv[q] >> 16);
          const float d0 = act_deriv_out(ACT, bf2f(hv[q] & 0xffff)) + p.flat;
          const float d1 = act_deriv_out(ACT, bf2f(hv[q] >> 16)) + p.flat;
          a0 = (n + 2 * q < p.n_valid) ? a0 * d0 : 0.f;
          a1 = (n + 2 * q + 1 < p.n_valid) ? a1 * d1 : 0.f;
          vv[q] = pack_bf16x2(a0, a1);
        }
        v = make_uint4(vv[0], vv[1], vv[2], vv[3]);
      }
      if (n + 8 <= p.N) {
        *(uint4*)(p.C + (size_t)m * p.ldc + n) = v;
      } else {                                             // N % 8 == 4 tail
        *(uint2*)(p.C + (size_t)m * p.ldc + n) = make_uint2(v.x, v.y);
      }
    }
    return;
  } else if constexpr (EPI == EPI_F32) {
    // each lane owns 4 consecutive output columns of one row: one 16-B store (C is float, ldc floats)
    // act != LINEAR applies the activation with the accurate libm forms (fp32 scoring: ops/gemm_ops.py)
    float* Cf = (float*)p.C;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = n0 + wc * 64 + i * 16 + (lane >> 4) * 4;
      if (nb >= p.N) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wr * 64 + j * 16 + (lane & 15);
        float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (p.act != ACT_LINEAR) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = act_fwd_precise(p.act, o[e]);
        }
        if (m < p.M) *(float4*)(Cf + (size_t)m * p.ldc + nb) = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
  } else {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nb = n0 + wc * 64 + i * 16 + (lane >> 4) * 4;
    if (nb >= p.N) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wr * 64 + j * 16 + (lane & 15);
      if (m >= p.M) continue;
      float o[4];
      if constexpr (EPI == EPI_ACT) {
        float d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + r;
          const float z = acc[i][j][r];
          if (n < p.n_valid) { o[r] = act_fwd(ACT, z); d[r] = act_deriv_pre(ACT, z) + p.flat; }
          else { o[r] = (n == p.n_valid && p.bias_col) ? 1.f : 0.f; d[r] = 0.f; }
        }
        uint2 w2;
        w2.x = pack_bf16x2(d[0], d[1]);
        w2.y = pack_bf16x2(d[2], d[3]);
        *(uint2*)(p.C2 + (size_t)m * p.ldc2 + nb) = w2;
      } else {   // EPI_DACT with a stored derivative (activations not derivable from the output)
        const uint2 h = *(const uint2*)(p.Hd + (size_t)m * p.ldhd + nb);
        const float dv[4] = {bf2f(h.x & 0xffff), bf2f(h.x >> 16), bf2f(h.y & 0xffff), bf2f(h.y >> 16)};
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (nb + r < p.n_valid) ? acc[i][j][r] * dv[r] : 0.f;
      }
      uint2 w;
      w.x = pack_bf16x2(o[0], o[1]);
      w.y = pack_bf16x2(o[2], o[3]);
      *(uint2*)(p.C + (size_t)m * p.ldc + nb) = w;
    }
  }
  }
}

// Staged epilogue of the 256 x 256 kernels (512 threads, 8 waves 2 M x 4 N, wave tile 128 x 64,
// acc[n-sub 0..3][m-sub 0..7]): the whole bf16 tile goes through LDS ([256][512 B], 16-B chunk ^
// (row & 15)) and leaves as 16-B row-segment stores (dgrad reads the matching H segments).
// The caller guarantees every wave has finished reading the LDS staging buffers.
template <int EPI, int ACT>
__device__ __forceinline__ void epilogue_256(const GemmArgs& p, f32x4 (&acc)[4][8], int m0, int n0, char* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  char* Cs = smem;
  auto tile_write = [&](auto FULL) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nl = wc * 64 + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ml = wr * 128 + j * 16 + (lane & 15);
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = acc[i][j][r];
          const int n = n0 + nl + r;
          if constexpr (decltype(FULL)::value) o[r] = EPI == EPI_ACT ? act_fwd(ACT, z) : z;
          else if constexpr (EPI == EPI_ACT) o[r] = n < p.n_valid ? act_fwd(ACT, z) : ((n == p.n_valid && p.bias_col) ? 1.f : 0.f);
          else if constexpr (EPI == EPI_STORE) o[r] = n < p.NB ? z : 0.f;
          else o[r] = z;
        }
        uint2 w;
        w.x = pack_bf16x2(o[0], o[1]);
        w.y = pack_bf16x2(o[2], o[3]);
        const int c = nl >> 3, half = (nl >> 2) & 1;
        *(uint2*)(Cs + ml * 512 + ((c ^ (ml & 15)) << 4) + half * 8) = w;
      }
    }
  };
  const bool full = EPI == EPI_DACT || n0 + 256 <= (EPI == EPI_ACT ? p.n_valid : p.NB);
  if (full) tile_write(std::integral_constant<bool, true>{});
  else tile_write(std::integral_constant<bool, false>{});
  __syncthreads();
  if (p.dbg & 8) return;                             // lab: no global tile stores
  const int c = tid & 31;
#pragma unroll 4
  for (int pass = 0; pass < 16; ++pass) {
    const int ml = pass * 16 + (tid >> 5);
    const int m = m0 + ml, n = n0 + c * 8;
    if (m >= p.M || n >= p.N) continue;
    uint4 v = *(const uint4*)(Cs + ml * 512 + ((c ^ (ml & 15)) << 4));
    if constexpr (EPI == EPI_DACT) {
      const uint4 hh = *(const uint4*)(p.H + (size_t)m * p.ldh + n);
      const uint32_t hv[4] = {hh.x, hh.y, hh.z, hh.w};
      uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float a0 = bf2f(vv[q] & 0xffff), a1 = bf2f(vv[q] >> 16);
        const float d0 = act_deriv_out(ACT, bf2f(hv[q] & 0xffff)) + p.flat;
        const float d1 = act_deriv_out(ACT, bf2f(hv[q] >> 16)) + p.flat;
        a0 = (n + 2 * q < p.n_valid) ? a0 * d0 : 0.f;
        a1 = (n + 2 * q + 1 < p.n_valid) ? a1 * d1 : 0.f;
        vv[q] = pack_bf16x2(a0, a1);
      }
      v = make_uint4(vv[0], vv[1], vv[2], vv[3]);
    }
    if (n + 8 <= p.N) *(uint4*)(p.C + (size_t)m * p.ldc + n) = v;
    else *(uint2*)(p.C + (size_t)m * p.ldc + n) = make_uint2(v.x, v.y);
  }
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((ext_vector_type(2))) unsigned int v2u32_t;
// ---------------------------------------------------------------------------------------
// 8-phase NT GEMM (256 x 256 x 64, 8 waves 2 M x 4 N, wave tile 128 x 64, 1 block per CU).
//
// The schedule follows the CDNA4 "256^2 8-phase" recipe (cdna_hip_programming.md §5): one
// iteration = 2 k-tiles = 8 phases; each phase is [ds_read fragments + one LDS-DMA half-tile
// prefetch] s_barrier [16 MFMAs on one quadrant of the wave tile] s_barrier, and the two wave
// rows run one barrier apart, so on every SIMD one wave's MFMAs overlap the other wave's
// reads / DMA issue.  LDS = 2 k-tile buffers x 4 half-tiles (A rows 0-127 / 128-255, B rows
// 0-127 / 128-255; 16 KiB each, [128 rows][128 B], 16-B chunk ^ ((row >> 1) & 7) swizzle that
// the DMA applies on the GLOBAL source address).
//
// Per iteration (even k-tile 2i in buffer 0, odd 2i+1 in buffer 1), per wave:
//   P1 DMA odd A-top(2i+1)   read A[mh0] B[nh0] (buf 0)  MFMA quadrant (0,0)
//   P2 DMA odd A-bot(2i+1)   read B[nh1], lgkmcnt(0) before the barrier      (0,1)
//   P3 DMA even B-0(2i+2)    read A[mh1]                                      (1,1)
//   P4 DMA even B-1(2i+2)    vmcnt(4): odd buffer landed                      (1,0)
//   P5-P8: the same on buffer 1 (DMA even A-top/A-bot(2i+2), odd B-0/B-1(2i+3)).
// Write-after-read: a half-tile is re-staged >= 2 phases after its last ds_read (B: 1 phase,
// its reads are retired before that phase's first barrier).  Read-after-DMA: the vmcnt(4) at
// P4 / P8 (the two youngest half-tiles stay in flight) retires every DMA into the buffer read
// in the next 3 phases, and a barrier separates the wait from the reads (no __syncthreads in
// the loop: its fence would drain vmcnt to 0).  DMA past the last k-tile re-reads k-tile nk-1
// into the buffer that is not read any more, so the counted waits stay exact.
// ---------------------------------------------------------------------------------------
constexpr int G8_T = 512, G8_HALF = 16384, G8_BUF = 4 * G8_HALF;
typedef __attribute__((ext_vector_type(4))) int v4i_t;

// Per-thread LDS-DMA source offsets of tile (m0, n0): half-tile h (0 A-top, 1 A-bot, 2 B-0, 3 B-1),
// instruction i (2 per thread): LDS byte P = i*8192 + wid*1024 + lane*16 of the half-tile holds
// logical chunk lc of row P>>7 (the swizzle is applied on the GLOBAL source address).
template <typename OffT = long>
__device__ __forceinline__ void gemm8_src(const GemmArgs& p, int m0, int n0, OffT (&off)[4][2]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int P = i * 8192 + wid * 1024 + lane * 16;
    const int row = P >> 7, lc = ((P >> 4) & 7) ^ ((row >> 1) & 7);
    int ma = min(m0 + row, p.M - 1), mb = min(m0 + 128 + row, p.M - 1);
    if (p.dbg & 32) { ma &= 4095; mb &= 4095; }        // lab: A rows from a 4096-row (L2-resident) window
    off[0][i] = (OffT)((long)ma * p.lda + lc * 8);
    off[1][i] = (OffT)((long)mb * p.lda + lc * 8);
    off[2][i] = (OffT)((long)min(n0 + row, p.NB - 1) * p.ldb + lc * 8);
    off[3][i] = (OffT)((long)min(n0 + 128 + row, p.NB - 1) * p.ldb + lc * 8);
  }
}

template <bool SEG = false, typename OffT = long>
__device__ __forceinline__ void gemm8_dma(const GemmArgs& p, const OffT (&off)[4][2], char* smem, int h, int kt) {
  const int wid = threadIdx.x >> 6;
  const int nk = p.K / 64;
  char* dst = smem + (kt & 1) * G8_BUF + h * G8_HALF + wid * 1024;
  int k0 = min(kt, nk - 1) * 64;
  const bf16_t* src = h < 2 ? p.A : p.B;
  if constexpr (SEG) {                 // wave-uniform shifts + scalar loads (no division: VALU)
    const int kk = min(kt, nk - 1), q = kk >> p.seg_shift;
    k0 = (kk & ((1 << p.seg_shift) - 1)) * 64;
    int pl = h < 2 ? p.segA[0] : p.segB[0];
#pragma unroll
    for (int i = 1; i < 7; ++i) pl = q == i ? (h < 2 ? p.segA[i] : p.segB[i]) : pl;
    src += (long)pl * p.seg_stride;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
    __builtin_amdgcn_global_load_lds((const void*)(src + off[h][i] + k0), (lds_ptr_t)(dst + i * 8192), 16, 0, 0);
}

// prologue DMAs of a tile: even k-tile 0 complete, odd k-tile 1 B halves (12 vector-memory ops)
template <bool SEG = false, typename OffT = long>
__device__ __forceinline__ void gemm8_prologue(const GemmArgs& p, const OffT (&off)[4][2], char* smem) {
  gemm8_dma<SEG>(p, off, smem, 2, 0); gemm8_dma<SEG>(p, off, smem, 3, 0); gemm8_dma<SEG>(p, off, smem, 0, 0);
  gemm8_dma<SEG>(p, off, smem, 1, 0); gemm8_dma<SEG>(p, off, smem, 2, 1); gemm8_dma<SEG>(p, off, smem, 3, 1);
}

// The 8-phase k-loop of one 256 x 256 output tile into acc (see the schedule above), after its
// prologue DMAs.
// I8: the operands are int8 (a k-tile = 128 int8 per row = the same 128 B that hold 64 bf16, so the
// staging is unchanged; p.K / p.lda stay in 2-byte units) and every MFMA is
// v_mfma_i32_16x16x64_i8 -- acc then holds int32 bits.  A and B fragments take the same 16 bytes
// of a row, so the hardware's k order inside the 64 does not matter.  zero = false accumulates
// onto acc (several operand pairs summed into one tile).
template <bool I8 = false, typename OffT = long>
__device__ __forceinline__ void gemm8_loop(const GemmArgs& p, f32x4 (&acc)[4][8], const OffT (&off)[4][2],
                                           char* smem, bool zero = true) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int nk = p.K / 64;
  auto dma = [&](int h, int kt) { gemm8_dma<I8, OffT>(p, off, smem, h, kt); };

  if (zero) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  bf16x8 af[4][2], bf0[2][2], bf1[2][2];
  const int lr = lane & 15, lq = lane >> 4;
  auto readA = [&](int buf, int mh) {
    const char* base = smem + buf * G8_BUF + wr * G8_HALF;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int c = 0; c < 2; ++c) af[t][c] = *(const bf16x8*)(base + swz_nt(mh * 64 + t * 16 + lr, c * 4 + lq));
  };
  auto readB = [&](int buf, int nh, bf16x8 (&bq)[2][2]) {
    const char* base = smem + buf * G8_BUF + (2 + (wc >> 1)) * G8_HALF;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        bq[t][c] = *(const bf16x8*)(base + swz_nt((wc & 1) * 64 + nh * 32 + t * 16 + lr, c * 4 + lq));
  };
  auto mma = [&](int mh, int nh, bf16x8 (&bq)[2][2]) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          f32x4& a_ = acc[nh * 2 + s_][mh * 4 + t];
          if constexpr (I8)
            a_ = __builtin_bit_cast(f32x4, __builtin_amdgcn_mfma_i32_16x16x64_i8(
                     __builtin_bit_cast(v4i_t, bq[s_][c]), __builtin_bit_cast(v4i_t, af[t][c]),
                     __builtin_bit_cast(v4i_t, a_), 0, 0, 0));
          else
            a_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[s_][c], af[t][c], a_, 0, 0, 0);
        }
  };
#define G8_BAR() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); \
                      __builtin_amdgcn_sched_barrier(0); } while (0)
#define G8_MMA(mh, nh, bq, on) do { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    if ((on) && !(p.dbg & 64)) { __builtin_amdgcn_s_setprio(1); mma(mh, nh, bq); __builtin_amdgcn_s_setprio(0); } } while (0)

  // even k-tile 0 landed (its 8 DMAs are the oldest), odd k-tile 1 B halves stay in flight
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  G8_BAR();
  if (wr == 1) G8_BAR();                      // stagger the two wave rows by one barrier

  for (int ke = 0; ke < nk; ke += 2) {
    const int ko = ke + 1;
    const bool odd_on = ko < nk;
    // ---- even k-tile (buffer 0)
    dma(0, ko); readB(0, 0, bf0); readA(0, 0);                                   // P1
    G8_BAR(); G8_MMA(0, 0, bf0, true); G8_BAR();
    dma(1, ko); readB(0, 1, bf1); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // P2
    G8_BAR(); G8_MMA(0, 1, bf1, true); G8_BAR();
    dma(2, ke + 2); readA(0, 1);                                                 // P3
    G8_BAR(); G8_MMA(1, 1, bf1, true); G8_BAR();
    dma(3, ke + 2); asm volatile("s_waitcnt vmcnt(4)" ::: "memory");            // P4
    G8_BAR(); G8_MMA(1, 0, bf0, true); G8_BAR();
    // ---- odd k-tile (buffer 1)
    dma(0, ke + 2); readB(1, 0, bf0); readA(1, 0);                               // P5
    G8_BAR(); G8_MMA(0, 0, bf0, odd_on); G8_BAR();
    dma(1, ke + 2); readB(1, 1, bf1); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // P6
    G8_BAR(); G8_MMA(0, 1, bf1, odd_on); G8_BAR();
    dma(2, ko + 2); readA(1, 1);                                                 // P7
    G8_BAR(); G8_MMA(1, 1, bf1, odd_on); G8_BAR();
    dma(3, ko + 2); asm volatile("s_waitcnt vmcnt(4)" ::: "memory");            // P8
    G8_BAR(); G8_MMA(1, 0, bf0, odd_on); G8_BAR();
  }
  if (wr == 0) G8_BAR();                      // re-align the rows
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain the trailing prefetches
  G8_BAR();
#undef G8_MMA
#undef G8_BAR
}

__device__ __forceinline__ void gemm8_mainloop(const GemmArgs& p, f32x4 (&acc)[4][8], int m0, int n0, char* smem) {
  long off[4][2];
  gemm8_src(p, m0, n0, off);
  gemm8_prologue(p, off, smem);
  gemm8_loop(p, acc, off, smem);
}

template <int EPI, int ACT>
__global__ __launch_bounds__(G8_T, 1) void gemm_nt_8ph_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntn = (p.N + 255) / 256;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / ntn) * 256, n0 = (wg % ntn) * 256;
  f32x4 acc[4][8];
  gemm8_mainloop(p, acc, m0, n0, smem);
  if (p.dbg & 2) {                                    // lab: main loop only (acc kept live)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  epilogue_256<EPI, ACT>(p, acc, m0, n0, smem);
}

// ---------------------------------------------------------------------------------------
// Fused network head: last hidden layer forward (8-phase GEMM, the whole hidden width N <= 256
// in one tile) + output layer (n_out = 1) + loss + output delta + last-hidden delta + output
// wgrad, all in the epilogue.  A block owns complete rows, so the output dot product, the loss
// and D = delta * w_out * (f'(a) + flat) are row-local; the last hidden activations never go to
// HBM (the unfused path writes them and mlp_output_kernel reads them back).
// Same per-row semantics as mlp_output_kernel (SubGradient.java:241-248 for the squared loss).
// ---------------------------------------------------------------------------------------
struct HeadArgs {
  const float* W;        // [KH] fp32 output weights (bias weight at kh_valid, zeros after)
  const float* Y;        // [M] targets
  const float* S;        // [M] significance (nullable -> 1)
  float* GW;             // [KH] output-weight gradient (atomic; unused when GWslab is set)
  float* GWslab;         // [tiles][KH] per-tile partials (nullable): summed in fixed order afterwards
  double* err;           // [2] error sum, weight sum (atomic; unused when errslab is set)
  double* errslab;       // [tiles][2] per-tile sums (nullable): summed in fixed order afterwards
  int KH, out_act, loss;
  float flat_out, flat_hid;
};
constexpr int HEAD_LDS = 2 * G8_BUF + 12288;    // ring / staging + row partials, deltas, gW partials

template <int ACT>
__global__ __launch_bounds__(G8_T, 1) void gemm_head_8ph_kernel(GemmArgs p, HeadArgs h) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * 256;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  // the epilogue's per-row inputs (targets, significance) are loaded before the main loop so
  // their HBM latency hides behind it (one block per CU: nothing else would cover it)
  const int my = min(m0 + (tid & 255), p.M - 1);
  const float y_pf = h.Y[my], s_pf = h.S ? h.S[my] : 1.f;
  f32x4 acc[4][8];
  gemm8_mainloop(p, acc, m0, 0, smem);
  if (p.dbg & 2) {                                    // lab: main loop only (acc kept live)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  float* red = (float*)(smem + 2 * G8_BUF);          // [2 wr][4 wc][128] row partials of z_out
  float* dl = red + 1024;                            // [256] output deltas
  float* gred = dl + 256;                            // [2 wr][256] output-wgrad partials
  double* ered = (double*)(gred + 512);              // [8 waves][2]
  const int nv = p.n_valid;
  // 1. hidden activations (bf16-rounded, as the unfused path stores them) + this lane's w_out
  float w3[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = wc * 64 + i * 16 + (lane >> 4) * 4 + r;
      w3[i][r] = (p.dbg & 16) ? 0.01f : (n < h.KH ? h.W[n] : 0.f);    // lab 16: no global loads
    }
  float zp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wc * 64 + i * 16 + (lane >> 4) * 4 + r;
        float a = n < nv ? act_fwd(ACT, acc[i][j][r]) : (n == nv ? 1.f : 0.f);
        a = bf2f(f2bf(a));
        acc[i][j][r] = a;
        t += a * w3[i][r];
      }
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    zp[j] = t;
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(wr * 4 + wc) * 128 + j * 16 + lane] = zp[j];
  }
  __syncthreads();
  // 2. per row: output, loss, delta (threads 0..255 = the tile's rows)
  double e_c = 0.0, e_w = 0.0;
  if (tid < 256) {
    const int rw = tid >> 7, rl = tid & 127;
    const float z = red[(rw * 4 + 0) * 128 + rl] + red[(rw * 4 + 1) * 128 + rl] + red[(rw * 4 + 2) * 128 + rl] +
                    red[(rw * 4 + 3) * 128 + rl];
    const int m = m0 + tid;
    float dlt = 0.f;
    if (m < p.M) {
      const float y = y_pf, sg = s_pf;
      const float a = act_fwd(h.out_act, z), e = y - a;
      const int lm = h.loss % 3;                       // loss >= 3: TF objective as the error
      if (lm == 1) {
        dlt = e * sg;
        const float ac = fminf(fmaxf(a, 1e-7f), 1.f - 1e-7f);
        e_c = h.loss >= 3 ? -(__logf(a + 1e-7f) * y + __logf(1.f - a + 1e-7f) * (1.f - y)) * sg
                          : -(__logf(ac) * y + __logf(1.f - ac) * (1.f - y));
      } else if (lm == 2) {
        dlt = (y < a ? 1.f : -1.f) * (act_deriv_out(h.out_act, a) + h.flat_out) * sg;
        e_c = fabsf(e) * sg;
      } else {
        dlt = (act_deriv_pre(h.out_act, z) + h.flat_out) * e * sg;
        e_c = h.loss >= 3 ? (double)(e * e) * sg : (double)(e * sg) * (e * sg);
      }
      e_w = sg;
    }
    dl[tid] = dlt;
  }
  e_c = wave_sum_d(e_c);
  e_w = wave_sum_d(e_w);
  if (lane == 0) { ered[wid * 2] = e_c; ered[wid * 2 + 1] = e_w; }
  __syncthreads();
  if (tid == 0 && !(p.dbg & 1)) {
    double a0 = 0.0, a1 = 0.0;
    for (int w = 0; w < 8; ++w) { a0 += ered[w * 2]; a1 += ered[w * 2 + 1]; }
    if (h.errslab) {                                 // 2 fp64 atomics from every tile on one line
      h.errslab[(size_t)(m0 >> 8) * 2] = a0;         // contended (~0.1 ms per 2M-row chunk)
      h.errslab[(size_t)(m0 >> 8) * 2 + 1] = a1;
    } else {
      atomicAdd(h.err, a0);
      atomicAdd(h.err + 1, a1);
    }
  }
  if (p.dbg & 4) return;                             // lab: stages 1-2 only
  // 3. last-hidden deltas (bf16, staged through LDS) and the output-wgrad partials
  char* Cs = smem;                                   // [256][512 B], 16-B chunk ^ (row & 15)
  float gw[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) gw[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ml = wr * 128 + j * 16 + (lane & 15);
    const float d = dl[ml];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nl = wc * 64 + i * 16 + (lane >> 4) * 4;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = acc[i][j][r];
        gw[i][r] += d * a;
        o[r] = (nl + r < nv) ? d * w3[i][r] * (act_deriv_out(ACT, a) + h.flat_hid) : 0.f;
      }
      uint2 w;
      w.x = pack_bf16x2(o[0], o[1]);
      w.y = pack_bf16x2(o[2], o[3]);
      const int c = nl >> 3, half = (nl >> 2) & 1;
      *(uint2*)(Cs + ml * 512 + ((c ^ (ml & 15)) << 4) + half * 8) = w;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = gw[i][r];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if ((lane & 15) == 0) gred[wr * 256 + wc * 64 + i * 16 + (lane >> 4) * 4 + r] = v;
    }
  __syncthreads();
  if (tid < 256 && tid < h.KH) {
    const float v = gred[tid] + gred[256 + tid];
    if (h.GWslab) h.GWslab[(size_t)(m0 >> 8) * h.KH + tid] = v;     // tile index = row block
    else atomicAdd(h.GW + tid, v);
  }
  if (p.dbg & 8) return;                             // lab: no global D stores
  const int c = tid & 31;
#pragma unroll 4
  for (int pass = 0; pass < 16; ++pass) {
    const int ml = pass * 16 + (tid >> 5);
    const int m = m0 + ml, n = c * 8;
    if (m >= p.M || n >= p.N) continue;
    const uint4 v = *(const uint4*)(Cs + ml * 512 + ((c ^ (ml & 15)) << 4));
    if (n + 8 <= p.N) *(uint4*)(p.C + (size_t)m * p.ldc + n) = v;
    else *(uint2*)(p.C + (size_t)m * p.ldc + n) = make_uint2(v.x, v.y);
  }
}

// ---------------------------------------------------------------------------------------
// wgrad: G[n][k] += sum_m D[m][n] * X[m][k]   (TN GEMM over rows, split over m)
// LDS images [64 m][128 cols] bf16, 256-B rows, quad XOR swizzle so that the 8 rows read
// by one 32-lane half of ds_read_b64_tr_b16 hit 8 distinct bank groups.
// ---------------------------------------------------------------------------------------
constexpr int WT_BN = 128, WT_BK = 128, WT_BM = 64;   // n-tile, k-tile, rows per step
constexpr int WT_TILE = WT_BM * 128 * 2;              // 16 KiB


struct WgradArgs {
  const bf16_t* D; long ldd;   // [M, Nd] deltas
  const bf16_t* X; long ldx;   // [M, Kx] layer inputs
  float* G; long ldg;          // [Nv, Kx] fp32 gradient (accumulated atomically)
  int M, Nv, Kx, rows_per_split;
  int nsplit, interleave;      // interleave: split s takes the 64-row steps s, s+nsplit, ...
};

template <int STAGES>
__global__ __launch_bounds__(NTHR) void wgrad_tn_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = (p.Nv + WT_BN - 1) / WT_BN, tiles_k = p.Kx / WT_BK;
  const int ntiles = tiles_n * tiles_k;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, t = wg % ntiles;
  const int n0 = (t / tiles_k) * WT_BN, k0 = (t % tiles_k) * WT_BK;
  // contiguous splits: rows [mbeg, mend); interleaved splits: 64-row steps split + i*nsplit (the
  // whole grid then sweeps one narrow window of rows together: shared L2/MALL/TLB locality)
  const int mbeg = p.interleave ? split * WT_BM : split * p.rows_per_split;
  const int mend = p.interleave ? p.M : min(p.M, mbeg + p.rows_per_split);
  if (mbeg >= mend) return;
  const int mstride = p.interleave ? p.nsplit * WT_BM : WT_BM;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wk = wid & 1;

  uint4 rd[4], rx[4];
  auto gload = [&](int mb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 4, ch = idx & 15;
      const int gm = mb + row;
      const bool ok = gm < mend;
      const int gn = n0 + ch * 8;
      rd[i] = (ok && gn < p.Nv) ? *(const uint4*)(p.D + (size_t)gm * p.ldd + gn) : make_uint4(0, 0, 0, 0);
      rx[i] = ok ? *(const uint4*)(p.X + (size_t)gm * p.ldx + k0 + ch * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto swrite = [&](int buf) {
    char* Ds = smem + buf * 2 * WT_TILE;
    char* Xs = Ds + WT_TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 4, ch = idx & 15;
      *(uint4*)(Ds + swz_tn_quad(row, ch * 2)) = rd[i];
      *(uint4*)(Xs + swz_tn_quad(row, ch * 2)) = rx[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // tr read addressing: group g = lane>>4; lane-in-group t = 4q+p supplies row (8g+q [+4]),
  // quad (col_base/4 + p); lane receives column (col_base + t) of the 4 rows.
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int nsteps = (mend - mbeg + mstride - 1) / mstride;
  gload(mbeg);
  swrite(0);
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = STAGES == 2 ? (st & 1) : 0;
    if (st + 1 < nsteps) gload(mbeg + (st + 1) * mstride);
    const char* Ds = smem + buf * 2 * WT_TILE;
    const char* Xs = Ds + WT_TILE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {          // two 32-row k-substeps
      bf16x8 af[4], bfr[4];
      const int mr = s * 32 + 8 * g + tq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = (wn * 64 + i * 16) / 4 + tp;
        const s16x4 lo = ds_read_tr16_b64(Ds + swz_tn_quad(mr, q));
        const s16x4 hi = ds_read_tr16_b64(Ds + swz_tn_quad(mr + 4, q));
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = (wk * 64 + j * 16) / 4 + tp;
        const s16x4 lo = ds_read_tr16_b64(Xs + swz_tn_quad(mr, q));
        const s16x4 hi = ds_read_tr16_b64(Xs + swz_tn_quad(mr + 4, q));
        bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (STAGES == 1) __syncthreads();
    if (st + 1 < nsteps) swrite(STAGES == 2 ? (buf ^ 1) : 0);
    __syncthreads();
  }
  // acc[i][j]: D_out[n][k]: k = lane&15 (+16j), n = 4*(lane>>4) + r (+16i)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4 + r;
      if (n >= p.Nv) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + wk * 64 + j * 16 + (lane & 15);
        atomicAdd(p.G + (size_t)n * p.ldg + k, acc[i][j][r]);
      }
    }
}


// ---------------------------------------------------------------------------------------
// K15 pairwise-complete correlation sums (CorrAccumulator, shifu_amd/algos/stats.py; the
// reference's FastCorrelationMapper J/core/correlation/FastCorrelationMapper.java:171-278 adds
// fp64 products row by row).  corr_kernels.hip writes, per row chunk, int8 DIGIT PLANES
// [P][F][kpad] (feature-major, rows contiguous): the validity mask m and S balanced base-128
// digits of the column-scaled shifted value u = (x - c) / 2^ex and of u^2 / 2^ey.  Every sum is
// then an exact integer NT GEMM over the chunk's rows on v_mfma_i32_16x16x64_i8 (the 8-phase
// pipeline above, 2x the bf16 rate): a JOB is a list of (A plane, B plane) pairs that share one
// power-of-two weight (e.g. the digit diagonal s + t = d of u_i u_j), accumulated in int32
// (|digit| <= 64, <= 7 pairs: < 2^31 for chunks <= 64K rows), and flushed once per tile into its
// own fp64 [F][F] sum with the exact scale 2^(ea_i + eb_j - wexp).  Symmetric jobs (m'm, u'u)
// run the upper tiles only.
// ---------------------------------------------------------------------------------------
struct CorrJob {
  int npairs, ka, kb, wexp;    // ka / kb: scale row (0 ones, 1 2^ex, 2 2^ey); weight 2^-wexp
  int pa[7], pb[7];            // plane indices (npairs <= 7)
};
struct CorrArgs {
  const int8_t* planes; long plane_stride; int kpad, F;
  const CorrJob* jobs; const int4* items;   // item: {job, tile m, tile n, -}
  const double* scale;                       // [3][F]
  double* out; long out_stride;              // [jobs][F][F]
};

__global__ __launch_bounds__(G8_T, 1) void corr_i8_kernel(CorrArgs c) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int4 it4 = c.items[blockIdx.x];
  const int job = __builtin_amdgcn_readfirstlane(it4.x);
  const int4 it{job, __builtin_amdgcn_readfirstlane(it4.y), __builtin_amdgcn_readfirstlane(it4.z), 0};
  const CorrJob& jb = c.jobs[job];
  const int m0 = it.y * 256, n0 = it.z * 256;
  // the job's plane pairs are consecutive K segments of one pipeline
  GemmArgs p{};
  p.A = p.B = (const bf16_t*)c.planes;
  p.lda = p.ldb = c.kpad / 2;
  p.seg_shift = __builtin_ctz(c.kpad / 128);
  const int npairs = __builtin_amdgcn_readfirstlane(jb.npairs);
  p.K = npairs * (c.kpad / 2);
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    p.segA[i] = __builtin_amdgcn_readfirstlane(jb.pa[i]);
    p.segB[i] = __builtin_amdgcn_readfirstlane(jb.pb[i]);
  }
  p.seg_stride = c.plane_stride / 2;
  p.M = p.NB = p.N = c.F;
  f32x4 acc[4][8];
  int off[4][2];                      // 32-bit DMA offsets: a plane is < 2 GiB (host check)
  gemm8_src<int>(p, m0, n0, off);
  gemm8_prologue<true, int>(p, off, smem);
  gemm8_loop<true, int>(p, acc, off, smem);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const double* sa = c.scale + (long)jb.ka * c.F;
  const double* sb = c.scale + (long)jb.kb * c.F;
  const double w = __builtin_ldexp(1.0, -jb.wexp);
  double* o = c.out + (long)it.x * c.out_stride;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = m0 + wr * 128 + j * 16 + (lane & 15);
    if (m >= c.F) continue;
    const double am = sa[m] * w;
    double* row = o + (long)m * c.F;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = n0 + wc * 64 + i * 16 + (lane >> 4) * 4;
      const v4i_t v = __builtin_bit_cast(v4i_t, acc[i][j]);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (nb + r < c.F) row[nb + r] += (double)v[r] * am * sb[nb + r];
    }
  }
}
}  // namespace

// =======================================================================================
// C ABI (called through ctypes; host-side shape checks live in shifu_amd/ops/mlp.py and
// are repeated here so a bad call fails loudly instead of faulting the GPU).
// =======================================================================================
#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

static int g_stages = 1;     // LDS stages of the MLP GEMMs (A/B switch for tuning; 1 = default)
static int g_big = 0;        // large-M path: 0 = auto (8-phase for M >= 64K, N >= 512, K >= 512; else 128x128),
                             // 3 = 8-phase whenever M >= 64K and N >= 256, 4 = 128x128 only
static int g_wg_interleave = 1;   // wgrad row splits: 1 interleaved 64-row steps (-3% wgrad1 at 1M rows), 0 contiguous
static int g_dbg = 0;             // lab ablation bits (GemmArgs::dbg)
static int g_ring_nt = 1;         // persistent ring forward (gemm_ring_nt.hip, tune key 12; 2.2 vs 2.3-2.5 ms
                                  // for the 8-phase per-tile kernel per 2M-row chunk, profiles/r5)
static int g_ring_nt_cap = 0;     // lab: grid cap of the ring forward (tune key 13; 0 = one block per CU)
static int g_strip_nt = 1;        // row-strip forward engine (gemm_strip_nt.hip, tune key 14): 1 = before the ring
// gemm_ring_nt.hip (same library): -1 when the shape is not one it takes
extern "C" int shifu_ring_nt(const void* A, long lda, const void* B, long ldb, int NB, void* C, long ldc, int M,
                             int N, int K, int epi, int act, int n_valid, int bias_col, int grid_cap,
                             hipStream_t stream);
extern "C" int shifu_strip_nt(const void* A, long lda, const void* B, long ldb, int NB, void* C, long ldc, int M,
                              int N, int K, int epi, int act, int n_valid, int bias_col, int grid_cap,
                              hipStream_t stream);
SHIFU_API int shifu_gemm_set_stages(int s) { g_stages = (s == 2) ? 2 : 1; return 0; }
SHIFU_API int shifu_gemm_set_tune(int key, int val) {
  if (key == 2) { g_wg_interleave = val; return 0; }
  if (key == 9) { g_dbg = val; return 0; }
  if (key == 12) { g_ring_nt = val; return 0; }
  if (key == 13) { g_ring_nt_cap = val; return 0; }
  if (key == 14) { g_strip_nt = val; return 0; }
  return -1;
}
SHIFU_API int shifu_gemm_set_big(int b) { g_big = (b == 3 || b == 4) ? b : 0; return 0; }

SHIFU_API int shifu_gemm_nt(const void* A, long lda, const void* B, long ldb, int NB, void* C, long ldc,
                            void* C2, long ldc2, const void* H, long ldh, const void* Hd, long ldhd,
                            int M, int N, int K, int epi, int act, int n_valid, int bias_col, float flat,
                            hipStream_t stream) {
  if (K % BK || N % 4 || ldc % 8 || lda % 8 || ldb % 8 || M <= 0 || N <= 0) return -1;
  if (epi == EPI_DACT && H != nullptr && ldh % 8) return -1;     // 16-B row-segment loads of H
  GemmArgs p{(const bf16_t*)A, lda, (const bf16_t*)B, ldb, (bf16_t*)C, ldc, (bf16_t*)C2, ldc2,
             (const bf16_t*)H, ldh, (const bf16_t*)Hd, ldhd, M, N, K, NB, n_valid, act, bias_col, flat, g_dbg};
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const size_t lds = 2 * g_stages * TILE_BYTES;
  if (act < 0 || act > 9 || epi < 0 || epi > 3) return -2;
  if (epi == EPI_F32) {             // fp32 tile out: the 128 x 128 kernel (ldc counted in floats)
    if (ldc % 4) return -1;
    if (g_stages == 2) hipLaunchKernelGGL((gemm_nt_kernel<EPI_F32, 2, 2>), dim3(grid), dim3(NTHR), lds, stream, p);
    else hipLaunchKernelGGL((gemm_nt_kernel<EPI_F32, 2, 1>), dim3(grid), dim3(NTHR), lds, stream, p);
    CHECK_HIP(hipGetLastError());
    return 0;
  }
  if (epi == EPI_ACT && !act_deriv_from_output(act) && C2 == nullptr) return -3;
  if (epi == EPI_DACT && !act_deriv_from_output(act) && Hd == nullptr) return -3;
  if (epi == EPI_DACT && act_deriv_from_output(act) && H == nullptr) return -3;
  const bool dfo_act = act_deriv_from_output(act);
  // persistent ring engine (forward).  dgrad stays on the 128 x 128 tile kernel: a ring dgrad
  // (H row segments loaded into registers after the tile's last MMA segment) measured 1.81 vs
  // 1.23 ms per 2M-row chunk (profiles/r5/NOTES_r5.md) -- with K = 256 a tile has 8 k-steps, and
  // the H round trip at every tile end is exposed.
  if (g_strip_nt && M >= 65536 && (epi == EPI_STORE || (epi == EPI_ACT && dfo_act)) && !g_dbg) {
    const int r = shifu_strip_nt(A, lda, B, ldb, NB, C, ldc, M, N, K, epi, act, n_valid, bias_col, g_ring_nt_cap,
                                 stream);
    if (r != -1) return r;          // -1: shape not taken, fall through
  }
  if (g_ring_nt && M >= 65536 && (epi == EPI_STORE || (epi == EPI_ACT && dfo_act)) && !g_dbg) {
    const int r = shifu_ring_nt(A, lda, B, ldb, NB, C, ldc, M, N, K, epi, act, n_valid, bias_col, g_ring_nt_cap,
                                stream);
    if (r != -1) return r;          // -1: shape not taken, fall through
  }
  const bool auto8 = g_big == 0 && M >= 65536 && N >= 512 && K >= 512;
  if ((g_big == 3 || auto8) && M >= 65536 && N >= 256 && (epi == EPI_STORE || dfo_act)) {
    const int grid8 = ((M + 255) / 256) * ((N + 255) / 256);
    const size_t lds8 = 2 * G8_BUF;
#define GEMM8_L(E, A) hipLaunchKernelGGL((gemm_nt_8ph_kernel<E, A>), dim3(grid8), dim3(G8_T), lds8, stream, p)
#define GEMM8_ACTS(E) switch (act) { case 0: GEMM8_L(E, 0); break; case 1: GEMM8_L(E, 1); break; \
    case 2: GEMM8_L(E, 2); break; case 3: GEMM8_L(E, 3); break; case 4: GEMM8_L(E, 4); break; \
    case 6: GEMM8_L(E, 6); break; case 9: GEMM8_L(E, 9); break; default: GEMM8_L(E, 7); break; }
    if (epi == EPI_ACT) { GEMM8_ACTS(EPI_ACT) }
    else if (epi == EPI_DACT) { GEMM8_ACTS(EPI_DACT) }
    else GEMM8_L(EPI_STORE, 2);
#undef GEMM8_ACTS
#undef GEMM8_L
    CHECK_HIP(hipGetLastError());
    return 0;
  }
#define GEMM_L(E, A) do { if (g_stages == 2) \
    hipLaunchKernelGGL((gemm_nt_kernel<E, A, 2>), dim3(grid), dim3(NTHR), lds, stream, p); \
  else hipLaunchKernelGGL((gemm_nt_kernel<E, A, 1>), dim3(grid), dim3(NTHR), lds, stream, p); } while (0)
#define GEMM_ACTS(E) switch (act) { case 0: GEMM_L(E, 0); break; case 1: GEMM_L(E, 1); break; \
    case 2: GEMM_L(E, 2); break; case 3: GEMM_L(E, 3); break; case 4: GEMM_L(E, 4); break; \
    case 5: GEMM_L(E, 5); break; case 6: GEMM_L(E, 6); break; case 7: GEMM_L(E, 7); break; \
    case 9: GEMM_L(E, 9); break; default: GEMM_L(E, 8); break; }
  if (epi == EPI_ACT) { GEMM_ACTS(EPI_ACT) }
  else if (epi == EPI_DACT) { GEMM_ACTS(EPI_DACT) }
  else GEMM_L(EPI_STORE, 2);
#undef GEMM_ACTS
#undef GEMM_L
  CHECK_HIP(hipGetLastError());
  return 0;
}

// per-tile (error, weight) sums of the head -> err[0..1] in a fixed order (one block)
__global__ __launch_bounds__(256) void err_slab_kernel(const double* slab, int T, double* err) {
  __shared__ double sh[2][256];
  double a0 = 0.0, a1 = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) { a0 += slab[2 * t]; a1 += slab[2 * t + 1]; }
  sh[0][threadIdx.x] = a0;
  sh[1][threadIdx.x] = a1;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + w];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {              // the two chunk lanes add into the same err: atomic
    atomicAdd(err, sh[0][0]);
    atomicAdd(err + 1, sh[1][0]);
  }
}

// Fused head (see gemm_head_8ph_kernel): A [M, K] last-hidden inputs, B [NB, K] last-hidden
// weights (bf16), D out [M, N] deltas of the last hidden layer (N = padded width <= 256).
SHIFU_API int shifu_gemm_head(const void* A, long lda, const void* B, long ldb, int NB, void* D, long ldd,
                              int M, int N, int K, int act, int n_valid, const float* W, const float* Y,
                              const float* S, float* GW, double* err, int KH, int out_act, int loss,
                              float flat_out, float flat_hid, float* GWslab, double* errslab,
                              hipStream_t stream) {
  if (K % 64 || N % 8 || N > 256 || KH > 256 || KH < n_valid + 1 || lda % 8 || ldb % 8 || ldd % 8 ||
      M <= 0 || NB <= 0 || NB > 256)
    return -1;
  if (!act_deriv_from_output(act) || act == 6 || out_act < 0 || out_act > 9) return -2;
  GemmArgs p{(const bf16_t*)A, lda, (const bf16_t*)B, ldb, (bf16_t*)D, ldd, nullptr, 0, nullptr, 0, nullptr, 0,
             M, N, K, NB, n_valid, act, 1, 0.f, g_dbg};
  HeadArgs h{W, Y, S, GW, GWslab, err, (g_dbg & 1) ? nullptr : errslab, KH, out_act, loss, flat_out, flat_hid};
  const int grid = (M + 255) / 256;
#define HEAD_L(A_) hipLaunchKernelGGL((gemm_head_8ph_kernel<A_>), dim3(grid), dim3(G8_T), HEAD_LDS, stream, p, h)
  switch (act) {
    case 0: HEAD_L(0); break; case 1: HEAD_L(1); break; case 2: HEAD_L(2); break;
    case 3: HEAD_L(3); break; case 4: HEAD_L(4); break; case 9: HEAD_L(9); break; default: HEAD_L(7); break;
  }
#undef HEAD_L
  if (h.errslab) hipLaunchKernelGGL(err_slab_kernel, dim3(1), dim3(256), 0, stream, h.errslab, grid, err);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// Fixed-order column sums of per-tile partials: G[k] += sum_t slab[t][k] (t ascending within each
// 128-tile block, blocks ascending in the second pass) -- the deterministic replacement of the
// head's output-wgrad atomics.  part: [ceil(T / 128)][K] scratch.
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* slab, int T, int K, float* part) {
  const int k = threadIdx.x;
  if (k >= K) return;
  const int t0 = blockIdx.x * 128, t1 = min(T, t0 + 128);
  float s = 0.f;
  for (int t = t0; t < t1; ++t) s += slab[(size_t)t * K + k];
  part[(size_t)blockIdx.x * K + k] = s;
}
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* part, int B, int K, float* G) {
  const int k = threadIdx.x;
  if (k >= K) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += part[(size_t)b * K + k];
  G[k] += s;
}

SHIFU_API long shifu_colsum_ws(int T, int K) { return (long)((T + 127) / 128) * K * 4; }

SHIFU_API int shifu_colsum_fixed(const float* slab, int T, int K, float* part, float* G, hipStream_t stream) {
  if (T <= 0) return 0;
  if (K <= 0 || K > 256) return -1;
  const int B = (T + 127) / 128;
  hipLaunchKernelGGL(colsum_part_kernel, dim3(B), dim3(256), 0, stream, slab, T, K, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(1), dim3(256), 0, stream, part, B, K, G);
  CHECK_HIP(hipGetLastError());
  return 0;
}


SHIFU_API int shifu_wgrad_tn(const void* D, long ldd, const void* X, long ldx, float* G, long ldg,
                             int M, int Nv, int Kx, int splits, hipStream_t stream) {
  if (Kx % WT_BK || ldd % 8 || ldx % 8 || M <= 0 || Nv <= 0) return -1;
  if (splits < 1) splits = 1;
  int rps = (M + splits - 1) / splits;
  rps = ((rps + WT_BM - 1) / WT_BM) * WT_BM;
  splits = (M + rps - 1) / rps;
  WgradArgs p{(const bf16_t*)D, ldd, (const bf16_t*)X, ldx, G, ldg, M, Nv, Kx, rps, splits, g_wg_interleave};
  const int ntiles = ((Nv + WT_BN - 1) / WT_BN) * (Kx / WT_BK);
  if (g_stages == 2)
    hipLaunchKernelGGL(wgrad_tn_kernel<2>, dim3(ntiles * splits), dim3(NTHR), 4 * WT_TILE, stream, p);
  else
    hipLaunchKernelGGL(wgrad_tn_kernel<1>, dim3(ntiles * splits), dim3(NTHR), 2 * WT_TILE, stream, p);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// K15 correlation sums: one launch per row chunk over n_items (job, tile) items (ordered by the
// caller); planes [P][F][kpad] int8, kpad a power of two in [128, 65536] (int32 accumulation
// bound: 7 pairs x 64^2 x 65536 < 2^31).
SHIFU_API int shifu_corr_gemm(const void* planes, long plane_stride, int kpad, int F, const void* jobs,
                              const void* items, int n_items, const double* scale, double* out,
                              long out_stride, hipStream_t stream) {
  if (kpad < 128 || (kpad & (kpad - 1)) || kpad > 65536 || F <= 0 || plane_stride < (long)F * kpad || plane_stride % 2 ||
      n_items < 0 ||
      out_stride < (long)F * F)
    return -1;
  if (n_items == 0) return 0;
  if ((long)F * kpad >= (1l << 31)) return -1;
  CorrArgs c{(const int8_t*)planes, plane_stride, kpad, F, (const CorrJob*)jobs, (const int4*)items, scale,
             out, out_stride};
  hipLaunchKernelGGL(corr_i8_kernel, dim3(n_items), dim3(G8_T), 2 * G8_BUF, stream, c);
  CHECK_HIP(hipGetLastError());
  return 0;
}
SHIFU_API int shifu_corr_job_bytes() { return (int)sizeof(CorrJob); }

// ---------------------------------------------------------------------------------------------
// Split-bf16 operand builder for the fp32-accurate GEMM (ops/gemm_ops.py): x [M, K] fp32 (ld ldx)
// -> A[:, t*K : (t+1)*K] = part_{xsel(t)}(x) for the T term pairs, parts hi = bf16(x),
// mid = bf16(x - hi), lo = bf16(x - hi - mid) (residuals exact in fp32).  One pass: each lane
// reads V consecutive floats once and writes its V bf16 per term (the torch form takes ~10
// elementwise passes).  xsel packs 2 bits per term.
// ---------------------------------------------------------------------------------------------
template <int V>
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ x, long ldx, long M, int K,
                                                          bf16_t* __restrict__ A, long lda, int T, int xsel) {
  const int KV = K / V;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * KV) return;
  const long r = idx / KV;
  const int k = (int)(idx - r * KV) * V;
  float v[V];
  if constexpr (V == 4) {
    const float4 q = *(const float4*)(x + r * ldx + k);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    v[0] = x[r * ldx + k];
  }
  bf16_t part[3][V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    float rem = v[e];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      part[q][e] = f2bf(rem);
      rem -= bf2f(part[q][e]);
    }
  }
  bf16_t* dst = A + r * lda + k;
  for (int t = 0; t < T; ++t) {
    const int s = (xsel >> (2 * t)) & 3;
    if constexpr (V == 4) {
      const bf16_t* p = s == 0 ? part[0] : (s == 1 ? part[1] : part[2]);
      *(uint2*)(dst + (long)t * K) = make_uint2((uint32_t)p[0] | ((uint32_t)p[1] << 16),
                                                (uint32_t)p[2] | ((uint32_t)p[3] << 16));
    } else {
      dst[(long)t * K] = s == 0 ? part[0][0] : (s == 1 ? part[1][0] : part[2][0]);
    }
  }
}

SHIFU_API int shifu_split_bf16_rows(const float* x, long ldx, long M, int K, void* A, long lda, int T, int xsel,
                                    hipStream_t stream) {
  if (M <= 0 || K <= 0) return 0;
  if (T < 1 || T > 15 || ldx < K || lda < (long)T * K) return -1;
  const bool vec = (K % 4 == 0) && (ldx % 4 == 0) && (lda % 4 == 0) && ((uintptr_t)x % 16 == 0) &&
                   ((uintptr_t)A % 8 == 0);
  const long n = M * (vec ? K / 4 : K);
  const long blocks = (n + 255) / 256;
  if (blocks > 0x7fffffffL) return -1;
  if (vec)
    hipLaunchKernelGGL(split_rows_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, stream, x, ldx, M, K,
                       (bf16_t*)A, lda, T, xsel);
  else
    hipLaunchKernelGGL(split_rows_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, stream, x, ldx, M, K,
                       (bf16_t*)A, lda, T, xsel);
  CHECK_HIP(hipGetLastError());
  return 0;
}
