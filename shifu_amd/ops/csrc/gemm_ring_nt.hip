// Persistent ring-pipelined MFMA NT GEMM for the MLP forward (gfx950 / CDNA4).
//
//   C[m][n] = act( sum_k A[m][k] B[n][k] )     A [M, K] layer inputs, B [NB, K] weights (bf16),
//                                              C [M, N] bf16 (FloatFlatNetwork.java:148-178 computes
//                                              the same per-record dot products one record at a time)
//
// Why (profiles/r4/NOTES_r4.md, "MLP forward GEMM ablation"): the one-tile-per-block 8-phase
// kernel spent 0.7 of its 2.64 ms per 2M-row chunk in the epilogue + next block's pipeline fill
// (one block per CU: nothing overlaps a block's store tail or its first HBM round trip), and its
// main loop paid 8 barriers per 64-deep k-tile.  This engine is the wgrad ring (gemm_ring.hip,
// ~1.3 PF on the same chunk) turned into an NT persistent kernel:
//   * one 512-thread block per CU walks its 256 x 256 output tiles t = lb, lb + G, ...; the
//     K axis of every tile is cut into 32-deep k-steps and the (tile, k-step) sequence is
//     flattened, so the LDS-DMA ring (5 slots x 32 KiB: A image [256 rows][64 B] + B image
//     [256 rows][64 B]) runs 4 steps ahead ACROSS tile boundaries -- the next tile's first
//     operands are in LDS when the current tile's epilogue starts;
//   * one LD segment (12 ds_read_b128 fragment reads + counted waits) and one MMA segment (32 x
//     mfma_f32_16x16x32_bf16 with the 4 LDS-DMA pieces of step t+4 interleaved) per k-step, raw
//     s_barriers between them; waves 4-7 run one barrier behind waves 0-3, so on every SIMD one
//     wave's MFMAs overlap the other's reads (and its epilogue VALU at tile ends);
//   * the epilogue writes straight from the accumulators: activation, bf16 pack, one
//     v_permlane16_swap per dword pair (cdna_hip_programming.md T21, the 16-lane form) so that
//     every lane holds 8 consecutive columns, and 16 buffer_store_dwordx4 per wave (rows >= M and
//     columns >= N fall outside the buffer resource and are dropped: the store count is the same
//     on every tile, which keeps the counted vmcnt waits exact).  No LDS staging, no barrier.
//   * 64-B image rows: 16-B chunk c of row r sits at c ^ x(r), x = [0, 2, 3, 1][(r >> 2) & 3] --
//     the 16 lanes of each ds_read_b128 lane group ({0-3,12-15,20-27}, ...) then hit 16 distinct
//     16-B bank slots (conflict-free); the DMA applies the swizzle on the SOURCE address.
// Numerics: the k order per accumulator is ascending 32-deep steps, exactly the 8-phase kernel's
// (c = 0, 1 within each 64-deep tile), so both kernels give bitwise-identical outputs.
//
// Schedule (per wave; "lag" = waves 4-7, one extra barrier up front):
//   prologue: DMA steps 0..3; vmcnt(12); BAR; [lag: BAR]
//   step t:   LD:  [tile start: epilogue of the previous tile]; read fragments of step t;
//                  vmcnt(8) (own DMAs of step t+1 landed; steps t+2, t+3 in flight) -- vmcnt(24)
//                  in the three LD segments after an epilogue, whose 16 stores are younger;
//                  lgkmcnt(0); BAR
//             MMA: 32 MFMAs + DMA of step t+4 into slot (t+4)%5 (= the slot of step t-1); BAR
//   end:      epilogue of the last tile; [lead: BAR]; vmcnt(0)
// RAW: every wave waits for its own step t+1 DMAs before the barrier that precedes any wave's
// reads of step t+1.  WAR: slot (t-1)%5 is refilled in MMA(t); every wave finished its reads of
// step t-1 (lgkmcnt(0)) before the barrier that ended its LD(t-1), which precedes MMA(t) of both
// wave groups.
#include "common.h"
#include <type_traits>
#include <utility>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((ext_vector_type(4))) int v4i_t;

constexpr int RN_T = 512;
constexpr int RN_NSLOT = 5;
constexpr int RN_IMG = 256 * 64;             // 16 KiB: [256 rows][32 bf16]
constexpr int RN_SLOT = 2 * RN_IMG;          // A image + B image
constexpr int RN_LDS = RN_NSLOT * RN_SLOT;   // 160 KiB
enum { RN_EPI_ACT = 0, RN_EPI_STORE = 2 };   // same codes as gemm_kernels.hip's Epi

__device__ __forceinline__ int rn_xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}
__device__ __forceinline__ int rn_xor(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

template <int OFF>
__device__ __forceinline__ bf16x8 rn_read(uint32_t a) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}

template <int I> struct RnIC { static constexpr int v = I; };
template <typename F, int... Is>
__device__ __forceinline__ void rn_for_impl(F&& f, std::integer_sequence<int, Is...>) { (f(RnIC<Is>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void rn_for(F&& f) { rn_for_impl(f, std::make_integer_sequence<int, N>{}); }

struct RingNTArgs {
  const bf16_t* A; long lda;   // [M, K]
  const bf16_t* B; long ldb;   // [NB, K] (rows >= NB read row NB-1; those columns are overwritten)
  bf16_t* C; long ldc;         // [M, N]
  int M, N, K, NB, n_valid, bias_col;
  int ntiles;                  // ceil(M / 256) * ceil(N / 256)
  // LAB builds only (never the shipped kernel): ablation bits and per-wave segment cycle sums
  //   dbg 1: no epilogue (acc kept live, zeroed), 2: epilogue stores z (no activation),
  //       4: no MFMAs (fragments kept live), 8: A rows from a 4096-row window (MALL), 16: from a
  //       256-row window (every block re-reads the same 512 KB: L2-resident), 32: every MFMA
  //       issued twice (wrong sums; the marginal cost of the MMA segment's MFMAs)
  int dbg;
  unsigned long long* stamps;  // [blocks][8 waves][8]: epilogue, reads, waits, LD barrier, MMA, MMA barrier, T, lb
};

template <int EPI, int ACT, bool LAB, int VAR>
__global__ __launch_bounds__(RN_T, 2) void ring_nt_kernel(RingNTArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = gridDim.x;
  const int lb = rn_xcd_remap(blockIdx.x, G);
  if (lb >= p.ntiles) return;                        // whole block
  const int ntn = (p.N + 255) >> 8;
  const int nk = p.K >> 5;
  const int T = ((p.ntiles - 1 - lb) / G + 1) * nk;  // flattened k-steps of this block
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  // the lag group: one barrier behind, so each SIMD pairs a computing wave with a reading one
  // (VAR bit 3: odd waves instead of waves 4-7 -- lab check of the wave -> SIMD placement)
  const bool lag = (VAR & 8) ? (wid & 1) != 0 : wid >= 4;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  // ---- LDS-DMA cursor over the flattened (tile, k-step) sequence
  int d_tile = lb, d_k = 0, d_left = T - 1;
  const char* dA;
  const char* dB;
  uint32_t offA[2], offB[2];
  auto dma_tile = [&](int t) __attribute__((always_inline)) {
    const int m0 = (t / ntn) * 256, n0 = (t % ntn) * 256;
    const bool win = LAB && (p.dbg & 24);            // lab: rows (m0 + r) & 4095 (8) / & 255 (16) of A
    dA = (const char*)(p.A + (size_t)(win ? 0 : m0) * p.lda);
    dB = (const char*)p.B;                           // absolute rows: a column tile may start at n0 >= NB
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int P = (i * 8 + wid) * 1024 + lane * 16;
      const int row = P >> 6, c = ((P >> 4) & 3) ^ rn_xor(row);
      const int ra = win ? (min(m0 + row, p.M - 1) & ((p.dbg & 16) ? 255 : 4095)) : min(m0 + row, p.M - 1) - m0;
      const int rb = min(n0 + row, p.NB - 1);      // rows >= NB read row NB-1 (columns overwritten)
      offA[i] = (uint32_t)(ra * p.lda + c * 8) * 2u;
      offB[i] = (uint32_t)(rb * p.ldb + c * 8) * 2u;
    }
  };
  dma_tile(d_tile);
  // one of the 4 LDS-DMA instructions of a step (q = 0, 1: A halves; 2, 3: B halves); q == 3 advances
  auto dma_piece = [&](int slot, int q) __attribute__((always_inline)) {
    char* base = smem + slot * RN_SLOT + wid_u * 1024 + (q >> 1) * RN_IMG + (q & 1) * 8192;
    const char* src = (q < 2 ? dA + offA[q & 1] : dB + offB[q & 1]) + d_k * 64;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)base, 16, 0, 0);
    if (q == 3 && d_left > 0) {                      // past the end: re-read the last step
      --d_left;
      if (++d_k == nk) { d_k = 0; d_tile += G; dma_tile(d_tile); }
    }
  };
  auto dma_step = [&](int slot) __attribute__((always_inline)) { dma_piece(slot, 0); dma_piece(slot, 1); dma_piece(slot, 2); dma_piece(slot, 3); };

  f32x4 acc[4][8];                                   // [n block][m block]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lq = lane >> 4;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const uint32_t oA = (uint32_t)((wr * 128 + lr) * 64 + ((lq ^ rn_xor(lr)) << 4));
  const uint32_t oB = (uint32_t)(RN_IMG + (wc * 64 + lr) * 64 + ((lq ^ rn_xor(lr)) << 4));
  bf16x8 af[8], bfr[4];
  constexpr int DMA_LD = (VAR & 3) == 1 ? 4 : (VAR & 3) == 2 ? 2 : 0;   // DMA pieces issued in the LD segment
  constexpr bool DEFER = (VAR & 4) != 0;     // epilogue: pack everything, then 16 stores whose data
                                             // registers stay untouched until the next MMA segment

  // ---- epilogue of tile t: activation + bf16 pack + permlane16 widening into pk
  uint32_t pk[2][8][4];
  // rows >= M / columns >= N: offsets outside the tile's buffer resource (dropped by the hardware)
  auto store_one_impl = [&](int t, int np, int mb) __attribute__((always_inline)) {
    const int m0 = (t / ntn) * 256, n0 = (t % ntn) * 256;
    const int rows = min(256, p.M - m0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.C + (size_t)m0 * p.ldc), (short)0, rows * (int)p.ldc * 2, 0x00020000);
    const int nl = wc * 64 + np * 32 + 16 * (lq & 1) + 8 * (lq >> 1);
    const int ml = wr * 128 + mb * 16 + lr;
    const int off = n0 + nl < p.N ? (int)((ml * p.ldc + n0 + nl) * 2) : (int)0x7ffffff0;
    const v4i_t v = {(int)pk[np][mb][0], (int)pk[np][mb][1], (int)pk[np][mb][2], (int)pk[np][mb][3]};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
  };
  (void)store_one_impl;
  auto pack_tile = [&](int t, auto FULL, auto USE_ACT) __attribute__((always_inline)) {
    const int n0 = (t % ntn) * 256;
#pragma unroll
    for (int np = 0; np < 2; ++np) {
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        uint32_t w[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float z = acc[2 * np + s][mb][r];
            const float a = (EPI == RN_EPI_ACT && decltype(USE_ACT)::value) ? act_fwd(ACT, z) : z;
            if constexpr (decltype(FULL)::value) {
              o[r] = a;
            } else {                                 // branch-free column masks
              const int n = n0 + wc * 64 + (2 * np + s) * 16 + 4 * lq + r;
              if constexpr (EPI == RN_EPI_ACT) o[r] = n < p.n_valid ? a : ((n == p.n_valid && p.bias_col) ? 1.f : 0.f);
              else o[r] = n < p.NB ? a : 0.f;
            }
          }
          w[s][0] = pack_bf16x2(o[0], o[1]);
          w[s][1] = pack_bf16x2(o[2], o[3]);
        }
        // odd 16-lane rows of w[0] <-> even rows of w[1]: lane row q then holds columns
        // 16(q & 1) + 8(q >> 1) .. +7 of the n-block pair (w[0] part first)
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r2 = __builtin_amdgcn_permlane16_swap(w[0][d], w[1][d], false, false);
          w[0][d] = r2[0];
          w[1][d] = r2[1];
        }
        pk[np][mb][0] = w[0][0]; pk[np][mb][1] = w[0][1]; pk[np][mb][2] = w[1][0]; pk[np][mb][3] = w[1][1];
        if constexpr (!DEFER) store_one_impl(t, np, mb);
      }
    }
  };
  auto pack = [&](int t) __attribute__((always_inline)) {
    const int n0 = (t % ntn) * 256;
    if (LAB && (p.dbg & 2)) { pack_tile(t, std::integral_constant<bool, true>{}, std::integral_constant<bool, false>{}); return; }
    if (n0 + 256 <= (EPI == RN_EPI_ACT ? p.n_valid : p.NB))
      pack_tile(t, std::integral_constant<bool, true>{}, std::integral_constant<bool, true>{});
    else pack_tile(t, std::integral_constant<bool, false>{}, std::integral_constant<bool, true>{});
  };
  // the epilogue of tile t (16 stores per wave); !DEFER: acc zeroed here
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    if (LAB && (p.dbg & 1)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" :: "v"(acc[i][j]));
#pragma unroll
      for (int np = 0; np < 2; ++np)
#pragma unroll
        for (int mb = 0; mb < 8; ++mb)
#pragma unroll
          for (int d = 0; d < 4; ++d) pk[np][mb][d] = 0;
    } else {
      pack(t);
    }
    if constexpr (DEFER) {
#pragma unroll
      for (int np = 0; np < 2; ++np)
#pragma unroll
        for (int mb = 0; mb < 8; ++mb) store_one_impl(t, np, mb);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // keeps the stored registers live (unreused) until after the LD segment's barrier
  auto keep_pk = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int np = 0; np < 2; ++np)
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        const v4i_t v = {(int)pk[np][mb][0], (int)pk[np][mb][1], (int)pk[np][mb][2], (int)pk[np][mb][3]};
        asm volatile("" :: "v"(v));
      }
  };

#define RN_BAR() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); \
                      __builtin_amdgcn_sched_barrier(0); } while (0)

  dma_step(0); dma_step(1); dma_step(2); dma_step(3);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  RN_BAR();
  if (lag) RN_BAR();

  unsigned long long st_sum[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if constexpr (LAB) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (k >= 0) st_sum[k] += now - st_prev;
      st_prev = now;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // the 32 MFMAs of a k-step (+ the DMA pieces of step t+4 not issued in the LD segment); ZC:
  // first step of a tile under DEFER -- a zero accumulator input instead of zeroed registers
  int slot = 0, dslot = 4, kk = 0, tile = lb, since_epi = 0;
  auto mma = [&](auto ZC) __attribute__((always_inline)) {
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      if (LAB && (p.dbg & 4)) {
        asm volatile("" :: "v"(af[mb]));
        if (mb == 0) {
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) asm volatile("" :: "v"(bfr[nb]));
        }
      } else {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              bfr[nb], af[mb], decltype(ZC)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[nb][mb], 0, 0, 0);
        if (LAB && (p.dbg & 32)) {                   // lab: every MFMA twice (marginal MFMA cost)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
            acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nb], af[mb], acc[nb][mb], 0, 0, 0);
        }
      }
      if constexpr (DMA_LD < 4) {
        if ((DMA_LD == 0 && (mb & 1)) || (DMA_LD == 2 && (mb == 3 || mb == 7))) {
          __builtin_amdgcn_sched_barrier(0);
          dma_piece(dslot, DMA_LD == 0 ? (mb >> 1) : (mb == 3 ? 2 : 3));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  };
  for (int t = 0; t < T; ++t) {
    // ---- LD segment (opened by the previous tile's epilogue at a tile start)
    stamp(-1);
    if (kk == 0 && t > 0) {
      __builtin_amdgcn_sched_barrier(0);
      epilogue(tile - G);
      since_epi = 3;
      __builtin_amdgcn_sched_barrier(0);
    }
    stamp(0);
    if constexpr (DMA_LD > 0) {
      __builtin_amdgcn_sched_barrier(0);
      dma_piece(dslot, 0);
      dma_piece(dslot, 1);
      if constexpr (DMA_LD == 4) { dma_piece(dslot, 2); dma_piece(dslot, 3); }
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t sa = lds0 + slot * RN_SLOT + oA, sb = lds0 + slot * RN_SLOT + oB;
    rn_for<4>([&](auto I) { bfr[I.v] = rn_read<I.v * 1024>(sb); });
    rn_for<8>([&](auto I) { af[I.v] = rn_read<I.v * 1024>(sa); });
    stamp(1);
    // own DMAs of step t+1 landed: younger are steps t+2, t+3 and the pieces of t+4 issued so far
    // (+16 epilogue stores in the three LD segments after a tile end)
    if (since_epi > 0) {
      --since_epi;
      if constexpr (DMA_LD == 4) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
      else if constexpr (DMA_LD == 2) asm volatile("s_waitcnt vmcnt(26)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    } else {
      if constexpr (DMA_LD == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if constexpr (DMA_LD == 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(2);
    RN_BAR();
    stamp(3);
    // ---- MMA segment
    __builtin_amdgcn_s_setprio(1);
    if constexpr (DEFER) {
      if (kk == 0) {
        if (t > 0) keep_pk();
        mma(std::integral_constant<bool, true>{});
      } else {
        mma(std::integral_constant<bool, false>{});
      }
    } else {
      mma(std::integral_constant<bool, false>{});
    }
    __builtin_amdgcn_s_setprio(0);
    stamp(4);
    RN_BAR();
    stamp(5);
    slot = slot == RN_NSLOT - 1 ? 0 : slot + 1;
    dslot = dslot == RN_NSLOT - 1 ? 0 : dslot + 1;
    if (++kk == nk) { kk = 0; tile += G; }
  }
  epilogue(tile - G);
  if (!lag) RN_BAR();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef RN_BAR
  if constexpr (LAB) {
    if (lane == 0 && p.stamps) {
      unsigned long long* d = p.stamps + ((size_t)blockIdx.x * 8 + wid) * 8;
      for (int k = 0; k < 6; ++k) d[k] = st_sum[k];
      d[6] = T;
      // HW_ID: wave slot [3:0], SIMD [5:4], CU [11:8] (gfx9 layout)
      d[7] = ((unsigned long long)lb << 32) | (unsigned)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    }
  }
}

}  // namespace

static int g_rn_dbg = -1;                    // LAB build switch: >= 0 runs ring_nt_kernel<.., LAB>
static unsigned long long* g_rn_stamps = nullptr;
constexpr int RN_DEFAULT_VAR = 0;            // DMA pieces in the MMA segment, per-pair stores
static int g_rn_var = RN_DEFAULT_VAR;        // sigmoid / store builds: schedule variant (lab A/B)
// Lab switch (tools/ring_lab.py): dbg >= 0 selects the LAB build (sigmoid / store only) with
// those ablation bits; buf (>= blocks * 64 u64, nullable) receives the segment cycle sums.
SHIFU_API int shifu_ring_nt_set_lab(int dbg, void* buf) {
  g_rn_dbg = dbg;
  g_rn_stamps = (unsigned long long*)buf;
  return 0;
}
// variant bits: 0-1 DMA placement (0: all 4 pieces in the MMA segment, 1: all in the LD segment,
// 2: two each), 2: deferred epilogue (pack all, 16 stores, registers untouched until the next MMA)
SHIFU_API int shifu_ring_nt_set_variant(int v) {
  if (v < 0 || (v & 4) || (v & 3) == 3 || v > 9) return -1;   // deferred-epilogue builds (bit 2) spill
  g_rn_var = v;
  return 0;
}

template <int EPI, int ACT, bool LAB>
static void rn_launch(int var, dim3 grid, hipStream_t stream, const RingNTArgs& p) {
#define RN_V(V) hipLaunchKernelGGL((ring_nt_kernel<EPI, ACT, LAB, V>), grid, dim3(RN_T), RN_LDS, stream, p)
  switch (var) {
    case 1: RN_V(1); break; case 2: RN_V(2); break; case 8: RN_V(8); break; case 9: RN_V(9); break;
    default: RN_V(0); break;
  }
#undef RN_V
}

// C ABI: returns -1 when the shape is not one this engine takes (the caller falls back).
// epi 0 = activation (derivative computable from the output: no f'(z) side output), 2 = store z.
SHIFU_API int shifu_ring_nt(const void* A, long lda, const void* B, long ldb, int NB, void* C, long ldc, int M,
                            int N, int K, int epi, int act, int n_valid, int bias_col, int grid_cap,
                            hipStream_t stream) {
  if (K % 32 || K < 128 || lda % 8 || ldb % 8 || ldc % 8 || N % 8 || M <= 0 || N <= 0 || NB <= 0) return -1;
  if (epi != RN_EPI_ACT && epi != RN_EPI_STORE) return -1;
  if (epi == RN_EPI_ACT && !act_deriv_from_output(act)) return -1;
  if ((long)K * 2 * 256 >= (1l << 31) || 256l * ldc * 2 >= (1l << 31)) return -1;   // 32-bit offsets
  if (lda < K || ldb < K || ldc < N) return -1;
  if ((long)NB * ldb * 2 >= (1l << 32)) return -1;                                     // B offsets are 32-bit
  const long ntiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  if (ntiles >= (1l << 31)) return -1;
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int grid = (int)(ntiles < ncu ? ntiles : ncu);
  if (grid_cap > 0 && grid > grid_cap) grid = grid_cap;
  RingNTArgs p{(const bf16_t*)A, lda, (const bf16_t*)B, ldb, (bf16_t*)C, ldc, M, N, K, NB, n_valid, bias_col,
               (int)ntiles, g_rn_dbg, g_rn_stamps};
  const dim3 g(grid);
  if (g_rn_dbg >= 0) {
    if (epi == RN_EPI_ACT && act == 0) rn_launch<RN_EPI_ACT, 0, true>(g_rn_var, g, stream, p);
    else if (epi == RN_EPI_STORE) rn_launch<RN_EPI_STORE, 2, true>(g_rn_var, g, stream, p);
    else return -1;
  } else if (epi == RN_EPI_STORE) {
    rn_launch<RN_EPI_STORE, 2, false>(g_rn_var, g, stream, p);
  } else if (act == 0) {
    rn_launch<RN_EPI_ACT, 0, false>(g_rn_var, g, stream, p);
  } else {
#define RN_L(A_) hipLaunchKernelGGL((ring_nt_kernel<RN_EPI_ACT, A_, false, RN_DEFAULT_VAR>), g, dim3(RN_T), RN_LDS, \
                                    stream, p)
    switch (act) {
      case 1: RN_L(1); break; case 2: RN_L(2); break; case 3: RN_L(3); break; case 4: RN_L(4); break;
      case 6: RN_L(6); break; case 9: RN_L(9); break; default: RN_L(7); break;
    }
#undef RN_L
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
