// Persistent "row-strip" MFMA NT GEMM for the MLP forward (gfx950 / CDNA4).
//
//   C[m][n] = act( sum_k A[m][k] B[n][k] )     A [M, K] layer inputs, B [NB, K] weights (bf16),
//                                              C [M, N] bf16 (FloatFlatNetwork.java:148-178 computes
//                                              the same per-record dot products one record at a time)
//
// Why a second forward engine (profiles/r5/NOTES_r5.md, section 1): the ring engine
// (gemm_ring_nt.hip) stages BOTH operands of its 256 x 256 tile by LDS-DMA in 32-deep k-steps, so
// every 1-KiB DMA piece covers 16 rows x 64 B -- half of each 128-B line -- and its ablations put
// the loop on that fill path (1.45-1.55 ms of the 2.3 ms per 2M-row chunk with the MFMAs removed,
// about the same with the A rows L2-resident).  Here:
//   * the k-step is 64 deep, so every global request covers whole 128-B lines;
//   * wave w of the 512-thread block owns the 32-row strip [32w, 32w + 32) of the 256-row tile and
//     all 256 columns, so no other wave needs its A rows: each lane loads its A fragments global ->
//     VGPR (4 global_load_dwordx4 per k-step: two m-blocks x the two 32-deep halves, the halves of a
//     row issued back to back = one whole line), 2 k-steps ahead into a 2-entry register ring;
//   * only the B tile (256 weight rows x 128 B = 32 KiB per k-step, shared by the 8 waves) goes
//     through LDS: 32 LDS-DMA pieces of 8 rows x 128 B per k-step, 4 per wave, into a 4-slot ring
//     running 2 k-steps ahead across tile boundaries (the (tile, k-step) sequence is flattened);
//     16-B chunk c of row r sits at c ^ ((r >> 1) & 7): every ds_read_b128 lane group hits 16
//     distinct bank slots;
//   * per k-step 32 B fragments are read (eight double-buffered groups of 4) and feed 64 x
//     mfma_f32_16x16x32_bf16 per wave; ONE barrier per k-step;
//   * the epilogue (activation, bf16 pack, v_permlane16_swap widening, 16 buffer_store_dwordx4 per
//     wave) is the ring engine's; rows >= M / columns >= N fall outside the store resource.
// The A loads are inline asm (hipcc waits vmcnt(0) at the first use of any ordinary load result
// while an LDS-DMA is in flight -- cdna_hip_programming.md §5 'Pipelining across barriers'); their
// completion is counted by hand with the DMA pieces and the epilogue stores in one vmcnt ladder.
// Numerics: every accumulator adds its 32-deep halves in ascending k order, like the ring and the
// 8-phase kernels, so the outputs are bitwise identical to theirs.
//
// Schedule per wave (D = 2 steps ahead, A ring of 2 entries; e = t mod 2):
//   prologue: groups 0, 1 (DMA x4, A x4 each); vmcnt(8); barrier
//   step t:   8 MMA groups (B fragments from slot t mod 4, A ring entry e);
//             group t+2: DMA x4 into slot (t+2) mod 4, A x4 into ring entry e;
//             [last k-step of a tile: epilogue, 16 stores];
//             vmcnt(8) (24 in the 2 steps after an epilogue) -> own group t+1 landed; barrier
// RAW: a wave's own pieces of step t+1 landed before the barrier that precedes every wave's reads
// of that slot.  WAR: slot (t+2) mod 4 was last read in step t-2, behind the barrier that ended
// step t-1.  (Issuing step t+2's loads between the MMA groups, with a 3-entry ring, measured the
// same: 2.19 ms vs 2.18-2.20, strip_lab_d.)
#include "common.h"
#include <type_traits>
#include <utility>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((ext_vector_type(4))) int v4i_t;

constexpr int SN_T = 512;
constexpr int SN_D = 2;                      // k-steps ahead: step t issues the loads of step t+D
constexpr int SN_P = SN_D;                   // A ring entries = unroll (entry t mod 2 reloaded after use)
constexpr int SN_NSLOT = SN_D + 2;           // B slots: + the slot being read + the one landed
constexpr int SN_SLOT = 256 * 128;           // 32 KiB: B image [256 rows][64 bf16]
constexpr int SN_LDS = SN_NSLOT * SN_SLOT;   // 128 KiB
enum { SN_EPI_ACT = 0, SN_EPI_STORE = 2 };   // same codes as gemm_kernels.hip's Epi

__device__ __forceinline__ int sn_xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <int OFF>
__device__ __forceinline__ bf16x8 sn_read(uint32_t a) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}
// "+v": the load's destination is tied to the ring entry's current register (the entry is
// overwritten in place; hipcc has no new value to place elsewhere)
template <int OFF>
__device__ __forceinline__ void sn_gload(bf16x8& v, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "+v"(v) : "v"(p), "n"(OFF) : "memory");
}

template <int I> struct SnIC { static constexpr int v = I; };
template <typename F, int... Is>
__device__ __forceinline__ void sn_for_impl(F&& f, std::integer_sequence<int, Is...>) { (f(SnIC<Is>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void sn_for(F&& f) { sn_for_impl(f, std::make_integer_sequence<int, N>{}); }

struct StripArgs {
  const bf16_t* A; long lda;   // [M, K]
  const bf16_t* B; long ldb;   // [NB, K] (rows >= NB read row NB-1; those columns are overwritten)
  bf16_t* C; long ldc;         // [M, N]
  int M, N, K, NB, n_valid, bias_col;
  int ntiles;                  // ceil(M / 256) * ceil(N / 256)
  int dbg;                     // LAB builds only: 1 no epilogue, 4 no MFMAs (operands kept live),
                               // 8 no B LDS-DMA, 16 no A loads (timing ablations: results invalid)
};

template <int EPI, int ACT, bool LAB>
__global__ __launch_bounds__(SN_T, 2) void strip_nt_kernel(StripArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = gridDim.x;
  const int lb = sn_xcd_remap(blockIdx.x, G);
  if (lb >= p.ntiles) return;                        // whole block
  const int ntn = (p.N + 255) >> 8;
  const int nk = p.K >> 6;
  const int T = ((p.ntiles - 1 - lb) / G + 1) * nk;  // flattened k-steps of this block
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int lr = lane & 15, lq = lane >> 4;

  // ---- load cursor over the flattened (tile, k-step) sequence, P steps ahead of the MMAs
  int c_tile = lb, c_k = 0, c_left = T - 1;
  const char* aptr[2];                               // this lane's A fragment rows (k-step 0)
  const char* bptr[4];                               // this lane's B DMA source rows (k-step 0)
  auto cursor_tile = [&](int t) __attribute__((always_inline)) {
    const int m0 = (t / ntn) * 256, n0 = (t % ntn) * 256;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = min(m0 + wid * 32 + i * 16 + lr, p.M - 1);   // rows >= M: stores dropped
      aptr[i] = (const char*)(p.A + (size_t)m * p.lda) + lq * 16;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (wid * 4 + i) * 8 + (lane >> 3);           // DMA piece: B rows 8q .. 8q+7
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int nb = min(n0 + row, p.NB - 1);
      bptr[i] = (const char*)(p.B + (size_t)nb * p.ldb) + c * 16;
    }
  };
  cursor_tile(c_tile);
  // the loads of the cursor's step: 4 DMA pieces into `slot`, 4 A fragments into a[mb][h] (the
  // two halves of a row's line back to back); advance() moves the cursor on afterwards
  auto issue_dma = [&](int slot, int i) __attribute__((always_inline)) {
    char* dst = smem + slot * SN_SLOT + (wid_u * 4 + i) * 1024;
    __builtin_amdgcn_global_load_lds((const void*)(bptr[i] + c_k * 128), (lds_ptr_t)dst, 16, 0, 0);
  };
  auto issue_a = [&](bf16x8 (&a)[2][2], int mb) __attribute__((always_inline)) {
    sn_gload<0>(a[mb][0], aptr[mb] + c_k * 128);
    sn_gload<64>(a[mb][1], aptr[mb] + c_k * 128);
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (c_left > 0) {                                // past the end: re-issue the last step
      --c_left;
      if (++c_k == nk) { c_k = 0; c_tile += G; cursor_tile(c_tile); }
    }
  };
  auto issue = [&](int slot, bf16x8 (&a)[2][2]) __attribute__((always_inline)) {
    if (!(LAB && (p.dbg & 8))) {                     // LAB dbg 8: no B LDS-DMA pieces
#pragma unroll
      for (int i = 0; i < 4; ++i) issue_dma(slot, i);
    }
    if (!(LAB && (p.dbg & 16))) {                    // LAB dbg 16: no A loads
      issue_a(a, 0);
      issue_a(a, 1);
    }
    advance();
  };

  f32x4 acc[16][2];                                  // [n block of 16][m block of 16]
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ar[SN_P][2][2] = {};                        // A register ring [entry][m block][k half]

  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const int sx = (lr >> 1) & 7;                      // the row swizzle of this lane's fragment rows
  const uint32_t oB0 = (uint32_t)(lr * 128 + ((lq ^ sx) << 4));          // k half 0; + nb * 2048
  const uint32_t oB1 = (uint32_t)(lr * 128 + (((lq ^ sx) ^ 4) << 4));    // k half 1

  // ---- epilogue of tile t (the ring engine's: activation, pack, permlane16 widening, 16 stores)
  auto store_tile = [&](int t, auto FULL) __attribute__((always_inline)) {
    const int m0 = (t / ntn) * 256, n0 = (t % ntn) * 256;
    const int rows = min(256, p.M - m0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.C + (size_t)m0 * p.ldc), (short)0, rows * (int)p.ldc * 2, 0x00020000);
#pragma unroll
    for (int np = 0; np < 8; ++np) {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        uint32_t w[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float z = acc[2 * np + s][mb][r];
            const float a = EPI == SN_EPI_ACT ? act_fwd(ACT, z) : z;
            if constexpr (decltype(FULL)::value) {
              o[r] = a;
            } else {                                 // branch-free column masks
              const int n = n0 + (2 * np + s) * 16 + 4 * lq + r;
              if constexpr (EPI == SN_EPI_ACT) o[r] = n < p.n_valid ? a : ((n == p.n_valid && p.bias_col) ? 1.f : 0.f);
              else o[r] = n < p.NB ? a : 0.f;
            }
          }
          w[s][0] = pack_bf16x2(o[0], o[1]);
          w[s][1] = pack_bf16x2(o[2], o[3]);
        }
        // odd 16-lane rows of w[0] <-> even rows of w[1]: lane row q then holds columns
        // 16(q & 1) + 8(q >> 1) .. +7 of the n-block pair
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r2 = __builtin_amdgcn_permlane16_swap(w[0][d], w[1][d], false, false);
          w[0][d] = r2[0];
          w[1][d] = r2[1];
        }
        const int nl = np * 32 + 16 * (lq & 1) + 8 * (lq >> 1);
        const int ml = wid * 32 + mb * 16 + lr;
        const int off = n0 + nl < p.N ? (int)((ml * p.ldc + n0 + nl) * 2) : (int)0x7ffffff0;
        const v4i_t v = {(int)w[0][0], (int)w[0][1], (int)w[1][0], (int)w[1][1]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
      }
    }
  };
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int n0 = (t % ntn) * 256;
    if (LAB && (p.dbg & 1)) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" :: "v"(acc[i][j]));
    } else if (n0 + 256 <= (EPI == SN_EPI_ACT ? p.n_valid : p.NB)) {
      store_tile(t, std::integral_constant<bool, true>{});
    } else {
      store_tile(t, std::integral_constant<bool, false>{});
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

#define SN_BAR() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); \
                      __builtin_amdgcn_sched_barrier(0); } while (0)
  // Every vmcnt wait names EVERY A ring register ("+v"): an asm load's destination counts as
  // written at the asm statement, so a loaded value that no later statement reads (the last
  // re-issued steps past the end of the sequence) would be dead to hipcc and its registers handed
  // to other values while the data is still in flight -- the late write then corrupts them (seen as
  // rare wrong last tiles before this).  Named here, each ring entry stays live and in place from
  // its load to the wait that retires it.
#define SN_WAIT_A(N, E) asm volatile("s_waitcnt vmcnt(" #N ")" \
    : "+v"(ar[0][0][0]), "+v"(ar[0][0][1]), "+v"(ar[0][1][0]), "+v"(ar[0][1][1]), \
      "+v"(ar[1][0][0]), "+v"(ar[1][0][1]), "+v"(ar[1][1][0]), "+v"(ar[1][1][1]) :: "memory")
#define SN_KEEP_A() asm volatile("" \
    : "+v"(ar[0][0][0]), "+v"(ar[0][0][1]), "+v"(ar[0][1][0]), "+v"(ar[0][1][1]), \
      "+v"(ar[1][0][0]), "+v"(ar[1][0][1]), "+v"(ar[1][1][0]), "+v"(ar[1][1][1]) :: "memory")
  static_assert(SN_P == 2, "SN_WAIT_A names a 2-entry ring");

  // prologue: steps 0 .. D-1 in flight
  sn_for<SN_D>([&](auto I) { issue(I.v, ar[I.v]); });
  SN_WAIT_A(8, 0);
  SN_BAR();

  // B fragments of n blocks 2g, 2g+1 (both k halves) x the wave's A fragments: 8 MFMAs, k ascending
  auto mma = [&](const bf16x8 (&b)[4], int g, const bf16x8 (&a)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (LAB && (p.dbg & 4)) {
          asm volatile("" :: "v"(b[2 * j + h]), "v"(a[0][h]), "v"(a[1][h]));
        } else {
#pragma unroll
          for (int mb = 0; mb < 2; ++mb)
            acc[2 * g + j][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[2 * j + h], a[mb][h], acc[2 * g + j][mb], 0, 0, 0);
        }
      }
  };
  // group g: fragments (nb 2g, h 0), (2g, 1), (2g+1, 0), (2g+1, 1)
  auto read_group = [&](bf16x8 (&b)[4], uint32_t sb, auto G_) __attribute__((always_inline)) {
    constexpr int g = decltype(G_)::v;
    b[0] = sn_read<(2 * g) * 2048>(sb + oB0);
    b[1] = sn_read<(2 * g) * 2048>(sb + oB1);
    b[2] = sn_read<(2 * g + 1) * 2048>(sb + oB0);
    b[3] = sn_read<(2 * g + 1) * 2048>(sb + oB1);
  };
#define SN_WAIT_B(N, b) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) \
                                     :: "memory")
  int kk = 0, tile = lb, since_epi = 0, rslot = 0, dslot = SN_D;
  for (int t0 = 0; t0 < T; t0 += SN_P) {          // T is a multiple of 2 (K % 128 == 0)
    sn_for<SN_P>([&](auto E) {
      constexpr int e = E.v;
      const int t = t0 + e;
      const uint32_t sb = lds0 + (uint32_t)(rslot * SN_SLOT);
      bf16x8 b0[4], b1[4];
      {
        read_group(b0, sb, SnIC<0>{});
        read_group(b1, sb, SnIC<1>{});
        __builtin_amdgcn_s_setprio(1);
        sn_for<8>([&](auto Gi) {
          constexpr int g = Gi.v;
          if constexpr ((g & 1) == 0) {
            if constexpr (g < 7) SN_WAIT_B(4, b0); else SN_WAIT_B(0, b0);
            __builtin_amdgcn_sched_barrier(0);
            mma(b0, g, ar[e]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g + 2 < 8) read_group(b0, sb, SnIC<g + 2>{});
          } else {
            if constexpr (g < 7) SN_WAIT_B(4, b1); else SN_WAIT_B(0, b1);
            __builtin_amdgcn_sched_barrier(0);
            mma(b1, g, ar[e]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g + 2 < 8) read_group(b1, sb, SnIC<g + 2>{});
          }
        });
        __builtin_amdgcn_s_setprio(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      // the loads of step t+2: B pieces into slot (t+2) mod 4 (last read in step t-2), A into the
      // ring entry e this step's MFMAs have just read
      issue(dslot, ar[e]);
      __builtin_amdgcn_sched_barrier(0);
      rslot = rslot == SN_NSLOT - 1 ? 0 : rslot + 1;
      dslot = dslot == SN_NSLOT - 1 ? 0 : dslot + 1;
      __builtin_amdgcn_sched_barrier(0);
      if (++kk == nk) {
        kk = 0;
        epilogue(tile);
        tile += G;
        since_epi = SN_D;
        __builtin_amdgcn_sched_barrier(0);
      }
      // own group t+1 landed (A ring entry (e+1) mod P, B pieces of slot t+1); younger: group
      // t+2 (+16 epilogue stores in the D steps after a tile end).  The waits carry no operands;
      // the statement naming the ring registers sits after the join: "+v" operands on waits in
      // two arms made hipcc give each arm its own register assignment and copy the in-flight ring
      // between them.  (A CFG audit of this reports the MFMAs after the join on the infeasible
      // path "since_epi > 0 without an epilogue"; tools/asm_vmcnt_audit.py --copies checks the rest.)
      if (since_epi > 0) {
        --since_epi;
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      }
      SN_KEEP_A();
      SN_BAR();
    });
  }
  SN_WAIT_A(0, 0);                                   // the trailing loads land before the exit
#undef SN_WAIT_B
#undef SN_WAIT_A
#undef SN_KEEP_A
#undef SN_BAR
}

}  // namespace

static int g_sn_dbg = -1;                    // LAB build switch: >= 0 runs strip_nt_kernel<.., LAB>
SHIFU_API int shifu_strip_nt_set_lab(int dbg) { g_sn_dbg = dbg; return 0; }

// C ABI: returns -1 when the shape is not one this engine takes (the caller falls back).
// epi 0 = activation (derivative computable from the output: no f'(z) side output), 2 = store z.
SHIFU_API int shifu_strip_nt(const void* A, long lda, const void* B, long ldb, int NB, void* C, long ldc, int M,
                             int N, int K, int epi, int act, int n_valid, int bias_col, int grid_cap,
                             hipStream_t stream) {
  if (K % 128 || K < 128 || lda % 8 || ldb % 8 || ldc % 8 || N % 8 || M <= 0 || N <= 0 || NB <= 0) return -1;
  if (epi != SN_EPI_ACT) return -1;                  // the store-z and tanh builds spill VGPRs: the A ring
  if (act == 1) return -1;                           // lives in asm-loaded registers, so those stay on the ring
  if (epi == SN_EPI_ACT && !act_deriv_from_output(act)) return -1;
  if (256l * ldc * 2 >= (1l << 31)) return -1;                                       // 32-bit store offsets
  if (lda < K || ldb < K || ldc < N) return -1;
  const long ntiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  if (ntiles >= (1l << 31)) return -1;
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int grid = (int)(ntiles < ncu ? ntiles : ncu);
  if (grid_cap > 0 && grid > grid_cap) grid = grid_cap;
  StripArgs p{(const bf16_t*)A, lda, (const bf16_t*)B, ldb, (bf16_t*)C, ldc, M, N, K, NB, n_valid, bias_col,
              (int)ntiles, g_sn_dbg};
  const dim3 g(grid);
  if (g_sn_dbg >= 0) {
    if (epi == SN_EPI_ACT && act == 0)
      hipLaunchKernelGGL((strip_nt_kernel<SN_EPI_ACT, 0, true>), g, dim3(SN_T), SN_LDS, stream, p);
    else return -1;
  } else {
#define SN_L(A_) hipLaunchKernelGGL((strip_nt_kernel<SN_EPI_ACT, A_, false>), g, dim3(SN_T), SN_LDS, stream, p)
    switch (act) {
      case 0: SN_L(0); break; case 2: SN_L(2); break; case 3: SN_L(3); break;
      case 4: SN_L(4); break; case 6: SN_L(6); break; case 9: SN_L(9); break; default: SN_L(7); break;
    }
#undef SN_L
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
