// Persistent row-strip fused network head + the dgrad of the layer below (gfx950 / CDNA4).
//
// One kernel per 2M-row chunk does what the 8-phase head kernel and the dgrad tile kernel did in
// two (profiles/r5/NOTES_r5.md: head 1.09 ms + dgrad 1.12 ms per chunk, 0.5 and 0.37 PFLOP/s):
//
//   Z2 = H1 W2^T                     H1 [M, K1] bf16 (the layer-below activations), W2 [NB, K1]
//   A2 = bf16(act(Z2)) (+ bias 1)    never leaves the chip
//   zo = A2 . Wo, a_o = out_act(zo), loss, output delta dl     (SubGradient.java:224-311)
//   D2 = bf16(dl * Wo * (f'(A2) + flat))     -> HBM (operand of the layer's wgrad)
//   gWo += A2^T dl, err += loss              (per-wave partials, summed in a fixed order)
//   DZ1 = bf16(bf16(D2 W2) * (f'(H1) + flat1))   -> HBM (the layer below's deltas)
//
// Layout (the row-strip engine of gemm_strip_nt.hip): a 512-thread block per CU walks 256-row
// tiles; wave w owns rows [32w, 32w + 32) of the tile and ALL 256 head columns, so the output dot
// product, the loss and the deltas are wave-local (no LDS reduction, no block barrier in the
// epilogue).  A tile is 2 x K1/64 "steps", each one 32-KiB B image through the 4-slot LDS-DMA ring
// and 64 MFMAs per wave:
//   * K1/64 forward steps: B = W2 rows [256 x 64 k], A = the wave's H1 fragments (global -> VGPR,
//     asm loads, 2 steps ahead in a 2-entry ring);
//   * K1/64 dgrad steps, 64 output columns each: B = W2^T rows [64 x 256 k], A = D2 -- kept in
//     registers: the head epilogue's bf16 pack + v_permlane16_swap leaves every lane with 8
//     consecutive D2 columns of one row, which IS an MFMA A fragment (k order inside a 32-block
//     permuted as 0,2,1,3 by lane quadrant; the B fragments are read with the same permutation).
//     The step's H1 values for the DACT multiply are loaded at its start and land during its MFMAs.
// D2 therefore never travels HBM -> chip again, and H1 is re-read once per tile (from MALL/HBM)
// instead of by a second kernel.
//
// Every load/store count between the vmcnt waits is a compile-time constant (the tile's steps are
// unrolled), so no wait depends on a runtime counter -- and no branch makes hipcc shuffle the
// in-flight registers (the lesson of gemm_strip_nt.hip; tools/asm_vmcnt_audit.py checks the ISA).
#include "common.h"
#include <type_traits>
#include <utility>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((ext_vector_type(4))) int v4i_t;

constexpr int SH_T = 512;
constexpr int SH_NSLOT = 4;
constexpr int SH_SLOT = 32768;                    // one step's B image
constexpr int SH_LDS = SH_NSLOT * SH_SLOT + 1024 + 8192 + 8192;   // + output weights, gWo / error partials

__device__ __forceinline__ int sh_xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <int OFF>
__device__ __forceinline__ bf16x8 sh_read(uint32_t a) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}
// Buffer resource in SGPRs for the asm loads (word3 = the raw-buffer format used throughout: rows
// past num_records read as 0, so a partial last tile needs no clamping)
__device__ __forceinline__ v4i_t sh_rsrc(const void* base, long bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  v4i_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)(uint32_t)bytes);    // caller keeps bytes < 2^32
  r[3] = 0x00020000;
  return r;
}
// "+v": the load's destination is tied to the ring entry's current register (in place)
template <int OFF>
__device__ __forceinline__ void sh_bload(bf16x8& v, uint32_t vo, v4i_t rs, int so) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4" : "+v"(v) : "v"(vo), "s"(rs), "s"(so), "n"(OFF)
               : "memory");
}
__device__ __forceinline__ void sh_gload_f(float& v, const float* p) {
  asm volatile("global_load_dword %0, %1, off" : "+v"(v) : "v"(p) : "memory");
}

// 4 output weights through LDS by asm (an ordinary LDS read makes hipcc wait for the LDS-DMA
// in flight first -- it cannot tell the regions apart); the caller waits lgkmcnt itself
template <int OFF>
__device__ __forceinline__ f32x4 sh_read_w(uint32_t a) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}

template <int I> struct ShIC { static constexpr int v = I; };
template <typename F, int... Is>
__device__ __forceinline__ void sh_for_impl(F&& f, std::integer_sequence<int, Is...>) { (f(ShIC<Is>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void sh_for(F&& f) { sh_for_impl(f, std::make_integer_sequence<int, N>{}); }

struct StripHeadArgs {
  const bf16_t* H; long ldh;     // [M, K1] layer-below activations: head GEMM input and DACT operand
  const bf16_t* W; long ldw;     // [NB, K1] head weights (bf16)
  const bf16_t* WT; long ldwt;   // [K1, 256] transposed head weights (dgrad B operand)
  bf16_t* D; long ldd;           // [M, 256] out: head-layer deltas
  bf16_t* DZ; long lddz;         // [M, K1] out: layer-below deltas
  const float* Wo;               // [KH] fp32 output weights (bias weight at nv)
  const float* Y;                // [M] targets
  const float* S;                // [M] significance (nullable -> 1)
  float* gw_slab;                // [grid * 8][KH] per-wave output-wgrad partials
  double* err_slab;              // [grid * 8][2] per-wave (error, weight) sums (err == nullptr)
  double* err;                   // non-null: per-wave sums added straight into err[2] (double atomics)
  int M, K1, NB, nv, nv1, KH, out_act, loss;
  float flat_out, flat_hid, flat1;
  int ntiles;
  float* dbg_rows;               // lab (nullable): per row {z_out, y, dl}
};

template <int ACT, int HACT, int NKF>
__global__ __launch_bounds__(SH_T, 2) void strip_head_kernel(StripHeadArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int S = 2 * NKF;                         // steps per tile: NKF forward + NKF dgrad
  static_assert(NKF >= 4 && (S % SH_NSLOT) == 0, "step slots are static: S % 4 == 0");
  const int G = gridDim.x;
  const int lb = sh_xcd_remap(blockIdx.x, G);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int lr = lane & 15, lq = lane >> 4;

  float* wo_s = (float*)(smem + SH_NSLOT * SH_SLOT);           // [256] output weights
  float* gw_s = wo_s + 256;                                    // [8 waves][256] output-wgrad partials
  double* er_s = (double*)(gw_s + 8 * 256);                    // [512 threads][2] error sums
  if (tid < 256) wo_s[tid] = tid < p.KH ? p.Wo[tid] : 0.f;
  for (int i = tid; i < 8 * 256; i += SH_T) gw_s[i] = 0.f;
  for (int i = tid; i < 2 * SH_T; i += SH_T) er_s[i] = 0.0;
  __syncthreads();

  // ---- addressing: per-lane 32-bit offsets (tile-invariant) + per-tile SGPR resources
  const long rowb = p.ldh * 2;                                 // H row pitch in bytes
  const int soD = __builtin_amdgcn_readfirstlane((int)(16 * p.ldd * 2));   // + m block 1 (stores)
  const int soZ = __builtin_amdgcn_readfirstlane((int)(16 * p.lddz * 2));
  // Lane-derived offsets are recomputed where they are used, from a laundered thread id: kept as
  // long-lived VGPRs (a dozen of them) they pushed the head epilogue over 256 and were spilled.
  struct Ids { int lane, lr, lq, w, coff; };
  auto ids = [&]() __attribute__((always_inline)) {
    int t = tid;
    asm volatile("" : "+v"(t));
    const int l = t & 63, q = l >> 4;
    return Ids{l, l & 15, q, t >> 6, 16 * (q & 1) + 8 * (q >> 1)};
  };
  // one resource per operand for the whole chunk (kernel constants: a handful of SGPRs, nothing
  // per tile to spill); the tile's row offset rides in voffset, which the range check covers
  // (rows past M read 0 / stores past M are dropped).  Chunks stay < 4 GiB per operand.
  const v4i_t rH = sh_rsrc(p.H, (long)p.M * rowb);
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.D, (short)0, (int)(uint32_t)((long)p.M * p.ldd * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rZ = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.DZ, (short)0, (int)(uint32_t)((long)p.M * p.lddz * 2), 0x00020000);
  // B DMA.  Forward step ss: W2 [256 rows x 64 k] image, 128-B rows, chunk c of row r at
  // c ^ ((r >> 1) & 7); wave w's piece i = rows 64i + 8w .. +7.  Dgrad step e: W2^T rows 64e ..
  // 64e + 63, 512-B rows, chunk c of row r at c ^ (r & 15); wave w's piece i = rows 16i + 2w, +1.
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0,
                                                                      (int)min((long)p.NB * p.ldw * 2, 0x7fffffffl), 0x00020000);
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc((void*)p.WT, (short)0,
                                                                      (int)min((long)p.K1 * p.ldwt * 2, 0x7fffffffl), 0x00020000);
  int soW = __builtin_amdgcn_readfirstlane((int)(64 * p.ldw * 2));   // per piece
  int soT = __builtin_amdgcn_readfirstlane((int)(16 * p.ldwt * 2));
  int soE = __builtin_amdgcn_readfirstlane((int)(64 * p.ldwt * 2));  // per dgrad step

  bf16x8 ar[2][2][2] = {};                           // A ring [entry][m block][k half]
  float yv = 0.f, sv = 0.f;                          // Y / S of row 32w + (lane & 31), one tile ahead

  // the loads of step ss (0 .. S-1) of the tile with resources rh / ry / rsg.  A buffer_load ... lds
  // adds its immediate offset to the LDS destination as well (M0 + inst_offset + lane * 16), so the
  // DMA's source offsets go in soffset; the asm VGPR loads use the immediate.
  auto issue = [&](auto SS_, int t) __attribute__((always_inline)) {
    constexpr int ss = decltype(SS_)::v;
    int wb = wid_u * 1024;                           // laundered per call (see the tile loop)
    asm volatile("" : "+s"(wb));
    char* dst = smem + (ss % SH_NSLOT) * SH_SLOT + wb;
    const Ids d = ids();
    if constexpr (ss < NKF) {
      int sw = soW;
      asm volatile("" : "+s"(sw));
      const int row = d.w * 8 + (d.lane >> 3);
      const uint32_t voW = (uint32_t)(row * (int)p.ldw * 2 + (((d.lane & 7) ^ ((row >> 1) & 7)) << 4));
      const uint32_t voA = (uint32_t)((t * 256 + d.w * 32 + d.lr) * rowb + d.lq * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)          // piece rows in voffset (range-checked), the k step in soffset
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_ptr_t)(dst + i * 8192), 16, voW + (uint32_t)(i * sw),
                                                 ss * 128, 0, 0);
      // row offsets in voffset: the range check (rows past M read 0) covers voffset + the
      // immediate, not soffset
      const uint32_t voA1 = voA + (uint32_t)(16 * rowb);
      sh_bload<ss * 128>(ar[ss % 2][0][0], voA, rH, 0);
      sh_bload<ss * 128 + 64>(ar[ss % 2][0][1], voA, rH, 0);
      sh_bload<ss * 128>(ar[ss % 2][1][0], voA1, rH, 0);
      sh_bload<ss * 128 + 64>(ar[ss % 2][1][1], voA1, rH, 0);
      if constexpr (ss == 0) {
        const int m = min(t * 256 + d.w * 32 + (d.lane & 31), p.M - 1);
        sh_gload_f(yv, p.Y + m);
        sh_gload_f(sv, (p.S ? p.S : p.Y) + m);
      }
    } else {
      constexpr int e = ss - NKF;
      int st = soT, se = soE;
      asm volatile("" : "+s"(st), "+s"(se));
      const int sbase = e * se;
      const int rt = d.w * 2 + (d.lane >> 5);
      const uint32_t voT = (uint32_t)(rt * (int)p.ldwt * 2 + (((d.lane & 31) ^ (rt & 15)) << 4));
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rT, (lds_ptr_t)(dst + i * 8192), 16, voT, sbase + i * st, 0, 0);
    }
  };
  // vm ops in group ss (DMA pieces + asm loads)
  constexpr auto gsize = [](int ss) constexpr { return ss < NKF ? (ss == 0 ? 10 : 8) : 4; };

#define SH_BAR() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); \
                      __builtin_amdgcn_sched_barrier(0); } while (0)
  // waits carry no operands; the statement after each names every asm-loaded register so hipcc
  // keeps them in place and orders their uses after the wait
#define SH_KEEP() asm volatile("" \
    : "+v"(ar[0][0][0]), "+v"(ar[0][0][1]), "+v"(ar[0][1][0]), "+v"(ar[0][1][1]), \
      "+v"(ar[1][0][0]), "+v"(ar[1][0][1]), "+v"(ar[1][1][0]), "+v"(ar[1][1][1]), "+v"(yv), "+v"(sv) :: "memory")
#define SH_VMWAIT(N) do { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); SH_KEEP(); } while (0)

  // forward B fragment offsets (as gemm_strip_nt.hip)
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  // prologue: groups 0, 1 of the first tile
  const int t_first = lb < p.ntiles ? lb : 0;
  issue(ShIC<0>{}, t_first);
  issue(ShIC<1>{}, t_first);
  SH_VMWAIT(8);
  SH_BAR();

  for (int tile = lb; tile < p.ntiles; tile += G) {
    // launder the address bases once per tile: hipcc would otherwise hoist every per-step /
    // per-piece derived offset (dozens of SGPRs and VGPRs) out of the tile loop and spill them
    asm volatile("" : "+s"(soW), "+s"(soT), "+s"(soE));
    const int m0 = tile * 256;
    const int tn = tile + G < p.ntiles ? tile + G : tile;     // past the end: valid re-loads
    const uint32_t toff = (uint32_t)m0 * (uint32_t)rowb;       // this tile's H rows (DACT loads)
    const float y_cur = yv, s_cur = p.S ? sv : 1.f;   // landed with group 0 (before this tile)

    f32x4 acc[16][2];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 d2f[8][2];                                // D2 as A fragments [k block][m block]

    sh_for<S>([&](auto SS_) {
      constexpr int s = decltype(SS_)::v;
      const uint32_t sb = lds0 + (uint32_t)((s % SH_NSLOT) * SH_SLOT);
      if constexpr (s < NKF) {
        // ---------------- forward step s: 8 groups of 4 B fragments (n blocks 2g, 2g+1)
        // this step's read bases, laundered (per-slot copies hoisted out of the loop cost VGPRs)
        uint32_t f0, f1;                               // forward B fragments (as gemm_strip_nt.hip)
        {
          const Ids d = ids();
          const int sx = (d.lr >> 1) & 7;
          f0 = sb + (uint32_t)(d.lr * 128 + ((d.lq ^ sx) << 4));
          f1 = sb + (uint32_t)(d.lr * 128 + (((d.lq ^ sx) ^ 4) << 4));
        }
        bf16x8 b0[4], b1[4];
        auto rg = [&](bf16x8 (&b)[4], auto G_) __attribute__((always_inline)) {
          constexpr int g = decltype(G_)::v;
          b[0] = sh_read<(2 * g) * 2048>(f0);
          b[1] = sh_read<(2 * g) * 2048>(f1);
          b[2] = sh_read<(2 * g + 1) * 2048>(f0);
          b[3] = sh_read<(2 * g + 1) * 2048>(f1);
        };
        rg(b0, ShIC<0>{});
        rg(b1, ShIC<1>{});
        __builtin_amdgcn_s_setprio(1);
        sh_for<8>([&](auto Gi) {
          constexpr int g = decltype(Gi)::v;
          bf16x8 (&b)[4] = (g & 1) ? b1 : b0;
          if constexpr (g < 7) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) :: "memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) :: "memory");
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int mb = 0; mb < 2; ++mb)
                acc[2 * g + j][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[2 * j + h], ar[s % 2][mb][h],
                                                                            acc[2 * g + j][mb], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (g + 2 < 8) rg(b, ShIC<g + 2>{});
        });
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (s + 2 < S) issue(ShIC<s + 2>{}, tile);
        else issue(ShIC<s + 2 - S>{}, tn);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (s == NKF - 1) {
          // ---------------- head epilogue (wave-local): A2, output, loss, D2, gWo partials
          // lane-relative limits, laundered per tile: hipcc would otherwise hoist the 64 column
          // compares of this epilogue (and their SGPR masks) out of the tile loop and spill
          const Ids d = ids();
          const int nvl = p.nv - 4 * d.lq;
          const uint32_t vd = (uint32_t)(((m0 + d.w * 32 + d.lr) * p.ldd + d.coff) * 2);
          uint32_t wa = lds0 + SH_NSLOT * SH_SLOT + d.lq * 16;   // output weights nb*16 + 4lq (+ nb*64 B)
          float zp[2] = {0.f, 0.f};
          uint32_t apk[16][2][2];                        // A2 (bf16-exact) packed: half the VGPRs of acc
          sh_for<4>([&](auto NB4) {
            constexpr int q4 = decltype(NB4)::v;
            f32x4 wq[4];
            wq[0] = sh_read_w<(4 * q4 + 0) * 64>(wa);
            wq[1] = sh_read_w<(4 * q4 + 1) * 64>(wa);
            wq[2] = sh_read_w<(4 * q4 + 2) * 64>(wa);
            wq[3] = sh_read_w<(4 * q4 + 3) * 64>(wa);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wq[0]), "+v"(wq[1]), "+v"(wq[2]), "+v"(wq[3]) :: "memory");
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int nb = 4 * q4 + u;
#pragma unroll
              for (int mb = 0; mb < 2; ++mb) {
                float av[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int n = nb * 16 + r;              // - 4 lq (vs nvl)
                  const float t = act_fwd(ACT, acc[nb][mb][r]);   // unconditional: selects, no branch
                  av[r] = n < nvl ? t : (n == nvl ? 1.f : 0.f);
                }
                apk[nb][mb][0] = pack_bf16x2(av[0], av[1]);
                apk[nb][mb][1] = pack_bf16x2(av[2], av[3]);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const uint32_t h = apk[nb][mb][r >> 1];
                  zp[mb] += bf2f((r & 1) ? (h >> 16) : (h & 0xffff)) * wq[u][r];
                }
              }
            }
            // pin this batch here: otherwise hipcc sinks half of it (the m block 1 rows) past the
            // loss code to its only use, with everything it needs kept alive across that code
#pragma unroll
            for (int u = 0; u < 4; ++u)
              asm volatile("" : "+v"(apk[4 * q4 + u][0][0]), "+v"(apk[4 * q4 + u][0][1]),
                           "+v"(apk[4 * q4 + u][1][0]), "+v"(apk[4 * q4 + u][1][1]));
            asm volatile("" : "+v"(zp[0]), "+v"(zp[1]));
            __builtin_amdgcn_sched_barrier(0);
          });
          float dl[2];
          double ec = 0.0, ew = 0.0;
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {
            float z = zp[mb];
            z += __shfl_xor(z, 16, 64);
            z += __shfl_xor(z, 32, 64);
            const int src = mb * 16 + lr;
            const float y = __shfl(y_cur, src, 64), sg = __shfl(s_cur, src, 64);
            const int m = m0 + wid * 32 + mb * 16 + lr;
            float dlt = 0.f;
            if (m < p.M) {
              const float a = act_fwd(p.out_act, z), e = y - a;
              const int lm = p.loss % 3;
              double e_c;
              if (lm == 1) {
                dlt = e * sg;
                const float ac = fminf(fmaxf(a, 1e-7f), 1.f - 1e-7f);
                e_c = p.loss >= 3 ? -(__logf(a + 1e-7f) * y + __logf(1.f - a + 1e-7f) * (1.f - y)) * sg
                                  : -(__logf(ac) * y + __logf(1.f - ac) * (1.f - y));
              } else if (lm == 2) {
                dlt = (y < a ? 1.f : -1.f) * (act_deriv_out(p.out_act, a) + p.flat_out) * sg;
                e_c = fabsf(e) * sg;
              } else {
                dlt = (act_deriv_pre(p.out_act, z) + p.flat_out) * e * sg;
                e_c = p.loss >= 3 ? (double)(e * e) * sg : (double)(e * sg) * (e * sg);
              }
              ec += e_c;
              ew += sg;
            }
            dl[mb] = dlt;
            if (p.dbg_rows && lq == 0 && m < p.M) {
              p.dbg_rows[(size_t)m * 3] = z;
              p.dbg_rows[(size_t)m * 3 + 1] = y;
              p.dbg_rows[(size_t)m * 3 + 2] = dlt;
            }
          }
          {                                              // per-lane running sums (asm: no DMA wait)
            const uint32_t ea = lds0 + (uint32_t)((char*)er_s - smem) + (uint32_t)(tid * 16);
            f32x4 ev;
            asm volatile("ds_read_b128 %0, %1" : "=v"(ev) : "v"(ea));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ev) :: "memory");
            double e2[2] = {__builtin_bit_cast(double, (f32x2_t){ev[0], ev[1]}),
                            __builtin_bit_cast(double, (f32x2_t){ev[2], ev[3]})};
            e2[0] += lq == 0 ? ec : 0.0;               // one copy of each row (the lq = 0 lanes)
            e2[1] += lq == 0 ? ew : 0.0;
            const f32x2_t lo = __builtin_bit_cast(f32x2_t, e2[0]), hi = __builtin_bit_cast(f32x2_t, e2[1]);
            ev = f32x4{lo[0], lo[1], hi[0], hi[1]};
            asm volatile("ds_write_b128 %0, %1" :: "v"(ea), "v"(ev) : "memory");
          }
          // D2 (bf16, 8-column runs after the swap) -> store + keep as A fragments; gWo partials
          // of this lane's 64 columns over its two rows
          float gp[64];
          int nvl2 = nvl;                                // fresh compares (not CSE'd with loop 1's)
          asm volatile("" : "+v"(nvl2), "+v"(wa));
          sh_for<8>([&](auto NP) {
            constexpr int np = decltype(NP)::v;
            f32x4 wq[2];
            wq[0] = sh_read_w<(2 * np) * 64>(wa);
            wq[1] = sh_read_w<(2 * np + 1) * 64>(wa);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wq[0]), "+v"(wq[1]) :: "memory");
            // fresh A2 words: without this hipcc keeps loop 1's unpacked floats (128 VGPRs) alive
            asm volatile("" : "+v"(apk[2 * np][0][0]), "+v"(apk[2 * np][0][1]), "+v"(apk[2 * np][1][0]),
                         "+v"(apk[2 * np][1][1]), "+v"(apk[2 * np + 1][0][0]), "+v"(apk[2 * np + 1][0][1]),
                         "+v"(apk[2 * np + 1][1][0]), "+v"(apk[2 * np + 1][1][1]));
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
              uint32_t w[2][2];
#pragma unroll
              for (int s2 = 0; s2 < 2; ++s2) {
                const int nb = 2 * np + s2;
                const f32x4 wv = wq[s2];
                float o[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int n = nb * 16 + r;              // - 4 lq (vs nvl)
                  const uint32_t h = apk[nb][mb][r >> 1];
                  const float a = bf2f((r & 1) ? (h >> 16) : (h & 0xffff));
                  const float t = dl[mb] * wv[r] * (act_deriv_out(ACT, a) + p.flat_hid);
                  o[r] = n < nvl2 ? t : 0.f;
                  if (mb == 0) gp[nb * 4 + r] = dl[0] * a;
                  else gp[nb * 4 + r] += dl[1] * a;
                }
                w[s2][0] = pack_bf16x2(o[0], o[1]);
                w[s2][1] = pack_bf16x2(o[2], o[3]);
              }
#pragma unroll
              for (int d = 0; d < 2; ++d) {
                const auto r2 = __builtin_amdgcn_permlane16_swap(w[0][d], w[1][d], false, false);
                w[0][d] = r2[0];
                w[1][d] = r2[1];
              }
              const v4i_t v = {(int)w[0][0], (int)w[0][1], (int)w[1][0], (int)w[1][1]};
              d2f[np][mb] = __builtin_bit_cast(bf16x8, v);
              __builtin_amdgcn_raw_buffer_store_b128(v, rD, vd + np * 64 + (mb ? soD : 0), 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
          });
          // reduce-scatter the 64 partials over the 16 lanes of this quadrant: lane lr keeps
          // columns 16 lr + 4 lq + (0..3)
          auto rs = [&](auto W_, int m) __attribute__((always_inline)) {
            constexpr int w = decltype(W_)::v;
            const bool up = (lr & m) != 0;
#pragma unroll
            for (int j = 0; j < w; ++j) {
              const float send = up ? gp[j] : gp[j + w];
              const float keep = up ? gp[j + w] : gp[j];
              gp[j] = keep + __shfl_xor(send, m, 64);
            }
          };
          rs(ShIC<32>{}, 8);
          rs(ShIC<16>{}, 4);
          rs(ShIC<8>{}, 2);
          rs(ShIC<4>{}, 1);
          {
            const uint32_t ga = lds0 + (uint32_t)((char*)gw_s - smem) + (uint32_t)((wid * 256 + lr * 16 + 4 * lq) * 4);
            f32x4 g4;
            asm volatile("ds_read_b128 %0, %1" : "=v"(g4) : "v"(ga));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(g4) :: "memory");
            g4[0] += gp[0]; g4[1] += gp[1]; g4[2] += gp[2]; g4[3] += gp[3];
            asm volatile("ds_write_b128 %0, %1" :: "v"(ga), "v"(g4) : "memory");
          }
          // own group NKF landed; younger: group NKF+1 and the 16 D2 stores
          SH_VMWAIT(gsize(NKF + 1) + 16);
        } else {
          SH_VMWAIT(gsize((s + 2) % S));
        }
        SH_BAR();
      } else {
        // ---------------- dgrad step e: DZ1 columns 64e .. 64e + 63 = D2 [32 x 256] x W2^T slice
        constexpr int e = s - NKF;
        bf16x8 hv[2][2];                             // H1 [pair][m block]: 8 columns of one row
        const Ids d = ids();
        const uint32_t voH = toff + (uint32_t)((d.w * 32 + d.lr) * (int)rowb + d.coff * 2);
        const uint32_t voH1 = voH + (uint32_t)(16 * rowb);
#pragma unroll
        for (int np2 = 0; np2 < 2; ++np2) {
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=v"(hv[np2][0])
                       : "v"(voH), "s"(rH), "n"((64 * e + 32 * np2) * 2) : "memory");
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=v"(hv[np2][1])
                       : "v"(voH1), "s"(rH), "n"((64 * e + 32 * np2) * 2) : "memory");
        }
        f32x4 ad[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) ad[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        // 8 groups (n block nb = g >> 1, k blocks 4 (g & 1) .. +3)
        // dgrad B fragment bases: row nb*16 + lr, chunk (4 kb + kp) ^ lr, kp = the lane quadrant's
        // permuted k octet; kb's low two bits meet lr's bits 2-3 -> one base per kb & 3, kb & 4
        // and the n block are immediates
        uint32_t d0, d1, d2, d3;
        {
          const int kp = 2 * (d.lq & 1) + (d.lq >> 1);
          const uint32_t bse = sb + (uint32_t)(d.lr * 512 + ((kp ^ (d.lr & 3)) << 4));
          const int u = d.lr >> 2;
          d0 = bse + (uint32_t)((0 ^ u) << 6);
          d1 = bse + (uint32_t)((1 ^ u) << 6);
          d2 = bse + (uint32_t)((2 ^ u) << 6);
          d3 = bse + (uint32_t)((3 ^ u) << 6);
        }
        bf16x8 b0[4], b1[4];
        auto rg = [&](bf16x8 (&b)[4], auto G_) __attribute__((always_inline)) {
          constexpr int g = decltype(G_)::v;
          constexpr int off = (g >> 1) * 8192 + ((g & 1) ? 256 : 0);
          b[0] = sh_read<off>(d0);
          b[1] = sh_read<off>(d1);
          b[2] = sh_read<off>(d2);
          b[3] = sh_read<off>(d3);
        };
        rg(b0, ShIC<0>{});
        rg(b1, ShIC<1>{});
        __builtin_amdgcn_s_setprio(1);
        sh_for<8>([&](auto Gi) {
          constexpr int g = decltype(Gi)::v;
          constexpr int nb = g >> 1;
          bf16x8 (&b)[4] = (g & 1) ? b1 : b0;
          if constexpr (g < 7) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) :: "memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) :: "memory");
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < 4; ++q)                // k block 4 (g & 1) + q, ascending
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
              ad[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[q], d2f[4 * (g & 1) + q][mb], ad[nb][mb], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (g + 2 < 8) rg(b, ShIC<g + 2>{});
        });
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        // everything in flight has landed: this step's H1 values (and group s+1, issued a step ago)
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(hv[0][0]), "+v"(hv[0][1]), "+v"(hv[1][0]), "+v"(hv[1][1]) :: "memory");
        SH_KEEP();
        const Ids d2i = ids();
        const int lim = p.nv1 - d2i.coff - 64 * e;
        const uint32_t vz = (uint32_t)(((m0 + d2i.w * 32 + d2i.lr) * p.lddz + d2i.coff) * 2);
#pragma unroll
        for (int np2 = 0; np2 < 2; ++np2) {
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {
            uint32_t w[2][2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              const f32x4 z = ad[2 * np2 + s2][mb];
              w[s2][0] = pack_bf16x2(z[0], z[1]);
              w[s2][1] = pack_bf16x2(z[2], z[3]);
            }
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              const auto r2 = __builtin_amdgcn_permlane16_swap(w[0][d], w[1][d], false, false);
              w[0][d] = r2[0];
              w[1][d] = r2[1];
            }
            const uint32_t zz[4] = {w[0][0], w[0][1], w[1][0], w[1][1]};
            const v4i_t hh = __builtin_bit_cast(v4i_t, hv[np2][mb]);
            const int n0 = 32 * np2;                     // - coff - 64 e (vs lim)
            uint32_t out[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const uint32_t hq = (uint32_t)hh[q];
              float a0 = bf2f(zz[q] & 0xffff), a1 = bf2f(zz[q] >> 16);
              const float d0 = act_deriv_out(HACT, bf2f(hq & 0xffff)) + p.flat1;
              const float d1 = act_deriv_out(HACT, bf2f(hq >> 16)) + p.flat1;
              a0 = (n0 + 2 * q < lim) ? a0 * d0 : 0.f;
              a1 = (n0 + 2 * q + 1 < lim) ? a1 * d1 : 0.f;
              out[q] = pack_bf16x2(a0, a1);
            }
            const v4i_t v = {(int)out[0], (int)out[1], (int)out[2], (int)out[3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, rZ, vz + (64 * e + 32 * np2) * 2 + (mb ? soZ : 0), 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (s + 2 < S) issue(ShIC<s + 2>{}, tile);
        else issue(ShIC<s + 2 - S>{}, tn);
        __builtin_amdgcn_sched_barrier(0);
        SH_KEEP();
        // group s+1 landed at the vmcnt(0) above
        SH_BAR();
      }
    });
  }
  SH_VMWAIT(0);                                      // the trailing re-loads land before the exit

  // ---- per-wave partials (fixed-order sums afterwards); blocks without tiles write zeros
  __syncthreads();
  const int srow = lb * 8 + wid;
  if (tid < 8 * 64) {
    const int c0 = lane * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (c0 + r < p.KH) p.gw_slab[(size_t)srow * p.KH + c0 + r] = gw_s[wid * 256 + c0 + r];
  }
  if (lane < 2) {
    double a = 0.0;
    for (int l = 0; l < 64; ++l) a += er_s[(wid * 64 + l) * 2 + lane];
    if (p.err) atomicAdd(p.err + lane, a);
    else p.err_slab[srow * 2 + lane] = a;
  }
#undef SH_VMWAIT
#undef SH_KEEP
#undef SH_BAR
}

__global__ __launch_bounds__(256) void sh_err_kernel(const double* slab, int T, double* err) {
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
  if (threadIdx.x == 0) {              // two chunk lanes add into the same err: atomic
    atomicAdd(err, sh[0][0]);
    atomicAdd(err + 1, sh[1][0]);
  }
}

int sh_grid(int M) {
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int ntiles = (M + 255) / 256;
  return ntiles < ncu ? ntiles : ncu;
}

}  // namespace

static float* g_sh_dbg_rows = nullptr;
SHIFU_API int shifu_strip_head_set_dbg_rows(float* p) { g_sh_dbg_rows = p; return 0; }

// Rows of the per-wave slabs shifu_strip_head writes for an M-row chunk (gw_slab [rows][KH],
// err_slab [rows][2]): the caller sums gw_slab with shifu_colsum_fixed.
SHIFU_API int shifu_strip_head_rows(int M) { return M > 0 ? sh_grid(M) * 8 : 0; }

// Fused head + layer-below dgrad (see above).  Returns -1 for shapes it does not take (the caller
// keeps the head + dgrad kernels): K1 = 512, head width padded to 256 (ldd = ldwt = 256),
// ACT == HACT (one instantiation per activation), both derivable from the output, not ptanh.
SHIFU_API int shifu_strip_head(const void* H, long ldh, const void* W, long ldw, int NB, const void* WT, long ldwt,
                               void* D, long ldd, void* DZ, long lddz, int M, int K1, int nv, int nv1,
                               const float* Wo, int KH, const float* Y, const float* S, float* gw_slab,
                               double* err_slab, double* err, int act, int hact, int out_act, int loss,
                               float flat_out, float flat_hid, float flat1, hipStream_t stream) {
  // K1 = 256 (4 + 4 steps per tile) is not taken: that build computed wrong, run-to-run different
  // head deltas for every block's second tile even with every wait made vmcnt(0) (a register-level
  // fault the ISA audit does not see; profiles/r6/NOTES_r6.md) -- its shapes keep the two kernels
  if (M <= 0 || K1 != 512 || ldh < K1 || ldh % 8 || ldw < K1 || ldw % 8 || ldd != 256 ||
      ldwt != 256 || lddz < K1 || lddz % 8 || NB <= 0 || NB > 256 || nv > 255 || nv < 0 || KH > 256 ||
      KH < nv + 1 || nv1 > K1)
    return -1;
  if (act != hact || !act_deriv_from_output(act) || act == ACT_PTANH || out_act < 0 || out_act > 9) return -1;
  // 32-bit buffer offsets over the whole chunk (row offsets ride in voffset)
  if ((long)M * ldh * 2 >= (1l << 32) || (long)M * lddz * 2 >= (1l << 32) || (long)M * ldd * 2 >= (1l << 32))
    return -1;
  const int grid = sh_grid(M);
  StripHeadArgs p{(const bf16_t*)H, ldh, (const bf16_t*)W, ldw, (const bf16_t*)WT, ldwt, (bf16_t*)D, ldd,
                  (bf16_t*)DZ, lddz, Wo, Y, S, gw_slab, err_slab, nullptr, M, K1, NB, nv, nv1, KH, out_act,
                  loss, flat_out, flat_hid, flat1, (M + 255) / 256, g_sh_dbg_rows};
  // the error sums: each wave's (error, weight) pair added into err by double atomics in the
  // kernel's tail (the two chunk lanes add into the same err already: order-free up to rounding).
  // A one-block reduction kernel after it sat on its lane's critical path for up to 1.5 ms per
  // chunk, waiting for a CU slot behind the other lane's persistent kernel (r6 MLP kernel trace).
  // SHIFU_SH_ERR_SLAB=1: per-wave slabs + the reduction kernel (lab A/B)
  static const bool err_slab_path = [] { const char* e = getenv("SHIFU_SH_ERR_SLAB"); return e && atoi(e) == 1; }();
  if (!err_slab_path) p.err = err;
#define SH_L(A_, N_) hipLaunchKernelGGL((strip_head_kernel<A_, A_, N_>), dim3(grid), dim3(SH_T), SH_LDS, stream, p)
#define SH_ACTS(N_) switch (act) { case 0: SH_L(0, N_); break; case 1: SH_L(1, N_); break; \
    case 2: SH_L(2, N_); break; case 3: SH_L(3, N_); break; case 4: SH_L(4, N_); break; \
    case 7: SH_L(7, N_); break; case 9: SH_L(9, N_); break; default: return -1; }
#ifdef SH_ONE                                        // lab builds: one instantiation
  if (act != 0) return -1;
  SH_L(0, 8);
#else
  SH_ACTS(8)
#endif
#undef SH_ACTS
#undef SH_L
  if (err_slab_path) hipLaunchKernelGGL(sh_err_kernel, dim3(1), dim3(256), 0, stream, err_slab, grid * 8, err);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
