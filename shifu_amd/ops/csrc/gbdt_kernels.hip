// Tree-ensemble (GBT / RF) kernels for MI355X (gfx950).
//
// Replaces the reference's DTWorker/DTMaster hot loops:
//   histogram   DTWorker.doCompute stats loop          J/core/dtrain/dt/DTWorker.java:789-863
//               Impurity.featureUpdate                 J/core/dtrain/dt/Impurity.java:238-242, 537-540
//   split find  Impurity.computeImpurity (Variance / FriedmanMSE / Entropy / Gini)
//                                                      J/core/dtrain/dt/Impurity.java:120-211, 269, 378, 563
//   routing     DTWorker.predictNodeIndex              J/core/dtrain/dt/DTWorker.java:1036-1096
//   GBT update  DTWorker.doCompute predict/output      J/core/dtrain/dt/DTWorker.java:620-670, Loss.java
//
// MI355X design:
//   * bins are uint8, quad-blocked [Q][N][128]: 128 features of a row form one 128-B record (one
//     L2 line), Q = Fp / 128; a histogram work item covers a 32-feature group = one 32-B quarter
//     of the record.  Rows are grouped per node through a position->row permutation that is
//     stably re-partitioned every level (rows of one node are a contiguous position range, so
//     a histogram pass reads only that node's rows).  Below the root those rows are a sparse,
//     ascending subset: each record read pulls its whole 128-B line, so the four groups of a
//     quad are consecutive work items placed on ONE XCD (xcd_remap) and consume every line from
//     that XCD's L2 -- the line-granularity gather that a [G][N][32] layout (a private 32-B slice
//     per line and group) wastes 3/4 of (profiles/r3, per-level table).
//   * histograms keep only (sum w, sum w*g) per bin: for variance / friedman-mse / binary
//     entropy / binary gini the best split depends on count and sum only (the sum-of-squares
//     terms cancel in the variance gain).  Both sums are int64 fixed point, packed into ONE
//     LDS atomic per (row, feature) (see gbdt_hist_kernel).
//   * a work item = (node, row range, 32-feature group); a block builds its item's histogram
//     in LDS and writes it to a per-item slab with coalesced stores (no global atomics); the
//     split kernel sums the slabs, derives the larger sibling by parent - smaller (histogram
//     subtraction) and scans the bins.
//   * deterministic: slab order is fixed and ties break to the lowest feature, then bin, so
//     every rank computes the identical split from the all-reduced histograms.
#include "common.h"
#include <cstdlib>
#include <type_traits>
typedef __attribute__((ext_vector_type(4))) int v4i_t;

namespace {

constexpr int NB = 256;        // max bins per feature (uint8 codes)
constexpr int FG = 32;         // features per work-item group
constexpr int QF = 128;        // features per row record (one 128-B line); 4 groups per record

// XCD-aware bijective block remap: consecutive logical ids land on the same XCD (blocks b, b+8,
// ... share an XCD under round-robin dispatch; speed only)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// byte offset of feature f of data row `row` in the quad-blocked layout (qs = N * 128)
__device__ __forceinline__ size_t bin_off(long qs, long row, int f) {
  return (size_t)(f >> 7) * qs + (size_t)row * QF + (f & (QF - 1));
}

struct HistArgs {
  const uint8_t* bins; long gs;      // quad-blocked bins [Q][N][128]: gs = N * 128 bytes per quad
  const int* pos2row;                // [N] position -> row id (nullptr: identity, the root level)
  const float* w;                    // [N] per-row weight (significance x subsample)
  const float* g;                    // [N] per-row target (label / pseudo residual)
  int wg_by_pos;                     // 1: w / g are position-ordered (permuted with pos2row): contiguous reads
  int rec;                           // row record bytes: 128 (quad-blocked) or 32 (group-blocked [G][N][32]
                                     // copy the dense root pass streams; gs = N * rec)
  const int* items;                  // [n_items][4] = {node, pos_lo, pos_hi, group}
  long long* slab;                   // [n_items][2][FG][NB] int64 fixed point
  int n_items, n_feat;
  float scale_w, scale_g;            // powers of two: w*scale_w < 2^16, |w*g*scale_g| < 2^23
  long nmod;                         // > 0: forest batch, pos2row holds tree * N + row -> bins row = v % N
};

// Histogram build (measured on gfx950 with tools/microbench_hist.hip, 16M rows x 1024 features):
//   * bins are stored group-blocked [G][N][32] so a block streams its group's 32-B row records
//     contiguously (row-major [N][1024] made every 32-B slice fetch its own 128-B line:
//     1.4 TB/s -> 4.1 TB/s);
//   * one packed ds_add_u64 per (row, feature): (qw << 36) + qg with qg signed.  Over <= 4096
//     rows a bin's sums stay inside their fields (qw < 2^16 -> 28 bits, |qg| < 2^23 -> 36 bits
//     signed), so the block unpacks the LDS histogram into int64 registers every 4096 rows.
//     Exact: identical sums to two separate int64 atomics;
//   * LDS layout [half][bin][16 features] + a per-lane rotation of the 16 feature bytes: lane
//     r of a 16-lane LDS group updates feature (j + r) & 15 at step j, so the group's 16 lanes
//     always hit 16 distinct bank pairs whatever the bins are.
constexpr int HT = 512;                       // threads per histogram block (8 waves)
constexpr int RPP = HT / 2;                   // rows per slot pass (2 threads x 16 B per row)
constexpr int HNE = 2 * NB * 16 / HT;         // LDS entries each thread unpacks (16)
constexpr int PACK_G = 36;                    // low field bits (signed qg)

__device__ __forceinline__ uint32_t pick(uint32_t a, uint32_t b, bool c) { return c ? b : a; }

__device__ __forceinline__ void unpack_add(unsigned long long v, long long& aw, long long& ag) {
  const long long gq = ((long long)(v << (64 - PACK_G))) >> (64 - PACK_G);
  ag += gq;
  aw += (long long)((v - (unsigned long long)gq) >> PACK_G);
}

// Root-level u32 modes (MODE 1 = sum w only, MODE 2 = sum w*g only): LDS u32 atomics move half
// the bytes of the packed u64 and run at ~2x its rate (profiles/microbench_lds_atomics.txt).  The
// root's sum-w histogram does not change between boosting rounds while the row weights do not,
// so the trainer builds it once (MODE 1) and re-builds only sum w*g (MODE 2) every round.  MODE 2
// quantises w*g at scale_g / 2^GSH32 (|q| < 2^20; 2048 rows between unpacks keep a bin's sum
// inside int32) and unpacks it shifted back to the scale_g grid, so the slab has the same units
// as the packed kernel's and the histogram subtraction below the root stays exact.
constexpr int GSH32 = 3;

template <bool PF, int HU, int MODE>
__global__ __launch_bounds__(HT) void gbdt_hist_kernel(HistArgs a) {
  // passes between unpacks: 4096 rows; in the u32 modes each of the two LDS copies sees exactly
  // half of them (2048), which keeps a bin's int32 sum in range
  constexpr int HFLUSH = 4096 / (RPP * HU);
  extern __shared__ __attribute__((aligned(16))) unsigned long long hsm[];   // [2][NB][16]
  uint32_t* hsm32 = (uint32_t*)hsm;
  const int item = xcd_remap(blockIdx.x, gridDim.x);     // a quad's 4 group items share an XCD
  const int lo = a.items[item * 4 + 1], hi = a.items[item * 4 + 2], grp = a.items[item * 4 + 3];
  if (lo >= hi) {        // an item past its node's rows (ranges resolved on the device): zero slab
    long long* out = a.slab + (size_t)item * 2 * FG * NB;
    for (int i = threadIdx.x; i < 2 * FG * NB; i += HT)
      if (!((MODE == 1 && i >= FG * NB) || (MODE == 2 && i < FG * NB))) out[i] = 0;
    return;
  }
  for (int i = threadIdx.x; i < 2 * NB * 16; i += HT) hsm[i] = 0ull;
  __syncthreads();
  const int half = threadIdx.x & 1, r = threadIdx.x & 15, t2 = threadIdx.x >> 1;
  const int gpr = a.rec / FG;                                   // groups per record (4 or 1)
  const uint8_t* gb = a.bins + (size_t)(grp / gpr) * a.gs + (grp % gpr) * FG + half * 16;
  unsigned long long* base = hsm + half * NB * 16;
  // u32 modes: two interleaved copies [half][bin][copy][16] (lane group parity picks the copy):
  // the 4 lanes that update the same feature then spread over 4 banks unless their bins agree
  // mod 2 (one 16-feature row per bin put them in 4 banks only when the bins differ mod 4)
  uint32_t* base32 = hsm32 + half * NB * 32 + (((threadIdx.x >> 4) & 1) << 4);
  // w / g are indexed by the (virtual) row id -- or by position when wg_by_pos -- the bins by
  // the data row
  auto rec = [&](int v) { return *(const uint4*)(gb + (size_t)(a.nmod ? (long)v % a.nmod : (long)v) * a.rec); };
  long long accw[HNE], accg[HNE];
#pragma unroll
  for (int k = 0; k < HNE; ++k) { accw[k] = 0; accg[k] = 0; }
  // one row slot: packed (w, w*g) fixed point added to the 16 features' bins of this half record
  auto update = [&](float wv, float gv, const uint4& bv) {
    if (wv == 0.f) return;
    unsigned long long q = 0;
    uint32_t q32 = 0;
    if constexpr (MODE == 0)
      q = ((unsigned long long)__float2uint_rn(wv * a.scale_w) << PACK_G) +
          (unsigned long long)(long long)__float2int_rn(wv * gv * a.scale_g);
    else if constexpr (MODE == 1)
      q32 = __float2uint_rn(wv * a.scale_w);
    else
      q32 = (uint32_t)__float2int_rn(wv * gv * a.scale_g);    // scale_g already / 2^GSH32
    // rotate the 16 bytes left by r: byte j of R = feature (j + r) & 15
    const uint32_t W[4] = {bv.x, bv.y, bv.z, bv.w};
    uint32_t X[4], Y[4], R[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) X[k] = pick(W[k], W[(k + 1) & 3], r & 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) Y[k] = pick(X[k], X[(k + 2) & 3], r & 8);
#pragma unroll
    for (int k = 0; k < 4; ++k) R[k] = __builtin_amdgcn_alignbyte(Y[(k + 1) & 3], Y[k], r & 3);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t b = (R[j >> 2] >> ((j & 3) * 8)) & 0xff;
      if constexpr (MODE == 0) atomicAdd(&base[(b << 4) | ((j + r) & 15)], q);
      else atomicAdd(&base32[(b << 5) | ((j + r) & 15)], q32);
    }
  };
  auto unpack32 = [&](uint32_t v, long long& aw, long long& ag) {
    if constexpr (MODE == 1) aw += (long long)v;
    else ag += (long long)(int32_t)v * (1ll << GSH32);
  };
  auto flush = [&](int& it) {
    if (++it == HFLUSH) {
      it = 0;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < HNE; ++k) {
        const int e = threadIdx.x + k * HT;
        if constexpr (MODE == 0) { unpack_add(hsm[e], accw[k], accg[k]); hsm[e] = 0ull; }
        else {
          const int i0 = ((e >> 12) * NB + ((e >> 4) & (NB - 1))) * 32 + (e & 15);
          unpack32(hsm32[i0], accw[k], accg[k]);
          unpack32(hsm32[i0 + 16], accw[k], accg[k]);
          hsm32[i0] = 0u;
          hsm32[i0 + 16] = 0u;
        }
      }
      __syncthreads();
    }
  };
  int it = 0;
  constexpr int STEP = RPP * HU;
  if constexpr (PF) {
    // Software pipeline over two static slots (as gbdt_hist64_kernel): slot k's (bins, w, g) are
    // added, then the slot is refilled with the pass two ahead whose row ids were gathered two
    // passes earlier.  Positions past `hi` are clamped to hi - 1 (valid memory, no branch around
    // a load) and get weight 0 when consumed.
    constexpr int SL = 2;
    auto row_of = [&](int p) { const int pc = min(p, hi - 1); return a.pos2row ? a.pos2row[pc] : pc; };
    auto wg_at = [&](int p, int rr) { return a.wg_by_pos ? min(p, hi - 1) : rr; };
    int rn[SL][HU];
    float wc[SL][HU], gc[SL][HU];
    uint4 bc[SL][HU];
#pragma unroll
    for (int k = 0; k < SL; ++k)
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int p = lo + k * STEP + t2 + u * RPP, rr = row_of(p), kk = wg_at(p, rr);
        wc[k][u] = a.w[kk]; gc[k][u] = a.g[kk]; bc[k][u] = rec(rr);
      }
#pragma unroll
    for (int k = 0; k < SL; ++k)
#pragma unroll
      for (int u = 0; u < HU; ++u) rn[k][u] = row_of(lo + (SL + k) * STEP + t2 + u * RPP);
    for (int p0 = lo; p0 < hi; p0 += SL * STEP) {     // block-uniform trip count (unpack barriers)
#pragma unroll
      for (int k = 0; k < SL; ++k) {
        const int pk = p0 + k * STEP;
#pragma unroll
        for (int u = 0; u < HU; ++u) update(pk + t2 + u * RPP < hi ? wc[k][u] : 0.f, gc[k][u], bc[k][u]);
        flush(it);
#pragma unroll
        for (int u = 0; u < HU; ++u) {
          const int kk = wg_at(pk + SL * STEP + t2 + u * RPP, rn[k][u]);
          wc[k][u] = a.w[kk]; gc[k][u] = a.g[kk]; bc[k][u] = rec(rn[k][u]);
          rn[k][u] = row_of(pk + 2 * SL * STEP + t2 + u * RPP);
        }
      }
    }
  } else {
    for (int p0 = lo; p0 < hi; p0 += STEP) {          // block-uniform trip count (unpack barriers)
      int rows[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int p = p0 + t2 + u * RPP;
        rows[u] = p < hi ? (a.pos2row ? a.pos2row[p] : p) : -1;
      }
      float wv[HU], gv[HU];
      uint4 bv[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int rr = rows[u], k = a.wg_by_pos ? p0 + t2 + u * RPP : rr;
        wv[u] = rr >= 0 ? a.w[k] : 0.f;
        gv[u] = rr >= 0 ? a.g[k] : 0.f;
        bv[u] = rr >= 0 ? rec(rr) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < HU; ++u) update(wv[u], gv[u], bv[u]);
      flush(it);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < HNE; ++k) {
    if constexpr (MODE == 0) unpack_add(hsm[threadIdx.x + k * HT], accw[k], accg[k]);
    else {
      const int e = threadIdx.x + k * HT, i0 = ((e >> 12) * NB + ((e >> 4) & (NB - 1))) * 32 + (e & 15);
      unpack32(hsm32[i0], accw[k], accg[k]);
      unpack32(hsm32[i0 + 16], accw[k], accg[k]);
    }
  }
  // transpose through LDS ([f][b] per statistic) for coalesced slab stores
  long long* out = a.slab + (size_t)item * 2 * FG * NB;
  long long* tsm = (long long*)hsm;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    if ((MODE == 1 && st == 1) || (MODE == 2 && st == 0)) continue;   // u32 modes own one half
    __syncthreads();
#pragma unroll
    for (int k = 0; k < HNE; ++k) {
      const int e = threadIdx.x + k * HT;
      const int f = (e >> 12) * 16 + (e & 15), b = (e >> 4) & (NB - 1);
      tsm[f * NB + b] = st ? accg[k] : accw[k];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < FG * NB; i += HT) out[st * FG * NB + i] = tsm[i];
  }
}

// ---------------------------------------------------------------------------------------
// Below-root histogram over HALF records: one 1024-thread block builds the packed u64
// histograms of 64 features (two 32-feature group items of one node and row range) for its
// rows, 4 threads per row each reading 16 B of the row's 64-B half line.  The per-group kernel
// above has 4 blocks read 32 B each of every 128-B line: its ablations put the non-root levels on
// that gather (14.4 of 15.7 ms per level with the LDS atomics removed, profiles/r5/gbdt), and
// every 32-B piece is its own L2 request.  Here a row's 64 B leave L2 as one request.
// LDS [4 quarters][NB][16] u64 = 128 KiB (one block per CU, 16 waves); the same per-lane byte
// rotation keeps each 16-lane group on 16 distinct bank pairs; 4096 rows between unpacks.
// ---------------------------------------------------------------------------------------
constexpr int H6_T = 1024;
constexpr int H6_RPP = H6_T / 4;                 // rows per pass
constexpr int H6_NE = 4 * NB * 16 / H6_T;        // entries each thread unpacks (16)

// PD: passes of (bins, w, g) in flight ahead of the one being added (row ids PD passes further):
// with one block of 16 waves per CU a single pass ahead keeps ~4 MB of gathers in flight over the
// chip, short of what HBM latency x bandwidth asks for
//
// PERM: LDS laid out [quarter pair][NB][2][16] instead of [quarter][NB][16], so a bin's row is 256
// bytes and each atomic's byte address {lane/step constant, bin, quarter pair, 0} is ONE v_perm_b32
// of the rotated record word and a per-(lane, step) constant (the [4][NB][16] layout needed a byte
// extract + shift-add per atomic).  Banks: a 16-lane group still hits 16 distinct bank pairs
// ((qt & 1) * 32 + 2 f for its 16 features, any bins).
template <int PD, bool PERM>
__global__ __launch_bounds__(H6_T) void gbdt_hist64_kernel(HistArgs a, const int* pairs) {
  constexpr int HFLUSH = 4096 / H6_RPP;
  extern __shared__ __attribute__((aligned(16))) unsigned long long h6[];    // [4][NB][16] (see PERM)
  const int pr = xcd_remap(blockIdx.x, gridDim.x);
  // items of groups 2j (ia) and 2j + 1 (ib) of one node and row range; either may be -1
  const int ia = pairs[pr * 2], ib = pairs[pr * 2 + 1], i0 = ia >= 0 ? ia : ib;
  const int lo = a.items[i0 * 4 + 1], hi = a.items[i0 * 4 + 2], grp = a.items[i0 * 4 + 3] & ~1;
  if (lo >= hi) {        // empty row range (device-resolved items): zero slabs
    for (int i = threadIdx.x; i < 2 * 2 * FG * NB; i += H6_T) {
      const int itm = (i / (2 * FG * NB)) ? ib : ia;
      if (itm >= 0) a.slab[(size_t)itm * 2 * FG * NB + (i % (2 * FG * NB))] = 0;
    }
    return;
  }
  for (int i = threadIdx.x; i < 4 * NB * 16; i += H6_T) h6[i] = 0ull;
  __syncthreads();
  const int qt = threadIdx.x & 3, r = threadIdx.x & 15, t4 = threadIdx.x >> 2;
  // grp is even: its 64-B half of the quad record starts at byte (grp & 3) * 32 (0 or 64)
  const uint8_t* gb = a.bins + (size_t)(grp >> 2) * a.gs + (grp & 3) * FG + qt * 16;
  unsigned long long* base = h6 + qt * NB * 16;
  const uint32_t cq = ((uint32_t)(qt >> 1) << 16) | ((uint32_t)(qt & 1) << 7);   // PERM layout
  auto rec = [&](int v) { return *(const uint4*)(gb + (size_t)(a.nmod ? (long)v % a.nmod : (long)v) * QF); };
  long long accw[H6_NE], accg[H6_NE];
#pragma unroll
  for (int k = 0; k < H6_NE; ++k) { accw[k] = 0; accg[k] = 0; }
  auto update = [&](float wv, float gv, const uint4& bv) {
    if (wv == 0.f) return;
    const unsigned long long q = ((unsigned long long)__float2uint_rn(wv * a.scale_w) << PACK_G) +
                                 (unsigned long long)(long long)__float2int_rn(wv * gv * a.scale_g);
    const uint32_t W[4] = {bv.x, bv.y, bv.z, bv.w};
    uint32_t X[4], Y[4], R[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) X[k] = pick(W[k], W[(k + 1) & 3], r & 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) Y[k] = pick(X[k], X[(k + 2) & 3], r & 8);
#pragma unroll
    for (int k = 0; k < 4; ++k) R[k] = __builtin_amdgcn_alignbyte(Y[(k + 1) & 3], Y[k], r & 3);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (PERM) {
        // {cq byte 0 + 8 f, bin, quarter pair, 0}: selector bytes 0 / 2 from src1, 4 + (j & 3) = the bin
        const uint32_t cj = cq | ((((uint32_t)(j + r)) & 15u) << 3);
        const uint32_t addr = __builtin_amdgcn_perm(R[j >> 2], cj, 0x0c020000u | ((4u + (j & 3)) << 8));
        asm volatile("ds_add_u64 %0, %1" : : "v"(addr), "v"(q) : "memory");
      } else {
        const uint32_t b = (R[j >> 2] >> ((j & 3) * 8)) & 0xff;
        atomicAdd(&base[(b << 4) | ((j + r) & 15)], q);
      }
    }
  };
  auto flush = [&](int& it) {
    if (++it == HFLUSH) {
      it = 0;
      if constexpr (PERM) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the asm atomics
      __syncthreads();
#pragma unroll
      for (int k = 0; k < H6_NE; ++k) {
        const int e = threadIdx.x + k * H6_T;
        unpack_add(h6[e], accw[k], accg[k]);
        h6[e] = 0ull;
      }
      __syncthreads();
    }
  };
  // software pipeline as gbdt_hist_kernel<PF>: next pass's (bins, w, g) and the pos2row gather
  // two passes ahead in flight while a pass's atomics run
  auto row_of = [&](int p) { const int pc = min(p, hi - 1); return a.pos2row ? a.pos2row[pc] : pc; };
  auto wg_at = [&](int p, int rr) { return a.wg_by_pos ? min(p, hi - 1) : rr; };
  int it = 0;
  // PD static slots: slot k is added, then refilled with the pass PD ahead (its row id was
  // gathered PD passes earlier; the slot's next row id is gathered now)
  float wr[PD], gr[PD];
  uint4 br[PD];
  int rn[PD];
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    const int p = lo + j * H6_RPP + t4, rr = row_of(p), k = wg_at(p, rr);
    wr[j] = a.w[k]; gr[j] = a.g[k]; br[j] = rec(rr);
  }
#pragma unroll
  for (int j = 0; j < PD; ++j) rn[j] = row_of(lo + (PD + j) * H6_RPP + t4);
  for (int p0 = lo; p0 < hi; p0 += PD * H6_RPP) {     // block-uniform trip count (unpack barriers)
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int pk = p0 + k * H6_RPP;                  // passes past hi add nothing (weight 0)
      update(pk + t4 < hi ? wr[k] : 0.f, gr[k], br[k]);
      flush(it);
      const int kw = wg_at(pk + PD * H6_RPP + t4, rn[k]);
      wr[k] = a.w[kw]; gr[k] = a.g[kw]; br[k] = rec(rn[k]);
      rn[k] = row_of(pk + 2 * PD * H6_RPP + t4);
    }
  }
  if constexpr (PERM) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int k = 0; k < H6_NE; ++k) unpack_add(h6[threadIdx.x + k * H6_T], accw[k], accg[k]);
  // slabs: entry e = (quarter e >> 12, bin (e >> 4) & 255, feature 16 quarter + (e & 15)) of the
  // 64; features 0-31 -> item ia, 32-63 -> item ib.  Transposed through LDS ([64 f][NB] int64 =
  // 128 KiB) per statistic for coalesced slab stores.
  long long* tsm = (long long*)h6;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < H6_NE; ++k) {
      const int e = threadIdx.x + k * H6_T;
      // PERM: e = (pair, bin, quarter & 1, feature) -> quarter ((e >> 13) << 1) | ((e >> 4) & 1)
      const int f = PERM ? ((((e >> 13) << 1) | ((e >> 4) & 1)) * 16 + (e & 15)) : ((e >> 12) * 16 + (e & 15));
      const int b = PERM ? ((e >> 5) & (NB - 1)) : ((e >> 4) & (NB - 1));
      tsm[f * NB + b] = st ? accg[k] : accw[k];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * FG * NB; i += H6_T) {
      const int half = i / (FG * NB);
      const int itm = half ? ib : ia;
      if (itm >= 0) a.slab[((size_t)itm * 2 + st) * FG * NB + (i % (FG * NB))] = tsm[i];
    }
  }
}

// ---------------------------------------------------------------------------------------
// Node histograms + split search.  One wave per (node, feature); 64 lanes x 4 bins.
// mode 0: built node  -> hist = sum of its items' slabs
// mode 1: derived node -> hist = parent_hist - sibling_hist (sibling built this level)
// Writes hist (fp32, for the next level's subtraction) and the best split candidate.
// ---------------------------------------------------------------------------------------
enum Imp : int { IMP_VARIANCE = 0, IMP_FRIEDMAN = 1, IMP_ENTROPY = 2, IMP_GINI = 3 };

struct SplitArgs {
  const long long* slab;        // [n_items][2][FG][NB] int64 fixed point
  const int* node_items;        // [n_nodes][n_groups][max_items] item ids (-1 padded) (mode 0)
  int max_items;
  const long long* parent_hist; // [n_parent][2][F][NB]                        (mode 1)
  const int* node_parent;       // [n_nodes] parent slot in parent_hist        (mode 1)
  const int* node_sibling;      // [n_nodes] sibling slot in hist              (mode 1)
  long long* hist;              // [n_nodes][2][F][NB] out (int64 fixed point)
  const int* node_list;         // nodes processed by this launch
  int n_list;
  const int* feat_list;         // candidate features (subset)
  int n_fsub;
  const int* nbins;             // [F]
  const uint8_t* is_cat;        // [F]
  const uint8_t* feat_mask;     // [n_nodes][F] optional per-node feature subset (nullable)
  float* cand;                  // [n_nodes][n_fsub][8]: gain, bin/k, lw, ls, rw, rs, valid, order_ref
  uint8_t* cat_order;           // [n_nodes][n_fsub][NB] sorted bin order for categorical (nullable)
  int F, mode, impurity, do_scan;
  float min_inst, min_gain;
  double inv_w, inv_g;          // 1 / fixed-point scales
};

__device__ __forceinline__ double imp_gain(int imp, double lw, double ls, double rw, double rs) {
  const double c = lw + rw, s = ls + rs;
  switch (imp) {
    case IMP_FRIEDMAN: { const double d = rw * ls - lw * rs; return d * d / (lw * rw * c); }
    case IMP_ENTROPY: {
      auto ent = [](double n, double p1) {   // binary classes: p1 = weight of class 1
        if (n <= 0.0) return 0.0;
        double r1 = p1 / n, r0 = 1.0 - r1, e = 0.0;
        if (r1 > 0.0) e -= r1 * log2(r1);
        if (r0 > 0.0) e -= r0 * log2(r0);
        return e;
      };
      return ent(c, s) - (lw / c) * ent(lw, ls) - (rw / c) * ent(rw, rs);
    }
    case IMP_GINI: {
      auto gin = [](double n, double p1) {
        if (n <= 0.0) return 0.0;
        double r1 = p1 / n, r0 = 1.0 - r1;
        return -(r1 * r1 + r0 * r0);
      };
      return gin(c, s) - (lw / c) * gin(lw, ls) - (rw / c) * gin(rw, rs);
    }
    default:   // variance: (sL^2/cL + sR^2/cR - s^2/c) / c  (sum-of-squares terms cancel)
      return (ls * ls / lw + rs * rs / rw - s * s / c) / c;
  }
}

__global__ __launch_bounds__(256) void gbdt_split_kernel(SplitArgs a) {
  __shared__ double skey[4][NB];
  __shared__ int sidx[4][NB];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long gw = (long)blockIdx.x * 4 + wv;
  if (gw >= (long)a.n_list * a.n_fsub) return;
  const int node = a.node_list[gw / a.n_fsub];
  const int fi = gw % a.n_fsub;
  const int f = a.feat_list[fi];
  float* cand = a.cand + ((size_t)node * a.n_fsub + fi) * 8;
  const size_t plane = (size_t)a.F * NB;              // stat plane stride inside a node
  long long* hw = a.hist + (size_t)node * 2 * plane + (size_t)f * NB;
  long long* hg = hw + plane;
  // ---- gather this (node, feature) histogram: 4 bins per lane (int64, exact) ----------
  long long qw[4], qg[4];
  const int b0 = lane * 4;
  if (a.mode == 0) {
    for (int k = 0; k < 4; ++k) { qw[k] = 0; qg[k] = 0; }
    // node_items is laid out [node][group][max_items]: the items of this node's feature group
    const int fg = f / FG, fl = f % FG;
    const int n_groups = (a.F + FG - 1) / FG;
    const int* its = a.node_items + ((size_t)node * n_groups + fg) * a.max_items;
    for (int t = 0; t < a.max_items; ++t) {
      const int it = its[t];
      if (it < 0) break;
      const long long* sw = a.slab + (size_t)it * 2 * FG * NB + (size_t)fl * NB + b0;
      const long long* sg = sw + FG * NB;
#pragma unroll
      for (int k = 0; k < 4; ++k) { qw[k] += sw[k]; qg[k] += sg[k]; }
    }
  } else if (a.mode == 2) {        // already-reduced histogram (after the cross-rank all-reduce)
#pragma unroll
    for (int k = 0; k < 4; ++k) { qw[k] = hw[b0 + k]; qg[k] = hg[b0 + k]; }
  } else {                         // derived sibling = parent - built sibling (exact in int64)
    const int par = a.node_parent[node], sib = a.node_sibling[node];
    const long long* pw = a.parent_hist + (size_t)par * 2 * plane + (size_t)f * NB;
    const long long* sw = a.hist + (size_t)sib * 2 * plane + (size_t)f * NB;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      qw[k] = pw[b0 + k] - sw[b0 + k];
      qg[k] = pw[plane + b0 + k] - sw[plane + b0 + k];
    }
  }
  if (a.mode != 2) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { hw[b0 + k] = qw[k]; hg[b0 + k] = qg[k]; }
  }
  if (!a.do_scan) return;
  double cw[4], cs[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) { cw[k] = (double)qw[k] * a.inv_w; cs[k] = (double)qg[k] * a.inv_g; }
  if (a.feat_mask && !a.feat_mask[(size_t)node * a.F + f]) {
    if (lane == 0) { cand[0] = -1.f; cand[6] = 0.f; }
    return;
  }
  const int nb = a.nbins[f];
  const bool cat = a.is_cat[f] != 0;
  // ---- categorical: order bins by mean target (ascending, stable by index) ----------------
  int order[4] = {b0, b0 + 1, b0 + 2, b0 + 3};
  if (cat) {
    for (int k = 0; k < 4; ++k) {
      const int b = b0 + k;
      // Impurity.getCategoricalOrderList: empty bin -> Double.MIN_VALUE; bins >= nb sort last
      double key = (b >= nb) ? 1e300 : (cw[k] != 0.0 ? cs[k] / cw[k] : 4.9e-324);
      skey[wv][b] = key;
      sidx[wv][b] = b;
    }
    __builtin_amdgcn_wave_barrier();
    // bitonic sort of 256 (key, idx) pairs, 4 per lane, lexicographic -> stable
    for (int size = 2; size <= NB; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int k = 0; k < 2; ++k) {
          const int t = lane + k * 64;          // 128 compare-exchange pairs
          const int i = 2 * stride * (t / stride) + (t % stride);
          const int j = i + stride;
          const bool up = ((i & size) == 0);
          const double ki = skey[wv][i], kj = skey[wv][j];
          const int ii = sidx[wv][i], ij = sidx[wv][j];
          const bool gt = (ki > kj) || (ki == kj && ii > ij);
          if (gt == up) { skey[wv][i] = kj; skey[wv][j] = ki; sidx[wv][i] = ij; sidx[wv][j] = ii; }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    // gather stats in sorted order: need stats by bin -> stash in LDS keyed by bin
    double tw[4], ts[4];
    for (int k = 0; k < 4; ++k) { tw[k] = cw[k]; ts[k] = cs[k]; }
    // write stats by bin into skey (reuse) after reading the order
    for (int k = 0; k < 4; ++k) order[k] = sidx[wv][b0 + k];
    __builtin_amdgcn_wave_barrier();
    for (int k = 0; k < 4; ++k) skey[wv][b0 + k] = tw[k];
    __builtin_amdgcn_wave_barrier();
    for (int k = 0; k < 4; ++k) cw[k] = skey[wv][order[k]];
    __builtin_amdgcn_wave_barrier();
    for (int k = 0; k < 4; ++k) skey[wv][b0 + k] = ts[k];
    __builtin_amdgcn_wave_barrier();
    for (int k = 0; k < 4; ++k) cs[k] = skey[wv][order[k]];
    if (a.cat_order) {
      uint8_t* co = a.cat_order + ((size_t)node * a.n_fsub + fi) * NB;
      for (int k = 0; k < 4; ++k) co[b0 + k] = (uint8_t)order[k];
    }
  }
  // ---- inclusive prefix over the 256 (ordered) bins ---------------------------------------
  double pw[4], ps[4];
  pw[0] = cw[0]; ps[0] = cs[0];
  for (int k = 1; k < 4; ++k) { pw[k] = pw[k - 1] + cw[k]; ps[k] = ps[k - 1] + cs[k]; }
  double xw = pw[3], xs = ps[3];
  for (int off = 1; off < 64; off <<= 1) {
    const double uw = __shfl_up(xw, off, 64), us = __shfl_up(xs, off, 64);
    if (lane >= off) { xw += uw; xs += us; }
  }
  const double ew = xw - pw[3], es = xs - ps[3];     // exclusive lane offset
  const double tw = __shfl(xw, 63, 64), ts = __shfl(xs, 63, 64);
  // candidates: left = ordered bins [0..b], b < nb - 1
  double best = -1.0;
  int bbin = -1;
  double blw = 0, bls = 0;
  for (int k = 0; k < 4; ++k) {
    const int b = b0 + k;
    if (b >= nb - 1) break;
    const double lw = ew + pw[k], ls = es + ps[k];
    const double rw = tw - lw, rs = ts - ls;
    if (lw <= a.min_inst || rw <= a.min_inst) continue;
    const double gain = imp_gain(a.impurity, lw, ls, rw, rs);
    if (!(gain > a.min_gain)) continue;
    if (gain > best) { best = gain; bbin = b; blw = lw; bls = ls; }
  }
  // wave argmax: max gain, ties -> lowest bin
  for (int off = 32; off > 0; off >>= 1) {
    const double og = __shfl_xor(best, off, 64);
    const int ob = __shfl_xor(bbin, off, 64);
    const double olw = __shfl_xor(blw, off, 64), ols = __shfl_xor(bls, off, 64);
    const bool take = (og > best) || (og == best && ob >= 0 && (bbin < 0 || ob < bbin));
    if (take) { best = og; bbin = ob; blw = olw; bls = ols; }
  }
  if (lane == 0) {
    cand[0] = (float)best;
    cand[1] = (float)bbin;
    cand[2] = (float)blw;
    cand[3] = (float)bls;
    cand[4] = (float)(tw - blw);
    cand[5] = (float)(ts - bls);
    cand[6] = bbin >= 0 ? 1.f : 0.f;
    cand[7] = (float)tw;
  }
}

// ---------------------------------------------------------------------------------------
// Partition: go-left flag per position for split nodes.  node_of_pos is computed by the
// caller as a per-position node slot array (int16) maintained alongside pos2row.
// split_feat < 0 -> node not split this level (rows stay, flag = 2 "keep").
// ---------------------------------------------------------------------------------------
struct PartArgs {
  const uint8_t* bins; long gs;   // quad-blocked [Q][N][128]
  // nullable: the feature-tiled copy of the same bins ([G][NT][32][128], the dense root pass's):
  // a row's split-feature byte then sits in a line of 128 consecutive rows of that feature, which
  // the node's other rows in the window share
  const uint8_t* bins32; long gs32;
  const int* pos2row;
  const int* pos_node;          // [N] node slot of each position (current level)
  const int* split_feat;        // [n_nodes]
  const int* split_bin;         // [n_nodes] numeric: left iff bin <= split_bin
  const uint32_t* cat_left;     // [n_nodes][8] categorical left bitset (bin b left iff bit set)
  const uint8_t* is_cat;        // [F]
  // out (nullable): left bit of every position (1 left, 0 right / not split) as one 64-bit word
  // per 64 positions (ballot), and the word's popcount -- 1/32 of an int32 flag array, and the
  // scatter ranks positions from the bits plus an exclusive scan of the per-word counts
  unsigned long long* fbits; int* wcnt;
  long n;
  long nmod;                    // > 0: forest batch (pos2row = tree * nmod + row)
  // fused GBT prediction update (replaces walking every row through the finished tree):
  // rows of nodes that stay leaves get pred += scale * node_val; on the final level rows of
  // split nodes get the value of the child they go to
  float* pred; const float* node_val; const float* child_l_val; const float* child_r_val;
  float scale; int final_level;
  // pos_node == nullptr: the node of a position comes from the level's node ranges sorted by
  // start (gbdt_range_index_kernel): r_start ascending, r_slot, node ends by slot
  const int* r_start; const int* r_slot; const int* r_end; int r_n;
};

// index r of the last sorted range starting at or before p (-1: none)
__device__ __forceinline__ int range_find(const int* rs, int nn, int p) {
  int lo = 0, hi = nn;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (rs[mid] <= p) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

// node slot of position p from the sorted ranges (-1: a finished node's position).  The search
// runs once per wave on the first active lane's position (uniform operands: scalar loads of the
// small index); lanes outside that node (a wave straddling a node boundary) search on their own
__device__ __forceinline__ int range_node(const int* rs, const int* rslot, const int* ren, int nn, int p) {
  const int p0 = __builtin_amdgcn_readfirstlane(p);
  const int r0 = range_find(rs, nn, p0);
  int s0 = -1, b0 = 0, e0 = 0;
  if (r0 >= 0) { s0 = rslot[r0]; b0 = rs[r0]; e0 = ren[s0]; }
  const bool in0 = r0 >= 0 && p >= b0 && p < e0;
  if (__all(in0)) return s0;
  const int r = range_find(rs, nn, p);
  if (r < 0) return -1;
  const int sl = rslot[r];
  return p < ren[sl] ? sl : -1;
}

// left bit of position p (+ the fused prediction update).  The node's parameters come from scalar
// loads of the wave's first lane's node when all 64 positions lie in it (nearly always), as in
// the scatter kernel
__device__ __forceinline__ int partition_flag(const PartArgs& a, long p) {
  const int node = a.pos_node ? a.pos_node[p] : range_node(a.r_start, a.r_slot, a.r_end, a.r_n, (int)p);
  const long v = a.pos2row[p], row = a.nmod ? v % a.nmod : v;
  const int nu = __builtin_amdgcn_readfirstlane(node);
  const int nd = __all(node == nu) ? nu : node;
  const int f = nd >= 0 ? a.split_feat[nd] : -1;
  int fl = 0;
  if (f >= 0) {
    const uint32_t b = a.bins32 ? a.bins32[(f >> 5) * a.gs32 + (row >> 7) * 4096 + (f & 31) * 128 + (row & 127)]
                                : a.bins[bin_off(a.gs, row, f)];
    if (a.is_cat[f]) fl = (a.cat_left[nd * 8 + (b >> 5)] >> (b & 31)) & 1;
    else fl = (int)b <= a.split_bin[nd] ? 1 : 0;
    if (a.pred && a.final_level) a.pred[row] += a.scale * (fl ? a.child_l_val[nd] : a.child_r_val[nd]);
  } else if (a.pred && nd >= 0) {
    a.pred[row] += a.scale * a.node_val[nd];
  }
  return fl;
}

__global__ void __launch_bounds__(256) gbdt_partition_flag_kernel(PartArgs a) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int fl = p < a.n ? partition_flag(a, p) : 0;
  if (a.fbits) {
    const unsigned long long m = __ballot(fl);
    if ((threadIdx.x & 63) == 0 && p < a.n) {
      a.fbits[p >> 6] = m;
      a.wcnt[p >> 6] = __popcll(m);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Final-level prediction update, row-window ordered.  Every current node's positions hold
// ascending rows (the stable partition keeps them so), so the positions of node k whose rows fall
// in window j = [j W, (j + 1) W) are one sub-range [bounds[k][j], bounds[k][j + 1]).  Block L works
// on window j = (L & 7) + 8 (L >> 3) / Y: each XCD walks its own windows in order, Y blocks per
// window, so the pred lines of a window (W x 4 B) are read-modify-written inside one XCD's L2
// while the window is open -- walking the positions node after node instead scattered
// 4-B updates over all of pred, one line fetch and one partial write-back per row.
// ---------------------------------------------------------------------------------------
struct LeafWinArgs {
  const uint8_t* bins; long gs;                  // quad-blocked [Q][N][128]
  const uint8_t* bins32; long gs32;              // nullable: feature-tiled copy
  const int* pos2row;
  const int* bounds;                             // [nn][NW + 1]
  int nn, NW, Y;
  const int* split_feat; const int* split_bin; const uint32_t* cat_left; const uint8_t* is_cat;
  float* pred; const float* node_val; const float* child_l_val; const float* child_r_val; float scale;
};

constexpr int LW_T = 256;
constexpr int LW_MAXN = 1024;

__global__ __launch_bounds__(LW_T) void gbdt_leaf_window_kernel(LeafWinArgs a) {
  __shared__ int pre[LW_MAXN + 1];
  const int L = blockIdx.x, j = (L & 7) + 8 * ((L >> 3) / a.Y), y = (L >> 3) % a.Y;
  if (j >= a.NW) return;
  const int nn = a.nn;
  for (int k = threadIdx.x; k < nn; k += LW_T)
    pre[k + 1] = a.bounds[(size_t)k * (a.NW + 1) + j + 1] - a.bounds[(size_t)k * (a.NW + 1) + j];
  if (threadIdx.x == 0) pre[0] = 0;
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k <= nn; ++k) pre[k] += pre[k - 1];
  __syncthreads();
  const int M = pre[nn];
  for (int v = y * LW_T + threadIdx.x; v < M; v += a.Y * LW_T) {
    int lo = 0, hi = nn;                                   // node k: pre[k] <= v < pre[k + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (pre[mid] <= v) lo = mid; else hi = mid;
    }
    const int k = lo;
    const long p = a.bounds[(size_t)k * (a.NW + 1) + j] + (v - pre[k]);
    const long row = a.pos2row[p];
    const int f = a.split_feat[k];
    float val;
    if (f >= 0) {
      const uint32_t b = a.bins32 ? a.bins32[(f >> 5) * a.gs32 + (row >> 7) * 4096 + (f & 31) * 128 + (row & 127)]
                                  : a.bins[bin_off(a.gs, row, f)];
      const bool left = a.is_cat[f] ? ((a.cat_left[k * 8 + (b >> 5)] >> (b & 31)) & 1) : ((int)b <= a.split_bin[k]);
      val = left ? a.child_l_val[k] : a.child_r_val[k];
    } else {
      val = a.node_val[k];
    }
    a.pred[row] += a.scale * val;
  }
}

// bounds[k][j] = first position of node k (in [start, end), ascending rows) with row >= j W
__global__ void gbdt_window_bounds_kernel(const int* pos2row, const int* starts, const int* ends, int nn, int NW,
                                          long W, int* bounds) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)nn * (NW + 1)) return;
  const int k = (int)(i / (NW + 1)), j = (int)(i % (NW + 1));
  int lo = starts[k], hi = max(starts[k], ends[k]);
  const long target = (long)j * W;
  while (lo < hi) {
    const int mid = lo + ((hi - lo) >> 1);
    if ((long)pos2row[mid] < target) lo = mid + 1; else hi = mid;
  }
  bounds[i] = lo;
}

// scatter: positions of split nodes move to [start + rank_left] or [start + n_left + rank_right]
struct ScatterArgs {
  const int* pos2row; const int* pos_node;
  const unsigned long long* fbits; const int* wpre;                          // left bits, exclusive word prefix
  const int* node_start; const int* node_nleft; const int* node_cum0;          // per node: start pos, #left, cum before start
  const int* split_feat;
  const int* child_left; const int* child_right;                               // new node slots
  int* new_pos2row; int* new_pos_node;
  // nullable: position-ordered per-row floats (w, g) moved with their rows (a pair of src / dst)
  const float* w_src; const float* g_src; float* w_dst; float* g_dst;
  long n;
  const int* r_start; const int* r_slot; const int* r_end; int r_n;   // pos_node == nullptr (as PartArgs)
};

__global__ void gbdt_partition_scatter_kernel(ScatterArgs a) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.n) return;
  // every per-position load first (independent of the node), then the node's parameters: a wave's
  // 64 positions almost always lie in one node, so those come from scalar loads of the wave's
  // first lane's node (vector loads only when the wave straddles a node boundary): 1.16 ->
  // 0.68 ms per 100M positions (profiles/r5/gbdt/partition_uniform_ab.txt)
  const int node = a.pos_node ? a.pos_node[p] : range_node(a.r_start, a.r_slot, a.r_end, a.r_n, (int)p);
  const int row = a.pos2row[p];
  float wv = 0.f, gv = 0.f;
  if (a.w_dst) { wv = a.w_src[p]; gv = a.g_src[p]; }
  const unsigned long long m = a.fbits[p >> 6];
  const int wp = a.wpre[p >> 6];
  const int nu = __builtin_amdgcn_readfirstlane(node);
  int sf, s, cum0, nleft, cl, cr;
  if (__all(node == nu)) {
    sf = nu >= 0 ? a.split_feat[nu] : -1;
    s = sf >= 0 ? a.node_start[nu] : 0; cum0 = sf >= 0 ? a.node_cum0[nu] : 0;
    nleft = sf >= 0 ? a.node_nleft[nu] : 0;
    cl = sf >= 0 ? a.child_left[nu] : -1; cr = sf >= 0 ? a.child_right[nu] : -1;
  } else {
    sf = node >= 0 ? a.split_feat[node] : -1;
    s = sf >= 0 ? a.node_start[node] : 0; cum0 = sf >= 0 ? a.node_cum0[node] : 0;
    nleft = sf >= 0 ? a.node_nleft[node] : 0;
    cl = sf >= 0 ? a.child_left[node] : -1; cr = sf >= 0 ? a.child_right[node] : -1;
  }
  long np = p;
  int child = -1;                                    // unsplit / finished rows keep their place
  if (sf >= 0) {
    const int lane = (int)(p & 63);
    const int cum = wp + __popcll(lane == 63 ? m : m & ((2ull << lane) - 1));   // inclusive
    const int before = cum - cum0;                   // #left in [s, p]
    if ((m >> lane) & 1) { np = s + before - 1; child = cl; }
    else { np = s + nleft + (int)(p - s) - before; child = cr; }
  }
  a.new_pos2row[np] = row;
  if (a.new_pos_node) a.new_pos_node[np] = child;
  if (a.w_dst) { a.w_dst[np] = wv; a.g_dst[np] = gv; }
}

// ---------------------------------------------------------------------------------------
// Tree application: walk a heap-ordered tree (<= 2^depth nodes) per row over its bins.
//   feat[id] < 0 -> leaf with value[id].  pred[row] += scale * value (or = value when set_mode).
// Used for validation rows, continuous-training recovery and GBT predict update.
// ---------------------------------------------------------------------------------------
struct TreeArgs {
  const uint8_t* bins; long gs;   // quad-blocked [Q][N][128]
  const int* rows;               // nullable: row ids (else 0..n-1)
  const int* feat; const int* thr; const uint32_t* cat_left; const float* value; const uint8_t* is_cat;
  float* pred; float scale; int set_mode;
  int* leaf_out;                 // nullable: leaf node id per row
  long n; int max_nodes;
};

__global__ void gbdt_apply_tree_kernel(TreeArgs a) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const long row = a.rows ? a.rows[i] : i;
  int id = 1;
  while (id < a.max_nodes && a.feat[id] >= 0) {
    const int f = a.feat[id];
    const uint32_t b = a.bins[bin_off(a.gs, row, f)];
    bool left;
    if (a.is_cat[f]) left = (a.cat_left[id * 8 + (b >> 5)] >> (b & 31)) & 1;
    else left = (int)b <= a.thr[id];
    id = left ? 2 * id : 2 * id + 1;
  }
  const float v = a.value[id];
  if (a.set_mode) a.pred[row] = v; else a.pred[row] += a.scale * v;
  if (a.leaf_out) a.leaf_out[row] = id;
}

// GBT residual refresh + error: output = -dLoss/dpredict (Loss.java), err += s * loss
struct ResidArgs {
  const float* pred; const float* y; const float* sig; float* out; double* err; long n; int loss;
};
__global__ __launch_bounds__(256) void gbdt_residual_kernel(ResidArgs a) {
  // grid-stride + block reduction: one pair of f64 atomics per block (not per wave)
  __shared__ double red[4][2];
  double e = 0.0, ws = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (long)gridDim.x * blockDim.x) {
    const float p = a.pred[i], y = a.y[i], s = a.sig ? a.sig[i] : 1.f;
    float grad, err;
    switch (a.loss) {
      case 1: grad = p - y; err = (p - y) * (p - y); break;                           // halfgradsquared
      case 2: grad = (y < p) ? 1.f : -1.f; err = fabsf(y - p); break;                   // absolute
      case 3: grad = (2.f - 4.f * y) / __expf(4.f * y * p - 2.f * p);                   // log
              err = log1pf(1.f + __expf(2.f * p - 4.f * p * y)); break;
      default: grad = 2.f * (p - y); err = (p - y) * (p - y); break;                    // squared
    }
    a.out[i] = -grad;
    e += (double)s * err;
    ws += s;
  }
  e = wave_sum_d(e);
  ws = wave_sum_d(ws);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[wv][0] = e; red[wv][1] = ws; }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(a.err, red[0][0] + red[1][0] + red[2][0] + red[3][0]);
    atomicAdd(a.err + 1, red[0][1] + red[1][1] + red[2][1] + red[3][1]);
  }
}

// Per-tree root statistics in one read of (w, g): sum w and sum w*g (f64, products of the f32
// inputs as in the host path) and max |w|, max |w*g| (the fixed-point scales).  Deterministic: a
// fixed grid of blocks writes per-block partials, one block sums them in a fixed order.
constexpr int WS_BLOCKS = 1024;

__device__ __forceinline__ float wave_max_f(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

__global__ __launch_bounds__(256) void gbdt_wg_stats_kernel(const float* w, const float* g, long n, double* part) {
  __shared__ double red[4][4];
  const long chunk = (n + WS_BLOCKS - 1) / WS_BLOCKS, lo = (long)blockIdx.x * chunk, hi = min(n, lo + chunk);
  double sw = 0.0, swg = 0.0;
  float mw = 0.f, mwg = 0.f;
  for (long i = lo + threadIdx.x; i < hi; i += 256) {
    const float wv = w[i], gv = g[i];
    sw += (double)wv;
    swg += (double)wv * (double)gv;
    mw = fmaxf(mw, fabsf(wv));
    mwg = fmaxf(mwg, fabsf(wv * gv));
  }
  sw = wave_sum_d(sw);
  swg = wave_sum_d(swg);
  mw = wave_max_f(mw);
  mwg = wave_max_f(mwg);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[wv][0] = sw; red[wv][1] = swg; red[wv][2] = mw; red[wv][3] = mwg; }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    double v = red[0][k];
    for (int j = 1; j < 4; ++j) v = k < 2 ? v + red[j][k] : fmax(v, red[j][k]);
    part[(long)blockIdx.x * 4 + k] = v;
  }
}

__global__ __launch_bounds__(256) void gbdt_wg_stats_final_kernel(const double* part, double* out) {
  __shared__ double red[4][4];
  double s0 = 0.0, s1 = 0.0, m0 = 0.0, m1 = 0.0;
  for (int b = threadIdx.x; b < WS_BLOCKS; b += 256) {
    s0 += part[b * 4]; s1 += part[b * 4 + 1];
    m0 = fmax(m0, part[b * 4 + 2]); m1 = fmax(m1, part[b * 4 + 3]);
  }
  s0 = wave_sum_d(s0);
  s1 = wave_sum_d(s1);
  for (int off = 32; off > 0; off >>= 1) { m0 = fmax(m0, __shfl_xor(m0, off, 64)); m1 = fmax(m1, __shfl_xor(m1, off, 64)); }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[wv][0] = s0; red[wv][1] = s1; red[wv][2] = m0; red[wv][3] = m1; }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    double v = red[0][k];
    for (int j = 1; j < 4; ++j) v = k < 2 ? v + red[j][k] : fmax(v, red[j][k]);
    out[k] = v;
  }
}

// ---------------------------------------------------------------------------------------
// Root level, sum w*g (MODE 2) over WHOLE 128-B records: one block builds the u32 histograms of
// all 128 features of a quad for its row range (128 x 256 u32 = 128 KiB of LDS), 8 threads per
// row each reading 16 B, so every fetched line is consumed by the CU that fetched it (the
// per-group items read a quarter of each line, 4x the L2->L1 traffic of the dense root pass).
// Bank = feature mod 64 ((bin * 128 + f) * 4 B); at step j lane (row slot r8, segment s)
// updates feature 16 s + ((j + rot) & 15) with rot = r8 + 8 (s >> 2): the 64 lanes of a wave
// hit 64 distinct banks whatever the bins are.  Sums stay exact: |q| < 2^20 - 1 on the root's
// coarser grid and 2048 rows between the int64 unpacks.
// ---------------------------------------------------------------------------------------
constexpr int RQ_T = 1024;                   // 16 waves: 128 rows per pass
constexpr int RQ_E = QF * NB / RQ_T;           // u32 entries each thread unpacks (64)

struct RootQuadArgs {
  const uint8_t* bins; long gs;              // quad-blocked [Q][N][128]
  const float* w; const float* g;
  const int* qitems;                         // [n][4] = {first item, lo, hi, quad}
  long long* slab;                           // [n_items][2][FG][NB]: this kernel writes the w*g half
  int n_groups;                              // 32-feature groups (G) = items per full quad
  float scale_g;                             // already / 2^GSH32
};

__global__ __launch_bounds__(RQ_T, 1) void gbdt_root_quad_kernel(RootQuadArgs a) {
  constexpr int RPQ = RQ_T / 8;               // rows per pass
  extern __shared__ __attribute__((aligned(16))) uint32_t hq[];    // [NB][128]
  const int qi = xcd_remap(blockIdx.x, gridDim.x);
  const int first = a.qitems[qi * 4], lo = a.qitems[qi * 4 + 1], hi = a.qitems[qi * 4 + 2],
            quad = a.qitems[qi * 4 + 3];
  for (int i = threadIdx.x; i < QF * NB; i += RQ_T) hq[i] = 0u;
  __syncthreads();
  const int seg = threadIdx.x & 7, rs = threadIdx.x >> 3;        // RPQ row slots x 8 segments
  const int rot = ((threadIdx.x >> 3) & 7) + ((seg >> 2) << 3);
  const uint8_t* qb = a.bins + (size_t)quad * a.gs + seg * 16;
  long long acc[RQ_E];
#pragma unroll
  for (int k = 0; k < RQ_E; ++k) acc[k] = 0;
  auto flush = [&]() {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RQ_E; ++k) {
      const int e = threadIdx.x + k * RQ_T;
      acc[k] += (long long)(int32_t)hq[e] * (1ll << GSH32);     // back on the scale_g grid (MODE 2)
      hq[e] = 0u;
    }
    __syncthreads();
  };
  int passes = 0;
  // software pipeline: next pass's record / w / g loaded before this pass's atomics
  auto load = [&](int r, uint4& b, float& q) {
    const int rc = min(r, hi - 1);
    b = *(const uint4*)(qb + (size_t)rc * QF);
    q = r < hi ? a.w[rc] * a.g[rc] * a.scale_g : 0.f;
  };
  uint4 bc; float qc;
  load(lo + rs, bc, qc);
  for (int r0 = lo; r0 < hi; r0 += RPQ) {                       // block-uniform trip count
    uint4 bn; float qn;
    load(r0 + RPQ + rs, bn, qn);
    const uint32_t q32 = (uint32_t)__float2int_rn(qc);
    if (qc != 0.f) {
      // rotate the 16 bytes left by rot: byte j of R = feature byte (j + rot) & 15
      const uint32_t W[4] = {bc.x, bc.y, bc.z, bc.w};
      uint32_t X[4], Y[4], R[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) X[k] = pick(W[k], W[(k + 1) & 3], rot & 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) Y[k] = pick(X[k], X[(k + 2) & 3], rot & 8);
#pragma unroll
      for (int k = 0; k < 4; ++k) R[k] = __builtin_amdgcn_alignbyte(Y[(k + 1) & 3], Y[k], rot & 3);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t b = (R[j >> 2] >> ((j & 3) * 8)) & 0xff;
        atomicAdd(&hq[(b << 7) | (seg << 4) | ((j + rot) & 15)], q32);
      }
    }
    if (++passes == 2048 / RPQ) { passes = 0; flush(); }
    bc = bn; qc = qn;
  }
  flush();
  // slabs: sub-group s of the quad -> item first + s, [1][fl][b] = feature 32 s + fl, bin b.
  // Thread t owns feature t & 127 and bins (t >> 7) + 4 k; transposed through LDS (64 features
  // x 256 bins of int64 = 128 KiB per half) so the slab rows leave as coalesced stores.
  const int nsub = min(4, a.n_groups - quad * 4);
  long long* tq = (long long*)hq;
  const int f_own = threadIdx.x & 127;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if ((f_own >> 6) == h) {
#pragma unroll
      for (int k = 0; k < RQ_E; ++k) tq[(f_own & 63) * NB + (threadIdx.x >> 7) + (RQ_T / 128) * k] = acc[k];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * NB; i += RQ_T) {
      const int f = h * 64 + (i >> 8), s = f >> 5;
      if (s < nsub) a.slab[((size_t)(first + s) * 2 + 1) * FG * NB + (size_t)(f & 31) * NB + (i & 255)] = tq[i];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Root pass over the feature-tiled copy of the bins: [G][NT][32][128], NT = ceil(N / 128).  A
// 4-KiB tile holds 128 rows x the 32 features of a group, each feature's 128 row bytes in one
// 128-B line.  The dense root pass streams whole tiles (every fetched byte used), and a
// partition below the root reads a node's split feature from lines that 128 consecutive rows
// share: the rows of one node that fall in one tile window hit one line (the row-record layout
// made every row fetch its own line; gbdt_partition_flag_kernel).
//
// Thread (tile slot ts, feature f = u & 31, chunk c = u >> 5) holds 16 row bytes of feature f and
// adds their per-row u32 q (precomputed by gbdt_root_q_kernel) to LDS [bin][copy][32] with
// copy = c & 1: the 64 lanes of a wave are 32 features x 2 copies -> 64 distinct banks for any
// bins (no rotation needed).  Each copy sees 128 of the 256 rows of a pass: 16 passes (2048
// rows per copy) between the int64 unpacks keep a bin's int32 sum exact (|q| < 2^20 - 1).
// ---------------------------------------------------------------------------------------
constexpr int RT_T = 512;                     // 8 waves: 2 tiles (256 rows) per pass
constexpr int RT_E = NB * FG / RT_T;          // (bin, feature) sums each thread owns (16)

struct RootTileArgs {
  const uint8_t* bins; long gs;              // [G][NT][32][128]: gs = NT * 4096 bytes per group
  const int* q;                              // [>= NT * 128] per-row u32 / i32 increment (0 past n)
  const int* items;                          // [n][4] = {node, lo, hi, group}
  long long* slab;                           // [n_items][2][FG][NB]
  int mode;                                  // 1: sum w (stat 0), 2: sum w*g (stat 1, x 2^GSH32)
  long n;                                    // rows (q is zero-padded past n to the tile end)
};

template <int MODE, int PD>
__global__ __launch_bounds__(RT_T) void gbdt_root_tile_kernel(RootTileArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t ht[];    // [NB][2][32]
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int lo = a.items[item * 4 + 1], hi = a.items[item * 4 + 2], grp = a.items[item * 4 + 3];
  for (int i = threadIdx.x; i < NB * 64; i += RT_T) ht[i] = 0u;
  __syncthreads();
  const int ts = threadIdx.x >> 8, u = threadIdx.x & 255, f = u & 31, c = u >> 5;
  const int lb = ((c & 1) << 5) | f;
  const uint8_t* gb = a.bins + (size_t)grp * a.gs + f * 128 + c * 16;
  long long acc[RT_E];
#pragma unroll
  for (int k = 0; k < RT_E; ++k) acc[k] = 0;
  auto flush = [&]() {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RT_E; ++k) {
      const int e = threadIdx.x + k * RT_T, i0 = ((e >> 5) << 6) | (e & 31);    // bin e >> 5, feature e & 31
      const uint32_t v0 = ht[i0], v1 = ht[i0 + 32];
      if constexpr (MODE == 1) acc[k] += (long long)v0 + (long long)v1;
      else acc[k] += ((long long)(int32_t)v0 + (long long)(int32_t)v1) * (1ll << GSH32);
      ht[i0] = 0u;
      ht[i0 + 32] = 0u;
    }
    __syncthreads();
  };
  const int t0 = lo >> 7, t1 = (hi + 127) >> 7;
  if (t1 <= t0) {                                             // no rows: zero slab
    long long* out = a.slab + ((size_t)item * 2 + (MODE == 1 ? 0 : 1)) * FG * NB;
    for (int i = threadIdx.x; i < FG * NB; i += RT_T) out[i] = 0;
    return;
  }
  // q of the chunk's 16 rows: lane (f & 3) = k of each 4-lane quad (same chunk) loads rows 4k..4k+3,
  // the others are broadcast from it by quad-permute DPP moves -- one 16-B q load per pass.
  // Loads are raw buffer loads: the per-lane part of the address in voffset (constant), the
  // wave-uniform tile in soffset (scalar arithmetic: no 64-bit VALU address math per pass)
  const int qk = f & 3;
  // Resources based at the item's first tile: the buffer offsets (and the range check) then span
  // only the item's own tiles, whatever the size of the copy (a group of 100M rows is 3.2 GB: a
  // whole-group resource clipped to 2^31 bytes read zeros past 67M rows)
  const long nt_item = (long)(t1 - t0);
  const __amdgpu_buffer_rsrc_t rb_bins = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.bins + (size_t)grp * a.gs + (size_t)t0 * 4096), (short)0, (int)(nt_item * 4096), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb_q = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.q + (size_t)t0 * 128), (short)0, (int)(nt_item * 512), 0x00020000);
  const int vo_b = f * 128 + c * 16, vo_q = (c * 16 + qk * 4) * 4;
  auto load = [&](int t, uint4& b, uint4& qv) {             // t: wave-uniform tile (clamped)
    const int tc = __builtin_amdgcn_readfirstlane(min(t, t1 - 1) - t0);
    const v4i_t bv = __builtin_amdgcn_raw_buffer_load_b128(rb_bins, vo_b, tc * 4096, 0);
    const v4i_t qq = __builtin_amdgcn_raw_buffer_load_b128(rb_q, vo_q, tc * 512, 0);
    b = make_uint4((uint32_t)bv[0], (uint32_t)bv[1], (uint32_t)bv[2], (uint32_t)bv[3]);
    qv = make_uint4((uint32_t)qq[0], (uint32_t)qq[1], (uint32_t)qq[2], (uint32_t)qq[3]);
  };
  // rows outside [lo, hi) add nothing (unaligned items only; applied when the pass is consumed)
  auto mask = [&](int t, uint4& qv) {
    const int tc = min(t, t1 - 1), r0 = tc * 128 + c * 16 + qk * 4;
    if (t >= t1 || r0 < lo || r0 + 4 > hi) {
      const int a0 = t >= t1 ? 4 : max(0, lo - r0), a1 = min(4, hi - r0);
      qv.x = (0 >= a0 && 0 < a1) ? qv.x : 0u;
      qv.y = (1 >= a0 && 1 < a1) ? qv.y : 0u;
      qv.z = (2 >= a0 && 2 < a1) ? qv.z : 0u;
      qv.w = (3 >= a0 && 3 < a1) ? qv.w : 0u;
    }
  };
  // The pass is VALU-bound (PMC: ~5.2 VALU per LDS atomic before, r6): each atomic's LDS byte
  // address bin * 256 + lane * 4 is ONE v_perm_b32 of the bin byte and the lane's byte offset, fed
  // to ds_add_u32 directly (the dynamic LDS array starts at byte 0: the kernel has no static LDS),
  // and items whose rows start and end on tile boundaries (the root items are chunked that way; q
  // is zero past n) skip the row mask: 2 VALU per atomic (perm + the q broadcast) plus the loop.
  const uint32_t lbyte = (uint32_t)lb * 4u;                   // < 256: byte 0 of every address
  auto consume = [&](const uint4& b, uint4 q0, int tt, auto masked) {
    if constexpr (decltype(masked)::value) mask(tt + ts, q0);
    const uint32_t B[4] = {b.x, b.y, b.z, b.w};
    const int Q[4] = {(int)q0.x, (int)q0.y, (int)q0.z, (int)q0.w};
    auto rows4 = [&](auto kc) {                               // rows 4k..4k+3 live in quad lane k
      constexpr int kq = decltype(kc)::value;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t qj = (uint32_t)__builtin_amdgcn_mov_dpp(Q[j], kq * 0x55, 0xf, 0xf, false);
        // bytes {lbyte, bin j of B[kq], 0, 0}: selector 0 = byte 0 of src1, 4 + j = byte j of src0
        const uint32_t addr = __builtin_amdgcn_perm(B[kq], lbyte, 0x0c0c0000u | ((4u + j) << 8));
        asm volatile("ds_add_u32 %0, %1" : : "v"(addr), "v"(qj) : "memory");
      }
    };
    rows4(std::integral_constant<int, 0>{});
    rows4(std::integral_constant<int, 1>{});
    rows4(std::integral_constant<int, 2>{});
    rows4(std::integral_constant<int, 3>{});
  };
  // the asm atomics are invisible to the compiler's LDS counter: drain them before the unpacks
  auto flush_asm = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); flush(); };
  // software pipeline over PD static slots: slot k is consumed, then refilled with the pass PD
  // ahead, so the other PD - 1 slots' loads stay in flight across its atomics.  Whole groups of PD
  // passes run branch-free; the last npass % PD passes are consumed after the loop.
  const int npass = (t1 - t0 + 1) >> 1;
  const bool aligned = (lo & 127) == 0 && ((hi & 127) == 0 || (long)hi == a.n);
  auto run = [&](auto masked) {
    uint4 br[PD], qr[PD];
#pragma unroll
    for (int j = 0; j < PD; ++j) load(t0 + 2 * j + ts, br[j], qr[j]);
    int passes = 0, pi = 0;
    // the last pass stays out of the branch-free loop: its second tile (waves with ts = 1) may lie
    // past t1 when the item has an odd tile count (the load clamps it to tile t1 - 1)
    for (; pi + PD < npass; pi += PD) {
#pragma unroll
      for (int k = 0; k < PD; ++k) {
        const int tt = t0 + 2 * (pi + k);
        consume(br[k], qr[k], tt, masked);
        load(tt + 2 * PD + ts, br[k], qr[k]);
        if (++passes == 16) { passes = 0; flush_asm(); }
      }
    }
#pragma unroll
    for (int k = 0; k < PD; ++k)
      if (pi + k < npass) {
        const int tt = t0 + 2 * (pi + k);
        if (tt + ts < t1) consume(br[k], qr[k], tt, masked);       // wave-uniform
        if (++passes == 16) { passes = 0; flush_asm(); }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  if (aligned) run(std::false_type{});
  else run(std::true_type{});
  flush();
  // slab [item][st][f][b]: transposed through LDS (32 x 256 int64 = 64 KiB) for coalesced stores
  long long* tt = (long long*)ht;
#pragma unroll
  for (int k = 0; k < RT_E; ++k) {
    const int e = threadIdx.x + k * RT_T;
    tt[(e & 31) * NB + (e >> 5)] = acc[k];
  }
  __syncthreads();
  long long* out = a.slab + ((size_t)item * 2 + (MODE == 1 ? 0 : 1)) * FG * NB;
  for (int i = threadIdx.x; i < FG * NB; i += RT_T) out[i] = tt[i];
}

// per-row increment of the tiled root pass: mode 1 u32(w * scale_w), mode 2 i32(w * g * scale_g)
// (scale_g already / 2^GSH32); rows [n, n_pad) get 0
__global__ void gbdt_root_q_kernel(const float* w, const float* g, long n, long n_pad, float scale, int mode, int* q) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pad) return;
  int v = 0;
  if (i < n) {
    const float wv = w[i];
    v = mode == 1 ? (int)__float2uint_rn(wv * scale) : __float2int_rn(wv * g[i] * scale);
  }
  q[i] = v;
}

// [Q][N][128] quad records -> [G][NT][32][128] feature tiles (one 4-KiB tile per block)
__global__ __launch_bounds__(256) void gbdt_tile_bins_kernel(const uint8_t* bins, long gs, long n, int G,
                                                            uint8_t* out, long gs_t) {
  __shared__ uint8_t tile[128][33];
  const long t = blockIdx.x;
  const int grp = blockIdx.y;
  const uint8_t* src = bins + (size_t)(grp >> 2) * gs + (grp & 3) * FG;
  for (int i = threadIdx.x; i < 128 * 32; i += 256) {
    const int r = i >> 5, f = i & 31;
    const long row = t * 128 + r;
    tile[r][f] = row < n ? src[(size_t)row * QF + f] : 0;
  }
  __syncthreads();
  uint8_t* dst = out + (size_t)grp * gs_t + (size_t)t * 4096;
  for (int i = threadIdx.x; i < 128 * 32; i += 256) {
    const int f = i >> 7, r = i & 127;
    dst[i] = tile[r][f];
  }
}

}  // namespace

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

// root histogram over the feature tiles: q scratch of >= NT * 128 ints (filled here from w, g)
SHIFU_API int shifu_gbdt_hist_root_tile(const void* tiles, long gs_t, long n, const float* w, const float* g,
                                        const int* items, int n_items, void* slab, double scale_w, double scale_g,
                                        int mode, int* q, hipStream_t stream) {
  const long nt = (n + 127) / 128;
  if (n <= 0 || n_items <= 0 || (mode != 1 && mode != 2) || gs_t != nt * 4096) return -1;
  if (nt * 128 > 0x7fffffffL) return -1;                      // row ids are int (items, q offsets)
  const float sc = mode == 1 ? (float)scale_w : (float)(scale_g / (1 << GSH32));
  hipLaunchKernelGGL(gbdt_root_q_kernel, dim3((unsigned)((nt * 128 + 255) / 256)), dim3(256), 0, stream, w, g, n,
                     nt * 128, sc, mode, q);
  RootTileArgs a{(const uint8_t*)tiles, gs_t, q, items, (long long*)slab, mode, n};
  const size_t lds = NB * 64 * 4;                              // 64 KiB (also the int64 transpose)
  // SHIFU_GBDT_ROOT_PD: tile passes in flight (lab A/B)
  static const int pd = [] { const char* e = getenv("SHIFU_GBDT_ROOT_PD"); return e ? atoi(e) : 6; }();   // 6: root 19.5-19.7 vs 19.8-20.0 ms with 4 (r6 gbdtenv_pd3)
  if (mode == 1) hipLaunchKernelGGL((gbdt_root_tile_kernel<1, 2>), dim3(n_items), dim3(RT_T), lds, stream, a);
  else if (pd >= 6) hipLaunchKernelGGL((gbdt_root_tile_kernel<2, 6>), dim3(n_items), dim3(RT_T), lds, stream, a);
  else if (pd >= 4) hipLaunchKernelGGL((gbdt_root_tile_kernel<2, 4>), dim3(n_items), dim3(RT_T), lds, stream, a);
  else if (pd == 3) hipLaunchKernelGGL((gbdt_root_tile_kernel<2, 3>), dim3(n_items), dim3(RT_T), lds, stream, a);
  else hipLaunchKernelGGL((gbdt_root_tile_kernel<2, 2>), dim3(n_items), dim3(RT_T), lds, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// out[4] (f64) = sum w, sum w*g, max |w|, max |w*g|; part: >= 4 * 1024 doubles of scratch
SHIFU_API int shifu_gbdt_wg_stats(const float* w, const float* g, long n, void* part, void* out, hipStream_t stream) {
  if (n < 0) return -1;
  hipLaunchKernelGGL(gbdt_wg_stats_kernel, dim3(WS_BLOCKS), dim3(256), 0, stream, w, g, n, (double*)part);
  hipLaunchKernelGGL(gbdt_wg_stats_final_kernel, dim3(1), dim3(256), 0, stream, (const double*)part, (double*)out);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// final-level fused prediction update in row windows (gbdt_leaf_window_kernel); bounds: scratch
// of >= nn * (NW + 1) ints, NW = ceil(n_rows / W) rounded up to a multiple of 8
SHIFU_API int shifu_gbdt_leaf_window(const void* bins, long gs, const void* bins32, long gs32, const int* pos2row,
                                     const int* starts, const int* ends, int nn, long n_rows, long W, int Y,
                                     int* bounds, const int* split_feat, const int* split_bin, const void* cat_left,
                                     const void* is_cat, float* pred, const float* node_val, const float* child_l_val,
                                     const float* child_r_val, float scale, hipStream_t stream) {
  if (nn <= 0) return 0;
  if (nn > LW_MAXN || W <= 0 || Y <= 0 || n_rows <= 0) return -1;
  const long nw = ((n_rows + W - 1) / W + 7) / 8 * 8;
  if (nw > (1L << 24) || nw * Y > 0x7fffffffL) return -1;
  const int NW = (int)nw;
  const long nb = (long)nn * (NW + 1);
  hipLaunchKernelGGL(gbdt_window_bounds_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, stream, pos2row,
                     starts, ends, nn, NW, W, bounds);
  LeafWinArgs a{(const uint8_t*)bins, gs, (const uint8_t*)bins32, gs32, pos2row, bounds, nn, NW, Y, split_feat,
                split_bin, (const uint32_t*)cat_left, (const uint8_t*)is_cat, pred, node_val, child_l_val,
                child_r_val, scale};
  hipLaunchKernelGGL(gbdt_leaf_window_kernel, dim3((unsigned)(nw * Y)), dim3(LW_T), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_tile_bins(const void* bins, long gs, long n, int G, void* out, long gs_t, hipStream_t stream) {
  const long nt = (n + 127) / 128;
  if (n <= 0 || G <= 0 || gs_t != nt * 4096 || nt > 0x7fffffffL) return -1;
  hipLaunchKernelGGL(gbdt_tile_bins_kernel, dim3((unsigned)nt, (unsigned)G), dim3(256), 0, stream,
                     (const uint8_t*)bins, gs, n, G, (uint8_t*)out, gs_t);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// Root sum w*g over whole quad records (gbdt_root_quad_kernel); qitems [n][4] = {first item, lo,
// hi, quad}, the items of a quad's groups consecutive in the slab.
SHIFU_API int shifu_gbdt_hist_root_quad(const void* bins, long gs, const float* w, const float* g, const int* qitems,
                                        int n_qitems, void* slab, int n_groups, double scale_g, hipStream_t stream) {
  if (gs % QF || n_qitems <= 0 || n_groups <= 0) return -1;
  RootQuadArgs a{(const uint8_t*)bins, gs, w, g, qitems, (long long*)slab, n_groups,
                 (float)(scale_g / (1 << GSH32))};
  hipLaunchKernelGGL(gbdt_root_quad_kernel, dim3(n_qitems), dim3(RQ_T), QF * NB * 4, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_hist(const void* bins, long gs, int rec, const int* pos2row, const float* w,
                              const float* g, int wg_by_pos, const int* items, int n_items, void* slab, int n_feat,
                              double scale_w, double scale_g, long nmod, int mode, hipStream_t stream) {
  if ((rec != QF && rec != FG) || gs % rec || n_items <= 0 || mode < 0 || mode > 2 || (wg_by_pos && nmod))
    return -1;
  HistArgs a{(const uint8_t*)bins, gs, pos2row, w, g, wg_by_pos, rec, items, (long long*)slab, n_items, n_feat,
             (float)scale_w, (float)(mode == 2 ? scale_g / (1 << GSH32) : scale_g), nmod};
  // SHIFU_HIST_PF: 3 (default) prefetching kernel, 1 row per thread and pass (2.9-3.07 TB/s of codes
  // below the root vs 2.3-2.5 with 2 rows: profiles/r5/gbdt_variants_r5k.txt); 1: 2 rows; 4: 4 rows;
  // 0: the non-prefetching kernel (lab A/B switch)
  static const int pf = [] { const char* e = getenv("SHIFU_HIST_PF"); return e ? atoi(e) : 3; }();
  const size_t lds = 2 * NB * 16 * 8;      // the u32 modes still use 64 KiB for the transposed store
  static const int root_hu = [] { const char* e = getenv("SHIFU_HIST_ROOT_HU"); return e ? atoi(e) : 2; }();
  if (mode == 1 && root_hu == 1) hipLaunchKernelGGL((gbdt_hist_kernel<true, 1, 1>), dim3(n_items), dim3(HT), lds, stream, a);
  else if (mode == 1) hipLaunchKernelGGL((gbdt_hist_kernel<true, 2, 1>), dim3(n_items), dim3(HT), lds, stream, a);
  else if (mode == 2 && root_hu == 1) hipLaunchKernelGGL((gbdt_hist_kernel<true, 1, 2>), dim3(n_items), dim3(HT), lds, stream, a);
  else if (mode == 2) hipLaunchKernelGGL((gbdt_hist_kernel<true, 2, 2>), dim3(n_items), dim3(HT), lds, stream, a);
  else if (pf == 4) hipLaunchKernelGGL((gbdt_hist_kernel<true, 4, 0>), dim3(n_items), dim3(HT), lds, stream, a);
  else if (pf == 3) hipLaunchKernelGGL((gbdt_hist_kernel<true, 1, 0>), dim3(n_items), dim3(HT), lds, stream, a);
  else if (pf) hipLaunchKernelGGL((gbdt_hist_kernel<true, 2, 0>), dim3(n_items), dim3(HT), lds, stream, a);
  else hipLaunchKernelGGL((gbdt_hist_kernel<false, 4, 0>), dim3(n_items), dim3(HT), lds, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// below-root histogram over half records (gbdt_hist64_kernel): pairs [n_pairs][2] of item ids
// (same node / rows, groups 2j and 2j + 1; the second -1 when the group count is odd)
SHIFU_API int shifu_gbdt_hist64(const void* bins, long gs, const int* pos2row, const float* w, const float* g,
                                int wg_by_pos, const int* items, int n_items, const int* pairs, int n_pairs,
                                void* slab, int n_feat, double scale_w, double scale_g, long nmod,
                                hipStream_t stream) {
  if (gs % QF || n_items <= 0 || n_pairs <= 0 || (wg_by_pos && nmod)) return -1;
  HistArgs a{(const uint8_t*)bins, gs, pos2row, w, g, wg_by_pos, QF, items, (long long*)slab, n_items, n_feat,
             (float)scale_w, (float)scale_g, nmod};
  // SHIFU_GBDT_H64_PD: passes in flight (lab A/B)
  static const int pd = [] { const char* e = getenv("SHIFU_GBDT_H64_PD"); return e ? atoi(e) : 3; }();
  // SHIFU_GBDT_H64_PERM=0: the [quarter][NB][16] layout with extract + shift-add addresses (lab A/B)
  static const bool perm = [] { const char* e = getenv("SHIFU_GBDT_H64_PERM"); return !e || atoi(e) != 0; }();
  const size_t lds = 4 * NB * 16 * 8;
  if (perm && pd >= 3) hipLaunchKernelGGL((gbdt_hist64_kernel<3, true>), dim3(n_pairs), dim3(H6_T), lds, stream, a, pairs);
  else if (perm) hipLaunchKernelGGL((gbdt_hist64_kernel<2, true>), dim3(n_pairs), dim3(H6_T), lds, stream, a, pairs);
  else if (pd >= 4) hipLaunchKernelGGL((gbdt_hist64_kernel<4, false>), dim3(n_pairs), dim3(H6_T), lds, stream, a, pairs);
  else if (pd == 3) hipLaunchKernelGGL((gbdt_hist64_kernel<3, false>), dim3(n_pairs), dim3(H6_T), lds, stream, a, pairs);
  else if (pd == 2) hipLaunchKernelGGL((gbdt_hist64_kernel<2, false>), dim3(n_pairs), dim3(H6_T), lds, stream, a, pairs);
  else hipLaunchKernelGGL((gbdt_hist64_kernel<1, false>), dim3(n_pairs), dim3(H6_T), lds, stream, a, pairs);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_split(const void* slab, const int* node_items, int max_items, const void* parent_hist,
                               const int* node_parent, const int* node_sibling, void* hist, const int* node_list,
                               int n_list, const int* feat_list, int n_fsub, const int* nbins, const void* is_cat,
                               const void* feat_mask, float* cand, void* cat_order, int F, int mode, int impurity,
                               int do_scan, float min_inst, float min_gain, double inv_w, double inv_g,
                               hipStream_t stream) {
  if (n_list <= 0 || n_fsub <= 0) return 0;
  SplitArgs a{(const long long*)slab, node_items, max_items, (const long long*)parent_hist, node_parent, node_sibling,
              (long long*)hist, node_list, n_list, feat_list, n_fsub, nbins, (const uint8_t*)is_cat,
              (const uint8_t*)feat_mask, cand, (uint8_t*)cat_order, F, mode, impurity, do_scan, min_inst, min_gain,
              inv_w, inv_g};
  const long waves = (long)n_list * n_fsub;
  hipLaunchKernelGGL(gbdt_split_kernel, dim3((waves + 3) / 4), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_partition_flag(const void* bins, long gs, const void* bins32, long gs32,
                                        const int* pos2row, const int* pos_node,
                                        const int* split_feat, const int* split_bin, const void* cat_left,
                                        const void* is_cat, void* fbits, int* wcnt, long n, long nmod, float* pred,
                                        const float* node_val, const float* child_l_val,
                                        const float* child_r_val, float scale, int final_level,
                                        const int* r_start, const int* r_slot, const int* r_end, int r_n,
                                        hipStream_t stream) {
  if (!pos_node && (!r_start || !r_slot || !r_end || r_n <= 0)) return -1;
  if (!pos_node && n >= 0x7fffffffL) return -1;
  PartArgs a{(const uint8_t*)bins, gs, (const uint8_t*)bins32, gs32, pos2row, pos_node, split_feat, split_bin, (const uint32_t*)cat_left,
             (const uint8_t*)is_cat, (unsigned long long*)fbits, wcnt, n, nmod, pred, node_val, child_l_val,
             child_r_val, scale,
             final_level, r_start, r_slot, r_end, r_n};
  // (a 4-positions-per-thread variant measured the same, 126.9 vs 127.9 ms per balanced round: the
  // pass is bound by the split-feature gather's line traffic, not by load parallelism; r5l)
  hipLaunchKernelGGL(gbdt_partition_flag_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_partition_scatter(const int* pos2row, const int* pos_node, const void* fbits, const int* wpre,
                                           const int* node_start, const int* node_nleft, const int* node_cum0,
                                           const int* split_feat, const int* child_left, const int* child_right,
                                           int* new_pos2row, int* new_pos_node, const float* w_src,
                                           const float* g_src, float* w_dst, float* g_dst, long n,
                                           const int* r_start, const int* r_slot, const int* r_end, int r_n,
                                           hipStream_t stream) {
  if ((w_dst != nullptr) != (g_dst != nullptr) || (w_dst && (!w_src || !g_src))) return -1;
  if (!pos_node && (!r_start || !r_slot || !r_end || r_n <= 0 || n >= 0x7fffffffL)) return -1;
  ScatterArgs a{pos2row, pos_node, (const unsigned long long*)fbits, wpre, node_start, node_nleft, node_cum0, split_feat, child_left,
                child_right, new_pos2row, new_pos_node, w_src, g_src, w_dst, g_dst, n, r_start, r_slot, r_end, r_n};
  hipLaunchKernelGGL(gbdt_partition_scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// inclusive left count cum[idx[i]] from the bits + word prefix (per-node boundaries for the host)
__global__ void gbdt_bitrank_kernel(const unsigned long long* fbits, const int* wpre, const long* idx, int m, int* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const long q = idx[i];
  const unsigned long long w = fbits[q >> 6];
  const int lane = (int)(q & 63);
  out[i] = wpre[q >> 6] + __popcll(lane == 63 ? w : w & ((2ull << lane) - 1));
}

// per node [start, end): left count before start (cum0) and #left in the node, from the bits +
// word prefix -- the scatter's node arrays, computed where the bits are (no host round trip)
// (chl / chr non-null: also the next level's node ranges, new_st / new_en by child slot -- the
// next level's histogram items resolve their row ranges from these on the device)
__global__ void gbdt_node_counts_kernel(const unsigned long long* fbits, const int* wpre, const int* starts,
                                        const int* ends, int nn, int* cum0, int* nleft, const int* chl,
                                        const int* chr, int* new_st, int* new_en) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  auto cum = [&](long q) {
    const unsigned long long w = fbits[q >> 6];
    const int lane = (int)(q & 63);
    return wpre[q >> 6] + __popcll(lane == 63 ? w : w & ((2ull << lane) - 1));
  };
  const int s = starts[i], e = ends[i];
  const int cb = s > 0 ? cum(s - 1) : 0;
  const int ce = e > s ? cum(e - 1) : cb;
  cum0[i] = cb;
  nleft[i] = ce - cb;
  if (chl && chl[i] >= 0) {
    new_st[chl[i]] = s; new_en[chl[i]] = s + (ce - cb);
    new_st[chr[i]] = s + (ce - cb); new_en[chr[i]] = e;
  }
}

SHIFU_API int shifu_gbdt_node_counts(const void* fbits, const int* wpre, const int* starts, const int* ends, int nn,
                                     int* cum0, int* nleft, const int* chl, const int* chr, int* new_st, int* new_en,
                                     hipStream_t stream) {
  if (nn <= 0) return 0;
  if (chl && (!chr || !new_st || !new_en)) return -1;
  hipLaunchKernelGGL(gbdt_node_counts_kernel, dim3((nn + 255) / 256), dim3(256), 0, stream,
                     (const unsigned long long*)fbits, wpre, starts, ends, nn, cum0, nleft, chl, chr, new_st, new_en);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_bitrank(const void* fbits, const int* wpre, const long* idx, int m, int* out,
                                 hipStream_t stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(gbdt_bitrank_kernel, dim3((m + 255) / 256), dim3(256), 0, stream,
                     (const unsigned long long*)fbits, wpre, idx, m, out);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_apply_tree(const void* bins, long gs, const int* rows, const int* feat, const int* thr,
                                    const void* cat_left, const float* value, const void* is_cat, float* pred,
                                    float scale, int set_mode, int* leaf_out, long n, int max_nodes,
                                    hipStream_t stream) {
  if (n <= 0) return 0;
  TreeArgs a{(const uint8_t*)bins, gs, rows, feat, thr, (const uint32_t*)cat_left, value, (const uint8_t*)is_cat,
             pred, scale, set_mode, leaf_out, n, max_nodes};
  hipLaunchKernelGGL(gbdt_apply_tree_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_gbdt_residual(const float* pred, const float* y, const float* sig, float* out, double* err,
                                  long n, int loss, hipStream_t stream) {
  if (n <= 0) return 0;
  ResidArgs a{pred, y, sig, out, err, n, loss};
  long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(gbdt_residual_kernel, dim3(blocks), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------
// Split decisions on the device.  After the split scan, one block turns the level's candidates
// into the partition's inputs (best feature per node with the lowest index on ties, split bin /
// categorical left set, leaf values, the children's next-level slots and values), so the
// partition is queued behind it at once and the host reads the same decisions later -- the
// level no longer waits on a host round trip between the split scan and the partition
// (DTMaster.java:298-355 makes these decisions on the master between two worker passes).
// The host applies the identical rules to the copied `best` rows (TreeTrainer._grow_levels_dev).
// ---------------------------------------------------------------------------------------
constexpr int DC_T = 1024;
constexpr int DC_MAXN = 512;

struct DecideArgs {
  const float* cand; int F, nn;                 // cand [nn][F][8]
  const int* meta;                              // [3][nn]: tree, node id, built
  const float* node_val;                        // [nn] leaf value of each node (fused prediction update)
  const uint8_t* cat_order;                     // [nn][F][NB] nullable
  const uint8_t* is_cat;
  int last;
  float* best;                                  // [nn][8]: feature, bin, gain, lw, ls, rw, rs, ok
  int* split_feat; int* split_bin; uint32_t* cat_left;   // [nn], [nn], [nn][8]
  int* child_l; int* child_r;                   // [nn] next-level slots (-1: leaf)
  float* lv;                                    // [3][nn]: node value, left / right child value
  float* next_val;                              // [2 nn] child values by next-level slot
};

__device__ __forceinline__ float leaf_value(float s, float w) {
  return w != 0.f ? (float)((double)s / (double)w) : 0.f;
}

__global__ __launch_bounds__(DC_T) void gbdt_decide_kernel(DecideArgs a) {
  __shared__ int s_ok[DC_MAXN];
  __shared__ int s_lb[DC_MAXN];                 // left child built (lw <= rw)
  __shared__ float s_cv[DC_MAXN][2];
  __shared__ long long s_key[2 * DC_MAXN];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nn = a.nn;
  for (int node = wv; node < nn; node += DC_T / 64) {
    float bg = -INFINITY;
    int bf = 0x7fffffff;
    for (int fi = lane; fi < a.F; fi += 64) {
      const float* c = a.cand + ((size_t)node * a.F + fi) * 8;
      const float gg = c[6] > 0.f ? c[0] : -INFINITY;
      if (gg > bg || (gg == bg && fi < bf)) { bg = gg; bf = fi; }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const float og = __shfl_xor(bg, off, 64);
      const int of = __shfl_xor(bf, off, 64);
      if (og > bg || (og == bg && of < bf)) { bg = og; bf = of; }
    }
    const int ok = bg > -INFINITY ? 1 : 0;
    if (!ok) bf = 0;
    const float* c = a.cand + ((size_t)node * a.F + bf) * 8;
    const int cat = ok && a.is_cat[bf];
    const int bin = (int)c[1];
    // categorical left set: the first bin + 1 entries of the node's mean-target order of bf
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (cat && a.cat_order) {
      const uint8_t* o = a.cat_order + ((size_t)node * a.F + bf) * NB;
      for (int k = lane * 4; k < lane * 4 + 4; ++k)
        if (k <= bin) { const int b = o[k]; words[b >> 5] |= 1u << (b & 31); }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        for (int off = 32; off > 0; off >>= 1) words[j] |= __shfl_xor(words[j], off, 64);
    }
    if (lane < 8) a.cat_left[node * 8 + lane] = words[lane];
    if (lane == 0) {
      float* b = a.best + (size_t)node * 8;
      b[0] = (float)bf; b[1] = c[1]; b[2] = c[0]; b[3] = c[2]; b[4] = c[3]; b[5] = c[4]; b[6] = c[5];
      b[7] = (float)ok;
      a.split_feat[node] = ok ? bf : -1;
      a.split_bin[node] = ok && !cat ? bin : -1;
      const float vl = ok ? leaf_value(c[3], c[2]) : 0.f, vr = ok ? leaf_value(c[5], c[4]) : 0.f;
      a.lv[node] = a.node_val[node];
      a.lv[nn + node] = vl;
      a.lv[2 * nn + node] = vr;
      s_ok[node] = ok;
      s_lb[node] = c[2] <= c[4];
      s_cv[node][0] = vl; s_cv[node][1] = vr;
    }
  }
  __syncthreads();
  if (a.last) {
    for (int i = threadIdx.x; i < nn; i += DC_T) { a.child_l[i] = -1; a.child_r[i] = -1; }
    return;
  }
  // next-level slot of child j = (node j / 2, side j % 2): its rank among the children by
  // (not built, tree, id) -- the host's _slot_key order
  for (int j = threadIdx.x; j < 2 * nn; j += DC_T) {
    const int node = j >> 1, side = j & 1;
    long long key = -1;
    if (s_ok[node]) {
      const int built = side == 0 ? s_lb[node] : !s_lb[node];
      key = ((long long)(built ? 0 : 1) << 62) | ((long long)a.meta[node] << 32) |
            (long long)(2 * a.meta[nn + node] + side);
    }
    s_key[j] = key;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * nn; j += DC_T) {
    const long long key = s_key[j];
    const int node = j >> 1, side = j & 1;
    if (key < 0) {
      if (side == 0) a.child_l[node] = -1; else a.child_r[node] = -1;
      continue;
    }
    int slot = 0;
    for (int t = 0; t < 2 * nn; ++t) slot += (s_key[t] >= 0 && s_key[t] < key) ? 1 : 0;
    if (side == 0) a.child_l[node] = slot; else a.child_r[node] = slot;
    a.next_val[slot] = s_cv[node][side];
  }
}

SHIFU_API int shifu_gbdt_decide(const float* cand, int F, int nn, const int* meta, const float* node_val,
                                const void* cat_order, const void* is_cat, int last, float* best, int* split_feat,
                                int* split_bin, void* cat_left, int* child_l, int* child_r, float* lv,
                                float* next_val, hipStream_t stream) {
  if (nn <= 0) return 0;
  if (nn > DC_MAXN || F <= 0 || F > (1 << 24)) return -1;
  DecideArgs a{cand, F, nn, meta, node_val, (const uint8_t*)cat_order, (const uint8_t*)is_cat, last, best,
               split_feat, split_bin, (uint32_t*)cat_left, child_l, child_r, lv, next_val};
  hipLaunchKernelGGL(gbdt_decide_kernel, dim3(1), dim3(DC_T), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// histogram items whose row ranges live on the device: items [n][4] = {slot, chunk, k, group} ->
// {slot, lo, hi, group}, chunk `chunk` of k equal pieces of the node's [start, end)
__global__ void gbdt_items_fix_kernel(int* items, int n, const int* starts, const int* ends) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int* it = items + (size_t)i * 4;
  const int slot = it[0], ch = it[1], k = max(1, it[2]);
  const int s = starts[slot], m = max(0, ends[slot] - s);
  const int step = (m + k - 1) / k;
  const long lo = min((long)m, (long)ch * step), hi = min((long)m, lo + step);
  it[1] = s + (int)lo;
  it[2] = s + (int)hi;
}

SHIFU_API int shifu_gbdt_items_fix(int* items, int n, const int* starts, const int* ends, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gbdt_items_fix_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, items, n, starts, ends);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// The level's node ranges sorted by start for range_node: empty ranges sort last (start INT_MAX).
// One block; nn <= DC_MAXN.
__global__ __launch_bounds__(256) void gbdt_range_index_kernel(const int* starts, const int* ends, int nn,
                                                               int* r_start, int* r_slot) {
  for (int i = threadIdx.x; i < nn; i += 256) {
    const int si = ends[i] > starts[i] ? starts[i] : 0x7fffffff;
    int rank = 0;
    for (int j = 0; j < nn; ++j) {
      const int sj = ends[j] > starts[j] ? starts[j] : 0x7fffffff;
      rank += (sj < si || (sj == si && j < i)) ? 1 : 0;
    }
    r_start[rank] = si;
    r_slot[rank] = i;
  }
}

SHIFU_API int shifu_gbdt_range_index(const int* starts, const int* ends, int nn, int* r_start, int* r_slot,
                                     hipStream_t stream) {
  if (nn <= 0 || nn > DC_MAXN) return -1;
  hipLaunchKernelGGL(gbdt_range_index_kernel, dim3(1), dim3(256), 0, stream, starts, ends, nn, r_start, r_slot);
  CHECK_HIP(hipGetLastError());
  return 0;
}
