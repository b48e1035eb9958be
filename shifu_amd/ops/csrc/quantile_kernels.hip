// K4: exact equal-population quantile binning + K19 HyperLogLog distinct counts (gfx950).
//
// Replaces the reference's per-mapper streaming histograms and reducer-side cut search
// (EqualPopulationBinning.java:491, UpdateBinningInfoMapper.java:349-599,
// MapReducerStatsWorker.java:105-176) with three mergeable passes over column-major fp64 data.
// Every pass accumulates into global state, so it runs unchanged over one resident column batch,
// over streamed row chunks, or per rank with an all-reduce between passes:
//
//   A  qprep   : per column min/max (as order-preserving u64 keys) of the selected finite values
//                and of all finite values, selected count, and p=14 HLL registers of all finite
//                values (splitmix64 of the canonical bits, rank = clz + 1).
//   B  qhist   : a 2048-bucket linear histogram of the selected values over [lo, hi] -- count,
//                fixed-point weight, and the min/max key inside each bucket -- plus min/max keys
//                per bucket of ALL finite values over their own range (exact distinct counts of
//                low-cardinality columns).  LDS-privatised (ds_add_u32/u64, ds_min/max_u64),
//                flushed once per block.
//   C  qgather : copies the selected values (and weights) of the buckets that hold a cut target
//                and more than one distinct value into per-bucket slots.  Two sweeps per block:
//                LDS counts, one global atomicAdd per (block, bucket) reserves a range, then the
//                values are placed -- no per-element global atomics.
//
// The host side (algos/quantile.py) turns the bucket prefix sums into the exact cut: a target
// bucket with min == max yields its value directly, otherwise the gathered slot is sorted on the
// device and searched.  The result equals binning.equal_population_boundaries bit for bit
// (integer ranks; fixed-point weights for the Weight* methods).
//
// Bucket mapping: floor((v - lo) * scale) clamped to [0, NB-1] -- monotone in v, so buckets
// partition the sorted order.  -0.0 is canonicalised to +0.0 (np.unique treats them as equal).
#include "common.h"

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

namespace {

constexpr int QNB = 2048;                 // histogram buckets per column
constexpr int HLL_P = 14;
constexpr int HLL_M = 1 << HLL_P;
constexpr int QT = 1024;                  // threads per block (16 waves)

__device__ __forceinline__ unsigned long long okey(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// numericalValueThreshold -> invalid; -0.0 -> +0.0; returns NaN for invalid
__device__ __forceinline__ double clean(double v, double thr) {
  return v > thr ? __longlong_as_double(0x7FF8000000000000ll) : v + 0.0;
}

__device__ __forceinline__ bool selected(const float* y, long r, int mode) {
  if (mode == 0) return true;
  const float t = y[r];
  return mode == 1 ? t > 0.5f : !(t > 0.5f);
}

__device__ __forceinline__ int bucket_of(double v, double lo, double scale) {
  const double f = (v - lo) * scale;
  int b = f <= 0.0 ? 0 : (f >= (double)(QNB - 1) ? QNB - 1 : (int)f);
  return b;
}

// A bucket's min/max keys only move outward, so a stale read that already lies strictly beyond k
// proves the atomic would change nothing.  Only the high dword is read (a 32-bit LDS read cannot
// tear against a concurrent 64-bit atomic); equal high dwords fall through to the atomic.
__device__ __forceinline__ bool covers_min(const unsigned long long* p, unsigned long long k) {
  return ((const volatile unsigned int*)p)[1] < (unsigned int)(k >> 32);
}
__device__ __forceinline__ bool covers_max(const unsigned long long* p, unsigned long long k) {
  return ((const volatile unsigned int*)p)[1] > (unsigned int)(k >> 32);
}

struct QArgs {
  const double* vals; long ldv; long n; int C;
  const float* y; const double* w; int sel_mode; double num_thr;
  long rows_per_block;
  const int* colmap;                      // blockIdx.y -> column (null = identity)
  const unsigned long long* win;          // [C][2] inclusive key window of the selected values
};

__device__ __forceinline__ int col_of(const QArgs& a) {
  return a.colmap ? a.colmap[blockIdx.x] : (int)blockIdx.x;
}

// ---------------------------------------------------------------------------------------------
// A: min/max keys + selected count + HLL registers
//    mm [C][4] u64: sel_min, sel_max, all_min, all_max (keys; min slots start at ~0)
//    scnt [C] u64; hll [C][HLL_M] u32
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(QT) qprep_kernel(QArgs a, unsigned long long* mm, unsigned long long* scnt,
                                                  unsigned int* hll) {
  __shared__ unsigned int reg[HLL_M];                 // 64 KiB
  __shared__ unsigned long long red[QT / WAVE][5];
  const int c = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < HLL_M; i += QT) reg[i] = 0u;
  __syncthreads();
  const long r0 = (long)blockIdx.y * a.rows_per_block;
  const long r1 = min(a.n, r0 + a.rows_per_block);
  const double* col = a.vals + (long)c * a.ldv;
  unsigned long long smin = ~0ull, smax = 0ull, amin = ~0ull, amax = 0ull, cnt = 0ull;
  for (long r = r0 + tid; r < r1; r += QT) {
    const double v = clean(col[r], a.num_thr);
    if (!isfinite(v)) continue;
    const unsigned long long k = okey(v);
    amin = min(amin, k); amax = max(amax, k);
    if (selected(a.y, r, a.sel_mode)) { smin = min(smin, k); smax = max(smax, k); cnt += 1ull; }
    const unsigned long long h = splitmix64((unsigned long long)__double_as_longlong(v));
    const unsigned int bkt = (unsigned int)(h >> (64 - HLL_P));
    const unsigned long long rest = (h << HLL_P) | (1ull << (HLL_P - 1));
    const unsigned int rk = (unsigned int)__clzll((long long)rest) + 1u;
    if (rk > reg[bkt]) atomicMax(&reg[bkt], rk);     // registers only grow: a stale read is safe
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    smin = min(smin, (unsigned long long)__shfl_xor((long long)smin, o, 64));
    smax = max(smax, (unsigned long long)__shfl_xor((long long)smax, o, 64));
    amin = min(amin, (unsigned long long)__shfl_xor((long long)amin, o, 64));
    amax = max(amax, (unsigned long long)__shfl_xor((long long)amax, o, 64));
    cnt += (unsigned long long)__shfl_xor((long long)cnt, o, 64);
  }
  const int wid = tid >> 6, lane = tid & 63;
  if (lane == 0) { red[wid][0] = smin; red[wid][1] = smax; red[wid][2] = amin; red[wid][3] = amax; red[wid][4] = cnt; }
  __syncthreads();
  if (tid == 0) {
    for (int k = 1; k < QT / WAVE; ++k) {
      red[0][0] = min(red[0][0], red[k][0]); red[0][1] = max(red[0][1], red[k][1]);
      red[0][2] = min(red[0][2], red[k][2]); red[0][3] = max(red[0][3], red[k][3]);
      red[0][4] += red[k][4];
    }
    if (red[0][4]) { atomicMin(&mm[c * 4 + 0], red[0][0]); atomicMax(&mm[c * 4 + 1], red[0][1]); }
    if (red[0][2] <= red[0][3]) { atomicMin(&mm[c * 4 + 2], red[0][2]); atomicMax(&mm[c * 4 + 3], red[0][3]); }
    if (red[0][4]) atomicAdd(&scnt[c], red[0][4]);
  }
  unsigned int* g = hll + (long)c * HLL_M;
  for (int i = tid; i < HLL_M; i += QT)
    if (reg[i]) atomicMax(&g[i], reg[i]);
}

// ---------------------------------------------------------------------------------------------
// B: bucket histograms.  prm [C][4] doubles: sel lo, sel scale, all lo, all scale.
//    cnt [C][QNB] u64, wq [C][QNB] u64 (weighted only), kmn/kmx [C][QNB] u64 (selected),
//    akmn/akmx [C][QNB] u64 (all finite; only when with_all)
// ---------------------------------------------------------------------------------------------
struct HistOut {
  unsigned long long *cnt, *wq, *kmn, *kmx, *akmn, *akmx;
};

template <bool WEIGHTED, bool WITH_ALL>
__global__ void __launch_bounds__(QT) qhist_kernel(QArgs a, const double* prm, double wscale, HistOut o) {
  __shared__ unsigned int lcnt[QNB];
  __shared__ unsigned long long lwq[WEIGHTED ? QNB : 1];
  __shared__ unsigned long long lmn[QNB], lmx[QNB];
  __shared__ unsigned long long lamn[WITH_ALL ? QNB : 1], lamx[WITH_ALL ? QNB : 1];
  const int c = col_of(a), tid = threadIdx.x;
  const unsigned long long wlo = a.win[2 * c], whi = a.win[2 * c + 1];
  for (int i = tid; i < QNB; i += QT) {
    lcnt[i] = 0u; lmn[i] = ~0ull; lmx[i] = 0ull;
    if (WEIGHTED) lwq[i] = 0ull;
    if (WITH_ALL) { lamn[i] = ~0ull; lamx[i] = 0ull; }
  }
  __syncthreads();
  const double lo = prm[c * 4 + 0], sc = prm[c * 4 + 1], alo = prm[c * 4 + 2], asc = prm[c * 4 + 3];
  const long r0 = (long)blockIdx.y * a.rows_per_block;
  const long r1 = min(a.n, r0 + a.rows_per_block);
  const double* col = a.vals + (long)c * a.ldv;
  for (long r = r0 + tid; r < r1; r += QT) {
    const double v = clean(col[r], a.num_thr);
    if (!isfinite(v)) continue;
    const unsigned long long k = okey(v);
    if (WITH_ALL) {
      const int ab = bucket_of(v, alo, asc);
      if (!covers_min(&lamn[ab], k)) atomicMin(&lamn[ab], k);
      if (!covers_max(&lamx[ab], k)) atomicMax(&lamx[ab], k);
    }
    if (!selected(a.y, r, a.sel_mode) || k < wlo || k > whi) continue;
    const int b = bucket_of(v, lo, sc);
    atomicAdd(&lcnt[b], 1u);
    if (!covers_min(&lmn[b], k)) atomicMin(&lmn[b], k);
    if (!covers_max(&lmx[b], k)) atomicMax(&lmx[b], k);
    if (WEIGHTED) {
      const double q = fmax(a.w[r], 0.0) * wscale;
      atomicAdd(&lwq[b], (unsigned long long)__double2ll_rn(q));
    }
  }
  __syncthreads();
  const long base = (long)c * QNB;
  for (int i = tid; i < QNB; i += QT) {
    if (lcnt[i]) {
      atomicAdd(&o.cnt[base + i], (unsigned long long)lcnt[i]);
      atomicMin(&o.kmn[base + i], lmn[i]);
      atomicMax(&o.kmx[base + i], lmx[i]);
      if (WEIGHTED && lwq[i]) atomicAdd(&o.wq[base + i], lwq[i]);
    }
    if (WITH_ALL && lamn[i] <= lamx[i]) {
      atomicMin(&o.akmn[base + i], lamn[i]);
      atomicMax(&o.akmx[base + i], lamx[i]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// C: gather the selected values of flagged buckets.  slot [C][QNB] int (-1 = not gathered);
//    sbase [S] i64 start of each slot in gv; scur [S] u32 running fill (persists across chunks)
// ---------------------------------------------------------------------------------------------
template <bool WEIGHTED>
__global__ void __launch_bounds__(QT) qgather_kernel(QArgs a, const double* prm, double wscale, const int* slot,
                                                    const long* sbase, unsigned int* scur, double* gv,
                                                    unsigned long long* gq) {
  __shared__ int lslot[QNB];
  __shared__ unsigned int lc[QNB], lb[QNB];
  const int c = col_of(a), tid = threadIdx.x;
  const unsigned long long wlo = a.win[2 * c], whi = a.win[2 * c + 1];
  for (int i = tid; i < QNB; i += QT) { lslot[i] = slot[(long)c * QNB + i]; lc[i] = 0u; }
  __syncthreads();
  const double lo = prm[c * 4 + 0], sc = prm[c * 4 + 1];
  const long r0 = (long)blockIdx.y * a.rows_per_block;
  const long r1 = min(a.n, r0 + a.rows_per_block);
  const double* col = a.vals + (long)c * a.ldv;
  for (long r = r0 + tid; r < r1; r += QT) {
    const double v = clean(col[r], a.num_thr);
    if (!isfinite(v) || !selected(a.y, r, a.sel_mode)) continue;
    const unsigned long long k = okey(v);
    if (k < wlo || k > whi) continue;
    const int b = bucket_of(v, lo, sc);
    if (lslot[b] >= 0) atomicAdd(&lc[b], 1u);
  }
  __syncthreads();
  for (int i = tid; i < QNB; i += QT) {
    if (lc[i]) lb[i] = atomicAdd(&scur[lslot[i]], lc[i]);
    lc[i] = 0u;
  }
  __syncthreads();
  for (long r = r0 + tid; r < r1; r += QT) {
    const double v = clean(col[r], a.num_thr);
    if (!isfinite(v) || !selected(a.y, r, a.sel_mode)) continue;
    const unsigned long long k = okey(v);
    if (k < wlo || k > whi) continue;
    const int b = bucket_of(v, lo, sc);
    const int s = lslot[b];
    if (s < 0) continue;
    const long at = sbase[s] + (long)lb[b] + (long)atomicAdd(&lc[b], 1u);
    gv[at] = v;
    if (WEIGHTED) gq[at] = (unsigned long long)__double2ll_rn(fmax(a.w[r], 0.0) * wscale);
  }
}

int grid_chunks(long n, int C) {
  // >= 8 blocks per CU over the batch, >= 16K rows per block (bounds the per-block flush)
  long by_rows = (n + 16383) / 16384;
  long want = (2048 + C - 1) / C;
  long ch = by_rows < want ? by_rows : want;
  return (int)(ch < 1 ? 1 : ch);
}

}  // namespace

SHIFU_API int shifu_qprep(const double* vals, long ldv, long n, int C, const float* y, int sel_mode, double num_thr,
                          void* mm, void* scnt, void* hll, hipStream_t stream) {
  if (n <= 0 || C <= 0) return 0;
  if (ldv < n || (sel_mode != 0 && !y)) return -1;
  const int ch = grid_chunks(n, C);
  QArgs a{vals, ldv, n, C, y, nullptr, sel_mode, num_thr, (n + ch - 1) / ch, nullptr, nullptr};
  hipLaunchKernelGGL(qprep_kernel, dim3(C, ch), dim3(QT), 0, stream, a, (unsigned long long*)mm,
                     (unsigned long long*)scnt, (unsigned int*)hll);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_qhist(const double* vals, long ldv, long n, int C, const float* y, const double* w, int sel_mode,
                          double num_thr, const int* colmap, int ncols, const void* win, const double* prm,
                          double wscale, int with_all, void* cnt, void* wq, void* kmn, void* kmx, void* akmn,
                          void* akmx, hipStream_t stream) {
  if (n <= 0 || C <= 0 || ncols <= 0) return 0;
  if (ldv < n || (sel_mode != 0 && !y) || (wq && !w) || (with_all && (!akmn || !akmx)) || !win) return -1;
  if (!colmap && ncols != C) return -1;
  const int ch = grid_chunks(n, ncols);
  QArgs a{vals, ldv, n, C, y, w, sel_mode, num_thr, (n + ch - 1) / ch, colmap, (const unsigned long long*)win};
  HistOut o{(unsigned long long*)cnt, (unsigned long long*)wq, (unsigned long long*)kmn, (unsigned long long*)kmx,
            (unsigned long long*)akmn, (unsigned long long*)akmx};
  dim3 g(ncols, ch), b(QT);
  if (wq) {
    if (with_all) hipLaunchKernelGGL((qhist_kernel<true, true>), g, b, 0, stream, a, prm, wscale, o);
    else hipLaunchKernelGGL((qhist_kernel<true, false>), g, b, 0, stream, a, prm, wscale, o);
  } else {
    if (with_all) hipLaunchKernelGGL((qhist_kernel<false, true>), g, b, 0, stream, a, prm, wscale, o);
    else hipLaunchKernelGGL((qhist_kernel<false, false>), g, b, 0, stream, a, prm, wscale, o);
  }
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_qgather(const double* vals, long ldv, long n, int C, const float* y, const double* w, int sel_mode,
                            double num_thr, const int* colmap, int ncols, const void* win, const double* prm,
                            double wscale, const int* slot, const long* sbase, void* scur, double* gv, void* gq,
                            hipStream_t stream) {
  if (n <= 0 || C <= 0 || ncols <= 0) return 0;
  if (ldv < n || (sel_mode != 0 && !y) || (gq && !w) || !win) return -1;
  if (!colmap && ncols != C) return -1;
  const int ch = grid_chunks(n, ncols);
  QArgs a{vals, ldv, n, C, y, w, sel_mode, num_thr, (n + ch - 1) / ch, colmap, (const unsigned long long*)win};
  dim3 g(ncols, ch), b(QT);
  if (gq) hipLaunchKernelGGL((qgather_kernel<true>), g, b, 0, stream, a, prm, wscale, slot, sbase,
                             (unsigned int*)scur, gv, (unsigned long long*)gq);
  else hipLaunchKernelGGL((qgather_kernel<false>), g, b, 0, stream, a, prm, wscale, slot, sbase,
                          (unsigned int*)scur, gv, (unsigned long long*)nullptr);
  CHECK_HIP(hipGetLastError());
  return 0;
}
