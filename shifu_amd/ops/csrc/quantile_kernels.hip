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

// row selection (EqualPositive / EqualNegative) as a packed bitmask: 1 bit per row instead of a
// 4-byte label per row per column -- a 64-column batch would otherwise re-read the labels 64 times
__device__ __forceinline__ bool selected(const unsigned int* sel, long r) {
  return !sel || ((sel[r >> 5] >> (r & 31)) & 1u);
}

__device__ __forceinline__ int bucket_of(double v, double lo, double scale) {
  const double f = (v - lo) * scale;
  int b = f <= 0.0 ? 0 : (f >= (double)(QNB - 1) ? QNB - 1 : (int)f);
  return b;
}

// A bucket's min/max keys only move outward, so a (stale) value that already covers k proves the
// atomic would change nothing.  The two dwords are read as 32-bit loads, high then low (one wave's
// LDS accesses execute in order): a mixed read (older high, newer low) of a decreasing minimum is
// >= the minimum at the time of the low read, of an increasing maximum <= it -- so "covers" never
// errs towards skipping a needed update.  Equal keys (single-valued buckets) skip the atomic too.
__device__ __forceinline__ bool covers_min(const unsigned long long* p, unsigned long long k) {
  const volatile unsigned int* q = (const volatile unsigned int*)p;
  const unsigned int hi = q[1], khi = (unsigned int)(k >> 32);
  if (hi != khi) return hi < khi;
  return q[0] <= (unsigned int)k;
}
__device__ __forceinline__ bool covers_max(const unsigned long long* p, unsigned long long k) {
  const volatile unsigned int* q = (const volatile unsigned int*)p;
  const unsigned int hi = q[1], khi = (unsigned int)(k >> 32);
  if (hi != khi) return hi > khi;
  return q[0] >= (unsigned int)k;
}

// A window of one column's selected values at the current refinement level: the inclusive key
// range [lo_key, hi_key], mapped onto `size` of the column's 2048 buckets starting at `base`, either
// linearly in value (msh < 0: floor((v - mlo) * msc)) or in key space ((key - mklo) >> msh).
// Level 1 is one window per column over everything; each later level refines every unresolved
// target bucket into its own window, so one pass serves all of a column's cut targets.
struct QWin {
  unsigned long long lo_key, hi_key;
  double mlo, msc;
  long long msh;
  unsigned long long mklo;
  int base, size;
};
static_assert(sizeof(QWin) == 56, "QWin layout is shared with algos/quantile.py");
constexpr int MAXW = 128;                 // windows per column (algos/quantile.py MAX_WINDOWS)

struct QArgs {
  const double* vals; long ldv; long n; int C;
  const unsigned int* sel; const double* w; int sel_mode; double num_thr;
  long rows_per_block;
  const int* colmap;                      // blockIdx.x -> column (null = identity)
  const int* wptr;                        // [C+1] window ranges of each column in `wins`
  const QWin* wins;
};

__device__ __forceinline__ int col_of(const QArgs& a) {
  return a.colmap ? a.colmap[blockIdx.x] : (int)blockIdx.x;
}

// the column's windows staged in LDS; returns the bucket of key k (value v) or -1 outside
struct WinLDS {
  unsigned long long lo[MAXW], hi[MAXW], klo[MAXW];
  double mlo[MAXW], msc[MAXW];
  int msh[MAXW], base[MAXW], size[MAXW];
  int n;
};

__device__ __forceinline__ void load_windows(WinLDS& W, const QArgs& a, int c) {
  const int w0 = a.wptr[c], nw = a.wptr[c + 1] - w0;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const QWin q = a.wins[w0 + i];
    W.lo[i] = q.lo_key; W.hi[i] = q.hi_key; W.klo[i] = q.mklo;
    W.mlo[i] = q.mlo; W.msc[i] = q.msc; W.msh[i] = (int)q.msh; W.base[i] = q.base; W.size[i] = q.size;
  }
  if (threadIdx.x == 0) W.n = nw;
}

__device__ __forceinline__ int win_bucket(const WinLDS& W, double v, unsigned long long k) {
  int t = 0;
  if (W.n > 1) {                          // last window with lo <= k (windows sorted, disjoint)
    int lo = 0, hi = W.n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (W.lo[mid] <= k) lo = mid; else hi = mid - 1;
    }
    t = lo;
  }
  if (W.n == 0 || k < W.lo[t] || k > W.hi[t]) return -1;
  const int sz = W.size[t];
  int b;
  if (W.msh[t] < 0) {
    const double f = (v - W.mlo[t]) * W.msc[t];
    b = f <= 0.0 ? 0 : (f >= (double)(sz - 1) ? sz - 1 : (int)f);
  } else {
    const unsigned long long q = (k - W.klo[t]) >> W.msh[t];
    b = q > (unsigned long long)(sz - 1) ? sz - 1 : (int)q;
  }
  return W.base[t] + b;
}

// ---------------------------------------------------------------------------------------------
// A: min/max keys + selected count + HLL registers
//    mm [C][4] u64: sel_min, sel_max, all_min, all_max (keys; min slots start at ~0)
//    scnt [C] u64; hll [C][HLL_M] u32
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(QT) qprep_kernel(QArgs a, unsigned long long* mm, unsigned long long* scnt,
                                                  unsigned int* hll, double* mom) {
  __shared__ unsigned int reg[HLL_M];                 // 64 KiB
  __shared__ unsigned long long red[QT / WAVE][5];
  __shared__ double redm[QT / WAVE][2];
  const int c = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < HLL_M; i += QT) reg[i] = 0u;
  __syncthreads();
  const long r0 = (long)blockIdx.y * a.rows_per_block;
  const long r1 = min(a.n, r0 + a.rows_per_block);
  const double* col = a.vals + (long)c * a.ldv;
  unsigned long long smin = ~0ull, smax = 0ull, amin = ~0ull, amax = 0ull, cnt = 0ull;
  double s1 = 0.0, s2 = 0.0;
  for_rows<4>(col, r0, r1, QT, [&](long r, double raw) {
    const double v = clean(raw, a.num_thr);
    if (!isfinite(v)) return;
    const unsigned long long k = okey(v);
    amin = min(amin, k); amax = max(amax, k);
    if (selected(a.sel, r)) { smin = min(smin, k); smax = max(smax, k); cnt += 1ull; s1 += v; s2 += v * v; }
    const unsigned long long h = splitmix64((unsigned long long)__double_as_longlong(v));
    const unsigned int bkt = (unsigned int)(h >> (64 - HLL_P));
    const unsigned long long rest = (h << HLL_P) | (1ull << (HLL_P - 1));
    const unsigned int rk = (unsigned int)__clzll((long long)rest) + 1u;
    if (rk > reg[bkt]) atomicMax(&reg[bkt], rk);     // registers only grow: a stale read is safe
  });

#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    smin = min(smin, (unsigned long long)__shfl_xor((long long)smin, o, 64));
    smax = max(smax, (unsigned long long)__shfl_xor((long long)smax, o, 64));
    amin = min(amin, (unsigned long long)__shfl_xor((long long)amin, o, 64));
    amax = max(amax, (unsigned long long)__shfl_xor((long long)amax, o, 64));
    cnt += (unsigned long long)__shfl_xor((long long)cnt, o, 64);
  }
  s1 = wave_sum_d(s1);
  s2 = wave_sum_d(s2);
  const int wid = tid >> 6, lane = tid & 63;
  if (lane == 0) {
    red[wid][0] = smin; red[wid][1] = smax; red[wid][2] = amin; red[wid][3] = amax; red[wid][4] = cnt;
    redm[wid][0] = s1; redm[wid][1] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    double m1 = 0.0, m2 = 0.0;
    for (int k = 0; k < QT / WAVE; ++k) { m1 += redm[k][0]; m2 += redm[k][1]; }
    if (m1 != 0.0 || m2 != 0.0) { atomicAdd(&mom[c * 2 + 0], m1); atomicAdd(&mom[c * 2 + 1], m2); }
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
// B: bucket histograms of the selected values through the column's windows:
//    cnt [C][QNB] u64, wq [C][QNB] u64 (weighted only), kmn/kmx [C][QNB] u64 (selected keys),
//    and at level 1 akmn/akmx [C][QNB] u64: min/max keys of ALL finite values over their own
//    linear map aprm [C][2] (lo, scale) -- exact distinct counts of low-cardinality columns.
// ---------------------------------------------------------------------------------------------
struct HistOut {
  unsigned long long *cnt, *wq, *kmn, *kmx, *akmn, *akmx;
};

template <bool WEIGHTED, bool WITH_ALL>
__global__ void __launch_bounds__(QT) qhist_kernel(QArgs a, const double* aprm, double wscale, HistOut o) {
  __shared__ unsigned int lcnt[QNB];
  __shared__ unsigned long long lwq[WEIGHTED ? QNB : 1];
  __shared__ unsigned long long lmn[QNB], lmx[QNB];
  __shared__ unsigned long long lamn[WITH_ALL ? QNB : 1], lamx[WITH_ALL ? QNB : 1];
  __shared__ WinLDS W;
  const int c = col_of(a), tid = threadIdx.x;
  for (int i = tid; i < QNB; i += QT) {
    lcnt[i] = 0u; lmn[i] = ~0ull; lmx[i] = 0ull;
    if (WEIGHTED) lwq[i] = 0ull;
    if (WITH_ALL) { lamn[i] = ~0ull; lamx[i] = 0ull; }
  }
  load_windows(W, a, c);
  __syncthreads();
  const double alo = WITH_ALL ? aprm[c * 2 + 0] : 0.0, asc = WITH_ALL ? aprm[c * 2 + 1] : 0.0;
  const long r0 = (long)blockIdx.y * a.rows_per_block;
  const long r1 = min(a.n, r0 + a.rows_per_block);
  const double* col = a.vals + (long)c * a.ldv;
  for_rows<4>(col, r0, r1, QT, [&](long r, double raw) {
    const double v = clean(raw, a.num_thr);
    if (!isfinite(v)) return;
    const unsigned long long k = okey(v);
    if (WITH_ALL) {
      const int ab = bucket_of(v, alo, asc);
      if (!covers_min(&lamn[ab], k)) atomicMin(&lamn[ab], k);
      if (!covers_max(&lamx[ab], k)) atomicMax(&lamx[ab], k);
    }
    if (!selected(a.sel, r)) return;
    const int b = win_bucket(W, v, k);
    if (b < 0) return;
    atomicAdd(&lcnt[b], 1u);
    if (!covers_min(&lmn[b], k)) atomicMin(&lmn[b], k);
    if (!covers_max(&lmx[b], k)) atomicMax(&lmx[b], k);
    if (WEIGHTED) {
      const double q = fmax(a.w[r], 0.0) * wscale;
      atomicAdd(&lwq[b], (unsigned long long)__double2ll_rn(q));
    }
  });

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
template <bool WEIGHTED, bool TWO_PHASE>
__global__ void __launch_bounds__(QT) qgather_kernel(QArgs a, double wscale, const int* slot, const long* sbase,
                                                    unsigned int* scur, double* gv, unsigned long long* gq) {
  __shared__ int lslot[QNB];
  __shared__ unsigned int lc[TWO_PHASE ? QNB : 1], lb[TWO_PHASE ? QNB : 1];
  __shared__ WinLDS W;
  const int c = col_of(a), tid = threadIdx.x;
  for (int i = tid; i < QNB; i += QT) {
    lslot[i] = slot[(long)c * QNB + i];
    if (TWO_PHASE) lc[i] = 0u;
  }
  load_windows(W, a, c);
  __syncthreads();
  const long r0 = (long)blockIdx.y * a.rows_per_block;
  const long r1 = min(a.n, r0 + a.rows_per_block);
  const double* col = a.vals + (long)c * a.ldv;
  if (!TWO_PHASE) {
    // few gathered values (refined buckets): one sweep, a global cursor atomic per value
    for_rows<4>(col, r0, r1, QT, [&](long r, double raw) {
      const double v = clean(raw, a.num_thr);
      if (!isfinite(v) || !selected(a.sel, r)) return;
      const int b = win_bucket(W, v, okey(v));
      const int s = b < 0 ? -1 : lslot[b];
      if (s < 0) return;
      const long at = sbase[s] + (long)atomicAdd(&scur[s], 1u);
      gv[at] = v;
      if (WEIGHTED) gq[at] = (unsigned long long)__double2ll_rn(fmax(a.w[r], 0.0) * wscale);
    });
    return;
  }
  // many gathered values: LDS counts, one global reservation per (block, bucket), then place
  for_rows<4>(col, r0, r1, QT, [&](long r, double raw) {
    const double v = clean(raw, a.num_thr);
    if (!isfinite(v) || !selected(a.sel, r)) return;
    const int b = win_bucket(W, v, okey(v));
    if (b >= 0 && lslot[b] >= 0) atomicAdd(&lc[b], 1u);
  });
  __syncthreads();
  for (int i = tid; i < QNB; i += QT) {
    if (lc[i]) lb[i] = atomicAdd(&scur[lslot[i]], lc[i]);
    lc[i] = 0u;
  }
  __syncthreads();
  for_rows<4>(col, r0, r1, QT, [&](long r, double raw) {
    const double v = clean(raw, a.num_thr);
    if (!isfinite(v) || !selected(a.sel, r)) return;
    const int b = win_bucket(W, v, okey(v));
    const int s = b < 0 ? -1 : lslot[b];
    if (s < 0) return;
    const long at = sbase[s] + (long)lb[b] + (long)atomicAdd(&lc[b], 1u);
    gv[at] = v;
    if (WEIGHTED) gq[at] = (unsigned long long)__double2ll_rn(fmax(a.w[r], 0.0) * wscale);
  });
}

// selection / class bitmask: bit r of word r/32 = (mode 1: y > 0.5, mode 2: !(y > 0.5)), one wave
// ballot per 64 rows
__global__ void __launch_bounds__(256) pack_bits_kernel(const float* __restrict__ y, long n, int mode,
                                                        unsigned int* __restrict__ out) {
  const long r = (long)blockIdx.x * 256 + threadIdx.x;
  const bool in = r < n;
  bool b = false;
  if (in) { const bool p = y[r] > 0.5f; b = mode == 2 ? !p : p; }
  const unsigned long long m = __ballot(b);
  const int lane = threadIdx.x & 63;
  const long w0 = (r - lane) >> 5;                 // first word of this wave's 64 rows
  if (lane == 0 && (r - lane) < n) out[w0] = (unsigned int)m;
  if (lane == 32 && r < n + 32 && (r - lane + 32) < n) out[w0 + 1] = (unsigned int)(m >> 32);
}

int grid_chunks(long n, int C) {
  // >= 8 blocks per CU over the batch, >= 16K rows per block (bounds the per-block flush)
  long by_rows = (n + 16383) / 16384;
  long want = (2048 + C - 1) / C;
  long ch = by_rows < want ? by_rows : want;
  return (int)(ch < 1 ? 1 : ch);
}

}  // namespace

SHIFU_API int shifu_pack_bits(const float* y, long n, int mode, unsigned int* out, hipStream_t stream) {
  if (n <= 0) return 0;
  if (mode != 1 && mode != 2) return -1;
  hipLaunchKernelGGL(pack_bits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, y, n, mode, out);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_qprep(const double* vals, long ldv, long n, int C, const unsigned int* y, int sel_mode, double num_thr,
                          void* mm, void* scnt, void* hll, double* mom, hipStream_t stream) {
  if (n <= 0 || C <= 0) return 0;
  if (ldv < n || (sel_mode != 0 && !y)) return -1;
  const int ch = grid_chunks(n, C);
  QArgs a{vals, ldv, n, C, y, nullptr, sel_mode, num_thr, (n + ch - 1) / ch, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(qprep_kernel, dim3(C, ch), dim3(QT), 0, stream, a, (unsigned long long*)mm,
                     (unsigned long long*)scnt, (unsigned int*)hll, mom);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// windows: wptr [C+1] (every column's range must hold <= MAXW windows), wins [wptr[C]] QWin
static int check_windows(const int* colmap, int ncols, int C) {
  return (!colmap && ncols != C) ? -1 : 0;
}

SHIFU_API int shifu_qhist(const double* vals, long ldv, long n, int C, const unsigned int* y, const double* w, int sel_mode,
                          double num_thr, const int* colmap, int ncols, const int* wptr, const void* wins,
                          const double* aprm, double wscale, int with_all, void* cnt, void* wq, void* kmn, void* kmx,
                          void* akmn, void* akmx, hipStream_t stream) {
  if (n <= 0 || C <= 0 || ncols <= 0) return 0;
  if (ldv < n || (sel_mode != 0 && !y) || (wq && !w) || (with_all && (!akmn || !akmx || !aprm)) || !wptr || !wins)
    return -1;
  if (check_windows(colmap, ncols, C)) return -1;
  const int ch = grid_chunks(n, ncols);
  QArgs a{vals, ldv, n, C, y, w, sel_mode, num_thr, (n + ch - 1) / ch, colmap, wptr, (const QWin*)wins};
  HistOut o{(unsigned long long*)cnt, (unsigned long long*)wq, (unsigned long long*)kmn, (unsigned long long*)kmx,
            (unsigned long long*)akmn, (unsigned long long*)akmx};
  dim3 g(ncols, ch), b(QT);
  if (wq) {
    if (with_all) hipLaunchKernelGGL((qhist_kernel<true, true>), g, b, 0, stream, a, aprm, wscale, o);
    else hipLaunchKernelGGL((qhist_kernel<true, false>), g, b, 0, stream, a, aprm, wscale, o);
  } else {
    if (with_all) hipLaunchKernelGGL((qhist_kernel<false, true>), g, b, 0, stream, a, aprm, wscale, o);
    else hipLaunchKernelGGL((qhist_kernel<false, false>), g, b, 0, stream, a, aprm, wscale, o);
  }
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_qgather(const double* vals, long ldv, long n, int C, const unsigned int* y, const double* w, int sel_mode,
                            double num_thr, const int* colmap, int ncols, const int* wptr, const void* wins,
                            double wscale, const int* slot, const long* sbase, void* scur, double* gv, void* gq,
                            int two_phase, hipStream_t stream) {
  if (n <= 0 || C <= 0 || ncols <= 0) return 0;
  if (ldv < n || (sel_mode != 0 && !y) || (gq && !w) || !wptr || !wins) return -1;
  if (check_windows(colmap, ncols, C)) return -1;
  const int ch = grid_chunks(n, ncols);
  QArgs a{vals, ldv, n, C, y, w, sel_mode, num_thr, (n + ch - 1) / ch, colmap, wptr, (const QWin*)wins};
  dim3 g(ncols, ch), b(QT);
  unsigned long long* q = (unsigned long long*)gq;
  unsigned int* cur = (unsigned int*)scur;
  if (gq) {
    if (two_phase) hipLaunchKernelGGL((qgather_kernel<true, true>), g, b, 0, stream, a, wscale, slot, sbase, cur, gv, q);
    else hipLaunchKernelGGL((qgather_kernel<true, false>), g, b, 0, stream, a, wscale, slot, sbase, cur, gv, q);
  } else {
    if (two_phase) hipLaunchKernelGGL((qgather_kernel<false, true>), g, b, 0, stream, a, wscale, slot, sbase, cur, gv, q);
    else hipLaunchKernelGGL((qgather_kernel<false, false>), g, b, 0, stream, a, wscale, slot, sbase, cur, gv, q);
  }
  CHECK_HIP(hipGetLastError());
  return 0;
}
