// Column statistics / normalization / LR / sensitivity kernels for MI355X (gfx950).
//
// Replaces the reference's per-row Java loops:
//   K1+K2  bin index + per-column moments and pos/neg histograms
//          UpdateBinningInfoMapper.populateStats  J/core/binning/UpdateBinningInfoMapper.java:427-615
//          UpdateBinningInfoReducer.reduce         J/core/binning/UpdateBinningInfoReducer.java:125-433
//   K5     normalization (z-score clip / WOE / pos-rate / discrete / index)
//          Normalizer.normalize / zScoreNormalize / woeNormalize  J/core/Normalizer.java:233-785
//   K1'    tree bin codes (CleanedData)         DTWorker.getBinIndex J/core/dtrain/dt/DTWorker.java:1001-1034
//   K9     logistic-regression gradient         LogisticRegressionWorker.doCompute :302-352
//   K14    sensitivity analysis (1 hidden layer) VarSelectMapper.map J/core/varselect/VarSelectMapper.java:277-333
//          with CacheFlatNetwork's first-layer cache (S - x_i * W1[:, i])
//
// Design notes:
//   * column-major raw values [F][ldv] fp64 (one column = one contiguous stream, exact double
//     comparisons against double bin boundaries, same as the Java code); boundaries are staged in
//     LDS per block and searched branch-free.
//   * histograms: LDS-privatised integer counters (ds_add_u32 for counts, ds_add_u64 for fixed-
//     point weights - integer LDS atomics are ~17x faster than ds_add_f32 on gfx950, see
//     profiles/microbench_lds_atomics.txt) flushed once per block; moments are fp64 wave/block
//     reductions written as per-block partials (no contended global atomics).
//   * normalize / bin-codes transpose column-major input to row-major output through a 64x64
//     LDS tile so both the loads and the stores are coalesced.
//   * LR: one fused pass over the row-major shard - dot, sigmoid, gradient accumulation in
//     registers (lane-strided vector loads), block partials reduced on the device.
#include "common.h"

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

namespace {

constexpr int MAXB = 1024;          // max boundaries per column staged in LDS

__device__ __forceinline__ int bin_search(const double* __restrict__ b, int nb, double v) {
  // number of boundaries <= v, minus one (b[0] = -inf); clipped to [0, nb-1]
  int lo = 0, hi = nb;                       // invariant: b[lo-1] <= v < b[hi]
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (b[mid] <= v) lo = mid + 1; else hi = mid;
  }
  int idx = lo - 1;
  return idx < 0 ? 0 : (idx > nb - 1 ? nb - 1 : idx);
}

// ---------------------------------------------------------------------------------------------
// K1+K2: per-column moments + pos/neg histograms
// ---------------------------------------------------------------------------------------------
struct StatsArgs {
  const double* vals; long ldv;
  const float* y; const double* w; long n;
  const double* bounds; const int* boff;
  int binary; double wscale; double num_thr;
  unsigned long long* hist; int hstride;     // [F][hstride][4]: cpos, cneg, wpos, wneg (fixed point)
  double* part; int nchunks; long rows_per_chunk;   // [F][nchunks][8]
  int unit_w;                                // every weight is 1: weight sums = counts
  const unsigned int* posbits;               // binary: bit r = (y[r] > 0.5), packed (1 bit per row)
  int max_nb;                                // max boundaries over the batch (sizes the LDS carve)
  int priv;                                  // per-thread private counters (unit_w, few bins)
};

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (unsigned long long)__shfl_xor((long long)v, o, 64);
  return v;
}

// Grid: x = column (fastest, so the blocks resident together read the same rows of y and w from
// L2), y = row chunk.  With few bins (the usual maxNumBin 10-30) and unit weights, every thread
// counts into its own LDS column ([key][thread], conflict-free, no atomics) and the block reduces
// the columns at the end; otherwise LDS atomics (u32 counts, u64 fixed-point weights).
constexpr int PRIV_KEYS = 48;                 // 2 * (bins + missing) <= 48 -> private counters

// dynamic LDS carve (bytes), shared by host and device
__host__ __device__ inline long cs_lds_bytes(int max_nb, int priv, int unit_w) {
  const long m1 = max_nb + 1;
  long b = (long)max_nb * 8 + 2 * m1 * 4;      // bounds, cp, cn
  b = (b + 15) & ~15L;
  if (priv) b += 2 * m1 * 256 * 4;            // [2 (nb+1)][256] u32
  else if (!unit_w) b += 2 * m1 * 8;          // wp, wn
  return b;
}

__global__ void __launch_bounds__(256) column_stats_kernel(StatsArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ double red[4][8];
  const long m1 = a.max_nb + 1;
  double* sb = (double*)smem;
  unsigned int* cp = (unsigned int*)(sb + a.max_nb);
  unsigned int* cn = cp + m1;
  unsigned char* tail = smem + ((((long)a.max_nb * 8 + 2 * m1 * 4) + 15) & ~15L);
  unsigned int* priv = (unsigned int*)tail;                       // [2 m1][256]
  unsigned long long* wp = (unsigned long long*)tail;             // [m1]
  unsigned long long* wn = wp + m1;
  const int f = blockIdx.x, chunk = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int b0 = a.boff[f], nb = a.boff[f + 1] - b0;
  const bool private_cnt = a.priv;
  for (int i = tid; i < nb; i += 256) sb[i] = a.bounds[b0 + i];
  for (int i = tid; i <= nb; i += 256) {
    cp[i] = 0; cn[i] = 0;
    if (!private_cnt && !a.unit_w) { wp[i] = 0ull; wn[i] = 0ull; }
  }
  if (private_cnt)
    for (int k = 0; k < 2 * (nb + 1); ++k) priv[k * 256 + tid] = 0u;
  __syncthreads();
  const long r0 = (long)chunk * a.rows_per_chunk;
  const long r1 = min(a.n, r0 + a.rows_per_chunk);
  const double* col = a.vals + (long)f * a.ldv;
  double cnt = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, mn = INFINITY, mx = -INFINITY;
  for_rows<4>(col, r0, r1, 256, [&](long r, double v) {
    if (v > a.num_thr) v = NAN;               // numericalValueThreshold -> invalid
    int bin;
    if (v != v) {
      bin = nb;                               // missing bin
    } else {
      bin = bin_search(sb, nb, v);
      if (isfinite(v)) {
        const double v2 = v * v;
        cnt += 1.0; s1 += v; s2 += v2; s3 += v2 * v; s4 += v2 * v2;
        mn = fmin(mn, v); mx = fmax(mx, v);
      }
    }
    const bool pos = !a.binary || ((a.posbits[r >> 5] >> (r & 31)) & 1u);
    if (private_cnt) {
      priv[(bin * 2 + (pos ? 1 : 0)) * 256 + tid] += 1u;
    } else if (a.unit_w) {
      atomicAdd(pos ? &cp[bin] : &cn[bin], 1u);
    } else {
      const unsigned long long q = (unsigned long long)__double2ll_rn(a.w[r] * a.wscale);
      if (pos) { atomicAdd(&cp[bin], 1u); atomicAdd(&wp[bin], q); }
      else     { atomicAdd(&cn[bin], 1u); atomicAdd(&wn[bin], q); }
    }
  });
  if (private_cnt) {                          // one wave per key: sum the 256 thread columns
    __syncthreads();
    const int wid = tid >> 6;
    for (int k = wid; k < 2 * (nb + 1); k += 4) {
      const unsigned int* pk = priv + k * 256;
      unsigned int t = pk[lane] + pk[lane + 64] + pk[lane + 128] + pk[lane + 192];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
      if (lane == 0) { if (k & 1) cp[k >> 1] = t; else cn[k >> 1] = t; }
    }
  }
  // moments: wave then block reduction
  cnt = wave_sum_d(cnt); s1 = wave_sum_d(s1); s2 = wave_sum_d(s2); s3 = wave_sum_d(s3); s4 = wave_sum_d(s4);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fmin(mn, __shfl_xor(mn, o, 64));
    mx = fmax(mx, __shfl_xor(mx, o, 64));
  }
  const int wid = tid >> 6;
  __syncthreads();
  if (lane == 0) {
    red[wid][0] = cnt; red[wid][1] = s1; red[wid][2] = s2; red[wid][3] = s3; red[wid][4] = s4;
    red[wid][5] = mn; red[wid][6] = mx;
  }
  __syncthreads();
  if (tid < 8) {
    double acc = red[0][tid];
    for (int k = 1; k < 4; ++k) {
      const double v = red[k][tid];
      acc = tid == 5 ? fmin(acc, v) : (tid == 6 ? fmax(acc, v) : acc + v);
    }
    if (tid == 7) acc = 0.0;
    a.part[((long)f * a.nchunks + chunk) * 8 + tid] = acc;
  }
  unsigned long long* h = a.hist + (long)f * a.hstride * 4;
  const unsigned long long unit_q = (unsigned long long)__double2ll_rn(a.wscale);
  for (int i = tid; i <= nb; i += 256) {
    const unsigned long long wpi = a.unit_w ? (unsigned long long)cp[i] * unit_q : wp[i];
    const unsigned long long wni = a.unit_w ? (unsigned long long)cn[i] * unit_q : wn[i];
    if (cp[i]) atomicAdd(&h[i * 4 + 0], (unsigned long long)cp[i]);
    if (cn[i]) atomicAdd(&h[i * 4 + 1], (unsigned long long)cn[i]);
    if (wpi) atomicAdd(&h[i * 4 + 2], wpi);
    if (wni) atomicAdd(&h[i * 4 + 3], wni);
  }
}

// ---------------------------------------------------------------------------------------------
// K5: normalization, column-major fp64 in -> row-major fp32 out (LDS-tiled transpose)
// ---------------------------------------------------------------------------------------------
enum NormMode : int { NM_ZSCORE = 0, NM_NUM_TABLE = 1, NM_CAT_TABLE = 2, NM_RAW = 3, NM_DISCRETE = 4,
                      NM_CAT_INDEX = 5 };

struct NormArgs {
  const double* vals; long ldv; long n; int F;
  const int* ip;        // [F][8]: mode, out_col, bnd_off, nbnd, tbl_off, ntbl, zflag, 0
  const double* dp;     // [F][8]: mean, std, cutoff, zmean, zstd, 0, 0, 0
  const double* bounds; const double* tables;
  float* out; long ldo;
};

__device__ __forceinline__ double zclip(double v, double mean, double std, double cutoff) {
  v = fmin(v, mean + cutoff * std);
  v = fmax(v, mean - cutoff * std);
  return std > 0.00001 ? (v - mean) / std : 0.0;
}

__global__ void __launch_bounds__(256) normalize_kernel(NormArgs a) {
  __shared__ float tile[64][65];
  const long r0 = (long)blockIdx.x * 64;
  const int f0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
  for (int k = ty; k < 64; k += 4) {
    const int f = f0 + k;
    const long r = r0 + tx;
    float res = 0.f;
    if (f < a.F && r < a.n) {
      const int* ip = a.ip + f * 8;
      const double* dp = a.dp + f * 8;
      const double v = a.vals[(long)f * a.ldv + r];
      const int mode = ip[0], nbnd = ip[3], ntbl = ip[5];
      const double* bnd = a.bounds + ip[2];
      const double* tbl = a.tables + ip[4];
      double o;
      switch (mode) {
        case NM_ZSCORE: o = zclip(isfinite(v) ? v : dp[0], dp[0], dp[1], dp[2]); break;
        case NM_NUM_TABLE: {
          int bin = (v != v) ? -1 : bin_search(bnd, nbnd, v);
          double t = tbl[bin < 0 ? ntbl - 1 : min(bin, ntbl - 1)];
          o = ip[6] ? zclip(t, dp[3], dp[4], dp[2]) : t;
          break;
        }
        case NM_CAT_TABLE: {
          int idx = (v != v || v < 0) ? -1 : (int)v;
          double t = tbl[(idx < 0 || idx >= ntbl) ? ntbl - 1 : idx];
          o = ip[6] ? zclip(t, dp[3], dp[4], dp[2]) : t;
          break;
        }
        case NM_RAW: o = isfinite(v) ? v : dp[0]; break;
        case NM_DISCRETE: {
          int bin = (v != v) ? -1 : bin_search(bnd, nbnd, v);
          double lo = (bin < 0 || bin >= ntbl) ? dp[0] : tbl[bin];
          o = zclip(lo, dp[0], dp[1], dp[2]);
          break;
        }
        default: {   // NM_CAT_INDEX
          int idx = (v != v || v < 0) ? -1 : (int)v;
          o = (double)(idx < 0 ? ntbl : idx);
        }
      }
      res = (float)o;
    }
    tile[k][tx] = res;
  }
  __syncthreads();
  // store: thread (tx = column in tile, ty = row group) -> out[r][out_col]
  for (int k = ty; k < 64; k += 4) {
    const long r = r0 + k;
    const int f = f0 + tx;
    if (r < a.n && f < a.F) a.out[r * a.ldo + a.ip[f * 8 + 1]] = tile[tx][k];
  }
}

// ---------------------------------------------------------------------------------------------
// K1': tree bin codes (CleanedData): numeric missing -> bin of 0.0, categorical missing -> ncat
// ---------------------------------------------------------------------------------------------
struct CodeArgs {
  const double* vals; long ldv; long n; int F;
  const int* ip;        // [F][4]: is_cat, bnd_off, nbnd, ncat
  const double* bounds;
  uint8_t* out; long ldo;
};

__global__ void __launch_bounds__(256) bin_codes_kernel(CodeArgs a) {
  __shared__ uint8_t tile[64][68];
  const long r0 = (long)blockIdx.x * 64;
  const int f0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int k = ty; k < 64; k += 4) {
    const int f = f0 + k;
    const long r = r0 + tx;
    uint8_t c = 0;
    if (f < a.F && r < a.n) {
      const int* ip = a.ip + f * 4;
      double v = a.vals[(long)f * a.ldv + r];
      if (ip[0]) {
        int idx = (v != v || v < 0) ? -1 : (int)v;
        c = (uint8_t)((idx < 0 || idx >= ip[3]) ? ip[3] : idx);
      } else {
        if (v != v) v = 0.0;                 // DTWorker.getFloatValue: missing -> 0f
        c = (uint8_t)bin_search(a.bounds + ip[1], ip[2], v);
      }
    }
    tile[k][tx] = c;
  }
  __syncthreads();
  for (int k = ty; k < 64; k += 4) {
    const long r = r0 + k;
    const int f = f0 + tx;
    if (r < a.n && f < a.F) a.out[r * a.ldo + f] = tile[tx][k];
  }
}

// ---------------------------------------------------------------------------------------------
// K5 fused (streamed `norm`): one read of a chunk's raw values -> every NormalizedData /
// CleanedData output of the chunk in the same pass: fp32 rows (the NormalizedData cache),
// bf16 GEMM-ready rows (the MLP's padded layout: the caller's buffer holds the bias column and
// the zero padding, the kernel fills the value columns) and uint8 tree codes.  Column-major fp64
// in, row-major out through one LDS transpose tile per output; each output is optional.
// ---------------------------------------------------------------------------------------------
struct NormCodesArgs {
  const double* vals; long ldv; long n; int F;
  const int* ip; const double* dp; const double* bounds; const double* tables;   // as NormArgs
  const int* cip; const double* cbounds;   // codes: [F][4] is_cat, bnd_off, nbnd, ncat (nullable)
  float* outf; long ldf;                   // [n][ldf] fp32 at out_col (nullable)
  bf16_t* outb; long ldb;                  // [n][ldb] bf16 at out_col (nullable)
  uint8_t* codes; long ldc;                // [n][ldc] uint8 at column f (nullable)
};

__device__ __forceinline__ double norm_value(const int* ip, const double* dp, const double* bounds,
                                             const double* tables, double v) {
  const int mode = ip[0], nbnd = ip[3], ntbl = ip[5];
  const double* bnd = bounds + ip[2];
  const double* tbl = tables + ip[4];
  switch (mode) {
    case NM_ZSCORE: return zclip(isfinite(v) ? v : dp[0], dp[0], dp[1], dp[2]);
    case NM_NUM_TABLE: {
      const int bin = (v != v) ? -1 : bin_search(bnd, nbnd, v);
      const double t = tbl[bin < 0 ? ntbl - 1 : min(bin, ntbl - 1)];
      return ip[6] ? zclip(t, dp[3], dp[4], dp[2]) : t;
    }
    case NM_CAT_TABLE: {
      const int idx = (v != v || v < 0) ? -1 : (int)v;
      const double t = tbl[(idx < 0 || idx >= ntbl) ? ntbl - 1 : idx];
      return ip[6] ? zclip(t, dp[3], dp[4], dp[2]) : t;
    }
    case NM_RAW: return isfinite(v) ? v : dp[0];
    case NM_DISCRETE: {
      const int bin = (v != v) ? -1 : bin_search(bnd, nbnd, v);
      const double lo = (bin < 0 || bin >= ntbl) ? dp[0] : tbl[bin];
      return zclip(lo, dp[0], dp[1], dp[2]);
    }
    default: {
      const int idx = (v != v || v < 0) ? -1 : (int)v;
      return (double)(idx < 0 ? ntbl : idx);
    }
  }
}

__global__ void __launch_bounds__(256) norm_codes_kernel(NormCodesArgs a) {
  __shared__ float tile[64][65];
  __shared__ uint8_t ctile[64][68];
  const long r0 = (long)blockIdx.x * 64;
  const int f0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
  for (int k = ty; k < 64; k += 4) {
    const int f = f0 + k;
    const long r = r0 + tx;
    float res = 0.f;
    uint8_t c = 0;
    if (f < a.F && r < a.n) {
      double v = a.vals[(long)f * a.ldv + r];          // coalesced: consecutive rows of column f
      if (a.outf || a.outb) res = (float)norm_value(a.ip + f * 8, a.dp + f * 8, a.bounds, a.tables, v);
      if (a.codes) {
        const int* cp = a.cip + f * 4;
        if (cp[0]) {
          const int idx = (v != v || v < 0) ? -1 : (int)v;
          c = (uint8_t)((idx < 0 || idx >= cp[3]) ? cp[3] : idx);
        } else {
          if (v != v) v = 0.0;                         // DTWorker.getFloatValue: missing -> 0f
          c = (uint8_t)bin_search(a.cbounds + cp[1], cp[2], v);
        }
      }
    }
    tile[k][tx] = res;
    ctile[k][tx] = c;
  }
  __syncthreads();
  for (int k = ty; k < 64; k += 4) {                   // thread (tx = column, ty = row group)
    const long r = r0 + k;
    const int f = f0 + tx;
    if (r >= a.n || f >= a.F) continue;
    if (a.outf || a.outb) {                          // a codes-only launch has no ip table
      const int oc = a.ip[f * 8 + 1];
      if (a.outf) a.outf[r * a.ldf + oc] = tile[tx][k];
      if (a.outb) a.outb[r * a.ldb + oc] = f2bf(tile[tx][k]);
    }
    if (a.codes) a.codes[r * a.ldc + f] = ctile[tx][k];
  }
}

// ---------------------------------------------------------------------------------------------
// K9: logistic regression fused gradient (one pass over X)
// ---------------------------------------------------------------------------------------------
template <typename T> struct Vec;
template <> struct Vec<float> { static constexpr int N = 4; };
template <> struct Vec<bf16_t> { static constexpr int N = 8; };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* o);
template <>
__device__ __forceinline__ void load_vec<float>(const float* p, float* o) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
__device__ __forceinline__ void load_vec<bf16_t>(const bf16_t* p, float* o) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { o[2 * i] = __uint_as_float(u[i] << 16); o[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u); }
}

struct LrArgs {
  const void* x; long ldx; long n; int F;
  const float* w; const float* y; const float* s;
  float* part; double* err_part;   // [nblk][F+1], [nblk]
};

template <typename T, int NK>
__global__ void __launch_bounds__(256) lr_grad_kernel(LrArgs a) {
  constexpr int V = Vec<T>::N;
  __shared__ float red[4][NK * 64 * V + 1];
  __shared__ double ered[4];
  const T* X = reinterpret_cast<const T*>(a.x);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float wv[NK][V], g[NK][V];
#pragma unroll
  for (int i = 0; i < NK; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (i * 64 + lane) * V + j;
      wv[i][j] = c < a.F ? a.w[c] : 0.f;
      g[i][j] = 0.f;
    }
  const float bias = a.w[a.F];
  float gb = 0.f;
  double err = 0.0;
  const long wave_id = (long)blockIdx.x * 4 + wid, nwaves = (long)gridDim.x * 4;
  for (long r = wave_id; r < a.n; r += nwaves) {
    float xv[NK][V];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int c0 = (i * 64 + lane) * V;
      if (c0 + V <= a.ldx) load_vec<T>(X + r * a.ldx + c0, xv[i]);
      else {
#pragma unroll
        for (int j = 0; j < V; ++j) xv[i][j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if (c0 + j >= a.F) xv[i][j] = 0.f;
        dot += xv[i][j] * wv[i][j];
      }
    }
    dot = wave_sum(dot);
    const float p = 1.f / (1.f + __expf(-(dot + bias)));
    const float e = a.y[r] - p;
    const float d = e * (p * (1.f - p) + 0.1f) * (a.s ? a.s[r] : 1.f);
#pragma unroll
    for (int i = 0; i < NK; ++i)
#pragma unroll
      for (int j = 0; j < V; ++j) g[i][j] += d * xv[i][j];
    gb += d;
    err += (double)e * e;
  }
#pragma unroll
  for (int i = 0; i < NK; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) red[wid][(i * 64 + lane) * V + j] = g[i][j];
  if (lane == 0) { red[wid][NK * 64 * V] = gb; ered[wid] = err; }
  __syncthreads();
  float* out = a.part + (long)blockIdx.x * (a.F + 1);
  for (int c = tid; c < a.F; c += 256) out[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  if (tid == 0) {
    const int B = NK * 64 * V;
    out[a.F] = red[0][B] + red[1][B] + red[2][B] + red[3][B];
    a.err_part[blockIdx.x] = ered[0] + ered[1] + ered[2] + ered[3];
  }
}

// ---------------------------------------------------------------------------------------------
// K14: sensitivity, 1-hidden-layer network: per (row, input f)
//   d = base[r] - act_o(b2 + sum_j W2[j] * act1(S[r][j] - x[r][f] * W1t[f][j]))
//   accumulate sum |d|, sum d^2 per input
// ---------------------------------------------------------------------------------------------
constexpr int SIPT = 8;    // inputs per thread (16 measured within 1%: 9.12 vs 9.02e9 pairs/s, 148 vs 92 VGPRs)
constexpr int SFT = 4 * SIPT;   // inputs per block (4 thread groups)
constexpr int SRT = 64;    // rows per tile (one per thread group member)
constexpr int SHC = 64;    // hidden units staged per chunk

struct SensArgs {
  const float* S; long lds; const float* X; long ldx; const float* W1t; const float* W2; float b2;
  const float* base; long n; int F; int H; int act_o;
  long rows_per_chunk; double* acc;   // [F][2]
};

// Register-blocked: thread = 1 row x SIPT inputs; per hidden unit j it reads S[r][j] (4 j per
// ds_read_b128 from the row's LDS strip) and W1[j][SIPT inputs] (SIPT/4 x ds_read_b128, same address for
// the 64 row-threads of a group -> broadcast), then SIPT x (fma, act, fma).  The activation's
// v_exp/v_rcp (quarter rate) bound the loop instead of scalar LDS reads (the previous 1x1
// version issued two ds_read_b32 per element).
template <int ACT1>
__global__ void __launch_bounds__(256) sensitivity_kernel(SensArgs a) {
  __shared__ __attribute__((aligned(16))) float st[SRT][SHC + 4];   // S strip per row
  __shared__ __attribute__((aligned(16))) float w1[SHC][SFT];       // W1 chunk, inputs contiguous
  __shared__ float w2s[SHC];
  __shared__ double red[4][2][SFT];
  const int tid = threadIdx.x, fg = tid & 3, rr = tid >> 2;
  const int f0 = blockIdx.y * SFT, fb = f0 + fg * SIPT;
  const long r0 = (long)blockIdx.x * a.rows_per_chunk, r1 = min(a.n, r0 + a.rows_per_chunk);
  double sa[SIPT], sq[SIPT];
#pragma unroll
  for (int k = 0; k < SIPT; ++k) { sa[k] = 0.0; sq[k] = 0.0; }
  for (long rb = r0; rb < r1; rb += SRT) {
    const long r = rb + rr;
    const bool rok = r < r1;
    float xv[SIPT], acc[SIPT];
#pragma unroll
    for (int k = 0; k < SIPT; ++k) {
      xv[k] = (rok && fb + k < a.F) ? a.X[r * a.ldx + fb + k] : 0.f;
      acc[k] = 0.f;
    }
    for (int h0 = 0; h0 < a.H; h0 += SHC) {
      const int hc = min(SHC, a.H - h0);
      __syncthreads();
      // sigmoid: the strips are staged pre-scaled by log2(e) (S as -S*log2e, W1 as W1*log2e), so
      // exp(-z) = exp2(x*W1' + S') is one packed FMA + v_exp_f32, and 1 + e and the w2-weighted
      // accumulation run as packed f32 pairs: fma, mul, add per element drop to half-rate pairs
      constexpr bool SIG = ACT1 == ACT_SIGMOID;
      const float sc = SIG ? -1.4426950408889634f : 1.f, wsc = SIG ? 1.4426950408889634f : 1.f;
      for (int i = tid; i < SRT * SHC; i += 256) {
        const int row = i / SHC, j = i % SHC;
        st[row][j] = (rb + row < r1 && j < hc) ? sc * a.S[(rb + row) * a.lds + h0 + j] : 0.f;
      }
      for (int i = tid; i < SFT * SHC; i += 256) {
        const int ff = i / SHC, j = i % SHC;
        w1[j][ff] = (f0 + ff < a.F && j < hc) ? wsc * a.W1t[(long)(f0 + ff) * a.H + h0 + j] : 0.f;
      }
      for (int j = tid; j < SHC; j += 256) w2s[j] = j < hc ? a.W2[h0 + j] : 0.f;
      __syncthreads();
      for (int j = 0; j < hc; j += 4) {
        const float4 s4 = *(const float4*)&st[rr][j];
        const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          float wv[SIPT];
#pragma unroll
          for (int q = 0; q < SIPT / 4; ++q) {
            const float4 w4 = *(const float4*)&w1[j + jj][fg * SIPT + 4 * q];
            wv[4 * q] = w4.x; wv[4 * q + 1] = w4.y; wv[4 * q + 2] = w4.z; wv[4 * q + 3] = w4.w;
          }
          const float w2j = w2s[j + jj];
          if constexpr (SIG) {
            // stage by stage over the SIPT inputs (independent chains between dependent ops: no
            // trans-result hazard nops)
            const f32x2_t s2 = {sv[jj], sv[jj]}, one = {1.f, 1.f}, w22 = {w2j, w2j};
            f32x2_t t[SIPT / 2];
#pragma unroll
            for (int q = 0; q < SIPT / 2; ++q)
              t[q] = __builtin_elementwise_fma(f32x2_t{xv[2 * q], xv[2 * q + 1]}, f32x2_t{wv[2 * q], wv[2 * q + 1]}, s2);
#pragma unroll
            for (int q = 0; q < SIPT / 2; ++q) t[q] = f32x2_t{__builtin_amdgcn_exp2f(t[q].x), __builtin_amdgcn_exp2f(t[q].y)};
#pragma unroll
            for (int q = 0; q < SIPT / 2; ++q) t[q] = t[q] + one;
#pragma unroll
            for (int q = 0; q < SIPT / 2; ++q) t[q] = f32x2_t{__builtin_amdgcn_rcpf(t[q].x), __builtin_amdgcn_rcpf(t[q].y)};
#pragma unroll
            for (int q = 0; q < SIPT / 2; ++q) {
              const f32x2_t a2 = __builtin_elementwise_fma(w22, t[q], f32x2_t{acc[2 * q], acc[2 * q + 1]});
              acc[2 * q] = a2.x;
              acc[2 * q + 1] = a2.y;
            }
          } else {
#pragma unroll
            for (int k = 0; k < SIPT; ++k) acc[k] += w2j * act_fwd(ACT1, sv[jj] - xv[k] * wv[k]);
          }
        }
      }
    }
    if (rok) {
      const float bse = a.base[r];
#pragma unroll
      for (int k = 0; k < SIPT; ++k) {
        const double d = (double)(bse - act_fwd(a.act_o, acc[k] + a.b2));
        sa[k] += fabs(d);
        sq[k] += d * d;
      }
    }
  }
  // reduce over the 64 rows of each input group: lanes l, l^4, l^8, ... share fg
#pragma unroll
  for (int k = 0; k < SIPT; ++k) {
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) { sa[k] += __shfl_xor(sa[k], o, 64); sq[k] += __shfl_xor(sq[k], o, 64); }
  }
  const int wv_ = tid >> 6, lane = tid & 63;
  if (lane < 4) {
#pragma unroll
    for (int k = 0; k < SIPT; ++k) { red[wv_][0][lane * SIPT + k] = sa[k]; red[wv_][1][lane * SIPT + k] = sq[k]; }
  }
  __syncthreads();
  if (tid < SFT && f0 + tid < a.F) {
    const double x = red[0][0][tid] + red[1][0][tid] + red[2][0][tid] + red[3][0][tid];
    const double y = red[0][1][tid] + red[1][1][tid] + red[2][1][tid] + red[3][1][tid];
    atomicAdd(&a.acc[(long)(f0 + tid) * 2], x);
    atomicAdd(&a.acc[(long)(f0 + tid) * 2 + 1], y);
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// C API
// ---------------------------------------------------------------------------------------------
SHIFU_API int shifu_column_stats(const double* vals, long ldv, const float* y, const double* w, long n, int F,
                                 const double* bounds, const int* boff, int max_nb, int binary, double wscale,
                                 double num_thr, void* hist, int hstride, double* part, int nchunks, int unit_w,
                                 const unsigned int* posbits, hipStream_t stream) {
  if (binary && !posbits) return -1;
  if (max_nb > MAXB || hstride < max_nb + 1 || nchunks <= 0 || nchunks > 65535 || F <= 0) return -1;
  const int priv = unit_w && 2 * (max_nb + 1) <= PRIV_KEYS;
  StatsArgs a{vals, ldv, y, w, n, bounds, boff, binary, wscale, num_thr, (unsigned long long*)hist, hstride,
              part, nchunks, (n + nchunks - 1) / nchunks, unit_w, posbits, max_nb, priv};
  const long lds = cs_lds_bytes(max_nb, priv, unit_w);
  if (lds > 150 * 1024) return -1;
  hipLaunchKernelGGL(column_stats_kernel, dim3(F, nchunks), dim3(256), (unsigned)lds, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_normalize(const double* vals, long ldv, long n, int F, const int* ip, const double* dp,
                              const double* bounds, const double* tables, float* out, long ldo, hipStream_t stream) {
  if (n <= 0 || F <= 0) return 0;
  NormArgs a{vals, ldv, n, F, ip, dp, bounds, tables, out, ldo};
  hipLaunchKernelGGL(normalize_kernel, dim3((n + 63) / 64, (F + 63) / 64), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_norm_codes(const double* vals, long ldv, long n, int F, const int* ip, const double* dp,
                               const double* bounds, const double* tables, const int* cip, const double* cbounds,
                               float* outf, long ldf, void* outb, long ldb, void* codes, long ldc,
                               hipStream_t stream) {
  if (n <= 0 || F <= 0) return 0;
  if ((outf || outb) && (!ip || !dp)) return -1;
  if (codes && (!cip || !cbounds || ldc < F)) return -1;
  NormCodesArgs a{vals, ldv, n, F, ip, dp, bounds, tables, cip, cbounds, outf, ldf, (bf16_t*)outb, ldb,
                  (uint8_t*)codes, ldc};
  hipLaunchKernelGGL(norm_codes_kernel, dim3((n + 63) / 64, (F + 63) / 64), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_bin_codes(const double* vals, long ldv, long n, int F, const int* ip, const double* bounds,
                              void* out, long ldo, hipStream_t stream) {
  if (n <= 0 || F <= 0) return 0;
  CodeArgs a{vals, ldv, n, F, ip, bounds, (uint8_t*)out, ldo};
  hipLaunchKernelGGL(bin_codes_kernel, dim3((n + 63) / 64, (F + 63) / 64), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

template <typename T>
static int lr_dispatch(int nk, dim3 g, hipStream_t s, const LrArgs& a) {
  switch (nk) {
    case 1: hipLaunchKernelGGL((lr_grad_kernel<T, 1>), g, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((lr_grad_kernel<T, 2>), g, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((lr_grad_kernel<T, 3>), g, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((lr_grad_kernel<T, 4>), g, dim3(256), 0, s, a); break;
    case 5: hipLaunchKernelGGL((lr_grad_kernel<T, 5>), g, dim3(256), 0, s, a); break;
    case 6: hipLaunchKernelGGL((lr_grad_kernel<T, 6>), g, dim3(256), 0, s, a); break;
    case 7: hipLaunchKernelGGL((lr_grad_kernel<T, 7>), g, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL((lr_grad_kernel<T, 8>), g, dim3(256), 0, s, a); break;
    default: return -2;
  }
  return 0;
}

// dtype: 0 = fp32 rows (ldx % 4 == 0), 1 = bf16 rows (ldx % 8 == 0); F <= 2048 / 4096
SHIFU_API int shifu_lr_grad(const void* x, long ldx, long n, int F, int dtype, const float* w, const float* y,
                            const float* s, float* part, double* err_part, int nblk, hipStream_t stream) {
  const int V = dtype ? 8 : 4;
  if (ldx % V || F <= 0 || nblk <= 0) return -1;
  const int nk = (F + 64 * V - 1) / (64 * V);
  LrArgs a{x, ldx, n, F, w, y, s, part, err_part};
  int rc = dtype ? lr_dispatch<bf16_t>(nk, dim3(nblk), stream, a) : lr_dispatch<float>(nk, dim3(nblk), stream, a);
  if (rc) return rc;
  CHECK_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------------
// K14b: SE for deeper nets -- the perturbed first hidden layer of (row, input) pairs, written as
// bf16 MLP rows [R * fc][Hpad] (bias column H = 1, padding 0) so the remaining layers run as
// MFMA GEMMs: out[(r*fc + f)][j] = act(S[r][j] - x[r][f0+f] * W1[j][f0+f]).  One thread per 2
// hidden units (packed bf16x2 store); rows of the pair matrix are independent.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) se_perturb_kernel(const float* __restrict__ S, long lds,
                                                         const float* __restrict__ X, long ldx,
                                                         const float* __restrict__ W1t, int f0, int fc, int H,
                                                         int Hpad, int act, uint32_t* __restrict__ out, long R) {
  const long pair = (long)blockIdx.x;              // r * fc + f
  const long r = pair / fc;
  const int f = (int)(pair - r * fc);
  if (r >= R) return;
  const float xv = X[r * ldx + f0 + f];
  const float* srow = S + r * lds;
  const float* wrow = W1t + (long)(f0 + f) * H;
  uint32_t* orow = out + pair * (Hpad / 2);
  for (int j2 = threadIdx.x; j2 < Hpad / 2; j2 += blockDim.x) {
    float v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = 2 * j2 + u;
      v[u] = j < H ? act_fwd(act, srow[j] - xv * wrow[j]) : (j == H ? 1.f : 0.f);
    }
    orow[j2] = pack_bf16x2(v[0], v[1]);
  }
}

SHIFU_API int shifu_se_perturb(const float* S, long lds, const float* X, long ldx, const float* W1t, int f0, int fc,
                               int F, int H, int Hpad, int act, void* out, long R, hipStream_t stream) {
  if (R <= 0 || fc <= 0) return 0;
  if (Hpad % 2 || Hpad < H + 1 || f0 < 0 || f0 + fc > F || lds < H || ldx < F) return -1;
  hipLaunchKernelGGL(se_perturb_kernel, dim3((unsigned)(R * fc)), dim3(256), 0, stream, S, lds, X, ldx, W1t, f0, fc,
                     H, Hpad, act, (uint32_t*)out, R);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_sensitivity(const float* S, long lds, const float* X, long ldx, const float* W1t, const float* W2,
                                float b2, const float* base, long n, int F, int H, int act1, int act_o, int nchunks,
                                double* acc, hipStream_t stream) {
  if (H <= 0 || H > 1024 || n <= 0 || nchunks <= 0) return -1;
  long rpc = (n + nchunks - 1) / nchunks;
  rpc = (rpc + SRT - 1) / SRT * SRT;
  nchunks = (int)((n + rpc - 1) / rpc);
  SensArgs a{S, lds, X, ldx, W1t, W2, b2, base, n, F, H, act_o, rpc, acc};
  const size_t sm = 0;
  dim3 g(nchunks, (F + SFT - 1) / SFT);
  switch (act1) {
    case ACT_SIGMOID: hipLaunchKernelGGL(sensitivity_kernel<ACT_SIGMOID>, g, dim3(256), sm, stream, a); break;
    case ACT_TANH: hipLaunchKernelGGL(sensitivity_kernel<ACT_TANH>, g, dim3(256), sm, stream, a); break;
    case ACT_LINEAR: hipLaunchKernelGGL(sensitivity_kernel<ACT_LINEAR>, g, dim3(256), sm, stream, a); break;
    case ACT_RELU: hipLaunchKernelGGL(sensitivity_kernel<ACT_RELU>, g, dim3(256), sm, stream, a); break;
    case ACT_LEAKYRELU: hipLaunchKernelGGL(sensitivity_kernel<ACT_LEAKYRELU>, g, dim3(256), sm, stream, a); break;
    case ACT_SWISH: hipLaunchKernelGGL(sensitivity_kernel<ACT_SWISH>, g, dim3(256), sm, stream, a); break;
    case ACT_PTANH: hipLaunchKernelGGL(sensitivity_kernel<ACT_PTANH>, g, dim3(256), sm, stream, a); break;
    case ACT_LOG: hipLaunchKernelGGL(sensitivity_kernel<ACT_LOG>, g, dim3(256), sm, stream, a); break;
    case ACT_SIN: hipLaunchKernelGGL(sensitivity_kernel<ACT_SIN>, g, dim3(256), sm, stream, a); break;
    default: return -2;
  }
  CHECK_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------------
// K3: KS / IV / WOE per column (ColumnStatsCalculator.calculateColumnMetrics,
// J/core/ColumnStatsCalculator.java): one wave per (column, variant) -- variant 0 = bin counts,
// 1 = weighted bins -- over the bins in 64-lane chunks: totals, per-bin WOE
// ln((n_i + eps) / (p_i + eps)), IV = sum (n_i - p_i) * woe_i, KS = max |cum p - cum n| with the
// cumulative sums carried across chunks by a wave scan.  All columns of a stats pass in one
// launch (bins are variable-length: offsets).
// ---------------------------------------------------------------------------------------------
namespace {
struct MetricsArgs {
  const double* neg; const double* pos;   // [2][total_bins]: counts, then weighted
  const int* off; int F; long total;      // bins of column f: [off[f], off[f+1])
  double* out;                            // [F][2][4]: ks * 100, iv, woe, valid
  double* bin_woe;                        // [2][total_bins]
};

__global__ void __launch_bounds__(256) column_metrics_kernel(MetricsArgs a) {
  const int wv = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (wv >= 2 * a.F) return;
  const int f = wv >> 1, var = wv & 1;
  const double* ng = a.neg + var * a.total;
  const double* ps = a.pos + var * a.total;
  const int b0 = a.off[f], b1 = a.off[f + 1];
  double sn = 0.0, sp = 0.0;
  for (int b = b0 + lane; b < b1; b += 64) { sn += ng[b]; sp += ps[b]; }
  sn = wave_sum_d(sn);
  sp = wave_sum_d(sp);
  double* o = a.out + ((long)f * 2 + var) * 4;
  if (sn == 0.0 || sp == 0.0) {
    if (lane == 0) { o[0] = 0.0; o[1] = 0.0; o[2] = 0.0; o[3] = 0.0; }
    return;
  }
  const double EPS = 1e-10;
  double iv = 0.0, ks = 0.0, cp = 0.0, cn = 0.0;     // cp / cn: cumulative sums before this chunk
  for (int c0 = b0; c0 < b1; c0 += 64) {
    const int b = c0 + lane;
    const bool ok = b < b1;
    const double p = ok ? ps[b] / sp : 0.0, n = ok ? ng[b] / sn : 0.0;
    const double bw = log((n + EPS) / (p + EPS));
    if (ok) { iv += (n - p) * bw; a.bin_woe[var * a.total + b] = bw; }
    double sp_inc = p, sn_inc = n;                    // inclusive wave scans
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const double tp = __shfl_up(sp_inc, d, 64), tn = __shfl_up(sn_inc, d, 64);
      if (lane >= d) { sp_inc += tp; sn_inc += tn; }
    }
    if (ok) ks = fmax(ks, fabs((cp + sp_inc) - (cn + sn_inc)));
    cp += __shfl(sp_inc, 63, 64);
    cn += __shfl(sn_inc, 63, 64);
  }
  iv = wave_sum_d(iv);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) ks = fmax(ks, __shfl_xor(ks, d, 64));
  if (lane == 0) { o[0] = ks * 100.0; o[1] = iv; o[2] = log((sn + EPS) / (sp + EPS)); o[3] = 1.0; }
}
}  // namespace

SHIFU_API int shifu_column_metrics(const double* neg, const double* pos, const int* off, int F, long total,
                                   double* out, double* bin_woe, hipStream_t stream) {
  if (F <= 0) return 0;
  MetricsArgs a{neg, pos, off, F, total, out, bin_woe};
  const long waves = 2L * F;
  hipLaunchKernelGGL(column_metrics_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// ---------------------------------------------------------------------------------------------
// K5 one-hot columns (ONEHOT, and ZSCALE_ONEHOT's categoricals): raw values column-major fp64
// [F][ldv] (categorical index, -1 / NaN missing) -> `width` 0/1 outputs per column at out_col,
// the missing / unknown slot last (normalize_column's ONEHOT branch).  ip [F][5]: is_cat,
// bnd_off, nbnd, width, out_col.  One thread per (row, column); the column-major read is
// coalesced over rows.
// ---------------------------------------------------------------------------------------------
struct OneHotArgs {
  const double* vals; long ldv; long n; int F;
  const int* ip; const double* bounds;
  float* outf; long ldf; bf16_t* outb; long ldb;
};

__global__ void __launch_bounds__(256) onehot_kernel(OneHotArgs a) {
  const long r = (long)blockIdx.x * 256 + threadIdx.x;
  const int f = blockIdx.y;
  if (r >= a.n) return;
  const int* p = a.ip + f * 5;
  const double v = a.vals[(long)f * a.ldv + r];
  int idx;
  if (p[0]) idx = (v != v || v < 0) ? -1 : (int)v;
  else idx = (v != v) ? -1 : bin_search(a.bounds + p[1], p[2], v);
  const int width = p[3], oc = p[4];
  if (idx < 0 || idx >= width) idx = width - 1;
  for (int j = 0; j < width; ++j) {
    const float o = j == idx ? 1.f : 0.f;
    if (a.outf) a.outf[r * a.ldf + oc + j] = o;
    if (a.outb) a.outb[r * a.ldb + oc + j] = f2bf(o);
  }
}

SHIFU_API int shifu_onehot(const double* vals, long ldv, long n, int F, const int* ip, const double* bounds,
                           float* outf, long ldf, void* outb, long ldb, hipStream_t stream) {
  if (n <= 0 || F <= 0) return 0;
  if (F > 65535 || !ip || ldv < n) return -1;
  OneHotArgs a{vals, ldv, n, F, ip, bounds, outf, ldf, (bf16_t*)outb, ldb};
  hipLaunchKernelGGL(onehot_kernel, dim3((unsigned)((n + 255) / 256), F), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}
