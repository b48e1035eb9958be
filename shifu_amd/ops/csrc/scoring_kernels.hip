// Scoring-side kernels for MI355X (gfx950): tree-ensemble inference (K13) and keyed weighted
// bin counts (K17 PSI unit x bin counts, K18 post-train per-bin score sums).
//
// Reference hot loops replaced:
//   tree walk     IndependentTreeModel.computeRegressionScore / predictNode
//                                         J/core/dtrain/dt/IndependentTreeModel.java:387-441, 465-520
//   PSI counts    PSICalculatorUDF / PopulationCounterUDF   J/udf/PSICalculatorUDF.java, J/udf/PopulationCounterUDF.java
//   bin avg score PostTrainMapper.map -> reducer            J/core/posttrain/PostTrainMapper.java:183-256
//
// MI355X design:
//   * tree inference: the input matrix is feature-major [C][N] fp64, so the 64 lanes of a wave
//     (64 consecutive rows) read one contiguous 512-B run whenever they sit on the same feature
//     (always at the root, mostly near it).  Node records are 16-B {feat, left, right, catrow}
//     plus fp64 threshold / leaf value: a whole 500-tree depth-7 ensemble is ~1.5 MB and stays in
//     L2.  Work = (256-row block, tree group); each group accumulates its trees in fixed order
//     into its own partial-score row, summed afterwards in group order -> deterministic scores.
//     Threshold compares stay fp64 so routing is bit-identical to the reference's double walk.
//   * keyed counts: one block per (row range, column) with an LDS-private int64 histogram
//     (count, fixed-point weight) flushed to global with integer atomics -> exact counts and
//     order-independent (deterministic) weighted sums; keys past the LDS budget go straight to
//     global integer atomics.
#include "common.h"

namespace {

struct TreeInferArgs {
  const double* X; long sf, sr;        // X[f * sf + row * sr]
  long n;
  const int4* node;                    // {feat (-1 = leaf), left, right, catrow}
  const double* thr;                   // numeric threshold / category count for categorical splits
  const double* value;                 // leaf value
  const uint8_t* catlut; int lut_w;    // [n_catrows][lut_w] 1 = goes left
  const int* roots; const double* lrs; int T, depth, tg;   // tg = trees per group
  double* part;                        // [n_groups][n] partial scores (nullable)
  int* leaf_out;                       // [n][T] leaf node ids (nullable)
};

// One (row, tree) walk is a chain of dependent loads (node -> input value -> next node), so a
// thread walks TI trees at once, level by level: TI independent chains per lane keep TI x the
// loads in flight (the kernel is latency-bound, not bandwidth-bound).  Leaves stay put, so the
// level loop has a fixed trip count (the ensemble depth) and every lane exits.
template <int TI>
__global__ __launch_bounds__(256) void tree_infer_kernel(TreeInferArgs a) {
  const long row = (long)blockIdx.x * 256 + threadIdx.x;
  if (row >= a.n) return;
  const int t0 = blockIdx.y * a.tg, t1 = min(a.T, t0 + a.tg);
  const double* xr = a.X + row * a.sr;
  double acc = 0.0;
  for (int tb = t0; tb < t1; tb += TI) {
    int id[TI];
    int4 nd[TI];
#pragma unroll
    for (int u = 0; u < TI; ++u) {
      id[u] = a.roots[min(tb + u, t1 - 1)];          // a short last batch repeats its last tree
      nd[u] = a.node[id[u]];
    }
    for (int d = 0; d < a.depth; ++d) {
      double v[TI], th[TI];
#pragma unroll
      for (int u = 0; u < TI; ++u) {
        const bool inner = nd[u].x >= 0;
        v[u] = inner ? xr[(long)nd[u].x * a.sf] : 0.0;
        th[u] = a.thr[id[u]];
      }
#pragma unroll
      for (int u = 0; u < TI; ++u) {
        if (nd[u].x < 0) continue;
        bool left;
        if (nd[u].w >= 0) {                            // categorical: category-index LUT
          int ci = (v[u] < 0.0 || v[u] >= th[u]) ? (int)th[u] : (int)floor(v[u] + 0.1);
          ci = min(max(ci, 0), a.lut_w - 1);
          left = a.catlut[(long)nd[u].w * a.lut_w + ci] != 0;
        } else {
          left = v[u] < th[u];
        }
        id[u] = left ? nd[u].y : nd[u].z;
      }
#pragma unroll
      for (int u = 0; u < TI; ++u) nd[u] = a.node[id[u]];
    }
#pragma unroll
    for (int u = 0; u < TI; ++u) {
      const int t = tb + u;
      if (t >= t1) break;
      if (a.leaf_out) a.leaf_out[row * a.T + t] = id[u];
      acc += a.lrs[t] * a.value[id[u]];
    }
  }
  if (a.part) a.part[(long)blockIdx.y * a.n + row] = acc;
}

// ---------------------------------------------------------------------------------------
// Coded tree walk.  The scattered fp64 input reads above move a 64-B+ transaction per (row,
// tree, level): at 500 trees x depth 7 that is ~1 TB per 5M rows, so the plain walk runs at
// the HBM rate, not the tree rate.  Instead every input value is first replaced by its rank
// among the ensemble's thresholds of that feature (u16 code: count of thresholds <= v, so
// v < t_k <=> code <= k exactly; NaN -> 0xFFFF goes right like the fp64 compare), the rows'
// codes are staged in LDS once (R rows x C codes, one coalesced read per row), and the walk
// reads only LDS + the L2-resident node table.
//   tree_code_kernel : 64-row x 64-feature tiles of the feature-major input, transposed
//                      through LDS into row-major u16 codes (coalesced both ways)
//   tree_walk_coded_kernel : R rows per block, TPR = 256 / R threads per row, thread sub walks
//                      trees sub, sub + TPR, ... (WCH at a time); per-row partial sums added in
//                      sub order (deterministic)
// ---------------------------------------------------------------------------------------
struct TreeCodeArgs {
  const double* XT; long ldx; long n; int C;  // feature-major: value (f, r) at XT[f * ldx + r]
  const double* bnd; const int* boff;       // sorted unique thresholds of feature f: bnd[boff[f] .. boff[f+1])
  const uint8_t* is_cat;                    // [C] categorical slot (value = category index)
  uint16_t* codes;                          // [n][C]
  int tb_cap;                               // thresholds the dynamic LDS buffer holds (0: search in global)
};

constexpr int TC_LDS = 4096;                // thresholds of the tile's features staged in LDS (32 KiB)
constexpr int TC_R = 256, TC_F = 32;        // tile: 256 rows (one per thread) x 32 features
constexpr int TCG = 16;                     // features per load group (TCG x 8 B in flight per lane)

// Thread t owns row r0 + t of the tile: its 32 feature values are loaded TCG at a time (TCG x 8 B in
// flight per lane, the next group's loads issued before this group's searches; a wave reads 512 contiguous bytes of one feature, the block 2 KiB), each is
// ranked by a branchless upper-bound search over the LDS-staged thresholds (wave-uniform step
// count: every lane of a wave is on the same feature), and the u16 codes are transposed
// through LDS into 64-B row segments of the row-major output.
__global__ __launch_bounds__(256) void tree_code_kernel(TreeCodeArgs a) {
  __shared__ uint16_t tile[TC_R][TC_F + 2];
  extern __shared__ double tb[];            // [a.tb_cap]: sized by the host to the largest tile's list
  // feature tile = blockIdx.x (fastest): the blocks in flight share a few row blocks, so every
  // feature column is read as one sequential stream (few pages live, TLB-friendly) instead of
  // each block opening 32 pages 8 B x N apart
  const long r0 = (long)blockIdx.y * TC_R;
  const int f0 = blockIdx.x * TC_F;
  const int fend = min(a.C, f0 + TC_F);
  const int b0 = a.boff[f0], nb = a.boff[fend] - b0;
  const bool lds = nb <= a.tb_cap;
  if (lds)
    for (int i = threadIdx.x; i < nb; i += 256) tb[i] = a.bnd[b0 + i];
  __syncthreads();
  // index the staged copy relative to b0 (never form tb - b0: an LDS address below the
  // allocation does not survive the generic-pointer conversion)
  auto thr_at = [&](int i) { return lds ? tb[i - b0] : a.bnd[i]; };
  const long r = r0 + threadIdx.x;
  const bool live = r < a.n;
  auto loadg = [&](int g, double* v) {
#pragma unroll
    for (int k = 0; k < TCG; ++k) {
      const int f = f0 + g + k;
      v[k] = (live && f < a.C) ? a.XT[(long)f * a.ldx + r] : 0.0;
    }
  };
  double v[TCG], vn[TCG];
  loadg(0, v);
  for (int g = 0; g < TC_F; g += TCG) {
    if (g + TCG < TC_F) loadg(g + TCG, vn);        // next group's loads in flight during this search
    // the TCG searches advance together (TCG independent LDS reads per step); a search whose
    // feature has fewer thresholds just fails the bound check on the extra steps
    int pos[TCG], base[TCG], L[TCG], lmax = 0;
#pragma unroll
    for (int k = 0; k < TCG; ++k) {
      const int f = min(f0 + g + k, a.C - 1);
      base[k] = a.boff[f];
      L[k] = a.boff[f + 1] - base[k];
      pos[k] = 0;
      lmax = max(lmax, L[k]);
    }
    for (int st = lmax ? 1 << (31 - __clz(lmax)) : 0; st > 0; st >>= 1) {
#pragma unroll
      for (int k = 0; k < TCG; ++k)
        if (pos[k] + st <= L[k] && thr_at(base[k] + pos[k] + st - 1) <= v[k]) pos[k] += st;
    }
#pragma unroll
    for (int k = 0; k < TCG; ++k) {
      const int f = f0 + g + k;
      uint16_t code = 0;
      if (f < a.C) {
        if (a.is_cat[f]) code = (v[k] >= 0.0) ? (uint16_t)fmin(floor(v[k] + 0.1), 65534.0) : (uint16_t)0xFFFF;
        else code = (v[k] != v[k]) ? (uint16_t)0xFFFF : (uint16_t)pos[k];      // NaN goes right
      }
      tile[threadIdx.x][g + k] = code;
    }
#pragma unroll
    for (int k = 0; k < TCG; ++k) v[k] = vn[k];
  }
  __syncthreads();
  const int nf = fend - f0;
#pragma unroll 4
  for (int i = 0; i < TC_R * TC_F / 256; ++i) {
    const int e = threadIdx.x + 256 * i, rr = e / TC_F, fl = e % TC_F;
    if (r0 + rr < a.n && fl < nf) a.codes[(r0 + rr) * a.C + f0 + fl] = tile[rr][fl];
  }
}

struct TreeWalkArgs {
  const uint16_t* codes; long n; int C;     // [n][C]
  const int4* node;                         // {feat (-1 leaf), left, right, w}: w >= 0 numeric threshold code k
                                            // (left iff code <= k), w < 0 categorical LUT row -w-1
  const int* catnc;                         // [n_catrows] category count of the split's column
  const double* value;
  const uint8_t* catlut; int lut_w;
  const int* roots; const double* lrs; int T, depth, tg, R;
  double* part; long ldp;                   // partial score of group g, row r at part[g * ldp + r]
  int* leaf_out;
};

__device__ __forceinline__ int walk_step(const TreeWalkArgs& a, const uint16_t* row, int4 nd) {
  const uint32_t code = row[nd.x];
  bool left;
  if (nd.w >= 0) {
    left = code <= (uint32_t)nd.w;
  } else {
    const int cr = -nd.w - 1, nc = a.catnc[cr];
    int ci = (code == 0xFFFFu || (int)code >= nc) ? nc : (int)code;
    ci = min(ci, a.lut_w - 1);
    left = a.catlut[(long)cr * a.lut_w + ci] != 0;
  }
  return left ? nd.y : nd.z;
}

constexpr int WCH = 4;                      // tree chains walked together per thread

__global__ __launch_bounds__(256) void tree_walk_coded_kernel(TreeWalkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
  uint16_t* rows = (uint16_t*)wsm;                                  // [R][C]
  double* red = (double*)(wsm + (((size_t)a.R * a.C * 2 + 15) & ~(size_t)15));   // [TPR][R]
  const long rb = (long)blockIdx.x * a.R;
  const int nr = (int)min((long)a.R, a.n - rb);
  const uint16_t* src = a.codes + rb * a.C;
  for (int i = threadIdx.x; i < nr * a.C; i += 256) rows[i] = src[i];
  __syncthreads();
  const int TPR = 256 / a.R, r = threadIdx.x % a.R, sub = threadIdx.x / a.R;
  const int t0 = blockIdx.y * a.tg, t1 = min(a.T, t0 + a.tg);
  const uint16_t* row = rows + r * a.C;
  double acc = 0.0;
  if (r < nr) {
    for (int t = t0 + sub; t < t1; t += WCH * TPR) {
      // WCH independent chains (trees t, t + TPR, ...): a chain past the group's end repeats the
      // last tree and is not accumulated
      int id[WCH];
      int4 nd[WCH];
#pragma unroll
      for (int c = 0; c < WCH; ++c) {
        id[c] = a.roots[min(t + c * TPR, t1 - 1)];
        nd[c] = a.node[id[c]];
      }
      for (int d = 0; d < a.depth; ++d) {                           // leaves stay put: fixed trip count
#pragma unroll
        for (int c = 0; c < WCH; ++c)
          if (nd[c].x >= 0) id[c] = walk_step(a, row, nd[c]);
#pragma unroll
        for (int c = 0; c < WCH; ++c) nd[c] = a.node[id[c]];
      }
#pragma unroll
      for (int c = 0; c < WCH; ++c) {
        const int tc = t + c * TPR;
        if (tc >= t1) break;
        if (a.leaf_out) a.leaf_out[(rb + r) * a.T + tc] = id[c];
        acc += a.lrs[tc] * a.value[id[c]];
      }
    }
  }
  red[sub * a.R + r] = acc;
  __syncthreads();
  if (sub == 0 && r < nr && a.part) {
    double s = 0.0;
    for (int k = 0; k < TPR; ++k) s += red[k * a.R + r];
    a.part[(long)blockIdx.y * a.ldp + rb + r] = s;
  }
}

// ---------------------------------------------------------------------------------------
// Keyed counts: out_cnt[f][k] += 1, out_w[f][k] += round(w * scale) for every row with
// 0 <= key < K.  keys[f * ks + r] (ks = 0: one key vector shared by every column),
// w[f * ws + r] (ws = 0: shared weights; w == nullptr: no weighted sums).
// ---------------------------------------------------------------------------------------
constexpr int KH_LDS_K = 2048;          // keys held in LDS (2 x 2048 x 8 B = 32 KiB)

struct KeyedArgs {
  const int* keys; long ks;
  const double* w; long ws;
  long n; int K;
  double scale;
  unsigned long long* cnt;               // [F][K]
  unsigned long long* wsum;              // [F][K] two's-complement int64 fixed point
};

__global__ __launch_bounds__(256) void keyed_hist_kernel(KeyedArgs a) {
  __shared__ unsigned long long hc[KH_LDS_K], hw[KH_LDS_K];
  const int f = blockIdx.y;
  const bool lds = a.K <= KH_LDS_K;
  if (lds)
    for (int i = threadIdx.x; i < a.K; i += 256) { hc[i] = 0ull; hw[i] = 0ull; }
  __syncthreads();
  const int* kc = a.keys + f * a.ks;
  const double* wc = a.w ? a.w + f * a.ws : nullptr;
  unsigned long long* gc = a.cnt + (long)f * a.K;
  unsigned long long* gw = a.wsum + (long)f * a.K;
  const long stride = (long)gridDim.x * 256;
  for (long r0 = (long)blockIdx.x * 256 + threadIdx.x; r0 < a.n; r0 += 4 * stride) {
    int k[4];
    double wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {               // four loads in flight before any atomic
      const long r = r0 + u * stride;
      k[u] = r < a.n ? kc[r] : -1;
      wv[u] = (wc && r < a.n) ? wc[r] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k[u] < 0 || k[u] >= a.K) continue;
      const unsigned long long q = (unsigned long long)__double2ll_rn(wv[u] * a.scale);
      if (lds) {
        atomicAdd(&hc[k[u]], 1ull);
        if (wc) atomicAdd(&hw[k[u]], q);
      } else {
        atomicAdd(&gc[k[u]], 1ull);
        if (wc) atomicAdd(&gw[k[u]], q);
      }
    }
  }
  if (!lds) return;
  __syncthreads();
  for (int i = threadIdx.x; i < a.K; i += 256) {
    if (hc[i]) atomicAdd(&gc[i], hc[i]);
    if (wc && hw[i]) atomicAdd(&gw[i], hw[i]);
  }
}

}  // namespace

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

SHIFU_API int shifu_tree_infer(const double* X, long sf, long sr, long n, const void* node, const double* thr,
                               const double* value, const void* catlut, int lut_w, const int* roots,
                               const double* lrs, int T, int depth, int n_groups, double* part, int* leaf_out,
                               hipStream_t stream) {
  if (n <= 0 || T <= 0) return 0;
  if (n_groups < 1 || n_groups > T || lut_w < 1 || depth < 0) return -1;
  const int tg = (T + n_groups - 1) / n_groups;
  if ((long)(n_groups - 1) * tg >= T) return -1;          // every group owns >= 1 tree
  TreeInferArgs a{X, sf, sr, n, (const int4*)node, thr, value, (const uint8_t*)catlut, lut_w, roots, lrs,
                  T, depth, tg, part, leaf_out};
  hipLaunchKernelGGL(tree_infer_kernel<4>, dim3((unsigned)((n + 255) / 256), n_groups), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_keyed_hist(const int* keys, long ks, const double* w, long ws, long n, int F, int K,
                               double scale, void* cnt, void* wsum, hipStream_t stream) {
  if (n <= 0 || F <= 0 || K <= 0) return 0;
  if (F > 65535) return -1;
  long bx = (n + 256 * 4 - 1) / (256 * 4);
  const long want = (2048 + F - 1) / F;                   // >= 2048 blocks over all columns
  if (bx > want) bx = want;
  if (bx < 1) bx = 1;
  KeyedArgs a{keys, ks, w, ws, n, K, scale, (unsigned long long*)cnt, (unsigned long long*)wsum};
  hipLaunchKernelGGL(keyed_hist_kernel, dim3((unsigned)bx, F), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_tree_code(const double* XT, long ldx, long n, int C, const double* bnd, const int* boff,
                              const void* is_cat, void* codes, int tb_cap, hipStream_t stream) {
  if (n <= 0 || C <= 0) return 0;
  if (C > 65535 * TC_F || ldx < n) return -1;
  // tb_cap: the largest 32-feature tile's threshold count (host-computed; tiles with more search in
  // global memory), so the LDS footprint is what the ensemble needs, not the TC_LDS maximum
  if (tb_cap < 0) return -1;
  TreeCodeArgs a{XT, ldx, n, C, bnd, boff, (const uint8_t*)is_cat, (uint16_t*)codes, min(tb_cap, TC_LDS)};
  if ((n + TC_R - 1) / TC_R > 65535) return -1;            // row blocks on grid y
  hipLaunchKernelGGL(tree_code_kernel, dim3((C + TC_F - 1) / TC_F, (unsigned)((n + TC_R - 1) / TC_R)), dim3(256),
                     (size_t)a.tb_cap * sizeof(double), stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_tree_walk_coded(const void* codes, long n, int C, const void* node, const int* catnc,
                                    const double* value, const void* catlut, int lut_w, const int* roots,
                                    const double* lrs, int T, int depth, int R, int n_groups, double* part,
                                    long ldp, int* leaf_out, hipStream_t stream) {
  if (n <= 0 || T <= 0) return 0;
  if (R < 1 || R > 256 || (R & (R - 1)) || (size_t)R * C * 2 > 65536 || n_groups < 1 || n_groups > T ||
      lut_w < 1 || depth < 0 || ldp < n) return -1;
  const int tg = (T + n_groups - 1) / n_groups;
  if ((long)(n_groups - 1) * tg >= T) return -1;
  TreeWalkArgs a{(const uint16_t*)codes, n, C, (const int4*)node, catnc, value, (const uint8_t*)catlut, lut_w,
                 roots, lrs, T, depth, tg, R, part, ldp, leaf_out};
  const size_t lds = (((size_t)R * C * 2 + 15) & ~(size_t)15) + 256 * sizeof(double);
  hipLaunchKernelGGL(tree_walk_coded_kernel, dim3((unsigned)((n + R - 1) / R), n_groups), dim3(256), lds, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}
