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
