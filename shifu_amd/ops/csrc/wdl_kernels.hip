// Wide & Deep input kernels for MI355X (gfx950) (K20).
//
// Reference: WideAndDeep.forward / backward (J/core/dtrain/wdl/WideAndDeep.java:112-232):
// the wide part sums one learned weight per (categorical field, category) -- a width-1
// embedding bag -- and the deep part feeds [dense | per-field embeddings] to the MLP.
//
// MI355X design: the per-field gathers that PyTorch would run as one launch per field (plus a
// concat) are one kernel that writes the deep input matrix row-major in a single coalesced pass
// (one thread per output element: consecutive threads = consecutive columns of a row) and one
// thread-per-row kernel for the wide sums; the backward scatters the gradients back into the
// concatenated tables with fp32 atomics (embedding rows are shared by many rows of a batch).
#include "common.h"

namespace {

struct WdlArgs {
  const float* dense; int nd;                 // [n][nd]
  const long* cats; int Fc;                   // [n][Fc] category index per field (< table rows)
  const float* wtab; const int* woff;         // wide tables concatenated; field f at woff[f]
  const float* etab; const int* eoff;         // embedding tables concatenated ([rows][D] each); e at eoff[e]
  const int* efield; int E, D;                // embedding e reads field efield[e]
  float* wide;                                // [n]           (fwd out / bwd in, nullable)
  float* A; long lda;                         // [n][nd + E*D] (fwd out / bwd in, nullable)
  float* dwtab; float* detab;                 // bwd out (accumulated)
  long nw, ne;                                // wide / embedding table sizes (floats): a table row
                                              // index past them is skipped (read as 0, never written)
  long n;
};

__global__ __launch_bounds__(256) void wdl_wide_fwd_kernel(WdlArgs a) {
  const long r = (long)blockIdx.x * 256 + threadIdx.x;
  if (r >= a.n) return;
  float s = 0.f;
  for (int f = 0; f < a.Fc; ++f) {
    const long c = a.cats[r * a.Fc + f], k = a.woff[f] + c;
    if (c >= 0 && k < a.nw) s += a.wtab[k];
  }
  a.wide[r] = s;
}

__global__ __launch_bounds__(256) void wdl_deep_fwd_kernel(WdlArgs a) {
  const long w = a.nd + (long)a.E * a.D;
  const long total = a.n * w;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / w;
    const int c = (int)(i - r * w);
    float v;
    if (c < a.nd) {
      v = a.dense[r * a.nd + c];
    } else {
      const int e = (c - a.nd) / a.D, d = (c - a.nd) - e * a.D;
      const long c = a.cats[r * a.Fc + a.efield[e]], k = ((long)a.eoff[e] + c) * a.D + d;
      v = (c >= 0 && k < a.ne) ? a.etab[k] : 0.f;
    }
    a.A[r * a.lda + c] = v;
  }
}

__global__ __launch_bounds__(256) void wdl_wide_bwd_kernel(WdlArgs a) {
  const long total = a.n * a.Fc;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / a.Fc;
    const int f = (int)(i - r * a.Fc);
    const long c = a.cats[i], k = a.woff[f] + c;
    if (c >= 0 && k < a.nw) atomicAdd(&a.dwtab[k], a.wide[r]);
  }
}

__global__ __launch_bounds__(256) void wdl_deep_bwd_kernel(WdlArgs a) {
  const long ew = (long)a.E * a.D;
  const long total = a.n * ew;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / ew;
    const int c = (int)(i - r * ew), e = c / a.D, d = c - e * a.D;
    const long cat = a.cats[r * a.Fc + a.efield[e]], k = ((long)a.eoff[e] + cat) * a.D + d;
    if (cat >= 0 && k < a.ne) atomicAdd(&a.detab[k], a.A[r * a.lda + a.nd + c]);
  }
}

long grid_of(long total) { long b = (total + 255) / 256; return b < 1 ? 1 : (b > 65536 ? 65536 : b); }

}  // namespace

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

// dir 0: forward (wide sums and/or deep input matrix), dir 1: backward (table gradients)
SHIFU_API int shifu_wdl_gather(int dir, const float* dense, int nd, const long* cats, int Fc, const float* wtab,
                               const int* woff, const float* etab, const int* eoff, const int* efield, int E, int D,
                               float* wide, float* A, long lda, float* dwtab, float* detab, long nw, long ne,
                               long n, hipStream_t stream) {
  if (n <= 0) return 0;
  if (Fc < 0 || E < 0 || (E > 0 && D <= 0) || (A && lda < nd + (long)E * D)) return -1;
  if (nw < 0 || ne < 0) return -1;
  WdlArgs a{dense, nd, cats, Fc, wtab, woff, etab, eoff, efield, E, D, wide, A, lda, dwtab, detab, nw, ne, n};
  if (dir == 0) {
    if (wide && Fc > 0) hipLaunchKernelGGL(wdl_wide_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
    if (A) hipLaunchKernelGGL(wdl_deep_fwd_kernel, dim3((unsigned)grid_of(n * (nd + (long)E * D))), dim3(256), 0,
                              stream, a);
  } else {
    if (wide && dwtab && Fc > 0)
      hipLaunchKernelGGL(wdl_wide_bwd_kernel, dim3((unsigned)grid_of(n * Fc)), dim3(256), 0, stream, a);
    if (A && detab && E > 0)
      hipLaunchKernelGGL(wdl_deep_bwd_kernel, dim3((unsigned)grid_of(n * (long)E * D)), dim3(256), 0, stream, a);
  }
  CHECK_HIP(hipGetLastError());
  return 0;
}

// ---- Output-neuron row / column dots (the WDL output unit, WideAndDeep.java:163-232, a linear
// unit over [h_L | 1]; the SE output neuron and base score, algos/varsel.py) ---------------------
// forward  out[i]   = sum_j H[i][j] w[j]          (bf16 activations, fp32 weights / sums)
// backward gw[j]    = sum_i g[i] H[i][j]          (per-256-row-block partials, then a fixed-order
//                                                  sum over blocks: deterministic, no atomics)
namespace {

__global__ __launch_bounds__(256) void wdl_rowdot_kernel(const bf16_t* __restrict__ H, long ldh, long n, int k,
                                                         const float* __restrict__ w, float* __restrict__ out) {
  // one wave per row, lanes over the columns
  const long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  float s = 0.f;
  for (int j = lane; j < k; j += 64) s += bf2f(((const uint16_t*)H)[i * ldh + j]) * w[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[i] = s;
}

__global__ __launch_bounds__(256) void wdl_coldot_part_kernel(const float* __restrict__ g, const bf16_t* __restrict__ H,
                                                              long ldh, long n, int k, float* __restrict__ part) {
  const long r0 = (long)blockIdx.x * 256, r1 = min(n, r0 + 256);
  for (int j = threadIdx.x; j < k; j += 256) {
    float s = 0.f;
    for (long i = r0; i < r1; ++i) s += g[i] * bf2f(((const uint16_t*)H)[i * ldh + j]);
    part[(long)blockIdx.x * k + j] = s;
  }
}

__global__ __launch_bounds__(256) void coldot_f32_part_kernel(const float* __restrict__ g, const float* __restrict__ X,
                                                              long ldx, long n, int k, float* __restrict__ part) {
  const long r0 = (long)blockIdx.x * 256, r1 = min(n, r0 + 256);
  for (int j = threadIdx.x; j < k; j += 256) {
    float s = 0.f;
    for (long i = r0; i < r1; ++i) s += g[i] * X[i * ldx + j];
    part[(long)blockIdx.x * k + j] = s;
  }
}

__global__ __launch_bounds__(256) void wdl_coldot_final_kernel(const float* __restrict__ part, long nb, int k,
                                                               float* __restrict__ gw) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= k) return;
  float s = 0.f;
  for (long b = 0; b < nb; ++b) s += part[b * k + j];
  gw[j] = s;
}

// out[i] = act_out(sum_j act_in(X[i][j]) w[j] + b)   (fp32 rows; act ids as models.nn.ACT_IDS,
// act_in < 0: identity)
__global__ __launch_bounds__(256) void rowdot_f32_act_kernel(const float* __restrict__ X, long ldx, long n, int k,
                                                             const float* __restrict__ w, float b, int act_in,
                                                             int act_out, float* __restrict__ out) {
  const long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  float s = 0.f;
  for (int j = lane; j < k; j += 64) {
    const float x = X[i * ldx + j];
    s += (act_in < 0 ? x : act_fwd(act_in, x)) * w[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[i] = act_out < 0 ? s + b : act_fwd(act_out, s + b);
}

}  // namespace

SHIFU_API int shifu_rowdot_f32_act(const float* X, long ldx, long n, int k, const float* w, float b, int act_in,
                                   int act_out, float* out, hipStream_t stream) {
  if (n <= 0) return 0;
  if (k <= 0 || ldx < k) return -1;
  hipLaunchKernelGGL(rowdot_f32_act_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, X, ldx, n, k, w, b,
                     act_in, act_out, out);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_rowdot_bf16(const void* H, long ldh, long n, int k, const float* w, float* out,
                               hipStream_t stream) {
  if (n <= 0) return 0;
  if (k <= 0 || ldh < k) return -1;
  hipLaunchKernelGGL(wdl_rowdot_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, (const bf16_t*)H, ldh,
                     n, k, w, out);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// part: >= ceil(n / 256) * k floats of scratch
SHIFU_API int shifu_coldot_bf16(const float* g, const void* H, long ldh, long n, int k, float* part, float* gw,
                               hipStream_t stream) {
  if (k <= 0 || ldh < k || n < 0) return -1;
  const long nb = (n + 255) / 256;
  if (nb > 0)
    hipLaunchKernelGGL(wdl_coldot_part_kernel, dim3((unsigned)nb), dim3(256), 0, stream, g, (const bf16_t*)H, ldh, n,
                       k, part);
  hipLaunchKernelGGL(wdl_coldot_final_kernel, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, stream, part, nb, k,
                     gw);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// the same over fp32 rows (LR gradient above K9's feature limit, models/lr.py)
SHIFU_API int shifu_coldot_f32(const float* g, const float* X, long ldx, long n, int k, float* part, float* gw,
                               hipStream_t stream) {
  if (k <= 0 || ldx < k || n < 0) return -1;
  const long nb = (n + 255) / 256;
  if (nb > 0)
    hipLaunchKernelGGL(coldot_f32_part_kernel, dim3((unsigned)nb), dim3(256), 0, stream, g, X, ldx, n, k, part);
  hipLaunchKernelGGL(wdl_coldot_final_kernel, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, stream, part, nb, k,
                     gw);
  CHECK_HIP(hipGetLastError());
  return 0;
}
