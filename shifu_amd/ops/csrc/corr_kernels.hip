// K15 correlation digit planes (the producer side of gemm_kernels.hip corr_i8_kernel).
//
// CorrAccumulator (shifu_amd/algos/stats.py) turns every pairwise-complete Pearson sum of a row
// chunk -- n = m'm, sx = u'm, sxx = (u*u)'m, sxy = u'u with u = x - c (c a per-column shift: the
// correlation is shift invariant, the shift removes the cancellation of large-mean columns) -- into
// exact int8 GEMMs.  This file writes their operands for one chunk of X [rows][ldx] fp64 (NaN/inf =
// missing, the reference's FastCorrelationMapper J/core/correlation/FastCorrelationMapper.java:
// 171-278 skips such pairs):
//   corr_colmax_kernel   max |x - c| over the finite values of every column (uint64 bit maxima:
//                        the order of non-negative doubles) -> per-column exponent ex (u / 2^ex in
//                        (-1/2, 1/2)) and ey = 2 ex - 1 for u^2
//   corr_planes_kernel   plane 0: m (0/1); planes 1..S: balanced base-128 digits q_s in [-64, 64]
//                        of u / 2^ex = sum_s q_s 128^-(s+1) + O(2^-(7S+1)); planes S+1..2S: the same
//                        for u^2 / 2^ey.  Layout [P][F][kpad] int8, feature-major so that one
//                        column's rows are the contiguous K axis of the NT GEMM; rows >= n are 0.
// A 128-row x 32-column fp64 tile is staged through LDS (coalesced 256-B row reads) and every lane
// then owns 16 rows of one column, so each plane is written as one 16-B store per lane (8 lanes
// cover a column's 128 contiguous bytes).
#include "common.h"

namespace {

constexpr int CP_ROWS = 128, CP_COLS = 32;

__global__ __launch_bounds__(256) void corr_colmax_kernel(const double* __restrict__ X, long ldx, int n, int F,
                                                          const double* __restrict__ shift, int rows_per_block,
                                                          unsigned long long* __restrict__ maxbits) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= F) return;
  const double c = shift ? shift[col] : 0.0;
  const long r0 = (long)blockIdx.y * rows_per_block, r1 = min((long)n, r0 + rows_per_block);
  double mx = 0.0;
  for (long r = r0; r < r1; r += 4) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = r + u < r1 ? X[(r + u) * ldx + col] : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (__builtin_isfinite(v[u])) mx = fmax(mx, fabs(v[u] - c));
  }
  if (mx > 0.0) atomicMax(maxbits + col, (unsigned long long)__double_as_longlong(mx));
}

__device__ __forceinline__ int col_exp(unsigned long long bits, bool square) {
  const double mx = __longlong_as_double((long long)bits);
  if (!(mx > 0.0) || !__builtin_isfinite(mx)) return 0;
  int E;
  (void)frexp(mx, &E);              // mx < 2^E
  return square ? 2 * E + 1 : E + 1;
}

template <int S>
__global__ __launch_bounds__(256) void corr_planes_kernel(const double* __restrict__ X, long ldx, int n, int F,
                                                          const double* __restrict__ shift,
                                                          const unsigned long long* __restrict__ maxbits,
                                                          int kpad, int8_t* __restrict__ planes, long plane_stride,
                                                          double* __restrict__ scale) {
  __shared__ double tile[CP_ROWS][CP_COLS + 1];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * CP_COLS;
  const long r0 = (long)blockIdx.y * CP_ROWS;
  // coalesced load: 8 rows x 32 columns per pass
#pragma unroll
  for (int k = 0; k < CP_ROWS / 8; ++k) {
    const int rr = k * 8 + (tid >> 5), cc = tid & 31;
    const long r = r0 + rr;
    const int col = c0 + cc;
    tile[rr][cc] = (r < n && col < F) ? X[r * ldx + col] : __builtin_nan("");
  }
  __syncthreads();
  const int wid = tid >> 6, lane = tid & 63;
  const int cl = wid * 8 + (lane >> 3), seg = lane & 7;
  const int col = c0 + cl;
  if (col >= F) return;
  const unsigned long long mb = maxbits[col];
  const int ex = col_exp(mb, false), ey = col_exp(mb, true);
  const double c = shift ? shift[col] : 0.0;
  if (blockIdx.y == 0 && seg == 0) {
    scale[col] = 1.0;
    scale[F + col] = __builtin_ldexp(1.0, ex);
    scale[2 * F + col] = __builtin_ldexp(1.0, ey);
  }
  int pm[4] = {0, 0, 0, 0}, px[S][4], py[S][4];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q) px[s][q] = py[s][q] = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const double x = tile[seg * 16 + i][cl];
    const bool ok = __builtin_isfinite(x);
    const double u = ok ? x - c : 0.0;
    double vx = __builtin_ldexp(u, -ex), vy = __builtin_ldexp(u * u, -ey);
    const int sh = (i & 3) * 8;
    pm[i >> 2] |= (ok ? 1 : 0) << sh;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double tx = vx * 128.0, ty = vy * 128.0;
      const double qx = __builtin_rint(tx), qy = __builtin_rint(ty);
      vx = tx - qx;                   // exact: |tx| <= 64 and qx is the nearest integer
      vy = ty - qy;
      px[s][i >> 2] |= ((int)qx & 0xff) << sh;
      py[s][i >> 2] |= ((int)qy & 0xff) << sh;
    }
  }
  typedef __attribute__((ext_vector_type(4))) int v4i;
  const long o = (long)col * kpad + r0 + seg * 16;
  *(v4i*)(planes + o) = v4i{pm[0], pm[1], pm[2], pm[3]};
#pragma unroll
  for (int s = 0; s < S; ++s) {
    *(v4i*)(planes + (long)(1 + s) * plane_stride + o) = v4i{px[s][0], px[s][1], px[s][2], px[s][3]};
    *(v4i*)(planes + (long)(1 + S + s) * plane_stride + o) = v4i{py[s][0], py[s][1], py[s][2], py[s][3]};
  }
}

}  // namespace

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

// Digit planes of one row chunk: X [n][ldx] fp64 (device), shift [F] (nullable = 0), S in 4..8,
// kpad % 128 == 0 and >= n; planes [1 + 2S][F][kpad] int8 (plane_stride >= F * kpad), scale [3][F]
// fp64 out (1, 2^ex, 2^ey), maxbits [F] uint64 scratch.
SHIFU_API int shifu_corr_planes(const double* X, long ldx, int n, int F, const double* shift, int S, int kpad,
                                void* planes, long plane_stride, double* scale, void* maxbits, hipStream_t stream) {
  if (n < 0 || F <= 0 || ldx < F || kpad % 128 || kpad < n || kpad <= 0 || plane_stride < (long)F * kpad ||
      S < 4 || S > 8)
    return -1;
  unsigned long long* mb = (unsigned long long*)maxbits;
  CHECK_HIP(hipMemsetAsync(mb, 0, sizeof(unsigned long long) * F, stream));
  if (n > 0) {
    const int rpb = 1024;
    hipLaunchKernelGGL(corr_colmax_kernel, dim3((F + 255) / 256, (n + rpb - 1) / rpb), dim3(256), 0, stream, X, ldx,
                       n, F, shift, rpb, mb);
    CHECK_HIP(hipGetLastError());
  }
  const dim3 grid((F + CP_COLS - 1) / CP_COLS, kpad / CP_ROWS);
  int8_t* P = (int8_t*)planes;
#define PL(S_) hipLaunchKernelGGL(corr_planes_kernel<S_>, grid, dim3(256), 0, stream, X, ldx, n, F, shift, mb, kpad, \
                                  P, plane_stride, scale)
  switch (S) { case 4: PL(4); break; case 5: PL(5); break; case 6: PL(6); break; case 7: PL(7); break; default: PL(8); }
#undef PL
  CHECK_HIP(hipGetLastError());
  return 0;
}
