// SVM C-SVC dual solver (SMO with libsvm's WSS3 second-order working-set selection) on the GPU.
//
// Reference: the legacy LOCAL SVM (J/core/alg/SVMTrainer.java:38-185) trains Encog's
// SupportVectorClassification, i.e. libsvm's solver.  models/svm.py drives the same algorithm;
// this kernel runs ITERS SMO iterations per launch inside one workgroup so the host synchronises
// once per batch (convergence check) instead of ~8 times per iteration.
//
// One 1024-thread workgroup (16 waves) owns the whole problem: per iteration
//   pass 1  Gmax = max_{t in I_up} -y_t G_t (first index on ties, as torch.argmax), Gmin over I_low
//   pass 2  j = argmin_{t in I_low, b_t > 0} -(b_t^2) / a_t,  b_t = Gmax + y_t G_t,
//           a_t = max(K_ii + K_tt - 2 K_it, TAU)                           (first index on ties)
//   scalar  the two-variable sub-problem with libsvm's clipping (thread 0, fp64)
//   pass 3  G_t += y_t (y_i da_i K_it + y_j da_j K_jt)
// K is the device-resident fp32 Gram matrix; alpha, G, y, C are fp64 (libsvm precision).  A
// single workgroup keeps the iteration free of grid-wide synchronisation: each pass streams
// 1-2 rows of K (n * 4 B) plus a few fp64 vectors, small next to a launch + host round trip.
#include "common.h"

namespace {

constexpr int ST = 1024;
constexpr int SW = ST / 64;

struct SmoArgs {
  const float* K; long ldk;     // [n][n] Gram matrix
  const double* Y;              // [n] +-1
  const double* C;              // [n] per-row box bound
  const double* Kd;             // [n] diagonal of K (fp64)
  double* alpha; double* G;     // [n] state
  int n, iters;
  double eps, tau;
  long* state;                  // [0] iterations done (accumulated), [1] converged flag
  double* gap;                  // [0] last Gmax - Gmin
};

// (value, index) reductions; ties resolve to the lower index
__device__ __forceinline__ void better_max(double& v, int& i, double v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
__device__ __forceinline__ void better_min(double& v, int& i, double v2, int i2) {
  if (v2 < v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

__global__ __launch_bounds__(ST) void svm_smo_kernel(SmoArgs a) {
#pragma clang fp contract(off)
  __shared__ double sv[SW], sv2[SW];
  __shared__ int si[SW];
  __shared__ double s_gmax, s_gmin, s_dai, s_daj, s_yi, s_yj;
  __shared__ int s_i, s_j, s_stop;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const double INF = __longlong_as_double(0x7ff0000000000000ll);
  int done = 0;
  for (int it = 0; it < a.iters; ++it) {
    // ---- pass 1
    double vmax = -INF, vmin = INF;
    int imax = 0x7fffffff;
    for (int t = tid; t < a.n; t += ST) {
      const double y = a.Y[t], al = a.alpha[t], c = a.C[t];
      const double mg = -y * a.G[t];
      const bool up = (y > 0 && al < c) || (y < 0 && al > 0);
      const bool low = (y > 0 && al > 0) || (y < 0 && al < c);
      if (up) better_max(vmax, imax, mg, t);
      if (low) vmin = fmin(vmin, mg);
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double v2 = __shfl_xor(vmax, o, 64);
      const int i2 = __shfl_xor(imax, o, 64);
      better_max(vmax, imax, v2, i2);
      vmin = fmin(vmin, __shfl_xor(vmin, o, 64));
    }
    if (lane == 0) { sv[wid] = vmax; si[wid] = imax; sv2[wid] = vmin; }
    __syncthreads();
    if (tid == 0) {
      double v = sv[0], m = sv2[0];
      int i = si[0];
      for (int w = 1; w < SW; ++w) { better_max(v, i, sv[w], si[w]); m = fmin(m, sv2[w]); }
      s_gmax = v; s_gmin = m; s_i = i;
      s_stop = (i == 0x7fffffff) || !(v - m >= a.eps);
      a.gap[0] = v - m;
    }
    __syncthreads();
    if (s_stop) { if (tid == 0) a.state[1] = 1; break; }
    const int i = s_i;
    const double gmax = s_gmax;
    const float* Ki = a.K + (size_t)i * a.ldk;
    const double kii = a.Kd[i];
    // ---- pass 2
    double omin = INF;
    int jmin = 0x7fffffff;
    for (int t = tid; t < a.n; t += ST) {
      const double y = a.Y[t], al = a.alpha[t], c = a.C[t];
      const bool low = (y > 0 && al > 0) || (y < 0 && al < c);
      const double b = gmax - (-y * a.G[t]);
      if (low && b > 0) {
        const double aa = fmax(kii + a.Kd[t] - 2.0 * (double)Ki[t], a.tau);
        better_min(omin, jmin, -(b * b) / aa, t);
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double v2 = __shfl_xor(omin, o, 64);
      const int i2 = __shfl_xor(jmin, o, 64);
      better_min(omin, jmin, v2, i2);
    }
    __syncthreads();                         // pass-1 partials consumed
    if (lane == 0) { sv[wid] = omin; si[wid] = jmin; }
    __syncthreads();
    if (tid == 0) {
      double v = sv[0];
      int j = si[0];
      for (int w = 1; w < SW; ++w) better_min(v, j, sv[w], si[w]);
      if (j == 0x7fffffff) j = i;            // no candidate (torch.argmin of all-inf: index 0 -> harmless)
      // two-variable sub-problem (libsvm Solver::solve, the clipping of models/svm.py)
      const double yi = a.Y[i], yj = a.Y[j];
      const double ai0 = a.alpha[i], aj0 = a.alpha[j], Ci = a.C[i], Cj = a.C[j];
      const double Gi = a.G[i], Gj = a.G[j];
      const double kjj = a.Kd[j], kij = (double)Ki[j];
      const double quad = fmax(kii + kjj - 2 * kij, a.tau);
      double ai = ai0, aj = aj0;
      if (yi != yj) {
        const double delta = (-Gi - Gj) / quad, diff = ai - aj;
        ai += delta; aj += delta;
        if (diff > 0 && aj < 0) { aj = 0; ai = diff; }
        else if (diff <= 0 && ai < 0) { ai = 0; aj = -diff; }
        if (diff > Ci - Cj && ai > Ci) { ai = Ci; aj = Ci - diff; }
        else if (diff <= Ci - Cj && aj > Cj) { aj = Cj; ai = Cj + diff; }
      } else {
        const double delta = (Gi - Gj) / quad, sm = ai + aj;
        ai -= delta; aj += delta;
        if (sm > Ci && ai > Ci) { ai = Ci; aj = sm - Ci; }
        else if (sm <= Ci && aj < 0) { aj = 0; ai = sm; }
        if (sm > Cj && aj > Cj) { aj = Cj; ai = sm - Cj; }
        else if (sm <= Cj && ai < 0) { ai = 0; aj = sm; }
      }
      s_j = j; s_yi = yi; s_yj = yj;
      s_dai = ai - ai0; s_daj = aj - aj0;
      a.alpha[i] = ai;
      a.alpha[j] = aj;
    }
    __syncthreads();
    // ---- pass 3
    const int j = s_j;
    const float* Kj = a.K + (size_t)j * a.ldk;
    const double ci = s_yi * s_dai, cj = s_yj * s_daj;
    for (int t = tid; t < a.n; t += ST) {
      const double u = ci * (double)Ki[t] + cj * (double)Kj[t];
      a.G[t] = a.G[t] + a.Y[t] * u;
    }
    ++done;
    __syncthreads();                         // G / alpha visible to the next pass 1
  }
  if (tid == 0) a.state[0] += done;
}

}  // namespace

// Run up to `iters` SMO iterations (stops early at gap < eps: state[1] = 1).  state[0] accumulates
// the iterations done.  One workgroup; n <= 2^31 - 1.
SHIFU_API int shifu_svm_smo(const float* K, long ldk, const double* Y, const double* C, const double* Kd,
                            double* alpha, double* G, int n, int iters, double eps, double tau, long* state,
                            double* gap, hipStream_t stream) {
  if (n <= 0 || iters <= 0 || ldk < n) return -1;
  SmoArgs a{K, ldk, Y, C, Kd, alpha, G, n, iters, eps, tau, state, gap};
  hipLaunchKernelGGL(svm_smo_kernel, dim3(1), dim3(ST), 0, stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
