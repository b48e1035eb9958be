// MLP row kernels for MI355X (gfx950): fused output layer/loss/delta, optimizer, weight casts.
// See gemm_kernels.hip for the layer GEMMs.
#include "common.h"

namespace {

constexpr int OUT_MAX = 8;
struct OutArgs {
  const bf16_t* H; long ldh;       // [M, KH]
  const bf16_t* Hd; long ldhd;     // optional stored hidden derivative
  const float* W;                  // [n_out, KH] fp32 (ld = KH)
  const float* Y; long ldy;        // [M, n_out] targets
  const float* S;                  // [M] significance (weights), nullable -> 1
  bf16_t* D; long ldd;             // [M, KH] hidden deltas out (nullable: no hidden layer dgrad)
  float* GW;                       // [n_out, KH] fp32 grads (atomic)
  double* err;                     // [2]: error sum, weight sum
  float* P; long ldp;              // optional predictions out [M, n_out]
  int M, KH, kh_valid, n_out, out_act, hid_act, loss, rows_per_wave;
  float flat_out, flat_hid;
};

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  f[0] = bf2f(v.x & 0xffff); f[1] = bf2f(v.x >> 16); f[2] = bf2f(v.y & 0xffff); f[3] = bf2f(v.y >> 16);
  f[4] = bf2f(v.z & 0xffff); f[5] = bf2f(v.z >> 16); f[6] = bf2f(v.w & 0xffff); f[7] = bf2f(v.w >> 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf16x2(f[0], f[1]);
  v.y = pack_bf16x2(f[2], f[3]);
  v.z = pack_bf16x2(f[4], f[5]);
  v.w = pack_bf16x2(f[6], f[7]);
  return v;
}

// LPR lanes per row (KH = 8*LPR), RPS = 64/LPR rows per wave step, U steps in flight.
template <int NOUT, int LPR>
__global__ __launch_bounds__(256) void mlp_output_kernel(OutArgs p) {
  constexpr int RPS = 64 / LPR, U = 4;
  const bool dfo = act_deriv_from_output(p.hid_act);   // wave-uniform
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, li = lane % LPR;
  const int c0 = li * 8;
  const long gw = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  float w[NOUT][8], gacc[NOUT][8];
#pragma unroll
  for (int o = 0; o < NOUT; ++o)
#pragma unroll
    for (int c = 0; c < 8; ++c) { w[o][c] = p.W[(size_t)o * p.KH + c0 + c]; gacc[o][c] = 0.f; }
  double esum = 0.0, wsum = 0.0;
  const long rows_per_iter = (long)RPS * U;
  for (long base = gw * rows_per_iter; base < p.M; base += nw * rows_per_iter) {
    uint4 hv[U], dv4[U];
    float yv[U][NOUT], sv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {          // issue every load of the U row-steps up front
      const long m = base + u * RPS + sub;
      const bool ok = m < p.M;
      hv[u] = ok ? *(const uint4*)(p.H + (size_t)m * p.ldh + c0) : make_uint4(0, 0, 0, 0);
      dv4[u] = (!dfo && ok && p.D) ? *(const uint4*)(p.Hd + (size_t)m * p.ldhd + c0) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int o = 0; o < NOUT; ++o) yv[u][o] = ok ? p.Y[(size_t)m * p.ldy + o] : 0.f;
      sv[u] = (ok && p.S) ? p.S[m] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long m = base + u * RPS + sub;
      const bool valid = m < p.M;
      float h[8];
      unpack8(hv[u], h);
      const float s = sv[u];
      float dlt[NOUT];
#pragma unroll
      for (int o = 0; o < NOUT; ++o) {
        float z = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) z += h[c] * w[o][c];
#pragma unroll
        for (int off = LPR / 2; off > 0; off >>= 1) z += __shfl_xor(z, off, 64);
        const float a = act_fwd(p.out_act, z);
        const float y = yv[u][o];
        const float e = y - a;
        if (p.P && valid && li == 0) p.P[(size_t)m * p.ldp + o] = a;
        float contrib;
        const int lm = p.loss % 3;                // loss >= 3: same deltas, TF objective as the error
        if (lm == 1) {              // log
          dlt[o] = e * s;
          const float ac = fminf(fmaxf(a, 1e-7f), 1.f - 1e-7f);
          contrib = p.loss >= 3 ? -(__logf(a + 1e-7f) * y + __logf(1.f - a + 1e-7f) * (1.f - y)) * s
                    : NOUT == 1 ? -(__logf(ac) * y + __logf(1.f - ac) * (1.f - y)) : -(__logf(ac) * y * s);
        } else if (lm == 2) {       // absolute
          dlt[o] = (y < a ? 1.f : -1.f) * (act_deriv_out(p.out_act, a) + p.flat_out) * s;
          contrib = fabsf(e) * s;
        } else {                    // squared (default)
          dlt[o] = (act_deriv_pre(p.out_act, z) + p.flat_out) * e * s;
          contrib = p.loss >= 3 ? e * e * s : (e * s) * (e * s);
        }
        if (!valid) dlt[o] = 0.f;
        if (valid && li == 0) esum += contrib;
      }
      if (valid && li == 0) wsum += s;
      float dsum[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) dsum[c] = 0.f;
#pragma unroll
      for (int o = 0; o < NOUT; ++o)
#pragma unroll
        for (int c = 0; c < 8; ++c) { dsum[c] += w[o][c] * dlt[o]; gacc[o][c] += dlt[o] * h[c]; }
      if (p.D && valid) {
        float dv[8], outv[8];
        if (dfo) {
#pragma unroll
          for (int c = 0; c < 8; ++c) dv[c] = act_deriv_out(p.hid_act, h[c]) + p.flat_hid;
        } else {
          unpack8(dv4[u], dv);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) outv[c] = (c0 + c) < p.kh_valid ? dsum[c] * dv[c] : 0.f;
        *(uint4*)(p.D + (size_t)m * p.ldd + c0) = pack8(outv);
      }
    }
  }
  // Reduce the gradient partials: over the RPS row-groups of the wave (shuffles), then over the
  // block's 4 waves (LDS), then ONE global atomic per column per block.  (Every block adding to
  // the same few hundred addresses is what made a naive per-wave atomic version 8x slower.)
  __shared__ float red[4][512];
  __shared__ double ered[4][2];
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float v = gacc[o][c];
#pragma unroll
      for (int off = LPR; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
      if (sub == 0) red[wv][c0 + c] = v;
    }
    __syncthreads();
    for (int col = threadIdx.x; col < p.KH; col += blockDim.x) {
      const float v = red[0][col] + red[1][col] + red[2][col] + red[3][col];
      atomicAdd(p.GW + (size_t)o * p.KH + col, v);
    }
    __syncthreads();
  }
  esum = wave_sum_d(esum);
  wsum = wave_sum_d(wsum);
  if (lane == 0) { ered[wv][0] = esum; ered[wv][1] = wsum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(p.err, ered[0][0] + ered[1][0] + ered[2][0] + ered[3][0]);
    atomicAdd(p.err + 1, ered[0][1] + ered[1][1] + ered[2][1] + ered[3][1]);
  }
}

// ---------------------------------------------------------------------------------------
// Output layer for ANY last-hidden width and ANY number of outputs (the row kernel above keeps
// every output's weights and gradient partials in registers: KH <= 512, n_out <= 8).  The
// reference builds any width / output count (J/core/dtrain/DTrainUtils.java:303-386; one output
// node per tag for NATIVE multi-class, ModelConfig.java:381-384), so this path has no limit but LDS.
//
// One wave per row, grid-stride.  Outputs in groups of 8: z over the row's 8-column groups (lane
// owns groups lane, lane + 64, ...; the H row is re-read from L1/L2 per output group), summed
// across the wave by xor shuffles, then activation / loss / output deltas computed redundantly by
// every lane; lane 0 stages the row's deltas in LDS (one n_out-float strip per wave) and stores
// them bf16 into L [M, ldl] (zero padded to ldl) for the output wgrad GEMM (GW += L^T H, wgrad_tn,
// called by the launcher).  Then the hidden deltas D = (sum_o dlt_o W[o]) * (f'(H) + flat) per
// column group, W rows read fp32 from L2 (n_out x KH x 4 B, shared by every wave).
// ---------------------------------------------------------------------------------------
struct WideArgs {
  const bf16_t* H; long ldh;
  const bf16_t* Hd; long ldhd;
  const float* W;                  // [n_out, KH] fp32
  const float* Y; long ldy;
  const float* S;
  bf16_t* D; long ldd;             // hidden deltas (nullable)
  bf16_t* L; long ldl;             // output deltas bf16 (nullable)
  double* err;
  float* P; long ldp;              // predictions (nullable)
  int M, KH, kh_valid, n_out, out_act, hid_act, loss;
  float flat_out, flat_hid;
};

__global__ __launch_bounds__(256) void mlp_output_wide_kernel(WideArgs p) {
  extern __shared__ float dl_lds[];                 // [4][n_out]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* dl = dl_lds + (size_t)wv * p.n_out;
  const bool dfo = act_deriv_from_output(p.hid_act);
  const long wave0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  const int ngroups = p.KH / 8;
  const int lm = p.loss % 3;
  double esum = 0.0, wsum = 0.0;
  for (long m = wave0; m < p.M; m += nwaves) {
    const bf16_t* hrow = p.H + (size_t)m * p.ldh;
    const float s = p.S ? p.S[m] : 1.f;
    for (int og = 0; og < p.n_out; og += 8) {
      float z[8];
#pragma unroll
      for (int o = 0; o < 8; ++o) z[o] = 0.f;
      for (int g = lane; g < ngroups; g += 64) {
        float h[8];
        unpack8(*(const uint4*)(hrow + g * 8), h);
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          const int oo = min(og + o, p.n_out - 1);             // clamped: branch-free loads
          const float4* wp = (const float4*)(p.W + (size_t)oo * p.KH + g * 8);
          const float4 w0 = wp[0], w1 = wp[1];
          z[o] += h[0] * w0.x + h[1] * w0.y + h[2] * w0.z + h[3] * w0.w +
                  h[4] * w1.x + h[5] * w1.y + h[6] * w1.z + h[7] * w1.w;
        }
      }
#pragma unroll
      for (int o = 0; o < 8; ++o)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) z[o] += __shfl_xor(z[o], off, 64);
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        const int oi = og + o;
        if (oi >= p.n_out) {
          if (p.L && lane == 0 && oi < p.ldl) p.L[(size_t)m * p.ldl + oi] = (bf16_t)0;
          continue;
        }
        const float a = act_fwd(p.out_act, z[o]);
        const float y = p.Y[(size_t)m * p.ldy + oi];
        const float e = y - a;
        float d, contrib;
        if (lm == 1) {
          d = e * s;
          const float ac = fminf(fmaxf(a, 1e-7f), 1.f - 1e-7f);
          contrib = p.loss >= 3 ? -(__logf(a + 1e-7f) * y + __logf(1.f - a + 1e-7f) * (1.f - y)) * s
                    : p.n_out == 1 ? -(__logf(ac) * y + __logf(1.f - ac) * (1.f - y)) : -(__logf(ac) * y * s);
        } else if (lm == 2) {
          d = (y < a ? 1.f : -1.f) * (act_deriv_out(p.out_act, a) + p.flat_out) * s;
          contrib = fabsf(e) * s;
        } else {
          d = (act_deriv_pre(p.out_act, z[o]) + p.flat_out) * e * s;
          contrib = p.loss >= 3 ? e * e * s : (e * s) * (e * s);
        }
        if (lane == 0) {
          esum += contrib;
          dl[oi] = d;
          if (p.L) p.L[(size_t)m * p.ldl + oi] = f2bf(d);
          if (p.P) p.P[(size_t)m * p.ldp + oi] = a;
        }
      }
    }
    if (lane == 0) wsum += s;
    if (p.D) {
      __builtin_amdgcn_s_waitcnt(0xc07f);          // lane 0's LDS stores of dl (lgkmcnt(0))
      __builtin_amdgcn_wave_barrier();
      for (int g = lane; g < ngroups; g += 64) {
        float ds[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) ds[c] = 0.f;
        for (int o = 0; o < p.n_out; ++o) {
          const float d = dl[o];
          const float4* wp = (const float4*)(p.W + (size_t)o * p.KH + g * 8);
          const float4 w0 = wp[0], w1 = wp[1];
          ds[0] += d * w0.x; ds[1] += d * w0.y; ds[2] += d * w0.z; ds[3] += d * w0.w;
          ds[4] += d * w1.x; ds[5] += d * w1.y; ds[6] += d * w1.z; ds[7] += d * w1.w;
        }
        float h[8], dv[8], outv[8];
        if (dfo) {
          unpack8(*(const uint4*)(hrow + g * 8), h);
#pragma unroll
          for (int c = 0; c < 8; ++c) dv[c] = act_deriv_out(p.hid_act, h[c]) + p.flat_hid;
        } else {
          unpack8(*(const uint4*)(p.Hd + (size_t)m * p.ldhd + g * 8), dv);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) outv[c] = (g * 8 + c) < p.kh_valid ? ds[c] * dv[c] : 0.f;
        *(uint4*)(p.D + (size_t)m * p.ldd + g * 8) = pack8(outv);
      }
      __builtin_amdgcn_wave_barrier();             // dl reads done before the next row's stores
    }
  }
  __shared__ double ered[4][2];
  esum = wave_sum_d(esum);
  wsum = wave_sum_d(wsum);
  if (lane == 0) { ered[wv][0] = esum; ered[wv][1] = wsum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(p.err, ered[0][0] + ered[1][0] + ered[2][0] + ered[3][0]);
    atomicAdd(p.err + 1, ered[0][1] + ered[1][1] + ered[2][1] + ered[3][1]);
  }
}

// ---------------------------------------------------------------------------------------
// Optimizer: one fused pass over the flat fp32 weights (J/core/dtrain/Weight.java:194-343,
// J/core/dtrain/nn/update/*.java).  Gradients are Encog ascent directions: every rule ADDS.
// ---------------------------------------------------------------------------------------
enum Rule : int { R_BACKPROP = 0, R_QUICK = 1, R_MANHATTAN = 2, R_RPROP = 3, R_ADAM = 4, R_ADAGRAD = 5,
                  R_RMSPROP = 6, R_MOMENTUM = 7, R_NESTEROV = 8,
                  R_RMSPROP_TF = 9 };   // tf.train.RMSPropOptimizer: c = rho c + (1 - rho) g^2 (train.py)
struct OptArgs {
  float* w; const float* g; float* s0; float* s1; float* s2; const uint8_t* fixed;
  long n; int rule, reg_level;     // reg_level 0 none, 1 L1, 2 L2 (legacy rules only)
  float lr, momentum, beta1, beta2, decay_rate, reg, num_train, q_eps, q_shrink, q_decay;
  int iteration;
  // TENSORFLOW algorithm (models/dnn_sgd.py): the accumulated Encog-direction gradient is scaled to
  // the mean loss of the batch (gscale) and the L2 term of tf.contrib.layers.l2_regularizer is
  // folded in on the weight entries (l2mask: 1 for weights, 0 for biases / padding)
  float gscale, l2; const uint8_t* l2mask;
};

__device__ __forceinline__ int sgn_tol(float v) { return fabsf(v) < 1e-7f ? 0 : (v > 0.f ? 1 : -1); }

__global__ void optimizer_kernel(OptArgs a) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  if (a.fixed && a.fixed[i]) return;
  float w = a.w[i];
  float g = a.g[i] * a.gscale;
  if (a.l2mask && a.l2mask[i]) g -= a.l2 * w;
  float delta = 0.f;
  switch (a.rule) {
    case R_BACKPROP: delta = g * a.lr + a.s0[i] * a.momentum; a.s0[i] = delta; break;
    case R_MANHATTAN: delta = fabsf(g) < 1e-17f ? 0.f : (g > 0.f ? a.lr : -a.lr); break;
    case R_QUICK: {
      const float d = a.s0[i], s = -g + a.q_decay * w, pp = -a.s1[i];
      float ns = 0.f;
      if (d < 0.f) { if (s > 0.f) ns -= a.q_eps * s; ns += (s >= a.q_shrink * pp) ? a.lr * d : d * s / (pp - s); }
      else if (d > 0.f) { if (s < 0.f) ns -= a.q_eps * s; ns += (s <= a.q_shrink * pp) ? a.lr * d : d * s / (pp - s); }
      else ns -= a.q_eps * s;
      a.s0[i] = ns; a.s1[i] = g; delta = ns; break;
    }
    case R_RPROP: {    // s0 = lastDelta, s1 = lastGradient, s2 = updateValues
      const int ch = sgn_tol(g * a.s1[i]);
      if (ch > 0) { float d = fminf(a.s2[i] * 1.2f, 50.f); delta = sgn_tol(g) * d; a.s2[i] = d; a.s1[i] = g; }
      else if (ch < 0) { float d = fmaxf(a.s2[i] * 0.5f, 1e-6f); a.s2[i] = d; delta = -a.s0[i]; a.s1[i] = 0.f; }
      else { delta = sgn_tol(g) * a.s2[i]; a.s1[i] = g; }
      a.s0[i] = delta; break;
    }
    case R_ADAM: {
      const float m = a.beta1 * a.s0[i] + (1.f - a.beta1) * g;
      const float v = a.beta2 * a.s1[i] + (1.f - a.beta2) * g * g;
      a.s0[i] = m; a.s1[i] = v;
      const float mc = m / (1.f - powf(a.beta1, (float)a.iteration));
      const float vc = v / (1.f - powf(a.beta2, (float)a.iteration));
      a.w[i] = w + a.lr * mc / (sqrtf(vc) + 1e-8f); return;
    }
    case R_ADAGRAD: { const float c = a.s0[i] + g * g; a.s0[i] = c; a.w[i] = w + a.lr * g / (sqrtf(c) + 1e-8f); return; }
    case R_RMSPROP: {  // RMSPropUpdate.java: cache += g^2 then cache = d*cache + (1-d) g^2
      float c = a.s0[i] + g * g; c = a.decay_rate * c + (1.f - a.decay_rate) * g * g; a.s0[i] = c;
      a.w[i] = w + a.lr * g / (sqrtf(c) + 1e-8f); return;
    }
    case R_MOMENTUM: { const float d = a.lr * g + a.momentum * a.s0[i]; a.s0[i] = d; a.w[i] = w + d; return; }
    case R_RMSPROP_TF: {
      const float c = a.decay_rate * a.s0[i] + (1.f - a.decay_rate) * g * g; a.s0[i] = c;
      a.w[i] = w + a.lr * g / (sqrtf(c) + 1e-10f); return;
    }
    case R_NESTEROV: {
      const float prev = a.s0[i]; const float ld = a.momentum * prev + g * a.lr; a.s0[i] = ld;
      a.w[i] = w + a.momentum * prev - (1.f + a.momentum) * ld; return;
    }
  }
  if (a.reg_level == 1 && a.reg != 0.f) {
    const float sh = a.reg / a.num_train;
    w = (delta > 0.f ? 1.f : (delta < 0.f ? -1.f : 0.f)) * fmaxf(0.f, fabsf(delta) - sh);
  } else if (a.reg_level == 2) {
    w += delta - a.reg * w / a.num_train;
  } else {
    w += delta;
  }
  a.w[i] = w;
}

// fp32 [R][C] (ld ldw) -> bf16 [R][C] (ld ldo)
__global__ void cast_bf16_kernel(const float* W, long ldw, bf16_t* O, long ldo, int R, int C) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)R * C) return;
  const int r = i / C, c = i % C;
  O[(size_t)r * ldo + c] = f2bf(W[(size_t)r * ldw + c]);
}
// fp32 W [R][C] -> bf16 WT [C][Rpad] (zero for r >= R)
__global__ void transpose_cast_kernel(const float* W, long ldw, bf16_t* O, int R, int C, int Rpad) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)C * Rpad) return;
  const int c = i / Rpad, r = i % Rpad;
  O[i] = r < R ? f2bf(W[(size_t)r * ldw + c]) : (bf16_t)0;
}

}  // namespace

// =======================================================================================
// C ABI (called through ctypes; host-side shape checks live in shifu_amd/ops/mlp.py and
// are repeated here so a bad call fails loudly instead of faulting the GPU).
// =======================================================================================
#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

static long g_out_waves = 8192;   // output-kernel grid cap in waves (tuning knob)
SHIFU_API int shifu_mlp_set_out_waves(int w) { g_out_waves = w >= 64 ? w : 4096; return 0; }

SHIFU_API int shifu_mlp_output(const void* H, long ldh, const void* Hd, long ldhd, const float* W, const float* Y,
                               long ldy, const float* S, void* D, long ldd, float* GW, double* err, float* P,
                               long ldp, int M, int KH, int kh_valid, int n_out, int out_act, int hid_act, int loss,
                               float flat_out, float flat_hid, hipStream_t stream) {
  if (KH % 64 || KH > 512 || n_out < 1 || n_out > OUT_MAX || M <= 0) return -1;
  if (D && !act_deriv_from_output(hid_act) && Hd == nullptr) return -3;
  OutArgs p{(const bf16_t*)H, ldh, (const bf16_t*)Hd, ldhd, W, Y, ldy, S, (bf16_t*)D, ldd, GW, err, P, ldp,
            M, KH, kh_valid, n_out, out_act, hid_act, loss, 0, flat_out, flat_hid};
  const int lpr = KH / 8;
  const long rows_per_wave_iter = (64 / lpr) * 4;
  long waves = (M + rows_per_wave_iter - 1) / rows_per_wave_iter;
  if (waves > g_out_waves) waves = g_out_waves;   // grid-stride cap (blocks x 4 waves)
  const long blocks = (waves + 3) / 4;
  // dispatch on (n_out, lanes-per-row)
#define OUT_L(NO, L) hipLaunchKernelGGL((mlp_output_kernel<NO, L>), dim3(blocks), dim3(256), 0, stream, p)
#define OUT_LPR(NO) switch (lpr) { case 8: OUT_L(NO, 8); break; case 16: OUT_L(NO, 16); break; \
    case 32: OUT_L(NO, 32); break; case 64: OUT_L(NO, 64); break; default: return -1; }
  switch (n_out) {
    case 1: OUT_LPR(1) break; case 2: OUT_LPR(2) break; case 3: OUT_LPR(3) break; case 4: OUT_LPR(4) break;
    case 5: OUT_LPR(5) break; case 6: OUT_LPR(6) break; case 7: OUT_LPR(7) break; default: OUT_LPR(8) break;
  }
#undef OUT_LPR
#undef OUT_L
  CHECK_HIP(hipGetLastError());
  return 0;
}

// gemm_kernels.hip (same library): split-K TN wgrad G[Nv, Kx] += D^T X
extern "C" int shifu_wgrad_tn(const void* D, long ldd, const void* X, long ldx, float* G, long ldg, int M, int Nv,
                              int Kx, int splits, hipStream_t stream);

// Any-shape output layer: row kernel (deltas, hidden deltas, errors, predictions) + the output
// wgrad GW [n_out, KH] += L^T H on the TN GEMM when GW is given (L [M, ldl] bf16 workspace,
// ldl >= round_up(n_out, 8)).
SHIFU_API int shifu_mlp_output_wide(const void* H, long ldh, const void* Hd, long ldhd, const float* W,
                                    const float* Y, long ldy, const float* S, void* D, long ldd, void* L,
                                    long ldl, float* GW, double* err, float* P, long ldp, int M, int KH,
                                    int kh_valid, int n_out, int out_act, int hid_act, int loss, float flat_out,
                                    float flat_hid, hipStream_t stream) {
  if (KH % 128 || KH < 128 || ldh < KH || ldh % 8 || n_out < 1 || n_out > 8192 || M <= 0) return -1;
  if (D && (ldd < KH || ldd % 8)) return -1;
  if (GW && (L == nullptr || ldl < ((n_out + 7) / 8) * 8 || ldl % 8)) return -1;
  if (D && !act_deriv_from_output(hid_act) && Hd == nullptr) return -3;
  WideArgs p{(const bf16_t*)H, ldh, (const bf16_t*)Hd, ldhd, W, Y, ldy, S, (bf16_t*)D, ldd,
             GW ? (bf16_t*)L : nullptr, ldl, err, P, ldp, M, KH, kh_valid, n_out, out_act, hid_act, loss,
             flat_out, flat_hid};
  long blocks = (M + 3) / 4;
  if (blocks > 4096) blocks = 4096;                 // 16 waves per CU, grid-stride over rows
  const size_t lds = (size_t)4 * n_out * sizeof(float);
  hipLaunchKernelGGL(mlp_output_wide_kernel, dim3(blocks), dim3(256), lds, stream, p);
  CHECK_HIP(hipGetLastError());
  if (GW) {
    int splits = M / 2048;
    const int tiles = ((n_out + 127) / 128) * (KH / 128);
    if (splits > 1024 / tiles) splits = 1024 / tiles;
    if (splits < 1) splits = 1;
    const int r = shifu_wgrad_tn(L, ldl, H, ldh, GW, KH, M, n_out, KH, splits, stream);
    if (r) return r;
  }
  return 0;
}

SHIFU_API int shifu_optimizer_step(float* w, const float* g, float* s0, float* s1, float* s2, const uint8_t* fixed,
                                   long n, int rule, int reg_level, float lr, float momentum, float beta1,
                                   float beta2, float decay_rate, float reg, float num_train, float q_eps,
                                   float q_shrink, float q_decay, int iteration, hipStream_t stream) {
  OptArgs a{w, g, s0, s1, s2, fixed, n, rule, reg_level, lr, momentum, beta1, beta2, decay_rate, reg, num_train,
            q_eps, q_shrink, q_decay, iteration, 1.f, 0.f, nullptr};
  hipLaunchKernelGGL(optimizer_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// TENSORFLOW-algorithm update: g' = gscale * g - l2 * w * l2mask, then `rule` (ADAM / momentum-free
// gradient descent / RMSPROP_TF) with the TF hyper-parameters.
SHIFU_API int shifu_optimizer_step_tf(float* w, const float* g, float* s0, float* s1, long n, int rule, float lr,
                                      float beta1, float beta2, float decay_rate, float gscale, float l2,
                                      const uint8_t* l2mask, int iteration, hipStream_t stream) {
  if (rule != R_ADAM && rule != R_MOMENTUM && rule != R_RMSPROP_TF) return -1;
  OptArgs a{w, g, s0, s1, nullptr, nullptr, n, rule, 0, lr, 0.f, beta1, beta2, decay_rate, 0.f, 1.f,
            0.f, 0.f, 0.f, iteration, gscale, l2, l2mask};
  hipLaunchKernelGGL(optimizer_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_cast_bf16(const float* W, long ldw, void* O, long ldo, int R, int C, hipStream_t stream) {
  const long n = (long)R * C;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, W, ldw, (bf16_t*)O, ldo, R, C);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_transpose_cast(const float* W, long ldw, void* O, int R, int C, int Rpad, hipStream_t stream) {
  const long n = (long)C * Rpad;
  hipLaunchKernelGGL(transpose_cast_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, W, ldw, (bf16_t*)O, R, C,
                     Rpad);
  CHECK_HIP(hipGetLastError());
  return 0;
}
