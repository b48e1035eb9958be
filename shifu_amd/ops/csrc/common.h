// Shared device helpers for the shifu_amd CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA 16x16x32 bf16 A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;    // MFMA 16x16 accumulator fragment
typedef uint16_t bf16_t;                                     // raw bf16 bits

#define SHIFU_API extern "C" __attribute__((visibility("default")))

static constexpr int WAVE = 64;   // CDNA wavefront: 64 lanes, never 32

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even f32 -> bf16 through the gfx950 hardware convert (v_cvt_pk_bf16_f32,
// emitted by hipcc for a plain cast; keeps NaN a NaN).  pack_bf16x2 converts two values with one
// instruction -- ~10x fewer VALU cycles per element than integer rounding on the f32 bits, which
// matters in the GEMM epilogues (64K conversions per 256x256 tile).
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------------------
// Activation functions, Encog/Shifu semantics (J/core/dtrain/DTrainUtils.java:303-386,
// J/core/dtrain/nn/Activation*.java).  derivative(b = pre-activation sum, a = output).
// ---------------------------------------------------------------------------------------
enum Act : int {
  ACT_SIGMOID = 0, ACT_TANH = 1, ACT_LINEAR = 2, ACT_RELU = 3, ACT_LEAKYRELU = 4,
  ACT_SWISH = 5, ACT_PTANH = 6, ACT_LOG = 7, ACT_SIN = 8,
  ACT_LEAKYRELU_TF = 9            // tf.nn.leaky_relu (alpha 0.2): the TENSORFLOW algorithm's leakyrelu
};

// Fast transcendental forms (v_exp_f32 + v_rcp_f32): the outputs are rounded to bf16 (8-bit
// mantissa) right after, so the ~1 ulp fp32 error of rcp/exp is invisible; tanh uses an odd
// polynomial near 0 to avoid the 1 - 2/(e^2x + 1) cancellation.
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_sigmoid(float x) { return fast_rcp(1.f + __expf(-x)); }
__device__ __forceinline__ float fast_tanh(float x) {
  const float x2 = x * x;
  const float poly = x * (1.f + x2 * (-0.333333333f + x2 * (0.133333333f + x2 * (-0.0539682540f + x2 * 0.0218694885f))));
  const float big = 1.f - 2.f * fast_rcp(__expf(2.f * x) + 1.f);
  return fabsf(x) < 0.3f ? poly : big;
}

__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case ACT_SIGMOID: return fast_sigmoid(x);
    case ACT_TANH: return fast_tanh(x);
    case ACT_LINEAR: return x;
    case ACT_RELU: return x <= 0.f ? 0.f : x;
    case ACT_LEAKYRELU: return x <= 0.f ? 0.01f * x : x;
    case ACT_SWISH: return x * fast_sigmoid(x);
    case ACT_PTANH: return x > 0.f ? fast_tanh(x) : 0.25f * fast_tanh(x);   // ActivationPTANH.java:54-59
    case ACT_LOG: return x >= 0.f ? __logf(1.f + x) : -__logf(1.f - x);
    case ACT_SIN: return __sinf(x);
    case ACT_LEAKYRELU_TF: return x <= 0.f ? 0.2f * x : x;
  }
  return x;
}

// fp32-accurate forms (libm expf/tanhf/log1pf/sinf) for outputs kept in fp32 (split-bf16 scoring)
__device__ __forceinline__ float act_fwd_precise(int act, float x) {
  switch (act) {
    case ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    case ACT_TANH: return tanhf(x);
    case ACT_SWISH: return x / (1.f + expf(-x));
    case ACT_PTANH: return x > 0.f ? tanhf(x) : 0.25f * tanhf(x);
    case ACT_LOG: return x >= 0.f ? log1pf(x) : -log1pf(-x);
    case ACT_SIN: return sinf(x);
  }
  return act_fwd(act, x);
}

// true when derivative can be computed from the activation output alone
__host__ __device__ constexpr inline bool act_deriv_from_output(int act) {
  return act == ACT_SIGMOID || act == ACT_TANH || act == ACT_LINEAR || act == ACT_RELU ||
         act == ACT_LEAKYRELU || act == ACT_LOG || act == ACT_PTANH || act == ACT_LEAKYRELU_TF;
}

// derivative given output a (only valid when act_deriv_from_output(act))
__device__ __forceinline__ float act_deriv_out(int act, float a) {
  switch (act) {
    case ACT_SIGMOID: return a * (1.f - a);
    case ACT_TANH: return 1.f - a * a;
    case ACT_LINEAR: return 1.f;
    case ACT_RELU: return a <= 0.f ? 0.f : 1.f;
    case ACT_LEAKYRELU: return a <= 0.f ? 0.01f : 1.f;
    case ACT_LOG: { float b = a >= 0.f ? __expf(a) - 1.f : 1.f - __expf(-a);
                    return b >= 0.f ? 1.f / (1.f + b) : 1.f / (1.f - b); }
    case ACT_PTANH: return a > 0.f ? 1.f - a * a : 0.25f * (1.f - 16.f * a * a);
    case ACT_LEAKYRELU_TF: return a <= 0.f ? 0.2f : 1.f;
  }
  return 1.f;
}

// derivative given pre-activation b (general)
__device__ __forceinline__ float act_deriv_pre(int act, float b) {
  switch (act) {
    case ACT_SWISH: { float s = 1.f / (1.f + __expf(-b)); return s + b * s * (1.f - s); }
    case ACT_SIN: return __cosf(b);
    default: return act_deriv_out(act, act_fwd(act, b));
  }
}

// Streaming row loop with U independent loads in flight per thread: the stats/quantile kernels
// are HBM-bound single passes, and one outstanding 8-byte load per lane leaves far too few bytes
// in flight per CU (Little's law at ~1 us HBM latency); loading U rows before processing any
// keeps U x the bytes in flight.  f(r, v) is called for every row r in [r0, r1) of this thread.
template <int U, typename F>
__device__ __forceinline__ void for_rows(const double* __restrict__ col, long r0, long r1, int stride, F&& f) {
  for (long rb = r0 + threadIdx.x; rb < r1; rb += (long)U * stride) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = rb + (long)u * stride;
      v[u] = r < r1 ? col[r] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = rb + (long)u * stride;
      if (r < r1) f(r, v[u]);
    }
  }
}
