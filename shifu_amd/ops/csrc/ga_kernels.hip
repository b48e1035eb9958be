// Population output heads for the voted (genetic) variable selection (algos/ga_varsel.py).
//
// The reference trains one small NN per seed (WrapperWorkerConductor / ValidationConductor
// J/core/dvarsel/wrapper/ValidationConductor.java:48-76, an Encog network per candidate column
// set).  Here the P seeds' first layers are one dense masked weight [P*H, K] on the MFMA GEMMs
// (gemm_kernels.hip forward, gemm_ring.hip wgrad); what remains per (row, seed) is the seed's own
// output neuron over its H hidden units -- H = 10 by default, far too narrow for a matrix core.
// This file does that part: one thread per seed walks a block of rows, so the H activations of a
// seed are contiguous 2H bytes and the 64 lanes of a wave read one contiguous span of a row.
//
//   train: z = sum_j h_j W2[p][j] + b2[p], o = sigmoid(z), dz = (y - o) o (1 - o) w  (ascent
//          direction, squared error), dH[n][p*H + j] = bf16(dz W2[p][j] f'(h_j)), and per-block
//          partials of the output-weight / bias gradients (sum over the block's rows of dz h_j,
//          dz), summed over blocks in a fixed order afterwards (deterministic, no atomics);
//   eval:  per-block partials of sum w (o - y)^2 per seed.
#include "common.h"

namespace {

constexpr int GA_ROWS = 256;                 // rows per block
constexpr int GA_T = 256;                    // threads (seeds) per block

template <int HMAX, bool TRAIN>
__global__ __launch_bounds__(GA_T) void ga_head_kernel(const bf16_t* __restrict__ Hs, long ldh, long n, int P, int H,
                                                       const float* __restrict__ W2, const float* __restrict__ b2,
                                                       const float* __restrict__ y, const float* __restrict__ w,
                                                       int act, bf16_t* __restrict__ dH, long lddh,
                                                       float* __restrict__ part) {
  const int p = blockIdx.x * GA_T + threadIdx.x;
  const long r0 = (long)blockIdx.y * GA_ROWS, r1 = min(n, r0 + GA_ROWS);
  if (p >= P) return;
  float w2[HMAX], g[HMAX];
#pragma unroll
  for (int j = 0; j < HMAX; ++j) {
    w2[j] = j < H ? W2[(long)p * H + j] : 0.f;
    g[j] = 0.f;
  }
  const float bb = b2[p];
  float gb = 0.f, err = 0.f;
  for (long r = r0; r < r1; ++r) {
    const bf16_t* hr = Hs + r * ldh + (long)p * H;
    float h[HMAX];
    float z = bb;
#pragma unroll
    for (int j = 0; j < HMAX; ++j) {
      h[j] = j < H ? bf2f(hr[j]) : 0.f;
      z += h[j] * w2[j];
    }
    const float o = 1.f / (1.f + __expf(-z));
    const float e = y[r] - o, wr = w[r];
    if constexpr (TRAIN) {
      const float dz = e * o * (1.f - o) * wr;
      gb += dz;
      bf16_t* dr = dH + r * lddh + (long)p * H;
#pragma unroll
      for (int j = 0; j < HMAX; ++j) {
        if (j < H) {
          g[j] += dz * h[j];
          dr[j] = f2bf(dz * w2[j] * act_deriv_out(act, h[j]));
        }
      }
    } else {
      err += wr * e * e;
    }
  }
  if constexpr (TRAIN) {
    const long base = (long)blockIdx.y * ((long)P * (H + 1));
#pragma unroll
    for (int j = 0; j < HMAX; ++j)
      if (j < H) part[base + (long)p * H + j] = g[j];
    part[base + (long)P * H + p] = gb;
  } else {
    part[(long)blockIdx.y * P + p] = err;
  }
}

// Any H (NumHiddenNodes > 64): the same math with nothing register-resident per hidden unit --
// z over the seed's H activations, then a second walk writing dH and accumulating the block's
// output-weight partials in place in `part` (each (block, seed) slot is owned by one thread, so
// the read-modify-writes are race-free and stay in L1/L2).  Same rounding order as above.
template <bool TRAIN>
__global__ __launch_bounds__(GA_T) void ga_head_any_kernel(const bf16_t* __restrict__ Hs, long ldh, long n, int P,
                                                           int H, const float* __restrict__ W2,
                                                           const float* __restrict__ b2, const float* __restrict__ y,
                                                           const float* __restrict__ w, int act,
                                                           bf16_t* __restrict__ dH, long lddh,
                                                           float* __restrict__ part) {
  const int p = blockIdx.x * GA_T + threadIdx.x;
  const long r0 = (long)blockIdx.y * GA_ROWS, r1 = min(n, r0 + GA_ROWS);
  if (p >= P) return;
  const float* w2 = W2 + (long)p * H;
  const long base = (long)blockIdx.y * ((long)P * (H + 1));
  float* g = part + base + (long)p * H;
  if constexpr (TRAIN)
    for (int j = 0; j < H; ++j) g[j] = 0.f;
  const float bb = b2[p];
  float gb = 0.f, err = 0.f;
  for (long r = r0; r < r1; ++r) {
    const bf16_t* hr = Hs + r * ldh + (long)p * H;
    float z = bb;
    for (int j = 0; j < H; ++j) z += bf2f(hr[j]) * w2[j];
    const float o = 1.f / (1.f + __expf(-z));
    const float e = y[r] - o, wr = w[r];
    if constexpr (TRAIN) {
      const float dz = e * o * (1.f - o) * wr;
      gb += dz;
      bf16_t* dr = dH + r * lddh + (long)p * H;
      for (int j = 0; j < H; ++j) {
        const float h = bf2f(hr[j]);
        g[j] += dz * h;
        dr[j] = f2bf(dz * w2[j] * act_deriv_out(act, h));
      }
    } else {
      err += wr * e * e;
    }
  }
  if constexpr (TRAIN) part[base + (long)P * H + p] = gb;
  else part[(long)blockIdx.y * P + p] = err;
}

// out[k] = sum over blocks b (ascending) of part[b][k]
__global__ __launch_bounds__(256) void ga_sum_blocks_kernel(const float* __restrict__ part, long nb, long k,
                                                            float* __restrict__ out, int accumulate) {
  const long j = (long)blockIdx.x * 256 + threadIdx.x;
  if (j >= k) return;
  float s = 0.f;
  for (long b = 0; b < nb; ++b) s += part[b * k + j];
  out[j] = accumulate ? out[j] + s : s;
}

}  // namespace

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

SHIFU_API long shifu_ga_part_floats(long n, int P, int H, int train) {
  const long nb = (n + GA_ROWS - 1) / GA_ROWS;
  return nb * (train ? (long)P * (H + 1) : (long)P);
}

// train != 0: dH [n][>= P*H] bf16 deltas and out[P*(H+1)] = output-weight then bias gradients
// (accumulated onto out when accumulate != 0); train == 0: out[P] = per-seed sum w (o - y)^2.
// part: >= shifu_ga_part_floats(n, P, H, train) floats of scratch.
SHIFU_API int shifu_ga_head(const void* Hs, long ldh, long n, int P, int H, const float* W2, const float* b2,
                            const float* y, const float* w, int act, void* dH, long lddh, float* part, float* out,
                            int train, int accumulate, hipStream_t stream) {
  if (n <= 0) return 0;
  if (P <= 0 || H <= 0 || ldh < (long)P * H || (train && (dH == nullptr || lddh < (long)P * H)))
    return -1;
  const long nb = (n + GA_ROWS - 1) / GA_ROWS;
  if (nb > 65535) return -1;
  const dim3 grid((P + GA_T - 1) / GA_T, (unsigned)nb);
#define GA_L(HM, TR) hipLaunchKernelGGL((ga_head_kernel<HM, TR>), grid, dim3(GA_T), 0, stream, (const bf16_t*)Hs, ldh, n, \
                                        P, H, W2, b2, y, w, act, (bf16_t*)dH, lddh, part)
#define GA_ANY(TR) hipLaunchKernelGGL((ga_head_any_kernel<TR>), grid, dim3(GA_T), 0, stream, (const bf16_t*)Hs, ldh, n, \
                                      P, H, W2, b2, y, w, act, (bf16_t*)dH, lddh, part)
  if (train) {
    if (H <= 16) GA_L(16, true); else if (H <= 64) GA_L(64, true); else GA_ANY(true);
  } else {
    if (H <= 16) GA_L(16, false); else if (H <= 64) GA_L(64, false); else GA_ANY(false);
  }
#undef GA_ANY
#undef GA_L
  const long k = train ? (long)P * (H + 1) : (long)P;
  hipLaunchKernelGGL(ga_sum_blocks_kernel, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, stream, part, nb, k, out,
                     accumulate);
  CHECK_HIP(hipGetLastError());
  return 0;
}
