// Fused MLP tail for MI355X (gfx950): last hidden layer forward + output layer + loss + output
// delta/wgrad + last hidden delta + backward GEMM into the previous hidden layer, per 128-row tile.
//
// Replaces, for the last hidden layer L-1 of a Shifu NN (J/core/dtrain/nn/SubGradient.java:224-311,
// J/core/dtrain/dataset/FloatFlatNetwork.java:69-223), four launches of the unfused path
//   z = h W^T (GEMM, gemm_kernels.hip)  ->  a = act(z) -> HBM
//   output layer + loss + delta_out + output wgrad + d = (delta_out W_out) f'(a)  (mlp_kernels.hip)
//   d_prev = (d W) f'(h)  (dgrad GEMM, gemm_kernels.hip)
// with one persistent kernel: the a tile never leaves the CU, d stays in LDS as the A operand of
// the backward GEMM, and only what later kernels need goes to HBM (d for the layer's wgrad,
// d_prev for the wgrad below).  Numerics match the unfused path: a is rounded to bf16 before
// the output layer reads it, output-layer math in fp32, deltas rounded to bf16.
//
// Block = 512 threads (8 waves, 2 M x 4 N), 128 rows x 256 hidden units per tile, 1 block / CU.
// LDS map (148 KiB): [0, 96K) forward k-tile double buffer (A 16K + B 32K per stage), reused as
// [0, 64K) d image (4 k-tiles [128][64] bf16, swizzled) + [64K, 128K) backward W double buffer /
// output-dot scratch / epilogue staging; [128K, 148K) per-block output-layer state.
#include "common.h"

namespace {

constexpr int TT = 512, TR = 128, TN = 256;
constexpr int T_OUTMAX = 8;
constexpr int L_FWD_A = 16384, L_FWD_STAGE = 49152;
constexpr int L_DIMG = 0, L_BWD = 65536, L_STATE = 131072;
constexpr int L_TOTAL = L_STATE + 4096 /*dl*/ + 8192 /*wout*/ + 8192 /*gacc*/;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

struct TailArgs {
  const bf16_t* H; long ldh;      // [M, KA] input of the last hidden layer (acts[L-1])
  const bf16_t* W; int nh;        // [nh, KA] bf16 weights of the last hidden layer (nh valid units)
  int KA, act_h;                  // KA multiple of 64; act of the last hidden layer
  float flat_h;
  const float* Wout;              // [n_out, KH] fp32 output weights (KH = TN padded hidden width)
  int KH;                         // <= 256, multiple of 64
  const float* Y; long ldy;       // [M, n_out]
  const float* S;                 // [M] significance, nullable
  int n_out, out_act, loss;
  float flat_out;
  bf16_t* D; long ldd;            // out: [M, KH] last hidden deltas
  float* GW;                      // [n_out, KH] output-layer gradient (atomic, once per block)
  double* err;                    // [2] error sum, weight sum
  // backward into the previous layer (do_bwd): Dp = (D Wt^T) * (f'(H) + flat_p) on cols < np_valid
  int do_bwd;
  const bf16_t* Wt; long ldwt;    // [KA, KH] bf16 (transposed weights of the last hidden layer)
  bf16_t* Dp; long lddp;          // out: [M, KA]
  int act_p, np_valid;
  float flat_p;
  int M;
};

__global__ __launch_bounds__(TT, 1) void mlp_tail_kernel(TailArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* dl_s = (float*)(smem + L_STATE);                   // [TR][T_OUTMAX]
  float* wo_s = (float*)(smem + L_STATE + 4096);            // [T_OUTMAX][TN]
  float* ga_s = (float*)(smem + L_STATE + 4096 + 8192);     // [T_OUTMAX][TN]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int lr = lane & 15, lq = lane >> 4;
  const int n_out = p.n_out;

  for (int i = tid; i < T_OUTMAX * TN; i += TT) {
    const int o = i / TN, n = i % TN;
    wo_s[i] = (o < n_out && n < p.KH) ? p.Wout[(size_t)o * p.KH + n] : 0.f;
    ga_s[i] = 0.f;
  }
  double esum = 0.0, wsum = 0.0;

  const int n_tiles = (p.M + TR - 1) / TR;
  const int nkA = p.KA / 64, nkB = p.KH / 64;
  for (int tile = xcd_remap(blockIdx.x, gridDim.x); tile < n_tiles; tile += gridDim.x) {
    const int m0 = tile * TR;
    __syncthreads();                                       // previous tile done with every LDS area

    // ---------------- phase A: Z[128 x 256] = H_tile W^T over KA ----------------
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto dmaA = [&](int kt, int buf) {
      char* base = smem + buf * L_FWD_STAGE;
#pragma unroll
      for (int i = 0; i < 6; ++i) {                       // 2 x 8 KiB of H, 4 x 8 KiB of W
        const int P = (i & 1) * 8192 + wid * 1024 + lane * 16;
        const int row = P >> 7, lc = ((P >> 4) & 7) ^ ((row >> 1) & 7);
        const bf16_t* src;
        char* dst;
        if (i < 2) {
          src = p.H + (size_t)min(m0 + row, p.M - 1) * p.ldh + kt * 64 + lc * 8;
          dst = base + i * 8192 + wid * 1024;
        } else {
          const int wrow = (i >> 1) * 64 + row - 64;       // i = 2,3 -> rows 0..127; 4,5 -> 128..255
          const int wrow2 = (i < 4 ? 0 : 128) + row;
          (void)wrow;
          src = p.W + (size_t)min(wrow2, p.nh - 1) * p.KA + kt * 64 + lc * 8;
          dst = base + L_FWD_A + (i - 2) * 8192 + wid * 1024;
        }
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)dst, 16, 0, 0);
      }
    };
    dmaA(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nkA; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nkA) dmaA(kt + 1, buf ^ 1);
      const char* As = smem + buf * L_FWD_STAGE;
      const char* Bs = As + L_FWD_A;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        bf16x8 af[4], bq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) af[j] = *(const bf16x8*)(As + swz(wr * 64 + j * 16 + lr, c * 4 + lq));
#pragma unroll
        for (int i = 0; i < 4; ++i) bq[i] = *(const bf16x8*)(Bs + swz(wc * 64 + i * 16 + lr, c * 4 + lq));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[i], af[j], acc[i][j], 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }

    // ---------------- phase B: a = bf16(act(z)), output layer, loss, delta_out ----------------
    // lane element acc[i][j][r]: unit n = 64 wc + 16 i + 4 lq + r, tile row m = 64 wr + 16 j + lr
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wc * 64 + i * 16 + lq * 4 + r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float z = acc[i][j][r];
          const float a = n < p.nh ? bf2f(f2bf(act_fwd(p.act_h, z))) : (n == p.nh ? 1.f : 0.f);
          acc[i][j][r] = a;
        }
      }
    float* red = (float*)(smem + L_BWD);                   // [4 wc][TR][T_OUTMAX]
    for (int o = 0; o < n_out; ++o) {
      float4 wv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) wv[i] = *(const float4*)(wo_s + o * TN + wc * 64 + i * 16 + lq * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          s += acc[i][j][0] * wv[i].x + acc[i][j][1] * wv[i].y + acc[i][j][2] * wv[i].z + acc[i][j][3] * wv[i].w;
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (lq == 0) red[(wc * TR + wr * 64 + j * 16 + lr) * T_OUTMAX + o] = s;
      }
    }
    __syncthreads();
    if (tid < TR) {
      const int m = m0 + tid;
      const bool valid = m < p.M;
      const float sv = (valid && p.S) ? p.S[m] : 1.f;
      for (int o = 0; o < n_out; ++o) {
        const float z = red[(0 * TR + tid) * T_OUTMAX + o] + red[(1 * TR + tid) * T_OUTMAX + o] +
                        red[(2 * TR + tid) * T_OUTMAX + o] + red[(3 * TR + tid) * T_OUTMAX + o];
        const float a = act_fwd(p.out_act, z);
        const float y = valid ? p.Y[(size_t)m * p.ldy + o] : 0.f;
        const float e = y - a;
        float dlt, contrib;
        if (p.loss == 1) {
          dlt = e * sv;
          const float ac = fminf(fmaxf(a, 1e-7f), 1.f - 1e-7f);
          contrib = n_out == 1 ? -(__logf(ac) * y + __logf(1.f - ac) * (1.f - y)) : -(__logf(ac) * y * sv);
        } else if (p.loss == 2) {
          dlt = (y < a ? 1.f : -1.f) * (act_deriv_out(p.out_act, a) + p.flat_out) * sv;
          contrib = fabsf(e) * sv;
        } else {
          dlt = (act_deriv_pre(p.out_act, z) + p.flat_out) * e * sv;
          contrib = (e * sv) * (e * sv);
        }
        dl_s[tid * T_OUTMAX + o] = valid ? dlt : 0.f;
        if (valid) esum += contrib;
      }
      if (valid) wsum += sv;
    }
    __syncthreads();

    // ---------------- phase C: output wgrad, d = (dl W_out) f'(a) -> HBM + LDS image ----------------
    float dlr[4][T_OUTMAX];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int o = 0; o < T_OUTMAX; ++o) dlr[j][o] = o < n_out ? dl_s[(wr * 64 + j * 16 + lr) * T_OUTMAX + o] : 0.f;
    for (int o = 0; o < n_out; ++o) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float g = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) g += dlr[j][o] * acc[i][j][r];
          g += __shfl_xor(g, 1, 64);
          g += __shfl_xor(g, 2, 64);
          g += __shfl_xor(g, 4, 64);
          g += __shfl_xor(g, 8, 64);
          if (lr == 0) atomicAdd(ga_s + o * TN + wc * 64 + i * 16 + lq * 4 + r, g);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = wc * 64 + i * 16 + lq * 4;
      float wo[T_OUTMAX][4];
#pragma unroll
      for (int o = 0; o < T_OUTMAX; ++o) {
        const float4 v = *(const float4*)(wo_s + o * TN + nb);
        wo[o][0] = v.x; wo[o][1] = v.y; wo[o][2] = v.z; wo[o][3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = wr * 64 + j * 16 + lr;
        float dv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float ds = 0.f;
#pragma unroll
          for (int o = 0; o < T_OUTMAX; ++o) ds += dlr[j][o] * wo[o][r];
          dv[r] = (nb + r) < p.nh ? ds * (act_deriv_out(p.act_h, acc[i][j][r]) + p.flat_h) : 0.f;
        }
        uint2 w2;
        w2.x = pack_bf16x2(dv[0], dv[1]);
        w2.y = pack_bf16x2(dv[2], dv[3]);
        const int kt = nb >> 6, ch = (nb & 63) >> 3, half = (nb >> 2) & 1;
        *(uint2*)(smem + L_DIMG + kt * 16384 + swz(ml, ch) + half * 8) = w2;
      }
    }
    __syncthreads();
    // coalesced copy of the d image rows to HBM (only the KH valid columns)
    for (int idx = tid; idx < TR * (p.KH / 8); idx += TT) {
      const int row = idx / (p.KH / 8), c = idx % (p.KH / 8);
      const int m = m0 + row;
      if (m < p.M)
        *(uint4*)(p.D + (size_t)m * p.ldd + c * 8) = *(const uint4*)(smem + L_DIMG + (c >> 3) * 16384 + swz(row, c & 7));
    }
    if (!p.do_bwd) continue;

    // ---------------- phase D: Dp[128 x KA] = D W (NT with Wt), * f'(H), 256 columns per pass ----------------
    for (int n0 = 0; n0 < p.KA; n0 += TN) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto dmaB = [&](int kt, int buf) {
        char* base = smem + L_BWD + buf * 32768;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int P = (i & 1) * 8192 + wid * 1024 + lane * 16;
          const int row = (i >> 1) * 128 + (P >> 7), lc = ((P >> 4) & 7) ^ (((P >> 7) >> 1) & 7);
          const bf16_t* src = p.Wt + (size_t)min(n0 + row, p.KA - 1) * p.ldwt + kt * 64 + lc * 8;
          __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(base + i * 8192 + wid * 1024), 16, 0, 0);
        }
      };
      __syncthreads();                                     // scratch / previous pass done with L_BWD
      dmaB(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int kt = 0; kt < nkB; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nkB) dmaB(kt + 1, buf ^ 1);
        const char* As = smem + L_DIMG + kt * 16384;
        const char* Bs = smem + L_BWD + buf * 32768;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          bf16x8 af[4], bq[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) af[j] = *(const bf16x8*)(As + swz(wr * 64 + j * 16 + lr, c * 4 + lq));
#pragma unroll
          for (int i = 0; i < 4; ++i) bq[i] = *(const bf16x8*)(Bs + swz(wc * 64 + i * 16 + lr, c * 4 + lq));
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[i], af[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      // staged epilogue: [128][256] bf16 tile in L_BWD ([128][512 B], chunk ^ (row & 15)), then
      // 16-B row segments with the matching H segment for the derivative
      char* Cs = smem + L_BWD;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nl = wc * 64 + i * 16 + lq * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ml = wr * 64 + j * 16 + lr;
          uint2 w2;
          w2.x = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
          w2.y = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
          const int c = nl >> 3, half = (nl >> 2) & 1;
          *(uint2*)(Cs + ml * 512 + ((c ^ (ml & 15)) << 4) + half * 8) = w2;
        }
      }
      __syncthreads();
      const int c = tid & 31;
#pragma unroll 2
      for (int pass = 0; pass < 8; ++pass) {
        const int ml = pass * 16 + (tid >> 5);
        const int m = m0 + ml, n = n0 + c * 8;
        if (m >= p.M || n >= p.KA) continue;
        const uint4 v = *(const uint4*)(Cs + ml * 512 + ((c ^ (ml & 15)) << 4));
        const uint4 hh = *(const uint4*)(p.H + (size_t)m * p.ldh + n);
        const uint32_t hv[4] = {hh.x, hh.y, hh.z, hh.w};
        uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float a0 = bf2f(vv[q] & 0xffff), a1 = bf2f(vv[q] >> 16);
          const float d0 = act_deriv_out(p.act_p, bf2f(hv[q] & 0xffff)) + p.flat_p;
          const float d1 = act_deriv_out(p.act_p, bf2f(hv[q] >> 16)) + p.flat_p;
          a0 = (n + 2 * q < p.np_valid) ? a0 * d0 : 0.f;
          a1 = (n + 2 * q + 1 < p.np_valid) ? a1 * d1 : 0.f;
          vv[q] = pack_bf16x2(a0, a1);
        }
        *(uint4*)(p.Dp + (size_t)m * p.lddp + n) = make_uint4(vv[0], vv[1], vv[2], vv[3]);
      }
    }
  }
  // per-block output-layer gradient and error sums -> global, once
  __syncthreads();
  for (int i = tid; i < n_out * p.KH; i += TT) {
    const int o = i / p.KH, n = i % p.KH;
    atomicAdd(p.GW + (size_t)o * p.KH + n, ga_s[o * TN + n]);
  }
  __shared__ double ered[8][2];
  esum = wave_sum_d(esum);
  wsum = wave_sum_d(wsum);
  if (lane == 0) { ered[wid][0] = esum; ered[wid][1] = wsum; }
  __syncthreads();
  if (tid == 0) {
    double e = 0.0, w = 0.0;
    for (int k = 0; k < 8; ++k) { e += ered[k][0]; w += ered[k][1]; }
    atomicAdd(p.err, e);
    atomicAdd(p.err + 1, w);
  }
}

}  // namespace

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

// Host entry.  Returns -1 on a shape the kernel does not cover (the caller then runs the
// unfused kernels): KH <= 256, KA and KH multiples of 64, n_out <= 8, activations whose
// derivative is a function of the output.
SHIFU_API int shifu_mlp_tail(const void* H, long ldh, const void* W, int nh, int KA, int act_h, float flat_h,
                             const float* Wout, int KH, const float* Y, long ldy, const float* S, int n_out,
                             int out_act, int loss, float flat_out, void* D, long ldd, float* GW, double* err,
                             int do_bwd, const void* Wt, long ldwt, void* Dp, long lddp, int act_p, int np_valid,
                             float flat_p, int M, int n_blocks, hipStream_t stream) {
  if (M <= 0) return 0;
  if (KA % 64 || KH % 64 || KH > TN || KH < 64 || n_out < 1 || n_out > T_OUTMAX || nh < 1 || nh >= KH) return -1;
  if (ldh % 8 || ldd % 8 || (do_bwd && (lddp % 8 || ldwt % 8 || ldwt < KH))) return -1;
  if (!act_deriv_from_output(act_h) || (do_bwd && !act_deriv_from_output(act_p))) return -1;
  if (act_h < 0 || act_h > 8 || out_act < 0 || out_act > 8 || (do_bwd && (act_p < 0 || act_p > 8))) return -1;
  TailArgs p{(const bf16_t*)H, ldh, (const bf16_t*)W, nh, KA, act_h, flat_h, Wout, KH, Y, ldy, S, n_out, out_act,
             loss, flat_out, (bf16_t*)D, ldd, GW, err, do_bwd, (const bf16_t*)Wt, ldwt, (bf16_t*)Dp, lddp, act_p,
             np_valid, flat_p, M};
  const int tiles = (M + TR - 1) / TR;
  int blocks = n_blocks > 0 ? n_blocks : 256;
  if (blocks > tiles) blocks = tiles;
  hipLaunchKernelGGL(mlp_tail_kernel, dim3(blocks), dim3(TT), L_TOTAL, stream, p);
  CHECK_HIP(hipGetLastError());
  return 0;
}
