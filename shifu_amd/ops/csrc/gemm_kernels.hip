// MFMA GEMM kernels for the MLP (gfx950 / CDNA4): fused forward/dgrad NT GEMM and TN wgrad.
//
// Replaces the reference's per-row Java scalar loops
//   forward  FloatFlatNetwork.compute/computeLayer  (J/core/dtrain/dataset/FloatFlatNetwork.java:69-223)
//   backward SubGradient.process/processLevel         (J/core/dtrain/nn/SubGradient.java:224-311)
//   update   Weight.calculateWeights + nn/update/*    (J/core/dtrain/Weight.java:194-343)
// with row-tiled MFMA GEMMs.  Layout decisions (MI355X-first, not a translation):
//   * Every layer is a pure GEMM: the Encog bias neuron is a real input column (value 1.0)
//     stored right after the last feature, and K is zero-padded to a multiple of 64.  So
//     W_l is [out_l, in_pad_l] with column in_l = bias (exactly Encog's flat layout per block).
//   * Activations are bf16 row-major [rows, in_pad]; the forward epilogue writes act(z),
//     the bias column (1.0) and zero padding in one pass.
//   * dgrad is an NT GEMM against a per-step transposed bf16 copy of W, with the
//     activation derivative (+ Encog flat spot) fused into the epilogue.
//   * wgrad is a TN GEMM over the row axis (split-K over rows) using the gfx950
//     ds_read_b64_tr_b16 transposed LDS read for both operands; fp32 atomics into the
//     flat gradient buffer.
//   * the output layer (n_out <= 8) + loss + output delta + last-hidden dgrad + output
//     wgrad are one row kernel (memory-bound, one wave per row strip).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int TILE_BYTES = BM * BK * 2;   // 16 KiB per operand tile

// XCD-aware bijective block remap: consecutive logical ids land on the same XCD
// (blocks b, b+8, ... share an XCD under round-robin dispatch; speed only).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// [128 rows][64 bf16] tile, 128-B rows, 16-B chunk XOR swizzle: rows 0..15 of a fragment
// read land on 16 distinct 16-B slots of the 256-B bank row (conflict-free ds_read_b128).
__device__ __forceinline__ int swz_nt(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

enum Epi : int { EPI_ACT = 0, EPI_DACT = 1, EPI_STORE = 2 };

struct GemmArgs {
  const bf16_t* A; long lda;   // [M, K] row-major
  const bf16_t* B; long ldb;   // [NB, K] row-major (rows >= NB read as 0)
  bf16_t* C; long ldc;         // [M, N] output
  bf16_t* C2; long ldc2;       // EPI_ACT optional: f'(z)+flat (activations not derivable from output)
  const bf16_t* H; long ldh;   // EPI_DACT: layer input activations (derivative from output)
  const bf16_t* Hd; long ldhd; // EPI_DACT: stored derivative (when !act_deriv_from_output)
  int M, N, K, NB, n_valid, act, bias_col;
  float flat;
};

template <int EPI, int ACT>
__global__ __launch_bounds__(NTHR) void gemm_nt_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntn = (p.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / ntn) * BM, n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  uint4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 3, ch = idx & 7;
      const int gm = m0 + row, gn = n0 + row;
      ra[i] = gm < p.M ? *(const uint4*)(p.A + (size_t)gm * p.lda + k0 + ch * 8) : make_uint4(0, 0, 0, 0);
      rb[i] = gn < p.NB ? *(const uint4*)(p.B + (size_t)gn * p.ldb + k0 + ch * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto swrite = [&](int buf) {
    char* As = smem + buf * 2 * TILE_BYTES;
    char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 3, ch = idx & 7;
      *(uint4*)(As + swz_nt(row, ch)) = ra[i];
      *(uint4*)(Bs + swz_nt(row, ch)) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);        // issue next tile's HBM loads early
    const char* As = smem + buf * 2 * TILE_BYTES;
    const char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) af[j] = *(const bf16x8*)(As + swz_nt(wr * 64 + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i) bfr[i] = *(const bf16x8*)(Bs + swz_nt(wc * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[i], af[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) swrite(buf ^ 1);
    __syncthreads();
  }

  // Epilogue.  acc[i][j] holds D[n][m]: m = lane&15 (+16j), n = 4*(lane>>4) + r (+16i):
  // each lane owns 4 consecutive output columns of one row -> one 8-byte store.
  constexpr bool dfo = act_deriv_from_output(ACT);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nb = n0 + wc * 64 + i * 16 + (lane >> 4) * 4;
    if (nb >= p.N) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wr * 64 + j * 16 + (lane & 15);
      if (m >= p.M) continue;
      float o[4];
      if constexpr (EPI == EPI_ACT) {
        float d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + r;
          const float z = acc[i][j][r];
          if (n < p.n_valid) { o[r] = act_fwd(ACT, z); if constexpr (!dfo) d[r] = act_deriv_pre(ACT, z) + p.flat; else d[r] = 0.f; }
          else { o[r] = (n == p.n_valid && p.bias_col) ? 1.f : 0.f; d[r] = 0.f; }
        }
        if constexpr (!dfo) {
          uint2 w2;
          w2.x = (uint32_t)f2bf(d[0]) | ((uint32_t)f2bf(d[1]) << 16);
          w2.y = (uint32_t)f2bf(d[2]) | ((uint32_t)f2bf(d[3]) << 16);
          *(uint2*)(p.C2 + (size_t)m * p.ldc2 + nb) = w2;
        }
      } else if constexpr (EPI == EPI_DACT) {
        float dv[4];
        if constexpr (dfo) {
          const uint2 h = *(const uint2*)(p.H + (size_t)m * p.ldh + nb);
          const float hv[4] = {bf2f(h.x & 0xffff), bf2f(h.x >> 16), bf2f(h.y & 0xffff), bf2f(h.y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r) dv[r] = act_deriv_out(ACT, hv[r]) + p.flat;
        } else {
          const uint2 h = *(const uint2*)(p.Hd + (size_t)m * p.ldhd + nb);
          dv[0] = bf2f(h.x & 0xffff); dv[1] = bf2f(h.x >> 16); dv[2] = bf2f(h.y & 0xffff); dv[3] = bf2f(h.y >> 16);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (nb + r < p.n_valid) ? acc[i][j][r] * dv[r] : 0.f;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r];
      }
      uint2 w;
      w.x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
      w.y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
      *(uint2*)(p.C + (size_t)m * p.ldc + nb) = w;
    }
  }
}

// ---------------------------------------------------------------------------------------
// wgrad: G[n][k] += sum_m D[m][n] * X[m][k]   (TN GEMM over rows, split over m)
// LDS images [64 m][128 cols] bf16, 256-B rows, quad XOR swizzle so that the 8 rows read
// by one 32-lane half of ds_read_b64_tr_b16 hit 8 distinct bank groups.
// ---------------------------------------------------------------------------------------
constexpr int WT_BN = 128, WT_BK = 128, WT_BM = 64;   // n-tile, k-tile, rows per step
constexpr int WT_TILE = WT_BM * 128 * 2;              // 16 KiB

__device__ __forceinline__ int tr_h(int m) { return (m & 3) | (((m >> 3) & 1) << 2); }
// byte offset of 8-byte quad q (4 bf16: cols 4q..4q+3) of row m
__device__ __forceinline__ int swz_tn_quad(int m, int q) { return m * 256 + ((q ^ (tr_h(m) << 2)) << 3); }

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
// gfx950 ds_read_b64_tr_b16 (compiler builtin: hipcc counts its lgkmcnt itself)
__device__ __forceinline__ s16x4 ds_read_tr16_b64(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
}

struct WgradArgs {
  const bf16_t* D; long ldd;   // [M, Nd] deltas
  const bf16_t* X; long ldx;   // [M, Kx] layer inputs
  float* G; long ldg;          // [Nv, Kx] fp32 gradient (accumulated atomically)
  int M, Nv, Kx, rows_per_split;
};

__global__ __launch_bounds__(NTHR) void wgrad_tn_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = (p.Nv + WT_BN - 1) / WT_BN, tiles_k = p.Kx / WT_BK;
  const int ntiles = tiles_n * tiles_k;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, t = wg % ntiles;
  const int n0 = (t / tiles_k) * WT_BN, k0 = (t % tiles_k) * WT_BK;
  const int mbeg = split * p.rows_per_split;
  const int mend = min(p.M, mbeg + p.rows_per_split);
  if (mbeg >= mend) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wk = wid & 1;

  uint4 rd[4], rx[4];
  auto gload = [&](int mb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 4, ch = idx & 15;
      const int gm = mb + row;
      const bool ok = gm < mend;
      const int gn = n0 + ch * 8;
      rd[i] = (ok && gn < p.Nv) ? *(const uint4*)(p.D + (size_t)gm * p.ldd + gn) : make_uint4(0, 0, 0, 0);
      rx[i] = ok ? *(const uint4*)(p.X + (size_t)gm * p.ldx + k0 + ch * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto swrite = [&](int buf) {
    char* Ds = smem + buf * 2 * WT_TILE;
    char* Xs = Ds + WT_TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NTHR, row = idx >> 4, ch = idx & 15;
      *(uint4*)(Ds + swz_tn_quad(row, ch * 2)) = rd[i];
      *(uint4*)(Xs + swz_tn_quad(row, ch * 2)) = rx[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // tr read addressing: group g = lane>>4; lane-in-group t = 4q+p supplies row (8g+q [+4]),
  // quad (col_base/4 + p); lane receives column (col_base + t) of the 4 rows.
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int nsteps = (mend - mbeg + WT_BM - 1) / WT_BM;
  gload(mbeg);
  swrite(0);
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    if (st + 1 < nsteps) gload(mbeg + (st + 1) * WT_BM);
    const char* Ds = smem + buf * 2 * WT_TILE;
    const char* Xs = Ds + WT_TILE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {          // two 32-row k-substeps
      bf16x8 af[4], bfr[4];
      const int mr = s * 32 + 8 * g + tq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = (wn * 64 + i * 16) / 4 + tp;
        const s16x4 lo = ds_read_tr16_b64(Ds + swz_tn_quad(mr, q));
        const s16x4 hi = ds_read_tr16_b64(Ds + swz_tn_quad(mr + 4, q));
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = (wk * 64 + j * 16) / 4 + tp;
        const s16x4 lo = ds_read_tr16_b64(Xs + swz_tn_quad(mr, q));
        const s16x4 hi = ds_read_tr16_b64(Xs + swz_tn_quad(mr + 4, q));
        bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nsteps) swrite(buf ^ 1);
    __syncthreads();
  }
  // acc[i][j]: D_out[n][k]: k = lane&15 (+16j), n = 4*(lane>>4) + r (+16i)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4 + r;
      if (n >= p.Nv) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + wk * 64 + j * 16 + (lane & 15);
        atomicAdd(p.G + (size_t)n * p.ldg + k, acc[i][j][r]);
      }
    }
}

// ---------------------------------------------------------------------------------------
// Output layer row kernel (n_out <= 8):
//   z_o = sum_j H[m][j] W[o][j]   (bias = column kh_valid of H, value 1)
//   p_o = act_out(z_o);  err += ((y-p)s)^2 (squared) | -(y ln p + (1-y) ln(1-p)) (log) | |y-p|s
//   delta_o = (y-p)(f'(p)+flat_out)s  (squared, J/core/dtrain/nn/SubGradient.java:241-248)
//           = (y-p)s                  (log)
//           = sign-loss (absolute, AbsoluteErrorFunction)
//   D[m][j] = (sum_o W[o][j] delta_o)(f'_hid(H[m][j]) + flat_hid)   j < kh_valid, else 0
//   GW[o][j] += delta_o H[m][j]
// One wave per row strip; each lane owns 8 columns (KH <= 512) - row read = 1 KiB per wave.
// ---------------------------------------------------------------------------------------
}  // namespace

// =======================================================================================
// C ABI (called through ctypes; host-side shape checks live in shifu_amd/ops/mlp.py and
// are repeated here so a bad call fails loudly instead of faulting the GPU).
// =======================================================================================
#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

SHIFU_API int shifu_gemm_nt(const void* A, long lda, const void* B, long ldb, int NB, void* C, long ldc,
                            void* C2, long ldc2, const void* H, long ldh, const void* Hd, long ldhd,
                            int M, int N, int K, int epi, int act, int n_valid, int bias_col, float flat,
                            hipStream_t stream) {
  if (K % BK || N % 4 || ldc % 4 || lda % 8 || ldb % 8 || M <= 0 || N <= 0) return -1;
  GemmArgs p{(const bf16_t*)A, lda, (const bf16_t*)B, ldb, (bf16_t*)C, ldc, (bf16_t*)C2, ldc2,
             (const bf16_t*)H, ldh, (const bf16_t*)Hd, ldhd, M, N, K, NB, n_valid, act, bias_col, flat};
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const size_t lds = 4 * TILE_BYTES;
  if (act < 0 || act > 8 || epi < 0 || epi > 2) return -2;
  if (epi == EPI_ACT && !act_deriv_from_output(act) && C2 == nullptr) return -3;
  if (epi == EPI_DACT && !act_deriv_from_output(act) && Hd == nullptr) return -3;
  if (epi == EPI_DACT && act_deriv_from_output(act) && H == nullptr) return -3;
#define GEMM_L(E, A) hipLaunchKernelGGL((gemm_nt_kernel<E, A>), dim3(grid), dim3(NTHR), lds, stream, p)
#define GEMM_ACTS(E) switch (act) { case 0: GEMM_L(E, 0); break; case 1: GEMM_L(E, 1); break; \
    case 2: GEMM_L(E, 2); break; case 3: GEMM_L(E, 3); break; case 4: GEMM_L(E, 4); break; \
    case 5: GEMM_L(E, 5); break; case 6: GEMM_L(E, 6); break; case 7: GEMM_L(E, 7); break; \
    default: GEMM_L(E, 8); break; }
  if (epi == EPI_ACT) { GEMM_ACTS(EPI_ACT) }
  else if (epi == EPI_DACT) { GEMM_ACTS(EPI_DACT) }
  else GEMM_L(EPI_STORE, 2);
#undef GEMM_ACTS
#undef GEMM_L
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_wgrad_tn(const void* D, long ldd, const void* X, long ldx, float* G, long ldg,
                             int M, int Nv, int Kx, int splits, hipStream_t stream) {
  if (Kx % WT_BK || ldd % 8 || ldx % 8 || M <= 0 || Nv <= 0) return -1;
  if (splits < 1) splits = 1;
  int rps = (M + splits - 1) / splits;
  rps = ((rps + WT_BM - 1) / WT_BM) * WT_BM;
  splits = (M + rps - 1) / rps;
  WgradArgs p{(const bf16_t*)D, ldd, (const bf16_t*)X, ldx, G, ldg, M, Nv, Kx, rps};
  const int ntiles = ((Nv + WT_BN - 1) / WT_BN) * (Kx / WT_BK);
  hipLaunchKernelGGL(wgrad_tn_kernel, dim3(ntiles * splits), dim3(NTHR), 4 * WT_TILE, stream, p);
  CHECK_HIP(hipGetLastError());
  return 0;
}

