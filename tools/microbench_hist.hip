// Microbenchmark: GBDT histogram build variants on gfx950 (uint8 bins, 32-feature groups).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_hist.hip -o tools/mb_hist && tools/mb_hist
// V0  two ds_add_u64 per (row, feature), feature-plane layout [2][32][257], row-major bins
//     [N][1024]                                                           (round-1 kernel)
// V3  one packed ds_add_u64 ((qw << 36) + qg) per (row, feature), bin-major LDS layout
//     [2][256][16] + per-lane byte rotation (the 16 lanes of an LDS lane group always hit 16
//     distinct bank pairs), unpacked into int64 registers every 4096 rows
// V4  loads + byte extraction only (memory ceiling of the same access pattern)
// BL  bins layout: 0 row-major [N][1024]; 1 group-blocked [32 groups][N][32]
// ID  1: positions are rows (root node, no pos2row gather)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int FG = 32, NB = 256, HP = 257;

struct Args {
  const uint8_t* bins; long ldb; const int* pos2row; const float* w; const float* g;
  int n_rows, per_item; long long* slab; float sw, sg;
  long gs;   // blocked layout: bytes per group
};

__device__ __forceinline__ uint32_t rotsel(uint32_t a, uint32_t b, bool c) { return c ? b : a; }

template <int V, int HU, int BL, int HT, int ID>
__global__ __launch_bounds__(HT) void hist(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long h[];
  constexpr int NW = V == 0 ? 2 * FG * HP : 2 * NB * 16;
  constexpr int NE = 2 * NB * 16 / HT;          // flush entries per thread
  const int grp = blockIdx.x & 31, rng = blockIdx.x >> 5;
  const int lo = rng * a.per_item, hi = min(a.n_rows, lo + a.per_item);
  for (int i = threadIdx.x; i < NW; i += HT) h[i] = 0ull;
  __syncthreads();
  const int half = threadIdx.x & 1, lane = threadIdx.x & 63, r = lane & 15;
  const int f0 = grp * FG + half * 16;
  long long accw[NE], accg[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) { accw[k] = 0; accg[k] = 0; }
  uint32_t xs = 0;
  constexpr int RPP = HT / 2;
  constexpr int FLUSH = 4096 / (RPP * HU);       // iterations between flushes
  int it = 0;
  const uint8_t* gbase = a.bins + (size_t)grp * a.gs + half * 16;
  for (int p0 = lo + (threadIdx.x >> 1); p0 - (int)(threadIdx.x >> 1) < hi; p0 += RPP * HU) {
    int rows[HU]; float wv[HU], gv[HU]; uint4 bv[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) { const int p = p0 + u * RPP; rows[u] = p < hi ? (ID ? p : a.pos2row[p]) : -1; }
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const int rr = rows[u];
      wv[u] = rr >= 0 ? a.w[rr] : 0.f; gv[u] = rr >= 0 ? a.g[rr] : 0.f;
      bv[u] = rr >= 0 ? *(const uint4*)(BL ? gbase + (size_t)rr * 32 : a.bins + (size_t)rr * a.ldb + f0)
                      : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      if (wv[u] == 0.f) continue;
      uint32_t W[4] = {bv[u].x, bv[u].y, bv[u].z, bv[u].w};
      if constexpr (V == 4) { xs += W[0] ^ W[1] ^ W[2] ^ W[3]; continue; }
      const float wg = wv[u] * gv[u];
      if constexpr (V == 0) {
        const unsigned long long qw = (unsigned long long)__float2ll_rn(wv[u] * a.sw);
        const unsigned long long qg = (unsigned long long)__float2ll_rn(wg * a.sg);
        unsigned long long* pw = h + half * 16 * HP;
        unsigned long long* pg = pw + FG * HP;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t b = (W[j >> 2] >> ((j & 3) * 8)) & 0xff;
          atomicAdd(&pw[j * HP + b], qw); atomicAdd(&pg[j * HP + b], qg);
        }
      } else {
        const unsigned long long q = ((unsigned long long)__float2uint_rn(wv[u] * a.sw) << 36) +
                                     (unsigned long long)(long long)__float2int_rn(wg * a.sg);
        const int q4 = r >> 2, s = r & 3;
        uint32_t X[4], Y[4], R[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) X[k] = rotsel(W[k], W[(k + 1) & 3], q4 & 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) Y[k] = rotsel(X[k], X[(k + 2) & 3], q4 & 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) R[k] = __builtin_amdgcn_alignbyte(Y[(k + 1) & 3], Y[k], s);
        unsigned long long* base = h + half * NB * 16;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t b = (R[j >> 2] >> ((j & 3) * 8)) & 0xff;
          atomicAdd(&base[(b << 4) | ((j + r) & 15)], q);
        }
      }
    }
    if constexpr (V == 3) {
      if (++it == FLUSH) {
        it = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          const unsigned long long v = h[threadIdx.x + k * HT];
          const long long gq = ((long long)(v << 28)) >> 28;
          accg[k] += gq; accw[k] += (long long)((v - (unsigned long long)gq) >> 36);
          h[threadIdx.x + k * HT] = 0ull;
        }
        __syncthreads();
      }
    }
  }
  __syncthreads();
  long long* out = a.slab + (size_t)blockIdx.x * 2 * FG * NB;
  if constexpr (V == 3) {
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int e = threadIdx.x + k * HT;
      const unsigned long long v = h[e];
      const long long gq = ((long long)(v << 28)) >> 28;
      const int hf = e >> 12, b = (e >> 4) & 255, f = hf * 16 + (e & 15);
      out[f * NB + b] = accw[k] + (long long)((v - (unsigned long long)gq) >> 36);
      out[FG * NB + f * NB + b] = accg[k] + gq;
    }
  } else if constexpr (V == 4) {
    out[threadIdx.x] = xs;
  } else {
    for (int i = threadIdx.x; i < 2 * FG * NB; i += HT)
      out[i] = (long long)h[(i / (FG * NB)) * FG * HP + ((i / NB) % FG) * HP + i % NB];
  }
}

template <int V, int HU, int BL, int HT = 512, int ID = 0>
float run(const Args& a, int items) {
  const size_t lds = V == 0 ? 2 * FG * HP * 8 : 2 * NB * 16 * 8;
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((hist<V, HU, BL, HT, ID>), dim3(items), dim3(HT), lds, 0, a);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  return best;
}

int main() {
  const int n = 16 << 20; const long ldb = 1024;
  uint8_t* bins; int* p2r; float *w, *g; long long* slab;
  (void)hipMalloc(&bins, (size_t)n * ldb); (void)hipMalloc(&p2r, n * 4);
  (void)hipMalloc(&w, n * 4); (void)hipMalloc(&g, n * 4);
  std::vector<uint8_t> hb((size_t)n * ldb); uint32_t s = 1;
  for (auto& x : hb) { s = s * 1664525u + 1013904223u; x = s >> 24; }
  (void)hipMemcpy(bins, hb.data(), hb.size(), hipMemcpyHostToDevice);
  std::vector<int> hp(n); std::vector<float> hw(n), hg(n);
  for (int i = 0; i < n; ++i) { hp[i] = i; hw[i] = 1.f; s = s * 1664525u + 1013904223u; hg[i] = (s >> 8) / 16777216.f - 0.5f; }
  (void)hipMemcpy(p2r, hp.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(w, hw.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(g, hg.data(), n * 4, hipMemcpyHostToDevice);
  int* p2r_half; (void)hipMalloc(&p2r_half, n / 2 * 4);
  { std::vector<int> h2; h2.reserve(n / 2);
    for (int i = 0; i < n && (int)h2.size() < n / 2; ++i) {
      s = s * 1664525u + 1013904223u;
      if ((s >> 31) || n - i <= n / 2 - (int)h2.size()) h2.push_back(i);
    }
    (void)hipMemcpy(p2r_half, h2.data(), h2.size() * 4, hipMemcpyHostToDevice); }
  for (int items : {2048, 4096}) {
    const int per = (n + items / 32 - 1) / (items / 32);
    (void)hipMalloc(&slab, (size_t)items * 2 * FG * NB * 8);
    Args a{bins, ldb, p2r, w, g, n, per, slab, 32768.f, 8388608.f, (long)n * 32};
    const double upd = (double)n * 1024;
    auto rep = [&](const char* name, float ms) {
      printf("items %5d %-40s %8.3f ms %8.1f G upd/s %7.2f TB/s\n", items, name, ms, upd / ms / 1e6,
             (double)n * ldb / ms / 1e9);
    };
    rep("V0 round-1 row-major", run<0, 4, 0>(a, items));
    rep("V3 blocked HT512 HU4", run<3, 4, 1>(a, items));
    rep("V3 blocked HT512 HU4 ident", run<3, 4, 1, 512, 1>(a, items));
    rep("V3 blocked HT1024 HU4", run<3, 4, 1, 1024>(a, items));
    rep("V3 blocked HT1024 HU8", run<3, 8, 1, 1024>(a, items));
    rep("V3 blocked HT1024 HU8 ident", run<3, 8, 1, 1024, 1>(a, items));
    rep("V4 blocked HT512 HU4 loads", run<4, 4, 1>(a, items));
    rep("V4 blocked HT1024 HU8 loads", run<4, 8, 1, 1024>(a, items));
    rep("V4 blocked HT1024 HU8 loads ident", run<4, 8, 1, 1024, 1>(a, items));
    {
      Args b = a; b.pos2row = p2r_half; b.n_rows = n / 2; b.per_item = (n / 2 + items / 32 - 1) / (items / 32);
      auto rep2 = [&](const char* name, float ms) {
        printf("items %5d %-40s %8.3f ms %8.1f G upd/s (50%% sorted subset)\n", items, name, ms,
               (double)n / 2 * 1024 / ms / 1e6);
      };
      rep2("V3 blocked HT512 HU4 subset", run<3, 4, 1>(b, items));
      rep2("V3 blocked HT1024 HU8 subset", run<3, 8, 1, 1024>(b, items));
    }
    // exactness: V3 (packed, blocked) == V0 (two atomics, row-major) on the same bins
    // (blocked view of the same bytes differs, so compare V3 row-major against V0 row-major)
    std::vector<long long> s0((size_t)items * 2 * FG * NB), s3(s0.size());
    run<0, 4, 0>(a, items); (void)hipMemcpy(s0.data(), slab, s0.size() * 8, hipMemcpyDeviceToHost);
    run<3, 4, 0>(a, items); (void)hipMemcpy(s3.data(), slab, s3.size() * 8, hipMemcpyDeviceToHost);
    size_t bad = 0; for (size_t i = 0; i < s0.size(); ++i) bad += s0[i] != s3[i];
    printf("items %5d V3 vs V0 mismatches: %zu of %zu\n", items, bad, s0.size());
    (void)hipFree(slab);
  }
  return 0;
}
