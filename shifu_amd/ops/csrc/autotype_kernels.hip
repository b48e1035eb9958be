// GPU auto-type statistics for `init` (B3 / H5) on MI355X: the text blocks `stats` already uploads
// for its field parser (data/gpu_parse.py) are coded and counted on the device instead of by the
// host scanner (runtime/csrc/autotype_scan.cpp, ~3.75 GB/s on 16 cores at 20M x 1600).
//
// Same per-field semantics as the host scanner (AutoTypeDistinctCountMapper.java:134-219):
//   * a line is a row unless blank (only ' ', '\t', '\r'); a trailing '\r' is not part of the last
//     field; with a tag column, rows whose trimmed tag is not a configured tag are skipped;
//   * per field of column c < ncols: missing-or-invalid when the lower-cased raw field equals a
//     missing token, else its 64-bit hash (the scanner's hash_field, bit for bit) and whether
//     Double.parseDouble accepts it (java_double);
//   * per column: row count, missing count, valid-number count, the exact set of value hashes up to
//     AT_EXACT_CAP distinct values (then a 2^14-register HyperLogLog built from the same hashes),
//     and for every distinct hash its first line, from which the host picks the column's first
//     distinct values ("items").
//
// Kernels:
//   at_codes_kernel  one 64-lane wave per line (the K0 tokenizer of csv_kernels.hip): the lane that
//                    owns a field's closing delimiter codes the field into codes[c][line];
//   at_apply_kernel  one 512-thread workgroup per column: the block's codes into LDS (exact set +
//                    first lines, counts), merged into the column's global set; columns past the
//                    cap update the global HLL registers directly;
//   at_spill_kernel  an overflowed column's exact set -> its HLL registers (once);
//   at_items_kernel  per column the AT_ITEMS distinct hashes with the smallest first line.
#include "common.h"
#include <string.h>

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

namespace {

constexpr int AT_MAXTOK = 8, AT_TOKLEN = 16;
constexpr int AT_MAXTAG = 16, AT_TAGLEN = 32;
constexpr int AT_WAVES = 4;
constexpr int AT_HLL_P = 14, AT_HLL_M = 1 << AT_HLL_P;
constexpr int AT_EXACT_CAP = 4096;                  // = autotype_scan.cpp
constexpr int AT_SLOTS = 8192;                      // open addressing, load <= 1/2
constexpr int AT_ITEMS = 200;
constexpr uint64_t AT_ABSENT = 0, AT_MISSING = 1;

struct AtArgs {
  const uint8_t* buf;                               // >= 16 readable bytes past the last line
  const long* ls; const long* le; long nl;
  int ncols;
  uint64_t* codes; long ldc;                        // codes[c * ldc + line]
  int* lflags;                                      // per line: 1 blank, 2 skipped (tag)
  int d0, ntok, tag_col, ntags;
  int toklen[AT_MAXTOK];
  unsigned char tok[AT_MAXTOK][AT_TOKLEN];          // as configured (compared with lower-cased fields)
  int taglen[AT_MAXTAG];
  unsigned char tag[AT_MAXTAG][AT_TAGLEN];          // trimmed
};

__device__ __forceinline__ bool at_ws(unsigned c) { return c == ' ' || c == '\t' || c == '\r'; }

__device__ __forceinline__ uint64_t at_mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// autotype_scan.cpp hash_field: <= 8 bytes one zero-padded little-endian word, else 8-byte words
__device__ uint64_t at_hash(const uint8_t* p, long n) {
  if (n <= 8) {
    uint64_t w = 0;
    for (long k = 0; k < n; ++k) w |= (uint64_t)p[k] << (8 * k);
    return at_mix64(w ^ ((uint64_t)n * 0xff51afd7ed558ccdull) ^ 0x2545f4914f6cdd1dull);
  }
  uint64_t h = 0x9e3779b97f4a7c15ull ^ ((uint64_t)n * 0xff51afd7ed558ccdull);
  long i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) w |= (uint64_t)p[i + k] << (8 * k);
    h = at_mix64(h ^ w) + 0x9e3779b97f4a7c15ull;
  }
  uint64_t t = 0;
  for (long k = 0; i + k < n; ++k) t |= (uint64_t)p[i + k] << (8 * k);
  return at_mix64(h ^ t ^ 0x2545f4914f6cdd1dull);
}

// Double.parseDouble's grammar (autotype_scan.cpp java_double)
__device__ bool at_java_double(const uint8_t* p, long n) {
  long a = 0, b = n;
  while (a < b && p[a] <= ' ') ++a;
  while (b > a && p[b - 1] <= ' ') --b;
  if (a == b) return false;
  if (p[a] == '+' || p[a] == '-') ++a;
  const long m = b - a;
  if (m == 3 && p[a] == 'N' && p[a + 1] == 'a' && p[a + 2] == 'N') return true;
  if (m == 8) {
    const char inf[8] = {'I', 'n', 'f', 'i', 'n', 'i', 't', 'y'};
    bool eq = true;
    for (int k = 0; k < 8; ++k) eq = eq && p[a + k] == (uint8_t)inf[k];
    if (eq) return true;
  }
  if (b > a && (p[b - 1] == 'd' || p[b - 1] == 'D' || p[b - 1] == 'f' || p[b - 1] == 'F')) --b;
  long i = a;
  int digits = 0;
  while (i < b && p[i] >= '0' && p[i] <= '9') { ++i; ++digits; }
  if (i < b && p[i] == '.') {
    ++i;
    while (i < b && p[i] >= '0' && p[i] <= '9') { ++i; ++digits; }
  }
  if (digits == 0) return false;
  if (i < b && (p[i] == 'e' || p[i] == 'E')) {
    ++i;
    if (i < b && (p[i] == '+' || p[i] == '-')) ++i;
    int ed = 0;
    while (i < b && p[i] >= '0' && p[i] <= '9') { ++i; ++ed; }
    if (ed == 0) return false;
  }
  return i == b;
}

__device__ __forceinline__ unsigned at_lower(unsigned c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// field [a, b) of a line, column f: its code (and the tag verdict when f is the tag column)
__device__ void at_field(const AtArgs& A, long line, int f, long a, long b, int* tag_ok) {
  const uint8_t* p = A.buf;
  const long n = b - a;
  if (f == A.tag_col) {
    long x = a, y = b;
    while (x < y && p[x] <= ' ') ++x;
    while (y > x && p[y - 1] <= ' ') --y;
    bool ok = false;
    for (int t = 0; t < A.ntags && !ok; ++t) {
      if (A.taglen[t] != y - x) continue;
      bool eq = true;
      for (long i = 0; i < y - x && eq; ++i) eq = p[x + i] == A.tag[t][i];
      ok = eq;
    }
    *tag_ok = ok ? 1 : 0;
  }
  if (f >= A.ncols) return;
  bool miss = false;
  for (int t = 0; t < A.ntok && !miss; ++t) {
    if (A.toklen[t] != n) continue;
    bool eq = true;
    for (long i = 0; i < n && eq; ++i) eq = at_lower(p[a + i]) == A.tok[t][i];
    miss = eq;
  }
  uint64_t code = AT_MISSING;
  if (!miss) {
    uint64_t h = at_hash(p + a, n) >> 1;
    if (!h) h = 1;
    code = (h << 1) | (at_java_double(p + a, n) ? 1u : 0u);
  }
  A.codes[(long)f * A.ldc + line] = code;
}

__device__ __forceinline__ int at_excl_sum(int v, int lane) {
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x - v;
}

__device__ __forceinline__ long at_incl_max(long v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long y = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, y);
  }
  return v;
}

__global__ __launch_bounds__(256) void at_codes_kernel(AtArgs A) {
  const int lane = threadIdx.x & 63;
  const long line = (long)blockIdx.x * AT_WAVES + (threadIdx.x >> 6);
  if (line >= A.nl) return;                          // whole wave exits together
  const long s = A.ls[line];
  long e = A.le[line];
  if (e > s && A.buf[e - 1] == '\r') --e;             // the scanner's line end (blank test keeps it)
  const long a0 = s & ~15l;
  int fields = 0;
  long prev = s - 1;
  bool nonblank = false;
  int tag_ok = -1;                                    // -1: tag field not seen (short row)
  const unsigned d0 = (unsigned)A.d0;
  for (long base = a0; base < e; base += 1024) {
    const long cb = base + 16 * lane;
    unsigned dm = 0;
    if (cb < e && cb + 16 > s) {
      const uint4 q = *(const uint4*)(A.buf + cb);
      const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const long pos = cb + j;
        const unsigned c = (w[j >> 2] >> (8 * (j & 3))) & 0xff;
        const bool in = pos >= s && pos < e;
        if (in && c == d0) dm |= 1u << j;
        if (in && !at_ws(c)) nonblank = true;
      }
    }
    const int cnt = __builtin_popcount(dm);
    const int pre = at_excl_sum(cnt, lane);
    const long mylast = dm ? cb + 31 - __builtin_clz(dm) : -1;
    const long incl = at_incl_max(mylast, lane);
    long before = __shfl_up(incl, 1, 64);
    if (lane == 0) before = -1;
    long st = max(prev, before) + 1;
    int f = fields + pre;
    unsigned mm = dm;
    while (mm) {
      const int j = __builtin_ctz(mm);
      mm &= mm - 1;
      at_field(A, line, f, st, cb + j, &tag_ok);
      st = cb + j + 1;
      ++f;
    }
    fields += __shfl(pre + cnt, 63, 64);
    prev = max(prev, __shfl(incl, 63, 64));
  }
  if (lane == 0) at_field(A, line, fields, prev + 1, e, &tag_ok);
  const int nf = fields + 1;
  for (int f = nf + lane; f < A.ncols; f += 64) A.codes[(long)f * A.ldc + line] = AT_ABSENT;
  const unsigned long long nb = __ballot(nonblank);
  // the tag verdict lives in the lane that coded the tag field
  const unsigned long long tagbad = __ballot(tag_ok == 0);
  if (lane == 0) {
    int fl = nb ? 0 : 1;
    if (A.tag_col >= 0 && nb && (tagbad || nf <= A.tag_col)) fl |= 2;
    A.lflags[line] = fl;
  }
}

// ---- per-column state in HBM (one rank):
//   cnt [ncols][3] int64 count / missing / valid-number; set [ncols][AT_SLOTS] u64 hashes (0 empty);
//   first [ncols][AT_SLOTS] u64 first line (global line number of the rank); used [ncols] int32;
//   ovf [ncols] int32 (1 overflowed, 2 overflowed and its set spilled into hll); hll [ncols][M] u32
struct AtState {
  long long* cnt; uint64_t* set; unsigned long long* first; int* used; int* ovf; unsigned* hll;
};

__device__ __forceinline__ void at_hll_add(unsigned* reg, uint64_t h) {
  const unsigned idx = (unsigned)(h >> (64 - AT_HLL_P));
  const uint64_t rest = (h << AT_HLL_P) | (1ull << (AT_HLL_P - 1));
  const unsigned rank = (unsigned)__builtin_clzll(rest) + 1;
  if (__builtin_nontemporal_load(reg + idx) < rank) atomicMax(reg + idx, rank);
}

// global set insert of hash h with first line ln; returns 1 when h was new, 0 if present, -1 full
__device__ int at_global_insert(const AtState& G, int c, uint64_t h, unsigned long long ln) {
  uint64_t* set = G.set + (size_t)c * AT_SLOTS;
  unsigned long long* first = G.first + (size_t)c * AT_SLOTS;
  unsigned k = (unsigned)h & (AT_SLOTS - 1);
  for (int probe = 0; probe < AT_SLOTS; ++probe, k = (k + 1) & (AT_SLOTS - 1)) {
    const uint64_t cur = atomicCAS((unsigned long long*)(set + k), 0ull, (unsigned long long)h);
    if (cur == 0 || cur == h) {
      atomicMin(first + k, ln);
      return cur == 0 ? 1 : 0;
    }
  }
  return -1;
}

constexpr int AT_APPLY_T = 512;

__global__ __launch_bounds__(AT_APPLY_T) void at_apply_kernel(const uint64_t* __restrict__ codes, long ldc, long nl,
                                                            const int* __restrict__ lflags, unsigned long long line0,
                                                            const int* __restrict__ cols, AtState G) {
  __shared__ uint64_t sset[AT_SLOTS];
  __shared__ unsigned sfirst[AT_SLOTS];
  __shared__ int sused, sovf;
  __shared__ long long scnt[3];
  const int c = cols[blockIdx.x];
  const int tid = threadIdx.x;
  for (int i = tid; i < AT_SLOTS; i += AT_APPLY_T) { sset[i] = 0; sfirst[i] = 0xffffffffu; }
  if (tid == 0) { sused = 0; sovf = G.ovf[c] ? 1 : 0; scnt[0] = scnt[1] = scnt[2] = 0; }
  __syncthreads();
  unsigned* hll = G.hll + (size_t)c * AT_HLL_M;
  const uint64_t* x = codes + (size_t)c * ldc;
  long long n0 = 0, n1 = 0, n2 = 0;
  for (long i = tid; i < nl; i += AT_APPLY_T) {
    if (lflags[i]) continue;
    const uint64_t v = x[i];
    if (v == AT_ABSENT) continue;
    ++n0;
    if (v == AT_MISSING) { ++n1; continue; }
    n2 += (long long)(v & 1);
    const uint64_t h = v | 1;
    if (*(volatile int*)&sovf) { at_hll_add(hll, h); continue; }
    unsigned k = (unsigned)h & (AT_SLOTS - 1);
    while (true) {
      const unsigned long long cur = atomicCAS((unsigned long long*)&sset[k], 0ull, (unsigned long long)h);
      if (cur == 0) {
        if (atomicAdd(&sused, 1) >= AT_EXACT_CAP) sovf = 1;   // the block's own cap: HLL from here
        atomicMin(&sfirst[k], (unsigned)i);
        break;
      }
      if (cur == h) { atomicMin(&sfirst[k], (unsigned)i); break; }
      k = (k + 1) & (AT_SLOTS - 1);
    }
    if (*(volatile int*)&sovf) at_hll_add(hll, h);
  }
  atomicAdd((unsigned long long*)&scnt[0], (unsigned long long)n0);
  atomicAdd((unsigned long long*)&scnt[1], (unsigned long long)n1);
  atomicAdd((unsigned long long*)&scnt[2], (unsigned long long)n2);
  __syncthreads();
  if (tid < 3) atomicAdd((unsigned long long*)&G.cnt[3 * c + tid], (unsigned long long)scnt[tid]);
  // merge the block's set: into the global set while the column stays exact, else into its HLL
  // (the global set's own entries are spilled into the HLL by at_spill_kernel)
  const bool block_ovf = *(volatile int*)&sovf != 0;
  for (int k = tid; k < AT_SLOTS; k += AT_APPLY_T) {
    const uint64_t h = sset[k];
    if (!h) continue;
    if (block_ovf || G.ovf[c]) { at_hll_add(hll, h); continue; }
    const int r = at_global_insert(G, c, h, line0 + sfirst[k]);
    if (r == 1 && atomicAdd(&G.used[c], 1) >= AT_EXACT_CAP) atomicMax(&G.ovf[c], 1);
    if (r < 0) { atomicMax(&G.ovf[c], 1); at_hll_add(hll, h); }
  }
  if (block_ovf && tid == 0) atomicMax(&G.ovf[c], 1);
}

// overflowed columns whose exact set has not been spilled: every set hash into the HLL registers
__global__ __launch_bounds__(256) void at_spill_kernel(const int* __restrict__ cols, AtState G) {
  const int c = cols[blockIdx.x];
  if (G.ovf[c] != 1) return;
  const uint64_t* set = G.set + (size_t)c * AT_SLOTS;
  unsigned* hll = G.hll + (size_t)c * AT_HLL_M;
  for (int k = threadIdx.x; k < AT_SLOTS; k += 256)
    if (set[k]) at_hll_add(hll, set[k]);
  __syncthreads();
  if (threadIdx.x == 0) G.ovf[c] = 2;
}

// every exact set of cols into its column's HLL registers (end of the scan: ranks merge HLL
// registers by max, so a column exact on this rank must still carry its sketch)
__global__ __launch_bounds__(256) void at_sets_to_hll_kernel(const int* __restrict__ cols, AtState G) {
  const int c = cols[blockIdx.x];
  const uint64_t* set = G.set + (size_t)c * AT_SLOTS;
  unsigned* hll = G.hll + (size_t)c * AT_HLL_M;
  for (int k = threadIdx.x; k < AT_SLOTS; k += 256)
    if (set[k]) at_hll_add(hll, set[k]);
}

// per column: the AT_ITEMS (hash, first line) pairs with the smallest first lines (ties: hash),
// out [ncols_sel][AT_ITEMS][2] u64 (hash 0 = none); bitonic sort of the 8192 slots in LDS
__global__ __launch_bounds__(1024) void at_items_kernel(const int* __restrict__ cols, AtState G, uint64_t* out) {
  __shared__ unsigned long long key[AT_SLOTS];       // first line (empty: ~0)
  __shared__ uint64_t val[AT_SLOTS];
  const int c = cols[blockIdx.x];
  const uint64_t* set = G.set + (size_t)c * AT_SLOTS;
  const unsigned long long* first = G.first + (size_t)c * AT_SLOTS;
  for (int k = threadIdx.x; k < AT_SLOTS; k += 1024) {
    const uint64_t h = set[k];
    key[k] = h ? first[k] : ~0ull;
    val[k] = h;
  }
  __syncthreads();
  for (int size = 2; size <= AT_SLOTS; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < AT_SLOTS / 2; t += 1024) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const bool gt = key[lo] > key[hi] || (key[lo] == key[hi] && val[lo] > val[hi]);
        if (gt == up) {
          const unsigned long long tk = key[lo]; key[lo] = key[hi]; key[hi] = tk;
          const uint64_t tv = val[lo]; val[lo] = val[hi]; val[hi] = tv;
        }
      }
      __syncthreads();
    }
  }
  uint64_t* o = out + (size_t)blockIdx.x * AT_ITEMS * 2;
  for (int k = threadIdx.x; k < AT_ITEMS; k += 1024) {
    o[2 * k] = key[k] == ~0ull ? 0 : val[k];
    o[2 * k + 1] = key[k];
  }
}

}  // namespace

SHIFU_API int shifu_at_gpu_caps(int* out) {
  out[0] = AT_HLL_P; out[1] = AT_EXACT_CAP; out[2] = AT_SLOTS; out[3] = AT_ITEMS;
  out[4] = AT_MAXTOK; out[5] = AT_TOKLEN; out[6] = AT_MAXTAG; out[7] = AT_TAGLEN;
  return 0;
}

// codes for the lines [ls, le) of a block in HBM: codes [ncols][ldc] u64, lflags [nl].
// toks / tags: '\0'-separated (tokens lower-case as the scanner compares them; tags trimmed)
SHIFU_API int shifu_at_gpu_codes(const void* buf, const long* ls, const long* le, long nl, int ncols, void* codes,
                                 long ldc, int* lflags, int delim, int ntok, const char* toks, int tag_col, int ntags,
                                 const char* tags, hipStream_t stream) {
  if (nl <= 0) return 0;
  if (ncols <= 0 || ldc < nl || ntok < 0 || ntok > AT_MAXTOK || ntags < 0 || ntags > AT_MAXTAG) return -1;
  AtArgs A{};
  A.buf = (const uint8_t*)buf; A.ls = ls; A.le = le; A.nl = nl; A.ncols = ncols;
  A.codes = (uint64_t*)codes; A.ldc = ldc; A.lflags = lflags;
  A.d0 = delim & 0xff; A.ntok = ntok; A.tag_col = tag_col; A.ntags = ntags;
  const char* t = toks;
  for (int i = 0; i < ntok; ++i) {
    const int n = (int)strlen(t);
    if (n >= AT_TOKLEN) return -1;
    A.toklen[i] = n;
    memcpy(A.tok[i], t, n);
    t += n + 1;
  }
  t = tags;
  for (int i = 0; i < ntags; ++i) {
    const int n = (int)strlen(t);
    if (n >= AT_TAGLEN) return -1;
    A.taglen[i] = n;
    memcpy(A.tag[i], t, n);
    t += n + 1;
  }
  const long blocks = (nl + AT_WAVES - 1) / AT_WAVES;
  if (blocks > 0x7fffffffl) return -1;
  hipLaunchKernelGGL(at_codes_kernel, dim3((unsigned)blocks), dim3(64 * AT_WAVES), 0, stream, A);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// the block's codes into the per-column state of columns cols[0 .. ncsel) (line0: the block's
// first line number in the rank's stream), then spill the columns that overflowed
SHIFU_API int shifu_at_gpu_apply(const void* codes, long ldc, long nl, const int* lflags, long line0,
                                 const int* cols, int ncsel, long long* cnt, void* set, void* first, int* used,
                                 int* ovf, unsigned* hll, hipStream_t stream) {
  if (nl <= 0 || ncsel <= 0) return 0;
  if (nl >= 0xffffffffl) return -1;                   // block-local first lines are u32 in LDS
  AtState G{cnt, (uint64_t*)set, (unsigned long long*)first, used, ovf, hll};
  hipLaunchKernelGGL(at_apply_kernel, dim3(ncsel), dim3(AT_APPLY_T), 0, stream, (const uint64_t*)codes, ldc, nl,
                     lflags, (unsigned long long)line0, cols, G);
  hipLaunchKernelGGL(at_spill_kernel, dim3(ncsel), dim3(256), 0, stream, cols, G);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// out [ncsel][AT_ITEMS][2] u64: per column the (hash, first line) pairs of its first distinct values
SHIFU_API int shifu_at_gpu_items(const int* cols, int ncsel, void* set, void* first, void* out, hipStream_t stream) {
  if (ncsel <= 0) return 0;
  AtState G{nullptr, (uint64_t*)set, (unsigned long long*)first, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(at_items_kernel, dim3(ncsel), dim3(1024), 0, stream, cols, G, (uint64_t*)out);
  CHECK_HIP(hipGetLastError());
  return 0;
}

SHIFU_API int shifu_at_gpu_hll_from_sets(const int* cols, int ncsel, void* set, unsigned* hll, hipStream_t stream) {
  if (ncsel <= 0) return 0;
  AtState G{nullptr, (uint64_t*)set, nullptr, nullptr, nullptr, hll};
  hipLaunchKernelGGL(at_sets_to_hll_kernel, dim3(ncsel), dim3(256), 0, stream, cols, G);
  CHECK_HIP(hipGetLastError());
  return 0;
}
