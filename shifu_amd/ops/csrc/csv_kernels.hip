// GPU numeric field parser (K0) for MI355X (gfx950): delimited text bytes already in HBM ->
// column-major fp64 values, bit-identical to the host parser (runtime/csrc/csv_parser.cpp).
//
// Replaces the per-record text parsing of the reference's loaders (NNWorker.load
// J/core/dtrain/nn/NNWorker.java:56-269, UpdateBinningInfoMapper.map
// J/core/binning/UpdateBinningInfoMapper.java:349-599, NormalizeUDF.exec J/udf/NormalizeUDF.java)
// for the bulk numeric columns: the host reads a block of lines into pinned memory, copies it to
// HBM (one ~50 GB/s DMA instead of 16 host cores tokenizing ~3 GB/s), and this kernel tokenizes
// and converts every wanted field; the host parser only frames rows and keeps the few
// target / weight / categorical columns (data/gpu_parse.py).
//
// MI355X design: one 64-lane wave per line.  Each step the wave covers 1 KB of the line (16 aligned
// bytes per lane, one 128-bit load), builds the lane's delimiter mask, and two wave scans give
// every delimiter its field index (exclusive popcount prefix) and its field's start (exclusive max
// of the previous delimiter positions, carried across steps).  The lane that owns a field's closing
// delimiter parses that field: trim (' ', '\t', '\r'), missing tokens, then the host parser's
// Clinger fast path ([+-]digits[.digits], <= 19 significant digits, < 2^53, <= 22 fraction digits:
// m / 10^k, one correctly rounded IEEE division == strtod).  Anything else (exponents, "1.0d",
// words) is appended to a fallback list the host finishes with its own strtod path, so the
// values equal the host parse bit for bit.  Short rows get NaN in their missing fields and every
// line reports (blank, field count != ncols) flags, the host parser's row rules.
#include "common.h"
#include <string.h>

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

namespace {

constexpr int CSV_MAXTOK = 8;
constexpr int CSV_TOKLEN = 16;
constexpr int CSV_WAVES = 4;                  // lines per 256-thread workgroup

struct CsvArgs {
  const uint8_t* buf;                         // padded: >= 16 readable bytes past the last line
  const long* ls; const long* le; long nl;    // line i = [ls[i], le[i]) ('\n' excluded)
  const int* slot; int ncols;                 // header column -> output row (-1: not parsed here)
  double* out; long ldo;                      // out[slot * ldo + line]
  int* lflags;                                // per line: 1 blank, 2 field count != ncols
  const int* mslot; int* moffs;               // header column -> host-column index (-1) ; its raw
                                              // field bounds moffs[(k * nl + line) * 2 + {0, 1}]
  long* fb; int fb_cap; int* fb_n;            // fallback fields (line, slot, start, end)
  int d0;
  int ntok;
  int toklen[CSV_MAXTOK];
  unsigned char tok[CSV_MAXTOK][CSV_TOKLEN];
};

__device__ __forceinline__ bool csv_ws(unsigned c) { return c == ' ' || c == '\t' || c == '\r'; }

__device__ const double kCsvPow10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                         1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// field [a, b) of `line`, header column f -> out (or the fallback list)
__device__ void csv_field(const CsvArgs& A, long line, int f, long a, long b) {
  if (f >= A.ncols) return;
  if (A.mslot) {                              // a host-parsed column: hand its bounds back
    const int k = A.mslot[f];
    if (k >= 0) {
      int* o = A.moffs + 2 * ((long)k * A.nl + line);
      o[0] = (int)a;
      o[1] = (int)b;
    }
  }
  const int s = A.slot[f];
  if (s < 0) return;
  const uint8_t* p = A.buf;
  while (a < b && csv_ws(p[a])) ++a;
  while (b > a && csv_ws(p[b - 1])) --b;
  double v = __builtin_nan("");
  const long n = b - a;
  if (n > 0) {
    bool miss = false;
    for (int t = 0; t < A.ntok && !miss; ++t) {
      if (A.toklen[t] != n) continue;
      bool eq = true;
      for (int i = 0; i < n && eq; ++i) eq = p[a + i] == A.tok[t][i];
      miss = eq;
    }
    if (!miss) {
      long i = a;
      bool neg = false;
      if (p[i] == '-' || p[i] == '+') { neg = p[i] == '-'; ++i; }
      unsigned long long m = 0;
      int nd = 0, frac = 0;
      bool any = false, dot = false, ok = true;
      for (; i < b; ++i) {
        const unsigned c = p[i];
        const unsigned d = c - '0';
        if (d < 10) {
          any = true;
          if (m == 0 && d == 0) { frac += dot; continue; }
          if (++nd > 19) { ok = false; break; }
          m = m * 10 + d;
          frac += dot;
        } else if (c == '.' && !dot) {
          dot = true;
        } else {
          ok = false;
          break;
        }
      }
      if (ok && any && m < (1ull << 53) && frac <= 22) {
        const double x = frac ? (double)m / kCsvPow10[frac] : (double)m;
        v = neg ? -x : x;
      } else {
        const int k = atomicAdd(A.fb_n, 1);
        if (k < A.fb_cap) {
          long* e = A.fb + 4 * (long)k;
          e[0] = line; e[1] = s; e[2] = a; e[3] = b;
        }
      }
    }
  }
  A.out[(long)s * A.ldo + line] = v;
}

__device__ __forceinline__ int wave_excl_sum(int v, int lane) {
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x - v;
}

__device__ __forceinline__ long wave_incl_max(long v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long y = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, y);
  }
  return v;
}

__global__ __launch_bounds__(256) void csv_parse_kernel(CsvArgs A) {
  const int lane = threadIdx.x & 63;
  const long line = (long)blockIdx.x * CSV_WAVES + (threadIdx.x >> 6);
  if (line >= A.nl) return;                   // whole wave exits together
  const long s = A.ls[line], e = A.le[line];
  const long a0 = s & ~15l;
  int fields = 0;                             // delimiters seen so far (= index of the open field)
  long prev = s - 1;                          // last delimiter position so far
  bool nonblank = false;
  const unsigned d0 = (unsigned)A.d0;
  for (long base = a0; base < e; base += 1024) {
    const long cb = base + 16 * lane;         // this lane's 16 aligned bytes
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
        if (in && !csv_ws(c)) nonblank = true;
      }
    }
    const int cnt = __builtin_popcount(dm);
    const int pre = wave_excl_sum(cnt, lane);
    const long mylast = dm ? cb + 31 - __builtin_clz(dm) : -1;
    const long incl = wave_incl_max(mylast, lane);
    long before = __shfl_up(incl, 1, 64);
    if (lane == 0) before = -1;
    long st = max(prev, before) + 1;          // start of the field this lane's first delimiter closes
    int f = fields + pre;
    unsigned mm = dm;
    while (mm) {
      const int j = __builtin_ctz(mm);
      mm &= mm - 1;
      csv_field(A, line, f, st, cb + j);
      st = cb + j + 1;
      ++f;
    }
    fields += __shfl(pre + cnt, 63, 64);
    prev = max(prev, __shfl(incl, 63, 64));
  }
  // the last field (after the last delimiter) and the missing fields of a short row
  if (lane == 0) csv_field(A, line, fields, prev + 1, e);
  const int nf = fields + 1;
  for (int f = nf + lane; f < A.ncols; f += 64) {
    const int sl = A.slot[f];
    if (sl >= 0) A.out[(long)sl * A.ldo + line] = __builtin_nan("");
  }
  const unsigned long long nb = __ballot(nonblank);
  if (lane == 0) A.lflags[line] = (nb ? 0 : 1) | (nf != A.ncols ? 2 : 0);
}

}  // namespace

// buf: device bytes (>= 16 readable bytes past the last line end); ls/le: int64 line bounds;
// slot[ncols]: output row per header column (-1 skip); out: [nslots][ldo] fp64; lflags[nl];
// fb: [fb_cap][4] int64 fallback fields, fb_n: int32 counter (zeroed by the caller);
// toks: ntok '\0'-separated trimmed missing tokens (each < 16 bytes).
// mslot (nullable): header column -> index of a host-parsed column whose raw field bounds are
// written to moffs [n_host][nl][2] int32 (block offsets < 2^31), so the host never scans the text.
SHIFU_API int shifu_csv_gpu_parse(const void* buf, const long* ls, const long* le, long nl, const int* slot,
                                  int ncols, double* out, long ldo, int* lflags, long* fb, int fb_cap, int* fb_n,
                                  int delim, int ntok, const char* toks, const int* mslot, int* moffs,
                                  hipStream_t stream) {
  if (nl <= 0) return 0;
  if (ncols <= 0 || ldo < nl || ntok < 0 || ntok > CSV_MAXTOK || fb_cap < 0 || (mslot && !moffs)) return -1;
  CsvArgs A{};
  A.buf = (const uint8_t*)buf; A.ls = ls; A.le = le; A.nl = nl; A.slot = slot; A.ncols = ncols;
  A.out = out; A.ldo = ldo; A.lflags = lflags; A.fb = fb; A.fb_cap = fb_cap; A.fb_n = fb_n;
  A.mslot = mslot; A.moffs = moffs;
  A.d0 = delim & 0xff; A.ntok = ntok;
  const char* t = toks;
  for (int i = 0; i < ntok; ++i) {
    const int n = (int)strlen(t);
    if (n >= CSV_TOKLEN) return -1;
    A.toklen[i] = n;
    memcpy(A.tok[i], t, n);
    t += n + 1;
  }
  const long blocks = (nl + CSV_WAVES - 1) / CSV_WAVES;
  if (blocks > 0x7fffffffl) return -1;
  hipLaunchKernelGGL(csv_parse_kernel, dim3((unsigned)blocks), dim3(64 * CSV_WAVES), 0, stream, A);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// ---- newline index: positions of every '\n' of a block in HBM (the line table the parse kernel
// takes).  Three launches, all on the device: per 64 KiB segment a count, one exclusive scan of
// the segment counts (one workgroup), then each segment's positions written in order (per-thread
// 256-byte runs, workgroup prefix of the run counts).  Replaces torch.nonzero(buf == '\n').
namespace {

constexpr int NL_SEG = 65536;                 // bytes per segment = 256 threads x 256 bytes
constexpr int NL_RUN = 256;

__device__ __forceinline__ int nl_count_run(const uint8_t* p, long len) {
  int c = 0;
  if (len == NL_RUN) {
#pragma unroll
    for (int i = 0; i < NL_RUN / 16; ++i) {
      const uint4 v = ((const uint4*)p)[i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t x = w[k] ^ 0x0a0a0a0au;                       // zero byte <=> '\n'
        c += __builtin_popcount(~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu));
      }
    }
  } else {
    for (long i = 0; i < len; ++i) c += p[i] == '\n';
  }
  return c;
}

__device__ __forceinline__ int nl_block_excl_scan(int v, int* sh, int* total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int u = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += u;
    __syncthreads();
  }
  const int incl = sh[t];
  *total = sh[255];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(256) void nl_count_kernel(const uint8_t* __restrict__ buf, long L, int* __restrict__ cnt) {
  __shared__ int sh[256];
  const long a = (long)blockIdx.x * NL_SEG + (long)threadIdx.x * NL_RUN;
  const long len = a < L ? min((long)NL_RUN, L - a) : 0;
  const int c = len > 0 ? nl_count_run(buf + a, len) : 0;
  int tot;
  nl_block_excl_scan(c, sh, &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// exclusive scan of the segment counts in place (+ the total at off[S])
__global__ __launch_bounds__(1024) void nl_scan_kernel(int* __restrict__ cnt, long S, long* __restrict__ off) {
  __shared__ long sh[1024];
  long carry = 0;
  for (long b = 0; b < S; b += 1024) {
    const long i = b + threadIdx.x;
    const long v = i < S ? cnt[i] : 0;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const long u = (int)threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
      __syncthreads();
      sh[threadIdx.x] += u;
      __syncthreads();
    }
    if (i < S) off[i] = carry + sh[threadIdx.x] - v;
    const long last = sh[1023];
    __syncthreads();
    carry += last;
  }
  if (threadIdx.x == 0) off[S] = carry;
}

__global__ __launch_bounds__(256) void nl_write_kernel(const uint8_t* __restrict__ buf, long L,
                                                       const long* __restrict__ off, long* __restrict__ ends) {
  __shared__ int sh[256];
  const long a = (long)blockIdx.x * NL_SEG + (long)threadIdx.x * NL_RUN;
  const long len = a < L ? min((long)NL_RUN, L - a) : 0;
  const int c = len > 0 ? nl_count_run(buf + a, len) : 0;
  int tot;
  const int pre = nl_block_excl_scan(c, sh, &tot);
  long o = off[blockIdx.x] + pre;
  for (long i = 0; i < len && c; ++i)
    if (buf[a + i] == '\n') ends[o++] = a + i;
}

}  // namespace

SHIFU_API long shifu_newline_ws_bytes(long L) {
  const long S = (L + NL_SEG - 1) / NL_SEG;
  return S * 4 + (S + 1) * 8 + 16;
}

// ws layout (16-B aligned): int32 segment counts [S], then at round16(4 S) the int64 exclusive
// offsets [S] and the total newline count
static long nl_off_bytes(long S) { return (S * 4 + 15) & ~15l; }
static long* nl_off(void* ws, long S) { return (long*)((char*)ws + nl_off_bytes(S)); }

// pass 1 (+ scan): the newline count lands at byte offset shifu_newline_count_offset(L) of ws
// (an int64; read it after the stream has run)
SHIFU_API long shifu_newline_count_offset(long L) {
  const long S = (L + NL_SEG - 1) / NL_SEG;
  return nl_off_bytes(S) + S * 8;
}

SHIFU_API int shifu_newline_count(const void* buf, long L, void* ws, hipStream_t stream) {
  if (L <= 0 || ((uintptr_t)buf & 15) || ((uintptr_t)ws & 15)) return -1;
  const long S = (L + NL_SEG - 1) / NL_SEG;
  if (S >= (1l << 31)) return -1;
  hipLaunchKernelGGL(nl_count_kernel, dim3((unsigned)S), dim3(256), 0, stream, (const uint8_t*)buf, L, (int*)ws);
  hipLaunchKernelGGL(nl_scan_kernel, dim3(1), dim3(1024), 0, stream, (int*)ws, S, nl_off(ws, S));
  CHECK_HIP(hipGetLastError());
  return 0;
}

// pass 2: ends[0 .. count) = the '\n' positions in order (ends sized by the count of pass 1)
SHIFU_API int shifu_newline_write(const void* buf, long L, const void* ws, long* ends, hipStream_t stream) {
  if (L <= 0) return -1;
  const long S = (L + NL_SEG - 1) / NL_SEG;
  hipLaunchKernelGGL(nl_write_kernel, dim3((unsigned)S), dim3(256), 0, stream, (const uint8_t*)buf, L,
                     nl_off((void*)ws, S), ends);
  CHECK_HIP(hipGetLastError());
  return 0;
}
