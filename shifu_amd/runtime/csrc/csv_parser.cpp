// Multithreaded delimited-text parser (host runtime, C++17).
//
// Replaces the reference's per-record text parsing in the Pig loaders / Guagua record readers
// (NNWorker.load J/core/dtrain/nn/NNWorker.java:56-269, DTWorker.load J/core/dtrain/dt/DTWorker.java:1099-1297,
// UpdateBinningInfoMapper.map) with a one-pass columnar parse:
//   * the buffer is split at line boundaries into T chunks parsed by T threads
//   * numeric columns -> double (NaN for missing / unparseable, the reference's "invalid")
//   * string columns  -> int32 dictionary codes (-1 = missing) + per-column dictionary
// Output is column-major so each column becomes one contiguous array (columnar cache).
// Two-phase use (shifu_csv_scan + shifu_csv_fill) writes the numeric columns straight into the
// caller's [n_numeric][ld] block: no internal per-column vectors, no serial zero-fill + copy-out
// (the destination's pages are first touched by the parsing threads).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>
#include <immintrin.h>

#define SHIFU_RT_API extern "C" __attribute__((visibility("default")))

namespace {

struct Parser {
  const char* buf = nullptr;
  size_t len = 0;
  std::string delim;
  int ncols = 0;
  std::vector<int> kinds;                  // 0 skip, 1 numeric, 2 string
  std::unordered_set<std::string> missing; // tokens treated as missing (trimmed)
  std::vector<std::string> miss_list;      // the same, scanned by length + memcmp (no per-field hash)
  bool numeric_missing = false;            // some missing token is itself a decimal ("-999", "0"):
                                           // the inline numeric fast path must check the token list
  bool is_missing(std::string_view v) const {
    for (const auto& t : miss_list)
      if (t.size() == v.size() && (v.empty() || memcmp(t.data(), v.data(), v.size()) == 0)) return true;
    return false;
  }
  int nthreads = 1;
  // results
  size_t nrows = 0;
  std::vector<std::vector<double>> num;    // per numeric column (internal storage, shifu_csv_parse)
  std::vector<double*> numptr;             // per numeric column: where its rows are written
  std::vector<struct Chunk>* chunks = nullptr;
  std::vector<std::vector<int32_t>> codes; // per string column
  std::vector<std::vector<std::string>> dicts;
  std::vector<int> num_idx, str_idx;       // column -> slot
  std::vector<int> next_wanted;            // column -> first column >= it with kind != 0 (ncols: none)
  int64_t bad_rows = 0;
};

inline std::string_view trim(std::string_view s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) --b;
  return s.substr(a, b - a);
}

// Clinger's fast path: [+-]digits[.digits] with <= 19 significant digits whose integer value is
// < 2^53 and <= 22 fraction digits is m / 10^k with both operands exact doubles, so ONE IEEE
// division gives the correctly rounded value -- bit-identical to strtod -- without strtod's
// locale / generic machinery (the common shape of the numeric text: "%.5f"-like fields).
// Anything else (exponents, more digits, inf/nan words, Java "1.0d") takes the strtod path.
static const double kPow10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

inline bool parse_decimal_fast(std::string_view s, double& out) {
  size_t i = 0;
  const size_t n = s.size();
  bool neg = false;
  if (i < n && (s[i] == '-' || s[i] == '+')) { neg = s[i] == '-'; ++i; }
  uint64_t m = 0;
  int nd = 0, frac = 0;
  bool any = false, dot = false;
  for (; i < n; ++i) {
    const char c = s[i];
    if (c >= '0' && c <= '9') {
      any = true;
      if (m == 0 && c == '0') { if (dot) ++frac; continue; }     // leading zeros
      if (++nd > 19) return false;
      m = m * 10 + (uint64_t)(c - '0');
      if (dot) ++frac;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      return false;
    }
  }
  if (!any || m >= (1ull << 53) || frac > 22) return false;
  const double v = frac ? (double)m / kPow10[frac] : (double)m;
  out = neg ? -v : v;
  return true;
}

inline double parse_double(std::string_view s, bool& ok) {
  ok = false;
  if (s.empty()) return NAN;
  double fast;
  if (parse_decimal_fast(s, fast)) { ok = true; return fast; }
  char tmp[64];
  if (s.size() >= sizeof(tmp)) return NAN;
  memcpy(tmp, s.data(), s.size());
  tmp[s.size()] = 0;
  char* end = nullptr;
  double v = strtod(tmp, &end);
  if (end == tmp) return NAN;
  while (*end == ' ' || *end == 'd' || *end == 'D' || *end == 'f' || *end == 'F') ++end;   // Java "1.0d"
  if (*end != 0) return NAN;
  ok = true;
  return v;
}

// SSSE3 / SSE4.1 form of the same fast path for fields of <= 16 bytes that lie inside the buffer:
// one 16-byte load gives the delimiter, dot, sign and digit masks; a table shuffle right-aligns the
// digits around the dot; two madd steps fold 16 digits into two 8-digit halves.  The mantissa m
// and the fraction length are exactly the scalar loop's, so the value (m / 10^frac, one IEEE
// division) is bit-identical.  Returns false (caller takes the scalar path) for anything else.
struct DigitShuffles {
  alignas(16) int8_t m[2][17][17][16];   // [sign][integer digits][fraction digits]
  DigitShuffles() {
    for (int s0 = 0; s0 < 2; ++s0)
      for (int di = 0; di <= 16; ++di)
        for (int df = 0; df <= 16; ++df) {
          const int nd = di + df;
          for (int j = 0; j < 16; ++j) {
            const int t = j - (16 - nd);
            m[s0][di][df][j] = (nd > 16 || t < 0) ? (int8_t)0x80 : (int8_t)(s0 + t + (t >= di ? 1 : 0));
          }
        }
  }
};
static const DigitShuffles kShuf;

__attribute__((target("ssse3,sse4.1,popcnt,bmi")))
inline bool parse_field_simd(const char* p, size_t avail, char d0, double& out, size_t& flen) {
  if (avail < 16) return false;
  const __m128i v = _mm_loadu_si128((const __m128i*)p);
  const unsigned md = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(v, _mm_set1_epi8(d0))) |
                      (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(v, _mm_set1_epi8('\n')));
  if (!md) return false;                                  // field longer than 15 bytes
  const int L = __builtin_ctz(md);
  if (L == 0) return false;                               // empty field: the caller's missing rule
  const int s0 = (p[0] == '-' || p[0] == '+') ? 1 : 0;
  const __m128i x = _mm_sub_epi8(v, _mm_set1_epi8('0'));
  const unsigned mdig = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_min_epu8(x, _mm_set1_epi8(9)), x));
  const unsigned mdot = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(v, _mm_set1_epi8('.')));
  const unsigned field = ((1u << L) - 1) & ~((1u << s0) - 1);
  const unsigned dg = mdig & field, dt = mdot & field;
  if ((dg | dt) != field || !dg || (dt & (dt - 1))) return false;
  const int nd = __builtin_popcount(dg);
  int di = nd, df = 0;
  if (dt) { const int pd = __builtin_ctz(dt); di = pd - s0; df = L - pd - 1; }
  const __m128i d = _mm_shuffle_epi8(x, _mm_load_si128((const __m128i*)kShuf.m[s0][di][df]));
  const __m128i t1 = _mm_maddubs_epi16(d, _mm_setr_epi8(10, 1, 10, 1, 10, 1, 10, 1, 10, 1, 10, 1, 10, 1, 10, 1));
  const __m128i t2 = _mm_madd_epi16(t1, _mm_setr_epi16(100, 1, 100, 1, 100, 1, 100, 1));
  const __m128i t3 = _mm_packus_epi32(t2, t2);
  const __m128i t4 = _mm_madd_epi16(t3, _mm_setr_epi16(10000, 1, 10000, 1, 10000, 1, 10000, 1));
  const uint64_t m = (uint64_t)(uint32_t)_mm_cvtsi128_si32(t4) * 100000000ull +
                     (uint32_t)_mm_extract_epi32(t4, 1);
  const double val = df ? (double)m / kPow10[df] : (double)m;
  out = (s0 && p[0] == '-') ? -val : val;
  flen = (size_t)L;
  return true;
}

// Position of the n-th (1-based) single-byte delimiter in [p, e), 16 bytes per step (compare +
// popcount); `found` = delimiters seen (n when returned position < e).  Runs of unparsed columns
// are skipped with this instead of one memchr per field (a norm pass over 200 of 1600 columns, or
// the GPU-parse framing pass that only keeps the target/weight columns, skips 1400+ per line).
__attribute__((target("sse2,popcnt,bmi")))
inline size_t nth_delim(const char* buf, size_t p, size_t e, char d0, long n, long& found) {
  long cnt = 0;
  size_t i = p;
  const __m128i vd = _mm_set1_epi8(d0);
  for (; i + 16 <= e; i += 16) {
    unsigned m = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(buf + i)), vd));
    const int c = __builtin_popcount(m);
    if (cnt + c >= n) {
      for (long t = cnt + 1; t < n; ++t) m &= m - 1;
      found = n;
      return i + (size_t)__builtin_ctz(m);
    }
    cnt += c;
  }
  for (; i < e; ++i)
    if (buf[i] == d0 && ++cnt == n) { found = n; return i; }
  found = cnt;
  return e;
}

struct Chunk {
  size_t begin, end;           // byte range (line aligned)
  std::vector<size_t> line_starts;
  size_t row_offset = 0;
  std::vector<std::unordered_map<std::string, int32_t>> local_dict;   // per string col
  std::vector<std::vector<std::string>> local_list;
};

void split_lines(const Parser& P, Chunk& c) {
  size_t i = c.begin;
  while (i < c.end) {
    const char* nl = (const char*)memchr(P.buf + i, '\n', c.end - i);
    const size_t j = nl ? (size_t)(nl - P.buf) : c.end;
    // skip blank lines
    size_t k = i;
    while (k < j && (P.buf[k] == ' ' || P.buf[k] == '\r' || P.buf[k] == '\t')) ++k;
    if (k < j) c.line_starts.push_back(i);
    i = j + 1;
  }
}

// One line: fields are tokenised and numeric fields converted in the same left-to-right pass.  A
// numeric field of the common shape ([+-]digits[.digits], <= 19 significant digits, < 2^53,
// <= 22 fraction digits) is accumulated while it is scanned and finished with one division
// (Clinger's fast path, == strtod); an empty field is missing; anything else (spaces, missing
// tokens, exponents, Java "1.0d", strings) is re-scanned to its delimiter and takes the general
// path (trim, missing tokens, strtod / dictionary).
// Numeric values go to row_out[slot] (a row of the caller's row-major tile); string codes straight
// to their column (one int per row, sequential).
void parse_line(Parser& P, Chunk& c, size_t s, size_t e, size_t r, double* row_out, std::atomic<int64_t>& bad) {
  const char d0 = P.delim[0];
  const size_t dl = P.delim.size();
  const char* buf = P.buf;
  int col = 0;
  size_t p = s;
  auto field_end = [&](size_t a) -> size_t {     // first delimiter at or after a (or e)
    if (dl == 1) {
      const void* q = memchr(buf + a, d0, e - a);
      return q ? (size_t)((const char*)q - buf) : e;
    }
    for (size_t i = a; i + dl <= e; ++i)
      if (buf[i] == d0 && memcmp(buf + i, P.delim.data(), dl) == 0) return i;
    return e;
  };
  auto general = [&](size_t a, size_t b) {
    const int k = P.kinds[col];
    std::string_view v = trim(std::string_view(buf + a, b - a));
    const bool miss = P.is_missing(v);
    if (k == 1) {
      bool ok = false;
      row_out[P.num_idx[col]] = miss ? NAN : parse_double(v, ok);
    } else {
      int32_t code = -1;
      if (!miss) {
        auto& m = c.local_dict[col];
        std::string key(v);
        auto it = m.find(key);
        if (it == m.end()) {
          code = (int32_t)c.local_list[col].size();
          m.emplace(key, code);
          c.local_list[col].push_back(std::move(key));
        } else {
          code = it->second;
        }
      }
      P.codes[P.str_idx[col]][r] = code;   // local code, remapped after merge
    }
  };
  while (true) {
    const int k = col < P.ncols ? P.kinds[col] : 0;
    if (k == 0 && dl == 1) {
      // a run of unparsed fields: jump to the next parsed column's field (or count the rest of
      // the line's fields for the column-count check)
      const long skip = col < P.ncols ? (long)(P.next_wanted[col] - col) : (long)1 << 62;
      long found = 0;
      const size_t q = nth_delim(buf, p, e, d0, skip, found);
      if (found < skip) {                            // the line ends inside the run
        col += (int)std::min<long>(found + 1, (long)1 << 30);
        break;
      }
      col += (int)skip;
      p = q + 1;
      continue;
    }
    size_t b;                                      // field end
    double sv;
    size_t sl;
    if (k == 1 && dl == 1 && p < e &&
        parse_field_simd(buf + p, P.len - p, d0, sv, sl) && p + sl <= e &&
        !(P.numeric_missing && P.is_missing(std::string_view(buf + p, sl)))) {
      b = p + sl;
      row_out[P.num_idx[col]] = sv;
    } else if (k == 1 && dl == 1) {
      size_t i = p;
      bool neg = false;
      if (i < e && (buf[i] == '-' || buf[i] == '+')) { neg = buf[i] == '-'; ++i; }
      uint64_t m = 0;
      int nd = 0, frac = 0;
      bool any = false, dot = false, fast = true;
      for (; i < e; ++i) {
        const char ch = buf[i];
        const unsigned dgt = (unsigned)(ch - '0');
        if (dgt < 10) {
          any = true;
          if (m == 0 && dgt == 0) { frac += dot; continue; }
          if (++nd > 19) { fast = false; break; }
          m = m * 10 + dgt;
          frac += dot;
        } else if (ch == '.' && !dot) {
          dot = true;
        } else {
          if (ch != d0) fast = false;
          break;
        }
      }
      if (fast && i == p) {                        // empty field: missing (token or not)
        b = i;
        row_out[P.num_idx[col]] = NAN;
      } else if (fast && any && m < (1ull << 53) && frac <= 22 &&
                 !(P.numeric_missing && P.is_missing(std::string_view(buf + p, i - p)))) {
        b = i;
        const double v = frac ? (double)m / kPow10[frac] : (double)m;
        row_out[P.num_idx[col]] = neg ? -v : v;
      } else {
        b = field_end(p);
        general(p, b);
      }
    } else {
      b = field_end(p);
      if (k != 0) general(p, b);
    }
    ++col;
    if (b >= e) break;
    p = b + dl;
  }
  if (col != P.ncols) {
    bad.fetch_add(1);
    for (int cc = col; cc < P.ncols; ++cc) {   // short row: rest missing
      if (P.kinds[cc] == 1) row_out[P.num_idx[cc]] = NAN;
      else if (P.kinds[cc] == 2) P.codes[P.str_idx[cc]][r] = -1;
    }
  }
}

// Lines are parsed TILE rows at a time into a row-major [TILE][n_numeric] scratch tile, which is
// then written out column by column (TILE consecutive doubles per column).  Writing each field
// straight to its column touched one page and one cache line per field (n_numeric pages per row:
// a DTLB miss per value at 1600 columns); the tile keeps the parse in L2 and the column writes
// contiguous.
constexpr int TILE = 32;

void parse_chunk(Parser& P, Chunk& c, std::atomic<int64_t>& bad) {
  c.local_dict.assign(P.ncols, {});
  c.local_list.assign(P.ncols, {});
  const size_t nn = P.numptr.size();
  std::vector<double> tile(std::max<size_t>(1, nn) * TILE);
  const size_t nl_total = c.line_starts.size();
  for (size_t l0 = 0; l0 < nl_total; l0 += TILE) {
    const size_t l1 = std::min(nl_total, l0 + TILE);
    for (size_t li = l0; li < l1; ++li) {
      const size_t s = c.line_starts[li];
      const size_t e = li + 1 < nl_total ? c.line_starts[li + 1] - 1 : c.end;
      const char* nl = (const char*)memchr(P.buf + s, '\n', e - s);   // blank lines were skipped
      parse_line(P, c, s, nl ? (size_t)(nl - P.buf) : e, c.row_offset + li, tile.data() + (li - l0) * nn, bad);
    }
    const size_t rows = l1 - l0, r0 = c.row_offset + l0;
    for (size_t k = 0; k < nn; ++k) {
      double* dst = P.numptr[k] + r0;
      const double* src = tile.data() + k;
      for (size_t i = 0; i < rows; ++i) dst[i] = src[i * nn];
    }
  }
}

}  // namespace

// Phase 1: split `buf` (len bytes) at line boundaries over `nthreads` threads and count the
// rows.  kinds[ncols]: 0 skip, 1 numeric, 2 string.  missing: '\n'-joined tokens.  Returns an
// opaque handle (nullptr on error); shifu_csv_nrows gives the row count for sizing the output.
SHIFU_RT_API void* shifu_csv_scan(const char* buf, long len, const char* delim, int ncols, const int* kinds,
                                  const char* missing, int nthreads) {
  auto* P = new Parser();
  P->buf = buf;
  P->len = (size_t)len;
  P->delim = delim && *delim ? delim : "|";
  P->ncols = ncols;
  P->kinds.assign(kinds, kinds + ncols);
  if (missing) {
    std::string m(missing);
    size_t a = 0;
    while (true) {
      size_t b = m.find('\n', a);
      std::string tok = m.substr(a, b == std::string::npos ? std::string::npos : b - a);
      P->missing.insert(std::string(trim(tok)));
      if (b == std::string::npos) break;
      a = b + 1;
    }
  }
  P->miss_list.assign(P->missing.begin(), P->missing.end());
  for (const auto& t : P->miss_list) {
    double v;
    if (!t.empty() && parse_decimal_fast(t, v)) P->numeric_missing = true;
  }
  P->nthreads = std::max(1, nthreads);
  for (int c = 0; c < ncols; ++c) {
    P->num_idx.push_back(-1);
    P->str_idx.push_back(-1);
  }
  int nn = 0, ns = 0;
  for (int c = 0; c < ncols; ++c) {
    if (P->kinds[c] == 1) P->num_idx[c] = nn++;
    else if (P->kinds[c] == 2) P->str_idx[c] = ns++;
  }
  P->next_wanted.assign(ncols + 1, ncols);
  for (int c = ncols - 1; c >= 0; --c) P->next_wanted[c] = P->kinds[c] ? c : P->next_wanted[c + 1];
  // chunking at line boundaries
  const int T = P->nthreads;
  P->chunks = new std::vector<Chunk>(T);
  auto& chunks = *P->chunks;
  size_t pos = 0;
  for (int t = 0; t < T; ++t) {
    size_t target = (P->len * (t + 1)) / T;
    if (t == T - 1) target = P->len;
    else {
      while (target < P->len && buf[target] != '\n') ++target;
      if (target < P->len) ++target;
    }
    chunks[t].begin = pos;
    chunks[t].end = std::max(pos, target);
    pos = chunks[t].end;
  }
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { split_lines(*P, chunks[t]); });
    for (auto& x : th) x.join();
  }
  size_t rows = 0;
  for (auto& c : chunks) { c.row_offset = rows; rows += c.line_starts.size(); }
  P->nrows = rows;
  return P;
}

// Phase 2: parse every row.  num_out: the numeric columns (in column order) as the rows of a
// [n_numeric][ld] double block (ld >= nrows), or nullptr for internal storage (then read them
// with shifu_csv_numeric).  String columns -> codes + dictionaries (shifu_csv_codes / _dict).
SHIFU_RT_API int shifu_csv_fill(void* h, double* num_out, long ld) {
  auto* P = (Parser*)h;
  if (!P || !P->chunks) return -1;
  auto& chunks = *P->chunks;
  const size_t rows = P->nrows;
  int nn = 0, ns = 0;
  for (int c = 0; c < P->ncols; ++c) nn += P->kinds[c] == 1, ns += P->kinds[c] == 2;
  P->numptr.assign(nn, nullptr);
  if (num_out) {
    if (ld < (long)rows) return -2;
    for (int i = 0; i < nn; ++i) P->numptr[i] = num_out + (size_t)i * (size_t)ld;
  } else {
    P->num.assign(nn, std::vector<double>(rows));
    for (int i = 0; i < nn; ++i) P->numptr[i] = P->num[i].data();
  }
  P->codes.assign(ns, std::vector<int32_t>(rows));
  std::atomic<int64_t> bad{0};
  {
    std::vector<std::thread> th;
    const int T = (int)chunks.size();
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { parse_chunk(*P, chunks[t], bad); });
    for (auto& x : th) x.join();
  }
  P->bad_rows = bad.load();
  // merge dictionaries in chunk order (first-seen order across the file) and remap codes
  P->dicts.assign(ns, {});
  for (int c = 0; c < P->ncols; ++c) {
    if (P->kinds[c] != 2) continue;
    const int si = P->str_idx[c];
    std::unordered_map<std::string, int32_t> global;
    for (auto& ch : chunks) {
      std::vector<int32_t> remap(ch.local_list[c].size());
      for (size_t i = 0; i < ch.local_list[c].size(); ++i) {
        const std::string& s = ch.local_list[c][i];
        auto it = global.find(s);
        if (it == global.end()) {
          const int32_t g = (int32_t)P->dicts[si].size();
          global.emplace(s, g);
          P->dicts[si].push_back(s);
          remap[i] = g;
        } else {
          remap[i] = it->second;
        }
      }
      int32_t* codes = P->codes[si].data();
      for (size_t li = 0; li < ch.line_starts.size(); ++li) {
        const size_t r = ch.row_offset + li;
        if (codes[r] >= 0) codes[r] = remap[codes[r]];
      }
    }
  }
  for (auto& ch : chunks) {                     // release the per-chunk line tables / local dicts
    std::vector<size_t>().swap(ch.line_starts);
    ch.local_dict.clear();
    ch.local_list.clear();
  }
  return 0;
}

// One-call form: scan + fill into internal storage.
SHIFU_RT_API void* shifu_csv_parse(const char* buf, long len, const char* delim, int ncols, const int* kinds,
                                   const char* missing, int nthreads) {
  void* h = shifu_csv_scan(buf, len, delim, ncols, kinds, missing, nthreads);
  if (h && shifu_csv_fill(h, nullptr, 0) != 0) {
    delete (Parser*)h;
    return nullptr;
  }
  return h;
}

SHIFU_RT_API long shifu_csv_nrows(void* h) { return (long)((Parser*)h)->nrows; }
SHIFU_RT_API long shifu_csv_bad_rows(void* h) { return (long)((Parser*)h)->bad_rows; }

SHIFU_RT_API int shifu_csv_numeric(void* h, int col, double* out) {
  auto* P = (Parser*)h;
  if (col < 0 || col >= P->ncols || P->num_idx[col] < 0) return -1;
  const double* v = P->numptr.empty() ? nullptr : P->numptr[P->num_idx[col]];
  if (v && P->nrows && v != out) memcpy(out, v, P->nrows * sizeof(double));   // (empty input: no rows)
  return 0;
}

SHIFU_RT_API int shifu_csv_codes(void* h, int col, int32_t* out) {
  auto* P = (Parser*)h;
  if (col < 0 || col >= P->ncols || P->str_idx[col] < 0) return -1;
  const auto& v = P->codes[P->str_idx[col]];
  if (!v.empty()) memcpy(out, v.data(), v.size() * sizeof(int32_t));
  return 0;
}

// dictionary of a string column serialized as '\n'-joined values; returns the byte size needed
SHIFU_RT_API long shifu_csv_dict(void* h, int col, char* out, long cap) {
  auto* P = (Parser*)h;
  if (col < 0 || col >= P->ncols || P->str_idx[col] < 0) return -1;
  const auto& d = P->dicts[P->str_idx[col]];
  long need = 0;
  for (size_t i = 0; i < d.size(); ++i) need += (long)d[i].size() + (i + 1 < d.size() ? 1 : 0);
  if (out && cap >= need) {
    long p = 0;
    for (size_t i = 0; i < d.size(); ++i) {
      if (!d[i].empty()) memcpy(out + p, d[i].data(), d[i].size());
      p += (long)d[i].size();
      if (i + 1 < d.size()) out[p++] = '\n';
    }
  }
  return need;
}

SHIFU_RT_API long shifu_csv_dict_size(void* h, int col) {
  auto* P = (Parser*)h;
  if (col < 0 || col >= P->ncols || P->str_idx[col] < 0) return -1;
  return (long)P->dicts[P->str_idx[col]].size();
}

SHIFU_RT_API void shifu_csv_free(void* h) {
  auto* P = (Parser*)h;
  if (!P) return;
  delete P->chunks;
  delete P;
}

// The GPU field parser's fallback list (ops/csrc/csv_kernels.hip): n entries (line, slot, start,
// end) of trimmed, non-missing fields its Clinger fast path did not take -> the same strtod path
// the host parser's general branch uses, so GPU-parsed blocks equal host-parsed ones bit for bit.
SHIFU_RT_API long shifu_parse_fields(const char* buf, const long* fb, long n, double* out) {
  for (long k = 0; k < n; ++k) {
    const long a = fb[4 * k + 2], b = fb[4 * k + 3];
    bool ok = false;
    out[k] = parse_double(std::string_view(buf + a, (size_t)(b - a)), ok);
  }
  return n;
}

// The host-parsed columns of a GPU-parsed block, from the field bounds the GPU field parser
// handed back (offs [k][nl][2] int32): one short line "f_0<d>f_1<d>...f_{k-1}<d>x\n" per non-blank
// line (lflags bit 0 clear; the trailing unparsed "x" field keeps a line of empty fields from
// reading as blank) -- the host parser then reads only these bytes instead of scanning the whole
// block.  Returns the bytes written, or -1 when `cap` is too small.
SHIFU_RT_API long shifu_gather_fields(const char* buf, const int* offs, long nl, int k, const int* lflags,
                                      const char* delim, char* out, long cap) {
  long p = 0;
  const char d = delim && *delim ? delim[0] : '|';
  for (long l = 0; l < nl; ++l) {
    if (lflags[l] & 1) continue;
    for (int j = 0; j < k; ++j) {
      const int* o = offs + 2 * ((long)j * nl + l);
      const long n = (long)o[1] - (long)o[0];
      if (n < 0 || p + n + 1 > cap) return -1;
      memcpy(out + p, buf + o[0], (size_t)n);
      p += n;
      out[p++] = d;
    }
    if (p + 2 > cap) return -1;
    out[p++] = 'x';
    out[p++] = '\n';
  }
  return p;
}
