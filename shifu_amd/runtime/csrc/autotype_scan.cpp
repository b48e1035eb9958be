// Streamed auto-type statistics for `init` with dataSet.autoType (B3 / H5).
//
// The reference runs a MapReduce job over every row (AutoTypeDistinctCountMapper.java:134-219 +
// AutoTypeDistinctCountReducer; InitModelProcessor.java:105-120, 143-254): per column the row
// count, the missing-or-invalid count, the count of values Double.parseDouble accepts, a
// HyperLogLog++ (p = 8) distinct estimate and up to 21 "frequent" (first seen) distinct values per
// mapper, 200 after the reducer's union; rows whose trimmed tag is not a configured tag are skipped.
//
// Here each rank scans its byte ranges of the text once (multi-threaded per block, every
// non-blank line a row exactly as the CSV parser frames them) and keeps per column:
//   * count / invalid / valid-number counts (int64);
//   * the exact set of 64-bit value hashes while it stays below AT_EXACT_CAP distinct values, and
//     always a HyperLogLog sketch with 2^14 registers (0.8 % standard error) -- the distinct
//     count is exact for the low-cardinality columns the type rule looks at (the reference's
//     p = 8 sketch is ~6.5 % off there), HLL above;
//   * the first 21 distinct non-missing values per thread, 200 per rank.
// Partial states merge by sums (counts), set union (exact hashes, below the cap), register max
// (HLL) and ordered union (items) -- within a rank here, across ranks in steps/create.py.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#define SHIFU_RT_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int AT_HLL_P = 14;
constexpr int AT_HLL_M = 1 << AT_HLL_P;
constexpr int AT_EXACT_CAP = 4096;            // distinct values tracked exactly per column
constexpr int AT_ITEMS_THREAD = 21;           // AutoTypeDistinctCountMapper: add while size <= 20
constexpr int AT_ITEMS_RANK = 200;            // the reducer's union limit (FREQUET_ITEM_MAX_SIZE * 10)

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

inline uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0x9e3779b97f4a7c15ull ^ (n * 0xff51afd7ed558ccdull);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = mix64(h ^ w) + 0x9e3779b97f4a7c15ull;
  }
  uint64_t t = 0;
  for (size_t k = 0; i + k < n; ++k) t |= (uint64_t)(uint8_t)p[i + k] << (8 * k);
  return mix64(h ^ t ^ 0x2545f4914f6cdd1dull);
}

// The field hash: fields of up to 8 bytes (most numeric text) are one zero-padded little-endian
// word -- loaded with one 8-byte read when `end` allows, else byte by byte: the same value
// hashes the same either way.
inline uint64_t hash_field(const char* p, size_t n, const char* end) {
  if (n > 8) return hash_bytes(p, n);
  uint64_t w = 0;
  if (p + 8 <= end) {
    memcpy(&w, p, 8);
    if (n < 8) w &= (1ull << (8 * n)) - 1;
  } else {
    for (size_t k = 0; k < n; ++k) w |= (uint64_t)(uint8_t)p[k] << (8 * k);
  }
  return mix64(w ^ (n * 0xff51afd7ed558ccdull) ^ 0x2545f4914f6cdd1dull);
}

// Double.parseDouble's grammar (whitespace-trimmed; NaN / Infinity, a trailing d/D/f/F type
// suffix; hexadecimal floats are not recognised)
bool java_double(const char* p, size_t n) {
  size_t a = 0, b = n;
  while (a < b && (uint8_t)p[a] <= ' ') ++a;
  while (b > a && (uint8_t)p[b - 1] <= ' ') --b;
  if (a == b) return false;
  if (p[a] == '+' || p[a] == '-') ++a;
  const size_t m = b - a;
  if (m == 3 && !memcmp(p + a, "NaN", 3)) return true;
  if (m == 8 && !memcmp(p + a, "Infinity", 8)) return true;
  if (b > a && (p[b - 1] == 'd' || p[b - 1] == 'D' || p[b - 1] == 'f' || p[b - 1] == 'F')) --b;
  size_t i = a;
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

// rank-level state of one column (sketches owned by one thread at a time, see shifu_at_feed)
struct Col {
  int64_t count = 0, invalid = 0, validnum = 0;
  std::vector<uint64_t> table;                // open addressing, 0 = empty
  int used = 0;
  bool overflow = false;
  std::vector<uint8_t> hll;                   // AT_HLL_M registers (allocated on first value)
  std::vector<std::string> items;
  std::unordered_set<std::string> item_set;

  void add_hash(uint64_t h) {                 // h != 0
    if (hll.empty()) hll.assign(AT_HLL_M, 0);
    const uint32_t idx = (uint32_t)(h >> (64 - AT_HLL_P));
    const uint64_t rest = (h << AT_HLL_P) | (1ull << (AT_HLL_P - 1));
    const uint8_t rank = (uint8_t)(__builtin_clzll(rest) + 1);
    if (rank > hll[idx]) hll[idx] = rank;
    if (overflow) return;
    if (table.empty()) table.assign(64, 0);
    if ((used + 1) * 2 > (int)table.size()) {
      if (used + 1 > AT_EXACT_CAP) {
        overflow = true;
        std::vector<uint64_t>().swap(table);
        return;
      }
      std::vector<uint64_t> t2(table.size() * 2, 0);
      for (uint64_t v : table)
        if (v) {
          size_t k = v & (t2.size() - 1);
          while (t2[k]) k = (k + 1) & (t2.size() - 1);
          t2[k] = v;
        }
      table.swap(t2);
    }
    size_t k = h & (table.size() - 1);
    while (table[k]) {
      if (table[k] == h) return;
      k = (k + 1) & (table.size() - 1);
    }
    table[k] = h;
    ++used;
  }
};

// first-seen distinct values of one column in one scanner thread (AT_ITEMS_THREAD of them)
struct Items {
  std::vector<std::string> items;
  std::unordered_set<std::string> set;
  void add(const char* p, size_t n) {
    if ((int)items.size() >= AT_ITEMS_THREAD) return;
    std::string s(p, n);
    if (set.insert(s).second) items.push_back(std::move(s));
  }
};

struct State {
  int ncols = 0, tag_col = -1;
  std::string delim;
  std::vector<std::string> tags;              // trimmed
  std::vector<std::string> missing;           // compared with the lower-cased raw field
  size_t missing_max = 0;                     // longest missing token
  std::vector<Col> cols;                      // counts and sketches
  std::vector<std::vector<Items>> part;       // per scanner thread, merged on query
  int64_t rows = 0, skipped_tag = 0;
  bool dirty = false;                         // per-thread items not merged yet
};

inline bool is_blank_line(const char* s, const char* e) {
  for (const char* q = s; q < e; ++q)
    if (*q != ' ' && *q != '\r' && *q != '\t') return false;
  return true;
}

// the raw field lower-cased equals one of the missing tokens (no allocation: tokens are short)
inline bool is_missing(const State& S, const char* v, size_t n) {
  if (n > S.missing_max) return false;
  for (const std::string& m : S.missing) {
    if (m.size() != n) continue;
    size_t i = 0;
    while (i < n && (char)tolower((unsigned char)v[i]) == m[i]) ++i;
    if (i == n) return true;
  }
  return false;
}

// per-field code of the row pass: 0 absent (short row), 1 missing-or-invalid, otherwise
// (63-bit value hash << 1) | parses-as-a-Java-double
constexpr uint64_t AT_ABSENT = 0, AT_MISSING = 1;

// Row pass of one thread over lines [s, e): tag / mask filter, field split, per field a code into
// the column-major buffer codes[c * cap + i] (i = kept row), first-seen items.  Returns kept rows.
int64_t code_rows(const State& S, std::vector<Items>& items, const char* s, const char* e, const uint8_t* mask,
                  int64_t row0, uint64_t* codes, int64_t cap, int64_t* skipped_out) {
  const char* d = S.delim.data();
  const size_t dl = S.delim.size();
  const int NC = S.ncols;
  int64_t r = row0, skipped = 0, nb = 0;
  std::vector<std::pair<const char*, size_t>> f;
  for (const char* p = s; p < e;) {
    const char* nl = (const char*)memchr(p, '\n', e - p);
    const char* le = nl ? nl : e;
    const char* next = nl ? nl + 1 : e;
    const char* lend = (le > p && le[-1] == '\r') ? le - 1 : le;
    if (is_blank_line(p, le)) { p = next; continue; }
    const int64_t row = r++;
    if (mask && !mask[row]) { p = next; continue; }
    f.clear();
    const char* q = p;
    while (true) {
      const char* hit = dl == 1 ? (const char*)memchr(q, d[0], lend - q) : nullptr;
      if (dl > 1) {
        for (const char* t = q; t + dl <= lend; ++t)
          if (!memcmp(t, d, dl)) { hit = t; break; }
      }
      if (!hit) { f.emplace_back(q, (size_t)(lend - q)); break; }
      f.emplace_back(q, (size_t)(hit - q));
      q = hit + dl;
    }
    if (S.tag_col >= 0) {
      if (S.tag_col >= (int)f.size()) { ++skipped; p = next; continue; }
      const char* t = f[S.tag_col].first;
      size_t a = 0, b = f[S.tag_col].second;
      while (a < b && (uint8_t)t[a] <= ' ') ++a;
      while (b > a && (uint8_t)t[b - 1] <= ' ') --b;
      bool ok = false;
      for (auto& tg : S.tags)
        if (tg.size() == b - a && !memcmp(tg.data(), t + a, b - a)) { ok = true; break; }
      if (!ok) { ++skipped; p = next; continue; }
    }
    if (nb >= cap) break;                     // cannot happen: cap = the chunk's line count
    const int nf = std::min((int)f.size(), NC);
    uint64_t* cr = codes + nb;
    for (int c = 0; c < nf; ++c) {
      const char* v = f[c].first;
      const size_t n = f[c].second;
      if (is_missing(S, v, n)) { cr[(size_t)c * cap] = AT_MISSING; continue; }
      uint64_t h = hash_field(v, n, e) >> 1;
      if (!h) h = 1;
      cr[(size_t)c * cap] = (h << 1) | (java_double(v, n) ? 1u : 0u);
      items[c].add(v, n);
    }
    for (int c = nf; c < NC; ++c) cr[(size_t)c * cap] = AT_ABSENT;
    ++nb;
    p = next;
  }
  *skipped_out = skipped;
  return nb;
}

// Column pass over columns [c0, c1): every chunk's codes (chunk order) into the column's counts,
// exact set and registers -- each column's sketch is touched by this thread only, for all the
// rows of the sub-block in a row, so it stays in this core's cache.
void apply_codes(State& S, int c0, int c1, const std::vector<std::vector<uint64_t>>& codes,
                 const std::vector<int64_t>& cap, const std::vector<int64_t>& kept) {
  for (int c = c0; c < c1; ++c) {
    Col& C = S.cols[c];
    for (size_t u = 0; u < codes.size(); ++u) {
      const uint64_t* x = codes[u].data() + (size_t)c * cap[u];
      for (int64_t i = 0; i < kept[u]; ++i) {
        const uint64_t v = x[i];
        if (v == AT_ABSENT) continue;
        C.count += 1;
        if (v == AT_MISSING) { C.invalid += 1; continue; }
        C.validnum += (int64_t)(v & 1);
        C.add_hash(v | 1);                  // top bits: the hash; odd: never the empty slot
      }
    }
  }
}

// per-thread item lists -> the rank's (thread order: the lists keep the text order)
void merge_parts(State& S) {
  if (!S.dirty) return;
  S.dirty = false;
  for (int c = 0; c < S.ncols; ++c) {
    Col& C = S.cols[c];
    for (auto& pt : S.part) {
      for (auto& it : pt[c].items) {
        if ((int)C.items.size() >= AT_ITEMS_RANK) break;
        if (C.item_set.insert(it).second) C.items.push_back(it);
      }
      pt[c] = Items();
    }
  }
}

constexpr long AT_SUB_BYTES = 32l << 20;      // sub-block: bounds the code buffers (~8 B per field)

std::vector<std::string> split_blob(const char* blob, bool trim) {
  std::vector<std::string> out;
  if (!blob) return out;
  const char* p = blob;
  while (*p) {
    const char* e = strchr(p, '\n');
    std::string s = e ? std::string(p, e - p) : std::string(p);
    if (trim) {
      size_t a = 0, b = s.size();
      while (a < b && (uint8_t)s[a] <= ' ') ++a;
      while (b > a && (uint8_t)s[b - 1] <= ' ') --b;
      s = s.substr(a, b - a);
    }
    out.push_back(s);
    if (!e) break;
    p = e + 1;
  }
  return out;
}

}  // namespace

// tags / missing: '\n'-joined (missing tokens as configured: the raw field is lower-cased and
// compared with them, as the mapper does); tag_col < 0: no tag filter
SHIFU_RT_API void* shifu_at_new(int ncols, int tag_col, const char* tags, const char* missing, const char* delim) {
  if (ncols <= 0 || !delim || !*delim) return nullptr;
  State* S = new State();
  S->ncols = ncols;
  S->tag_col = tag_col;
  S->delim = delim;
  S->tags = split_blob(tags, true);
  for (auto& m : split_blob(missing, false)) {
    S->missing_max = std::max(S->missing_max, m.size());
    S->missing.push_back(m);
  }
  S->cols.resize(ncols);
  return S;
}

// Scan a block of complete lines; mask (nullable): keep flag per non-blank line of the block (the
// purifier's filter expression).  Returns the rows counted (tag filter passed) or -1.
// Sub-blocks of AT_SUB_BYTES: `nthreads` threads code their line-aligned chunks (row pass), then
// the same threads each own a slice of the columns and apply every chunk's codes to it.
SHIFU_RT_API long shifu_at_feed(void* h, const char* buf, long len, const uint8_t* mask, int nthreads) {
  if (!h || len < 0) return -1;
  State& S = *(State*)h;
  const int NC = S.ncols;
  long tot = 0;
  int64_t mrow = 0;                             // mask rows before the sub-block
  for (long sb0 = 0; sb0 < len;) {
    long sb1 = std::min(len, sb0 + AT_SUB_BYTES);
    if (sb1 < len) {
      const char* nl = (const char*)memchr(buf + sb1, '\n', len - sb1);
      sb1 = nl ? (long)(nl - buf) + 1 : len;
    }
    const char* s0 = buf + sb0;
    const long sl = sb1 - sb0;
    const int T = std::max(1, std::min(nthreads, (int)(sl >> 20) + 1));
    if ((int)S.part.size() < T) {
      S.part.resize(T);
      for (auto& pt : S.part)
        if ((int)pt.size() != NC) pt.resize(NC);
    }
    std::vector<const char*> cut(T + 1);
    cut[0] = s0;
    cut[T] = s0 + sl;
    for (int t = 1; t < T; ++t) {
      const char* c = std::max(s0 + (sl * t) / T, cut[t - 1]);
      const char* nl = (const char*)memchr(c, '\n', s0 + sl - c);
      cut[t] = nl ? nl + 1 : s0 + sl;
    }
    // lines per chunk (buffer rows) and non-blank rows before each chunk (mask numbering)
    std::vector<int64_t> lines(T, 0), row0(T, 0);
    {
      std::vector<std::thread> th;
      auto count = [&](int t) {
        int64_t nlines = 0, nonblank = 0;
        for (const char* p = cut[t]; p < cut[t + 1];) {
          const char* nl = (const char*)memchr(p, '\n', cut[t + 1] - p);
          const char* le = nl ? nl : cut[t + 1];
          ++nlines;
          if (mask && !is_blank_line(p, le)) ++nonblank;
          p = nl ? nl + 1 : cut[t + 1];
        }
        lines[t] = nlines;
        row0[t] = nonblank;                      // prefix-summed below
      };
      for (int t = 1; t < T; ++t) th.emplace_back(count, t);
      count(0);
      for (auto& x : th) x.join();
    }
    int64_t r = mrow;
    for (int t = 0; t < T; ++t) { const int64_t nbk = row0[t]; row0[t] = r; r += nbk; }
    mrow = r;
    std::vector<std::vector<uint64_t>> codes(T);
    std::vector<int64_t> cap(T), kept(T, 0), skipped(T, 0);
    for (int t = 0; t < T; ++t) {
      cap[t] = std::max<int64_t>(1, lines[t]);
      codes[t].resize((size_t)cap[t] * NC);
    }
    {
      std::vector<std::thread> th;
      auto rowpass = [&](int t) {
        kept[t] = code_rows(S, S.part[t], cut[t], cut[t + 1], mask, row0[t], codes[t].data(), cap[t], &skipped[t]);
      };
      for (int t = 1; t < T; ++t) th.emplace_back(rowpass, t);
      rowpass(0);
      for (auto& x : th) x.join();
    }
    {
      const int TC = std::max(1, std::min(T, (NC + 15) / 16));
      std::vector<std::thread> th;
      auto colpass = [&](int t) {
        apply_codes(S, (int)((int64_t)NC * t / TC), (int)((int64_t)NC * (t + 1) / TC), codes, cap, kept);
      };
      for (int t = 1; t < TC; ++t) th.emplace_back(colpass, t);
      colpass(0);
      for (auto& x : th) x.join();
    }
    for (int t = 0; t < T; ++t) { tot += kept[t]; S.skipped_tag += skipped[t]; }
    sb0 = sb1;
  }
  S.rows += tot;
  S.dirty = true;
  return tot;
}

// out[3 * ncols]: count, invalid, valid-number per column; returns the rows scanned
SHIFU_RT_API long shifu_at_counts(void* h, int64_t* out) {
  State& S = *(State*)h;
  merge_parts(S);
  for (int c = 0; c < S.ncols; ++c) {
    out[3 * c] = S.cols[c].count;
    out[3 * c + 1] = S.cols[c].invalid;
    out[3 * c + 2] = S.cols[c].validnum;
  }
  return (long)S.rows;
}

// the exact hash set of a column (sorted) into out (cap entries); -1 when the column overflowed
SHIFU_RT_API long shifu_at_exact(void* h, int col, uint64_t* out, long cap) {
  State& S = *(State*)h;
  merge_parts(S);
  if (col < 0 || col >= S.ncols) return -2;
  Col& C = S.cols[col];
  if (C.overflow) return -1;
  long n = 0;
  for (uint64_t v : C.table)
    if (v) {
      if (n >= cap) return -3;
      out[n++] = v;
    }
  std::sort(out, out + n);
  return n;
}

SHIFU_RT_API int shifu_at_hll_p() { return AT_HLL_P; }
SHIFU_RT_API int shifu_at_exact_cap() { return AT_EXACT_CAP; }

// HLL registers of every column: out[ncols][2^p]
SHIFU_RT_API int shifu_at_hll(void* h, uint8_t* out) {
  State& S = *(State*)h;
  merge_parts(S);
  for (int c = 0; c < S.ncols; ++c) {
    if (S.cols[c].hll.empty()) memset(out + (size_t)c * AT_HLL_M, 0, AT_HLL_M);
    else memcpy(out + (size_t)c * AT_HLL_M, S.cols[c].hll.data(), AT_HLL_M);
  }
  return 0;
}

// HyperLogLog estimate (with the small-range linear-counting correction) of registers [2^p]
SHIFU_RT_API double shifu_at_hll_estimate(const uint8_t* reg) {
  const double m = AT_HLL_M;
  double z = 0.0;
  int zeros = 0;
  for (int i = 0; i < AT_HLL_M; ++i) {
    z += std::ldexp(1.0, -reg[i]);
    zeros += reg[i] == 0;
  }
  const double alpha = 0.7213 / (1.0 + 1.079 / m);
  const double e = alpha * m * m / z;
  if (e <= 2.5 * m && zeros) return m * std::log(m / zeros);
  return e;
}

// the column's items, '\n'-joined, into out (cap bytes); returns the bytes written or -1
SHIFU_RT_API long shifu_at_items(void* h, int col, char* out, long cap) {
  State& S = *(State*)h;
  merge_parts(S);
  if (col < 0 || col >= S.ncols) return -1;
  long n = 0;
  for (size_t i = 0; i < S.cols[col].items.size(); ++i) {
    const std::string& s = S.cols[col].items[i];
    if (n + (long)s.size() + 1 > cap) return -1;
    memcpy(out + n, s.data(), s.size());
    n += (long)s.size();
    out[n++] = '\n';
  }
  return n;
}

SHIFU_RT_API long shifu_at_skipped(void* h) { return (long)((State*)h)->skipped_tag; }

SHIFU_RT_API void shifu_at_free(void* h) { delete (State*)h; }
