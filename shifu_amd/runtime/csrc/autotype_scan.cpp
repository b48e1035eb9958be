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

struct Col {
  int64_t count = 0, invalid = 0, validnum = 0;
  std::vector<uint64_t> table;                // open addressing, 0 = empty (hash 0 stored as 1)
  int used = 0;
  bool overflow = false;
  std::vector<uint8_t> hll;                   // AT_HLL_M registers (allocated on first value)
  std::vector<std::string> items;
  std::unordered_set<std::string> item_set;

  void add_hash(uint64_t h) {
    if (hll.empty()) hll.assign(AT_HLL_M, 0);
    const uint32_t idx = (uint32_t)(h >> (64 - AT_HLL_P));
    const uint64_t rest = (h << AT_HLL_P) | (1ull << (AT_HLL_P - 1));
    const uint8_t rank = (uint8_t)(__builtin_clzll(rest) + 1);
    if (rank > hll[idx]) hll[idx] = rank;
    if (overflow) return;
    if (h == 0) h = 1;
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
  void add_item(const char* p, size_t n, int cap) {
    if ((int)items.size() >= cap) return;
    std::string s(p, n);
    if (item_set.insert(s).second) items.push_back(std::move(s));
  }
  void merge(Col& o, int item_cap) {
    count += o.count; invalid += o.invalid; validnum += o.validnum;
    if (!o.hll.empty()) {
      if (hll.empty()) hll.assign(AT_HLL_M, 0);
      for (int i = 0; i < AT_HLL_M; ++i) hll[i] = std::max(hll[i], o.hll[i]);
    }
    if (o.overflow) {
      overflow = true;
      std::vector<uint64_t>().swap(table);
    } else if (!overflow) {
      for (uint64_t v : o.table)
        if (v) {
          if (overflow) break;
          // re-insert without touching the HLL (already merged)
          if (table.empty()) table.assign(64, 0);
          if ((used + 1) * 2 > (int)table.size()) {
            if (used + 1 > AT_EXACT_CAP) { overflow = true; std::vector<uint64_t>().swap(table); break; }
            std::vector<uint64_t> t2(table.size() * 2, 0);
            for (uint64_t w : table)
              if (w) {
                size_t k = w & (t2.size() - 1);
                while (t2[k]) k = (k + 1) & (t2.size() - 1);
                t2[k] = w;
              }
            table.swap(t2);
          }
          size_t k = v & (table.size() - 1);
          bool dup = false;
          while (table[k]) {
            if (table[k] == v) { dup = true; break; }
            k = (k + 1) & (table.size() - 1);
          }
          if (!dup) { table[k] = v; ++used; }
        }
    }
    for (auto& s : o.items) {
      if ((int)items.size() >= item_cap) break;
      if (item_set.insert(s).second) items.push_back(s);
    }
    o = Col();
  }
};

struct State {
  int ncols = 0, tag_col = -1;
  std::string delim;
  std::vector<std::string> tags;              // trimmed
  std::unordered_set<std::string> missing;    // compared with the lower-cased raw field
  std::vector<Col> cols;                      // merged (rank) state
  std::vector<std::vector<Col>> part;         // per thread, merged on query
  int64_t rows = 0, skipped_tag = 0;
};

inline bool is_blank_line(const char* s, const char* e) {
  for (const char* q = s; q < e; ++q)
    if (*q != ' ' && *q != '\r' && *q != '\t') return false;
  return true;
}

// one thread: lines in [s, e) (line-aligned), rows numbered from row0 for the mask
void scan_range(State& S, std::vector<Col>& cols, const char* s, const char* e, const uint8_t* mask, int64_t row0,
                int64_t* rows_out, int64_t* skipped_out) {
  const char* d = S.delim.data();
  const size_t dl = S.delim.size();
  int64_t r = row0, skipped = 0, rows = 0;
  std::string low;
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
    ++rows;
    const int nf = std::min((int)f.size(), S.ncols);
    for (int c = 0; c < nf; ++c) {
      Col& C = cols[c];
      const char* v = f[c].first;
      const size_t n = f[c].second;
      C.count += 1;
      low.assign(v, n);
      for (auto& ch : low) ch = (char)tolower((unsigned char)ch);
      if (S.missing.count(low)) { C.invalid += 1; continue; }
      C.add_hash(hash_bytes(v, n));
      if (java_double(v, n)) C.validnum += 1;
      C.add_item(v, n, AT_ITEMS_THREAD);
    }
    p = next;
  }
  *rows_out = rows;
  *skipped_out = skipped;
}

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

void merge_parts(State& S) {
  for (auto& pc : S.part)
    for (int c = 0; c < S.ncols; ++c) S.cols[c].merge(pc[c], AT_ITEMS_RANK);
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
  for (auto& m : split_blob(missing, false)) S->missing.insert(m);
  S->cols.resize(ncols);
  return S;
}

// Scan a block of complete lines; mask (nullable): keep flag per non-blank line of the block (the
// purifier's filter expression).  Returns the rows counted (tag filter passed) or -1.
SHIFU_RT_API long shifu_at_feed(void* h, const char* buf, long len, const uint8_t* mask, int nthreads) {
  if (!h || len < 0) return -1;
  State& S = *(State*)h;
  const int T = std::max(1, std::min(nthreads, (int)(len >> 20) + 1));
  if ((int)S.part.size() < T) {
    S.part.resize(T);
    for (auto& pc : S.part)
      if ((int)pc.size() != S.ncols) pc.resize(S.ncols);
  }
  std::vector<const char*> cut(T + 1);
  cut[0] = buf;
  cut[T] = buf + len;
  for (int t = 1; t < T; ++t) {
    const char* c = buf + (len * t) / T;
    if (c < cut[t - 1]) c = cut[t - 1];
    const char* nl = (const char*)memchr(c, '\n', buf + len - c);
    cut[t] = nl ? nl + 1 : buf + len;
  }
  std::vector<int64_t> row0(T, 0);
  if (mask) {                                   // rows before each chunk (non-blank lines)
    int64_t r = 0;
    for (int t = 0; t < T; ++t) {
      row0[t] = r;
      for (const char* p = cut[t]; p < cut[t + 1];) {
        const char* nl = (const char*)memchr(p, '\n', cut[t + 1] - p);
        const char* le = nl ? nl : cut[t + 1];
        if (!is_blank_line(p, le)) ++r;
        p = nl ? nl + 1 : cut[t + 1];
      }
    }
  }
  std::vector<int64_t> rows(T, 0), skipped(T, 0);
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t)
    th.emplace_back([&, t] { scan_range(S, S.part[t], cut[t], cut[t + 1], mask, row0[t], &rows[t], &skipped[t]); });
  scan_range(S, S.part[0], cut[0], cut[1], mask, row0[0], &rows[0], &skipped[0]);
  for (auto& x : th) x.join();
  long tot = 0;
  for (int t = 0; t < T; ++t) { tot += rows[t]; S.skipped_tag += skipped[t]; }
  S.rows += tot;
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
