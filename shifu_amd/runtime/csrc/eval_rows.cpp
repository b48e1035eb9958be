// EvalScore text rows for the streamed `eval` (B9): the reference writes EvalScore through Pig
// (P/Eval.pig:29-41: EvalScoreUDF.exec J/udf/EvalScoreUDF.java:226, then ORDER BY score DESC).
// Here every rank scores its byte range chunk by chunk; this file formats a chunk's columns into
// '|'-joined lines in one native pass (no per-row Python), and k-way merges the ranks' sorted
// line runs into one EvalScore (stable: ties keep rank order = the single-process row order).
//
// Number formats match the Python writer they replace byte for byte:
//   FIXED6  f"{x:.6f}"   (std::to_chars fixed, precision 6: correctly rounded, like CPython)
//   REPR    repr(float)  (shortest round-trip digits, CPython's fixed/scientific switch)
//   REPR_OR_EMPTY  the same, '' for NaN (a numeric tag / meta column's missing value)
//   DICT    dictionary string of an int32 code ('' for a missing code < 0)
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <queue>
#include <thread>
#include <vector>

#define SHIFU_RT_API extern "C" __attribute__((visibility("default")))

namespace {

enum Kind : int { FIXED6 = 0, REPR = 1, DICT = 2, REPR_OR_EMPTY = 3 };

int put_fixed6(char* p, double x) {
  if (std::isnan(x)) { std::memcpy(p, "nan", 3); return 3; }
  if (std::isinf(x)) { if (x < 0) { std::memcpy(p, "-inf", 4); return 4; } std::memcpy(p, "inf", 3); return 3; }
  auto r = std::to_chars(p, p + 400, x, std::chars_format::fixed, 6);
  return (int)(r.ptr - p);
}

// CPython float_repr_style 'short': repr(x) = shortest digits; fixed when -4 <= exp10 < 16
int put_repr(char* p, double x) {
  if (std::isnan(x)) { std::memcpy(p, "nan", 3); return 3; }
  if (std::isinf(x)) { if (x < 0) { std::memcpy(p, "-inf", 4); return 4; } std::memcpy(p, "inf", 3); return 3; }
  char* q = p;
  if (std::signbit(x)) { *q++ = '-'; x = -x; }
  if (x == 0.0) { std::memcpy(q, "0.0", 3); return (int)(q - p) + 3; }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  *r.ptr = 0;
  // buf = d[.ddd]e[+-]XX
  char digits[32];
  int nd = 0;
  const char* s = buf;
  for (; *s && *s != 'e'; ++s)
    if (*s != '.') digits[nd++] = *s;
  const int e = std::atoi(s + 1);
  if (e >= -4 && e < 16) {
    if (e >= 0) {
      for (int i = 0; i <= e; ++i) *q++ = i < nd ? digits[i] : '0';
      *q++ = '.';
      if (nd > e + 1) for (int i = e + 1; i < nd; ++i) *q++ = digits[i];
      else *q++ = '0';
    } else {
      *q++ = '0'; *q++ = '.';
      for (int i = 0; i < -e - 1; ++i) *q++ = '0';
      for (int i = 0; i < nd; ++i) *q++ = digits[i];
    }
  } else {
    *q++ = digits[0];
    if (nd > 1) { *q++ = '.'; for (int i = 1; i < nd; ++i) *q++ = digits[i]; }
    *q++ = 'e';
    *q++ = e < 0 ? '-' : '+';
    const int ae = e < 0 ? -e : e;
    if (ae < 10) *q++ = '0';
    q += std::snprintf(q, 8, "%d", ae);
  }
  return (int)(q - p);
}

}  // namespace

// Format n rows of ncols columns into '|'-joined, '\n'-terminated lines.
//   kinds[c]: FIXED6 / REPR / REPR_OR_EMPTY (cols[c] -> double[n]) or DICT (cols[c] -> int32[n],
//   dict_blob[c] + dict_off[c][k..k+1] = string k, dict_n[c] strings).
//   line_end[i] = byte offset just past row i's '\n'.  Returns bytes written, or -1 if cap is short.
//   sep / slen: the field separator (shifu_format_rows: '|').
SHIFU_RT_API long shifu_format_rows_sep(long n, int ncols, const int* kinds, const void* const* cols,
                                        const char* const* dict_blob, const long* const* dict_off,
                                        const long* dict_n, char* out, long cap, long* line_end,
                                        const char* sep, int slen) {
  if (slen < 1 || slen > 64) return -1;
  long pos = 0;
  for (long i = 0; i < n; ++i) {
    for (int c = 0; c < ncols; ++c) {
      if (cap - pos < 512) return -1;
      if (c) { std::memcpy(out + pos, sep, (size_t)slen); pos += slen; }
      const int k = kinds[c];
      if (k == DICT) {
        const int code = ((const int32_t*)cols[c])[i];
        if (code >= 0 && code < dict_n[c]) {
          const long a = dict_off[c][code], b = dict_off[c][code + 1];
          if (cap - pos < (b - a) + 512) return -1;
          std::memcpy(out + pos, dict_blob[c] + a, (size_t)(b - a));
          pos += b - a;
        }
      } else {
        const double v = ((const double*)cols[c])[i];
        if (k == FIXED6) pos += put_fixed6(out + pos, v);
        else if (k == REPR || !std::isnan(v)) pos += put_repr(out + pos, v);
      }
    }
    out[pos++] = '\n';
    line_end[i] = pos;
  }
  return pos;
}

SHIFU_RT_API long shifu_format_rows(long n, int ncols, const int* kinds, const void* const* cols,
                                    const char* const* dict_blob, const long* const* dict_off,
                                    const long* dict_n, char* out, long cap, long* line_end) {
  return shifu_format_rows_sep(n, ncols, kinds, cols, dict_blob, dict_off, dict_n, out, cap, line_end, "|", 1);
}

// Joined rows for `combo` (DataJoin of the sub-model scores, ComboModelProcessor.java:278-356) and
// `encode` (tree leaf-path columns): every non-blank line of a block of complete lines (blank =
// only ' ', '\t', '\r'; the parser's row framing) is written as its first `nf` fields (a short
// row padded with empty fields, fields past the header dropped, a trailing '\r' removed), then
// the separator and suffix line i (from shifu_format_rows_sep, '\n'-terminated).  The raw field
// bytes pass through untouched.  Two passes over `nthreads` line-aligned chunks: (1) per line the
// kept length and the number of padding separators (memchr over the separator's first byte),
// per chunk the row count and output bytes; (2) every chunk copies to its prefix-summed offset.
// Returns bytes written, -1 if cap is short, -2 if the block does not hold exactly n non-blank
// lines.
namespace {

struct JoinLine { const char* p; int64_t keep; int32_t pad; };

inline bool blank_line(const char* p, const char* le) {
  for (const char* q = p; q < le; ++q)
    if (*q != ' ' && *q != '\r' && *q != '\t') return false;
  return true;
}

void join_scan(const char* s, const char* e, const char* sep, int slen, int nf, std::vector<JoinLine>& out,
               int64_t* bytes) {
  int64_t tot = 0;
  for (const char* p = s; p < e;) {
    const char* nl = (const char*)std::memchr(p, '\n', (size_t)(e - p));
    const char* le = nl ? nl : e;
    const char* next = nl ? nl + 1 : e;
    if (blank_line(p, le)) { p = next; continue; }
    if (le > p && le[-1] == '\r') --le;
    const char* cut = le;
    int seen = 1;
    for (const char* q = p; q + slen <= le;) {
      const char* h = (const char*)std::memchr(q, sep[0], (size_t)(le - q));
      if (!h || h + slen > le) break;
      if (slen == 1 || std::memcmp(h, sep, (size_t)slen) == 0) {
        if (seen == nf) { cut = h; break; }
        ++seen;
        q = h + slen;
      } else {
        q = h + 1;
      }
    }
    const int pad = nf - seen + 1;            // separators after the kept bytes (incl. the suffix's)
    out.push_back({p, (int64_t)(cut - p), pad});
    tot += (cut - p) + (int64_t)pad * slen;
    p = next;
  }
  *bytes = tot;
}

}  // namespace

SHIFU_RT_API long shifu_join_lines(const char* buf, long len, const char* sep, int slen, int nf,
                                   const char* suffix, const long* suffix_end, long n, char* out, long cap,
                                   int nthreads) {
  if (slen < 1 || nf < 1) return -2;
  const int T = std::max(1, std::min(nthreads, (int)(len >> 20) + 1));
  std::vector<const char*> cut(T + 1);
  cut[0] = buf;
  cut[T] = buf + len;
  for (int t = 1; t < T; ++t) {
    const char* c = std::max(buf + (len * t) / T, cut[t - 1]);
    const char* nl = (const char*)std::memchr(c, '\n', (size_t)(buf + len - c));
    cut[t] = nl ? nl + 1 : buf + len;
  }
  std::vector<std::vector<JoinLine>> lines(T);
  std::vector<int64_t> raw(T, 0);
  {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t)
      th.emplace_back([&, t] { join_scan(cut[t], cut[t + 1], sep, slen, nf, lines[t], &raw[t]); });
    join_scan(cut[0], cut[1], sep, slen, nf, lines[0], &raw[0]);
    for (auto& x : th) x.join();
  }
  std::vector<int64_t> row0(T + 1, 0), off0(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    row0[t + 1] = row0[t] + (int64_t)lines[t].size();
    if (row0[t + 1] > n) return -2;
    const int64_t sa = row0[t] ? suffix_end[row0[t] - 1] : 0;
    const int64_t sb = row0[t + 1] ? suffix_end[row0[t + 1] - 1] : 0;
    off0[t + 1] = off0[t] + raw[t] + (sb - sa);
  }
  if (row0[T] != n) return -2;
  if (off0[T] > cap) return -1;
  auto write = [&](int t) {
    char* o = out + off0[t];
    int64_t r = row0[t];
    for (const JoinLine& L : lines[t]) {
      std::memcpy(o, L.p, (size_t)L.keep);
      o += L.keep;
      for (int k = 0; k < L.pad; ++k) { std::memcpy(o, sep, (size_t)slen); o += slen; }
      const int64_t a = r ? suffix_end[r - 1] : 0, b = suffix_end[r];
      std::memcpy(o, suffix + a, (size_t)(b - a));
      o += b - a;
      ++r;
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(write, t);
    write(0);
    for (auto& x : th) x.join();
  }
  return (long)off0[T];
}

// k-way merge of R sorted runs of lines into `out_path` (appending).  Run r: lines blob + line_end
// offsets (ascending) + keys (the run's order: descending key); ties go to the lower run index,
// so runs = ranks in order reproduces a stable single-process sort.  Returns lines written or -1.
// Output staging of the merge / gather below: lines are copied into a fixed-size buffer that is
// written out whenever it fills (the merging rank's memory stays bounded whatever the score file's
// size; one fwrite per line was ~1-2 s at 20M rows).
static size_t kFlushBytes = (size_t)256 << 20;
SHIFU_RT_API long shifu_eval_set_flush_bytes(long b) {      // tests: a small buffer (flush paths)
  const long old = (long)kFlushBytes;
  if (b > 0) kFlushBytes = (size_t)b;
  return old;
}

SHIFU_RT_API long shifu_merge_runs(int R, const char* const* blobs, const long* const* ends, const double* const* keys,
                                   const long* counts, const char* out_path) {
  FILE* f = std::fopen(out_path, "ab");
  if (!f) return -1;
  long total = 0;
  int live = 0, only = -1;
  for (int r = 0; r < R; ++r)
    if (counts[r] > 0) { total += counts[r]; ++live; only = r; }
  if (live == 1) {                                  // one run: it is the merge, written from the blob
    const size_t bytes = (size_t)ends[only][counts[only] - 1];
    if (bytes && std::fwrite(blobs[only], 1, bytes, f) != bytes) { std::fclose(f); return -1; }
    return std::fclose(f) == 0 ? total : -1;
  }
  std::vector<char> out(kFlushBytes);
  size_t o = 0;
  bool ok = true;
  auto put = [&](const char* p, size_t len) {
    if (o + len > out.size()) {
      if (o && std::fwrite(out.data(), 1, o, f) != o) ok = false;
      o = 0;
      if (len > out.size()) {                       // a line longer than the buffer: straight out
        if (std::fwrite(p, 1, len, f) != len) ok = false;
        return;
      }
    }
    std::memcpy(out.data() + o, p, len);
    o += len;
  };
  struct Head { double key; int run; };
  auto worse = [](const Head& a, const Head& b) {        // priority: larger key, then lower run
    return a.key < b.key || (a.key == b.key && a.run > b.run);
  };
  std::priority_queue<Head, std::vector<Head>, decltype(worse)> pq(worse);
  std::vector<long> at(R, 0);
  for (int r = 0; r < R; ++r)
    if (counts[r] > 0) pq.push({keys[r][0], r});
  while (!pq.empty() && ok) {
    const Head h = pq.top();
    pq.pop();
    const int r = h.run;
    const long i = at[r]++;
    const long a = i ? ends[r][i - 1] : 0, b = ends[r][i];
    put(blobs[r] + a, (size_t)(b - a));
    if (at[r] < counts[r]) pq.push({keys[r][at[r]], r});
  }
  if (ok && o && std::fwrite(out.data(), 1, o, f) != o) ok = false;
  if (std::fclose(f) != 0 || !ok) return -1;
  return total;
}

// Reorder one run's lines: write lines order[0], order[1], ... of (blob, line_end) to out_path and
// their new end offsets to new_end (the rank-local ORDER BY before the k-way merge).
SHIFU_RT_API long shifu_gather_lines(const char* blob, const long* ends, const long* order, long n,
                                     const char* out_path, long* new_end) {
  // output offsets of the reordered lines (one O(n) pass), then the lines copied by several threads
  // into a fixed-size buffer, written whenever it fills (a window of lines per fill)
  long pos = 0;
  for (long i = 0; i < n; ++i) {
    const long j = order[i];
    pos += ends[j] - (j ? ends[j - 1] : 0);
    new_end[i] = pos;
  }
  FILE* f = std::fopen(out_path, "wb");
  if (!f) return -1;
  std::vector<char> out(std::min<size_t>(kFlushBytes, (size_t)std::max(pos, 1L)));
  long i0 = 0;
  while (i0 < n) {
    // the window [i0, i1): as many whole lines as fit (at least one)
    const long base = i0 ? new_end[i0 - 1] : 0;
    long i1 = i0 + 1;
    {
      long lo = i0 + 1, hi = n;                     // largest i1 with new_end[i1 - 1] - base <= size
      while (lo <= hi) {
        const long mid = lo + (hi - lo) / 2;
        if (new_end[mid - 1] - base <= (long)out.size()) { i1 = mid; lo = mid + 1; } else hi = mid - 1;
      }
    }
    const long wbytes = new_end[i1 - 1] - base;
    if (wbytes > (long)out.size()) {                 // one line longer than the buffer
      const long j = order[i0];
      const long a = j ? ends[j - 1] : 0;
      if (std::fwrite(blob + a, 1, (size_t)wbytes, f) != (size_t)wbytes) { std::fclose(f); return -1; }
      i0 = i1;
      continue;
    }
    const long cnt = i1 - i0;
    const long T = std::max(1L, std::min<long>(16, cnt >> 16));
    std::vector<std::thread> th;
    for (long t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        for (long i = i0 + cnt * t / T, e = i0 + cnt * (t + 1) / T; i < e; ++i) {
          const long j = order[i];
          const long a = j ? ends[j - 1] : 0, b = ends[j];
          std::memcpy(out.data() + ((i ? new_end[i - 1] : 0) - base), blob + a, (size_t)(b - a));
        }
      });
    for (auto& x : th) x.join();
    if (wbytes && std::fwrite(out.data(), 1, (size_t)wbytes, f) != (size_t)wbytes) { std::fclose(f); return -1; }
    i0 = i1;
  }
  if (std::fclose(f) != 0) return -1;
  return pos;
}
