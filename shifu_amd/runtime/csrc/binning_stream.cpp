// Reference-parity streaming quantile sketches for numeric binning (host runtime, C++17).
//
// ``stats.binningAlgorithm`` SPDT/SPDTI and MunroPat/MunroPatI of the reference compute a
// column's cut points from a streaming sketch fed with the column's values in row order
// (udf/BinningDataUDF.java:72-97):
//   * SPDT -- Ben-Haim & Tom-Tov streaming histogram of at most min(100 * bins, 10000) centroids,
//     closest-pair merging, trapezoid "uniform" procedure for the cuts
//     (core/binning/EqualPopulationBinning.java:185-600);
//   * MunroPat -- Munro-Paterson multi-level buffers with alternate-element collapse
//     (core/MunroPatEstimator.java), cuts = every (1/(bins-1)) quantile, deduplicated
//     (core/binning/MunroPatBinning.java:53-96).
// The default path of this framework computes EXACT equal-population cuts on the GPU
// (algos/quantile.py); these sketches exist so a model set can reproduce the reference's
// approximate cuts bit for bit when ``shifu.stats.binning.parity=true``.  Tie rules, merge
// arithmetic order and the reference's quirks (a small-bin merge that reuses the updated
// count, the stale unit count after small-bin merging) are kept on purpose.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

namespace {

struct Unit {
  double v, c;
};

// java.lang.Double.compare for non-NaN values: -0.0 orders before +0.0
inline int jcmp(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  const bool na = std::signbit(a), nb = std::signbit(b);
  return na == nb ? 0 : (na ? -1 : 1);
}

class Spdt {
 public:
  explicit Spdt(int bins) : bins_(bins) {
    long m = (long)bins * 100;
    max_units_ = (int)(m > 10000 ? 10000 : m);
  }

  void add(double v, double f) {
    if (u_.empty() && max_units_ > 1) {
      u_.push_back({v, f});
      count_ = 1;
      return;
    }
    insert_with_trim({v, f});
  }

  std::vector<double> cuts(int to_bins) {
    std::vector<double> out{-std::numeric_limits<double>::infinity()};
    double total = 0;
    for (const Unit& x : u_) total += x.c;
    merge_small(total, to_bins);
    if (count_ <= to_bins) {
      for (size_t i = 0; i + 1 < u_.size(); ++i) out.push_back((u_[i].v + u_[i + 1].v) / 2);
      return out;
    }
    // sum at each centroid: everything before it + half of its own count
    std::vector<double> sc(u_.size());
    double run = 0;
    for (size_t i = 0; i < u_.size(); ++i) {
      sc[i] = run + u_[i].c / 2.0;
      run += u_[i].c;
    }
    long cur = -1;  // -1 = not started (the reference's null start position)
    const long last = (long)u_.size() - 1;
    for (int j = 1; j < to_bins; ++j) {
      const double s = (j * total) / to_bins;
      long pos = locate(s, cur, sc, last);
      if (pos < 0 || pos == cur || pos == last) continue;
      const Unit& ch = u_[pos];
      const Unit& nh = u_[pos + 1];
      const double d = s - sc[pos];
      if (d < 0) {
        out.push_back((ch.v + nh.v) / 2);
        cur = pos;
        continue;
      }
      const double a = nh.c - ch.c, b = 2 * ch.c, c = -2 * d;
      const double z = a == 0.0 ? -1 * c / b : (-1 * b + std::sqrt(b * b - 4 * a * c)) / (2 * a);
      out.push_back(ch.v + (nh.v - ch.v) * z);
      cur = pos;
    }
    return out;
  }

 private:
  // the reference's linked list as a sorted vector; the scan runs tail -> head with strict '<'
  // on the intervals, so among equal minimum intervals the right-most pair is merged
  void insert_with_trim(Unit node) {
    const long n = (long)u_.size();
    long ins = -2;                      // index the node goes after (-1 = head), -2 = not found
    double min_iv = std::numeric_limits<double>::max();
    long min_at = -3;                   // merge target: index into the post-insert list
    bool min_is_node = false;
    for (long i = n - 1; i >= 0; --i) {
      if (ins == -2) {
        const int r = jcmp(u_[i].v, node.v);
        if (r == 0) {
          u_[i].c += node.c;
          return;
        }
        if (r < 0) {
          ins = i;
          double iv = node.v - u_[i].v;
          if (iv < min_iv) { min_iv = iv; min_at = i; min_is_node = false; }
          if (i + 1 < n) {
            iv = u_[i + 1].v - node.v;
            if (iv < min_iv) { min_iv = iv; min_is_node = true; }
          }
        }
      }
      if (i + 1 < n) {
        const double iv = u_[i + 1].v - u_[i].v;
        if (iv < min_iv) { min_iv = iv; min_at = i; min_is_node = false; }
      }
    }
    const long at = ins == -2 ? 0 : ins + 1;           // insert position in the vector
    u_.insert(u_.begin() + at, node);
    const long m = min_is_node ? at : (min_at < 0 ? -1 : (min_at >= at ? min_at + 1 : min_at));
    if (count_ == max_units_ && m >= 0 && m + 1 < (long)u_.size()) {
      Unit& ch = u_[m];
      Unit& nh = u_[m + 1];
      nh.v = (ch.v * ch.c + nh.v * nh.c) / (ch.c + nh.c);
      nh.c = ch.c + nh.c;
      u_.erase(u_.begin() + m);
    } else {
      ++count_;
    }
  }

  void merge_small(double total, int to_bins) {
    if (u_.size() <= 1) return;
    const double min_cnt = (total / to_bins) * 0.003;
    size_t i = 0;
    while (i < u_.size()) {
      if (u_[i].c < min_cnt) {
        const Unit ch = u_[i];
        if (i == 0) {
          if (u_.size() == 1) break;
          Unit& nh = u_[1];
          nh.c = ch.c + nh.c;                     // reference order: count first, then value
          nh.v = (ch.v * ch.c + nh.v * nh.c) / (ch.c + nh.c);
          u_.erase(u_.begin());
          continue;                               // the new head is examined next
        } else if (i + 1 == u_.size()) {
          Unit& ph = u_[i - 1];
          ph.c = ch.c + ph.c;
          ph.v = (ch.v * ch.c + ph.v * ph.c) / (ch.c + ph.c);
          u_.pop_back();
          break;
        } else {
          Unit& ph = u_[i - 1];
          Unit& nh = u_[i + 1];
          if (ch.v - ph.v < nh.v - ch.v) {
            ph.c = ch.c + ph.c;
            ph.v = (ch.v * ch.c + ph.v * ph.c) / (ch.c + ph.c);
          } else {
            nh.c = ch.c + nh.c;
            nh.v = (ch.v * ch.c + nh.v * nh.c) / (ch.c + nh.c);
          }
          u_.erase(u_.begin() + i);
          continue;                               // u_[i] is now the old next
        }
      }
      ++i;
    }
    // the reference does not update its unit count here (its later check uses the stale count)
  }

  long locate(double s, long start, const std::vector<double>& sc, long last) const {
    while (start != last) {
      if (start < 0) start = 0;
      if (start == last) return start;
      const double a = sc[start], b = sc[start + 1];
      if (a >= s || (a < s && s <= b)) return start;
      ++start;
    }
    return -1;
  }

  int bins_;
  int max_units_ = 0;
  int count_ = 0;
  std::vector<Unit> u_;
};

class MunroPat {
 public:
  explicit MunroPat(int nq) : nq_(nq) {
    const double eps = 1.0 / (nq - 1.0);
    const double max_tot = 1024.0 * 1024.0 * 1024.0 * 1024.0;
    int b = 2;
    while ((double)((long long)(b - 2) * (1LL << (b - 2))) + 0.5 <= eps * max_tot) ++b;
    m_ = (long)(max_tot / (double)(1LL << (b - 1)));
  }

  void add(double e) {
    if (total_ == 0 || e < min_) min_ = e;
    if (total_ == 0 || max_ < e) max_ = e;
    if (total_ > 0 && total_ % (2 * m_) == 0) {
      std::sort(buf_[0].begin(), buf_[0].end());
      std::sort(buf_[1].begin(), buf_[1].end());
      std::vector<double> b0 = std::move(buf_[0]);
      buf_[0].clear();
      collapse_up(b0, 1);
    }
    ensure(1);
    (buf_[0].size() < (size_t)m_ ? buf_[0] : buf_[1]).push_back(e);
    ++total_;
  }

  std::vector<double> cuts() {
    std::vector<double> q;
    if (total_ == 0) return merge_bins(q);
    q.push_back(min_);
    std::sort(buf_[0].begin(), buf_[0].end());
    std::sort(buf_[1].begin(), buf_[1].end());
    std::vector<size_t> idx(buf_.size(), 0);
    long long S = 0;
    for (int i = 1; i <= nq_ - 2; ++i) {
      const long long target = (long long)std::ceil(i * (total_ / (nq_ - 1.0)));
      for (;;) {
        double smallest = max_;
        int id = -1;
        for (size_t j = 0; j < buf_.size(); ++j)
          if (idx[j] < buf_[j].size() && smallest >= buf_[j][idx[j]]) { smallest = buf_[j][idx[j]]; id = (int)j; }
        const long long inc = id <= 1 ? 1LL : (1LL << (id - 1));
        if (S + inc >= target || id < 0) {
          q.push_back(smallest);
          break;
        }
        ++idx[id];
        S += inc;
      }
    }
    q.push_back(max_);
    return merge_bins(q);
  }

 private:
  void ensure(size_t level) {
    while (buf_.size() < level + 1) buf_.emplace_back();
  }

  // buffers a (level) and b (the incoming sorted run) -> every other element of their merge;
  // ties take from b first (the reference's compareTo >= 0)
  std::vector<double> collapse(std::vector<double>& a, std::vector<double>& b) {
    std::vector<double> out;
    out.reserve(m_);
    long ia = 0, ib = 0, cnt = 0;
    while (ia < m_ || ib < m_) {
      double s;
      if (ia >= m_ || (ib < m_ && a[ia] >= b[ib])) s = b[ib++];
      else s = a[ia++];
      if (cnt++ % 2 == 0) out.push_back(s);
    }
    a.clear();
    b.clear();
    return out;
  }

  void collapse_up(std::vector<double>& run, size_t level) {
    ensure(level + 1);
    const bool empty_above = buf_[level + 1].empty();
    std::vector<double> merged = collapse(buf_[level], run);
    if (empty_above) {
      buf_[level + 1] = std::move(merged);
    } else {
      collapse_up(merged, level + 1);
    }
  }

  std::vector<double> merge_bins(std::vector<double> bins) const {
    if (bins.empty()) return {std::numeric_limits<double>::quiet_NaN()};
    std::vector<double> nb{bins[0]};
    double cur = bins[0];
    for (size_t i = 1; i < bins.size(); ++i) {
      if (std::fabs(cur - bins[i]) > 1e-10) nb.push_back(bins[i]);
      cur = bins[i];
    }
    const double ninf = -std::numeric_limits<double>::infinity();
    if (nb.size() == 1) return {ninf, nb[0]};
    nb[0] = ninf;
    if (nb.size() > 2) nb.pop_back();
    return nb;
  }

  int nq_;
  long m_ = 0;
  long long total_ = 0;
  double min_ = 0, max_ = 0;
  std::vector<std::vector<double>> buf_{std::vector<double>(), std::vector<double>()};
};

long emit(const std::vector<double>& c, double* out, long cap) {
  const long n = (long)c.size();
  for (long i = 0; i < n && i < cap; ++i) out[i] = c[i];
  return n;
}

}  // namespace

extern "C" {

// values in row order (NaN = missing, skipped); optional weights (null = 1); returns the number
// of cut points (first = -inf); writes min(n, cap) of them
long shifu_spdt_bins(const double* vals, const double* w, long n, int bins, double* out, long cap) {
  if (bins < 1 || n < 0) return -1;
  Spdt s(bins);
  for (long i = 0; i < n; ++i)
    if (!std::isnan(vals[i])) s.add(vals[i], w ? w[i] : 1.0);
  return emit(s.cuts(bins), out, cap);
}

long shifu_munropat_bins(const double* vals, long n, int bins, double* out, long cap) {
  if (bins < 2 || n < 0) return -1;
  MunroPat m(bins);
  for (long i = 0; i < n; ++i)
    if (!std::isnan(vals[i])) m.add(vals[i]);
  return emit(m.cuts(), out, cap);
}

}  // extern "C"
