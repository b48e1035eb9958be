// Synthetic tabular CSV generator for the pipeline benchmark (bench.py --model pipeline): the
// shape of the reference's published runs (CHANGES.txt:233-237, 264-268: 20M rows x 1600
// variables, '|'-delimited Pig text), written by T threads into T part files at disk speed.
//
// Row i (deterministic in (seed, i), independent of the thread count):
//   id<i> | tag (M/B) | weight U(0.5, 2) | num_0..num_{F-1} ('%.5f', ~missing_rate empty) | cat_0..cat_{C-1} (k0..k4)
// The tag is a planted SPARSE rule: z = sum over the k_strong "strong" numeric columns (every
// (F / k_strong)-th column, alternating sign, decaying weight) + 0.5 * noise > 0, so a
// sensitivity varsel can be checked for recovering exactly those columns.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define SHIFU_RT_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline double uni(uint64_t& s) { return (double)(splitmix(s) >> 11) * (1.0 / 9007199254740992.0); }
// N(0,1) by inverse-CDF table lookup (4096 quantiles, linear between them): generation runs at
// formatting speed instead of a log + cos per value
struct NormTable {
  double q[4097];
  NormTable() {
    for (int i = 0; i <= 4096; ++i) {          // Acklam-style rational approximation of the probit
      double p = (i + 0.5) / 4097.0;
      const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                          1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00};
      const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                          6.680131188771972e+01, -1.328068155288572e+01};
      const double c[] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                          -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00};
      const double d[] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                          3.754408661907416e+00};
      double x;
      if (p < 0.02425) {
        const double t = std::sqrt(-2 * std::log(p));
        x = (((((c[0] * t + c[1]) * t + c[2]) * t + c[3]) * t + c[4]) * t + c[5]) /
            ((((d[0] * t + d[1]) * t + d[2]) * t + d[3]) * t + 1);
      } else if (p > 1 - 0.02425) {
        const double t = std::sqrt(-2 * std::log(1 - p));
        x = -(((((c[0] * t + c[1]) * t + c[2]) * t + c[3]) * t + c[4]) * t + c[5]) /
            ((((d[0] * t + d[1]) * t + d[2]) * t + d[3]) * t + 1);
      } else {
        const double t = p - 0.5, r = t * t;
        x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * t /
            (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
      }
      q[i] = x;
    }
  }
};
const NormTable kNorm;
inline double gauss(uint64_t& s) {
  const uint64_t r = splitmix(s);
  const int i = (int)(r >> 52);
  const double f = (double)((r >> 20) & 0xFFFFFFFFull) * (1.0 / 4294967296.0);
  return kNorm.q[i] + f * (kNorm.q[i + 1] - kNorm.q[i]);
}

bool is_strong(int j, int F, int k) { return k > 0 && (j % (F / k > 0 ? F / k : 1)) == 0 && j / (F / k > 0 ? F / k : 1) < k; }

void gen_rows(const std::string& path, long r0, long r1, int F, int C, uint64_t seed, double miss, int k,
              int* status) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) { *status = -1; return; }
  std::vector<char> buf(1 << 24);
  std::vector<double> x(F);
  long pos = 0;
  const int step = (k > 0 && F / k > 0) ? F / k : 1;
  for (long i = r0; i < r1; ++i) {
    uint64_t s = seed * 0x100000001B3ull + (uint64_t)i * 0x9E3779B97F4A7C15ull;
    double z = 0.0;
    for (int j = 0; j < F; ++j) {
      x[j] = gauss(s);
      if (is_strong(j, F, k)) {
        const int q = j / step;
        z += ((q & 1) ? -1.0 : 1.0) * (1.0 / (1.0 + 0.15 * q)) * x[j];
      }
    }
    z += 0.5 * gauss(s);
    const double w = 0.5 + 1.5 * uni(s);
    if ((long)buf.size() - pos < (long)F * 24 + C * 8 + 128) {
      std::fwrite(buf.data(), 1, (size_t)pos, f);
      pos = 0;
    }
    char* p = buf.data() + pos;
    char* p0 = p;
    *p++ = 'i'; *p++ = 'd';
    p = std::to_chars(p, p + 24, i).ptr;
    *p++ = '|'; *p++ = z > 0 ? 'M' : 'B'; *p++ = '|';
    p = std::to_chars(p, p + 32, w, std::chars_format::fixed, 4).ptr;
    for (int j = 0; j < F; ++j) {
      *p++ = '|';
      if (uni(s) >= miss) p = std::to_chars(p, p + 32, x[j], std::chars_format::fixed, 5).ptr;
    }
    for (int j = 0; j < C; ++j) {
      *p++ = '|';
      if (uni(s) >= miss) { *p++ = 'k'; *p++ = (char)('0' + (int)(uni(s) * 5.0)); }
    }
    *p++ = '\n';
    pos += p - p0;
  }
  std::fwrite(buf.data(), 1, (size_t)pos, f);
  *status = std::fclose(f) == 0 ? 0 : -1;
}

}  // namespace

// Writes `nparts` files dir/part-00000.. holding rows [0, n) split evenly; returns 0 on success.
SHIFU_RT_API int shifu_gen_csv(const char* dir, long n, int n_num, int n_cat, long seed, double missing_rate,
                               int k_strong, int nparts) {
  if (n < 0 || n_num <= 0 || n_cat < 0 || nparts <= 0) return -1;
  std::vector<std::thread> th;
  std::vector<int> st(nparts, 0);
  for (int t = 0; t < nparts; ++t) {
    char name[64];
    std::snprintf(name, sizeof name, "/part-%05d", t);
    const long r0 = n * t / nparts, r1 = n * (t + 1) / nparts;
    th.emplace_back(gen_rows, std::string(dir) + name, r0, r1, n_num, n_cat, (uint64_t)seed, missing_rate, k_strong,
                    &st[t]);
  }
  for (auto& t : th) t.join();
  for (int s : st)
    if (s) return -1;
  return 0;
}

// The strong columns of the planted rule (out[0..k) = column indices), for recall checks.
SHIFU_RT_API int shifu_gen_strong_cols(int n_num, int k_strong, int* out) {
  int m = 0;
  for (int j = 0; j < n_num; ++j)
    if (is_strong(j, n_num, k_strong)) out[m++] = j;
  return m;
}
