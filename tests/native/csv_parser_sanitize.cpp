// Host-side sanitizer driver for the native CSV parser (race detection /
// sanitizers).  Built with -fsanitize=address,undefined (and separately -fsanitize=thread)
// by tests/test_native_sanitizers.py; exercises edge cases and the multi-threaded chunking.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
void* shifu_csv_parse(const char* buf, long len, const char* delim, int ncols, const int* kinds,
                      const char* missing, int nthreads);
long shifu_csv_nrows(void* h);
long shifu_csv_bad_rows(void* h);
int shifu_csv_numeric(void* h, int col, double* out);
int shifu_csv_codes(void* h, int col, int* out);
long shifu_csv_dict(void* h, int col, char* out, long cap);
long shifu_csv_dict_size(void* h, int col);
void shifu_csv_free(void* h);
}

static int check(const std::string& text, int ncols, long want_rows, int nthreads) {
  std::vector<int> kinds(ncols, 2);
  kinds[0] = 1;
  const char missing[] = "\n?";           // newline-joined list: "" and "?"
  void* h = shifu_csv_parse(text.data(), (long)text.size(), "|", ncols, kinds.data(), missing, nthreads);
  if (!h) { std::printf("parse returned null\n"); return 1; }
  const long n = shifu_csv_nrows(h);
  if (want_rows >= 0 && n != want_rows) { std::printf("rows %ld != %ld\n", n, want_rows); return 1; }
  std::vector<double> num(n > 0 ? n : 1);
  shifu_csv_numeric(h, 0, num.data());
  for (int c = 1; c < ncols; ++c) {
    std::vector<int> codes(n > 0 ? n : 1);
    shifu_csv_codes(h, c, codes.data());
    (void)shifu_csv_dict_size(h, c);
    const long need = shifu_csv_dict(h, c, nullptr, 0);
    std::vector<char> d(need + 1);
    shifu_csv_dict(h, c, d.data(), need);
  }
  shifu_csv_free(h);
  return 0;
}

int main() {
  int rc = 0;
  rc |= check("", 3, 0, 4);
  rc |= check("1|a|b\n", 3, 1, 4);
  rc |= check("1|a|b", 3, 1, 4);                         // no trailing newline
  rc |= check("1|a|b\r\n2|c|d\r\n", 3, 2, 2);            // CRLF
  rc |= check("1|a\n2|c|d|e\n|||\n?|x|y\n", 3, 4, 3);    // short / long / empty fields
  rc |= check("\n\n1|a|b\n\n", 3, -1, 8);                 // blank lines
  std::string big;
  for (int i = 0; i < 200000; ++i) {
    big += std::to_string(i * 0.5) + "|k" + std::to_string(i % 97) + "|" + std::string(i % 13, 'z') + "\n";
  }
  rc |= check(big, 3, 200000, 8);                         // multi-threaded chunk boundaries
  std::string longfield(1 << 20, 'q');
  rc |= check("1|" + longfield + "|x\n2|y|z\n", 3, 2, 4);
  std::printf(rc ? "FAIL\n" : "OK\n");
  return rc;
}
