// Host check of FastDiv (bolt_amd/csrc/bm_common.h): the mul-hi division the
// copy kernels use for every index decomposition must equal n / d exactly.
#include "../../bolt_amd/csrc/bm_common.h"
#include <cstdio>
#include <random>

void bm_set_error(const char *, ...) {}

int main() {
  std::mt19937_64 rng(12345);
  const uint64_t ds[] = {1, 2, 3, 5, 7, 31, 32, 33, 64, 65, 100, 255, 256, 257, 1000, 2000, 4096, 65535,
                         65536, 65537, 262144, 1000003, (1ull << 31) - 1, 1ull << 31, (1ull << 32) + 15,
                         (1ull << 40) + 7, (1ull << 62) + 3, (1ull << 63) - 1};
  long bad = 0, n_checks = 0;
  for (uint64_t d : ds) {
    FastDiv f = make_fastdiv(d);
    for (int i = 0; i < 200000; ++i) {
      uint64_t n;
      switch (i % 4) {
        case 0: n = rng(); break;
        case 1: n = rng() >> (rng() % 64); break;
        case 2: n = (rng() % 1000) * d + (rng() % (d < 3 ? 1 : 3)); break;
        default: n = (uint64_t)i; break;
      }
      if (n == 0 && i % 4 == 2) n = d - 1;
      uint64_t q = fd_div(n, f);
      ++n_checks;
      if (q != n / d) {
        if (bad < 10) printf("bad: n=%llu d=%llu got %llu want %llu\n", (unsigned long long)n,
                             (unsigned long long)d, (unsigned long long)q, (unsigned long long)(n / d));
        ++bad;
      }
    }
    // boundary values
    const uint64_t mx = ~(uint64_t)0;
    for (uint64_t n : {(uint64_t)0, d - 1, d, d + 1, 2 * d - 1, mx, mx - 1, (mx / d) * d, (mx / d) * d - 1}) {
      ++n_checks;
      if (fd_div(n, f) != n / d) ++bad;
    }
  }
  printf("%ld checks, %ld bad\n", n_checks, bad);
  return bad ? 1 : 0;
}
