/* local_step.c -- the reference LOCAL mode's C2 step on host cores (OpenMP).
 *
 * TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it as an extra
 * multi-core CPU line ("an OpenMP C++ CPU permute on all
 * cores may be reported as an extra line, not as 'reference'"), and
 * tests/test_cpu_baseline_c.py checks it against numpy.  Never linked or
 * loaded by bolt_amd.
 *
 * What it restates: bolt's local mode is a numpy subclass
 * (bolt/local/array.py:8); BoltArrayLocal.swap((0,), (0, 1)) is
 * ascontiguousarray(x.transpose(1, 2, 0)) (local/array.py swap -> transpose),
 * and mean / std over the last axis are numpy's reductions.  Here:
 *   swap : y[p][t] = x[t][p] for x of shape [T][P] (P = 512 * 512), cache-
 *          blocked 64 x 64 tiles, threads over blocks of p;
 *   mean : per p, sum over t in float64, divided by T, rounded to float32;
 *   std  : per p, two passes in float64 (mean, then the sum of squared
 *          deviations), sqrt(m2 / T) rounded to float32 (numpy's ddof = 0).
 * The statistics read the swapped array, as the reference's calls do.
 */
#include <math.h>
#include <stdint.h>
#include <omp.h>

enum { TB = 64 };

void local_swap(const float *x, float *y, int64_t T, int64_t P, int threads) {
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int64_t p0 = 0; p0 < P; p0 += TB) {
    const int64_t p1 = p0 + TB < P ? p0 + TB : P;
    for (int64_t t0 = 0; t0 < T; t0 += TB) {
      const int64_t t1 = t0 + TB < T ? t0 + TB : T;
      for (int64_t p = p0; p < p1; ++p)
        for (int64_t t = t0; t < t1; ++t) y[p * T + t] = x[t * P + p];
    }
  }
}

void local_mean(const float *y, float *out, int64_t T, int64_t P, int threads) {
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int64_t p = 0; p < P; ++p) {
    const float *r = y + p * T;
    double s = 0.0;
    for (int64_t t = 0; t < T; ++t) s += r[t];
    out[p] = (float)(s / (double)T);
  }
}

void local_std(const float *y, float *out, int64_t T, int64_t P, int threads) {
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int64_t p = 0; p < P; ++p) {
    const float *r = y + p * T;
    double s = 0.0;
    for (int64_t t = 0; t < T; ++t) s += r[t];
    const double mu = s / (double)T;
    double m2 = 0.0;
    for (int64_t t = 0; t < T; ++t) {
      const double d = r[t] - mu;
      m2 += d * d;
    }
    out[p] = (float)sqrt(m2 / (double)T);
  }
}

int local_max_threads(void) { return omp_get_max_threads(); }
