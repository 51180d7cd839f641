/* ORACLE-SIDE BASELINE (test/bench infrastructure only; never linked into the product).
 *
 * "host-parallel" CPU baseline of bench.py's subspace-update step ("also time an
 * OpenMP variant on all host cores, reported as host-parallel, not reference"). The same op
 * sequence as oracle.CpuUpdateStep — 2 x gemm_inner(m x k), 2 x [fill x m + gemm_outer(k -> m)],
 * m axpy, m dot — but written the way a tuned host code would: OpenMP over index tiles,
 * cache-blocked gemm_inner / gemm_outer that read each vector once per call (not the reference's
 * pairwise loops), compiler-vectorised inner loops.
 */
#include <omp.h>
#include <stddef.h>
#include <string.h>

#define HP_TILE 1024
#define HP_MAXM 16
#define HP_MAXK 64

int hp_threads(void) { return omp_get_max_threads(); }

static void gemm_inner(double* const* x, int m, double* const* y, int k, size_t n, double* out) {
  memset(out, 0, sizeof(double) * (size_t)m * (size_t)k);
#pragma omp parallel
  {
    double acc[HP_MAXM * HP_MAXK];
    memset(acc, 0, sizeof acc);
#pragma omp for schedule(static)
    for (size_t t = 0; t < n; t += HP_TILE) {
      const size_t e = t + HP_TILE < n ? t + HP_TILE : n;
      for (int i = 0; i < m; ++i)
        for (int j = 0; j < k; ++j) {
          const double* xi = x[i];
          const double* yj = y[j];
          double s = 0;
#pragma omp simd reduction(+ : s)
          for (size_t p = t; p < e; ++p) s += xi[p] * yj[p];
          acc[i * k + j] += s;
        }
    }
#pragma omp critical
    for (int q = 0; q < m * k; ++q) out[q] += acc[q];
  }
}

static void gemm_outer(const double* alpha, double* const* x, int k, double* const* y, int m, size_t n) {
#pragma omp parallel for schedule(static)
  for (size_t t = 0; t < n; t += HP_TILE) {
    const size_t e = t + HP_TILE < n ? t + HP_TILE : n;
    for (int j = 0; j < m; ++j) {
      double* yj = y[j];
      for (int i = 0; i < k; ++i) {
        const double a = alpha[(size_t)i * m + j];
        const double* xi = x[i];
#pragma omp simd
        for (size_t p = t; p < e; ++p) yj[p] += a * xi[p];
      }
    }
  }
}

static void fill0(double* x, size_t n) {
#pragma omp parallel for schedule(static)
  for (size_t p = 0; p < n; ++p) x[p] = 0;
}

static void axpy(double a, const double* x, double* y, size_t n) {
#pragma omp parallel for simd schedule(static)
  for (size_t p = 0; p < n; ++p) y[p] += a * x[p];
}

static double dot(const double* x, const double* y, size_t n) {
  double s = 0;
#pragma omp parallel for simd reduction(+ : s) schedule(static)
  for (size_t p = 0; p < n; ++p) s += x[p] * y[p];
  return s;
}

int hp_update_step(double* const* rp, double* const* ra, double* const* qp, double* const* qa, int m, int k, size_t n,
                   const double* coef, const double* lam, double* out) {
  if (m > HP_MAXM || k > HP_MAXK) return 1;
  gemm_inner(rp, m, qp, k, n, out);
  gemm_inner(rp, m, qa, k, n, out);
  for (int i = 0; i < m; ++i) fill0(rp[i], n);
  gemm_outer(coef, qp, k, rp, m, n);
  for (int i = 0; i < m; ++i) fill0(ra[i], n);
  gemm_outer(coef, qa, k, ra, m, n);
  for (int i = 0; i < m; ++i) axpy(-lam[i], rp[i], ra[i], n);
  double e = 0;
  for (int i = 0; i < m; ++i) {
    const double d = dot(ra[i], ra[i], n);
    e = d > e ? d : e;
  }
  out[0] += 0 * e;
  return 0;
}

/* First-touch initialisation by the threads that will stream the data (NUMA placement). */
void hp_first_touch(double* x, size_t n, double v) {
#pragma omp parallel for schedule(static)
  for (size_t p = 0; p < n; ++p) x[p] = v;
}
