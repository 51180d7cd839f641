/* ORACLE — test infrastructure only (see oracle_ops.h).  CPU restatement of the reference's
 * ArrayHandlerIterable / ArrayHandlerIterableSparse kernels, single-threaded, reference order. */
#include "oracle_ops.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* OR_OMP (liboracle_itsolv_omp.so, tests/golden/make_traces.py --omp only): the loops whose elements are
 * independent run on several threads.  Every element sees the same operations in the same order as
 * the sequential build, so results are bit-identical; the sequential sums of dot stay sequential. */
#ifdef OR_OMP
#define OR_PRAGMA(x) _Pragma(#x)
#define OR_PAR_FOR(len) OR_PRAGMA(omp parallel for schedule(static) if ((len) > 65536))
#else
#define OR_PAR_FOR(len)
#endif

int or_fill(double alpha, double* x, size_t n) {
  OR_PAR_FOR(n)
  for (size_t i = 0; i < n; ++i) x[i] = alpha;
  return 0;
}

int or_scal(double alpha, double* x, size_t n) {
  OR_PAR_FOR(n)
  for (size_t i = 0; i < n; ++i) x[i] *= alpha;
  return 0;
}

int or_copy(double* x, size_t nx, const double* y, size_t ny) {
  if (ny > nx) return 1; /* std::copy(begin(y), end(y), begin(x)) would overrun x */
  OR_PAR_FOR(ny)
  for (size_t i = 0; i < ny; ++i) x[i] = y[i];
  return 0;
}

int or_axpy(double alpha, const double* x, size_t nx, double* y, size_t ny) {
  if (nx < ny) return 1;
  OR_PAR_FOR(ny)
  for (size_t i = 0; i < ny; ++i) y[i] = y[i] + alpha * x[i];
  return 0;
}

/* Summation order of dot / gemm_inner (a checker knob, never the product): 0 = the reference's
 * sequential std::inner_product (ArrayHandlerIterable.h:76-82), the default and the only order the
 * parity fixtures are generated with; 1 = 8 interleaved partial sums folded pairwise, the order a
 * vectorising build of the same loop (-ffast-math / AVX-512) produces.  Order 1 exists to measure
 * how sensitive the REFERENCE algorithm itself is to a valid change of summation order
 * (tests/golden/make_traces.py: the "reordered" runs).  2 = sequential partial sums over consecutive
 * 1024-element blocks, the block sums folded pairwise: the shape of a blocked / threaded reduction
 * (an OpenMP-parallel build of the loop, numpy's pairwise sum) and of the GPU's ("reordered_blocked").
 * 100 + P (P = 2..64) = the reference's distributed build on P MPI ranks with rank-order sums: the index range split
 * by make_distribution_spread_remainder (util/Distribution.h:99-109), each rank's local
 * std::inner_product sequential, the P partials summed in rank order (DistrArray.cpp:124-138, the
 * MPI_Allreduce of util/gemm.h:179-182) ("mpiP" runs) -- one valid association of MPI_Allreduce.
 * 200 + P = the same rank partials combined in the association MPICH's MPI_Allreduce(MPI_SUM) of doubles
 * gives them on one node: with pof2 the largest power of two <= P and rem = P - pof2, ranks 2i and
 * 2i+1 (i < rem) first add their partials, and the pof2 values left are combined pairwise at distance
 * 1, 2, 4, ... (the recursive-doubling / reduce-scatter tree MPICH 3.3 uses for buffers over 2048
 * bytes).  Buffers of at most 2048 bytes MPICH reduces along a binomial tree ((p0 + p1) + (p2 + p3)) +
 * p4 ...; the two trees are the same association for P = 2, 3, 4, 6, 7, 8 (and every power of two),
 * so there the model holds for every buffer length (measured: /opt/conda MPICH 3.3.2, random
 * partials, tests/test_mpi_bridge.py::test_mpich_allreduce_association).  For P = 2 and 3 it is the
 * rank order, for P = 4 (p0 + p1) + (p2 + p3).  Pinned against MPICH's own MPI_Allreduce by the C-API
 * loops of tests/mpi_worker.py ("mpichP" runs). */
static int g_sum_order = 0;

int or_set_sum_order(int order) {
  if (order < 0 || (order > 2 && (order < 102 || order > 164) && (order < 202 || order > 264))) return 1;
  g_sum_order = order;
  return 0;
}

int or_dot(const double* x, size_t nx, const double* y, size_t ny, double* out) {
  if (nx > ny) return 1;
  if (g_sum_order >= 200) {
    const size_t P = (size_t)(g_sum_order - 200), blk = nx / P, extra = nx % P;
    double v[64];
    size_t pof2 = 1;
    while (2 * pof2 <= P) pof2 *= 2;
    const size_t rem = P - pof2;
    for (size_t r = 0; r < P; ++r) {
      const size_t b = r * blk + (r < extra ? r : extra), e = b + blk + (r < extra ? 1 : 0);
      double l = 0;
      for (size_t i = b; i < e; ++i) l = l + x[i] * y[i];
      /* new rank of r: i for the pair (2i, 2i+1), i < rem; r - rem above the pairs */
      if (r < 2 * rem) {
        if (r & 1) v[r / 2] = v[r / 2] + l;
        else v[r / 2] = l;
      } else {
        v[r - rem] = l;
      }
    }
    for (size_t mask = 1; mask < pof2; mask *= 2)
      for (size_t i = 0; i < pof2; i += 2 * mask) v[i] = v[i] + v[i + mask];
    *out = v[0];
    return 0;
  }
  if (g_sum_order >= 100) {
    const size_t P = (size_t)(g_sum_order - 100), blk = nx / P, extra = nx % P;
    double s = 0;
    for (size_t r = 0; r < P; ++r) {
      const size_t b = r * blk + (r < extra ? r : extra), e = b + blk + (r < extra ? 1 : 0);
      double l = 0;
      for (size_t i = b; i < e; ++i) l = l + x[i] * y[i];
      s = r ? s + l : l;
    }
    *out = s;
    return 0;
  }
  if (g_sum_order == 2) {
    const size_t B = 1024;
    size_t nb = (nx + B - 1) / B;
    if (nb == 0) {
      *out = 0;
      return 0;
    }
    double* p = (double*)malloc(nb * sizeof(double));
    if (!p) return 3;
    OR_PAR_FOR(nx)
    for (size_t b = 0; b < nb; ++b) {
      double s = 0;
      size_t e = (b + 1) * B < nx ? (b + 1) * B : nx;
      for (size_t i = b * B; i < e; ++i) s = s + x[i] * y[i];
      p[b] = s;
    }
    while (nb > 1) {
      size_t h = nb / 2;
      for (size_t j = 0; j < h; ++j) p[j] = p[2 * j] + p[2 * j + 1];
      if (nb & 1) p[h] = p[nb - 1];
      nb = h + (nb & 1);
    }
    *out = p[0];
    free(p);
    return 0;
  }
  if (g_sum_order == 1) {
    double p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    size_t i = 0;
    for (; i + 8 <= nx; i += 8)
      for (int l = 0; l < 8; ++l) p[l] = p[l] + x[i + l] * y[i + l];
    for (int l = 0; i < nx; ++i, ++l) p[l] = p[l] + x[i] * y[i];
    *out = ((p[0] + p[4]) + (p[2] + p[6])) + ((p[1] + p[5]) + (p[3] + p[7]));
    return 0;
  }
  double s = 0;
  for (size_t i = 0; i < nx; ++i) s = s + x[i] * y[i];
  *out = s;
  return 0;
}

int or_gemm_inner(const double* const* xx, int m, const double* const* yy, int k, size_t n, double* out) {
  int status = 0;
  /* the m*k dots are independent: OR_OMP spreads whole (sequential) dots over threads */
  OR_PAR_FOR((size_t)m * k * n)
  for (int ij = 0; ij < m * k; ++ij) {
    int s = or_dot(xx[ij / k], n, yy[ij % k], n, &out[ij]);
    if (s) {
#ifdef OR_OMP
#pragma omp critical
#endif
      if (!status) status = s;
    }
  }
  return status;
}

int or_gemm_outer(const double* alphas, const double* const* xx, int k, double* const* yy, int m, size_t n) {
  for (int ii = 0; ii < k; ++ii)
    for (int jj = 0; jj < m; ++jj) {
      int s = or_axpy(alphas[(size_t)ii * m + jj], xx[ii], n, yy[jj], n);
      if (s) return s;
    }
  return 0;
}

/* ---- std::priority_queue<pair<double,size_t>, vector<...>, greater<...>> restated ---------- */
typedef struct {
  double v;
  size_t i;
} pair_t;

/* std::pair operator< */
static int pair_less(const pair_t* a, const pair_t* b) {
  if (a->v < b->v) return 1;
  if (b->v < a->v) return 0;
  return a->i < b->i;
}

/* min-heap: parent <= child under pair_less (top is the smallest pair, popped first) */
static void heap_push(pair_t* h, size_t* size, pair_t p) {
  size_t c = (*size)++;
  h[c] = p;
  while (c > 0) {
    size_t par = (c - 1) / 2;
    if (!pair_less(&h[c], &h[par])) break;
    pair_t t = h[c];
    h[c] = h[par];
    h[par] = t;
    c = par;
  }
}

static void heap_pop(pair_t* h, size_t* size) {
  h[0] = h[--(*size)];
  size_t c = 0;
  for (;;) {
    size_t l = 2 * c + 1, r = l + 1, s = c;
    if (l < *size && pair_less(&h[l], &h[s])) s = l;
    if (r < *size && pair_less(&h[r], &h[s])) s = r;
    if (s == c) break;
    pair_t t = h[c];
    h[c] = h[s];
    h[s] = t;
    c = s;
  }
}

static int cmp_index(const void* a, const void* b) {
  const pair_t* p = (const pair_t*)a;
  const pair_t* q = (const pair_t*)b;
  return (p->i > q->i) - (p->i < q->i);
}

/* Keeps the nsel largest pairs of vals (indices 0..n-1) and writes them in index order. */
static int select_pairs(const double* vals, size_t n, size_t nsel, int negate_out, size_t* idx_out, double* val_out,
                        size_t* nout) {
  pair_t* h = (pair_t*)malloc((nsel + 1) * sizeof(pair_t));
  if (!h) return 3;
  size_t size = 0;
  for (size_t i = 0; i < n; ++i) {
    pair_t p = {vals[i], i};
    if (i < nsel) {
      heap_push(h, &size, p);
    } else {
      heap_push(h, &size, p);
      heap_pop(h, &size);
    }
  }
  qsort(h, size, sizeof(pair_t), cmp_index); /* std::map<size_t, value> order */
  for (size_t e = 0; e < size; ++e) {
    if (idx_out) idx_out[e] = h[e].i;
    if (val_out) val_out[e] = negate_out ? -h[e].v : h[e].v;
  }
  *nout = size;
  free(h);
  return 0;
}

int or_select(const double* x, size_t n, size_t nsel, int max, int ignore_sign, size_t* idx_out, double* val_out,
              size_t* nout) {
  if (nsel > n) return 1; /* "ArrayHandlerIterable::select() n is too large" */
  double* v = (double*)malloc((n ? n : 1) * sizeof(double));
  if (!v) return 3;
  OR_PAR_FOR(n)
  for (size_t i = 0; i < n; ++i)
    v[i] = max ? (ignore_sign ? fabs(x[i]) : x[i]) : (ignore_sign ? -fabs(x[i]) : -x[i]);
  int s = select_pairs(v, n, nsel, !max, idx_out, val_out, nout);
  free(v);
  return s;
}

int or_select_max_dot(const double* x, const double* y, size_t n, size_t nsel, size_t* idx_out, double* val_out,
                      size_t* nout) {
  if (nsel > n) return 1;
  double* v = (double*)malloc((n ? n : 1) * sizeof(double));
  if (!v) return 3;
  OR_PAR_FOR(n)
  for (size_t i = 0; i < n; ++i) v[i] = fabs(x[i] * y[i]);
  int s = select_pairs(v, n, nsel, 0, idx_out, val_out, nout);
  free(v);
  return s;
}

int or_sparse_copy(double* x, size_t n, const size_t* idx, const double* val, size_t nnz) {
  for (size_t i = 0; i < n; ++i) x[i] = 0;
  for (size_t e = 0; e < nnz; ++e) {
    if (idx[e] >= n) return 3; /* the reference writes out of bounds here */
    x[idx[e]] = val[e];
  }
  return 0;
}

int or_sparse_axpy(double alpha, const size_t* idx, const double* val, size_t nnz, double* y, size_t n) {
  for (size_t e = 0; e < nnz; ++e)
    if (idx[e] < n) y[idx[e]] = y[idx[e]] + alpha * val[e];
  return 0;
}

int or_sparse_dot(const double* x, size_t n, const size_t* idx, const double* val, size_t nnz, double* out) {
  double tot = 0;
  for (size_t e = 0; e < nnz; ++e)
    if (idx[e] < n) tot = tot + x[idx[e]] * val[e];
  *out = tot;
  return 0;
}

int or_precondition(double* const* a, int nvec, const double* d, const double* shift, size_t n) {
  for (int k = 0; k < nvec; ++k) {
    OR_PAR_FOR(n)
    for (size_t i = 0; i < n; ++i) a[k][i] = a[k][i] / (d[i] - shift[k] + 1e-15);
  }
  return 0;
}

int or_distribution(size_t dimension, int nchunks, size_t* borders) {
  if (nchunks <= 0) return 3;
  size_t block = dimension / (size_t)nchunks, extra = dimension % (size_t)nchunks;
  borders[0] = 0;
  for (int c = 0; c < nchunks; ++c) borders[c + 1] = borders[c] + block + ((size_t)c < extra ? 1 : 0);
  return 0;
}
