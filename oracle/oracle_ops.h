/*
 * ORACLE — test infrastructure only.  CPU restatement of the reference's ArrayHandlerIterable /
 * ArrayHandlerIterableSparse kernels (knowles-group/iterative-solver @ 2025-03-04).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker
 * (never as the thing measured for `value`, never as a fallback of the product path).
 *
 * Every function follows the reference loop it names, in the same element order, single-threaded,
 * so a result here is the reference's result for the same inputs (up to the compiler's
 * floating-point contraction, which the Makefile disables to match an x86-64 build without FMA).
 *
 * Pinned by tests/test_oracle.py against the reference's own known answers (select_max_dot
 * {6:4, 4:3, 1:2}, testArrayHandlerIterable.cpp:57-69; gemm_inner == pairwise dot, testGemm.cpp:58-88)
 * and golden vectors in tests/golden/.
 *
 * Return codes: 0 ok, 1 size error (ArrayHandlerError), 3 bad argument.
 */
#ifndef ORACLE_OPS_H
#define ORACLE_OPS_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ArrayHandlerIterable.h:59-63 */
int or_fill(double alpha, double* x, size_t n);
/* ArrayHandlerIterable.h:54-57 */
int or_scal(double alpha, double* x, size_t n);
/* ArrayHandlerIterable.h:48-52  (x <- y, y.size() elements) */
int or_copy(double* x, size_t nx, const double* y, size_t ny);
/* ArrayHandlerIterable.h:65-74  (error if x.size() < y.size()) */
int or_axpy(double alpha, const double* x, size_t nx, double* y, size_t ny);
/* ArrayHandlerIterable.h:76-82  (error if x.size() > y.size()), std::inner_product from 0 */
int or_set_sum_order(int order); /* 0 = reference sequential (default), 1 = 8 interleaved sums */
int or_dot(const double* x, size_t nx, const double* y, size_t ny, double* out);
/* util/gemm.h:267-279 gemm_inner_default: out[i*k+j] = dot(xx[i], yy[j]) */
int or_gemm_inner(const double* const* xx, int m, const double* const* yy, int k, size_t n, double* out);
/* util/gemm.h:257-265 gemm_outer_default: for ii (rows of alphas): for jj: axpy(alphas(ii,jj), xx[ii], yy[jj]) */
int or_gemm_outer(const double* alphas, const double* const* xx, int k, double* const* yy, int m, size_t n);
/* util/select.h:28-55 (via ArrayHandlerIterable::select :98-102, error if n > x.size()) */
int or_select(const double* x, size_t n, size_t nsel, int max, int ignore_sign, size_t* idx_out, double* val_out,
              size_t* nout);
/* util/select_max_dot.h:166-190 */
int or_select_max_dot(const double* x, const double* y, size_t n, size_t nsel, size_t* idx_out, double* val_out,
                      size_t* nout);
/* ArrayHandlerIterableSparse.h:167-172: x = 0, x[i] = v */
int or_sparse_copy(double* x, size_t n, const size_t* idx, const double* val, size_t nnz);
/* ArrayHandlerIterableSparse.h:178-182: y[i] += alpha * v for i < y.size() */
int or_sparse_axpy(double alpha, const size_t* idx, const double* val, size_t nnz, double* y, size_t n);
/* ArrayHandlerIterableSparse.h:184-190: sum of x[i] * v for i < x.size() */
int or_sparse_dot(const double* x, size_t n, const size_t* idx, const double* val, size_t nnz, double* out);
/* itsolv/IterativeSolver.h:46-55 precondition_default: a[k][i] = a[k][i] / (d[i] - shift[k] + 1e-15) */
int or_precondition(double* const* a, int nvec, const double* d, const double* shift, size_t n);
/* util/Distribution.h:376-387 make_distribution_spread_remainder: borders[0..nchunks] */
int or_distribution(size_t dimension, int nchunks, size_t* borders);

#ifdef __cplusplus
}
#endif
#endif
