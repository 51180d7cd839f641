/*
 * itsolv_hbm.h — C ABI of libitsolv_hbm.so: the host C++ solvers (LinearEigensystemDavidson,
 * NonLinearEquationsDIIS; restated from the reference's itsolv headers) running over the HBM handlers of
 * libsubspace_hip.so.  These entry points drive a complete solve on a problem whose action is
 * computed on the device, and report what the reference's tests check: eigenvalues, errors,
 * statistics().iterations, and recomputed residual norms.
 *
 * The context is a libsubspace_hip.so ssp_ctx (with an RCCL communicator attached for more than
 * one rank); every rank calls the same entry point with the same arguments (SPMD, as the
 * reference's MPI build requires).  The oracle (oracle/itsolv_oracle.cpp) exports the same
 * functions with an `oracle_` prefix and std::vector<double> CPU handlers.
 */
#ifndef ITSOLV_HBM_H
#define ITSOLV_HBM_H
#include <stddef.h>

#include "subspace_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ITSOLV_MAX_ROOTS 64
#define ITSOLV_TRACE_ITER 256
#define ITSOLV_TRACE_ROOTS 8

typedef struct {
  int nroots;                  /* n_roots (reference Options::n_roots)                    */
  int nwork;                   /* number of R buffers handed to solve(); 0 -> nroots       */
  int max_iter;                /* reference IterativeSolverTemplate m_max_iter (default 100) */
  int max_size_qspace;         /* reference option max_size_qspace (<= 0: unlimited)       */
  int reset_D;                 /* reference option reset_D (<= 0: never)                   */
  int reset_D_max_Q_size;      /* <= 0: unlimited                                          */
  int max_p;                   /* P-space size limit (0: no P space)                       */
  double p_threshold;          /* P-space selection threshold (<= 0: infinity)             */
  double convergence_threshold;
  int hermitian;
  int generate_initial_guess;  /* 1: initial guess from the n smallest diagonals           */
  int verbosity;               /* 0 none .. 3 detailed                                     */
  double augmented_hessian;    /* LinearEquationsDavidson augmented-Hessian parameter (0: off) */
  int block_gram_schmidt;      /* extension (-1: the vector type's default, 0: the reference's MGS,
                                  1: on): orthogonalise the new
                                  R vectors against P, Q, D with coefficients from the overlaps
                                  already computed for redundancy screening (forward substitution
                                  through the stored S) and one gemm_outer per space; same result
                                  in exact arithmetic, not bit-identical */
} itsolv_options;

typedef struct {
  int converged;
  int iterations;      /* statistics().iterations                                          */
  int r_creations;
  int q_creations;
  int nroots;
  double eigenvalues[ITSOLV_MAX_ROOTS];
  double errors[ITSOLV_MAX_ROOTS];
  double residual_norms[ITSOLV_MAX_ROOTS]; /* |H x - e x| / |x| recomputed from solution() */
  double seconds;      /* wall time of the solve                                            */
  int n_eig_trace;     /* iterations recorded in eig_trace (<= 256)                          */
  double eig_trace[256]; /* lowest eigenvalue after each add_vector                          */
  /* Per-iteration trace (the parity observables of IterativeSolverTemplate.h:322-408), one row
   * per solve() iteration, n_eig_trace rows: eigenvalues (Davidson) and errors of the first
   * trace_roots roots, Q-space size and working-set size after the iteration. */
  int trace_roots;
  int trace_nq[ITSOLV_TRACE_ITER];
  int trace_nwork[ITSOLV_TRACE_ITER];
  double trace_eigenvalues[ITSOLV_TRACE_ITER * ITSOLV_TRACE_ROOTS];
  double trace_errors[ITSOLV_TRACE_ITER * ITSOLV_TRACE_ROOTS];
  /* propose_rspace's screening (extension): new R vectors removed by the redundancy screen and as
   * null after orthogonalisation, in all, and cumulative after each iteration */
  int redundant_params;
  int null_params;
  int trace_screened[ITSOLV_TRACE_ITER];
  /* host time of the subspace algebra (extension, instrumentation): wall seconds, calls and the
   * largest dimension of the eigenproblem / svd_system / solve_DIIS / solve_LinearEquations calls
   * of the solve (itsolv_hbm/dense.h AlgebraClock) */
  double host_algebra_seconds;
  int host_algebra_calls;
  int host_algebra_max_dim;
} itsolv_result;

const char* itsolv_last_error(void);
void itsolv_default_options(itsolv_options* opt);

/* Davidson on H = diag(1+g) + rho * sum_{l<rank} u_l u_l^T (global length n, sharded over the
 * context's ranks).  solutions_out (optional): this rank's shard of each root, nroots x n_local. */
int itsolv_davidson_synthetic(ssp_ctx* ctx, size_t n, double rho, int rank, unsigned long long seed,
                              const itsolv_options* opt, itsolv_result* out, double* solutions_out);

/* Davidson on a dense n x n row-major matrix (small fixtures; single rank). */
int itsolv_davidson_dense(ssp_ctx* ctx, const double* h, size_t n, const itsolv_options* opt, itsolv_result* out,
                          double* solutions_out);

/* DIIS on the residual r(x) = H (x - 1) of the synthetic H (solution x = 1), diagonal
 * preconditioner, x0 = 0 except x0[0] = 1.  x_out (optional): this rank's shard of the solution. */
int itsolv_diis_synthetic(ssp_ctx* ctx, size_t n, double rho, int rank, unsigned long long seed,
                          const itsolv_options* opt, itsolv_result* out, double* x_out);

/* The same two solves on any synthetic family (subspace_hip.h sspx_synth), e.g. BASELINE config
 * C5's well-posed DIIS instance: diag_kind SSPX_DIAG_BOUNDED, rho = 1/n, rank 1, alpha 0.5
 * (itsolv_hbm/problems.h c5_spec). */
int itsolv_davidson_synth(ssp_ctx* ctx, size_t n, const sspx_synth* spec, const itsolv_options* opt,
                          itsolv_result* out, double* solutions_out);
int itsolv_diis_synth(ssp_ctx* ctx, size_t n, const sspx_synth* spec, const itsolv_options* opt, itsolv_result* out,
                      double* x_out);

/* DIIS on r(x) = H (x - 1) for a dense row-major H (reference test_NonLinearEquations.cpp:38-49). */
/* LinearEquationsDavidson (reference itsolv/LinearEquationsDavidson.h): A x_r = b_r for nrhs
 * right-hand sides b (row-major nrhs x n, host), dense row-major A resident in HBM (single rank).
 * x_out (nrhs x n, host) may be NULL. */
int itsolv_linear_equations_dense(ssp_ctx* ctx, const double* a, size_t n, const double* rhs, int nrhs,
                                  const itsolv_options* opt, itsolv_result* out, double* x_out);
/* OptimizeBFGS (algorithm 0) or OptimizeSD (1) minimising the Rayleigh quotient x.Hx / x.x of a
 * dense row-major H (HBM, single rank) from x = e_0; eigenvalues[0] = final function value, x_out
 * (n, host) may be NULL. */
int itsolv_optimize_dense(ssp_ctx* ctx, const double* h, size_t n, int algorithm, const itsolv_options* opt,
                          itsolv_result* out, double* x_out);
int itsolv_diis_dense(ssp_ctx* ctx, const double* h, size_t n, const itsolv_options* opt, itsolv_result* out,
                      double* x_out);

#ifdef __cplusplus
}
#endif
#endif /* ITSOLV_HBM_H */
