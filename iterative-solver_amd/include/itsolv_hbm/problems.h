// Problem definitions shared by the device solver entry points (host/itsolv_capi.cpp) and the CPU
// oracle (oracle/itsolv_oracle.cpp), and the generic solve drivers both run.
//
// Synthetic H = diag(1 + g) + rho * sum_{l<rank} u_l u_l^T with u_0 = 1 and u_l(g) = +/-1 from
// splitmix64 (the rank-one case is reference test/itsolv/test_rayleigh_quotient.cpp:37-42).  The
// hash is the same function the HIP kernels (csrc/synthetic.hip) and oracle/oracle.py evaluate.
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <functional>
#include <vector>

#include "itsolv_hbm.h"
#include "solvers.h"

namespace molpro::linalg::itsolv::problems {

inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t stream_key(uint64_t seed, uint64_t stream) { return splitmix64(seed ^ (stream * 0xD1B54A32D192ED03ull)); }

// Equidistributed fractions frac(g * phi) for the bounded diagonal (exact in IEEE double on host and
// device: one rounded product, an exact floor and an exact subtraction; csrc/synthetic.hip evaluates
// the same expressions with contraction off).
constexpr double kPhi1 = 0x1.3c6ef372fe950p-1;  // (sqrt(5) - 1) / 2
constexpr double kPhi2 = 0x1.827f5352054c6p-1;  // 1 / plastic number
inline double frac_phi(size_t g, double phi) {
  const double f = double(g) * phi;
  return f - std::floor(f);
}

// Diagonal families of the synthetic H (SSPX_DIAG_* in include/subspace_hip.h):
//   SSPX_DIAG_LINEAR   d_g = 1 + g: the Davidson configurations C1-C4.
//   SSPX_DIAG_BOUNDED  d_g = 1 + 2 frac(g phi1) in [1, 3): the C5 DIIS instance.  Its problem hands
//                      the preconditioner an approximate diagonal p_g = d_g (1 + alpha (2 frac(g phi2)
//                      - 1)) (an approximate Jacobian diagonal, as orbital-energy differences are for
//                      the DIIS of SCF / coupled cluster), so the preconditioned operator has a
//                      continuous spectrum and DIIS converges geometrically (~0.4 per iteration), and
//                      the coupling rho is O(1/N), so |r_0| = |H (e_0 - 1)| ~ 3 sqrt(N): the
//                      threshold 1e-8 sits four orders above the rounding floor eps |H| |x| ~ 1e-12.
struct SyntheticSpec {
  size_t n;
  double rho;
  int rank;
  uint64_t seed;
  int diag_kind = SSPX_DIAG_LINEAR;
  double alpha = 0;
  //! The nonlinear-equations solution's components: r = H (x - target 1) (the reference test's x = 1,
  //! test_NonLinearEquations.cpp:25-49, is target 1; C5 uses 1 / sqrt(n), a unit-norm solution).
  double target = 1.0;
  std::vector<uint64_t> keys;  // per low-rank vector
  SyntheticSpec(size_t n_, double rho_, int rank_, uint64_t seed_, int diag_kind_ = SSPX_DIAG_LINEAR,
                double alpha_ = 0, double target_ = 1.0)
      : n(n_), rho(rho_), rank(rank_), seed(seed_), diag_kind(diag_kind_), alpha(alpha_),
        target(target_ == 0.0 ? 1.0 : target_) {
    for (int l = 0; l < rank; ++l) keys.push_back(stream_key(seed, 1000 + uint64_t(l)));
  }
  double u(int l, size_t g) const { return l == 0 ? 1.0 : ((splitmix64(keys[l] ^ uint64_t(g)) & 1ull) ? -1.0 : 1.0); }
  //! The diagonal part d_g of H (without the low-rank term).
  double d(size_t g) const { return diag_kind == SSPX_DIAG_BOUNDED ? 1.0 + 2.0 * frac_phi(g, kPhi1) : 1.0 + double(g); }
  double h(size_t i, size_t j) const {
    double s = 0;
    for (int l = 0; l < rank; ++l) s += u(l, i) * u(l, j);
    return (i == j ? d(i) : 0.0) + rho * s;
  }
  //! What the problem's diagonals() reports (the preconditioner's diagonal).
  double diagonal(size_t g) const {
    if (diag_kind == SSPX_DIAG_BOUNDED) {
      const double t = 2.0 * frac_phi(g, kPhi2) - 1.0;
      const double s = alpha * t;
      return d(g) * (1.0 + s);
    }
    return 1.0 + double(g) + rank * rho;
  }
  sspx_synth c_spec() const { return sspx_synth{rho, rank, seed, diag_kind, alpha, target}; }
};

//! BASELINE config C5 as a well-posed instance: r = H (x - t 1), H = diag(1 + 2 frac(g phi1)) + (1/N) 1 1^T
//! (the reference's DIIS test form 1 1^T + diag, test_NonLinearEquations.cpp:25-31, with the coupling
//! scaled to the length and the diagonal bounded), preconditioner mismatch alpha = 0.2 and the solution
//! t 1 of unit norm (t = 1/sqrt(N)).  10 steps at every N from |r_0| = 3.2 to the 1e-8 threshold, the
//! last two errors 2.8x above and 1.5x below it, while valid reorderings of the CPU path's sums move
//! them by at most 3 %.  Round 2's alpha = 0.5 with x = 1 stagnated at ~1.4e-8
//! for its last steps, where reorderings moved the errors by up to 43 % and the count followed.
inline SyntheticSpec c5_spec(size_t n, int rank = 1, uint64_t seed = 3, double alpha = 0.2) {
  return SyntheticSpec(n, 1.0 / double(n), rank, seed, SSPX_DIAG_BOUNDED, alpha, 1.0 / std::sqrt(double(n)));
}

// One row of itsolv_result's per-iteration trace (called from solve()'s iteration_hook).
template <class S>
void record_trace(const S& solver, const std::vector<double>& eigenvalues, itsolv_result& out) {
  const int it = out.n_eig_trace;
  if (it >= ITSOLV_TRACE_ITER) return;
  const auto& err = solver.errors();
  out.trace_roots = int(std::min<size_t>(std::max(err.size(), eigenvalues.size()), ITSOLV_TRACE_ROOTS));
  for (int r = 0; r < out.trace_roots; ++r) {
    out.trace_eigenvalues[it * ITSOLV_TRACE_ROOTS + r] = size_t(r) < eigenvalues.size() ? eigenvalues[r] : 0.0;
    out.trace_errors[it * ITSOLV_TRACE_ROOTS + r] = size_t(r) < err.size() ? err[r] : 0.0;
  }
  out.trace_nq[it] = int(solver.dimensions().nQ);
  out.trace_nwork[it] = int(solver.working_set().size());
  out.trace_screened[it] = solver.statistics().redundant_params + solver.statistics().null_params;
  out.eig_trace[it] = eigenvalues.empty() ? 0.0 : eigenvalues.front();
  out.n_eig_trace = it + 1;
}

inline void apply_options(const itsolv_options& o, Options& base) {
  base.n_roots = o.nroots;
  base.convergence_threshold = o.convergence_threshold;
  if (o.max_iter > 0) base.max_iter = o.max_iter;
  base.max_p = o.max_p;
  if (o.p_threshold > 0) base.p_threshold = o.p_threshold;
  base.verbosity = Verbosity(o.verbosity);
}

// Runs LinearEigensystemDavidson::solve and fills `out`.  make_vec() creates a zeroed R vector;
// residual_norm(x, e) returns |H x - e x| (computed by the caller's action).
// The solutions of roots [0, nroots) after solve(), written into the solver's own parameter and
// action buffers (free once solve() has returned) in batches of their count: one solution() call
// per batch reads every Q / D vector once for all the batch's roots (construct_solution's sources
// are summed per destination in the same order either way, so each solution is the one a single-root
// call gives, bit for bit), where a call per root re-reads them per root (C3: 16 passes over 41
// vectors against 2 over 41 + 8).  each(root, solution) runs before the next batch overwrites it.
template <class Solver, class R, class F>
void extract_solutions(Solver& solver, std::vector<R>& params, std::vector<R>& actions, int nroots, F&& each) {
  const size_t batch = std::min(params.size(), actions.size());
  if (batch == 0) return;
  for (size_t r0 = 0; r0 < size_t(std::max(nroots, 0)); r0 += batch) {
    const size_t nb = std::min(batch, size_t(nroots) - r0);
    std::vector<int> roots(nb);
    for (size_t i = 0; i < nb; ++i) roots[i] = int(r0 + i);
    solver.solution(roots, params, actions);
    for (size_t i = 0; i < nb; ++i) each(int(r0 + i), params[i]);
  }
}

// Batched form of residual_norm: out[i] = |H x_i - e_i x_i| / |x_i| for a batch of solutions at once.
template <class R>
using ResidualNormsBatch = std::function<void(const std::vector<const R*>&, const std::vector<double>&, std::vector<double>&)>;

// extract_solutions with the whole batch handed over: each_batch(first root, count, params).
template <class Solver, class R, class F>
void extract_solution_batches(Solver& solver, std::vector<R>& params, std::vector<R>& actions, int nroots,
                              F&& each_batch) {
  const size_t batch = std::min(params.size(), actions.size());
  if (batch == 0) return;
  for (size_t r0 = 0; r0 < size_t(std::max(nroots, 0)); r0 += batch) {
    const size_t nb = std::min(batch, size_t(nroots) - r0);
    std::vector<int> roots(nb);
    for (size_t i = 0; i < nb; ++i) roots[i] = int(r0 + i);
    solver.solution(roots, params, actions);
    each_batch(r0, nb, params);
  }
}

template <class R, class Q, class P>
void run_davidson(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers, const Problem<R, P>& problem,
                  const std::function<R()>& make_vec, const std::function<double(const R&, double)>& residual_norm,
                  const itsolv_options& o, itsolv_result& out, const std::function<void(size_t, const R&)>& emit,
                  const ResidualNormsBatch<R>& residual_norms_batch = {}) {
  LinearEigensystemDavidson<R, Q, P> solver(handlers);
  LinearEigensystemDavidsonOptions opt;
  apply_options(o, opt);
  if (o.max_size_qspace > 0) opt.max_size_qspace = o.max_size_qspace;
  if (o.reset_D > 0) opt.reset_D = o.reset_D;
  if (o.reset_D_max_Q_size > 0) opt.reset_D_max_Q_size = o.reset_D_max_Q_size;
  opt.hermiticity = o.hermitian != 0;
  if (o.block_gram_schmidt >= 0) opt.block_gram_schmidt = o.block_gram_schmidt != 0;
  solver.set_options(opt);
  const size_t nwork = size_t(o.nwork > 0 ? o.nwork : o.nroots);
  std::vector<R> params, actions;
  for (size_t i = 0; i < nwork; ++i) {
    params.push_back(make_vec());
    actions.push_back(make_vec());
  }
  out.n_eig_trace = 0;
  solver.iteration_hook = [&] { record_trace(solver, solver.eigenvalues(), out); };
  dense::AlgebraClock::reset();
  const auto t0 = std::chrono::steady_clock::now();
  out.converged = solver.solve(params, actions, problem, o.generate_initial_guess != 0);
  out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  out.host_algebra_seconds = dense::AlgebraClock::seconds;
  out.host_algebra_calls = dense::AlgebraClock::calls;
  out.host_algebra_max_dim = int(dense::AlgebraClock::max_dim);
  const auto& st = solver.statistics();
  out.iterations = st.iterations;
  out.r_creations = st.r_creations;
  out.q_creations = st.q_creations;
  out.redundant_params = st.redundant_params;
  out.null_params = st.null_params;
  const auto ev = solver.eigenvalues();
  out.nroots = int(std::min<size_t>(ev.size(), ITSOLV_MAX_ROOTS));
  for (int i = 0; i < out.nroots; ++i) {
    out.eigenvalues[i] = ev[i];
    out.errors[i] = i < int(solver.errors().size()) ? solver.errors()[i] : 0.0;
  }
  // Solutions, residuals recomputed from the problem's action (per root, or per batch of extracted
  // roots when the caller has the batched form: one action over the batch, the residuals with their
  // norms in one pass).
  if (residual_norms_batch) {
    extract_solution_batches(solver, params, actions, out.nroots, [&](size_t r0, size_t nb, std::vector<R>& xs) {
      std::vector<const R*> px;
      std::vector<double> e, rn(nb);
      for (size_t i = 0; i < nb; ++i) {
        px.push_back(&xs[i]);
        e.push_back(ev[r0 + i]);
      }
      residual_norms_batch(px, e, rn);
      for (size_t i = 0; i < nb; ++i) {
        out.residual_norms[r0 + i] = rn[i];
        if (emit) emit(r0 + i, xs[i]);
      }
    });
    return;
  }
  extract_solutions(solver, params, actions, out.nroots, [&](int r, const R& x) {
    out.residual_norms[r] = residual_norm(x, ev[size_t(r)]);
    if (emit) emit(size_t(r), x);
  });
}

// Runs LinearEquationsDavidson::solve on A x = b for the given right-hand sides and fills `out`;
// residual_norms are |A x - b| / |b| recomputed by residual_norm(x, root).
template <class R, class Q, class P>
void run_linear_equations(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers, const Problem<R, P>& problem,
                          const std::function<R()>& make_vec, std::vector<R>& rhs,
                          const std::function<double(const R&, size_t)>& residual_norm, const itsolv_options& o,
                          itsolv_result& out, const std::function<void(size_t, const R&)>& emit) {
  LinearEquationsDavidson<R, Q, P> solver(handlers);
  solver.add_equations(rhs);
  LinearEquationsDavidsonOptions opt;
  apply_options(o, opt);
  opt.n_roots = int(rhs.size());
  if (o.max_size_qspace > 0) opt.max_size_qspace = o.max_size_qspace;
  if (o.reset_D > 0) opt.reset_D = o.reset_D;
  if (o.reset_D_max_Q_size > 0) opt.reset_D_max_Q_size = o.reset_D_max_Q_size;
  opt.hermiticity = o.hermitian != 0;
  if (o.augmented_hessian > 0) opt.augmented_hessian = o.augmented_hessian;
  if (o.block_gram_schmidt >= 0) opt.block_gram_schmidt = o.block_gram_schmidt != 0;
  solver.set_options(opt);
  const size_t nwork = rhs.size();
  std::vector<R> params, actions;
  for (size_t i = 0; i < nwork; ++i) {
    params.push_back(make_vec());
    actions.push_back(make_vec());
  }
  out.n_eig_trace = 0;
  solver.iteration_hook = [&] { record_trace(solver, std::vector<double>{}, out); };
  dense::AlgebraClock::reset();
  const auto t0 = std::chrono::steady_clock::now();
  out.converged = solver.solve(params, actions, problem, o.generate_initial_guess != 0);
  out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  out.host_algebra_seconds = dense::AlgebraClock::seconds;
  out.host_algebra_calls = dense::AlgebraClock::calls;
  out.host_algebra_max_dim = int(dense::AlgebraClock::max_dim);
  const auto& st = solver.statistics();
  out.iterations = st.iterations;
  out.r_creations = st.r_creations;
  out.q_creations = st.q_creations;
  out.redundant_params = st.redundant_params;
  out.null_params = st.null_params;
  out.nroots = int(std::min<size_t>(nwork, ITSOLV_MAX_ROOTS));
  for (int i = 0; i < out.nroots; ++i) {
    out.eigenvalues[i] = 0;
    out.errors[i] = i < int(solver.errors().size()) ? solver.errors()[i] : 0.0;
  }
  extract_solutions(solver, params, actions, out.nroots, [&](int r, const R& x) {
    out.residual_norms[r] = residual_norm(x, size_t(r));
    if (emit) emit(size_t(r), x);
  });
}

// Runs OptimizeBFGS (algorithm 0) or OptimizeSD (1) from x0 (set by init); eigenvalues[0] is
// the final function value (reference OptimizeBFGS.h, OptimizeSD.h).
template <class R, class Q, class P>
void run_optimize(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers, const Problem<R, P>& problem,
                  const std::function<R()>& make_vec, const std::function<void(R&)>& init, int algorithm,
                  const itsolv_options& o, itsolv_result& out, const std::function<void(const R&)>& emit) {
  std::unique_ptr<IterativeSolverTemplate<R, Q, P>> solver;
  if (algorithm == 0) {
    auto b = std::make_unique<OptimizeBFGS<R, Q, P>>(handlers);
    OptimizeBFGSOptions opt;
    apply_options(o, opt);
    opt.n_roots = 1;
    if (o.max_size_qspace > 0) opt.max_size_qspace = o.max_size_qspace;
    b->set_options(opt);
    solver = std::move(b);
  } else {
    solver = std::make_unique<OptimizeSD<R, Q, P>>(handlers);
    Options opt;
    apply_options(o, opt);
    opt.n_roots = 1;
    solver->set_options(opt);
  }
  R x = make_vec(), g = make_vec();
  init(x);
  out.n_eig_trace = 0;
  solver->iteration_hook = [&] { record_trace(*solver, std::vector<double>{solver->value()}, out); };
  dense::AlgebraClock::reset();
  const auto t0 = std::chrono::steady_clock::now();
  out.converged = solver->solve(x, g, problem);
  out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  out.host_algebra_seconds = dense::AlgebraClock::seconds;
  out.host_algebra_calls = dense::AlgebraClock::calls;
  out.host_algebra_max_dim = int(dense::AlgebraClock::max_dim);
  const auto& st = solver->statistics();
  out.iterations = st.iterations;
  out.r_creations = st.r_creations;
  out.q_creations = st.q_creations;
  out.redundant_params = st.redundant_params;
  out.null_params = st.null_params;
  out.nroots = 1;
  out.errors[0] = solver->errors().empty() ? 0.0 : solver->errors().front();
  out.eigenvalues[0] = solver->value();
  R xs = make_vec(), gs = make_vec();
  solver->solution(xs, gs);
  problem.residual(xs, gs);
  out.residual_norms[0] = std::sqrt(std::abs(handlers->rr().dot(gs, gs)));
  if (emit) emit(xs);
}

// Runs NonLinearEquationsDIIS::solve from x0 (set by init) and fills `out`.
template <class R, class Q, class P>
void run_diis(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers, const Problem<R, P>& problem,
              const std::function<R()>& make_vec, const std::function<void(R&)>& init,
              const itsolv_options& o, itsolv_result& out, const std::function<void(const R&)>& emit) {
  NonLinearEquationsDIIS<R, Q, P> solver(handlers);
  NonLinearEquationsDIISOptions opt;
  apply_options(o, opt);
  opt.n_roots = 1;
  if (o.max_size_qspace > 0) opt.max_size_qspace = o.max_size_qspace;
  solver.set_options(opt);
  R x = make_vec(), g = make_vec();
  init(x);
  out.n_eig_trace = 0;
  solver.iteration_hook = [&] { record_trace(solver, std::vector<double>{}, out); };
  dense::AlgebraClock::reset();
  const auto t0 = std::chrono::steady_clock::now();
  out.converged = solver.solve(x, g, problem);
  out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  out.host_algebra_seconds = dense::AlgebraClock::seconds;
  out.host_algebra_calls = dense::AlgebraClock::calls;
  out.host_algebra_max_dim = int(dense::AlgebraClock::max_dim);
  const auto& st = solver.statistics();
  out.iterations = st.iterations;
  out.r_creations = st.r_creations;
  out.q_creations = st.q_creations;
  out.redundant_params = st.redundant_params;
  out.null_params = st.null_params;
  out.nroots = 1;
  out.errors[0] = solver.errors().empty() ? 0.0 : solver.errors().front();
  out.eigenvalues[0] = 0;
  // the solution's parameters only: its residual is recomputed from the problem right after (the
  // solver's residual combination would be overwritten unread)
  R xs = make_vec(), gs = make_vec();
  solver.solution_params(std::vector<int>{0}, VecRef<R>{std::ref(xs)});
  problem.residual(xs, gs);
  out.residual_norms[0] = std::sqrt(std::abs(handlers->rr().dot(gs, gs)));
  if (emit) emit(xs);
}

inline void default_options(itsolv_options* o) {
  o->nroots = 1;
  o->nwork = 0;
  o->max_iter = 100;
  o->max_size_qspace = 0;
  o->reset_D = 0;
  o->reset_D_max_Q_size = 0;
  o->augmented_hessian = 0;
  o->block_gram_schmidt = -1;
  o->max_p = 0;
  o->p_threshold = 0;
  o->convergence_threshold = 1e-8;
  o->hermitian = 1;
  o->generate_initial_guess = 1;
  o->verbosity = 0;
}

}  // namespace molpro::linalg::itsolv::problems
