// Iterative solvers over the ArrayHandlers boundary: LinearEigensystemDavidson and
// NonLinearEquationsDIIS, with the reverse-communication interface (add_vector / end_iteration /
// solution) and the one-call solve(parameters, actions, problem).
//
// Restated from the reference:
//   Problem                         itsolv/IterativeSolver.h:76-172, precondition_default :34-63
//   detail::construct_solution etc. itsolv/IterativeSolverTemplate.h:19-117
//   IterativeSolverTemplate          :126-600 (add_vector :140-166, add_p :176-187, solution :191-215,
//                                    solve :322-408, solve_and_generate_working_set :518-563)
//   SubspaceSolverLinEig             itsolv/subspace/SubspaceSolverLinEig.h:23-124
//   SubspaceSolverDIIS               itsolv/subspace/SubspaceSolverDIIS.h:19-96
//   LinearEigensystemDavidson        itsolv/LinearEigensystemDavidson.h:27-199
//   NonLinearEquationsDIIS           itsolv/NonLinearEquationsDIIS.h:28-185
// All vector work goes through the handlers; these classes only move small matrices around, so
// with HBM handlers the same code is the GPU solver and with the oracle's CPU handlers it is the
// reference CPU path.
#pragma once
#include <algorithm>
#include <cmath>
#include <functional>
#include <iomanip>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "interpolate.h"
#include "rspace.h"

namespace molpro::linalg::itsolv {

using subspace::EqnData;
using subspace::Matrix;

// Generic preconditioner for iterable containers (reference IterativeSolver.h:46-55).  Device vector
// types supply their own overload.
template <class T, typename = typename T::iterator>
void precondition_default(const VecRef<T>& action, const std::vector<double>& shift, const T& diagonals) {
  for (size_t k = 0; k < action.size(); ++k) {
    auto& a = action[k].get();
    auto d = diagonals.begin();
    for (auto it = a.begin(); it != a.end(); ++it, ++d) *it = *it / (*d - shift[k] + 1e-15);
  }
}

template <typename R, typename P = std::map<size_t, typename R::value_type>>
class Problem {
 public:
  using container_t = R;
  using value_t = typename R::value_type;
  virtual ~Problem() = default;
  virtual value_t residual(const R& parameters, R& residual) const { return 0; }
  virtual void action(const CVecRef<R>& parameters, const VecRef<R>& action) const {}
  virtual bool diagonals(container_t& d) const { return false; }
  virtual void precondition(const VecRef<R>& residual, const std::vector<value_t>& shift) const {}
  virtual void precondition(const VecRef<R>& residual, const std::vector<value_t>& shift, const R& diagonals) const {
    precondition_default(residual, shift, diagonals);
  }
  virtual std::vector<double> pp_action_matrix(const std::vector<P>& pparams) const {
    if (!pparams.empty()) throw std::logic_error("P-space unavailable: unimplemented pp_action_matrix() in Problem class");
    return {};
  }
  virtual void p_action(const std::vector<std::vector<value_t>>& p_coefficients, const CVecRef<P>& pparams,
                        const VecRef<container_t>& actions) const {
    if (!pparams.empty()) throw std::logic_error("P-space unavailable: unimplemented p_action() in Problem class");
  }
  // Parameter sets for IterativeSolverTemplate::test_problem (reference IterativeSolver.h:163-171):
  // fill `parameters` for instance 0, 1, ... and return false when there are no more.
  virtual bool test_parameters(unsigned int instance, R& parameters) const { return false; }
};

namespace detail {

inline std::vector<std::pair<size_t, size_t>> parameter_batches(size_t nsol, size_t nparam) {
  std::vector<std::pair<size_t, size_t>> b;
  if (nparam && nsol)
    for (size_t s = 0; s < nsol; s += nparam) b.emplace_back(s, std::min(s + nparam, nsol));
  return b;
}

// params[i] = sum over P, Q, D of solutions(roots[i], .) (reference IterativeSolverTemplate.h:33-65):
// fill(0) then one gemm_outer per space.
template <class R, class Q, class P>
void construct_solution(const VecRef<R>& params, const std::vector<int>& roots, const Matrix<double>& sol,
                        const CVecRef<P>& pp, const CVecRef<Q>& qp, const CVecRef<Q>& dp, size_t oP, size_t oQ,
                        size_t oD, ArrayHandlers<R, Q, P>& h) {
  if (roots.empty()) return;
  {
    // Handlers with a one-pass form write the solutions without reading them: each destination
    // still sums its sources from zero in the order P, Q, D.
    Matrix<double> cp({pp.size(), roots.size()}), cqd({qp.size() + dp.size(), roots.size()});
    for (size_t i = 0; i < roots.size(); ++i) {
      for (size_t j = 0; j < pp.size(); ++j) cp(j, i) = sol(roots[i], oP + j);
      for (size_t j = 0; j < qp.size(); ++j) cqd(j, i) = sol(roots[i], oQ + j);
      for (size_t j = 0; j < dp.size(); ++j) cqd(qp.size() + j, i) = sol(roots[i], oD + j);
    }
    CVecRef<Q> qd(qp.begin(), qp.end());
    qd.insert(qd.end(), dp.begin(), dp.end());
    using array::fused_construct_solution;
    if (fused_construct_solution(h.rp(), cp, pp, cqd, qd, params)) return;
  }
  for (size_t i = 0; i < roots.size(); ++i) h.rr().fill(0, params.at(i));
  Matrix<double> cp({pp.size(), roots.size()}), cq({qp.size(), roots.size()}), cd({dp.size(), roots.size()});
  for (size_t i = 0; i < roots.size(); ++i) {
    for (size_t j = 0; j < pp.size(); ++j) cp(j, i) = sol(roots[i], oP + j);
    for (size_t j = 0; j < qp.size(); ++j) cq(j, i) = sol(roots[i], oQ + j);
    for (size_t j = 0; j < dp.size(); ++j) cd(j, i) = sol(roots[i], oD + j);
  }
  h.rp().gemm_outer(cp, pp, params);
  h.rq().gemm_outer(cq, qp, params);
  h.rq().gemm_outer(cd, dp, params);
}

inline std::vector<std::vector<double>> construct_vectorP(const std::vector<int>& roots, const Matrix<double>& sol,
                                                          size_t oP, size_t nP) {
  std::vector<std::vector<double>> v;
  for (auto r : roots) {
    v.emplace_back();
    for (size_t j = 0; j < nP; ++j) v.back().push_back(sol(r, oP + j));
  }
  return v;
}

template <class R>
void normalise_pairs(size_t n, const VecRef<R>& params, const VecRef<R>& actions, array::ArrayHandler<R, R>& h,
                     Logger& log) {
  const auto dots = self_dots(VecRef<R>(params.begin(), params.begin() + long(n)), h);
  for (size_t i = 0; i < n; ++i) {
    const double d = std::sqrt(std::abs(dots[i]));
    if (d > 1.0e-14) {
      h.scal(1. / d, params.at(i));
      h.scal(1. / d, actions.at(i));
    } else {
      log.msg("solution parameter's length is too small, dot = " + Logger::scientific(d), Logger::Warn);
    }
  }
}

// reference IterativeSolverTemplate.h:95-102, the root norms as one lazy batch (detail::self_dots)
template <class R>
void update_errors(std::vector<double>& errors, const CVecRef<R>& residual, array::ArrayHandler<R, R>& h) {
  const auto dots = self_dots(CVecRef<R>(residual.begin(), residual.begin() + long(errors.size())), h);
  for (size_t i = 0; i < errors.size(); ++i) errors[i] = std::sqrt(std::abs(dots[i]));
}

// The nw roots with the largest errors above threshold, in ascending root order (reference :104-117).
inline std::vector<int> select_working_set(size_t nw, const std::vector<double>& errors, double thr,
                                           const std::vector<double>& value_errors, double value_thr) {
  std::multimap<double, size_t, std::greater<double>> ordered;
  for (size_t i = 0; i < errors.size(); ++i)
    if (errors[i] > thr || (i < value_errors.size() && value_errors[i] > value_thr)) ordered.emplace(errors[i], i);
  std::vector<int> ws;
  for (auto it = ordered.begin(); it != ordered.end() && ws.size() < nw; ++it) ws.push_back(int(it->second));
  std::sort(ws.begin(), ws.end());
  return ws;
}

}  // namespace detail

// ---- subspace problem solvers -------------------------------------------------------------------

class SubspaceSolver {
 public:
  virtual ~SubspaceSolver() = default;
  virtual void solve(const subspace::SubspaceData& data, size_t nroots_max) = 0;
  void set_error(int root, double e) { m_errors.at(root) = e; }
  void set_error(const std::vector<int>& roots, const std::vector<double>& e) {
    for (size_t i = 0; i < roots.size(); ++i) set_error(roots[i], e[i]);
  }
  const Matrix<double>& solutions() const { return m_solutions; }
  virtual const std::vector<double>& eigenvalues() const { return m_eigenvalues; }
  const std::vector<double>& errors() const { return m_errors; }
  size_t size() const { return m_solutions.rows(); }

 protected:
  Matrix<double> m_solutions;  // one row per root
  std::vector<double> m_eigenvalues;
  std::vector<double> m_errors;
};

// Dense eigenproblem (or linear equations when rhs is present) in the subspace.
class SubspaceSolverLinEig : public SubspaceSolver {
 public:
  explicit SubspaceSolverLinEig(std::shared_ptr<Logger> log) : m_logger(std::move(log)) {}
  void solve(const subspace::SubspaceData& data, size_t nroots_max) override {
    // reference SubspaceSolverLinEig.h:27-34: linear equations when a rhs block is present
    const auto rhs = data.find(EqnData::rhs);
    if (rhs != data.end() && !rhs->second.empty()) {
      solve_linear_equations(data);
      return;
    }
    const auto& h = data.at(EqnData::H);
    const auto& s = data.at(EqnData::S);
    const size_t dim = h.rows();
    std::vector<double> evec;
    eigenproblem(evec, m_eigenvalues, h.data(), s.data(), dim, m_hermitian, m_svd_solver_threshold, 0, true, nroots_max);
    const size_t nsol = dim ? evec.size() / dim : 0;
    const size_t nroots = std::min(nroots_max, nsol);
    m_eigenvalues.resize(nroots);
    m_solutions = Matrix<double>({nroots, dim});
    for (size_t k = 0; k < nroots; ++k)
      for (size_t j = 0; j < dim; ++j) m_solutions(k, j) = evec[j + dim * k];
    m_errors.assign(nroots, std::numeric_limits<double>::max());
    if (m_logger->data_dump) m_logger->msg("eigenvectors = " + as_string(m_solutions), Logger::Info);
  }
  // reference SubspaceSolverLinEig.h:62-85
  void solve_linear_equations(const subspace::SubspaceData& data) {
    const auto& h = data.at(EqnData::H);
    const auto& s = data.at(EqnData::S);
    const auto& rhs = data.at(EqnData::rhs);
    const size_t dim = h.rows(), nsol = rhs.cols();
    std::vector<double> solution;
    m_eigenvalues.assign(nsol, 0);
    solve_LinearEquations(solution, m_eigenvalues, h.data(), s.data(), rhs.data(), dim, nsol, m_augmented_hessian,
                          m_svd_solver_threshold, 0);
    m_solutions = Matrix<double>({nsol, dim});
    for (size_t r = 0; r < nsol; ++r)
      for (size_t k = 0; k < dim; ++k) m_solutions(r, k) = solution[k + dim * r];
    m_errors.assign(nsol, std::numeric_limits<double>::max());
  }
  void set_augmented_hessian(double a) { m_augmented_hessian = a; }
  double get_augmented_hessian() const { return m_augmented_hessian; }
  void set_hermiticity(bool h) { m_hermitian = h; }
  bool get_hermiticity() const { return m_hermitian; }
  double m_svd_solver_threshold = 1.0e-14;

 private:
  std::shared_ptr<Logger> m_logger;
  bool m_hermitian = false;
  double m_augmented_hessian = 0;
};

// Rayleigh-Schroedinger perturbation theory in the subspace (reference
// itsolv/subspace/SubspaceSolverRSPT.h:6-25): the variational subspace eigenproblem is solved (for
// eigenvalues()), then the solution is the unit vector on the first Q parameter.
class SubspaceSolverRSPT : public SubspaceSolverLinEig {
 public:
  using SubspaceSolverLinEig::SubspaceSolverLinEig;
  void solve(const subspace::SubspaceData& data, size_t nroots_max) override {
    SubspaceSolverLinEig::solve(data, nroots_max);
    m_solutions.fill(0);
    m_solutions(0, 0) = 1;
  }
};

class SubspaceSolverDIIS : public SubspaceSolver {
 public:
  SubspaceSolverDIIS(std::shared_ptr<Logger> log, const bool& converged) : m_converged(converged), m_logger(std::move(log)) {}
  void solve(const subspace::SubspaceData& data, size_t) override {
    const auto& kH = data.at(EqnData::H);
    const size_t dim = kH.rows();
    m_solutions = Matrix<double>({1, dim});
    if (m_converged) {
      m_solutions.fill(0);
      if (dim) m_solutions(0, 0) = 1;
      return;
    }
    std::vector<double> matrix;
    matrix.reserve(dim * dim);
    for (size_t i = 0; i < dim; ++i)
      for (size_t j = 0; j < dim; ++j) matrix.push_back(kH(j, i));
    std::vector<double> sol(dim);
    solve_DIIS(sol, matrix, dim, 1e-10, 1);
    for (size_t i = 0; i < dim; ++i) m_solutions(0, i) = sol[i];
    m_errors.assign(1, dim ? kH(0, 0) : 0.0);
  }
  const std::vector<double>& eigenvalues() const override {
    throw std::logic_error("eigenvalues() not available in non-linear method");
  }

 private:
  const bool& m_converged;
  std::shared_ptr<Logger> m_logger;
};

// ---- the solver template ------------------------------------------------------------------------

template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class IterativeSolverTemplate {
 public:
  using value_type = typename R::value_type;
  using scalar_type = double;
  using VectorP = std::vector<value_type>;
  using fapply_on_p_type = std::function<void(const std::vector<VectorP>&, const CVecRef<P>&, const VecRef<R>&)>;

  virtual ~IterativeSolverTemplate() = default;
  IterativeSolverTemplate(const IterativeSolverTemplate&) = delete;

  virtual bool nonlinear() const = 0;

  // Consistency check of a Problem (reference IterativeSolverTemplate.h:420-473): for a non-linear
  // problem, the change of the value between test parameter sets against the mean residual dotted
  // with the step; for a linear one, that the action is linear under scaling by 10.
  bool test_problem(const Problem<R, P>& problem, R& v0, R& v1, int verbosity, double threshold) const {
    auto& h = *m_handlers;
    bool success = true;
    if (nonlinear()) {
      if (!problem.test_parameters(0, v0)) return true;
      const auto value0 = problem.residual(v0, v1);
      Q parameters0{h.qr().copy(v0)};
      Q residual0{h.qr().copy(v1)};
      for (unsigned int instance = 1; problem.test_parameters(instance, v0); ++instance) {
        const auto value1 = problem.residual(v0, v1);
        Q parameters1{h.qr().copy(v0)};
        Q residual1{h.qr().copy(v1)};
        h.rq().copy(v0, residual1);
        h.rr().scal(0.5, v0);
        h.rq().axpy(0.5, residual0, v0);
        h.rq().copy(v1, parameters1);
        h.rq().axpy(-1, parameters0, v1);
        const auto dv_analytic = h.rr().dot(v0, v1);
        success = success && std::abs(dv_analytic - (value1 - value0)) < threshold;
        if (verbosity > 0 || (verbosity > -1 && !success))
          std::cout << "{actual, extrapolated} value change: {" << value1 - value0 << ", " << dv_analytic << "}"
                    << std::endl;
      }
    } else {
      for (unsigned int instance = 0; problem.test_parameters(instance, v0); ++instance) {
        problem.action(cwrap_arg(v0), wrap_arg(v1));
        Q residual{h.qr().copy(v1)};
        const auto norm2_residual = std::sqrt(h.rr().dot(v1, v1));
        constexpr double scale_factor{10.0};
        h.rr().scal(scale_factor, v0);
        problem.action(cwrap_arg(v0), wrap_arg(v1));
        h.rq().axpy(-scale_factor, residual, v1);
        const auto norm2 = std::sqrt(h.rr().dot(v1, v1));
        success = success && std::abs(norm2 / norm2_residual) < threshold;
        if (verbosity > 0 || (verbosity > -1 && !success))
          std::cout << "Length of residual: " << norm2_residual << ", scaling defect: " << norm2 << std::endl;
      }
    }
    return success;
  }

  // Adds the working-set parameters and their actions (residuals for non-linear solvers) to the
  // subspace, solves it and returns the new working set in parameters / actions.
  virtual int add_vector(const VecRef<R>& parameters, const VecRef<R>& actions) {
    if (m_xspace->dimensions().nP != 0 && !m_apply_p)
      throw std::runtime_error("Solver contains P space but no valid apply_p function. Make sure add_p was called correctly.");
    const size_t nW = std::min(m_working_set.size(), parameters.size());
    auto cp = cwrap(parameters.begin(), parameters.begin() + nW);
    auto ca = cwrap(actions.begin(), actions.begin() + nW);
    m_stats->r_creations += int(nW);
    m_xspace->update_qspace(cp, ca);
    m_stats->q_creations += int(2 * nW);
    auto ws = solve_and_generate_working_set(parameters, actions);
    read_handler_counts(*m_stats, *m_handlers);
    m_end_iteration_needed = true;
    return int(ws);
  }
  int add_vector(std::vector<R>& parameters, std::vector<R>& actions) { return add_vector(wrap(parameters), wrap(actions)); }
  virtual int add_vector(R& parameters, R& actions, value_type value = 0) {
    return add_vector(wrap_arg(parameters), wrap_arg(actions));
  }

  size_t add_p(const CVecRef<P>& pparams, const std::vector<double>& pp_action_matrix, const VecRef<R>& parameters,
               const VecRef<R>& actions, fapply_on_p_type apply_p) {
    if (!pparams.empty() && pparams.size() < n_roots())
      throw std::runtime_error("P space must be empty or at least as large as number of roots sought");
    if (apply_p) m_apply_p = std::move(apply_p);
    m_xspace->update_pspace(pparams, pp_action_matrix);
    auto ws = solve_and_generate_working_set(parameters, actions);
    read_handler_counts(*m_stats, *m_handlers);
    return ws;
  }

  void solution(const std::vector<int>& roots, const VecRef<R>& parameters, const VecRef<R>& residual) {
    check_roots(roots, parameters.size());
    const auto& d = m_xspace->dimensions();
    detail::construct_solution(parameters, roots, m_subspace_solver->solutions(), m_xspace->cparamsp(),
                               m_xspace->cparamsq(), m_xspace->cparamsd(), d.oP, d.oQ, d.oD, *m_handlers);
    detail::construct_solution(residual, roots, m_subspace_solver->solutions(), CVecRef<P>{}, m_xspace->cactionsq(),
                               m_xspace->cactionsd(), d.oP, d.oQ, d.oD, *m_handlers);
    auto pvec = detail::construct_vectorP(roots, m_subspace_solver->solutions(), d.oP, d.nP);
    if (m_normalise_solution) detail::normalise_pairs(roots.size(), parameters, residual, m_handlers->rr(), *m_logger);
    if (m_apply_p) m_apply_p(pvec, m_xspace->cparamsp(), residual);
    construct_residual(roots, cwrap(parameters), residual);
    read_handler_counts(*m_stats, *m_handlers);
  }
  void solution(const std::vector<int>& roots, std::vector<R>& parameters, std::vector<R>& residual) {
    solution(roots, wrap(parameters), wrap(residual));
  }
  void solution(R& parameters, R& residual) { solution(std::vector<int>(1, 0), wrap_arg(parameters), wrap_arg(residual)); }

  void solution_params(const std::vector<int>& roots, const VecRef<R>& parameters) {
    check_roots(roots, parameters.size());
    const auto& d = m_xspace->dimensions();
    detail::construct_solution(parameters, roots, m_subspace_solver->solutions(), m_xspace->cparamsp(),
                               m_xspace->cparamsq(), m_xspace->cparamsd(), d.oP, d.oQ, d.oD, *m_handlers);
  }

  virtual size_t end_iteration(const VecRef<R>& parameters, const VecRef<R>& actions) = 0;
  size_t end_iteration(std::vector<R>& parameters, std::vector<R>& actions) {
    return end_iteration(wrap(parameters), wrap(actions));
  }
  size_t end_iteration(R& parameters, R& actions) { return end_iteration(wrap_arg(parameters), wrap_arg(actions)); }
  bool end_iteration_needed() const { return m_end_iteration_needed; }

  const std::vector<int>& working_set() const { return m_working_set; }
  virtual std::vector<double> working_set_eigenvalues() const { return std::vector<double>(m_working_set.size(), 0); }
  size_t n_roots() const { return m_nroots; }
  void set_n_roots(size_t n) {
    m_nroots = n;
    m_working_set.resize(n);
    std::iota(m_working_set.begin(), m_working_set.end(), 0);
  }
  const std::vector<double>& errors() const { return m_errors; }
  const Statistics& statistics() const { return *m_stats; }
  const subspace::Dimensions& dimensions() const { return m_xspace->dimensions(); }
  //! Latest function value of an Optimize solver, NaN otherwise (reference IterativeSolverTemplate.h:312-315)
  double value() const {
    const auto it = m_xspace->data.find(EqnData::value);
    return it != m_xspace->data.end() && !it->second.empty() ? it->second(0, 0)
                                                               : std::nan("molpro::linalg::itsolv::IterativeSolver::value");
  }
  void set_convergence_threshold(double t) { m_convergence_threshold = t; }
  double convergence_threshold() const { return m_convergence_threshold; }
  void set_convergence_threshold_value(double t) { m_convergence_threshold_value = t; }
  void set_verbosity(Verbosity v) { m_verbosity = v; }
  Verbosity get_verbosity() const { return m_verbosity; }
  void set_max_iter(int n) { m_max_iter = n; }
  int get_max_iter() const { return m_max_iter; }
  void set_max_p(int n) { m_max_p = size_t(n); }
  int get_max_p() const { return int(m_max_p); }
  void set_p_threshold(double t) { m_p_threshold = t; }
  double get_p_threshold() const { return m_p_threshold; }
  std::shared_ptr<Logger> logger() const { return m_logger; }
  subspace::XSpace<R, Q, P>& xspace() { return *m_xspace; }

  //! The current settings (reference IterativeSolverTemplate.h:262-267; derived solvers add theirs).
  virtual std::shared_ptr<Options> get_options() const {
    auto o = std::make_shared<Options>();
    o->n_roots = int(n_roots());
    o->convergence_threshold = convergence_threshold();
    return o;
  }

  virtual void set_options(const Options& o) {
    if (o.n_roots) set_n_roots(size_t(*o.n_roots));
    if (o.convergence_threshold) set_convergence_threshold(*o.convergence_threshold);
    if (o.verbosity) set_verbosity(*o.verbosity);
    if (o.max_iter) set_max_iter(*o.max_iter);
    if (o.max_p) set_max_p(int(*o.max_p));
    if (o.p_threshold) set_p_threshold(*o.p_threshold);
  }

  // One-call driver (reference IterativeSolverTemplate.h:322-408).
  bool solve(const VecRef<R>& parameters, const VecRef<R>& actions, const Problem<R, P>& problem,
             bool generate_initial_guess = false) {
    if (parameters.empty()) throw std::runtime_error("Empty container passed to IterativeSolver::solve()");
    if (parameters.size() != actions.size()) throw std::runtime_error("Inconsistent container sizes in IterativeSolver::solve()");
    const bool use_diagonals = problem.diagonals(actions.at(0));
    std::unique_ptr<Q> diagonals;
    if (use_diagonals) diagonals = std::make_unique<Q>(m_handlers->qr().copy(actions.at(0)));
    if (generate_initial_guess) {
      if (!use_diagonals) throw std::runtime_error("Default initial guess requested, but diagonal elements are not available");
      auto guess = m_handlers->qq().select(parameters.size(), *diagonals);
      size_t root = 0;
      for (const auto& g : guess) m_handlers->rp().copy(parameters[root++], P{{g.first, 1}});
    }
    int nwork = int(parameters.size());
    std::vector<P> pspace;
    if (use_diagonals && m_max_p > 0) {
      auto selectp = m_handlers->qq().select(m_max_p, *diagonals);
      for (auto s = selectp.begin(); s != selectp.end(); ++s)
        if (s->second > selectp.begin()->second + m_p_threshold) {
          selectp.erase(s, selectp.end());
          break;
        }
      for (const auto& s : selectp) pspace.push_back(P{{s.first, 1}});
      fapply_on_p_type apply = [&problem](const std::vector<VectorP>& c, const CVecRef<P>& pp, const VecRef<R>& a) {
        problem.p_action(c, pp, a);
      };
      auto ppm = problem.pp_action_matrix(pspace);
      nwork = int(add_p(cwrap(pspace), ppm, parameters, actions, apply));
    }
    for (int iter = 0; iter < m_max_iter && nwork > 0; ++iter) {
      if (nonlinear()) {
        const auto value = problem.residual(parameters.front(), actions.front());
        nwork = add_vector(parameters.front().get(), actions.front().get(), value);
      } else if (iter > 0 || pspace.empty()) {
        problem.action(cwrap(parameters.begin(), parameters.begin() + nwork), wrap(actions.begin(), actions.begin() + nwork));
        nwork = add_vector(parameters, actions);
      }
      while (end_iteration_needed()) {
        if (nwork > 0) {
          if (use_diagonals) {
            m_handlers->rq().copy(parameters.at(0), *diagonals);
            problem.precondition(wrap(actions.begin(), actions.begin() + nwork), working_set_eigenvalues(),
                                 parameters.at(0));
          } else {
            problem.precondition(wrap(actions.begin(), actions.begin() + nwork), working_set_eigenvalues());
          }
        }
        nwork = int(end_iteration(parameters, actions));
      }
      if (iteration_hook) iteration_hook();
      if (m_verbosity >= Verbosity::Iteration) report();
    }
    const double emax = m_errors.empty() ? 0 : *std::max_element(m_errors.begin(), m_errors.end());
    return nwork == 0 && emax <= m_convergence_threshold;
  }
  bool solve(std::vector<R>& parameters, std::vector<R>& actions, const Problem<R, P>& problem,
             bool generate_initial_guess = false) {
    return solve(wrap(parameters), wrap(actions), problem, generate_initial_guess);
  }
  bool solve(R& parameters, R& actions, const Problem<R, P>& problem, bool generate_initial_guess = false) {
    return solve(wrap_arg(parameters), wrap_arg(actions), problem, generate_initial_guess);
  }

  //! Called after every iteration of solve() (measurement / tracing; not part of the reference API).
  std::function<void()> iteration_hook;

  virtual void report(std::ostream& o = std::cout) const {
    o << "iteration " << m_stats->iterations;
    if (!m_errors.empty()) {
      auto it = std::max_element(m_errors.begin(), m_errors.end());
      o << (n_roots() > 1 ? ", |residual[" + std::to_string(it - m_errors.begin()) + "]| = " : ", |residual| = ")
        << std::scientific << *it << std::defaultfloat;
    }
    o << std::endl;
  }

 protected:
  IterativeSolverTemplate(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers, std::shared_ptr<SubspaceSolver> ss,
                          std::shared_ptr<Logger> logger)
      : m_handlers(std::move(handlers)),
        m_xspace(std::make_shared<subspace::XSpace<R, Q, P>>(m_handlers, logger)),
        m_subspace_solver(std::move(ss)),
        m_stats(std::make_shared<Statistics>()),
        m_logger(std::move(logger)) {
    set_n_roots(1);
  }

  virtual void set_value_errors() {}
  virtual void construct_residual(const std::vector<int>& roots, const CVecRef<R>& params, const VecRef<R>& actions) = 0;

  // reference IterativeSolverTemplate.h:518-563
  size_t solve_and_generate_working_set(const VecRef<R>& parameters, const VecRef<R>& action) {
    m_subspace_solver->solve(m_xspace->data, n_roots());
    const size_t nsol = m_subspace_solver->size();
    std::vector<std::pair<Q, Q>> temp;
    const auto batches = detail::parameter_batches(nsol, parameters.size());
    for (const auto& [s0, s1] : batches) {
      std::vector<int> roots(s1 - s0);
      std::iota(roots.begin(), roots.end(), int(s0));
      m_residual_norms2.clear();
      solution(roots, parameters, action);
      std::vector<double> errors(roots.size(), 0);
      if (m_residual_norms2.size() == roots.size()) {  // from a fused construct_residual
        for (size_t i = 0; i < errors.size(); ++i) errors[i] = std::sqrt(std::abs(m_residual_norms2[i]));
        m_handlers->rr().count_replaced(0, int(roots.size()), 0);  // update_errors' self-dots
      } else {
        detail::update_errors(errors, cwrap(action), m_handlers->rr());
      }
      m_residual_norms2.clear();
      if (batches.size() > 1) {
        for (size_t i = 0; i < roots.size(); ++i)
          temp.emplace_back(m_handlers->qr().copy(parameters[i]), m_handlers->qr().copy(action[i]));
        m_stats->q_creations += int(2 * roots.size());
      }
      m_subspace_solver->set_error(roots, errors);
    }
    set_value_errors();
    m_errors = m_subspace_solver->errors();
    m_working_set = detail::select_working_set(parameters.size(), m_errors, m_convergence_threshold, m_value_errors,
                                               m_convergence_threshold_value);
    for (size_t i = 0; i < m_working_set.size(); ++i) {
      const size_t root = size_t(m_working_set[i]);
      if (batches.size() > 1) {
        m_handlers->rq().copy(parameters[i], temp.at(root).first);
        m_handlers->rq().copy(action[i], temp.at(root).second);
      } else {
        if (root < i) throw std::logic_error("incorrect ordering of roots");
        if (root > i) {
          m_handlers->rr().copy(parameters[i], parameters[root]);
          m_handlers->rr().copy(action[i], action[root]);
        }
      }
    }
    return m_working_set.size();
  }

  void check_roots(const std::vector<int>& roots, size_t nparams) const {
    if (roots.size() > nparams) throw std::runtime_error("asking for more roots than parameters");
    if (!roots.empty() && size_t(*std::max_element(roots.begin(), roots.end())) >= m_subspace_solver->solutions().rows())
      throw std::runtime_error("asking for more roots than there are solutions");
  }

  std::shared_ptr<ArrayHandlers<R, Q, P>> m_handlers;
  std::shared_ptr<subspace::XSpace<R, Q, P>> m_xspace;
  std::shared_ptr<SubspaceSolver> m_subspace_solver;
  std::shared_ptr<Statistics> m_stats;
  std::shared_ptr<Logger> m_logger;
  std::vector<double> m_errors, m_value_errors;
  std::vector<double> m_residual_norms2;  // <r_i, r_i> left by a fused construct_residual (solution())
  std::vector<int> m_working_set;
  size_t m_nroots = 0;
  double m_convergence_threshold = 1.0e-8;
  double m_convergence_threshold_value = std::numeric_limits<double>::max();
  bool m_normalise_solution = false;
  fapply_on_p_type m_apply_p{};
  Verbosity m_verbosity = Verbosity::Iteration;
  int m_max_iter = 100;
  size_t m_max_p = 0;
  double m_p_threshold = std::numeric_limits<double>::max();
  bool m_end_iteration_needed = true;
};

// ---- Davidson ----------------------------------------------------------------------------------

// What LinearEigensystemDavidson and LinearEquationsDavidson share (reference
// LinearEigensystemDavidson.h:63-83 and LinearEquationsDavidson.h:48-62 have the same end_iteration,
// both over detail::propose_rspace, propose_rspace.h:553-624, and the DSpaceResetter).
template <class R, class Q, class P>
class DavidsonSolver : public IterativeSolverTemplate<R, Q, P> {
  using Base = IterativeSolverTemplate<R, Q, P>;

 public:
  DavidsonSolver(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers, std::shared_ptr<Logger> logger)
      : Base(std::move(handlers), std::make_shared<SubspaceSolverLinEig>(logger), logger) {
    this->m_normalise_solution = false;
  }

  bool nonlinear() const override { return false; }

  size_t end_iteration(const VecRef<R>& parameters, const VecRef<R>& action) override {
    if (m_resetter.do_reset(size_t(this->m_stats->iterations), this->m_xspace->dimensions())) {
      m_resetting = true;
      this->m_working_set = m_resetter.run(parameters, *this->m_xspace, this->m_subspace_solver->solutions(),
                                           norm_thresh, svd_thresh, *this->m_handlers, *this->m_logger);
    } else {
      m_resetting = false;
      this->m_working_set = propose_rspace(parameters, action);
    }
    this->m_stats->iterations++;
    read_handler_counts(*this->m_stats, *this->m_handlers);
    this->m_end_iteration_needed = false;
    return this->m_working_set.size();
  }
  using Base::end_iteration;

  void set_reset_D(size_t n) { m_resetter.set_nreset(n); }
  int get_reset_D() const { return m_resetter.get_nreset(); }
  void set_reset_D_maxQ_size(size_t n) { m_resetter.set_max_Qsize(n); }
  int get_reset_D_maxQ_size() const { return m_resetter.get_max_Qsize(); }
  int get_max_size_qspace() const { return m_max_size_qspace; }
  void set_max_size_qspace(int n) {
    m_max_size_qspace = n;
    if (m_resetter.get_max_Qsize() > m_max_size_qspace) m_resetter.set_max_Qsize(size_t(m_max_size_qspace));
  }
  void set_hermiticity(bool h) {
    m_hermiticity = h;
    this->m_xspace->set_hermiticity(h);
    subspace_solver().set_hermiticity(h);
  }
  bool get_hermiticity() const { return m_hermiticity; }

  double norm_thresh = 1e-10;  // propose_rspace_norm_thresh
  double svd_thresh = 1e-12;   // propose_rspace_svd_thresh

 protected:
  SubspaceSolverLinEig& subspace_solver() { return static_cast<SubspaceSolverLinEig&>(*this->m_subspace_solver); }

  template <class O>
  std::shared_ptr<O> davidson_options() const {
    auto o = std::make_shared<O>();
    o->copy(*Base::get_options());
    o->reset_D = get_reset_D();
    o->reset_D_max_Q_size = get_reset_D_maxQ_size();
    o->max_size_qspace = get_max_size_qspace();
    o->norm_thresh = norm_thresh;
    o->svd_thresh = svd_thresh;
    o->hermiticity = get_hermiticity();
    o->block_gram_schmidt = m_block_gram_schmidt;
    return o;
  }

  template <class O>
  void set_davidson_options(const O& d) {
    if (d.reset_D) set_reset_D(size_t(*d.reset_D));
    if (d.reset_D_max_Q_size) set_reset_D_maxQ_size(size_t(*d.reset_D_max_Q_size));
    if (d.max_size_qspace) set_max_size_qspace(*d.max_size_qspace);
    if (d.norm_thresh) norm_thresh = *d.norm_thresh;
    if (d.svd_thresh) svd_thresh = *d.svd_thresh;
    if (d.hermiticity) set_hermiticity(*d.hermiticity);
    if (d.block_gram_schmidt) m_block_gram_schmidt = *d.block_gram_schmidt;
  }

 public:
  void set_block_gram_schmidt(bool on) { m_block_gram_schmidt = on; }
  //! The option as set (unset: the R type's default for the vectors' length, block_gram_schmidt_default).
  std::optional<bool> block_gram_schmidt() const { return m_block_gram_schmidt; }

 protected:
  // reference propose_rspace.h:553-624
  std::vector<int> propose_rspace(const VecRef<R>& parameters, const VecRef<R>& residuals) {
    auto& xs = *this->m_xspace;
    auto& ss = *this->m_subspace_solver;
    auto& h = *this->m_handlers;
    auto& log = *this->m_logger;
    const auto solutions = ss.solutions();
    auto q_delete = detail::limit_qspace_size(xs.dimensions(), size_t(m_max_size_qspace), solutions, log);
    if (!q_delete.empty()) {
      auto [dp, da] = detail::construct_dspace(solutions, xs, q_delete, norm_thresh, svd_thresh, h.qq(), log);
      std::sort(q_delete.begin(), q_delete.end(), std::greater<int>());
      for (int iq : q_delete) xs.eraseq(size_t(iq));
      auto wdp = wrap(dp);
      auto wda = wrap(da);
      xs.update_dspace(wdp, wda);
      ss.solve(xs.data, solutions.rows());
    }
    auto wres = wrap(residuals.begin(), residuals.begin() + this->working_set().size());
    detail::normalise(wres, h.rr(), log);
    const auto full = detail::append_overlap_with_r(xs.data.at(EqnData::S), cwrap(wres), xs.cparamsp(), xs.cparamsq(),
                                                    xs.cparamsd(), h);
    auto redundant = detail::redundant_parameters(full, xs.dimensions().nX, wres.size(), svd_thresh, log);
    std::vector<size_t> rows(wres.size());
    std::iota(rows.begin(), rows.end(), xs.dimensions().nX);
    detail::delete_parameters(redundant, wres);
    detail::delete_parameters(redundant, rows);
    const bool block_gs = m_block_gram_schmidt.value_or(
        array::block_gram_schmidt_default<R>::for_length(wres.empty() ? 0 : wres.front().get().size()));
    auto null_params =
        block_gs
            ? detail::block_gram_schmidt(wres, full, rows, xs.dimensions(), xs.cparamsp(), xs.cparamsq(),
                                         xs.cparamsd(), norm_thresh, h)
            : detail::modified_gram_schmidt(wres, xs.data.at(EqnData::S), xs.dimensions(), xs.cparamsp(),
                                            xs.cparamsq(), xs.cparamsd(), norm_thresh, h);
    detail::delete_parameters(null_params, wres);
    this->m_stats->redundant_params += int(redundant.size());
    this->m_stats->null_params += int(null_params.size());
    detail::normalise(wres, h.rr(), log);
    for (size_t i = 0; i < wres.size(); ++i) h.rr().copy(parameters.at(i), wres.at(i));
    return detail::get_new_working_set(this->working_set(), cwrap(residuals), cwrap(wres));
  }

  int m_max_size_qspace = std::numeric_limits<int>::max();
  detail::DSpaceResetter<Q> m_resetter;
  bool m_hermiticity = false;
  bool m_resetting = false;
  std::optional<bool> m_block_gram_schmidt;
};

template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class LinearEigensystemDavidson : public DavidsonSolver<R, Q, P> {
  using Base = DavidsonSolver<R, Q, P>;

 public:
  explicit LinearEigensystemDavidson(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers,
                                     std::shared_ptr<Logger> logger = std::make_shared<Logger>())
      : Base(std::move(handlers), std::move(logger)) {
    this->set_hermiticity(this->m_hermiticity);
  }

  std::vector<double> eigenvalues() const { return this->m_subspace_solver->eigenvalues(); }
  std::vector<double> working_set_eigenvalues() const override {
    std::vector<double> e;
    for (auto i : this->working_set()) e.push_back(this->m_subspace_solver->eigenvalues().at(i));
    return e;
  }

  void set_options(const Options& o) override {
    Base::set_options(o);
    if (auto* d = dynamic_cast<const LinearEigensystemDavidsonOptions*>(&o)) this->set_davidson_options(*d);
  }
  //! reference LinearEigensystemDavidson.h:168-178
  std::shared_ptr<Options> get_options() const override {
    return this->template davidson_options<LinearEigensystemDavidsonOptions>();
  }

 protected:
  void set_value_errors() override {
    const auto cur = this->m_subspace_solver->eigenvalues();
    this->m_value_errors.assign(cur.size(), std::numeric_limits<double>::max());
    for (size_t i = 0; i < std::min(m_last_values.size(), cur.size()); ++i)
      this->m_value_errors[i] = std::abs(cur[i] - m_last_values[i]);
    if (!this->m_resetting) m_last_values = cur;
  }

  // r_i -= lambda_i x_i (reference LinearEigensystemDavidson.h:186-192); where the handler fuses the
  // axpys with the residual norms (array::fused_residual_norms), the norms are kept for
  // solve_and_generate_working_set's update_errors instead of being read back in a second pass.
  void construct_residual(const std::vector<int>& roots, const CVecRef<R>& params, const VecRef<R>& actions) override {
    const auto& ev = eigenvalues();
    std::vector<double> c(roots.size());
    for (size_t i = 0; i < roots.size(); ++i) c[i] = -ev.at(roots[i]);
    using array::fused_residual_norms;
    if (fused_residual_norms(this->m_handlers->rr(), c, params, VecRef<R>(actions.begin(), actions.begin() + long(roots.size())),
                             this->m_residual_norms2)) {
      this->m_handlers->rr().count_replaced(int(roots.size()), 0, 0);  // the axpys it replaced
      return;
    }
    for (size_t i = 0; i < roots.size(); ++i) this->m_handlers->rr().axpy(c[i], params.at(i), actions.at(i));
  }

  std::vector<double> m_last_values;
};

// Lowest eigenvalue by Rayleigh-Schroedinger perturbation theory (reference
// itsolv/LinearEigensystemRSPT.h:32-198).  The caller's loop (test_RSPT.cpp:105-128) adds x = psi(k)
// and g = H psi(k); construct_residual appends E(k+1) = <psi(0), H psi(k)> to the perturbation series
// and forms g = H psi(k) - E(0..) psi(..) from the stored Q parameters (q(j) holds psi(n-j-1)); after
// the caller's preconditioner end_iteration makes the next correction x = -g (the first one from
// x = 0).  One root, hermitian, unnormalised solutions.
template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class LinearEigensystemRSPT : public IterativeSolverTemplate<R, Q, P> {
  using Base = IterativeSolverTemplate<R, Q, P>;

 public:
  explicit LinearEigensystemRSPT(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers,
                                 std::shared_ptr<Logger> logger = std::make_shared<Logger>())
      : Base(std::move(handlers), std::make_shared<SubspaceSolverRSPT>(logger), logger) {
    set_hermiticity(true);
    this->set_n_roots(1);
    this->m_normalise_solution = false;
  }

  bool nonlinear() const override { return false; }

  // reference LinearEigensystemRSPT.h:74-81
  size_t end_iteration(const VecRef<R>& parameters, const VecRef<R>& actions) override {
    R& x = parameters.front().get();
    R& g = actions.front().get();
    if (this->m_xspace->size() == 1) this->m_handlers->rr().fill(0, x);
    this->m_handlers->rr().axpy(-1, g, x);
    this->m_end_iteration_needed = false;
    return this->m_errors.front() < this->m_convergence_threshold ? 0 : 1;
  }
  using Base::end_iteration;

  std::vector<double> eigenvalues() const { return this->m_subspace_solver->eigenvalues(); }
  std::vector<double> working_set_eigenvalues() const override {
    std::vector<double> e;
    for (auto i : this->working_set()) e.push_back(this->m_subspace_solver->eigenvalues().at(i));
    return e;
  }
  //! The perturbation series: element k (k >= 1) is the k-th order energy contribution, with
  //! element 1 = E(0) + E(1) = <psi(0)|H|psi(0)>; element 0 is 0 (LinearEigensystemRSPT.h:175-179).
  const std::vector<double>& rspt_values() const { return m_rspt_values; }

  void set_hermiticity(bool hermitian) {
    this->m_xspace->set_hermiticity(hermitian);
    std::static_pointer_cast<SubspaceSolverRSPT>(this->m_subspace_solver)->set_hermiticity(hermitian);
  }
  bool get_hermiticity() const { return true; }

  //! reference LinearEigensystemRSPT.h:139-151 (options norm_thresh / svd_thresh)
  void set_options(const Options& o) override {
    Base::set_options(o);
    if (auto* r = dynamic_cast<const LinearEigensystemRSPTOptions*>(&o)) {
      if (r->norm_thresh) propose_rspace_norm_thresh = *r->norm_thresh;
      if (r->svd_thresh) propose_rspace_svd_thresh = *r->svd_thresh;
    }
  }
  std::shared_ptr<Options> get_options() const override {
    auto o = std::make_shared<LinearEigensystemRSPTOptions>();
    o->copy(*Base::get_options());
    o->norm_thresh = propose_rspace_norm_thresh;
    o->svd_thresh = propose_rspace_svd_thresh;
    return o;
  }
  double propose_rspace_norm_thresh = 1e-10;
  double propose_rspace_svd_thresh = 1e-12;

  void report(std::ostream& o = std::cout) const override {
    o << "Perturbed energies " << std::fixed << std::setprecision(8);
    for (double e : m_rspt_values) o << e << ", ";
    o << std::defaultfloat << std::endl;
  }

 protected:
  // reference LinearEigensystemRSPT.h:163-190
  void construct_residual(const std::vector<int>&, const CVecRef<R>& params, const VecRef<R>& actions) override {
    const auto q = this->m_xspace->cparamsq();
    const size_t n = q.size();
    const R& c = params.back().get();
    R& hc = actions.back().get();
    if (n == 1) m_rspt_values.assign(1, 0);
    m_rspt_values.push_back(this->m_handlers->qr().dot(q.at(n - 1).get(), hc));
    this->m_handlers->rr().axpy(-m_rspt_values[0], c, hc);
    for (size_t k = 0; k < n; ++k) this->m_handlers->rq().axpy(-m_rspt_values[n - k], q.at(n - k - 1).get(), hc);
  }

  std::vector<double> m_rspt_values;
};

// A x = b for several right-hand sides in the same Krylov/P/D subspace machinery
// (reference LinearEquationsDavidson.h:27-191).  Residuals are scaled by 1/|b| (:175-186).
template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class LinearEquationsDavidson : public DavidsonSolver<R, Q, P> {
  using Base = DavidsonSolver<R, Q, P>;

 public:
  explicit LinearEquationsDavidson(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers,
                                   std::shared_ptr<Logger> logger = std::make_shared<Logger>())
      : Base(std::move(handlers), std::move(logger)) {
    this->set_hermiticity(true);  // reference LinearEquationsDavidson.h:189 (m_hermiticity = true)
  }

  // reference :73-78
  void add_equations(const CVecRef<R>& rhs) {
    this->m_xspace->add_rhs_equations(rhs);
    this->set_n_roots(this->m_xspace->dimensions().nRHS);
  }
  void add_equations(const R& rhs) { add_equations(cwrap_arg(rhs)); }
  void add_equations(const std::vector<R>& rhs) { add_equations(cwrap(rhs)); }
  CVecRef<Q> rhs() const { return this->m_xspace->rhs(); }

  //! Augmented-Hessian parameter of the subspace solve; 0 = plain linear equations (reference :119-127)
  void set_augmented_hessian(double a) { this->subspace_solver().set_augmented_hessian(a); }
  double get_augmented_hessian() { return this->subspace_solver().get_augmented_hessian(); }

  void set_options(const Options& o) override {
    Base::set_options(o);
    if (auto* d = dynamic_cast<const LinearEquationsDavidsonOptions*>(&o)) {
      this->set_davidson_options(*d);
      if (d->augmented_hessian) set_augmented_hessian(*d->augmented_hessian);
    }
  }
  //! reference LinearEquationsDavidson.h:147-158
  std::shared_ptr<Options> get_options() const override {
    auto o = this->template davidson_options<LinearEquationsDavidsonOptions>();
    o->augmented_hessian = const_cast<LinearEquationsDavidson*>(this)->get_augmented_hessian();
    return o;
  }

 protected:
  // r_i = (A x_i - b_i) / |b_i| (reference :175-186)
  void construct_residual(const std::vector<int>& roots, const CVecRef<R>& params, const VecRef<R>& actions) override {
    const auto& norm = this->m_xspace->rhs_norm();
    for (size_t i = 0; i < roots.size(); ++i) {
      const auto ii = size_t(roots[i]);
      this->m_handlers->rq().axpy(-1, rhs().at(ii), actions.at(i));
      if (norm.at(ii) != 0) this->m_handlers->rr().scal(1 / norm[ii], actions.at(i));
    }
  }
};

// ---- DIIS --------------------------------------------------------------------------------------

template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class NonLinearEquationsDIIS : public IterativeSolverTemplate<R, Q, P> {
  using Base = IterativeSolverTemplate<R, Q, P>;

 public:
  using typename Base::value_type;
  explicit NonLinearEquationsDIIS(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers,
                                  std::shared_ptr<Logger> logger = std::make_shared<Logger>())
      : Base(std::move(handlers), std::make_shared<SubspaceSolverDIIS>(logger, m_converged), logger) {
    this->m_xspace->set_hermiticity(true);
    this->m_xspace->set_action_action();
  }

  bool nonlinear() const override { return true; }

  // reference NonLinearEquationsDIIS.h:285-304
  int add_vector(R& parameters, R& residual, value_type value = 0) override {
    const double error = std::sqrt(this->m_handlers->rr().dot(residual, residual));
    m_converged = error < this->m_convergence_threshold;
    auto& xs = *this->m_xspace;
    for (auto del = least_important_vector(xs.data[EqnData::H]);
         xs.size() >= size_t(m_max_size_qspace) || del.second < m_svd_thresh;
         del = least_important_vector(xs.data[EqnData::H]))
      xs.eraseq(del.first);
    const int nwork = Base::add_vector(wrap_arg(parameters), wrap_arg(residual));
    this->m_errors.front() = error;
    return nwork;
  }
  using Base::add_vector;

  // reference NonLinearEquationsDIIS.h:305-321
  size_t end_iteration(const VecRef<R>& parameters, const VecRef<R>& action) override {
    this->solution_params(this->m_working_set, parameters);
    this->m_end_iteration_needed = false;
    if (this->m_errors.front() < this->m_convergence_threshold) {
      this->m_working_set.clear();
      return 0;
    }
    this->m_working_set.assign(1, 0);
    this->m_handlers->rr().axpy(-1, action.front(), parameters.front());
    this->m_stats->iterations++;
    return 1;
  }
  using Base::end_iteration;

  void set_norm_thresh(double t) { m_norm_thresh = t; }
  void set_svd_thresh(double t) { m_svd_thresh = t; }
  void set_max_size_qspace(int n) { m_max_size_qspace = n; }
  int get_max_size_qspace() const { return m_max_size_qspace; }

  void set_options(const Options& o) override {
    Base::set_options(o);
    if (auto* d = dynamic_cast<const NonLinearEquationsDIISOptions*>(&o)) {
      if (d->max_size_qspace) set_max_size_qspace(*d->max_size_qspace);
      if (d->norm_thresh) set_norm_thresh(*d->norm_thresh);
      if (d->svd_thresh) set_svd_thresh(*d->svd_thresh);
    }
  }
  //! reference NonLinearEquationsDIIS.h:150-157
  std::shared_ptr<Options> get_options() const override {
    auto o = std::make_shared<NonLinearEquationsDIISOptions>();
    o->copy(*Base::get_options());
    o->max_size_qspace = m_max_size_qspace;
    o->norm_thresh = m_norm_thresh;
    o->svd_thresh = m_svd_thresh;
    return o;
  }

 protected:
  void construct_residual(const std::vector<int>&, const CVecRef<R>&, const VecRef<R>&) override {}

  // reference NonLinearEquationsDIIS.h:254-282
  std::pair<size_t, double> least_important_vector(const Matrix<double>& H) const {
    std::pair<size_t, double> result{0, std::numeric_limits<double>::max()};
    const size_t n = H.cols();
    if (n < 2) return result;
    std::vector<double> ev, vec;
    dense::sym_eigen(n, H.data(), ev, vec);
    double evmax = 0;
    for (size_t i = 0; i < n; ++i) {
      evmax = std::max(evmax, ev[i]);
      if (ev[i] < result.second) {
        result.second = ev[i];
        result.first = 1;
        for (size_t j = 1; j < n; ++j)
          if (std::abs(vec[j + n * i]) > std::abs(vec[result.first + n * i])) result.first = j;
      }
    }
    result.second /= evmax;
    if (result.second > m_svd_thresh) result = {n - 1, std::numeric_limits<double>::max()};
    return result;
  }

  bool m_converged = false;
  double m_norm_thresh = 1e-10;
  double m_svd_thresh = 1e-12;
  int m_max_size_qspace = std::numeric_limits<int>::max();
};

// ---- Optimize ------------------------------------------------------------------------------------

// Subspace "solution" of the optimisers: the latest point (reference SubspaceSolverOptBFGS.h:27-46,
// SubspaceSolverOptSD.h); the step itself is formed in end_iteration.
class SubspaceSolverOptLatest : public SubspaceSolver {
 public:
  void solve(const subspace::SubspaceData& data, size_t) override {
    const size_t dim = data.at(EqnData::H).rows();
    m_solutions = Matrix<double>({1, dim});
    m_solutions.fill(0);
    if (dim) m_solutions(0, 0) = 1;
    m_errors.assign(1, dim ? data.at(EqnData::H)(0, 0) : 0.0);
  }
  const std::vector<double>& eigenvalues() const override {
    throw std::logic_error("eigenvalues() not available in non-linear method");
  }
};

template <class R, class Q, class P>
class OptimizeSolver : public IterativeSolverTemplate<R, Q, P> {
  using Base = IterativeSolverTemplate<R, Q, P>;

 public:
  OptimizeSolver(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers, std::shared_ptr<Logger> logger)
      : Base(std::move(handlers), std::make_shared<SubspaceSolverOptLatest>(), std::move(logger)) {}
  bool nonlinear() const override { return true; }

 protected:
  // reference OptimizeBFGS.h:208-213, OptimizeSD.h:57-62
  void set_value_errors() override {
    auto& v = this->m_xspace->data[EqnData::value];
    this->m_value_errors.assign(1, std::numeric_limits<double>::max());
    if (this->m_xspace->size() > 1 && v(0, 0) < v(1, 0)) this->m_value_errors.front() = v(1, 0) - v(0, 0);
  }
  void construct_residual(const std::vector<int>&, const CVecRef<R>&, const VecRef<R>&) override {}
};

// Steepest descent with the caller's preconditioner (reference itsolv/OptimizeSD.h:20-104).
template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class OptimizeSD : public OptimizeSolver<R, Q, P> {
  using Base = OptimizeSolver<R, Q, P>;

 public:
  explicit OptimizeSD(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers,
                      std::shared_ptr<Logger> logger = std::make_shared<Logger>())
      : Base(std::move(handlers), std::move(logger)) {}

  int add_vector(R& parameters, R& residual, double value) override {
    auto& v = this->m_xspace->data[EqnData::value];
    v.resize({this->m_xspace->dimensions().nX + 1, 1});
    v(0, 0) = value;
    return IterativeSolverTemplate<R, Q, P>::add_vector(wrap_arg(parameters), wrap_arg(residual));
  }
  using Base::add_vector;

  size_t end_iteration(const VecRef<R>& parameters, const VecRef<R>& action) override {
    this->solution_params(this->m_working_set, parameters);
    this->m_end_iteration_needed = false;
    if (this->m_errors.front() < this->m_convergence_threshold) {
      this->m_working_set.clear();
      return 0;
    }
    this->m_working_set.assign(1, 0);
    this->m_handlers->rr().axpy(-1, action.front(), parameters.front());
    this->m_stats->iterations++;
    return 1;
  }
  using Base::end_iteration;

  //! reference OptimizeSD.h:70-74
  std::shared_ptr<Options> get_options() const override {
    auto o = std::make_shared<OptimizeSDOptions>();
    o->copy(*IterativeSolverTemplate<R, Q, P>::get_options());
    return o;
  }
};

// Limited-memory quasi-Newton (BFGS two-loop recursion over the Q space) with a cubic line search
// under the Wolfe conditions (reference itsolv/OptimizeBFGS.h:20-265).
template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class OptimizeBFGS : public OptimizeSolver<R, Q, P> {
  using Base = OptimizeSolver<R, Q, P>;

 public:
  explicit OptimizeBFGS(std::shared_ptr<ArrayHandlers<R, Q, P>> handlers,
                        std::shared_ptr<Logger> logger = std::make_shared<Logger>())
      : Base(std::move(handlers), std::move(logger)) {}

  // reference :38-106; returns -1 when a line-search point was proposed in `parameters`
  int add_vector(R& parameters, R& residual, double value) override {
    auto& xs = *this->m_xspace;
    auto& xdata = xs.data;
    while (xs.size() >= size_t(m_max_size_qspace)) xs.eraseq(xs.size() - 1);
    auto& val = xdata[EqnData::value];
    const Matrix<double> old = val;
    val.resize({xs.size() + 1, 1});
    for (size_t i = 0; i < xs.size(); ++i) val(i + 1, 0) = old(i, 0);
    val(0, 0) = value;
    const int nwork = IterativeSolverTemplate<R, Q, P>::add_vector(wrap_arg(parameters), wrap_arg(residual));
    const auto& H = xdata.at(EqnData::H);
    const auto& S = xdata.at(EqnData::S);
    if (xs.size() > 1) {  // line search needed?
      const auto& V = xdata.at(EqnData::value);
      const double fprev = V(1, 0), fcur = V(0, 0);
      const double gprev = H(0, 1) - H(1, 1), gcur = H(0, 0) - H(1, 0);
      const bool wolfe1 = fcur <= fprev + m_Wolfe_1 * gprev;
      const bool wolfe2 = m_strong_Wolfe ? gcur >= m_Wolfe_2 * gprev : std::abs(gcur) <= m_Wolfe_2 * std::abs(gprev);
      (void)S;
      if (!(wolfe1 && wolfe2)) {
        Interpolate inter({-1, fprev, gprev}, {0, fcur, gcur});
        const auto p = inter.minimize(-1 - m_linesearch_grow_factor, m_linesearch_grow_factor);
        if (std::abs(p.x) > m_linesearch_tolerance) {
          this->m_logger->msg("Line search step taken", Logger::Info);
          this->m_handlers->rr().scal(1 + p.x, parameters);
          this->m_handlers->rq().axpy(-p.x, xs.cparamsq().at(1).get(), parameters);
          xs.eraseq(fprev < fcur ? 0 : 1);
          m_linesearch = true;
          return -1;
        }
      }
    }
    m_linesearch = false;
    this->m_logger->msg("Quasi-Newton step taken", Logger::Info);
    for (bool again = true; again;) {
      again = false;
      const auto& Hc = xdata.at(EqnData::H);
      for (size_t a = 0; a < m_alpha.size() && a + 1 < xs.size(); ++a)
        if (std::abs(curv(Hc, a)) < std::max(5e-14 * std::abs(Hc(a, a)), 1e-15)) {
          xs.eraseq(a + 1);
          this->m_logger->msg("Erase redundant Q", Logger::Info);
          again = true;
          break;
        }
    }
    bfgs_update_1(residual);
    return nwork;
  }
  using Base::add_vector;

  // reference :170-205
  size_t end_iteration(const VecRef<R>& parameters, const VecRef<R>& action) override {
    this->m_working_set = {0};
    this->m_end_iteration_needed = false;
    if (!m_linesearch) {
      m_last_linesearching = false;
      this->solution_params(this->m_working_set, parameters);
      if (this->m_errors.front() < this->m_convergence_threshold) {
        this->m_working_set.clear();
        return 0;
      }
      this->m_working_set.assign(1, 0);
      auto& z = action.front().get();
      bfgs_update_2(z);
      this->m_handlers->rr().axpy(-1, z, parameters.front());
    } else {
      this->m_stats->line_search_steps++;
      if (!m_last_linesearching) this->m_stats->line_searches++;
      m_last_linesearching = true;
    }
    this->m_stats->iterations++;
    return this->errors().front() < this->m_convergence_threshold ? 0 : 1;
  }
  using Base::end_iteration;

  void set_max_size_qspace(int n) { m_max_size_qspace = n; }
  int get_max_size_qspace() const { return m_max_size_qspace; }
  //! reference OptimizeBFGS.h:229-239 (which reports Wolfe_1 as the strong_Wolfe flag; the value here)
  std::shared_ptr<Options> get_options() const override {
    auto o = std::make_shared<OptimizeBFGSOptions>();
    o->copy(*IterativeSolverTemplate<R, Q, P>::get_options());
    o->max_size_qspace = m_max_size_qspace;
    o->strong_Wolfe = m_strong_Wolfe;
    o->Wolfe_1 = m_Wolfe_1;
    o->Wolfe_2 = m_Wolfe_2;
    o->linesearch_tolerance = m_linesearch_tolerance;
    o->linesearch_grow_factor = m_linesearch_grow_factor;
    return o;
  }
  void set_options(const Options& o) override {
    Base::set_options(o);
    if (auto* b = dynamic_cast<const OptimizeBFGSOptions*>(&o)) {
      if (b->max_size_qspace) set_max_size_qspace(*b->max_size_qspace);
      if (b->strong_Wolfe) m_strong_Wolfe = *b->strong_Wolfe;
      if (b->Wolfe_1) m_Wolfe_1 = *b->Wolfe_1;
      if (b->Wolfe_2) m_Wolfe_2 = *b->Wolfe_2;
      if (b->linesearch_tolerance) m_linesearch_tolerance = *b->linesearch_tolerance;
      if (b->linesearch_grow_factor) m_linesearch_grow_factor = *b->linesearch_grow_factor;
    }
  }

 private:
  static double curv(const Matrix<double>& H, size_t a) { return H(a, a) - H(a, a + 1) - H(a + 1, a) + H(a + 1, a + 1); }

  // first loop of the two-loop recursion (reference :108-120)
  void bfgs_update_1(R& residual) {
    auto& xs = *this->m_xspace;
    const auto& H = xs.data.at(EqnData::H);
    m_alpha.assign(xs.size() ? xs.size() - 1 : 0, 0.0);
    const auto q = xs.cparamsq();
    const auto u = xs.cactionsq();
    auto& h = *this->m_handlers;
    for (size_t a = 0; a < m_alpha.size(); ++a) {
      m_alpha[a] = (h.rq().dot(residual, q[a].get()) - h.rq().dot(residual, q[a + 1].get())) / curv(H, a);
      h.rq().axpy(-m_alpha[a], u[a].get(), residual);
      h.rq().axpy(m_alpha[a], u[a + 1].get(), residual);
    }
  }
  // second loop (reference :122-132)
  void bfgs_update_2(R& z) {
    auto& xs = *this->m_xspace;
    const auto& H = xs.data.at(EqnData::H);
    const auto q = xs.cparamsq();
    const auto u = xs.cactionsq();
    auto& h = *this->m_handlers;
    for (int a = int(m_alpha.size()) - 1; a >= 0; --a) {
      const double beta = (h.rq().dot(z, u[a].get()) - h.rq().dot(z, u[a + 1].get())) / curv(H, size_t(a));
      h.rq().axpy(m_alpha[a] - beta, q[a].get(), z);
      h.rq().axpy(-m_alpha[a] + beta, q[a + 1].get(), z);
    }
  }

  std::vector<double> m_alpha;
  bool m_linesearch = false;
  bool m_last_linesearching = false;
  int m_max_size_qspace = std::numeric_limits<int>::max();
  bool m_strong_Wolfe = true;
  double m_Wolfe_1 = 1e-4;
  double m_Wolfe_2 = 0.9;
  double m_linesearch_tolerance = .2;
  double m_linesearch_grow_factor = 2;
};

}  // namespace molpro::linalg::itsolv

#include "interpolate_morse.h"  // Interpolate("morse") fits by NonLinearEquationsDIIS, defined above
