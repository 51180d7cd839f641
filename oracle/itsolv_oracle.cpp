// ORACLE — test infrastructure only (see oracle_ops.h).
//
// The reference CPU path: the restated solvers (the same host templates the device library runs)
// over CPU handlers that call the oracle's restatement of ArrayHandlerIterable /
// ArrayHandlerIterableSparse (oracle_ops.c): sequential std::inner_product dots, element-order
// axpys, pairwise gemm_inner_default / gemm_outer_default (reference util/gemm.h:257-279).
// Exports oracle_* twins of the include/itsolv_hbm.h entry points; tests compare the two.
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "itsolv_hbm.h"
#include "itsolv_hbm/problems.h"
#include "itsolv_hbm/sparse_handler.h"
#include "oracle_handlers.h"
#include "oracle_ops.h"

using molpro::linalg::array::ArrayHandler;
using molpro::linalg::hbm::ArrayHandlerSparse;
using molpro::linalg::itsolv::ArrayHandlers;
using molpro::linalg::itsolv::CVecRef;
using molpro::linalg::itsolv::Problem;
using molpro::linalg::itsolv::VecRef;
using molpro::linalg::itsolv::subspace::Matrix;
namespace pr = molpro::linalg::itsolv::problems;

using V = std::vector<double>;
using SP = std::map<size_t, double>;
using oracle::cpu_handlers;
using oracle::IterableHandler;
using oracle::ok;

#ifdef OR_OMP  // liboracle_itsolv_omp.so: independent elements on several threads, bit-identical
#define OR_PAR_FOR _Pragma("omp parallel for schedule(static)")
#else
#define OR_PAR_FOR
#endif

namespace {

thread_local std::string g_error;


class SyntheticCpu : public Problem<V, SP> {
 public:
  explicit SyntheticCpu(const pr::SyntheticSpec& s) : m_s(s) {
    m_u.resize(size_t(s.rank));
    for (int l = 0; l < s.rank; ++l) {
      m_u[l].resize(s.n);
      auto& u = m_u[l];
      OR_PAR_FOR
      for (size_t g = 0; g < s.n; ++g) u[g] = s.u(l, g);
    }
  }
  bool diagonals(V& d) const override {
    OR_PAR_FOR
    for (size_t g = 0; g < d.size(); ++g) d[g] = m_s.diagonal(g);
    return true;
  }
  void apply(const V& x, V& y) const {
    std::vector<double> c(size_t(m_s.rank));
    OR_PAR_FOR
    for (int l = 0; l < m_s.rank; ++l) or_dot(m_u[l].data(), x.size(), x.data(), x.size(), &c[l]);
    OR_PAR_FOR
    for (size_t g = 0; g < x.size(); ++g) {
      double s = 0;
      for (int l = 0; l < m_s.rank; ++l) s += m_u[l][g] * c[l];
      y[g] = m_s.d(g) * x[g] + m_s.rho * s;
    }
  }
  void action(const CVecRef<V>& p, const VecRef<V>& a) const override {
    for (size_t k = 0; k < p.size(); ++k) apply(p[k].get(), a[k].get());
  }
  double residual(const V& x, V& r) const override {
    V t(x);
    for (auto& v : t) v -= m_s.target;
    apply(t, r);
    return 0;
  }
  std::vector<double> pp_action_matrix(const std::vector<SP>& pp) const override {
    std::vector<double> m;
    for (auto& a : pp)
      for (auto& b : pp) m.push_back(m_s.h(a.begin()->first, b.begin()->first));
    return m;
  }
  void p_action(const std::vector<std::vector<double>>& c, const CVecRef<SP>& pp, const VecRef<V>& a) const override {
    for (size_t k = 0; k < c.size(); ++k) {
      auto& y = a[k].get();
      std::vector<double> w(size_t(m_s.rank), 0.0);
      for (size_t p = 0; p < pp.size(); ++p)
        for (auto& [i, coef] : pp[p].get()) {
          y[i] += m_s.d(i) * coef * c[k][p];
          for (int l = 0; l < m_s.rank; ++l) w[l] += c[k][p] * coef * m_s.u(l, i);
        }
      OR_PAR_FOR
      for (size_t g = 0; g < y.size(); ++g) {
        double s = 0;
        for (int l = 0; l < m_s.rank; ++l) s += m_u[l][g] * w[l];
        y[g] += m_s.rho * s;
      }
    }
  }

 private:
  pr::SyntheticSpec m_s;
  std::vector<std::vector<double>> m_u;
};

class DenseCpu : public Problem<V, SP> {
 public:
  DenseCpu(const double* h, size_t n) : m_h(h, h + n * n), m_n(n) {}
  bool diagonals(V& d) const override {
    for (size_t i = 0; i < m_n; ++i) d[i] = m_h[i * m_n + i];
    return true;
  }
  void apply(const V& x, V& y) const {
    for (size_t i = 0; i < m_n; ++i) {
      double s = 0;
      for (size_t j = 0; j < m_n; ++j) s += m_h[i * m_n + j] * x[j];
      y[i] = s;
    }
  }
  void action(const CVecRef<V>& p, const VecRef<V>& a) const override {
    for (size_t k = 0; k < p.size(); ++k) apply(p[k].get(), a[k].get());
  }
  double residual(const V& x, V& r) const override {
    V t(x);
    for (auto& v : t) v -= 1.0;
    apply(t, r);
    return 0;
  }
  std::vector<double> pp_action_matrix(const std::vector<SP>& pp) const override {
    std::vector<double> m;
    for (auto& a : pp)
      for (auto& b : pp) m.push_back(m_h[a.begin()->first * m_n + b.begin()->first]);
    return m;
  }
  void p_action(const std::vector<std::vector<double>>& c, const CVecRef<SP>& pp, const VecRef<V>& a) const override {
    for (size_t k = 0; k < c.size(); ++k)
      for (size_t p = 0; p < pp.size(); ++p)
        for (auto& [i, coef] : pp[p].get())
          for (size_t j = 0; j < m_n; ++j) a[k].get()[j] += m_h[j * m_n + i] * coef * c[k][p];
  }

 private:
  std::vector<double> m_h;
  size_t m_n;
};

class RayleighCpu : public DenseCpu {
 public:
  using DenseCpu::DenseCpu;
  double residual(const V& x, V& g) const override {
    apply(x, g);
    double xx = 0, xg = 0;
    for (size_t i = 0; i < x.size(); ++i) {
      xx += x[i] * x[i];
      xg += x[i] * g[i];
    }
    const double f = xg / xx;
    for (size_t i = 0; i < x.size(); ++i) {
      g[i] += -f * x[i];
      g[i] *= 2 / xx;
    }
    return f;
  }
};

template <class P>
double residual_norm(const P& problem, const V& x, double e) {
  V ax(x.size());
  problem.apply(x, ax);
  double rr = 0, xx = 0;
  for (size_t i = 0; i < x.size(); ++i) {
    const double r = ax[i] - e * x[i];
    rr += r * r;
    xx += x[i] * x[i];
  }
  return std::sqrt(rr / xx);
}

template <class F>
int guarded(F f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_error = e.what();
    return 1;
  }
}

itsolv_options opts_or_default(const itsolv_options* o) {
  itsolv_options d;
  pr::default_options(&d);
  return o ? *o : d;
}

template <class P>
int davidson(const P& problem, size_t n, const itsolv_options* opt, itsolv_result* out, double* sol) {
  return guarded([&] {
    std::memset(out, 0, sizeof(*out));
    pr::run_davidson<V, V, SP>(
        cpu_handlers(), problem, [&] { return V(n, 0.0); },
        [&](const V& x, double e) { return residual_norm(problem, x, e); }, opts_or_default(opt), *out,
        [&](size_t r, const V& x) {
          if (sol) std::memcpy(sol + r * n, x.data(), n * sizeof(double));
        });
  });
}

template <class P>
int diis(const P& problem, size_t n, const itsolv_options* opt, itsolv_result* out, double* xo) {
  return guarded([&] {
    std::memset(out, 0, sizeof(*out));
    pr::run_diis<V, V, SP>(
        cpu_handlers(), problem, [&] { return V(n, 0.0); }, [](V& x) { x.at(0) = 1.0; }, opts_or_default(opt), *out,
        [&](const V& x) {
          if (xo) std::memcpy(xo, x.data(), n * sizeof(double));
        });
  });
}

// Reverse-communication twin of include/iterative_solver_c.h over the CPU handlers: the same solver
// construction and the same per-call routing as iterative-solver_amd/host/iterative_solver_c.cpp
// (reference IterativeSolverCMPI.cpp:158-534), with host vectors.  Tests drive one loop through both
// (problems defined in Python: Rosenbrock, trig, quadratic forms) and compare iteration by iteration.
namespace it = molpro::linalg::itsolv;
struct RcInstance {
  std::unique_ptr<it::IterativeSolverTemplate<V, V, SP>> solver;
  size_t n = 0;
  std::vector<V> rp, ra;
  VecRef<V> first(std::vector<V>& v, size_t k) {
    VecRef<V> r;
    for (size_t i = 0; i < k; ++i) r.emplace_back(v[i]);
    return r;
  }
  void in(size_t k, const double* x, const double* g) {
    while (rp.size() < k) {
      rp.emplace_back(n, 0.0);
      ra.emplace_back(n, 0.0);
    }
    for (size_t i = 0; i < k; ++i) {
      std::memcpy(rp[i].data(), x + i * n, n * sizeof(double));
      std::memcpy(ra[i].data(), g + i * n, n * sizeof(double));
    }
  }
  void out(size_t k, double* x, double* g) {
    for (size_t i = 0; i < k; ++i) {
      std::memcpy(x + i * n, rp[i].data(), n * sizeof(double));
      std::memcpy(g + i * n, ra[i].data(), n * sizeof(double));
    }
  }
};

}  // namespace

extern "C" {

const char* oracle_itsolv_last_error(void) { return g_error.c_str(); }

// test_problem on the reference's trigProblem (test_NonLinearEquations.cpp:160-204): value
// sum_i sin^2((i+1) x_i) + couple (sum x)^2; test parameters all 1, then x_{instance-1} += 1e-4.
// wrong_gradient scales the residual by 1.1 (a problem test_problem must reject).
int oracle_test_problem_trig(size_t n, double threshold, int wrong_gradient) {
  struct Trig : Problem<V, SP> {
    double scale = 1;
    double residual(const V& x, V& g) const override {
      double value = 0;
      const double couple = 1e-2;
      for (size_t i = 0; i < x.size(); ++i) {
        value += std::pow(std::sin((i + 1) * x[i]), 2);
        g[i] = 2 * (i + 1) * std::sin((i + 1) * x[i]) * std::cos((i + 1) * x[i]);
        for (size_t j = 0; j < x.size(); ++j) {
          value += couple * x[i] * x[j];
          g[i] += 2 * couple * x[j];
        }
        g[i] *= scale;
      }
      return value;
    }
    bool test_parameters(unsigned int instance, V& p) const override {
      p.assign(p.size(), 1.0);
      if (instance == 0) return true;
      if (instance <= p.size()) {
        p[instance - 1] += 0.0001;
        return true;
      }
      return false;
    }
  } problem;
  problem.scale = wrong_gradient ? 1.1 : 1.0;
  int ok = -1;
  guarded([&] {
    molpro::linalg::itsolv::NonLinearEquationsDIIS<V, V, SP> solver(cpu_handlers());
    V v0(n), v1(n);
    ok = solver.test_problem(problem, v0, v1, -1, threshold) ? 1 : 0;
  });
  return ok;
}

// The cubic line-search model of OptimizeBFGS (iterative-solver_amd/include/itsolv_hbm/interpolate.h,
// reference itsolv/Interpolate.cpp): value, first and second derivative at x of the cubic through
// (x0, f0, g0), (x1, f1, g1); and its analytic minimiser (out: x, f, f1, f2).
void oracle_interpolate_cubic(const double* p0, const double* p1, double x, double* out) {
  it::Interpolate inter({p0[0], p0[1], p0[2]}, {p1[0], p1[1], p1[2]});
  const auto p = inter(x);
  out[0] = p.x;
  out[1] = p.f;
  out[2] = p.f1;
  out[3] = p.f2;
}
// Interpolate(p0, p1, interpolant) evaluated at x, and minimize(xa, xb, bracket_grid,
// max_bracket_grid, analytic) (reference Interpolate.cpp:55-186); out: x, f, f1, f2 then the four
// parameters.  Returns nonzero with oracle_itsolv_last_error() on a throw (unknown interpolant).
int oracle_interpolate_ex(const double* p0, const double* p1, const char* interpolant, double x, double xa, double xb,
                          size_t bracket_grid, size_t max_bracket_grid, int analytic, double* at_x, double* minimum,
                          double* parameters) {
  return guarded([&] {
    it::Interpolate inter({p0[0], p0[1], p0[2]}, {p1[0], p1[1], p1[2]}, interpolant ? interpolant : "cubic", 0);
    const auto p = inter(x);
    const auto m = inter.minimize(xa, xb, bracket_grid, max_bracket_grid, analytic != 0);
    const double v[4] = {p.x, p.f, p.f1, p.f2}, w[4] = {m.x, m.f, m.f1, m.f2};
    for (int i = 0; i < 4; ++i) {
      at_x[i] = v[i];
      minimum[i] = w[i];
      parameters[i] = inter.parameters()[i];
    }
  });
}
void oracle_interpolate_minimize(const double* p0, const double* p1, double xa, double xb, double* out) {
  it::Interpolate inter({p0[0], p0[1], p0[2]}, {p1[0], p1[1], p1[2]});
  const auto p = inter.minimize(xa, xb);
  out[0] = p.x;
  out[1] = p.f;
  out[2] = p.f1;
  out[3] = p.f2;
}

// kind: "LinearEigensystem", "NonLinearEquations" (DIIS), "Optimize" (algorithm BFGS or SD),
// "LinearEquations" (rhs: nroot x n).  Returns NULL on error (oracle_itsolv_last_error).
void* oracle_rc_create(const char* kind, size_t n, size_t nroot, const double* rhs, double thresh, double thresh_value,
                       int hermitian, const char* algorithm, const char* options) {
  auto* h = new RcInstance;
  h->n = n;
  const std::string k = kind ? kind : "", alg = algorithm ? algorithm : "", opt = options ? options : "";
  const int s = guarded([&] {
    if (k == "LinearEigensystem" && alg == "RSPT") {  // LinearEigensystemRSPT.h:32-198
      auto d = std::make_unique<it::LinearEigensystemRSPT<V, V, SP>>(cpu_handlers());
      if (!opt.empty()) d->set_options(it::Options(it::parse_options(opt)));
      d->set_convergence_threshold(thresh);
      d->set_convergence_threshold_value(thresh_value);
      h->solver = std::move(d);
    } else if (k == "LinearEigensystem") {
      auto d = std::make_unique<it::LinearEigensystemDavidson<V, V, SP>>(cpu_handlers());
      if (!opt.empty()) d->set_options(it::LinearEigensystemDavidsonOptions(it::parse_options(opt)));
      d->set_n_roots(nroot);
      d->set_hermiticity(hermitian != 0);
      d->set_convergence_threshold(thresh);
      d->set_convergence_threshold_value(thresh_value);
      h->solver = std::move(d);
    } else if (k == "NonLinearEquations") {
      auto d = std::make_unique<it::NonLinearEquationsDIIS<V, V, SP>>(cpu_handlers());
      if (!opt.empty()) d->set_options(it::NonLinearEquationsDIISOptions(it::parse_options(opt)));
      d->set_convergence_threshold(thresh);
      h->solver = std::move(d);
    } else if (k == "Optimize") {
      std::unique_ptr<it::IterativeSolverTemplate<V, V, SP>> d;
      if (alg.empty() || alg == "BFGS") {
        auto b = std::make_unique<it::OptimizeBFGS<V, V, SP>>(cpu_handlers());
        if (!opt.empty()) b->set_options(it::OptimizeBFGSOptions(it::parse_options(opt)));
        d = std::move(b);
      } else if (alg == "SD") {
        d = std::make_unique<it::OptimizeSD<V, V, SP>>(cpu_handlers());
        if (!opt.empty()) d->set_options(it::Options(it::parse_options(opt)));
      } else {
        throw std::runtime_error("oracle_rc_create: unknown algorithm " + alg);
      }
      d->set_n_roots(1);
      d->set_convergence_threshold(thresh);
      d->set_convergence_threshold_value(thresh_value);
      h->solver = std::move(d);
    } else if (k == "LinearEquations") {
      auto d = std::make_unique<it::LinearEquationsDavidson<V, V, SP>>(cpu_handlers());
      std::vector<V> b;
      for (size_t r = 0; r < nroot; ++r) b.emplace_back(rhs + r * n, rhs + (r + 1) * n);
      if (!opt.empty()) d->set_options(it::LinearEquationsDavidsonOptions(it::parse_options(opt)));
      d->set_hermiticity(hermitian != 0);
      d->set_n_roots(nroot);
      d->add_equations(b);
      d->set_convergence_threshold(thresh);
      d->set_convergence_threshold_value(thresh_value);
      h->solver = std::move(d);
    } else {
      throw std::runtime_error("oracle_rc_create: unknown kind " + k);
    }
  });
  if (s) {
    delete h;
    return nullptr;
  }
  return h;
}

void oracle_rc_destroy(void* h) { delete static_cast<RcInstance*>(h); }

long long oracle_rc_add_vector(void* hp, size_t nbuf, double* x, double* g) {
  auto& h = *static_cast<RcInstance*>(hp);
  long long r = -1;
  guarded([&] {
    h.in(nbuf, x, g);
    r = h.solver->nonlinear() && nbuf >= 1 ? (long long)h.solver->add_vector(h.rp[0], h.ra[0], 0.0)
                                           : (long long)h.solver->add_vector(h.first(h.rp, nbuf), h.first(h.ra, nbuf));
    h.out(nbuf, x, g);
  });
  return r;
}

long long oracle_rc_add_value(void* hp, double value, double* x, double* g) {
  auto& h = *static_cast<RcInstance*>(hp);
  long long r = -1;
  guarded([&] {
    h.in(1, x, g);
    r = h.solver->add_vector(h.rp[0], h.ra[0], value) > 0 ? 1 : 0;
    h.out(1, x, g);
  });
  return r;
}

long long oracle_rc_end_iteration(void* hp, size_t nbuf, double* x, double* g) {
  auto& h = *static_cast<RcInstance*>(hp);
  long long r = -1;
  guarded([&] {
    h.in(nbuf, x, g);
    r = (long long)h.solver->end_iteration(h.first(h.rp, nbuf), h.first(h.ra, nbuf));
    h.out(nbuf, x, g);
  });
  return r;
}

// IterativeSolverAddP's twin: func(pcoeff (nvec x nP), actions (nvec rows of n), nvec, ranges).
long long oracle_rc_add_p(void* hp, size_t nbuf, size_t nP, const size_t* offsets, const size_t* indices,
                          const double* coefficients, const double* pp, double* x, double* g,
                          void (*func)(const double*, double*, const size_t, const size_t*)) {
  auto& h = *static_cast<RcInstance*>(hp);
  long long r = -1;
  guarded([&] {
    h.in(nbuf, x, g);
    std::vector<SP> pvectors(nP);
    for (size_t p = 0; p < nP; ++p)
      for (size_t k = offsets[p]; k < offsets[p + 1]; ++k) pvectors[p].emplace(indices[k], coefficients[k]);
    const size_t npp = (h.solver->dimensions().oP + nP) * nP;
    std::vector<double> ppm(pp, pp + npp);
    // stored by the solver and called again from later add_vector / solution calls: capture by value
    const size_t n = h.n;
    auto apply = [n, func](const std::vector<std::vector<double>>& pvecs, const CVecRef<SP>&, const VecRef<V>& act) {
      const size_t nu = pvecs.size();
      std::vector<double> flat;
      for (const auto& v : pvecs) flat.insert(flat.end(), v.begin(), v.end());
      std::vector<size_t> ranges;
      for (size_t k = 0; k < nu; ++k) {
        ranges.push_back(0);
        ranges.push_back(n);
      }
      std::vector<double> host(nu * n);
      for (size_t k = 0; k < nu; ++k) std::memcpy(host.data() + k * n, act[k].get().data(), n * sizeof(double));
      func(flat.data(), host.data(), nu, ranges.data());
      for (size_t k = 0; k < nu; ++k) std::memcpy(act[k].get().data(), host.data() + k * n, n * sizeof(double));
    };
    r = (long long)h.solver->add_p(molpro::linalg::itsolv::cwrap(pvectors), ppm, h.first(h.rp, nbuf),
                                   h.first(h.ra, nbuf), apply);
    h.out(nbuf, x, g);
  });
  return r;
}

int oracle_rc_working_set_eigenvalues(void* hp, double* ev) {
  auto& h = *static_cast<RcInstance*>(hp);
  return guarded([&] {
    size_t k = 0;
    for (double e : h.solver->working_set_eigenvalues()) ev[k++] = e;
  });
}

int oracle_rc_solution(void* hp, int nroot, const int* roots, double* x, double* g) {
  auto& h = *static_cast<RcInstance*>(hp);
  return guarded([&] {
    h.in(size_t(nroot), x, g);
    h.solver->solution(std::vector<int>(roots, roots + nroot), h.first(h.rp, size_t(nroot)),
                       h.first(h.ra, size_t(nroot)));
    h.out(size_t(nroot), x, g);
  });
}

// iterations, r_creations, errors (nroot), value, eigenvalues (nroot; Davidson only)
int oracle_rc_stats(void* hp, int* iterations, int* r_creations, double* errors, double* value, double* eigenvalues) {
  auto& h = *static_cast<RcInstance*>(hp);
  return guarded([&] {
    const auto& st = h.solver->statistics();
    *iterations = st.iterations;
    *r_creations = st.r_creations;
    size_t k = 0;
    for (double e : h.solver->errors()) errors[k++] = e;
    *value = h.solver->value();
    if (auto* d = dynamic_cast<it::LinearEigensystemDavidson<V, V, SP>*>(h.solver.get())) {
      k = 0;
      for (double e : d->eigenvalues()) eigenvalues[k++] = e;
    }
  });
}

int oracle_davidson_synthetic(size_t n, double rho, int rank, unsigned long long seed, const itsolv_options* opt,
                              itsolv_result* out, double* solutions_out) {
  SyntheticCpu p(pr::SyntheticSpec(n, rho, rank, seed));
  return davidson(p, n, opt, out, solutions_out);
}

// itsolv_davidson_synth / itsolv_diis_synth's twins (any synthetic family, include/subspace_hip.h sspx_synth)
int oracle_davidson_synth(size_t n, const sspx_synth* s, const itsolv_options* opt, itsolv_result* out,
                          double* solutions_out) {
  SyntheticCpu p(pr::SyntheticSpec(n, s->rho, s->rank, s->seed, s->diag_kind, s->alpha, s->target));
  return davidson(p, n, opt, out, solutions_out);
}

int oracle_diis_synth(size_t n, const sspx_synth* s, const itsolv_options* opt, itsolv_result* out, double* x_out) {
  SyntheticCpu p(pr::SyntheticSpec(n, s->rho, s->rank, s->seed, s->diag_kind, s->alpha, s->target));
  return diis(p, n, opt, out, x_out);
}

int oracle_davidson_dense(const double* h, size_t n, const itsolv_options* opt, itsolv_result* out,
                          double* solutions_out) {
  DenseCpu p(h, n);
  return davidson(p, n, opt, out, solutions_out);
}

int oracle_diis_synthetic(size_t n, double rho, int rank, unsigned long long seed, const itsolv_options* opt,
                          itsolv_result* out, double* x_out) {
  SyntheticCpu p(pr::SyntheticSpec(n, rho, rank, seed));
  return diis(p, n, opt, out, x_out);
}

int oracle_linear_equations_dense(const double* h, size_t n, const double* rhs, int nrhs, const itsolv_options* opt,
                                  itsolv_result* out, double* x_out) {
  DenseCpu p(h, n);
  return guarded([&] {
    std::memset(out, 0, sizeof(*out));
    std::vector<V> b;
    for (int r = 0; r < nrhs; ++r) b.emplace_back(rhs + size_t(r) * n, rhs + size_t(r + 1) * n);
    pr::run_linear_equations<V, V, SP>(
        cpu_handlers(), p, [&] { return V(n, 0.0); }, b,
        [&](const V& x, size_t r) {
          V ax(n);
          p.apply(x, ax);
          double rr = 0, bb = 0;
          for (size_t i = 0; i < n; ++i) {
            rr += (ax[i] - b[r][i]) * (ax[i] - b[r][i]);
            bb += b[r][i] * b[r][i];
          }
          return std::sqrt(rr / (bb > 0 ? bb : 1.0));
        },
        opts_or_default(opt), *out,
        [&](size_t r, const V& x) {
          if (x_out) std::memcpy(x_out + r * n, x.data(), n * sizeof(double));
        });
  });
}

int oracle_optimize_dense(const double* h, size_t n, int algorithm, const itsolv_options* opt, itsolv_result* out,
                          double* x_out) {
  RayleighCpu p(h, n);
  return guarded([&] {
    std::memset(out, 0, sizeof(*out));
    pr::run_optimize<V, V, SP>(
        cpu_handlers(), p, [&] { return V(n, 0.0); }, [](V& x) { x.at(0) = 1.0; }, algorithm, opts_or_default(opt),
        *out, [&](const V& x) {
          if (x_out) std::memcpy(x_out, x.data(), n * sizeof(double));
        });
  });
}

int oracle_diis_dense(const double* h, size_t n, const itsolv_options* opt, itsolv_result* out, double* x_out) {
  DenseCpu p(h, n);
  return diis(p, n, opt, out, x_out);
}

}  // extern "C"
