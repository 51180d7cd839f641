// libitsolv_hbm.so: the restated solvers (include/itsolv_hbm/solvers.h) over HBM vectors and the
// HIP handlers, behind the C ABI of include/itsolv_hbm.h.  Problem actions run on the device
// (sspx_* kernels), so R, Q and the diagonals never leave HBM during a solve.
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "itsolv_hbm.h"
#include "itsolv_hbm/hbm_handlers.h"
#include "itsolv_hbm/problems.h"

using molpro::linalg::hbm::check;
using molpro::linalg::hbm::Device;
using molpro::linalg::hbm::SparseP;
using molpro::linalg::hbm::Vec;
using molpro::linalg::itsolv::CVecRef;
using molpro::linalg::itsolv::Problem;
using molpro::linalg::itsolv::VecRef;
namespace pr = molpro::linalg::itsolv::problems;

namespace {

thread_local std::string g_error;

std::shared_ptr<Device> borrow(ssp_ctx* ctx) {
  // The caller owns the context; the Device must not destroy it.
  return std::make_shared<Device>(ctx, true);
}

// zero-initialised (deferred, hbm_vec.h: stored only if something reads it before overwriting it)
Vec zero_vec(const std::shared_ptr<Device>& dev, size_t n) {
  Vec v(dev, n);
  v.fill_deferred(0.0);
  return v;
}

// write-only outputs (the problems' actions overwrite them in full)
std::vector<double*> ptrs(const VecRef<Vec>& v) {
  std::vector<double*> p;
  for (auto& x : v) p.push_back(x.get().data_wo());
  return p;
}
std::vector<const double*> cptrs(const CVecRef<Vec>& v) {
  std::vector<const double*> p;
  for (auto& x : v) p.push_back(x.get().data());
  return p;
}

// H = diag(d) + rho sum_l u_l u_l^T (itsolv_hbm/problems.h SyntheticSpec), applied on the device.
class SyntheticProblem : public Problem<Vec, SparseP> {
 public:
  SyntheticProblem(std::shared_ptr<Device> dev, const pr::SyntheticSpec& s)
      : m_dev(std::move(dev)), m_s(s), m_c(s.c_spec()) {}

  bool diagonals(Vec& d) const override {
    check(sspx_synth_diagonal(ctx(), &m_c, d.data_wo(), d.local_size(), d.offset()), "sspx_synth_diagonal");
    return true;
  }
  void action(const CVecRef<Vec>& params, const VecRef<Vec>& actions) const override {
    if (params.empty()) return;
    // the parameters' deferred normalisation scal (hbm_vec.h) is applied as they are read
    std::vector<const double*> x;
    std::vector<double> xs;
    for (auto& p : params) {
      x.push_back(p.get().data_deferred());
      xs.push_back(p.get().scale());
    }
    auto y = ptrs(actions);
    const auto& v0 = params.front().get();
    check(sspx_synth_action_scaled(ctx(), &m_c, x.data(), xs.data(), y.data(), int(params.size()), v0.local_size(),
                                   v0.offset()),
          "sspx_synth_action_scaled");
  }
  // r = H (x - target 1); value = 0 (unused by DIIS)
  double residual(const Vec& x, Vec& r) const override {
    Vec t(x);
    Vec ones(m_dev, x.size());
    check(ssp_fill(ctx(), m_s.target, ones.data_wo(), ones.local_size()), "ssp_fill");
    check(ssp_axpy(ctx(), -1.0, ones.data(), t.data_rw(), t.local_size()), "ssp_axpy");
    const double* xp[1] = {t.data()};
    double* yp[1] = {r.data_wo()};
    check(sspx_synth_action(ctx(), &m_c, xp, yp, 1, t.local_size(), t.offset()), "sspx_synth_action");
    return 0;
  }
  std::vector<double> pp_action_matrix(const std::vector<SparseP>& pp) const override {
    std::vector<size_t> idx;
    for (auto& p : pp) idx.push_back(p.begin()->first);
    std::vector<double> m;
    for (size_t i : idx)
      for (size_t j : idx) m.push_back(m_s.h(i, j));
    return m;
  }
  // actions[k] += sum_p c[k][p] H e_{i_p}: diagonal part as one batched sparse axpy, then the
  // low-rank part of every action in one device pass (the sign table read once for all of them;
  // per element the same two updates in the same order as action by action).
  void p_action(const std::vector<std::vector<double>>& c, const CVecRef<SparseP>& pp,
                const VecRef<Vec>& actions) const override {
    if (c.empty()) return;
    const size_t rank = size_t(m_s.rank);
    std::vector<double> w(c.size() * rank, 0.0);
    std::vector<double*> yp;
    std::vector<size_t> ptr{0}, idx;
    std::vector<double> val;
    for (size_t k = 0; k < c.size(); ++k) {
      auto& a = actions[k].get();
      for (size_t p = 0; p < pp.size(); ++p) {
        for (auto& [i, coef] : pp[p].get()) {
          idx.push_back(i);
          val.push_back(m_s.d(i) * coef * c[k][p]);
          for (size_t l = 0; l < rank; ++l) w[k * rank + l] += c[k][p] * coef * m_s.u(int(l), i);
        }
      }
      ptr.push_back(idx.size());
      yp.push_back(a.data_rw());
    }
    const auto& a0 = actions.front().get();
    check(ssp_sparse_axpy_batch(ctx(), int(yp.size()), ptr.data(), idx.data(), val.data(), yp.data(), a0.local_size(),
                                a0.offset()),
          "ssp_sparse_axpy_batch");
    check(sspx_synth_add_lowrank(ctx(), &m_c, yp.data(), int(yp.size()), a0.local_size(), a0.offset(), w.data()),
          "sspx_synth_add_lowrank");
  }

 private:
  ssp_ctx* ctx() const { return m_dev->ctx(); }
  std::shared_ptr<Device> m_dev;
  pr::SyntheticSpec m_s;
  sspx_synth m_c;
};

pr::SyntheticSpec spec_of(size_t n, const sspx_synth* s) {
  if (!s) throw std::invalid_argument("null sspx_synth");
  return pr::SyntheticSpec(n, s->rho, s->rank, s->seed, s->diag_kind, s->alpha, s->target);
}

// Dense row-major H, single rank: H resident in HBM, action by a row-per-lane kernel.
class DenseProblem : public Problem<Vec, SparseP> {
 public:
  DenseProblem(std::shared_ptr<Device> dev, const double* h, size_t n) : m_dev(std::move(dev)), m_h(h, h + n * n), m_n(n) {
    if (m_dev->nranks() != 1) throw std::invalid_argument("dense fixture problems run on a single rank");
    check(ssp_alloc(ctx(), n * n, &m_dh), "ssp_alloc");
    check(ssp_upload(ctx(), m_dh, h, n * n), "ssp_upload");
  }
  ~DenseProblem() override { ssp_free(ctx(), m_dh); }
  bool diagonals(Vec& d) const override {
    std::vector<double> v(m_n);
    for (size_t i = 0; i < m_n; ++i) v[i] = m_h[i * m_n + i];
    d.set_local_values(v);
    return true;
  }
  void action(const CVecRef<Vec>& params, const VecRef<Vec>& actions) const override {
    if (params.empty()) return;
    auto x = cptrs(params);
    auto y = ptrs(actions);
    check(sspx_dense_action(ctx(), m_dh, m_n, x.data(), y.data(), int(params.size()), m_n, 0), "sspx_dense_action");
  }
  double residual(const Vec& x, Vec& r) const override {
    Vec t(x);
    Vec ones(m_dev, x.size());
    check(ssp_fill(ctx(), 1.0, ones.data_wo(), m_n), "ssp_fill");
    check(ssp_axpy(ctx(), -1.0, ones.data(), t.data_rw(), m_n), "ssp_axpy");
    const double* xp[1] = {t.data()};
    double* yp[1] = {r.data_wo()};
    check(sspx_dense_action(ctx(), m_dh, m_n, xp, yp, 1, m_n, 0), "sspx_dense_action");
    return 0;
  }
  std::vector<double> pp_action_matrix(const std::vector<SparseP>& pp) const override {
    std::vector<double> m;
    for (auto& a : pp)
      for (auto& b : pp) m.push_back(m_h[a.begin()->first * m_n + b.begin()->first]);
    return m;
  }
  void p_action(const std::vector<std::vector<double>>& c, const CVecRef<SparseP>& pp,
                const VecRef<Vec>& actions) const override {
    // one column term at a time, added into the action as the reference's test drivers do
    // (a_j += H_ji coef c), so that the parity fixtures see the same sums
    Vec t(m_dev, m_n);
    std::vector<double> col(m_n);
    for (size_t k = 0; k < c.size(); ++k) {
      auto& a = actions[k].get();
      for (size_t p = 0; p < pp.size(); ++p)
        for (auto& [i, coef] : pp[p].get()) {
          for (size_t j = 0; j < m_n; ++j) col[j] = m_h[j * m_n + i] * coef * c[k][p];
          t.set_local_values(col);
          check(ssp_axpy(ctx(), 1.0, t.data(), a.data_rw(), m_n), "ssp_axpy");
        }
    }
  }

 private:
  ssp_ctx* ctx() const { return m_dev->ctx(); }
  std::shared_ptr<Device> m_dev;
  std::vector<double> m_h;
  size_t m_n;
  double* m_dh = nullptr;
};

// f(x) = x.Hx / x.x with gradient 2 (Hx - f x) / x.x: the objective of the reference's Python
// Rayleigh-quotient tests (python/test/test_rayleigh_quotient.py:8-33), H dense in HBM.
class RayleighProblem : public DenseProblem {
 public:
  using DenseProblem::DenseProblem;
  double residual(const Vec& x, Vec& g) const override {
    action(CVecRef<Vec>{std::cref(x)}, VecRef<Vec>{std::ref(g)});
    double xx = 0, xg = 0;
    check(ssp_dot(x.ctx(), x.data(), x.data(), x.local_size(), &xx), "ssp_dot");
    check(ssp_dot(x.ctx(), x.data(), g.data(), x.local_size(), &xg), "ssp_dot");
    const double f = xg / xx;
    check(ssp_axpy(x.ctx(), -f, x.data(), g.data_rw(), g.local_size()), "ssp_axpy");
    check(ssp_scal(x.ctx(), 2 / xx, g.data_rw(), g.local_size()), "ssp_scal");
    return f;
  }
};

template <class P>
double residual_norm(const P& problem, const std::shared_ptr<Device>& dev, const Vec& x, double e) {
  Vec ax(dev, x.size());
  problem.action(CVecRef<Vec>{std::cref(x)}, VecRef<Vec>{std::ref(ax)});
  check(ssp_axpy(dev->ctx(), -e, x.data(), ax.data_rw(), ax.local_size()), "ssp_axpy");
  double rr = 0, xx = 0;
  check(ssp_dot(dev->ctx(), ax.data(), ax.data(), ax.local_size(), &rr), "ssp_dot");
  check(ssp_dot(dev->ctx(), x.data(), x.data(), x.local_size(), &xx), "ssp_dot");
  return std::sqrt(std::abs(rr) / std::abs(xx));
}

// residual_norm for a batch of solutions (run_davidson's batched form): one action over the batch,
// r_i = H x_i - e_i x_i with |r_i|^2 in one pass (ssp_axpy_pairs_norm: element for element
// ssp_axpy's), |x_i|^2 from one symmetric overlap.  Batches of more than 16 roots (one fused launch's
// destinations) run as consecutive chunks of 16.  From the fused-pass size up (shorter vectors keep
// the per-root form and its sequential dots).
template <class P>
pr::ResidualNormsBatch<Vec> residual_norms_batch(const P& problem, const std::shared_ptr<Device>& dev, size_t n) {
  if (n < molpro::linalg::hbm::fused_min_size()) return {};
  return [&problem, dev, n](const std::vector<const Vec*>& xs, const std::vector<double>& e, std::vector<double>& out) {
    constexpr size_t kChunk = 16;
    for (size_t i0 = 0; i0 < xs.size(); i0 += kChunk) {
      const size_t m = std::min(kChunk, xs.size() - i0);
      std::vector<Vec> ax;
      ax.reserve(m);
      for (size_t i = 0; i < m; ++i) ax.emplace_back(dev, n);
      CVecRef<Vec> cx;
      VecRef<Vec> wa;
      for (size_t i = 0; i < m; ++i) {
        cx.emplace_back(std::cref(*xs[i0 + i]));
        wa.emplace_back(std::ref(ax[i]));
      }
      problem.action(cx, wa);
      std::vector<const double*> xp;
      std::vector<double*> ap;
      std::vector<double> c(m), rr(m), g(m * m);
      for (size_t i = 0; i < m; ++i) {
        xp.push_back(xs[i0 + i]->data());
        ap.push_back(ax[i].data_rw());
        c[i] = -e[i0 + i];
      }
      const size_t local = xs[i0]->local_size();
      check(ssp_axpy_pairs_norm(dev->ctx(), c.data(), xp.data(), nullptr, ap.data(), nullptr, int(m), local, rr.data()),
            "ssp_axpy_pairs_norm");
      check(ssp_gemm_inner(dev->ctx(), xp.data(), int(m), xp.data(), int(m), local, g.data()), "ssp_gemm_inner");
      for (size_t i = 0; i < m; ++i) out[i0 + i] = std::sqrt(std::abs(rr[i]) / std::abs(g[i * m + i]));
    }
  };
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

}  // namespace

extern "C" {

const char* itsolv_last_error(void) { return g_error.c_str(); }

void itsolv_default_options(itsolv_options* opt) { pr::default_options(opt); }

int itsolv_davidson_synthetic(ssp_ctx* ctx, size_t n, double rho, int rank, unsigned long long seed,
                              const itsolv_options* opt, itsolv_result* out, double* solutions_out) {
  const sspx_synth s{rho, rank, seed, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return itsolv_davidson_synth(ctx, n, &s, opt, out, solutions_out);
}

int itsolv_davidson_synth(ssp_ctx* ctx, size_t n, const sspx_synth* spec, const itsolv_options* opt,
                          itsolv_result* out, double* solutions_out) {
  return guarded([&] {
    auto dev = borrow(ctx);
    const auto o = opts_or_default(opt);
    SyntheticProblem problem(dev, spec_of(n, spec));
    std::memset(out, 0, sizeof(*out));
    pr::run_davidson<Vec, Vec, SparseP>(
        molpro::linalg::hbm::make_handlers(), problem, [&] { return zero_vec(dev, n); },
        [&](const Vec& x, double e) { return residual_norm(problem, dev, x, e); }, o, *out,
        [&](size_t r, const Vec& x) {
          if (!solutions_out) return;
          auto v = x.local_values();
          std::memcpy(solutions_out + r * v.size(), v.data(), v.size() * sizeof(double));
        },
        residual_norms_batch(problem, dev, n));
  });
}

int itsolv_davidson_dense(ssp_ctx* ctx, const double* h, size_t n, const itsolv_options* opt, itsolv_result* out,
                          double* solutions_out) {
  return guarded([&] {
    auto dev = borrow(ctx);
    const auto o = opts_or_default(opt);
    DenseProblem problem(dev, h, n);
    std::memset(out, 0, sizeof(*out));
    pr::run_davidson<Vec, Vec, SparseP>(
        molpro::linalg::hbm::make_handlers(), problem, [&] { return zero_vec(dev, n); },
        [&](const Vec& x, double e) { return residual_norm(problem, dev, x, e); }, o, *out,
        [&](size_t r, const Vec& x) {
          if (!solutions_out) return;
          auto v = x.local_values();
          std::memcpy(solutions_out + r * n, v.data(), n * sizeof(double));
        });
  });
}

int itsolv_diis_synthetic(ssp_ctx* ctx, size_t n, double rho, int rank, unsigned long long seed,
                          const itsolv_options* opt, itsolv_result* out, double* x_out) {
  const sspx_synth s{rho, rank, seed, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return itsolv_diis_synth(ctx, n, &s, opt, out, x_out);
}

int itsolv_diis_synth(ssp_ctx* ctx, size_t n, const sspx_synth* spec, const itsolv_options* opt, itsolv_result* out,
                      double* x_out) {
  return guarded([&] {
    auto dev = borrow(ctx);
    const auto o = opts_or_default(opt);
    SyntheticProblem problem(dev, spec_of(n, spec));
    std::memset(out, 0, sizeof(*out));
    pr::run_diis<Vec, Vec, SparseP>(
        molpro::linalg::hbm::make_handlers(), problem, [&] { return zero_vec(dev, n); },
        [&](Vec& x) {
          const size_t i0 = 0;
          const double one = 1.0;
          check(ssp_sparse_copy(x.ctx(), x.data_wo(), x.local_size(), x.offset(), &i0, &one, 1), "ssp_sparse_copy");
        },
        o, *out,
        [&](const Vec& x) {
          if (!x_out) return;
          auto v = x.local_values();
          std::memcpy(x_out, v.data(), v.size() * sizeof(double));
        });
  });
}

int itsolv_linear_equations_dense(ssp_ctx* ctx, const double* a, size_t n, const double* rhs, int nrhs,
                                  const itsolv_options* opt, itsolv_result* out, double* x_out) {
  return guarded([&] {
    auto dev = borrow(ctx);
    const auto o = opts_or_default(opt);
    DenseProblem problem(dev, a, n);
    std::memset(out, 0, sizeof(*out));
    std::vector<Vec> b;
    for (int r = 0; r < nrhs; ++r) {
      b.emplace_back(dev, n);
      check(ssp_upload(dev->ctx(), b.back().data_wo(), rhs + size_t(r) * n + b.back().offset(), b.back().local_size()),
            "ssp_upload");
    }
    pr::run_linear_equations<Vec, Vec, SparseP>(
        molpro::linalg::hbm::make_handlers(), problem, [&] { return zero_vec(dev, n); }, b,
        [&](const Vec& x, size_t r) {
          Vec ax(dev, x.size());
          problem.action(CVecRef<Vec>{std::cref(x)}, VecRef<Vec>{std::ref(ax)});
          check(ssp_axpy(dev->ctx(), -1.0, b[r].data(), ax.data_rw(), ax.local_size()), "ssp_axpy");
          double rr = 0, bb = 0;
          check(ssp_dot(dev->ctx(), ax.data(), ax.data(), ax.local_size(), &rr), "ssp_dot");
          check(ssp_dot(dev->ctx(), b[r].data(), b[r].data(), b[r].local_size(), &bb), "ssp_dot");
          return std::sqrt(std::abs(rr) / (bb > 0 ? bb : 1.0));
        },
        o, *out,
        [&](size_t r, const Vec& x) {
          if (!x_out) return;
          auto v = x.local_values();
          std::memcpy(x_out + r * n, v.data(), v.size() * sizeof(double));
        });
  });
}

int itsolv_optimize_dense(ssp_ctx* ctx, const double* h, size_t n, int algorithm, const itsolv_options* opt,
                          itsolv_result* out, double* x_out) {
  return guarded([&] {
    auto dev = borrow(ctx);
    const auto o = opts_or_default(opt);
    RayleighProblem problem(dev, h, n);
    std::memset(out, 0, sizeof(*out));
    pr::run_optimize<Vec, Vec, SparseP>(
        molpro::linalg::hbm::make_handlers(), problem, [&] { return zero_vec(dev, n); },
        [&](Vec& x) {
          const size_t i0 = 0;
          const double one = 1.0;
          check(ssp_sparse_copy(x.ctx(), x.data_wo(), x.local_size(), x.offset(), &i0, &one, 1), "ssp_sparse_copy");
        },
        algorithm, o, *out,
        [&](const Vec& x) {
          if (!x_out) return;
          auto v = x.local_values();
          std::memcpy(x_out, v.data(), v.size() * sizeof(double));
        });
  });
}

int itsolv_diis_dense(ssp_ctx* ctx, const double* h, size_t n, const itsolv_options* opt, itsolv_result* out,
                      double* x_out) {
  return guarded([&] {
    auto dev = borrow(ctx);
    const auto o = opts_or_default(opt);
    DenseProblem problem(dev, h, n);
    std::memset(out, 0, sizeof(*out));
    pr::run_diis<Vec, Vec, SparseP>(
        molpro::linalg::hbm::make_handlers(), problem, [&] { return zero_vec(dev, n); },
        [&](Vec& x) {
          const size_t i0 = 0;
          const double one = 1.0;
          check(ssp_sparse_copy(x.ctx(), x.data_wo(), x.local_size(), x.offset(), &i0, &one, 1), "ssp_sparse_copy");
        },
        o, *out,
        [&](const Vec& x) {
          if (!x_out) return;
          auto v = x.local_values();
          std::memcpy(x_out, v.data(), v.size() * sizeof(double));
        });
  });
}

}  // extern "C"
