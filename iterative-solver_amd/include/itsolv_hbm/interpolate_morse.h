// Fit of the "morse" interpolant (reference itsolv/Interpolate.cpp:30-53, :74-97): the four
// parameters (L0, k, a, y0) are the root of the four conditions "value and slope match at both
// points", found by NonLinearEquationsDIIS from the cubic's minimum.  The parameters are four host
// doubles -- not solver vectors -- so they get a private container type and a private four-element
// handler here; no HBM vector is involved.  Included at the end of solvers.h.
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <vector>

#include "interpolate.h"

namespace molpro::linalg::itsolv {
namespace detail {

struct MorseParameters : std::vector<double> {
  using std::vector<double>::vector;
};
using MorseP = std::map<size_t, double>;

// The reference's ArrayHandlerIterable loops on four elements (ArrayHandlerIterable.h:46-110).
class MorseHandler : public array::ArrayHandler<MorseParameters, MorseParameters> {
  using V = MorseParameters;

 public:
  using typename array::ArrayHandler<MorseParameters, MorseParameters>::ProxyHandle;
  using array::ArrayHandler<MorseParameters, MorseParameters>::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }
  V copy(const V& s) override { return s; }
  void copy(V& x, const V& y) override { x = y; }
  void scal(double a, V& x) override {
    for (auto& e : x) e *= a;
  }
  void fill(double a, V& x) override { std::fill(x.begin(), x.end(), a); }
  void axpy(double a, const V& x, V& y) override {
    for (size_t i = 0; i < y.size(); ++i) y[i] += a * x[i];
  }
  double dot(const V& x, const V& y) override {
    double s = 0;
    for (size_t i = 0; i < x.size(); ++i) s += x[i] * y[i];
    return s;
  }
  void gemm_outer(const Matrix<double> al, const CVecRef<V>& xx, const VecRef<V>& yy) override {
    for (size_t i = 0; i < al.rows(); ++i)
      for (size_t j = 0; j < al.cols(); ++j) axpy(al(i, j), xx.at(i).get(), yy[j].get());
  }
  Matrix<double> gemm_inner(const CVecRef<V>& xx, const CVecRef<V>& yy) override {
    Matrix<double> m({xx.size(), yy.size()});
    for (size_t i = 0; i < m.rows(); ++i)
      for (size_t j = 0; j < m.cols(); ++j) m(i, j) = dot(xx.at(i).get(), yy.at(j).get());
    return m;
  }
  std::map<size_t, double> select_max_dot(size_t, const V&, const V&) override { return unused(); }
  std::map<size_t, double> select(size_t, const V&, bool, bool) override { return unused(); }

 private:
  static std::map<size_t, double> unused() { throw std::logic_error("Morse fit: select is not used by DIIS"); }
};

// DIIS has no P space: the P handlers complete the bundle and refuse every call that would touch a
// P vector.
template <class A, class B>
class MorseNoP : public array::ArrayHandler<A, B> {
  using T = typename array::ArrayHandler<A, B>::value_type;
  using TA = typename array::ArrayHandler<A, B>::value_type_abs;
  [[noreturn]] static void no() { throw std::logic_error("Morse fit: no P space"); }

 public:
  using typename array::ArrayHandler<A, B>::ProxyHandle;
  using array::ArrayHandler<A, B>::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }
  A copy(const B&) override { no(); }
  void copy(A&, const B&) override { no(); }
  void scal(T, A&) override { no(); }
  void fill(T, A&) override { no(); }
  void axpy(T, const B&, A&) override { no(); }
  T dot(const A&, const B&) override { no(); }
  // the subspace bookkeeping forms overlaps with the (empty) P set
  void gemm_outer(const Matrix<T>, const CVecRef<B>& xx, const VecRef<A>& yy) override {
    if (!xx.empty() && !yy.empty()) no();
  }
  Matrix<T> gemm_inner(const CVecRef<A>& xx, const CVecRef<B>& yy) override {
    if (!xx.empty() && !yy.empty()) no();
    return Matrix<T>({xx.size(), yy.size()});
  }
  std::map<size_t, TA> select_max_dot(size_t, const A&, const B&) override { no(); }
  std::map<size_t, T> select(size_t, const A&, bool, bool) override { no(); }
};

// reference Interpolate.cpp:30-53: residual = (f(x0), f(x1), f'(x0), f'(x1)) of the interpolant
// minus the given values and slopes
class MorseProblem : public Problem<MorseParameters, MorseP> {
 public:
  MorseProblem(Interpolate::point p0, Interpolate::point p1) : m_p0(p0), m_p1(p1) {}
  double residual(const MorseParameters& p, MorseParameters& r) const override {
    const auto a = Interpolate::morse(m_p0.x, p), b = Interpolate::morse(m_p1.x, p);
    r[0] = a.f - m_p0.f;
    r[1] = b.f - m_p1.f;
    r[2] = a.f1 - m_p0.f1;
    r[3] = b.f1 - m_p1.f1;
    return 0;
  }

 private:
  Interpolate::point m_p0, m_p1;
};

}  // namespace detail

inline std::vector<double> Interpolate::fit_morse(const point& p0, const point& p1, std::vector<double> guess,
                                                  int verbosity) {
  using V = detail::MorseParameters;
  using P = detail::MorseP;
  auto dense = std::make_shared<detail::MorseHandler>();
  auto handlers = ArrayHandlers<V, V, P>::create()
                      .rr(dense)
                      .qq(dense)
                      .rq(dense)
                      .qr(dense)
                      .pp(std::make_shared<detail::MorseNoP<P, P>>())
                      .rp(std::make_shared<detail::MorseNoP<V, P>>())
                      .qp(std::make_shared<detail::MorseNoP<V, P>>())
                      .build_shared();
  NonLinearEquationsDIIS<V, V, P> solver(handlers);  // create_NonLinearEquations<R>("DIIS") defaults
  solver.set_verbosity(Verbosity(verbosity));
  V parameters(guess.begin(), guess.end()), residual(4);
  detail::MorseProblem problem(p0, p1);
  if (!solver.solve(parameters, residual, problem)) throw std::runtime_error("Cannot find Morse interpolant");
  solver.solution(parameters, residual);
  return {parameters.begin(), parameters.end()};
}

}  // namespace molpro::linalg::itsolv
