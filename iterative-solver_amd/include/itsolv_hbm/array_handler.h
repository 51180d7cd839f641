// The drop-in boundary: ArrayHandler<AL, AR>.
//
// Same virtual operations, argument meaning and error behaviour as the reference's abstract handler
// (reference src/molpro/linalg/array/ArrayHandler.h:161-437):
//   copy / scal / fill / axpy / dot                            :184-190
//   gemm_outer(alphas (xx.size() x yy.size()), xx, yy)         :195   yy[j] += sum_i alphas(i,j) xx[i]
//   gemm_inner(xx, yy) -> Matrix (xx.size() x yy.size())       :200   M(i,j) = <xx[i], yy[j]>
//   select_max_dot / select -> std::map ordered by index       :212, :222
//   op Counter feeding Statistics                              :167-176, :224-253
//   errors throw util::ArrayHandlerError                       :25-27, :268
//   lazy_handle(): registers dot / axpy and evaluates them on eval() or destruction (:298-432);
//   here evaluation goes through fused_dot / fused_axpy, which device handlers override with
//   one gemm_inner / gemm_outer launch.
#pragma once
#include <cmath>
#include <complex>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "matrix.h"
#include "vecref.h"

namespace molpro::linalg::array {

using molpro::linalg::itsolv::CVecRef;
using molpro::linalg::itsolv::VecRef;
using molpro::linalg::itsolv::subspace::Matrix;

namespace util {
struct ArrayHandlerError : public std::logic_error {
  using std::logic_error::logic_error;
};
}  // namespace util

// Element type of a container: mapped_type for maps (P space), value_type otherwise.
template <class A, class = void>
struct element_type {
  using type = typename A::value_type;
};
template <class A>
struct element_type<A, std::void_t<typename A::mapped_type>> {
  using type = typename A::mapped_type;
};
template <class A>
using element_type_t = typename element_type<A>::type;

template <class AL, class AR = AL>
class ArrayHandler {
 public:
  using value_type_L = element_type_t<AL>;
  using value_type_R = element_type_t<AR>;
  using value_type = decltype(value_type_L{} * value_type_R{});
  using value_type_abs = decltype(std::abs(value_type{}));

  struct Counter {
    int scal = 0;
    int dot = 0;
    int axpy = 0;
    int copy = 0;
    int gemm_inner = 0;
    int gemm_outer = 0;
  };

  virtual ~ArrayHandler() = default;

  virtual AL copy(const AR& source) = 0;
  //! Copy content of y into x
  virtual void copy(AL& x, const AR& y) = 0;
  virtual void scal(value_type alpha, AL& x) = 0;
  virtual void fill(value_type alpha, AL& x) = 0;
  virtual void axpy(value_type alpha, const AR& x, AL& y) = 0;
  virtual value_type dot(const AL& x, const AR& y) = 0;
  virtual void gemm_outer(const Matrix<value_type> alphas, const CVecRef<AR>& xx, const VecRef<AL>& yy) = 0;
  virtual Matrix<value_type> gemm_inner(const CVecRef<AL>& xx, const CVecRef<AR>& yy) = 0;
  virtual std::map<size_t, value_type_abs> select_max_dot(size_t n, const AL& x, const AR& y) = 0;
  virtual std::map<size_t, value_type> select(size_t n, const AL& x, bool max = false, bool ignore_sign = false) = 0;

  const Counter& counter() const { return *m_counter; }
  void clear_counter() { *m_counter = Counter{}; }

  std::string counter_to_string(const std::string& L, const std::string& R) const {
    std::string s;
    const auto& c = *m_counter;
    if (c.scal > 0) s += std::to_string(c.scal) + " scaling operations of the " + L + " vectors, ";
    if (c.copy > 0) s += std::to_string(c.copy) + " " + L + "<-" + R + " copy operations, ";
    if (c.dot > 0) s += std::to_string(c.dot) + " dot product operations between the " + L + " and " + R + " vectors, ";
    if (c.axpy > 0) s += std::to_string(c.axpy) + " axpy (" + R + " = a*" + L + " + " + R + ") operations, ";
    if (c.gemm_inner > 0)
      s += std::to_string(c.gemm_inner) + " gemm_inner operations between the " + L + " and " + R + " vectors, ";
    if (c.gemm_outer > 0)
      s += std::to_string(c.gemm_outer) + " gemm_outer operations between the " + L + " and " + R + " vectors, ";
    return s;
  }

  // Deferred dot / axpy (reference ArrayHandler.h:298-432).  Only one kind of operation may be
  // registered at a time; eval() runs them through fused_dot / fused_axpy and clears the register.
  class LazyHandle {
   public:
    explicit LazyHandle(ArrayHandler& h) : m_handler(&h) {}
    LazyHandle(const LazyHandle&) = delete;
    ~LazyHandle() {
      try {
        eval();
      } catch (...) {
      }
    }
    void axpy(value_type a, const AR& x, AL& y) {
      kind("axpy");
      m_axpy.emplace_back(a, &x, &y);
      if (m_off) eval();
    }
    void dot(const AL& x, const AR& y, value_type& out) {
      kind("dot");
      m_dot.emplace_back(&x, &y, &out);
      if (m_off) eval();
    }
    void eval() {
      if (!m_handler) return;
      if (!m_axpy.empty()) m_handler->fused_axpy(m_axpy);
      if (!m_dot.empty()) m_handler->fused_dot(m_dot);
      m_axpy.clear();
      m_dot.clear();
      m_kind.clear();
    }
    void off() { m_off = true; }
    void on() { m_off = false; }
    bool is_off() const { return m_off; }
    void invalidate() { m_handler = nullptr; }
    bool invalid() const { return m_handler == nullptr; }

   private:
    void kind(const std::string& k) {
      if (!m_kind.empty() && m_kind != k)
        throw util::ArrayHandlerError("Failed to register operation type " + k + " with the current state of the LazyHandle");
      m_kind = k;
    }
    ArrayHandler* m_handler;
    bool m_off = false;
    std::string m_kind;
    std::vector<std::tuple<value_type, const AR*, AL*>> m_axpy;
    std::vector<std::tuple<const AL*, const AR*, value_type*>> m_dot;
  };
  using ProxyHandle = std::shared_ptr<LazyHandle>;
  ProxyHandle lazy_handle() { return std::make_shared<LazyHandle>(*this); }

 protected:
  ArrayHandler() : m_counter(std::make_unique<Counter>()) {}
  ArrayHandler(const ArrayHandler& o) : m_counter(std::make_unique<Counter>(*o.m_counter)) {}
  virtual void error(const std::string& message) { throw util::ArrayHandlerError{message}; }

  // Default fusion: one call per registered operation, in registration order.
  virtual void fused_axpy(const std::vector<std::tuple<value_type, const AR*, AL*>>& ops) {
    for (auto& [a, x, y] : ops) axpy(a, *x, *y);
  }
  virtual void fused_dot(const std::vector<std::tuple<const AL*, const AR*, value_type*>>& ops) {
    for (auto& [x, y, out] : ops) *out = dot(*x, *y);
  }

  std::unique_ptr<Counter> m_counter;
};

// Capabilities of a vector type's handlers beyond the reference interface.
// Both default to off, so the reference call sequence is kept for every other type (the CPU
// oracle path in particular); the HBM handlers switch them on (hbm_handlers.h).
//  * batched_symmetric_overlap: the symmetric overlap of one set is one gemm_inner(xx, xx) with the
//    lower triangle mirrored, in place of the pairwise dots of subspace/util.h:55-62.
template <class T>
struct batched_symmetric_overlap : std::false_type {};

// Fused MGS step hook: y_j += c_j x for all j, then dots_j = <y_j, z>, in one pass; returns false
// when the handler has no fused form (the caller then issues gemm_outer + gemm_inner).  Found by
// argument-dependent lookup; the HBM overload lives in namespace molpro::linalg::hbm.
template <class H, class Q, class RefR>
bool fused_axpy_inner(H&, const std::vector<double>&, const Q&, const RefR&, const Q&, std::vector<double>&) {
  return false;
}

// Hook for construct_solution (reference IterativeSolverTemplate.h:33-65: fill(0), then gemm_outer
// over the P, Q and D spaces) as one pass that writes the destinations without reading them:
// returns false when the handler has no such form.  `hp` is the R x P handler; the Q and D
// sources arrive concatenated (`qd`, coefficients `cqd`).  Found by argument-dependent lookup.
template <class HP, class RefP, class RefQ, class RefR>
bool fused_construct_solution(HP&, const Matrix<double>&, const RefP&, const Matrix<double>&, const RefQ&,
                              const RefR&) {
  return false;
}

// Hook for a fused sequential self-orthonormalisation of R (reference propose_rspace.h:450-465):
// returns false when the handler has no fused form (the caller then runs the reference loop of
// dot / scal / dot / axpy calls).  Found by argument-dependent lookup.
template <class H, class RefR>
bool fused_orthonormalise(H&, const RefR&, double, std::vector<int>&) {
  return false;
}

}  // namespace molpro::linalg::array
