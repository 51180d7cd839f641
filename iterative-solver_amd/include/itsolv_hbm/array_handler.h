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
//   lazy_handle(): registers dot / axpy and evaluates them on eval() or destruction (:298-437)
//   through the protected fused_dot / fused_axpy, which device handlers override with one
//   gemm_inner / gemm_outer launch.
#pragma once
#include <cmath>
#include <complex>
#include <exception>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <set>
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

// Ordered register of deferred operations (reference ArrayHandler.h:29-57).  push(args...) appends;
// push<N>(args..., equal) inserts after the last registered operation whose N-th argument equals
// this one's, so operations sharing that argument end up consecutive, groups in arrival order.
template <typename... Args>
struct OperationRegister {
  using OP = std::tuple<Args...>;
  std::list<OP> m_register;

  template <int N, class ArgEqual>
  void push(const Args&... args, ArgEqual equal) {
    OP op{args...};
    auto pos = m_register.end();
    for (auto it = m_register.end(); it != m_register.begin();) {
      --it;
      if (equal(std::get<N>(op), std::get<N>(*it))) {
        pos = std::next(it);
        break;
      }
    }
    m_register.insert(pos, std::move(op));
  }
  void push(const Args&... args) { m_register.emplace_back(args...); }
  bool empty() { return m_register.empty(); }
  void clear() { m_register.clear(); }
};

// Turns a register of (x, y, z) operations into index triples over the distinct x, y and z
// (first-appearance order, equality by the given predicates) -- reference ArrayHandler.h:59-97.
template <typename X, typename Y, typename Z, class EqualX, class EqualY, class EqualZ>
std::tuple<std::vector<std::tuple<size_t, size_t, size_t>>, std::vector<X>, std::vector<Y>, std::vector<Z>>
remove_duplicates(const std::list<std::tuple<X, Y, Z>>& reg, EqualX equal_x, EqualY equal_y, EqualZ equal_z) {
  std::vector<std::tuple<size_t, size_t, size_t>> index;
  std::vector<X> xs;
  std::vector<Y> ys;
  std::vector<Z> zs;
  auto slot = [](auto& seen, const auto& v, auto& eq) {
    for (size_t i = 0; i < seen.size(); ++i)
      if (eq(v, seen[i])) return i;
    seen.push_back(v);
    return seen.size() - 1;
  };
  index.reserve(reg.size());
  for (const auto& op : reg) {
    const size_t ix = slot(xs, std::get<0>(op), equal_x);
    const size_t iy = slot(ys, std::get<1>(op), equal_y);
    const size_t iz = slot(zs, std::get<2>(op), equal_z);
    index.emplace_back(ix, iy, iz);
  }
  return {index, xs, ys, zs};
}

// Identity of referenced objects (reference ArrayHandler.h:100-106).
template <typename T = int>
struct RefEqual {
  bool operator()(const std::reference_wrapper<T>& l, const std::reference_wrapper<T>& r) {
    return std::addressof(l.get()) == std::addressof(r.get());
  }
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

// The abstract handler: the member names, signatures and protected customisation points of the
// reference's ArrayHandler<AL, AR> (ArrayHandler.h:161-437), so that a handler written for one
// base compiles against the other (include/itsolv_hbm/reference_handler.h builds the HBM handlers
// on the reference's own header).
template <class AL, class AR = AL>
class ArrayHandler {
 protected:
  struct Counter {
    int scal = 0;
    int dot = 0;
    int axpy = 0;
    int copy = 0;
    int gemm_inner = 0;
    int gemm_outer = 0;
  };
  std::unique_ptr<Counter> m_counter;

  ArrayHandler() : m_counter(std::make_unique<Counter>()) {}
  ArrayHandler(const ArrayHandler& o) : m_counter(std::make_unique<Counter>(*o.m_counter)) {}

 public:
  using value_type_L = element_type_t<AL>;
  using value_type_R = element_type_t<AR>;
  using value_type = decltype(value_type_L{} * value_type_R{});
  using value_type_abs = decltype(std::abs(value_type{}));

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
  // Extension (not in the reference): a fused call site (e.g. the residuals with
  // their norms, the block Gram-Schmidt update) records the handler operations its one pass
  // replaced, so Statistics reads the same operation counts whether or not the pass was fused.
  void count_replaced(int axpy, int dot, int gemm_outer) {
    m_counter->axpy += axpy;
    m_counter->dot += dot;
    m_counter->gemm_outer += gemm_outer;
  }

  std::string counter_to_string(std::string L, std::string R) {
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

  //! Destroying the handler invalidates the lazy handles it made: they no longer evaluate.
  virtual ~ArrayHandler() {
    for (auto& w : m_lazy_handles)
      if (auto h = w.lock()) h->invalidate();
  }

 protected:
  virtual void error(const std::string& message) { throw util::ArrayHandlerError{message}; }

  // Customisation points of lazy evaluation (reference :270-292): `reg` holds one (alpha, x, y)
  // index triple per registered axpy, (x, y, out) per registered dot, over the distinct operands.
  // The defaults evaluate one operation at a time in registration order; device handlers override
  // them with one batched launch.
  virtual void fused_axpy(const std::vector<std::tuple<size_t, size_t, size_t>>& reg,
                          const std::vector<value_type>& alphas, const std::vector<std::reference_wrapper<const AR>>& xx,
                          std::vector<std::reference_wrapper<AL>>& yy) {
    for (const auto& [a, x, y] : reg) axpy(alphas[a], xx[x].get(), yy[y].get());
  }
  virtual void fused_dot(const std::vector<std::tuple<size_t, size_t, size_t>>& reg,
                         const std::vector<std::reference_wrapper<const AL>>& xx,
                         const std::vector<std::reference_wrapper<const AR>>& yy,
                         std::vector<std::reference_wrapper<value_type>>& out) {
    for (const auto& [x, y, z] : reg) out[z].get() = dot(xx[x].get(), yy[y].get());
  }

  // Deferred dot / axpy (reference :298-381): one kind of operation at a time; eval() (or the
  // destructor) hands the de-duplicated register to fused_axpy / fused_dot and clears it.
  class LazyHandle {
   public:
    using value_type = typename ArrayHandler<AL, AR>::value_type;
    template <typename T>
    using ref_wrap = std::reference_wrapper<T>;

    explicit LazyHandle(ArrayHandler<AL, AR>& handler)
        : m_handler{handler}, m_uncaught_at_creation{std::uncaught_exceptions()} {}
    // As the reference, destruction evaluates what is still registered -- except while an exception
    // thrown in this handle's own scope unwinds it (a failed eval() or handler call): then the
    // register is dropped, so a recoverable device or size error reaches the caller (e.g. the C API's
    // status codes) instead of std::terminate from a second throw in this destructor.  Scope-guard
    // rule: only an unwind that began after the handle was made counts, so a handle created and
    // finished inside a cleanup path of some unrelated unwind still evaluates its operations.
    virtual ~LazyHandle() {
      if (std::uncaught_exceptions() > m_uncaught_at_creation)
        clear();
      else
        LazyHandle::eval();
    }

    virtual void axpy(value_type alpha, const AR& x, AL& y) {
      if (!register_op_type("axpy"))
        return error("Failed to register operation type axpy with the current state of the LazyHandle");
      m_axpy.push(alpha, std::cref(x), std::ref(y));
    }
    virtual void dot(const AL& x, const AR& y, value_type& out) {
      if (!register_op_type("dotLR"))
        return error("Failed to register operation type dot with the current state of the LazyHandle");
      m_dot.push(std::cref(x), std::cref(y), std::ref(out));
    }
    // The registers are taken and cleared before the handler runs them, so an operation that throws
    // leaves nothing behind to be evaluated again.
    virtual void eval() {
      if (m_invalid) return;
      auto axpys = std::move(m_axpy.m_register);
      auto dots = std::move(m_dot.m_register);
      clear();
      if (!axpys.empty()) {
        auto [reg, alphas, xx, yy] = util::remove_duplicates(axpys, std::equal_to<value_type>{},
                                                             util::RefEqual<const AR>{}, util::RefEqual<AL>{});
        m_handler.fused_axpy(reg, alphas, xx, yy);
      }
      if (!dots.empty()) {
        auto [reg, xx, yy, out] = util::remove_duplicates(dots, util::RefEqual<const AL>{}, util::RefEqual<const AR>{},
                                                          util::RefEqual<value_type>{});
        m_handler.fused_dot(reg, xx, yy, out);
      }
    }
    void invalidate() { m_invalid = true; }
    bool invalid() { return m_invalid; }

   protected:
    virtual bool register_op_type(const std::string& type) {
      if (!m_op_types.empty() && m_op_types.count(type) == 0) return false;
      m_op_types.insert(type);
      return true;
    }
    void clear() {
      m_op_types.clear();
      m_axpy.clear();
      m_dot.clear();
    }
    void error(std::string message) { m_handler.error(message); }

    std::set<std::string> m_op_types;
    util::OperationRegister<value_type, ref_wrap<const AR>, ref_wrap<AL>> m_axpy;
    util::OperationRegister<ref_wrap<const AL>, ref_wrap<const AR>, ref_wrap<value_type>> m_dot;
    ArrayHandler<AL, AR>& m_handler;
    bool m_invalid = false;
    int m_uncaught_at_creation = 0;  // std::uncaught_exceptions() when the handle was made
  };

  // What lazy_handle() returns (reference :384-414): forwards to the LazyHandle; with off(), every
  // registered operation is evaluated at once.
  class ProxyHandle {
   public:
    ProxyHandle(std::shared_ptr<LazyHandle> handle) : m_lazy_handle{std::move(handle)} {}
    template <typename... Args>
    void axpy(Args&&... args) {
      m_lazy_handle->axpy(std::forward<Args>(args)...);
      if (m_off) eval();
    }
    template <typename... Args>
    void dot(Args&&... args) {
      m_lazy_handle->dot(std::forward<Args>(args)...);
      if (m_off) eval();
    }
    void eval() { m_lazy_handle->eval(); }
    void invalidate() { m_lazy_handle->invalidate(); }
    bool invalid() { return m_lazy_handle->invalid(); }
    void off() { m_off = true; }
    void on() { m_off = false; }
    bool is_off() { return m_off; }

   protected:
    std::shared_ptr<LazyHandle> m_lazy_handle;
    bool m_off = false;
  };

  std::vector<std::weak_ptr<LazyHandle>> m_lazy_handles;

  void save_handle(const std::shared_ptr<LazyHandle>& handle) {
    for (auto& w : m_lazy_handles)
      if (w.expired()) {
        w = handle;
        return;
      }
    m_lazy_handles.push_back(handle);
  }
  ProxyHandle lazy_handle(ArrayHandler<AL, AR>& handler) {
    auto h = std::make_shared<LazyHandle>(handler);
    save_handle(h);
    return h;
  }

 public:
  //! A lazy handle on this handler; implementations return lazy_handle(*this).
  virtual ProxyHandle lazy_handle() = 0;
};

// Capabilities of a vector type's handlers beyond the reference interface.
// Both default to off, so the reference call sequence is kept for every other type (the CPU
// oracle path in particular); the HBM handlers switch them on (hbm_handlers.h).
//  * batched_symmetric_overlap: the symmetric overlap of one set is one gemm_inner(xx, xx) with the
//    lower triangle mirrored, in place of the pairwise dots of subspace/util.h:55-62.
template <class T>
struct batched_symmetric_overlap : std::false_type {};

//  * block_gram_schmidt_default: whether Davidson solvers over this R type orthogonalise new R
//    vectors by block Gram-Schmidt (rspace.h block_gram_schmidt) unless the option says otherwise;
//    for_length(n): the same for vectors of global length n.
template <class T>
struct block_gram_schmidt_default : std::false_type {
  static bool for_length(size_t) { return false; }
};

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

// Hook for the block Gram-Schmidt update (rspace.h block_gram_schmidt): yy[j] += P and Q/D
// combinations in that order, as one pass over the destinations; returns false when the handler has
// no such form (the caller then issues the two gemm_outer).  `hp` is the R x P handler.  Found by
// argument-dependent lookup.
template <class HP, class RefP, class RefQ, class RefR>
bool fused_block_update(HP&, const Matrix<double>&, const RefP&, const Matrix<double>&, const RefQ&, const RefR&) {
  return false;
}

// Hook for new Q vectors that are linear combinations of existing ones (construct_dspace,
// reference propose_rspace.h:380-394: a copy of a prototype, fill(0), then the axpy loops):
// out[i] = sum_j coeff(i, j) src[j], sources applied in order j = 0..; returns false when the
// handler has no form that writes the new vectors without copying, zeroing and re-reading them.
// Found by argument-dependent lookup.
template <class H, class Q>
bool fused_new_combinations(H&, const Matrix<double>&, const std::vector<const Q*>&, std::vector<Q>&) {
  return false;
}

// Hook for the new rows of the subspace matrices (xspace::update_qspace_data, reference
// XSpace.h:30-83, which issues one overlap per block): out = the overlaps of `rows` with the column
// sets `cols` concatenated, in one batched gemm_inner that reads the rows once per launch instead of
// once per block; returns false when the handler has no such form.  Found by argument-dependent
// lookup.
template <class H, class RefL, class RefC, class M>
bool fused_overlap_rows(H&, const RefL&, const std::vector<RefC>&, M&) {
  return false;
}

// Hook for an overlap whose result is needed only after more work has been queued (the subspace
// update's S(R, P) / H(P, R) rows, queued ahead of the dense rows so that one wait covers both):
// returns a function delivering gemm_inner(rows, cols), or an empty function when the handler has no
// such form.  Found by argument-dependent lookup.
template <class H, class RefL, class RefC>
std::function<Matrix<double>()> queued_overlap(H&, const RefL&, const RefC&) {
  return {};
}

// Hook for the residuals and their norms in one pass (construct_residual, reference
// LinearEigensystemDavidson.h:186-192: r_i += c_i x_i, then update_errors' self-dots,
// IterativeSolverTemplate.h:95-102): norms2[i] = <r_i, r_i> of the updated residuals; returns false
// when the handler has no such form.  Found by argument-dependent lookup.
template <class H, class RefX, class RefR>
bool fused_residual_norms(H&, const std::vector<double>&, const RefX&, const RefR&, std::vector<double>&) {
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
