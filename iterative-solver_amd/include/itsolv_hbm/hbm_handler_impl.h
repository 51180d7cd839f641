// The HBM ArrayHandlers, written once over whichever ArrayHandler base the translation unit has:
//
//   * itsolv_hbm/hbm_handlers.h includes this after the restated base (itsolv_hbm/array_handler.h):
//     the handlers this package's solvers and C ABI run on;
//   * itsolv_hbm/reference_handler.h includes it after the reference's own
//     molpro/linalg/array/ArrayHandler.h: the same classes as a drop-in for the reference's
//     ArrayHandlers<R, Q, P> injection (reference itsolv/ArrayHandlers.h:57-103).
//
// Both bases declare molpro::linalg::array::ArrayHandler<AL, AR>, ::util::ArrayHandlerError,
// molpro::linalg::itsolv::subspace::Matrix and itsolv::{CVecRef, VecRef} with the reference's
// signatures (reference ArrayHandler.h:161-437, subspace/Matrix.h, wrap.h), which is all this
// header uses.  Every operation is one libsubspace_hip.so C-ABI call on HBM-resident shards:
//
//   copy / scal / fill / axpy / dot   ArrayHandlerIterable.h:46-82     ssp_copy/scal/fill/axpy/dot
//   gemm_inner(xx, yy)                util/gemm.h:267-279 (+ :157-184)  ssp_gemm_inner (+ RCCL allreduce)
//   gemm_outer(alphas, xx, yy)        util/gemm.h:257-265 (+ :186-203)  ssp_gemm_outer
//   select / select_max_dot           util/select.h:28-55, DistrArray.cpp:170-276   ssp_select*
//   lazy dot (fused_dot)              ArrayHandler.h:283-292           one ssp_gemm_inner over the
//                                                                      distinct registered operands
//   lazy axpy (fused_axpy)            ArrayHandler.h:271-280           one ssp_gemm_outer when every
//                                     destination's sources arrive in first-appearance order (the
//                                     kernel applies them in that order with one fma each: bit-for-
//                                     bit the sequence of axpys); otherwise the sequence itself
//   sparse R x P (ArrayHandlerHbmSparse)  ArrayHandlerIterableSparse.h:35-58, DistrArray.cpp:419-465
//
// Error behaviour: size mismatches call error() (util::ArrayHandlerError, as
// ArrayHandlerIterable.h:68-69, :77-78 throw), alphas dimension mismatch -> std::out_of_range
// (gemm.h:66-71), sparse copy-construction -> std::logic_error (ArrayHandlerDistrSparse.h:26-28).
//
// No include guard on purpose: it is included once per translation unit, by one of the two headers
// above (each has #pragma once).
#include <algorithm>
#include <cmath>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "hbm_vec.h"

namespace molpro::linalg::hbm {

namespace detail {
template <class Refs>
std::vector<const double*> cptrs(const Refs& v) {
  std::vector<const double*> p;
  p.reserve(v.size());
  for (auto& x : v) p.push_back(x.get().data());
  return p;
}
// Destinations: read-modify-write (a shared block is copied first) or write-only (a shared block is
// replaced without a copy), hbm_vec.h.
template <class Refs>
std::vector<double*> rw_ptrs(const Refs& v) {
  std::vector<double*> p;
  p.reserve(v.size());
  for (auto& x : v) p.push_back(x.get().data_rw());
  return p;
}
// Operands of the *_scaled entry points (deferred scal, hbm_vec.h): the stored blocks and their
// pending scales; read-modify-write destinations hand their scale to the kernel.
template <class Refs>
std::vector<const double*> deferred_ptrs(const Refs& v, std::vector<double>& scales) {
  std::vector<const double*> p;
  p.reserve(v.size());
  scales.clear();
  for (auto& x : v) {
    p.push_back(x.get().data_deferred());
    scales.push_back(x.get().scale());
  }
  return p;
}
template <class Refs>
std::vector<double*> rw_deferred_ptrs(const Refs& v, std::vector<double>& scales) {
  std::vector<double*> p(v.size());
  scales.assign(v.size(), 1.0);
  for (size_t i = 0; i < v.size(); ++i) p[i] = v[i].get().data_rw_deferred(&scales[i]);
  return p;
}
// After a successful *_scaled call: the destinations' pending scales are in their blocks now.
template <class Refs>
void scales_applied(const Refs& v) {
  for (auto& x : v) x.get().scale_applied();
}
template <class Refs>
std::vector<double*> wo_ptrs(const Refs& v) {
  std::vector<double*> p;
  p.reserve(v.size());
  for (auto& x : v) p.push_back(x.get().data_wo());
  return p;
}
// (ptr, idx, val) CSR packing of sparse P vectors, indices ascending (std::map order).
template <class PRefs>
void pack(const PRefs& ps, std::vector<size_t>& ptr, std::vector<size_t>& idx, std::vector<double>& val) {
  ptr.assign(1, 0);
  for (auto& p : ps) {
    for (auto& [i, v] : p.get()) {
      idx.push_back(i);
      val.push_back(v);
    }
    ptr.push_back(idx.size());
  }
}
inline std::map<size_t, double> run_select(size_t n, const std::function<int(size_t*, double*, size_t*)>& f) {
  std::vector<size_t> idx(std::max<size_t>(n, 1));
  std::vector<double> val(std::max<size_t>(n, 1));
  size_t cnt = 0;
  check_status<array::util::ArrayHandlerError>(f(idx.data(), val.data(), &cnt), "ssp_select");
  std::map<size_t, double> out;
  for (size_t e = 0; e < cnt; ++e) out.emplace(idx[e], val[e]);
  return out;
}
}  // namespace detail

// Dense HBM x HBM handler (R x R, Q x Q, R x Q, Q x R).
class ArrayHandlerHbm : public array::ArrayHandler<Vec, Vec> {
  using Base = array::ArrayHandler<Vec, Vec>;
  static void check(int status, const char* what) { check_status<array::util::ArrayHandlerError>(status, what); }

 public:
  using typename Base::ProxyHandle;
  using Base::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }

  // Copies share the source's HBM block until one side is written (hbm_vec.h): no bytes move here.
  Vec copy(const Vec& source) override {
    m_counter->copy++;
    return Vec(source);
  }
  void copy(Vec& x, const Vec& y) override {
    m_counter->copy++;
    same(x, y, "copy");
    x.assign_shared(y);
  }
  // Deferred (hbm_vec.h): applied by the next kernel that reads x.
  void scal(double alpha, Vec& x) override {
    m_counter->scal++;
    x.scale_by(alpha);
  }
  // deferred to the next access that needs the block (hbm_vec.h): a write-only access drops it
  void fill(double alpha, Vec& x) override { x.fill_deferred(alpha); }
  void axpy(double alpha, const Vec& x, Vec& y) override {
    m_counter->axpy++;
    if (x.size() < y.size()) error("ArrayHandlerHbm::axpy() incompatible x and y arrays, x.size() < y.size()");
    same(x, y, "axpy");
    const double* xp = x.data_deferred();
    const double xs = x.scale();
    double ys = 1.0;
    double* yp = y.data_rw_deferred(&ys);
    check(ssp_axpy_scaled(y.ctx(), alpha, xp, xs, yp, ys, y.local_size()), "ssp_axpy_scaled");
    y.scale_applied();
  }
  double dot(const Vec& x, const Vec& y) override {
    m_counter->dot++;
    if (x.size() > y.size()) error("ArrayHandlerHbm::dot() incompatible x and y arrays, x.size() > y.size()");
    same(x, y, "dot");
    double out = 0;
    check(ssp_dot_scaled(x.ctx(), x.data_deferred(), x.scale(), y.data_deferred(), y.scale(), x.local_size(), &out),
          "ssp_dot_scaled");
    return out;
  }
  void gemm_outer(const itsolv::subspace::Matrix<double> alphas, const itsolv::CVecRef<Vec>& xx,
                  const itsolv::VecRef<Vec>& yy) override {
    m_counter->gemm_outer++;
    if (yy.empty() || xx.empty()) return;
    if (alphas.rows() != xx.size())
      throw std::out_of_range("gemm_outer: dimensions of xx and alphas are different: " + std::to_string(alphas.rows()) +
                              " " + std::to_string(xx.size()));
    // As gemm_outer_default (util/gemm.h:257-265): alphas.cols() destinations, the first of yy
    // (construct_solution fills a batch of roots into a larger parameter buffer).
    if (alphas.cols() > yy.size())
      throw std::out_of_range("gemm_outer: dimensions of yy and alphas are different: " + std::to_string(alphas.cols()) +
                              " " + std::to_string(yy.size()));
    for (auto& x : xx) same(x.get(), yy.front().get(), "gemm_outer");
    std::vector<double> xs, ys;
    auto xp = detail::deferred_ptrs(xx, xs);
    // only the alphas.cols() destinations the kernel updates
    const itsolv::VecRef<Vec> dest(yy.begin(), yy.begin() + long(alphas.cols()));
    auto yp = detail::rw_deferred_ptrs(dest, ys);
    const auto& y0 = yy.front().get();
    check(ssp_gemm_outer_scaled(y0.ctx(), alphas.data().data(), xp.data(), xs.data(), int(xx.size()), yp.data(),
                                ys.data(), int(alphas.cols()), y0.local_size()),
          "ssp_gemm_outer_scaled");
    detail::scales_applied(dest);
  }
  itsolv::subspace::Matrix<double> gemm_inner(const itsolv::CVecRef<Vec>& xx, const itsolv::CVecRef<Vec>& yy) override {
    m_counter->gemm_inner++;
    std::vector<double> buf(xx.size() * yy.size(), 0.0);
    if (!xx.empty() && !yy.empty()) {
      for (auto& y : yy) same(xx.front().get(), y.get(), "gemm_inner");
      std::vector<double> xs, ys;
      auto xp = detail::deferred_ptrs(xx, xs);
      auto yp = detail::deferred_ptrs(yy, ys);
      const auto& x0 = xx.front().get();
      check(ssp_gemm_inner_scaled(x0.ctx(), xp.data(), xs.data(), int(xx.size()), yp.data(), ys.data(), int(yy.size()),
                                  x0.local_size(), buf.data()),
            "ssp_gemm_inner_scaled");
    }
    return itsolv::subspace::Matrix<double>(std::move(buf), {xx.size(), yy.size()});
  }
  std::map<size_t, double> select_max_dot(size_t n, const Vec& x, const Vec& y) override {
    if (n > x.size() || n > y.size()) error("ArrayHandlerHbm::select_max_dot() n is too large");
    same(x, y, "select_max_dot");
    return detail::run_select(n, [&](size_t* i, double* v, size_t* c) {
      return ssp_select_max_dot(x.ctx(), x.data(), y.data(), x.local_size(), x.offset(), n, i, v, c);
    });
  }
  std::map<size_t, double> select(size_t n, const Vec& x, bool max = false, bool ignore_sign = false) override {
    if (n > x.size()) error("ArrayHandlerHbm::select() n is too large");
    return detail::run_select(n, [&](size_t* i, double* v, size_t* c) {
      return ssp_select(x.ctx(), x.data(), x.local_size(), x.offset(), n, max, ignore_sign, i, v, c);
    });
  }

 protected:
  void same(const Vec& a, const Vec& b, const char* op) {
    if (!a.compatible(b)) error(std::string("ArrayHandlerHbm::") + op + "() arrays have different distributions");
  }

  // Registered lazy dots: one gemm_inner over the distinct x and y (each vector read once).
  void fused_dot(const std::vector<std::tuple<size_t, size_t, size_t>>& reg,
                 const std::vector<std::reference_wrapper<const Vec>>& xx,
                 const std::vector<std::reference_wrapper<const Vec>>& yy,
                 std::vector<std::reference_wrapper<double>>& out) override {
    // a batch of self-dots whose values the kernels that wrote the vectors have recorded
    // (Vec::set_known_norm2: the block self-orthonormalisation's last Gram pass): no pass
    bool known = !reg.empty();
    std::vector<double> kv(reg.size());
    for (size_t r = 0; known && r < reg.size(); ++r) {
      const auto& [x, y, z] = reg[r];
      known = &xx[x].get() == &yy[y].get() && xx[x].get().known_norm2(&kv[r]);
    }
    if (known) {
      for (size_t r = 0; r < reg.size(); ++r) out[std::get<2>(reg[r])].get() = kv[r];
      return;
    }
    const auto m = gemm_inner(itsolv::CVecRef<Vec>(xx.begin(), xx.end()), itsolv::CVecRef<Vec>(yy.begin(), yy.end()));
    for (const auto& [x, y, z] : reg) out[z].get() = m(x, y);
  }

  // Registered lazy axpys: one gemm_outer (alphas(x, y) = the registered coefficient) when each
  // (x, y) pair occurs once and every destination receives its sources in increasing x order --
  // the order the kernel applies them -- so the result is the axpy sequence bit for bit.
  void fused_axpy(const std::vector<std::tuple<size_t, size_t, size_t>>& reg, const std::vector<double>& alphas,
                  const std::vector<std::reference_wrapper<const Vec>>& xx,
                  std::vector<std::reference_wrapper<Vec>>& yy) override {
    const size_t nx = xx.size(), ny = yy.size();
    std::vector<double> coef(nx * ny, 0.0);
    std::vector<char> seen(nx * ny, 0);
    std::vector<long> last(ny, -1);
    bool batched = nx > 0 && ny > 0;
    for (const auto& [a, x, y] : reg) {
      if (seen[x * ny + y] || long(x) < last[y]) {
        batched = false;
        break;
      }
      seen[x * ny + y] = 1;
      last[y] = long(x);
      coef[x * ny + y] = alphas[a];
    }
    if (!batched) {
      for (const auto& [a, x, y] : reg) axpy(alphas[a], xx[x].get(), yy[y].get());
      return;
    }
    for (size_t y = 1; y < ny; ++y) same(yy[y].get(), yy[0].get(), "fused_axpy");
    for (size_t x = 0; x < nx; ++x) same(xx[x].get(), yy[0].get(), "fused_axpy");
    m_counter->gemm_outer++;
    std::vector<double> xs, ys;
    auto xp = detail::deferred_ptrs(xx, xs);
    auto yp = detail::rw_deferred_ptrs(yy, ys);
    const auto& y0 = yy.front().get();
    check(ssp_gemm_outer_scaled(y0.ctx(), coef.data(), xp.data(), xs.data(), int(nx), yp.data(), ys.data(), int(ny),
                                y0.local_size()),
          "ssp_gemm_outer_scaled");
    detail::scales_applied(yy);
  }
};

// HBM x sparse (R x P, Q x P) handler; P = std::map<size_t, double>.
class ArrayHandlerHbmSparse : public array::ArrayHandler<Vec, SparseP> {
  using Base = array::ArrayHandler<Vec, SparseP>;
  static void check(int status, const char* what) { check_status<array::util::ArrayHandlerError>(status, what); }

 public:
  using typename Base::ProxyHandle;
  using Base::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }

  Vec copy(const SparseP&) override {
    throw std::logic_error("ArrayHandlerHbmSparse: cannot construct a distributed array from a sparse one");
  }
  void copy(Vec& x, const SparseP& y) override {
    m_counter->copy++;
    std::vector<size_t> idx;
    std::vector<double> val;
    for (auto& [i, v] : y) {
      idx.push_back(i);
      val.push_back(v);
    }
    check(ssp_sparse_copy(x.ctx(), x.data_wo(), x.local_size(), x.offset(), idx.data(), val.data(), idx.size()),
          "ssp_sparse_copy");
  }
  void scal(double, Vec&) override {}
  void fill(double, Vec&) override {}
  void axpy(double alpha, const SparseP& x, Vec& y) override {
    m_counter->axpy++;
    std::vector<size_t> idx;
    std::vector<double> val;
    for (auto& [i, v] : x)
      if (i < y.size()) {
        idx.push_back(i);
        val.push_back(v);
      }
    check(ssp_sparse_axpy(y.ctx(), alpha, idx.data(), val.data(), idx.size(), y.data_rw(), y.local_size(), y.offset()),
          "ssp_sparse_axpy");
  }
  double dot(const Vec& x, const SparseP& y) override {
    m_counter->dot++;
    std::vector<size_t> idx;
    std::vector<double> val;
    for (auto& [i, v] : y)
      if (i < x.size()) {
        idx.push_back(i);
        val.push_back(v);
      }
    double out = 0;
    const size_t ptr[2] = {0, idx.size()};
    const double* xp = x.data_deferred();
    const double xs = x.scale();
    check(ssp_gemm_inner_sparse_scaled(x.ctx(), &xp, &xs, 1, x.local_size(), x.offset(), ptr, idx.data(), val.data(),
                                       1, &out),
          "ssp_sparse_dot");
    return out;
  }
  void gemm_outer(const itsolv::subspace::Matrix<double> alphas, const itsolv::CVecRef<SparseP>& xx,
                  const itsolv::VecRef<Vec>& yy) override {
    m_counter->gemm_outer++;
    if (xx.empty() || yy.empty()) return;
    if (alphas.rows() != xx.size() || alphas.cols() > yy.size())
      throw std::out_of_range("gemm_outer (sparse): dimensions of alphas do not match xx, yy");
    std::vector<size_t> ptr, idx;
    std::vector<double> val;
    detail::pack(xx, ptr, idx, val);
    auto yp = detail::rw_ptrs(itsolv::VecRef<Vec>(yy.begin(), yy.begin() + long(alphas.cols())));
    const auto& y0 = yy.front().get();
    check(ssp_gemm_outer_sparse(y0.ctx(), alphas.data().data(), ptr.data(), idx.data(), val.data(), int(xx.size()),
                                yp.data(), int(alphas.cols()), y0.local_size(), y0.offset()),
          "ssp_gemm_outer_sparse");
  }
  itsolv::subspace::Matrix<double> gemm_inner(const itsolv::CVecRef<Vec>& xx,
                                              const itsolv::CVecRef<SparseP>& yy) override {
    m_counter->gemm_inner++;
    std::vector<double> buf(xx.size() * yy.size(), 0.0);
    if (!xx.empty() && !yy.empty()) {
      std::vector<size_t> ptr, idx;
      std::vector<double> val;
      detail::pack(yy, ptr, idx, val);
      std::vector<double> xs;
      auto xp = detail::deferred_ptrs(xx, xs);
      const auto& x0 = xx.front().get();
      check(ssp_gemm_inner_sparse_scaled(x0.ctx(), xp.data(), xs.data(), int(xx.size()), x0.local_size(), x0.offset(),
                                         ptr.data(), idx.data(), val.data(), int(yy.size()), buf.data()),
            "ssp_gemm_inner_sparse_scaled");
    }
    return itsolv::subspace::Matrix<double>(std::move(buf), {xx.size(), yy.size()});
  }
  // gemm_inner in two halves (ssp_gemm_inner_sparse_begin / _end; the array::queued_overlap hook):
  // the products are queued now, the returned function delivers them.  The same kernel and operands
  // as gemm_inner above, so the same numbers.
  std::function<itsolv::subspace::Matrix<double>()> gemm_inner_queued(const itsolv::CVecRef<Vec>& xx,
                                                                       const itsolv::CVecRef<SparseP>& yy) {
    m_counter->gemm_inner++;
    const size_t m = xx.size(), k = yy.size();
    if (m == 0 || k == 0)
      return [m, k] { return itsolv::subspace::Matrix<double>(std::vector<double>(m * k, 0.0), {m, k}); };
    std::vector<size_t> ptr, idx;
    std::vector<double> val;
    detail::pack(yy, ptr, idx, val);
    std::vector<double> xs;
    auto xp = detail::deferred_ptrs(xx, xs);
    const auto& x0 = xx.front().get();
    ssp_ctx* ctx = x0.ctx();
    check(ssp_gemm_inner_sparse_begin(ctx, xp.data(), xs.data(), int(m), x0.local_size(), x0.offset(), ptr.data(),
                                      idx.data(), val.data(), int(k)),
          "ssp_gemm_inner_sparse_begin");
    return [ctx, m, k] {
      std::vector<double> buf(m * k, 0.0);
      check(ssp_gemm_inner_sparse_end(ctx, buf.data()), "ssp_gemm_inner_sparse_end");
      return itsolv::subspace::Matrix<double>(std::move(buf), {m, k});
    };
  }
  // |x_i v_i| over the entries of y, reduced over ranks, then the reference's top-n rule of
  // select_max_dot_iter_sparse (util/select_max_dot.h:59-85): the first n entries of y are pushed
  // onto its heap without pops, out-of-range ones skipped, and every later in-range entry is pushed
  // and then the smallest popped -- so the result holds the largest n - k in-range products, k = the
  // number of out-of-range indices among y's first n entries (ties: the larger index stays).
  std::map<size_t, double> select_max_dot(size_t n, const Vec& x, const SparseP& y) override {
    if (n > x.size() || n > y.size()) error("ArrayHandlerHbmSparse::select_max_dot() n is too large");
    size_t keep = n;
    {
      auto it = y.begin();
      for (size_t e = 0; e < n; ++e, ++it)
        if (it->first >= x.size()) --keep;
    }
    std::vector<SparseP> storage;
    for (auto& [i, v] : y)
      if (i < x.size()) storage.push_back(SparseP{{i, v}});
    itsolv::CVecRef<SparseP> singles(storage.begin(), storage.end());
    const auto prod = gemm_inner(itsolv::CVecRef<Vec>{std::cref(x)}, singles);
    std::vector<std::pair<double, size_t>> c;
    for (size_t e = 0; e < storage.size(); ++e) c.emplace_back(std::abs(prod(0, e)), storage[e].begin()->first);
    std::sort(c.begin(), c.end(), [](auto& a, auto& b) { return b < a; });
    std::map<size_t, double> out;
    for (size_t k = 0; k < std::min(keep, c.size()); ++k) out.emplace(c[k].second, c[k].first);
    return out;
  }
  std::map<size_t, double> select(size_t n, const Vec& x, bool max = false, bool ignore_sign = false) override {
    if (n > x.size()) error("ArrayHandlerHbmSparse::select() n is too large");
    return detail::run_select(n, [&](size_t* i, double* v, size_t* c) {
      return ssp_select(x.ctx(), x.data(), x.local_size(), x.offset(), n, max, ignore_sign, i, v, c);
    });
  }
};

}  // namespace molpro::linalg::hbm
