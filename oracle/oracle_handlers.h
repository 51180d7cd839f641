// ORACLE — test infrastructure only (see oracle_ops.h).
//
// The reference's CPU handlers restated over oracle_ops.c: ArrayHandlerIterable<std::vector<double>>
// (reference array/ArrayHandlerIterable.h:34-128: sequential std::inner_product dots, element-order
// axpys, pairwise gemm_inner_default / gemm_outer_default, util/gemm.h:257-279, the heap select of
// util/select.h:28-55) and ArrayHandlerIterableSparse<std::vector<double>, std::map<size_t, double>>
// (ArrayHandlerIterableSparse.h:151-217), on the restated ArrayHandler base.  Used by the oracle's
// solver path (itsolv_oracle.cpp) and the host-layer component tests (tests/cpp/host_layer_test.cpp).
#pragma once
#include <cmath>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "itsolv_hbm/array_handlers.h"
#include "itsolv_hbm/sparse_handler.h"
#include "oracle_ops.h"

namespace oracle {

using molpro::linalg::array::ArrayHandler;
using molpro::linalg::hbm::ArrayHandlerSparse;
using molpro::linalg::itsolv::ArrayHandlers;
using molpro::linalg::itsolv::CVecRef;
using molpro::linalg::itsolv::VecRef;
using molpro::linalg::itsolv::subspace::Matrix;
using V = std::vector<double>;
using SP = std::map<size_t, double>;

inline void ok(int s, const char* what) {
  if (s == 1) throw molpro::linalg::array::util::ArrayHandlerError(std::string(what) + ": incompatible sizes");
  if (s != 0) throw std::runtime_error(std::string(what) + ": oracle error");
}

// reference ArrayHandlerIterable<std::vector<double>> (ArrayHandlerIterable.h:34-128)
class IterableHandler : public ArrayHandler<V, V> {
 public:
  using typename ArrayHandler<V, V>::ProxyHandle;
  using ArrayHandler<V, V>::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }
  V copy(const V& s) override { return V(s); }
  void copy(V& x, const V& y) override { ok(or_copy(x.data(), x.size(), y.data(), y.size()), "copy"); }
  void scal(double a, V& x) override { or_scal(a, x.data(), x.size()); }
  void fill(double a, V& x) override { or_fill(a, x.data(), x.size()); }
  void axpy(double a, const V& x, V& y) override { ok(or_axpy(a, x.data(), x.size(), y.data(), y.size()), "axpy"); }
  double dot(const V& x, const V& y) override {
    double r = 0;
    ok(or_dot(x.data(), x.size(), y.data(), y.size(), &r), "dot");
    return r;
  }
  // gemm_outer_default / gemm_inner_default: pairwise axpy / dot
  void gemm_outer(const Matrix<double> al, const CVecRef<V>& xx, const VecRef<V>& yy) override {
    for (size_t i = 0; i < al.rows(); ++i)
      for (size_t j = 0; j < al.cols(); ++j) axpy(al(i, j), xx.at(i).get(), yy[j].get());
  }
  Matrix<double> gemm_inner(const CVecRef<V>& xx, const CVecRef<V>& yy) override {
    Matrix<double> m({xx.size(), yy.size()});
    if (xx.empty() || yy.empty()) return m;
#ifdef OR_OMP
    // the pairwise dots are independent: whole (sequential) dots spread over threads, bit-identical
    const long np = long(m.rows() * m.cols()), nc = long(m.cols());
    std::vector<int> st(size_t(np), 0);
    std::vector<double> out(size_t(np), 0.0);
#pragma omp parallel for schedule(dynamic) if (np > 1 && xx.at(0).get().size() > 65536)
    for (long ij = 0; ij < np; ++ij) {
      const V& x = xx.at(size_t(ij / nc)).get();
      const V& y = yy.at(size_t(ij % nc)).get();
      st[size_t(ij)] = or_dot(x.data(), x.size(), y.data(), y.size(), &out[size_t(ij)]);
    }
    for (long ij = 0; ij < np; ++ij) {
      ok(st[size_t(ij)], "dot");
      m(size_t(ij / nc), size_t(ij % nc)) = out[size_t(ij)];
    }
#else
    for (size_t i = 0; i < m.rows(); ++i)
      for (size_t j = 0; j < m.cols(); ++j) m(i, j) = dot(xx.at(i).get(), yy.at(j).get());
#endif
    return m;
  }
  std::map<size_t, double> select_max_dot(size_t n, const V& x, const V& y) override {
    if (n > x.size() || n > y.size()) error("ArrayHandlerIterable::select_max_dot() n is too large");
    return to_map(n, [&](size_t* i, double* v, size_t* c) {
      return or_select_max_dot(x.data(), y.data(), std::min(x.size(), y.size()), n, i, v, c);
    });
  }
  std::map<size_t, double> select(size_t n, const V& x, bool max = false, bool ignore_sign = false) override {
    if (n > x.size()) error("ArrayHandlerIterable::select() n is too large");
    return to_map(n, [&](size_t* i, double* v, size_t* c) { return or_select(x.data(), x.size(), n, max, ignore_sign, i, v, c); });
  }
  template <class F>
  static std::map<size_t, double> to_map(size_t n, F f) {
    std::vector<size_t> idx(std::max<size_t>(n, 1));
    std::vector<double> val(std::max<size_t>(n, 1));
    size_t c = 0;
    ok(f(idx.data(), val.data(), &c), "select");
    std::map<size_t, double> out;
    for (size_t e = 0; e < c; ++e) out.emplace(idx[e], val[e]);
    return out;
  }
};

// reference ArrayHandlerIterableSparse<std::vector<double>, std::map<size_t,double>> (:151-217)
class IterableSparseHandler : public ArrayHandler<V, SP> {
 public:
  using typename ArrayHandler<V, SP>::ProxyHandle;
  using ArrayHandler<V, SP>::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }
  V copy(const SP& s) override {
    V r;
    copy(r, s);
    return r;
  }
  void copy(V& x, const SP& y) override {
    std::fill(x.begin(), x.end(), 0.0);
    for (auto& [i, v] : y) x.at(i) = v;
  }
  void scal(double, V&) override {}
  void fill(double, V&) override {}
  void axpy(double a, const SP& x, V& y) override {
    for (auto& [i, v] : x)
      if (i < y.size()) y[i] = y[i] + a * v;
  }
  double dot(const V& x, const SP& y) override {
    double t = 0;
    for (auto& [i, v] : y)
      if (i < x.size()) t = t + x[i] * v;
    return t;
  }
  void gemm_outer(const Matrix<double> al, const CVecRef<SP>& xx, const VecRef<V>& yy) override {
    for (size_t i = 0; i < al.rows(); ++i)
      for (size_t j = 0; j < al.cols(); ++j) axpy(al(i, j), xx.at(i).get(), yy[j].get());
  }
  Matrix<double> gemm_inner(const CVecRef<V>& xx, const CVecRef<SP>& yy) override {
    Matrix<double> m({xx.size(), yy.size()});
    for (size_t i = 0; i < m.rows(); ++i)
      for (size_t j = 0; j < m.cols(); ++j) m(i, j) = dot(xx.at(i).get(), yy.at(j).get());
    return m;
  }
  // reference select_max_dot_iter_sparse (util/select_max_dot.h:59-85): a min-heap that receives the
  // in-range entries among y's first n without pops, then push + pop for every later in-range entry
  std::map<size_t, double> select_max_dot(size_t n, const V& x, const SP& y) override {
    if (n > x.size() || n > y.size()) error("ArrayHandlerIterableSparse::select_max_dot() n is too large");
    std::vector<double> prod;
    std::vector<size_t> keys;
    size_t keep = 0, e = 0;
    for (auto& [i, v] : y) {
      if (i < x.size()) {
        keys.push_back(i);
        prod.push_back(std::abs(x[i] * v));
        if (e < n) ++keep;
      }
      ++e;
    }
    auto sel = IterableHandler::to_map(keep, [&](size_t* i, double* v, size_t* c) {
      return or_select_max_dot(prod.data(), std::vector<double>(prod.size(), 1.0).data(), prod.size(), keep, i, v, c);
    });
    std::map<size_t, double> out;
    for (auto& [k, v] : sel) out.emplace(keys[k], v);
    return out;
  }
  std::map<size_t, double> select(size_t n, const V& x, bool max = false, bool ignore_sign = false) override {
    return IterableHandler::to_map(n, [&](size_t* i, double* v, size_t* c) { return or_select(x.data(), x.size(), n, max, ignore_sign, i, v, c); });
  }
};

inline std::shared_ptr<ArrayHandlers<V, V, SP>> cpu_handlers() {
  auto dense = [] { return std::make_shared<IterableHandler>(); };
  auto sparse = [] { return std::make_shared<IterableSparseHandler>(); };
  return ArrayHandlers<V, V, SP>::create()
      .rr(dense())
      .qq(dense())
      .pp(std::make_shared<ArrayHandlerSparse>())
      .rq(dense())
      .rp(sparse())
      .qr(dense())
      .qp(sparse())
      .build_shared();
}

}  // namespace oracle
