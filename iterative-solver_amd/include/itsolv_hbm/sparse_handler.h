// P x P handler (std::map<size_t, double> x std::map<size_t, double>), host only.
// Restates the reference's ArrayHandlerSparse (src/molpro/linalg/array/ArrayHandlerSparse.h): the P
// space is a handful of unit vectors, so these operations never touch the device.
#pragma once
#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

#include "array_handler.h"

namespace molpro::linalg::hbm {

using itsolv::CVecRef;
using itsolv::VecRef;
using itsolv::subspace::Matrix;
using SparseP = std::map<size_t, double>;

// P x P (sparse x sparse) handler on the host (reference ArrayHandlerSparse.h).
class ArrayHandlerSparse : public array::ArrayHandler<SparseP, SparseP> {
 public:
  using typename array::ArrayHandler<SparseP, SparseP>::ProxyHandle;
  using array::ArrayHandler<SparseP, SparseP>::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }
  SparseP copy(const SparseP& s) override {
    m_counter->copy++;
    return s;
  }
  void copy(SparseP& x, const SparseP& y) override {
    m_counter->copy++;
    x = y;
  }
  void scal(double a, SparseP& x) override {
    m_counter->scal++;
    for (auto& e : x) e.second *= a;
  }
  void fill(double a, SparseP& x) override {
    for (auto& e : x) e.second = a;
  }
  void axpy(double a, const SparseP& x, SparseP& y) override {
    m_counter->axpy++;
    for (auto& [i, v] : x) y[i] += a * v;
  }
  double dot(const SparseP& x, const SparseP& y) override {
    m_counter->dot++;
    double s = 0;
    for (auto& [i, v] : x) {
      auto it = y.find(i);
      if (it != y.end()) s += v * it->second;
    }
    return s;
  }
  void gemm_outer(const Matrix<double> alphas, const CVecRef<SparseP>& xx, const VecRef<SparseP>& yy) override {
    m_counter->gemm_outer++;
    for (size_t i = 0; i < alphas.rows(); ++i)
      for (size_t j = 0; j < alphas.cols(); ++j) axpy(alphas(i, j), xx.at(i).get(), yy[j].get());
  }
  Matrix<double> gemm_inner(const CVecRef<SparseP>& xx, const CVecRef<SparseP>& yy) override {
    m_counter->gemm_inner++;
    Matrix<double> m({xx.size(), yy.size()});
    for (size_t i = 0; i < xx.size(); ++i)
      for (size_t j = 0; j < yy.size(); ++j) m(i, j) = dot(xx[i].get(), yy[j].get());
    return m;
  }
  std::map<size_t, double> select_max_dot(size_t n, const SparseP& x, const SparseP& y) override {
    std::vector<std::pair<double, size_t>> c;
    for (auto& [i, v] : x) {
      auto it = y.find(i);
      if (it != y.end()) c.emplace_back(std::abs(v * it->second), i);
    }
    return top(n, c, false);
  }
  std::map<size_t, double> select(size_t n, const SparseP& x, bool max = false, bool ignore_sign = false) override {
    std::vector<std::pair<double, size_t>> c;
    for (auto& [i, v] : x) c.emplace_back(max ? (ignore_sign ? std::abs(v) : v) : (ignore_sign ? -std::abs(v) : -v), i);
    return top(n, c, !max);
  }

 private:
  static std::map<size_t, double> top(size_t n, std::vector<std::pair<double, size_t>>& c, bool negate) {
    std::sort(c.begin(), c.end(), [](auto& a, auto& b) { return b < a; });
    std::map<size_t, double> out;
    for (size_t k = 0; k < std::min(n, c.size()); ++k) out.emplace(c[k].second, negate ? -c[k].first : c[k].first);
    return out;
  }
};

}  // namespace molpro::linalg::hbm
