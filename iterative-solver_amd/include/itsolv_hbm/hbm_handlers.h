// HBM-resident vectors and the ArrayHandlers that operate on them through libsubspace_hip.so.
//
// hbm::Vec is the R / Q container: one rank's contiguous shard [offset, offset + local_size) of a
// global vector of length size(), distributed as the reference's make_distribution_spread_remainder
// (reference array/util/Distribution.h:376-387; DistrArraySpan.cpp:35-37).  It owns its HBM block
// (unlike DistrArraySpan, whose copies alias, reference DistrArraySpan.cpp:47-51), is movable and
// deep-copyable, and value_type is double.
//
// ArrayHandlerHbm (R x R, Q x Q, R x Q, Q x R) and ArrayHandlerHbmSparse (Vec x std::map P) implement
// every ArrayHandler operation with one C-ABI call; ArrayHandlerSparse (P x P) is host-only.
// Error codes map to the reference's exceptions: size mismatch -> util::ArrayHandlerError,
// alphas dimension mismatch -> std::out_of_range (reference util/gemm.h:287-292), unsupported
// sparse copy-construction -> std::logic_error (reference ArrayHandlerDistrSparse.h:26-28).
#pragma once
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "array_handlers.h"
#include "sparse_handler.h"
#include "subspace_hip.h"

namespace molpro::linalg::hbm {

using itsolv::CVecRef;
using itsolv::VecRef;
using itsolv::subspace::Matrix;

inline void check(int status, const char* what) {
  if (status == SSP_OK) return;
  std::string msg = std::string(what) + ": " + ssp_last_error();
  switch (status) {
    case SSP_ERR_SIZE: throw array::util::ArrayHandlerError(msg);
    case SSP_ERR_RANGE: throw std::out_of_range(msg);
    case SSP_ERR_UNSUPPORTED: throw std::logic_error(msg);
    default: throw std::runtime_error(msg);
  }
}

// One process's device: the ssp context (HIP stream, HBM arena, optional RCCL communicator).
class Device {
 public:
  explicit Device(int device) { check(ssp_ctx_create(device, &m_ctx), "ssp_ctx_create"); }
  // Wraps a context owned by the caller (borrowed = true: not destroyed here).
  Device(ssp_ctx* ctx, bool borrowed) : m_ctx(ctx), m_owned(!borrowed) {
    if (!ctx) throw std::invalid_argument("hbm::Device: null ssp_ctx");
  }
  Device(const Device&) = delete;
  virtual ~Device() {
    if (m_owned) ssp_ctx_destroy(m_ctx);
  }
  void attach_comm(int nranks, int rank, const char* unique_id) {
    check(ssp_ctx_attach_comm(m_ctx, nranks, rank, unique_id), "ssp_ctx_attach_comm");
  }
  ssp_ctx* ctx() const { return m_ctx; }
  int rank() const { return ssp_ctx_rank(m_ctx); }
  int nranks() const { return ssp_ctx_nranks(m_ctx); }
  // Shard of a global length n owned by this rank.
  std::pair<size_t, size_t> shard(size_t n) const {
    size_t offset = 0, length = 0;
    check(ssp_shard_range(n, nranks(), rank(), &offset, &length), "ssp_shard_range");
    return {offset, length};
  }

 private:
  ssp_ctx* m_ctx = nullptr;
  bool m_owned = true;
};

class Vec {
 public:
  using value_type = double;

  Vec() = default;
  Vec(std::shared_ptr<Device> dev, size_t n_global) : m_dev(std::move(dev)), m_size(n_global) {
    auto [off, n] = m_dev->shard(n_global);
    m_offset = off;
    m_local = n;
    check(ssp_alloc(m_dev->ctx(), m_local, &m_data), "ssp_alloc");
  }
  Vec(const Vec& o) : Vec(o.m_dev, o.m_size) { check(ssp_copy(ctx(), m_data, o.m_data, m_local), "ssp_copy"); }
  Vec(Vec&& o) noexcept { swap(o); }
  Vec& operator=(const Vec& o) {
    if (this != &o) {
      Vec t(o);
      swap(t);
    }
    return *this;
  }
  Vec& operator=(Vec&& o) noexcept {
    Vec t(std::move(o));
    swap(t);
    return *this;
  }
  ~Vec() {
    if (m_data) ssp_free(ctx(), m_data);
  }
  void swap(Vec& o) noexcept {
    std::swap(m_dev, o.m_dev);
    std::swap(m_data, o.m_data);
    std::swap(m_size, o.m_size);
    std::swap(m_local, o.m_local);
    std::swap(m_offset, o.m_offset);
  }

  size_t size() const { return m_size; }
  size_t local_size() const { return m_local; }
  size_t offset() const { return m_offset; }
  double* data() { return m_data; }
  const double* data() const { return m_data; }
  ssp_ctx* ctx() const { return m_dev->ctx(); }
  const std::shared_ptr<Device>& device() const { return m_dev; }
  bool compatible(const Vec& o) const { return m_size == o.m_size && m_offset == o.m_offset && m_local == o.m_local; }

  std::vector<double> local_values() const {
    std::vector<double> v(m_local);
    check(ssp_download(ctx(), v.data(), m_data, m_local), "ssp_download");
    return v;
  }
  void set_local_values(const std::vector<double>& v) {
    if (v.size() != m_local) throw std::invalid_argument("Vec::set_local_values: wrong length");
    check(ssp_upload(ctx(), m_data, v.data(), m_local), "ssp_upload");
  }

 private:
  std::shared_ptr<Device> m_dev;
  double* m_data = nullptr;
  size_t m_size = 0, m_local = 0, m_offset = 0;
};


namespace detail {
inline std::vector<const double*> cptrs(const CVecRef<Vec>& v) {
  std::vector<const double*> p;
  for (auto& x : v) p.push_back(x.get().data());
  return p;
}
inline std::vector<double*> mptrs(const VecRef<Vec>& v) {
  std::vector<double*> p;
  for (auto& x : v) p.push_back(x.get().data());
  return p;
}
// (ptr, idx, val) CSR packing of sparse P vectors, indices ascending (std::map order).
inline void pack(const CVecRef<SparseP>& ps, std::vector<size_t>& ptr, std::vector<size_t>& idx,
                 std::vector<double>& val) {
  ptr.assign(1, 0);
  for (auto& p : ps) {
    for (auto& [i, v] : p.get()) {
      idx.push_back(i);
      val.push_back(v);
    }
    ptr.push_back(idx.size());
  }
}
}  // namespace detail

// Dense HBM x HBM handler.
class ArrayHandlerHbm : public array::ArrayHandler<Vec, Vec> {
 public:
  Vec copy(const Vec& source) override {
    m_counter->copy++;
    return Vec(source);
  }
  void copy(Vec& x, const Vec& y) override {
    m_counter->copy++;
    same(x, y, "copy");
    check(ssp_copy(x.ctx(), x.data(), y.data(), x.local_size()), "ssp_copy");
  }
  void scal(double alpha, Vec& x) override {
    m_counter->scal++;
    check(ssp_scal(x.ctx(), alpha, x.data(), x.local_size()), "ssp_scal");
  }
  void fill(double alpha, Vec& x) override { check(ssp_fill(x.ctx(), alpha, x.data(), x.local_size()), "ssp_fill"); }
  void axpy(double alpha, const Vec& x, Vec& y) override {
    m_counter->axpy++;
    if (x.size() < y.size()) error("ArrayHandlerHbm::axpy() incompatible x and y arrays, x.size() < y.size()");
    same(x, y, "axpy");
    check(ssp_axpy(y.ctx(), alpha, x.data(), y.data(), y.local_size()), "ssp_axpy");
  }
  double dot(const Vec& x, const Vec& y) override {
    m_counter->dot++;
    if (x.size() > y.size()) error("ArrayHandlerHbm::dot() incompatible x and y arrays, x.size() > y.size()");
    same(x, y, "dot");
    double out = 0;
    check(ssp_dot(x.ctx(), x.data(), y.data(), x.local_size(), &out), "ssp_dot");
    return out;
  }
  void gemm_outer(const Matrix<double> alphas, const CVecRef<Vec>& xx, const VecRef<Vec>& yy) override {
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
    auto xp = detail::cptrs(xx);
    auto yp = detail::mptrs(yy);
    const auto& y0 = yy.front().get();
    check(ssp_gemm_outer(y0.ctx(), alphas.data().data(), xp.data(), int(xx.size()), yp.data(), int(alphas.cols()),
                         y0.local_size()),
          "ssp_gemm_outer");
  }
  Matrix<double> gemm_inner(const CVecRef<Vec>& xx, const CVecRef<Vec>& yy) override {
    m_counter->gemm_inner++;
    Matrix<double> m({xx.size(), yy.size()});
    if (xx.empty() || yy.empty()) return m;
    for (auto& y : yy) same(xx.front().get(), y.get(), "gemm_inner");
    auto xp = detail::cptrs(xx);
    auto yp = detail::cptrs(yy);
    const auto& x0 = xx.front().get();
    check(ssp_gemm_inner(x0.ctx(), xp.data(), int(xx.size()), yp.data(), int(yy.size()), x0.local_size(), m.raw()),
          "ssp_gemm_inner");
    return m;
  }
  std::map<size_t, double> select_max_dot(size_t n, const Vec& x, const Vec& y) override {
    if (n > x.size() || n > y.size()) error("ArrayHandlerHbm::select_max_dot() n is too large");
    same(x, y, "select_max_dot");
    return run_select(n, [&](size_t* i, double* v, size_t* c) {
      return ssp_select_max_dot(x.ctx(), x.data(), y.data(), x.local_size(), x.offset(), n, i, v, c);
    });
  }
  std::map<size_t, double> select(size_t n, const Vec& x, bool max = false, bool ignore_sign = false) override {
    if (n > x.size()) error("ArrayHandlerHbm::select() n is too large");
    return run_select(n, [&](size_t* i, double* v, size_t* c) {
      return ssp_select(x.ctx(), x.data(), x.local_size(), x.offset(), n, max, ignore_sign, i, v, c);
    });
  }

  template <class F>
  static std::map<size_t, double> run_select(size_t n, F f) {
    std::vector<size_t> idx(std::max<size_t>(n, 1));
    std::vector<double> val(std::max<size_t>(n, 1));
    size_t cnt = 0;
    check(f(idx.data(), val.data(), &cnt), "ssp_select");
    std::map<size_t, double> out;
    for (size_t e = 0; e < cnt; ++e) out.emplace(idx[e], val[e]);
    return out;
  }

 protected:
  void same(const Vec& a, const Vec& b, const char* op) {
    if (!a.compatible(b)) error(std::string("ArrayHandlerHbm::") + op + "() arrays have different distributions");
  }
  // Registered lazy dots become one gemm_inner over the distinct x and y vectors.
  void fused_dot(const std::vector<std::tuple<const Vec*, const Vec*, double*>>& ops) override {
    std::vector<const Vec*> xs, ys;
    auto index = [](std::vector<const Vec*>& v, const Vec* p) {
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == p) return i;
      v.push_back(p);
      return v.size() - 1;
    };
    std::vector<std::pair<size_t, size_t>> at;
    for (auto& [x, y, out] : ops) at.emplace_back(index(xs, x), index(ys, y));
    CVecRef<Vec> cx, cy;
    for (auto p : xs) cx.emplace_back(*p);
    for (auto p : ys) cy.emplace_back(*p);
    auto m = gemm_inner(cx, cy);
    for (size_t k = 0; k < ops.size(); ++k) *std::get<2>(ops[k]) = m(at[k].first, at[k].second);
  }
};

// HBM x sparse (R x P, Q x P) handler.
class ArrayHandlerHbmSparse : public array::ArrayHandler<Vec, SparseP> {
 public:
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
    check(ssp_sparse_copy(x.ctx(), x.data(), x.local_size(), x.offset(), idx.data(), val.data(), idx.size()),
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
    check(ssp_sparse_axpy(y.ctx(), alpha, idx.data(), val.data(), idx.size(), y.data(), y.local_size(), y.offset()),
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
    check(ssp_sparse_dot(x.ctx(), x.data(), x.local_size(), x.offset(), idx.data(), val.data(), idx.size(), &out),
          "ssp_sparse_dot");
    return out;
  }
  void gemm_outer(const Matrix<double> alphas, const CVecRef<SparseP>& xx, const VecRef<Vec>& yy) override {
    m_counter->gemm_outer++;
    if (xx.empty() || yy.empty()) return;
    if (alphas.rows() != xx.size() || alphas.cols() > yy.size())
      throw std::out_of_range("gemm_outer (sparse): dimensions of alphas do not match xx, yy");
    std::vector<size_t> ptr, idx;
    std::vector<double> val;
    detail::pack(xx, ptr, idx, val);
    auto yp = detail::mptrs(yy);
    const auto& y0 = yy.front().get();
    check(ssp_gemm_outer_sparse(y0.ctx(), alphas.data().data(), ptr.data(), idx.data(), val.data(), int(xx.size()),
                                yp.data(), int(alphas.cols()), y0.local_size(), y0.offset()),
          "ssp_gemm_outer_sparse");
  }
  Matrix<double> gemm_inner(const CVecRef<Vec>& xx, const CVecRef<SparseP>& yy) override {
    m_counter->gemm_inner++;
    Matrix<double> m({xx.size(), yy.size()});
    if (xx.empty() || yy.empty()) return m;
    std::vector<size_t> ptr, idx;
    std::vector<double> val;
    detail::pack(yy, ptr, idx, val);
    auto xp = detail::cptrs(xx);
    const auto& x0 = xx.front().get();
    check(ssp_gemm_inner_sparse(x0.ctx(), xp.data(), int(xx.size()), x0.local_size(), x0.offset(), ptr.data(),
                                idx.data(), val.data(), int(yy.size()), m.raw()),
          "ssp_gemm_inner_sparse");
    return m;
  }
  // |x_i v_i| over the entries of y, reduced over ranks, then the reference's top-n rule.
  std::map<size_t, double> select_max_dot(size_t n, const Vec& x, const SparseP& y) override {
    if (n > x.size() || n > y.size()) error("ArrayHandlerHbmSparse::select_max_dot() n is too large");
    CVecRef<SparseP> singles;
    std::vector<SparseP> storage;
    for (auto& [i, v] : y)
      if (i < x.size()) storage.push_back(SparseP{{i, v}});
    for (auto& s : storage) singles.emplace_back(s);
    auto prod = gemm_inner(CVecRef<Vec>{std::cref(x)}, singles);
    std::vector<std::pair<double, size_t>> c;
    for (size_t e = 0; e < storage.size(); ++e) c.emplace_back(std::abs(prod(0, e)), storage[e].begin()->first);
    std::sort(c.begin(), c.end(), [](auto& a, auto& b) { return b < a; });
    std::map<size_t, double> out;
    for (size_t k = 0; k < std::min(n, c.size()); ++k) out.emplace(c[k].second, c[k].first);
    return out;
  }
  std::map<size_t, double> select(size_t n, const Vec& x, bool max = false, bool ignore_sign = false) override {
    if (n > x.size()) error("ArrayHandlerHbmSparse::select() n is too large");
    return ArrayHandlerHbm::run_select(n, [&](size_t* i, double* v, size_t* c) {
      return ssp_select(x.ctx(), x.data(), x.local_size(), x.offset(), n, max, ignore_sign, i, v, c);
    });
  }
};

// The bundle for R = Q = hbm::Vec, P = std::map<size_t, double>.
inline std::shared_ptr<itsolv::ArrayHandlers<Vec, Vec, SparseP>> make_handlers() {
  auto dense = [] { return std::make_shared<ArrayHandlerHbm>(); };
  auto sparse = [] { return std::make_shared<ArrayHandlerHbmSparse>(); };
  return itsolv::ArrayHandlers<Vec, Vec, SparseP>::create()
      .rr(dense())
      .qq(dense())
      .pp(std::make_shared<ArrayHandlerSparse>())
      .rq(dense())
      .rp(sparse())
      .qr(dense())
      .qp(sparse())
      .build_shared();
}

// Fused MGS step on HBM vectors (array::fused_axpy_inner hook, found by argument-dependent lookup).
inline bool fused_axpy_inner(array::ArrayHandler<Vec, Vec>&, const std::vector<double>& c, const Vec& x,
                             const itsolv::VecRef<Vec>& rr, const Vec& z, std::vector<double>& dots) {
  std::vector<double*> y;
  for (auto& r : rr) y.push_back(r.get().data());
  check(ssp_axpy_inner(x.ctx(), c.data(), x.data(), y.data(), int(y.size()), z.data(), x.local_size(), dots.data()),
        "ssp_axpy_inner");
  return true;
}

// construct_solution as one pass (array::fused_construct_solution hook): ssp_construct_solution
// writes the destinations without reading them, bit-identical to fill(0) + the three gemm_outer.
inline bool fused_construct_solution(array::ArrayHandler<Vec, SparseP>&, const itsolv::subspace::Matrix<double>& cp,
                                     const itsolv::CVecRef<SparseP>& pp, const itsolv::subspace::Matrix<double>& cqd,
                                     const itsolv::CVecRef<Vec>& qd, const itsolv::VecRef<Vec>& yy) {
  if (yy.empty() || cqd.cols() > yy.size() || cqd.rows() != qd.size() || cp.rows() != pp.size() ||
      (!pp.empty() && cp.cols() != cqd.cols()))
    return false;
  std::vector<size_t> ptr{0}, idx;
  std::vector<double> val;
  if (!pp.empty()) detail::pack(pp, ptr, idx, val);
  auto xp = detail::cptrs(qd);
  auto yp = detail::mptrs(yy);
  const auto& y0 = yy.front().get();
  check(ssp_construct_solution(y0.ctx(), cp.data().data(), ptr.data(), idx.data(), val.data(), int(pp.size()),
                               cqd.data().data(), xp.data(), int(qd.size()), yp.data(), int(cqd.cols()),
                               y0.local_size(), y0.offset()),
        "ssp_construct_solution");
  return true;
}

// Sequential self-orthonormalisation of R (reference propose_rspace.h:450-465) in two passes per
// vector: ssp_scal_inner (r_i *= 1/|r_i|, then <r_i, r_j> for j > i) and ssp_axpy_norm
// (r_j -= <r_i, r_j> r_i for j > i, then |r_{i+1}|^2).  The vector updates are the reference loop's
// scal and axpys, element for element; the dots are taken from the same values (array::
// fused_orthonormalise hook, found by argument-dependent lookup).
inline bool fused_orthonormalise(array::ArrayHandler<Vec, Vec>&, const itsolv::VecRef<Vec>& rr, double norm_thresh,
                                 std::vector<int>& null_params) {
  const size_t nR = rr.size();
  if (nR == 0) return true;
  ssp_ctx* ctx = rr[0].get().ctx();
  const size_t n = rr[0].get().local_size();
  double nrm2 = 0;
  check(ssp_dot(ctx, rr[0].get().data(), rr[0].get().data(), n, &nrm2), "ssp_dot");
  for (size_t i = 0; i < nR; ++i) {
    const double nrm = std::sqrt(std::abs(nrm2));
    if (nrm > norm_thresh) {
      std::vector<const double*> yc;
      std::vector<double*> y;
      for (size_t j = i + 1; j < nR; ++j) {
        yc.push_back(rr[j].get().data());
        y.push_back(rr[j].get().data());
      }
      std::vector<double> ov(std::max<size_t>(1, y.size()));
      check(ssp_scal_inner(ctx, 1. / nrm, rr[i].get().data(), yc.data(), int(yc.size()), n, ov.data()),
            "ssp_scal_inner");
      if (y.empty()) break;
      for (auto& o : ov) o = -o;
      check(ssp_axpy_norm(ctx, ov.data(), rr[i].get().data(), y.data(), int(y.size()), n, &nrm2), "ssp_axpy_norm");
    } else {
      null_params.push_back(int(i));
      if (i + 1 < nR) check(ssp_dot(ctx, rr[i + 1].get().data(), rr[i + 1].get().data(), n, &nrm2), "ssp_dot");
    }
  }
  return true;
}

// Davidson preconditioner on HBM vectors: reference precondition_default (IterativeSolver.h:34-55)
// as one fused kernel over all working-set vectors (d read once).  Found by argument-dependent
// lookup from Problem<R>::precondition.
inline void precondition_default(const itsolv::VecRef<Vec>& action, const std::vector<double>& shift,
                                 const Vec& diagonals) {
  if (action.empty()) return;
  std::vector<double*> a;
  for (auto& v : action) a.push_back(v.get().data());
  check(ssp_precondition(diagonals.ctx(), a.data(), int(a.size()), diagonals.data(), shift.data(),
                         diagonals.local_size()),
        "ssp_precondition");
}

}  // namespace molpro::linalg::hbm

namespace molpro::linalg::array {
// HBM handlers form symmetric overlaps with one gemm_inner (reads each vector once).
template <>
struct batched_symmetric_overlap<hbm::Vec> : std::true_type {};
}  // namespace molpro::linalg::array
