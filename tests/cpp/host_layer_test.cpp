// Component tests of the restated host layer (iterative-solver_amd/include/itsolv_hbm/*.h) -- the code
// the GPU solvers and the CPU oracle share, so these are its only pins below whole-solve results.
// Each case restates a reference test (file:line under test/itsolv/) with the reference's inputs and
// expected values; run by tests/test_host_layer_cpp.py over the oracle's CPU handlers
// (oracle/oracle_handlers.h).
//
//   overlap_*, parameter_batches                 subspace/test_util.cpp:26-76, :176-187
//   resize_qspace, max_overlap_with_R_*          testDSpaceResetter.cpp:16-76
//   is_iota_*, construct_zeroed_copy,
//   delete_parameters_*, StringFacet_*           test_util.cpp:1-115
//   solver_factory_string_constructor            test_SolverFactory.cpp:9-66
//   qspace_* (prepend order, S/H splicing, erase) subspace/QSpace.h:76-116 -- the reference's own
//                                                testQSpace.cpp is not compiled by its build
//                                                (test/itsolv/subspace/CMakeLists.txt:1) and targets
//                                                functions its QSpace.h no longer has
//   dspace_resetter_do_reset                     DSpaceResetter.h:80-83
//   ordered_gemm_*, eigenproblem_kept_vectors,   the host algebra's fast paths against their plain
//   screen_cholesky_proof                        forms (dense.h; no reference test)
//   "svd" mode prints the restated eigensolver_lapacke_dsyev / svd_system on the matrix of
//   test_svd_system.cpp:17-35 for the Python side to check against LAPACK (numpy), as :64-90 does
//   against Eigen.
// Not restated, so not tested: subspace::util::eye_order, gram_schmidt and the vector-list
// modified_gram_schmidt of subspace/gram_schmidt.h (no solver path calls them; the Davidson MGS
// is propose_rspace.h:421-466, pinned through the solves).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <list>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "itsolv_hbm/dense.h"
#include "itsolv_hbm/rspace.h"
#include "itsolv_hbm/solver_factory.h"
#include "itsolv_hbm/solvers.h"
#include "oracle_handlers.h"

namespace it = molpro::linalg::itsolv;
namespace array = molpro::linalg::array;
using it::CVecRef;
using it::cwrap;
using it::VecRef;
using it::wrap;
using Mat = it::subspace::Matrix<double>;
using V = std::vector<double>;
using SP = std::map<size_t, double>;

namespace {
int g_fail = 0;
struct Failure {
  std::string why;
};
void expect(bool ok, const std::string& why) {
  if (!ok) throw Failure{why};
}
void run(const char* name, const std::function<void()>& f) {
  try {
    f();
    std::printf("PASS %s\n", name);
  } catch (const Failure& e) {
    ++g_fail;
    std::printf("FAIL %s: %s\n", name, e.why.c_str());
  } catch (const std::exception& e) {
    ++g_fail;
    std::printf("FAIL %s: exception %s\n", name, e.what());
  }
}
template <class E, class F>
bool throws(F f) {
  try {
    f();
  } catch (const E&) {
    return true;
  } catch (...) {
    return false;
  }
  return false;
}

// A second vector type, so that overlap() sees a handler whose (left, right) types are reversed.
struct W : std::vector<double> {
  using std::vector<double>::vector;
};
// Loops over two container types (dot / gemm_inner only; the overlap tests need nothing else).
template <class X, class Y>
struct DotHandler : array::ArrayHandler<X, Y> {
  using typename array::ArrayHandler<X, Y>::ProxyHandle;
  using array::ArrayHandler<X, Y>::lazy_handle;
  ProxyHandle lazy_handle() override { return this->lazy_handle(*this); }
  X copy(const Y& s) override { return X(s.begin(), s.end()); }
  void copy(X&, const Y&) override { throw std::logic_error("unused"); }
  void scal(double, X&) override { throw std::logic_error("unused"); }
  void fill(double, X&) override { throw std::logic_error("unused"); }
  void axpy(double, const Y&, X&) override { throw std::logic_error("unused"); }
  double dot(const X& x, const Y& y) override {
    double s = 0;
    for (size_t i = 0; i < x.size(); ++i) s = s + x[i] * y[i];
    return s;
  }
  void gemm_outer(const Mat, const CVecRef<Y>&, const VecRef<X>&) override { throw std::logic_error("unused"); }
  Mat gemm_inner(const CVecRef<X>& xx, const CVecRef<Y>& yy) override {
    Mat m({xx.size(), yy.size()});
    for (size_t i = 0; i < xx.size(); ++i)
      for (size_t j = 0; j < yy.size(); ++j) m(i, j) = dot(xx[i].get(), yy[j].get());
    return m;
  }
  std::map<size_t, double> select_max_dot(size_t, const X&, const Y&) override { return {}; }
  std::map<size_t, double> select(size_t, const X&, bool, bool) override { return {}; }
};

void subspace_util_cases() {
  const std::vector<double> alphas{1, 2, 3};
  const size_t nx = 5;
  std::vector<V> x;
  for (double a : alphas) x.emplace_back(nx, a);
  Mat ref({3, 3});
  for (size_t i = 0; i < 3; ++i)
    for (size_t j = 0; j < 3; ++j) ref(i, j) = double(nx) * alphas[i] * alphas[j];
  oracle::IterableHandler h;
  run("overlap_null_vectors", [&] { expect(it::subspace::util::overlap<V, V>({}, {}, h).empty(), "empty"); });
  run("overlap_one_param", [&] { expect(it::subspace::util::overlap(cwrap(x), h).data() == ref.data(), "S"); });
  run("overlap_two_params", [&] {
    expect(it::subspace::util::overlap(cwrap(x), cwrap(x), h).data() == ref.data(), "S");
  });
  run("overlap_reverse_params", [] {
    std::vector<V> xs{{1}, {2}, {3}};
    std::vector<W> ys{{4}, {5}, {6}};
    DotHandler<V, W> fwd;
    DotHandler<W, V> rev;
    auto m = it::subspace::util::overlap(cwrap(xs), cwrap(ys), fwd);
    auto mr = it::subspace::util::overlap(cwrap(xs), cwrap(ys), rev);
    expect(m.rows() == 3 && m.cols() == 3 && m(0, 2) == 6 && m(2, 0) == 12, "forward");
    expect(mr.data() == m.data(), "reversed handler transposes back");
  });
  run("parameter_batches", [] {
    using B = std::vector<std::pair<size_t, size_t>>;
    expect(it::detail::parameter_batches(3, 3) == B{{0, 3}}, "3,3");
    expect(it::detail::parameter_batches(2, 3) == B{{0, 2}}, "2,3");
    expect(it::detail::parameter_batches(9, 3) == B{{0, 3}, {3, 6}, {6, 9}}, "9,3");
    expect(it::detail::parameter_batches(4, 3) == B{{0, 3}, {3, 4}}, "4,3");
  });
}

void dspace_resetter_cases() {
  run("resize_qspace", [] {
    struct XS {
      int nQ = 3;
      std::vector<size_t> erased;
      it::subspace::Dimensions dims{0, 3, 0};
      const it::subspace::Dimensions& dimensions() const { return dims; }
      void eraseq(size_t i) {
        --nQ;
        erased.push_back(i);
        dims = it::subspace::Dimensions(0, size_t(nQ), 0);
      }
    } xs;
    Mat solutions(std::vector<double>{0.0, 0.5, -0.3, 0.0, 0.1, -0.4, 0.1, 0.2, 0.1}, {3, 3});
    it::Logger log;
    it::detail::resize_qspace(xs, solutions, 0, log);
    expect(xs.nQ == 0 && xs.erased == std::vector<size_t>({2, 1, 0}), "erased Q in descending order");
  });
  std::vector<V> rparams{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  oracle::IterableHandler h;
  auto case_ = [&](const char* name, std::vector<V> q, std::vector<int> want) {
    run(name, [&, q, want] {
      expect(it::detail::max_overlap_with_R(cwrap(rparams), cwrap(q), h) == want, "indices");
    });
  };
  case_("max_overlap_with_R_qparams_3", {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, {2, 1, 0});
  case_("max_overlap_with_R_qparams_2", {{1, 0, 0}, {0, 0, 1}}, {1, 0});
  case_("max_overlap_with_R_qparams_1", {{0, 1, 0}}, {0});
  case_("max_overlap_with_R_qparams_0", {}, {});
  run("dspace_resetter_do_reset", [] {
    it::detail::DSpaceResetter<V> r;
    r.set_nreset(3);
    expect(!r.do_reset(2, it::subspace::Dimensions(0, 4, 0)), "no D space: no reset");
    expect(r.do_reset(2, it::subspace::Dimensions(0, 4, 1)), "iteration 3 with D: reset");
    expect(!r.do_reset(3, it::subspace::Dimensions(0, 4, 1)), "iteration 4: no reset");
  });
}

void itsolv_util_cases() {
  using it::util::is_iota;
  run("is_iota_null", [] {
    std::vector<int> v;
    expect(is_iota(v.begin(), v.end(), 0), "empty");
  });
  run("is_iota_true", [] {
    std::vector<int> v{1, 2, 3, 4, 5};
    expect(is_iota(v.begin(), v.end(), 1), "1..5");
  });
  run("is_iota_false", [] {
    std::vector<int> v{1, 2, 3, 4, 5}, v2{1, 3, 4, 5}, v3{3, 2, 1};
    expect(!is_iota(v.begin(), v.end(), 0) && !is_iota(v2.begin(), v2.end(), v2[0]) &&
               !is_iota(v3.begin(), v3.end(), v3[0]),
           "not iota");
  });
  run("construct_zeroed_copy", [] {
    oracle::IterableHandler h;
    V r(10);
    std::iota(r.begin(), r.end(), 0.);
    auto q = it::util::construct_zeroed_copy(r, h);
    expect(q.size() == r.size() && q == V(10, 0.0), "zeroed copy");
  });
  run("delete_parameters_empty_params", [] {
    std::vector<int> p;
    it::util::delete_parameters({}, p);
    expect(p.empty(), "empty");
  });
  run("delete_parameters_empty_indices", [] {
    std::vector<int> p{1, 2, 3, 4};
    it::util::delete_parameters({}, p);
    expect(p == std::vector<int>({1, 2, 3, 4}), "unchanged");
  });
  run("delete_parameters", [] {
    std::vector<int> p{1, 2, 3, 4};
    it::util::delete_parameters({1, 3}, p);
    expect(p == std::vector<int>({1, 3}), "deleted");
  });
  using it::util::StringFacet;
  run("StringFacet_toupper", [] { expect(StringFacet{}.toupper("MixeD C@sE") == "MIXED C@SE", "upper"); });
  run("StringFacet_tolower", [] { expect(StringFacet{}.tolower("MixeD C@sE") == "mixed c@se", "lower"); });
  run("StringFacet_crop_space", [] {
    for (std::string s : {std::string(" some_words"), std::string("some_words "), std::string(" some_words ")}) {
      StringFacet::crop_space(s);
      expect(s == "some_words", "crop");
    }
  });
  run("StringFacet_tobool_true", [] {
    for (std::string s : {"TRUE", "True", "tRuE", "true", " true", "    true    ", "T", "t", "1"})
      expect(StringFacet{}.tobool(s), s);
  });
  run("StringFacet_tobool_false", [] {
    for (std::string s : {"FALSE", "False", "fAlSe", "false", " false", "  false    ", "F", "f", "0"})
      expect(!StringFacet{}.tobool(s), s);
  });
  run("StringFacet_tobool_exception", [] {
    for (std::string s : {"Tr", "fal", "2", ""})
      expect(throws<std::runtime_error>([&] { StringFacet{}.tobool(s); }), "'" + s + "' must throw");
  });
  run("StringFacet_parse_keyval_string", [] {
    auto m = StringFacet::parse_keyval_string(" key1=value1 , key2=value2,key3=  , key4=value4");
    expect(m["key1"] == "value1" && m["key2"] == "value2" && m["key3"] == "" && m["key4"] == "value4", "good");
    expect(throws<std::runtime_error>([] { StringFacet::parse_keyval_string("keywithoutvalue"); }), "bad");
    auto m2 = StringFacet::parse_keyval_string("a:1; b = 2;");
    expect(m2.size() == 2 && m2["a"] == "1" && m2["b"] == "2", "':' and ';' separators");
    // reference util.cpp:47-48: parsing stops at the first empty field
    auto m3 = StringFacet::parse_keyval_string("A=1,,B=2");
    expect(m3.size() == 1 && m3["A"] == "1", "consecutive separators end the list");
    auto m4 = StringFacet::parse_keyval_string("A=1; ;B=2");
    expect(m4.size() == 1, "a blank field ends the list");
    expect(StringFacet::parse_keyval_string("").empty() && StringFacet::parse_keyval_string(" , A=1").empty(),
           "leading empty field");
    auto m5 = StringFacet::parse_keyval_string("k=a=b");
    expect(m5["k"] == "a=b", "value keeps later separators");
  });
}

void solver_factory_cases() {
  run("solver_factory_string_constructor", [] {
    auto h = oracle::cpu_handlers();
    {
      auto s = it::create_LinearEigensystem("Davidson", "convergence_threshold=1e-3,max_size_qspace=73, n_roots=4", h);
      auto o = s->get_options();
      expect(o->convergence_threshold.has_value() && *o->convergence_threshold == 1e-3, "threshold");
      auto d = std::dynamic_pointer_cast<it::LinearEigensystemDavidsonOptions>(o);
      expect(d && d->norm_thresh.has_value() && d->norm_thresh.value_or(777) != 777, "norm_thresh");
      expect(d->max_size_qspace.value() == 73 && d->n_roots.value() == 4, "max_size_qspace, n_roots");
    }
    {
      auto s = it::create_LinearEquations("Davidson", "convergence_threshold=1e-3,max_size_qspace=73, rubbish=trash", h);
      auto d = std::dynamic_pointer_cast<it::LinearEquationsDavidsonOptions>(s->get_options());
      expect(d && *d->convergence_threshold == 1e-3 && d->norm_thresh.has_value() && d->max_size_qspace.value() == 73,
             "LinearEquations");
    }
    {
      auto s = it::create_NonLinearEquations("DIIS", "convergence_threshold=1e-3,max_size_qspace=73, rubbish=trash", h);
      auto d = std::dynamic_pointer_cast<it::NonLinearEquationsDIISOptions>(s->get_options());
      expect(d && *d->convergence_threshold == 1e-3 && d->norm_thresh.has_value() && d->max_size_qspace.value() == 73,
             "DIIS");
    }
    for (std::string m : {"BFGS", "SD"}) {
      auto s = it::create_Optimize(m, std::string("convergence_threshold=1e-3") + (m == "BFGS" ? ",max_size_qspace=73" : ""),
                                   h);
      auto o = s->get_options();
      expect(*o->convergence_threshold == 1e-3, m + " threshold");
      if (m == "BFGS") {
        auto b = std::dynamic_pointer_cast<it::OptimizeBFGSOptions>(o);
        expect(b && b->max_size_qspace.value() == 73, "BFGS max_size_qspace");
      } else {
        expect(std::dynamic_pointer_cast<it::OptimizeSDOptions>(o) != nullptr, "SD options type");
      }
    }
    {
      auto s = it::create_LinearEigensystem("RSPT", "norm_thresh=1e-9, SVD_THRESH=1e-11", h);
      auto r = std::dynamic_pointer_cast<it::LinearEigensystemRSPTOptions>(s->get_options());
      expect(r && *r->norm_thresh == 1e-9 && *r->svd_thresh == 1e-11, "RSPT thresholds");
    }
    expect(throws<std::runtime_error>([&] { it::create_LinearEigensystem("Lanczos", "", h); }), "unknown method");
    expect(throws<std::runtime_error>([&] { it::create_LinearEigensystem("Davidson", "bad", h); }), "bad option string");
  });
}

void qspace_cases() {
  // XSpace::update_qspace twice: new vectors are prepended to Q (QSpace.h:80-84) and S / H are the
  // overlaps of the Q vectors in that order (XSpace.h:30-83, QSpace.h:86-110).
  const size_t n = 7;
  std::mt19937_64 g(5);
  std::uniform_real_distribution<double> u(-1, 1);
  Mat A({n, n});
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j <= i; ++j) A(i, j) = A(j, i) = u(g) + (i == j ? 3.0 * i : 0.0);
  auto act = [&](const V& x) {
    V y(n, 0.0);
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j < n; ++j) y[i] += A(i, j) * x[j];
    return y;
  };
  std::vector<V> p;
  for (int k = 0; k < 3; ++k) {
    V v(n);
    for (auto& e : v) e = u(g);
    p.push_back(v);
  }
  auto h = oracle::cpu_handlers();
  auto dot = [](const V& a, const V& b) {
    double s = 0;
    for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
    return s;
  };
  run("qspace_prepend_and_blocks", [&] {
    it::subspace::XSpace<V, V, SP> xs(h, std::make_shared<it::Logger>());
    xs.set_hermiticity(true);
    std::vector<V> a01{act(p[0]), act(p[1])}, a2{act(p[2])};
    xs.update_qspace(CVecRef<V>{std::cref(p[0]), std::cref(p[1])}, cwrap(a01));
    xs.update_qspace(CVecRef<V>{std::cref(p[2])}, cwrap(a2));
    const auto q = xs.cparamsq();
    expect(q.size() == 3 && q[0].get() == p[2] && q[1].get() == p[0] && q[2].get() == p[1], "Q order: newest first");
    const std::vector<const V*> order{&p[2], &p[0], &p[1]};
    const auto& S = xs.data.at(it::subspace::EqnData::S);
    const auto& H = xs.data.at(it::subspace::EqnData::H);
    for (size_t i = 0; i < 3; ++i)
      for (size_t j = 0; j < 3; ++j) {
        expect(std::abs(S(i, j) - dot(*order[i], *order[j])) < 1e-12, "S(" + std::to_string(i) + "," + std::to_string(j) + ")");
        expect(std::abs(H(i, j) - dot(*order[i], act(*order[j]))) < 1e-12, "H");
      }
    xs.eraseq(1);  // p[0]
    expect(xs.dimensions().nQ == 2 && xs.cparamsq()[1].get() == p[1], "erase");
    const auto& S2 = xs.data.at(it::subspace::EqnData::S);
    expect(S2.rows() == 2 && std::abs(S2(0, 1) - dot(p[2], p[1])) < 1e-12, "S after erase");
  });
}

// The host algebra's fast paths against their plain forms (dense.h): the register-tiled products are
// the triple loop's numbers, the eigenproblem's kept eigenvectors do not depend on how many are
// kept, and the redundancy screen's Cholesky proof never skips a decomposition that would have
// reported an eigenvalue at or below the threshold.
void dense_cases() {
  std::mt19937_64 g(11);
  std::uniform_real_distribution<double> u(-1, 1);
  run("ordered_gemm_is_the_triple_loop", [&] {
    for (size_t M : {1, 5, 8, 13, 64})
      for (size_t N : {1, 3, 4, 9})
        for (size_t K : {1, 7, 40}) {
          std::vector<double> A(M * K), B(K * N), C(M * N), R(M * N, 0.0);
          for (auto& x : A) x = u(g);
          for (auto& x : B) x = u(g);
          it::dense::ordered_gemm(M, N, K, A.data(), M, B.data(), K, C.data(), M);
          for (size_t j = 0; j < N; ++j)
            for (size_t l = 0; l < K; ++l)
              for (size_t i = 0; i < M; ++i) R[i + M * j] += A[i + M * l] * B[l + K * j];
          expect(std::memcmp(C.data(), R.data(), sizeof(double) * M * N) == 0, "bitwise");
        }
  });
  run("eigenproblem_kept_vectors", [&] {
    for (size_t n : {1, 6, 24, 40}) {
      std::vector<double> H(n * n), S(n * n, 0.0);
      for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j <= i; ++j) {
          H[i * n + j] = H[j * n + i] = u(g) + (i == j ? double(i) : 0.0);
          S[i * n + j] = S[j * n + i] = (i == j ? 1.0 : 1e-3 * u(g));
        }
      std::vector<double> v_all, e_all, v_few, e_few;
      it::eigenproblem(v_all, e_all, H, S, n, true, 1e-14, 0, true);
      const size_t keep = std::min<size_t>(3, n);
      it::eigenproblem(v_few, e_few, H, S, n, true, 1e-14, 0, true, keep);
      expect(e_all == e_few && e_all.size() == n, "eigenvalues of every root");
      expect(v_few.size() == n * keep && v_all.size() == n * n, "vector counts");
      expect(std::memcmp(v_all.data(), v_few.data(), sizeof(double) * n * keep) == 0, "kept vectors bitwise");
    }
  });
  run("screen_cholesky_proof", [&] {
    int proven = 0, skipped_wrongly = 0;
    for (int trial = 0; trial < 400; ++trial) {
      const size_t n = 2 + size_t(trial % 30), r = 1 + size_t(trial % 7);
      // Gram matrices of n vectors in d dimensions, some near-dependent, and scaled
      const size_t d = (trial % 4 == 0 && n > r) ? n - r : n;  // rank-deficient every fourth trial
      std::vector<double> X(n * d);
      for (auto& x : X) x = u(g);
      if (trial % 5 == 1)
        for (size_t j = 0; j < d; ++j) X[(n - 1) * d + j] = X[j] + 1e-9 * u(g);
      const double scale = std::pow(10.0, double(trial % 9) - 4.0);
      std::vector<double> A(n * n);
      for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j < n; ++j) {
          double s = 0;
          for (size_t k = 0; k < d; ++k) s += X[i * d + k] * X[j * d + k];
          A[i * n + j] = scale * s;
        }
      for (double thresh : {1e-12, 1e-8 * scale}) {
        const bool ok = it::dense::eigenvalues_exceed(n, A, thresh);
        const bool none = it::svd_system(n, n, A, thresh, true).empty();
        proven += ok;
        skipped_wrongly += ok && !none;
      }
    }
    expect(skipped_wrongly == 0, "a proof skipped a decomposition with an eigenvalue <= threshold");
    expect(proven > 200, "the proof holds on the well-conditioned cases");
    std::vector<double> nan(9, 0.0);
    nan[0] = nan[4] = nan[8] = 1.0;
    nan[4] = std::nan("");
    expect(!it::dense::eigenvalues_exceed(3, nan, 1e-12), "NaN: not proven");
    expect(!it::dense::eigenvalues_exceed(0, {}, 1e-12), "empty: not proven");
  });
}

// test_svd_system.cpp:17-35: the symmetric test matrix from the C library's rand() (unseeded).
void svd_dump() {
  const size_t dim = 5;
  std::vector<double> m(dim * dim, 0.0);
  for (size_t i = 0; i < dim; i++)
    for (size_t j = 0; j < dim; j++) {
      if (i <= j) {
        float r2 = static_cast<float>(rand()) / (static_cast<float>(RAND_MAX / 1.0));
        m[i + j * dim] = i == j ? double(i + 1) : 0.01 * r2 * double(i + j);
      } else {
        m[i + j * dim] = m[j + i * dim];
      }
    }
  std::vector<double> vecs(dim * dim), vals(dim);
  it::eigensolver_lapacke_dsyev(m, vecs, vals, dim);
  auto svds = it::svd_system(dim, dim, m, 1e300, true);
  auto list = [](const std::vector<double>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i]).substr(0, 0);
    char b[64];
    s = "[";
    for (size_t i = 0; i < v.size(); ++i) {
      std::snprintf(b, sizeof b, "%s%.17g", i ? "," : "", v[i]);
      s += b;
    }
    return s + "]";
  };
  std::vector<double> sv, sval;
  for (auto& x : svds) {
    sval.push_back(x.value);
    sv.insert(sv.end(), x.v.begin(), x.v.end());
  }
  std::printf("{\"dim\": %zu, \"matrix\": %s, \"eigenvalues\": %s, \"eigenvectors\": %s, \"svd_values\": %s, "
              "\"svd_vectors\": %s}\n",
              dim, list(m).c_str(), list(vals).c_str(), list(vecs).c_str(), list(sval).c_str(), list(sv).c_str());
}
}  // namespace

// "sym_eigen" mode: reads n and an n x n row-major matrix from stdin, prints the restated
// dense::sym_eigen result (eigenvalues ascending, then the eigenvector columns) for the Python side.
int sym_eigen_io() {
  size_t n = 0;
  if (std::scanf("%zu", &n) != 1) return 2;
  std::vector<double> a(n * n);
  for (auto& x : a)
    if (std::scanf("%lf", &x) != 1) return 2;
  std::vector<double> ev, vec;
  it::dense::sym_eigen(n, a, ev, vec);
  for (double x : ev) std::printf("%.17g\n", x);
  for (double x : vec) std::printf("%.17g\n", x);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "svd") {
    svd_dump();
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "sym_eigen") return sym_eigen_io();
  subspace_util_cases();
  dspace_resetter_cases();
  itsolv_util_cases();
  solver_factory_cases();
  qspace_cases();
  dense_cases();
  std::printf("%s %d failure(s)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
