// subspace::Matrix: the cases of the reference's test/itsolv/subspace/testMatrix.cpp:1-238, built
// against the restated itsolv_hbm/matrix.h (default) or the reference's own
// molpro/linalg/itsolv/subspace/Matrix.h (-DWITH_REFERENCE_BASE -I<reference>/src), so both must
// behave the same.  Run by tests/test_host_layer_cpp.py.
#include <array>
#include <cstdio>
#include <functional>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#ifdef WITH_REFERENCE_BASE
#include <molpro/linalg/itsolv/subspace/Matrix.h>
#else
#include "itsolv_hbm/matrix.h"
#endif

using molpro::linalg::itsolv::subspace::Matrix;
using molpro::linalg::itsolv::subspace::transpose_copy;
using M = Matrix<double>;
using coord = M::coord_type;

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
bool all_eq(const std::vector<double>& v, double x) {
  for (double e : v)
    if (e != x) return false;
  return true;
}
bool all_ne(const std::vector<double>& a, const std::vector<double>& b) {
  for (size_t i = 0; i < a.size(); ++i)
    if (a[i] == b[i]) return false;
  return true;
}
const size_t r = 3, c = 4;
M iota_matrix() {
  M m({r, c});
  for (size_t i = 0, ij = 0; i < m.rows(); ++i)
    for (size_t j = 0; j < m.cols(); ++j, ++ij) m(i, j) = double(ij);
  return m;
}
}  // namespace

int main() {
#ifdef WITH_REFERENCE_BASE
  std::printf("base: reference molpro/linalg/itsolv/subspace/Matrix.h\n");
#else
  std::printf("base: restated itsolv_hbm/matrix.h\n");
#endif
  run("default_constructor", [] {
    M m;
    expect(m.rows() == 0 && m.cols() == 0 && m.size() == 0 && m.dimensions() == coord{0, 0}, "empty");
  });
  run("constructor", [] {
    M m({3, 5});
    expect(m.rows() == 3 && m.cols() == 5 && m.size() == 15 && m.dimensions() == coord{3, 5}, "dims");
  });
  run("to_coord", [] {
    M m({r, c});
    expect(m.to_coord(0) == coord{0, 0} && m.to_coord(1) == coord{0, 1} && m.to_coord(c) == coord{1, 0}, "coords");
    expect(m.to_coord(c + 1) == coord{1, 1} && m.to_coord(2 * c + 2) == coord{2, 2}, "coords 2");
    expect(m.to_coord(m.size() - 1) == coord{r - 1, c - 1}, "last");
    expect(throws<std::out_of_range>([&] { m.to_coord(m.size()); }), "out of range");
  });
  run("fill", [] {
    M m({r, c});
    m.fill(3.14);
    expect(all_eq(m.data(), 3.14), "fill");
  });
  run("assignment", [] {
    auto m = iota_matrix();
    std::vector<double> ref(m.size());
    std::iota(ref.begin(), ref.end(), 0.);
    expect(m.data() == ref, "iota");
  });
  run("remove_row", [] {
    auto m = iota_matrix();
    std::array<std::vector<double>, 3> ref{
        {{4, 5, 6, 7, 8, 9, 10, 11}, {0, 1, 2, 3, 8, 9, 10, 11}, {0, 1, 2, 3, 4, 5, 6, 7}}};
    for (size_t i = 0; i < 3; ++i) {
      auto m0 = m;
      m0.remove_row(i);
      expect(m0.dimensions() == coord{r - 1, c} && m0.data() == ref[i], "row " + std::to_string(i));
    }
  });
  run("remove_col", [] {
    auto m = iota_matrix();
    std::vector<size_t> cols{0, 2, 3};
    std::array<std::vector<double>, 3> ref{
        {{1, 2, 3, 5, 6, 7, 9, 10, 11}, {0, 1, 3, 4, 5, 7, 8, 9, 11}, {0, 1, 2, 4, 5, 6, 8, 9, 10}}};
    for (size_t i = 0; i < cols.size(); ++i) {
      auto m0 = m;
      m0.remove_col(cols[i]);
      expect(m0.dimensions() == coord{r, c - 1} && m0.data() == ref[i], "col " + std::to_string(cols[i]));
    }
  });
  run("remove_row_col", [] {
    auto m = iota_matrix();
    std::vector<std::pair<size_t, size_t>> rc{{0, 0}, {1, 2}, {2, 3}};
    std::array<std::vector<double>, 3> ref{{{5, 6, 7, 9, 10, 11}, {0, 1, 3, 8, 9, 11}, {0, 1, 2, 4, 5, 6}}};
    for (size_t i = 0; i < rc.size(); ++i) {
      auto m0 = m;
      m0.remove_row_col(rc[i].first, rc[i].second);
      expect(m0.dimensions() == coord{r - 1, c - 1} && m0.data() == ref[i], "case " + std::to_string(i));
    }
  });
  run("slice_constructor", [] {
    M m({r, c});
    m.slice({0, 0}, {0, 0});
    m.slice({0, 0}, {r, c});
    expect(throws<std::runtime_error>([&] { m.slice({0, 0}, {r + 1, c + 1}); }), "beyond the matrix");
    expect(throws<std::runtime_error>([&] { m.slice({size_t(-1), size_t(-1)}, {r, c}); }), "negative corner");
    expect(throws<std::runtime_error>([&] { m.slice({size_t(-1), 0}, {r, c + 1}); }), "negative + beyond");
  });
  run("slice_copy_empty", [] {
    M m({r, c});
    auto right = m;
    m.fill(0);
    right.fill(1);
    const auto ref = m.data();
    m.slice({0, 0}, {0, 0}) = right.slice({0, 0}, {0, 0});
    m.slice({0, 0}, {0, c}) = right.slice({0, 0}, {0, c});
    m.slice({0, 0}, {r, 0}) = right.slice({0, 0}, {r, 0});
    m.slice({r, 0}, {r, c}) = right.slice({r, 0}, {r, c});
    m.slice({0, c}, {r, c}) = right.slice({0, c}, {r, c});
    m.slice({r, c}, {r, c}) = right.slice({r, c}, {r, c});
    expect(m.data() == ref, "empty slices copy nothing");
  });
  run("slice_no_params", [] {
    M m({r, c});
    auto right = m;
    right.fill(0.1);
    expect(all_ne(m.data(), right.data()), "differ before");
    m.slice() = right;
    expect(m.data() == right.data(), "whole-matrix slice");
  });
  run("slice_copy_full_matrix", [] {
    M m({r, c});
    auto right = m;
    m.fill(0.);
    right.fill(3.14);
    expect(throws<std::runtime_error>([&] { m.slice({0, 0}, {1, 1}) = right.slice({0, 0}, {2, 2}); }),
           "incompatible dimensions");
    m.slice({0, 0}, m.dimensions()) = right.slice({0, 0}, m.dimensions());
    expect(m.data() == right.data(), "copied");
  });
  run("cslice_copy_full_matrix", [] {
    M m({r, c});
    auto right = m;
    m.fill(0.);
    right.fill(3.14);
    const auto cm = right;
    m.slice({0, 0}, m.dimensions()) = cm.slice({0, 0}, m.dimensions());
    expect(m.data() == right.data(), "copied from const");
  });
  run("slice_copy_block", [] {
    M m({r, c});
    const size_t br = r / 2, bc = c / 2;
    M right({br, bc});
    m.fill(3.14);
    std::vector<double> ref(m.size(), 3.14);
    for (size_t i = 0, ij = 0; i < br; ++i)
      for (size_t j = 0; j < bc; ++j, ++ij) {
        right(i, j) = double(ij);
        ref[i * bc + j] = double(ij);  // as the reference test indexes it
      }
    m.slice({0, 0}, {br, bc}) = right.slice({0, 0}, right.dimensions());
    expect(m.data() == ref, "block");
  });
  run("slice_axpy", [] {
    M m({r, c});
    auto right = m;
    m.fill(3.14);
    right.fill(1.1);
    m.slice().axpy(-0.5, right.slice());
    expect(all_eq(m.data(), 3.14 + -0.5 * 1.1), "axpy");
  });
  run("slice_scal", [] {
    M m({r, c});
    m.fill(3.14);
    m.slice().scal(-0.5);
    expect(all_eq(m.data(), 3.14 * -0.5), "scal");
  });
  run("transpose_copy", [] {
    const size_t nr = 4, nc = 3;
    M ml({nr, nc}), mr({nc, nr}), mref({nr, nc});
    for (size_t i = 0; i < nr; ++i)
      for (size_t j = 0; j < nc; ++j) {
        mr(j, i) = double(j);
        mref(i, j) = double(j);
      }
    transpose_copy(ml, mr);
    expect(ml.data() == mref.data(), "transpose");
  });
  run("resize_keeps_data", [] {
    auto m = iota_matrix();
    m.resize({r + 1, c + 1});
    expect(m.rows() == r + 1 && m.cols() == c + 1 && m(2, 3) == 11 && m(3, 4) == 0 && m(1, 4) == 0, "grown");
    m.resize({2, 2});
    expect(m.data() == std::vector<double>({0, 1, 4, 5}), "shrunk");
  });
  std::printf("%s %d failure(s)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
