// Host dense subspace algebra timings (development tool): sym_eigen, eigenproblem, svd_system at the
// subspace sizes of the C3/C4 solves.  Build: g++ -O3 -march=x86-64-v3 -ffp-contract=off -std=c++17
//   -I iterative-solver_amd/include -I include tools/hostalg_bench.cpp -o tools/hostalg_bench
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
#include "itsolv_hbm/dense.h"
using namespace molpro::linalg::itsolv;
int main() {
  for (size_t n : {24, 48, 64, 72}) {
    std::mt19937 g(1);
    std::uniform_real_distribution<double> u(-1, 1);
    std::vector<double> a(n * n), s(n * n, 0.0);
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j <= i; ++j) a[i * n + j] = a[j * n + i] = u(g) + (i == j ? double(i) : 0.0);
    for (size_t i = 0; i < n; ++i) s[i * n + i] = 1.0;
    for (size_t i = 0; i + 1 < n; ++i) s[i * n + i + 1] = s[(i + 1) * n + i] = 1e-3;
    auto t0 = std::chrono::steady_clock::now();
    int reps = 200;
    for (int r = 0; r < reps; ++r) {
      std::vector<double> ev, val;
      eigenproblem(ev, val, a, s, n, true, 1e-14, 0, true);
    }
    auto t1 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
      auto sv = svd_system(n, n, s, 1e-12, true);
    }
    auto t2 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
      std::vector<double> ev, vec;
      dense::sym_eigen(n, a, ev, vec);
    }
    auto t3 = std::chrono::steady_clock::now();
    auto us = [&](auto x, auto y) { return std::chrono::duration<double, std::micro>(y - x).count() / reps; };
    printf("n=%zu eigenproblem %.1f us  svd_system %.1f us  sym_eigen %.1f us\n", n, us(t0, t1), us(t1, t2),
           us(t2, t3));
  }
}
