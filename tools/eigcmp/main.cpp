#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
void old_sym(size_t, const std::vector<double>&, std::vector<double>&, std::vector<double>&);
void new_sym(size_t, const std::vector<double>&, std::vector<double>&, std::vector<double>&);
void old_eig(size_t, const std::vector<double>&, const std::vector<double>&, std::vector<double>&, std::vector<double>&);
void new_eig(size_t, const std::vector<double>&, const std::vector<double>&, std::vector<double>&, std::vector<double>&);
static bool same(const std::vector<double>& a, const std::vector<double>& b) {
  return a.size() == b.size() && (a.empty() || std::memcmp(a.data(), b.data(), a.size() * 8) == 0);
}
int main() {
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(-1, 1);
  long bad = 0, cases = 0;
  for (int rep = 0; rep < 30; ++rep)
    for (size_t n = 1; n <= 80; ++n)
      for (int kind = 0; kind < 5; ++kind) {
        std::vector<double> a(n * n, 0.0), s(n * n, 0.0);
        for (size_t i = 0; i < n; ++i)
          for (size_t j = 0; j <= i; ++j) {
            double v = 0;
            if (kind == 0) v = u(g);
            else if (kind == 1) v = (i == j ? 1.0 : (j + 1 == i ? 1e-3 * u(g) : 0.0));
            else if (kind == 2) v = (i == j ? double(i) : 0.0) + (u(g) > 0.7 ? u(g) : 0.0);
            else if (kind == 3) v = (i == j ? 1.0 : 0.0);
            else v = (i == j ? -0.0 : (u(g) > 0.5 ? -0.0 : 1e-300 * u(g)));
            a[i * n + j] = a[j * n + i] = v;
            const double w = (i == j ? 1.0 + 0.1 * std::abs(u(g)) : 1e-2 * u(g));
            s[i * n + j] = s[j * n + i] = w;
          }
        std::vector<double> e1, v1, e2, v2;
        int t1 = 0, t2 = 0;
        try { old_sym(n, a, e1, v1); } catch (...) { t1 = 1; }
        try { new_sym(n, a, e2, v2); } catch (...) { t2 = 1; }
        if (t1 != t2) { printf("throw differs n=%zu kind=%d\n", n, kind); ++bad; }
        ++cases;
        if (!same(e1, e2) || !same(v1, v2)) { if (bad < 5) printf("sym_eigen differs n=%zu kind=%d\n", n, kind); ++bad; }
        if (kind == 2) {  // a rank-deficient metric: S = B B^T, B n x (n/2 + 1)
          const size_t r = n / 2 + 1;
          std::vector<double> B(n * r);
          for (auto& b : B) b = u(g);
          for (size_t i = 0; i < n; ++i)
            for (size_t j = 0; j < n; ++j) {
              double t = 0;
              for (size_t q = 0; q < r; ++q) t += B[i * r + q] * B[j * r + q];
              s[i * n + j] = t;
            }
        }
        if (kind != 4) {
          std::vector<double> x1, l1, x2, l2;
          int u1 = 0, u2 = 0;
          try { old_eig(n, a, s, x1, l1); } catch (...) { u1 = 1; }
          try { new_eig(n, a, s, x2, l2); } catch (...) { u2 = 1; }
          if (u1 != u2) { printf("eig throw differs n=%zu kind=%d\n", n, kind); ++bad; }
          ++cases;
          if (!same(x1, x2) || !same(l1, l2)) { if (bad < 5) printf("eigenproblem differs n=%zu kind=%d\n", n, kind); ++bad; }
        }
      }
  printf("cases %ld differing %ld\n", cases, bad);
  return bad != 0;
}
