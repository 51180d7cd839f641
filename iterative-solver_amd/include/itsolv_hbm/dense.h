// Small dense linear algebra of the subspace problem (host, matrices of at most a few hundred rows).
//
// The reference delegates these to LAPACKE dsyev and Eigen 3.3.7 (reference
// itsolv/helper-implementation.h).  Neither is available here, so they are restated on top of one
// symmetric eigensolver of dsyev's method (Householder tridiagonalisation + implicit QL, backward
// stable; pinned against LAPACK in tests/test_host_layer_cpp.py), reproducing the reference's
// conventions:
//   * eigensolver_lapacke_dsyev: eigenvalues ascending, eigenvector i in column i   (:122-158)
//   * svd_system(hermitian): eigenpairs listed largest first, value <= threshold kept (:184-192, :263-296)
//   * get_rank: count of eigenvalues >= threshold * max                              (:221-231)
//   * eigenproblem: Hbar = S^-1/2 U^T H U S^-1/2 on the first `rank` eigenpairs of S in ascending
//     order, eigenvalues ascending, back-transform, sign fixed so that the largest-|.| component is
//     positive                                                                        (:318-543)
//   * solve_DIIS: augmented [B -1; -1 0] system solved by a pseudo-inverse (SVD threshold 0) (:619-669)
// The non-hermitian branch (JacobiSVD of S + general real EigenSolver) uses a one-sided Jacobi SVD and
// a Hessenberg-QR eigensolver; those paths are only exercised by the non-hermitian tests.
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <limits>
#include <list>
#include <numeric>
#include <stdexcept>
#include <vector>

namespace molpro::linalg::itsolv {

template <typename T>
struct SVD {
  using value_type = T;
  value_type value;
  std::vector<value_type> u;
  std::vector<value_type> v;
};

namespace dense {

// Host time of the subspace algebra (instrumentation only): the outermost eigenproblem /
// svd_system / solve_DIIS / solve_LinearEquations call of this thread adds its wall time, its
// count and its dimension; run_davidson / run_diis reset it per solve and report it in
// itsolv_result.host_algebra_*.  Two clock reads per call.
struct AlgebraClock {
  static inline thread_local double seconds = 0;
  static inline thread_local int calls = 0;
  static inline thread_local int depth = 0;
  static inline thread_local size_t max_dim = 0;
  static void reset() { seconds = 0, calls = 0, depth = 0, max_dim = 0; }
};
class AlgebraScope {
 public:
  explicit AlgebraScope(size_t dim) : m_outer(AlgebraClock::depth++ == 0) {
    if (m_outer) {
      m_t0 = std::chrono::steady_clock::now();
      AlgebraClock::max_dim = std::max(AlgebraClock::max_dim, dim);
    }
  }
  ~AlgebraScope() {
    --AlgebraClock::depth;
    if (m_outer) {
      AlgebraClock::seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - m_t0).count();
      ++AlgebraClock::calls;
    }
  }
  AlgebraScope(const AlgebraScope&) = delete;
  AlgebraScope& operator=(const AlgebraScope&) = delete;

 private:
  bool m_outer;
  std::chrono::steady_clock::time_point m_t0;
};

// True when every eigenvalue that sym_eigen would compute for the symmetric n x n matrix a (row-major,
// either triangle) is certainly above `thresh`: the Cholesky factorisation of a - tau I runs to the
// end with positive pivots, tau = thresh + margin.  A factorisation that succeeds in floating point
// proves lambda_min(a) > tau - (n + 1) eps max_i a_ii (its backward error), and sym_eigen's
// eigenvalues lie within a small multiple of n eps ||a||_F of the exact ones (backward-stable
// Householder + QL); margin = 1e3 n eps ||a||_F covers both with room to spare.  A false return
// only means "not proven" (near-null directions, NaN, n = 0): the caller then decomposes.  O(n^3 / 6),
// against O(9 n^3) for the decomposition it lets the redundancy screen skip.
inline bool eigenvalues_exceed(size_t n, const std::vector<double>& a, double thresh) {
  if (n == 0 || a.size() < n * n) return false;
  AlgebraScope clock_(n);
  double fro = 0;
  for (size_t i = 0; i < n * n; ++i) fro += a[i] * a[i];
  fro = std::sqrt(fro);
  if (!(fro < std::numeric_limits<double>::infinity())) return false;
  const double tau = std::max(thresh, 0.0) + 1e3 * double(n) * std::numeric_limits<double>::epsilon() * fro;
  std::vector<double> L(n * n, 0.0);  // lower triangle, row-major
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j <= i; ++j) {
      double s = 0.5 * (a[i * n + j] + a[j * n + i]) - (i == j ? tau : 0.0);
      for (size_t k = 0; k < j; ++k) s -= L[i * n + k] * L[j * n + k];
      if (i == j) {
        if (!(s > 0)) return false;
        L[i * n + i] = std::sqrt(s);
      } else {
        L[i * n + j] = s / L[j * n + j];
      }
    }
  return true;
}

// C = A B (column-major; A M x K, lda; B K x N, ldb; C M x N, ldc), each element the sum over
// l = 0..K-1 in order of the rounded products A[i,l] B[l,j] -- the numbers of the plain triple loop
// (with -ffp-contract=off, as every host build here is) -- in 8 x 4 register tiles: the same
// operations per element, several elements per instruction.
inline void ordered_gemm(size_t M, size_t N, size_t K, const double* A, size_t lda, const double* B, size_t ldb,
                         double* C, size_t ldc) {
  typedef double v4d __attribute__((vector_size(32), aligned(8), may_alias));
  size_t j = 0;
  for (; j + 4 <= N; j += 4) {
    size_t i = 0;
    for (; i + 8 <= M; i += 8) {
      v4d c[4][2] = {};
      const double* b = B + ldb * j;
      for (size_t l = 0; l < K; ++l) {
        const double* a = A + lda * l + i;
        const v4d a0 = *reinterpret_cast<const v4d*>(a), a1 = *reinterpret_cast<const v4d*>(a + 4);
        for (int q = 0; q < 4; ++q) {
          const double bq = b[l + ldb * size_t(q)];
          c[q][0] = c[q][0] + a0 * bq;
          c[q][1] = c[q][1] + a1 * bq;
        }
      }
      for (int q = 0; q < 4; ++q) {
        *reinterpret_cast<v4d*>(C + i + ldc * (j + size_t(q))) = c[q][0];
        *reinterpret_cast<v4d*>(C + i + 4 + ldc * (j + size_t(q))) = c[q][1];
      }
    }
    for (; i < M; ++i)
      for (size_t q = 0; q < 4; ++q) {
        double s = 0;
        for (size_t l = 0; l < K; ++l) s += A[i + lda * l] * B[l + ldb * (j + q)];
        C[i + ldc * (j + q)] = s;
      }
  }
  for (; j < N; ++j)
    for (size_t i = 0; i < M; ++i) {
      double s = 0;
      for (size_t l = 0; l < K; ++l) s += A[i + lda * l] * B[l + ldb * j];
      C[i + ldc * j] = s;
    }
}

// Symmetric eigen-decomposition of the n x n matrix a (either storage order: only the symmetric
// part is used).  On return evals is ascending and column i of evecs (evecs[j + n*i]) is the
// unit eigenvector of evals[i].
//
// The method of the reference's own solvers (LAPACK dsyev = dsytrd + dsteqr, helper-implementation.h:
// 122-158; Eigen's SelfAdjointEigenSolver, :356-382): Householder reduction to tridiagonal form with
// the transformations accumulated, then the implicit QL iteration with Wilkinson-type shifts on the
// tridiagonal matrix, rotations applied to the accumulated basis.  O(n^3) with a small constant:
// 0.1 ms at n = 72 against 1.6 ms for cyclic Jacobi (which the host side of every iteration runs
// two to four times; at the C4 shard size it was a fifth of the solve).
inline void sym_eigen(size_t n, const std::vector<double>& a, std::vector<double>& evals, std::vector<double>& evecs) {
  // Z: row-major working matrix, ends as the accumulated orthogonal basis (columns = eigenvectors).
  std::vector<double> Z(n * n);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) Z[i * n + j] = 0.5 * (a[i * n + j] + a[j * n + i]);
  std::vector<double> d(n, 0.0), e(n, 0.0), gacc_t(n, 0.0);
  if (n == 0) {
    evals.clear();
    evecs.clear();
    return;
  }
  // Householder tridiagonalisation, last row first: row i is reduced against columns 0..i-1.
  for (size_t i = n - 1; i > 0; --i) {
    const size_t l = i - 1;
    double h = 0, scale = 0;
    if (l > 0) {
      for (size_t k = 0; k <= l; ++k) scale += std::abs(Z[i * n + k]);
      if (scale == 0) {
        e[i] = Z[i * n + l];
      } else {
        for (size_t k = 0; k <= l; ++k) {
          Z[i * n + k] /= scale;
          h += Z[i * n + k] * Z[i * n + k];
        }
        double f = Z[i * n + l];
        const double g = f >= 0 ? -std::sqrt(h) : std::sqrt(h);
        e[i] = scale * g;
        h -= f * g;
        Z[i * n + l] = f - g;
        f = 0;
        // gg_j = sum_{k<=j} Z[j][k] z_k, then + Z[k][j] z_k for k = j+1..l, in that order (the
        // symmetric product with the lower triangle, z = row i).  The second part is accumulated
        // row k at a time (unit stride) -- each gg_j still receives its terms in increasing k.
        // Column i, written here, is read by none of these sums (they read columns <= l < i).
        const double* zi = &Z[i * n];
        for (size_t j = 0; j <= l; ++j) {
          Z[j * n + i] = zi[j] / h;
          double gg = 0;
          for (size_t k = 0; k <= j; ++k) gg += Z[j * n + k] * zi[k];
          gacc_t[j] = gg;
        }
        for (size_t k = 1; k <= l; ++k) {
          const double zk = zi[k];
          const double* rk = &Z[k * n];
          for (size_t j = 0; j < k; ++j) gacc_t[j] += rk[j] * zk;
        }
        for (size_t j = 0; j <= l; ++j) {
          e[j] = gacc_t[j] / h;
          f += e[j] * zi[j];
        }
        const double hh = f / (h + h);
        for (size_t j = 0; j <= l; ++j) {
          const double fj = Z[i * n + j];
          const double gj = e[j] - hh * fj;
          e[j] = gj;
          for (size_t k = 0; k <= j; ++k) Z[j * n + k] -= fj * e[k] + gj * Z[i * n + k];
        }
      }
    } else {
      e[i] = Z[i * n + l];
    }
    d[i] = h;
  }
  d[0] = 0;
  e[0] = 0;
  // Accumulate the transformations.  For row i, g_j = sum_k Z[i][k] Z[k][j] (k = 0..i-1 in order)
  // reads row i and column j only, and the update of column j touches neither row i nor any other
  // column, so all g_j are formed first and the columns updated after -- the same operations on
  // every element in the same order as the column-at-a-time loop, with unit-stride inner loops.
  std::vector<double> gacc(n);
  for (size_t i = 0; i < n; ++i) {
    if (d[i] != 0) {
      std::fill(gacc.begin(), gacc.begin() + long(i), 0.0);
      for (size_t k = 0; k < i; ++k) {
        const double zik = Z[i * n + k];
        const double* zk = &Z[k * n];
        for (size_t j = 0; j < i; ++j) gacc[j] += zik * zk[j];
      }
      for (size_t k = 0; k < i; ++k) {
        const double zki = Z[k * n + i];
        double* zk = &Z[k * n];
        for (size_t j = 0; j < i; ++j) zk[j] -= gacc[j] * zki;
      }
    }
    d[i] = Z[i * n + i];
    Z[i * n + i] = 1;
    for (size_t j = 0; j < i; ++j) Z[j * n + i] = Z[i * n + j] = 0;
  }
  // The basis transposed: W row i = column i of Z, so each QL rotation updates two contiguous rows.
  std::vector<double> W(n * n);
  for (size_t i = 0; i < n; ++i)
    for (size_t k = 0; k < n; ++k) W[i * n + k] = Z[k * n + i];
  // Implicit QL with shifts on (d, e); e[i] couples d[i-1] and d[i] -> shift down by one.
  for (size_t i = 1; i < n; ++i) e[i - 1] = e[i];
  e[n - 1] = 0;
  const double eps = std::numeric_limits<double>::epsilon();
  for (size_t l = 0; l < n; ++l) {
    for (int iter = 0;; ++iter) {
      size_t m = l;
      for (; m + 1 < n; ++m) {
        const double dd = std::abs(d[m]) + std::abs(d[m + 1]);
        if (std::abs(e[m]) <= eps * dd) break;
      }
      if (m == l) break;
      if (iter == 60) throw std::runtime_error("sym_eigen: QL iteration did not converge");
      double g = (d[l + 1] - d[l]) / (2 * e[l]);
      double r = std::hypot(g, 1.0);
      g = d[m] - d[l] + e[l] / (g + (g >= 0 ? r : -r));
      double s = 1, c = 1, p = 0;
      bool deflated = false;
      for (size_t i = m; i-- > l;) {
        double f = s * e[i];
        const double b = c * e[i];
        r = std::hypot(f, g);
        e[i + 1] = r;
        if (r == 0) {
          d[i + 1] -= p;
          e[m] = 0;
          deflated = true;
          break;
        }
        s = f / r;
        c = g / r;
        g = d[i + 1] - p;
        r = (d[i] - g) * s + 2 * c * b;
        p = s * r;
        d[i + 1] = g + p;
        g = c * r - b;
        double* wi = &W[i * n];
        double* wj = &W[(i + 1) * n];
        for (size_t k = 0; k < n; ++k) {
          const double wk1 = wj[k], wk0 = wi[k];
          wj[k] = s * wk0 + c * wk1;
          wi[k] = c * wk0 - s * wk1;
        }
      }
      if (deflated) continue;
      d[l] -= p;
      e[l] = g;
      e[m] = 0;
    }
  }
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return d[x] < d[y]; });
  evals.resize(n);
  evecs.assign(n * n, 0.0);
  for (size_t i = 0; i < n; ++i) {
    evals[i] = d[order[i]];
    for (size_t j = 0; j < n; ++j) evecs[j + n * i] = W[order[i] * n + j];
  }
}

// One-sided Jacobi SVD of the nrows x ncols column-major matrix m (nrows >= ncols assumed padded):
// singular values descending, thin U (nrows x ncols) and V (ncols x ncols), column-major.
inline void jacobi_svd(size_t nrows, size_t ncols, const std::vector<double>& m, std::vector<double>& sv,
                       std::vector<double>& U, std::vector<double>& V) {
  const size_t n = ncols, r = std::max(nrows, ncols);
  std::vector<double> W(r * n, 0.0);  // column-major r x n
  for (size_t j = 0; j < n; ++j)
    for (size_t i = 0; i < nrows; ++i) W[i + r * j] = m[i + nrows * j];
  std::vector<double> Vm(n * n, 0.0);
  for (size_t i = 0; i < n; ++i) Vm[i + n * i] = 1;
  for (int sweep = 0; sweep < 100; ++sweep) {
    bool rotated = false;
    for (size_t p = 0; p + 1 < n; ++p)
      for (size_t q = p + 1; q < n; ++q) {
        double alpha = 0, beta = 0, gamma = 0;
        for (size_t i = 0; i < r; ++i) {
          alpha += W[i + r * p] * W[i + r * p];
          beta += W[i + r * q] * W[i + r * q];
          gamma += W[i + r * p] * W[i + r * q];
        }
        if (gamma == 0 || std::abs(gamma) <= 1e-16 * std::sqrt(alpha * beta)) continue;
        rotated = true;
        const double zeta = (beta - alpha) / (2 * gamma);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::abs(zeta) + std::sqrt(1 + zeta * zeta));
        const double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (size_t i = 0; i < r; ++i) {
          const double wp = W[i + r * p], wq = W[i + r * q];
          W[i + r * p] = c * wp - s * wq;
          W[i + r * q] = s * wp + c * wq;
        }
        for (size_t i = 0; i < n; ++i) {
          const double vp = Vm[i + n * p], vq = Vm[i + n * q];
          Vm[i + n * p] = c * vp - s * vq;
          Vm[i + n * q] = s * vp + c * vq;
        }
      }
    if (!rotated) break;
  }
  std::vector<double> norms(n);
  for (size_t j = 0; j < n; ++j) {
    double s = 0;
    for (size_t i = 0; i < r; ++i) s += W[i + r * j] * W[i + r * j];
    norms[j] = std::sqrt(s);
  }
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return norms[x] > norms[y]; });
  sv.resize(n);
  U.assign(nrows * n, 0.0);
  V.assign(n * n, 0.0);
  for (size_t k = 0; k < n; ++k) {
    const size_t j = order[k];
    sv[k] = norms[j];
    for (size_t i = 0; i < nrows; ++i) U[i + nrows * k] = norms[j] > 0 ? W[i + r * j] / norms[j] : 0.0;
    for (size_t i = 0; i < n; ++i) V[i + n * k] = Vm[i + n * j];
  }
}

// Eigenvalues / eigenvectors of a general real n x n matrix (column-major), via Hessenberg reduction
// and the shifted QR algorithm on the complex Schur form (small n only).
inline void general_eigen(size_t n, const std::vector<double>& a, std::vector<std::complex<double>>& evals,
                          std::vector<std::complex<double>>& evecs) {
  using cd = std::complex<double>;
  // Complex Schur via unshifted-then-Wilkinson-shifted QR on the complex matrix (n is tiny).
  std::vector<cd> T(n * n), Q(n * n, cd(0));
  for (size_t i = 0; i < n; ++i) {
    Q[i + n * i] = 1;
    for (size_t j = 0; j < n; ++j) T[i + n * j] = a[i + n * j];
  }
  auto givens = [&](size_t k, cd x, cd y, cd& c, cd& s) {
    double r = std::sqrt(std::norm(x) + std::norm(y));
    if (r == 0) {
      c = 1;
      s = 0;
      return;
    }
    c = x / r;
    s = y / r;
  };
  // Unitary reduction to upper Hessenberg form (Givens rotations, accumulated in Q): the shifted
  // QR sweeps below and their subdiagonal deflation test assume it.
  for (size_t j = 0; j + 2 < n; ++j)
    for (size_t i = n - 1; i >= j + 2; --i) {
      const cd x = T[(i - 1) + n * j], y = T[i + n * j];
      if (std::abs(y) == 0) continue;
      cd c, s;
      givens(0, x, y, c, s);
      for (size_t k = 0; k < n; ++k) {
        const cd a = T[(i - 1) + n * k], b = T[i + n * k];
        T[(i - 1) + n * k] = std::conj(c) * a + std::conj(s) * b;
        T[i + n * k] = -s * a + c * b;
      }
      for (size_t k = 0; k < n; ++k) {
        const cd a = T[k + n * (i - 1)], b = T[k + n * i];
        T[k + n * (i - 1)] = a * c + b * s;
        T[k + n * i] = -a * std::conj(s) + b * std::conj(c);
        const cd qa = Q[k + n * (i - 1)], qb = Q[k + n * i];
        Q[k + n * (i - 1)] = qa * c + qb * s;
        Q[k + n * i] = -qa * std::conj(s) + qb * std::conj(c);
      }
      T[i + n * j] = 0;
    }
  for (size_t hi = n; hi > 1;) {
    int iter = 0;
    for (;;) {
      const double sub = std::abs(T[(hi - 1) + n * (hi - 2)]);
      const double scale = std::abs(T[(hi - 1) + n * (hi - 1)]) + std::abs(T[(hi - 2) + n * (hi - 2)]);
      if (sub <= 1e-15 * (scale > 0 ? scale : 1) || iter > 300) {
        T[(hi - 1) + n * (hi - 2)] = 0;
        --hi;
        break;
      }
      ++iter;
      // Wilkinson shift from the trailing 2x2 block.
      cd a11 = T[(hi - 2) + n * (hi - 2)], a12 = T[(hi - 2) + n * (hi - 1)], a21 = T[(hi - 1) + n * (hi - 2)],
         a22 = T[(hi - 1) + n * (hi - 1)];
      cd tr = a11 + a22, det = a11 * a22 - a12 * a21;
      cd disc = std::sqrt(tr * tr / 4.0 - det);
      cd mu1 = tr / 2.0 + disc, mu2 = tr / 2.0 - disc;
      cd mu = std::abs(mu1 - a22) < std::abs(mu2 - a22) ? mu1 : mu2;
      if (iter % 11 == 0) mu += cd(std::abs(a21), 0);  // exceptional shift
      for (size_t i = 0; i < hi; ++i) T[i + n * i] -= mu;
      std::vector<cd> cs(hi), sn(hi);
      for (size_t k = 0; k + 1 < hi; ++k) {
        cd c, s;
        givens(k, T[k + n * k], T[(k + 1) + n * k], c, s);
        cs[k] = c;
        sn[k] = s;
        for (size_t j = 0; j < n; ++j) {
          cd x = T[k + n * j], y = T[(k + 1) + n * j];
          T[k + n * j] = std::conj(c) * x + std::conj(s) * y;
          T[(k + 1) + n * j] = -s * x + c * y;
        }
      }
      for (size_t k = 0; k + 1 < hi; ++k) {
        cd c = cs[k], s = sn[k];
        for (size_t i = 0; i < n; ++i) {
          cd x = T[i + n * k], y = T[i + n * (k + 1)];
          T[i + n * k] = x * c + y * s;
          T[i + n * (k + 1)] = -x * std::conj(s) + y * std::conj(c);
          cd qx = Q[i + n * k], qy = Q[i + n * (k + 1)];
          Q[i + n * k] = qx * c + qy * s;
          Q[i + n * (k + 1)] = -qx * std::conj(s) + qy * std::conj(c);
        }
      }
      for (size_t i = 0; i < hi; ++i) T[i + n * i] += mu;
    }
  }
  evals.resize(n);
  for (size_t i = 0; i < n; ++i) evals[i] = T[i + n * i];
  // Eigenvectors of the triangular T by back substitution, then rotate by Q; unit 2-norm.
  evecs.assign(n * n, cd(0));
  for (size_t k = 0; k < n; ++k) {
    std::vector<cd> y(n, cd(0));
    y[k] = 1;
    for (size_t i = k; i-- > 0;) {
      cd s = 0;
      for (size_t j = i + 1; j <= k; ++j) s += T[i + n * j] * y[j];
      cd d = T[i + n * i] - T[k + n * k];
      if (std::abs(d) < 1e-300) d = 1e-300;
      y[i] = -s / d;
    }
    double nrm = 0;
    std::vector<cd> x(n, cd(0));
    for (size_t i = 0; i < n; ++i) {
      for (size_t j = 0; j <= k; ++j) x[i] += Q[i + n * j] * y[j];
      nrm += std::norm(x[i]);
    }
    nrm = std::sqrt(nrm);
    // Remove the arbitrary complex phase: the largest component becomes real positive, so the
    // eigenvector of a real eigenvalue is real (as Eigen::EigenSolver returns it).
    size_t big = 0;
    for (size_t i = 0; i < n; ++i)
      if (std::abs(x[i]) > std::abs(x[big])) big = i;
    const cd phase = std::abs(x[big]) > 0 ? x[big] / std::abs(x[big]) : cd(1);
    for (size_t i = 0; i < n; ++i) evecs[i + n * k] = x[i] / (nrm * phase);
  }
}

}  // namespace dense

// ---- reference helper conventions -----------------------------------------------------------------

// LAPACK dsyev role: eigenvalues ascending, eigenvectors column-major.  Returns 0.
inline int eigensolver_lapacke_dsyev(const std::vector<double>& matrix, std::vector<double>& eigenvectors,
                                     std::vector<double>& eigenvalues, const size_t dimension) {
  if (eigenvectors.size() != matrix.size())
    throw std::runtime_error("Matrix of eigenvectors and input matrix are not the same size!");
  if (eigenvectors.size() != dimension * dimension || eigenvalues.size() != dimension)
    throw std::runtime_error("Size of eigenvectors/eigenvlaues do not match dimension!");
  dense::sym_eigen(dimension, matrix, eigenvalues, eigenvectors);
  return 0;
}

// Eigenpairs of a symmetric matrix as a list, largest eigenvalue first (reference :167-195).
inline std::list<SVD<double>> eigensolver_lapacke_dsyev(size_t dimension, const std::vector<double>& matrix) {
  std::vector<double> vecs(dimension * dimension), vals(dimension);
  eigensolver_lapacke_dsyev(matrix, vecs, vals, dimension);
  std::list<SVD<double>> out;
  for (size_t i = dimension; i-- > 0;) {
    SVD<double> s;
    s.value = vals[i];
    s.v.assign(vecs.begin() + dimension * i, vecs.begin() + dimension * (i + 1));
    out.push_back(std::move(s));
  }
  return out;
}

template <typename value_type>
size_t get_rank(const std::vector<value_type>& eigenvalues, value_type threshold) {
  if (eigenvalues.empty()) return 0;
  const value_type thr = threshold * *std::max_element(eigenvalues.begin(), eigenvalues.end());
  return size_t(std::count_if(eigenvalues.begin(), eigenvalues.end(), [&](value_type v) { return v >= thr; }));
}

template <typename value_type>
size_t get_rank(const std::list<SVD<value_type>>& svds, value_type threshold) {
  value_type mx = 0;
  for (auto& s : svds) mx = std::max(mx, s.value);
  size_t r = 0;
  for (auto& s : svds)
    if (s.value > threshold * mx) ++r;
  return r;
}

// Singular (eigen, when hermitian) pairs with value below `threshold` (reference :263-296).
// m is row-major nrows x ncols.
inline std::list<SVD<double>> svd_system(size_t nrows, size_t ncols, const std::vector<double>& m, double threshold,
                                         bool hermitian = false, bool reduce_to_rank = false) {
  dense::AlgebraScope clock_(std::max(nrows, ncols));
  std::list<SVD<double>> svds;
  if (m.empty()) return svds;
  if (hermitian) {
    svds = eigensolver_lapacke_dsyev(nrows, m);
    for (auto s = svds.begin(); s != svds.end();)
      if (s->value > threshold)
        s = svds.erase(s);
      else
        ++s;
  } else {
    // Eigen::Map<Matrix> of the row-major buffer reads it column-major: the SVD is of m^T viewed
    // as nrows x ncols column-major, exactly as the reference's svd_eigen_jacobi does.
    std::vector<double> sv, U, V;
    dense::jacobi_svd(nrows, ncols, m, sv, U, V);
    for (size_t i = ncols; i-- > 0;) {
      if (std::abs(sv[i]) < threshold) {
        SVD<double> t;
        t.value = sv[i];
        for (size_t j = 0; j < ncols; ++j) t.v.push_back(V[j + ncols * i]);
        svds.push_back(std::move(t));
      }
    }
  }
  if (reduce_to_rank) {
    const size_t rank = get_rank(svds, threshold);
    for (size_t i = ncols; i > rank && !svds.empty(); --i) svds.pop_back();
  }
  return svds;
}

// Generalised eigenproblem H c = e S c of the subspace (reference :318-543).  matrix (H) is
// row-major, metric (S) is read column-major as the reference's Eigen::Map does (S is symmetric in
// the hermitian case).  eigenvectors: column-major dimension x nsol (column k = root k).  nvec
// (hermitian case): only the eigenvectors of the nvec lowest roots are formed (the Davidson solver
// keeps nroots of them; eigenvalues are returned for every root).
inline void eigenproblem(std::vector<double>& eigenvectors, std::vector<double>& eigenvalues,
                         const std::vector<double>& matrix, const std::vector<double>& metric, size_t dimension,
                         bool hermitian, double svdThreshold, int verbosity, bool condone_complex,
                         size_t nvec = std::numeric_limits<size_t>::max()) {
  dense::AlgebraScope clock_(dimension);
  using cd = std::complex<double>;
  const size_t n = dimension;
  std::vector<double> H(n * n);  // column-major copy of the row-major input
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) H[i + n * j] = matrix[i * n + j];
  std::vector<double> sing, U, V;  // U, V column-major n x n
  size_t rank = 0;
  if (hermitian) {
    std::vector<double> vecs(n * n), vals(n);
    if (eigensolver_lapacke_dsyev(metric, vecs, vals, n) != 0) throw std::runtime_error("Eigensolver did not converge");
    sing = vals;
    U = V = vecs;
    rank = get_rank(vals, svdThreshold);
  } else {
    dense::jacobi_svd(n, n, metric, sing, U, V);
    // Eigen's JacobiSVD::rank(): singular values above max * max(n,n) * machine epsilon.
    const double thr = (sing.empty() ? 0 : sing[0]) * double(n) * std::numeric_limits<double>::epsilon();
    rank = size_t(std::count_if(sing.begin(), sing.end(), [&](double s) { return s > thr; }));
  }
  std::vector<double> svmh(rank);
  for (size_t k = 0; k < rank; ++k) svmh[k] = sing[k] > 1e-14 ? 1 / std::sqrt(sing[k]) : 0;
  // Hbar = diag(svmh) U_r^T H V_r diag(svmh)  (rank x rank, column-major): HV[i,j] = sum_l H[i,l]
  // V[l,j] and then Hbar[i,j] = svmh[i] (sum_l U[l,i] HV[l,j]) svmh[j], every sum over l = 0..n-1 in
  // order (ordered_gemm).
  std::vector<double> HV(n * rank);
  dense::ordered_gemm(n, rank, n, H.data(), n, V.data(), n, HV.data(), n);
  std::vector<double> Hbar(rank * rank), Ut(n * rank);
  for (size_t i = 0; i < rank; ++i)
    for (size_t l = 0; l < n; ++l) Ut[l * rank + i] = U[l + n * i];
  dense::ordered_gemm(rank, rank, n, Ut.data(), rank, HV.data(), n, Hbar.data(), rank);
  for (size_t j = 0; j < rank; ++j)
    for (size_t i = 0; i < rank; ++i) Hbar[i + rank * j] = svmh[i] * Hbar[i + rank * j] * svmh[j];
  if (hermitian) {
    // The Hermitian case in real arrays: the complex form below carries zero imaginary parts through
    // the back-transform, the sort and the sign fix, and its real parts are these numbers exactly
    // (the same operations in the same order), so the results are bit for bit the same.
    std::vector<double> ev, vec;
    dense::sym_eigen(rank, Hbar, ev, vec);
    // Selection sort ascending (first minimum wins) of all `rank` eigenvalues; the back-transformed
    // vectors X[:, k] = sum_l (V[:, l] svmh[l]) vec[l, k] (l in order) only for the first `nvec` of
    // that order -- each column is formed on its own, so the kept ones are the same numbers.
    std::vector<size_t> order;
    {
      std::vector<char> used(rank, 0);
      for (size_t k = 0; k < rank; ++k) {
        size_t ll = 0;
        while (used[ll]) ++ll;
        for (size_t l = 0; l < rank; ++l)
          if (!used[l] && ev[l] < ev[ll]) ll = l;
        used[ll] = 1;
        order.push_back(ll);
      }
    }
    const size_t nkeep = std::min(nvec, rank);
    std::vector<double> Vs(n * rank), Y(rank * nkeep);
    for (size_t l = 0; l < rank; ++l)
      for (size_t i = 0; i < n; ++i) Vs[i + n * l] = V[i + n * l] * svmh[l];
    for (size_t k = 0; k < nkeep; ++k)
      std::copy(vec.begin() + long(rank * order[k]), vec.begin() + long(rank * (order[k] + 1)), Y.begin() + long(rank * k));
    eigenvectors.resize(n * nkeep);
    eigenvalues.resize(rank);
    dense::ordered_gemm(n, nkeep, rank, Vs.data(), n, Y.data(), rank, eigenvectors.data(), n);
    for (size_t k = 0; k < rank; ++k) eigenvalues[k] = ev[order[k]];
    // sign fixed on the largest of the first `rank` components
    for (size_t k = 0; k < nkeep; ++k) {
      double* col = &eigenvectors[n * k];
      size_t mc = 0;
      for (size_t l = 0; l < rank && l < n; ++l)
        if (std::abs(col[l]) > std::abs(col[mc])) mc = l;
      if (col[mc] < 0)
        for (size_t i = 0; i < n; ++i) col[i] = -col[i];
    }
    (void)verbosity;
    (void)condone_complex;
    return;
  }
  std::vector<cd> evals_c(rank), y(rank * rank);
  if (hermitian) {
    std::vector<double> ev, vec;
    dense::sym_eigen(rank, Hbar, ev, vec);
    for (size_t i = 0; i < rank; ++i) evals_c[i] = ev[i];
    for (size_t i = 0; i < rank * rank; ++i) y[i] = vec[i];
  } else {
    dense::general_eigen(rank, Hbar, evals_c, y);
    double imag_norm = 0;
    for (auto& e : evals_c) imag_norm += e.imag() * e.imag();
    if (std::sqrt(imag_norm) < 1e-10) {
      for (auto& e : evals_c) e = e.real();
      for (size_t i = 0; i < rank; ++i) {
        double in = 0;
        for (size_t l = 0; l < rank; ++l) in += std::norm(y[l + rank * i].imag());
        if (std::sqrt(in) > 1e-10 && i + 1 < rank && std::abs(evals_c[i] - evals_c[i + 1]) < 1e-10) {
          double rn = 0, imn = 0;
          for (size_t l = 0; l < rank; ++l) {
            rn += std::pow(y[l + rank * i].real(), 2);
            imn += std::pow(y[l + rank * i].imag(), 2);
          }
          for (size_t l = 0; l < rank; ++l) {
            const cd v = y[l + rank * i];
            y[l + rank * (i + 1)] = v.imag() / std::sqrt(imn);
            y[l + rank * i] = v.real() / std::sqrt(rn);
          }
        }
      }
    }
  }
  // Back-transform: X = V_r diag(svmh) Y  (n x rank), each X[i,k] summed over l = 0..rank-1 in order.
  // Hermitian: Y is real, and (V svmh) * (y + 0i) accumulated in complex arithmetic has exactly
  // these real parts (and zero imaginary parts), so the real loop, unit stride in i, is used.
  std::vector<cd> X(n * rank, cd(0));
  if (hermitian) {
    std::vector<double> Xr(n);
    for (size_t k = 0; k < rank; ++k) {
      std::fill(Xr.begin(), Xr.end(), 0.0);
      for (size_t l = 0; l < rank; ++l) {
        const double ylk = y[l + rank * k].real(), sl = svmh[l];
        const double* vl = &V[n * l];
        for (size_t i = 0; i < n; ++i) Xr[i] += vl[i] * sl * ylk;
      }
      for (size_t i = 0; i < n; ++i) X[i + n * k] = Xr[i];
    }
  } else {
    for (size_t k = 0; k < rank; ++k)
      for (size_t i = 0; i < n; ++i) {
        cd s = 0;
        for (size_t l = 0; l < rank; ++l) s += V[i + n * l] * svmh[l] * y[l + rank * k];
        X[i + n * k] = s;
      }
  }
  // Selection sort ascending by real part (first minimum wins), sign fix on the largest component.
  std::vector<char> used(rank, 0);
  std::vector<cd> sv(rank), sX(n * rank);
  for (size_t k = 0; k < rank; ++k) {
    size_t ll = 0;
    while (used[ll]) ++ll;
    for (size_t l = 0; l < rank; ++l)
      if (!used[l] && evals_c[l].real() < evals_c[ll].real()) ll = l;
    used[ll] = 1;
    sv[k] = evals_c[ll];
    for (size_t i = 0; i < n; ++i) sX[i + n * k] = X[i + n * ll];
    // (the reference scans the first `rank` components for the largest)
    size_t mc = 0;
    for (size_t l = 0; l < rank && l < n; ++l)
      if (std::abs(sX[l + n * k].real()) > std::abs(sX[mc + n * k].real())) mc = l;
    if (sX[mc + n * k].real() < 0)
      for (size_t i = 0; i < n; ++i) sX[i + n * k] = -sX[i + n * k];
  }
  if (!hermitian) {
    // Normalise each eigenvector in the S metric and fix its phase (reference :451-506).
    std::vector<double> Sc(n * n);
    for (size_t i = 0; i < n * n; ++i) Sc[i] = metric[i];
    for (int repeat = 0; repeat < 3; ++repeat)
      for (size_t k = 0; k < rank; ++k) {
        if (std::abs(sv[k]) < 1e-12) {
          for (size_t i = 0; i < n; ++i) sX[i + n * k] = cd(sX[i + n * k].real() + 0.3256897 * sX[i + n * k].imag(), 0);
        }
        cd ovl = 0;
        for (size_t i = 0; i < n; ++i) {
          cd t = 0;
          for (size_t j = 0; j < n; ++j) t += Sc[i + n * j] * sX[j + n * k];
          ovl += std::conj(sX[i + n * k]) * t;
        }
        for (size_t i = 0; i < n; ++i) sX[i + n * k] /= std::sqrt(ovl.real());
        size_t lmax = 0;
        for (size_t l = 0; l < n; ++l)
          if (std::abs(sX[l + n * k]) > std::abs(sX[lmax + n * k])) lmax = l;
        if (sX[lmax + n * k].real() < 0)
          for (size_t i = 0; i < n; ++i) sX[i + n * k] = -sX[i + n * k];
      }
  }
  if (condone_complex) {
    for (size_t root = 0; root < rank; ++root) {
      if (sv[root].imag() != 0 && root + 1 < rank) {
        sv[root] = sv[root + 1] = sv[root].real();
        for (size_t i = 0; i < n; ++i) {
          const cd a = sX[i + n * root], b = sX[i + n * (root + 1)];
          sX[i + n * root] = a.real();
          sX[i + n * (root + 1)] = b.imag();
        }
        ++root;
      }
    }
  }
  double imag = 0;
  for (auto& x : sX) imag += x.imag() * x.imag();
  for (auto& e : sv) imag += e.imag() * e.imag();
  if (std::sqrt(imag) > 1e-10) throw std::runtime_error("unexpected complex solution found");
  eigenvectors.resize(n * rank);
  eigenvalues.resize(rank);
  for (size_t i = 0; i < n * rank; ++i) eigenvectors[i] = sX[i].real();
  for (size_t k = 0; k < rank; ++k) eigenvalues[k] = sv[k].real();
  (void)verbosity;
}

// Householder QR solve of a square system A X = B (A column-major n x n, B column-major n x m),
// the role of Eigen's householderQr().solve.
inline void householder_qr_solve(size_t n, std::vector<double> A, std::vector<double>& B, size_t m) {
  std::vector<double> v(n);
  for (size_t k = 0; k < n; ++k) {
    double norm = 0;
    for (size_t i = k; i < n; ++i) norm += A[i + n * k] * A[i + n * k];
    norm = std::sqrt(norm);
    if (norm == 0) continue;
    const double alpha = A[k + n * k] > 0 ? -norm : norm;
    double vnorm = 0;
    for (size_t i = k; i < n; ++i) {
      v[i] = A[i + n * k] - (i == k ? alpha : 0.0);
      vnorm += v[i] * v[i];
    }
    if (vnorm == 0) continue;
    auto reflect = [&](double* col) {
      double d = 0;
      for (size_t i = k; i < n; ++i) d += v[i] * col[i];
      d *= 2 / vnorm;
      for (size_t i = k; i < n; ++i) col[i] -= d * v[i];
    };
    for (size_t j = k; j < n; ++j) reflect(&A[n * j]);
    for (size_t j = 0; j < m; ++j) reflect(&B[n * j]);
  }
  for (size_t j = 0; j < m; ++j)
    for (size_t i = n; i-- > 0;) {
      double s = B[i + n * j];
      for (size_t l = i + 1; l < n; ++l) s -= A[i + n * l] * B[l + n * j];
      B[i + n * j] = A[i + n * i] != 0 ? s / A[i + n * i] : 0.0;
    }
}

// DIIS extrapolation coefficients (reference :619-669).  matrix: column-major dimension^2.
inline void solve_DIIS(std::vector<double>& solution, const std::vector<double>& matrix, const size_t dimension,
                       double svdThreshold, int verbosity = 0) {
  dense::AlgebraScope clock_(dimension);
  const size_t na = dimension + 1;
  std::vector<double> B(na * na, 0.0), rhs(na, 0.0);
  for (size_t i = 0; i < dimension; ++i)
    for (size_t j = 0; j < dimension; ++j) B[i + na * j] = matrix[i + dimension * j];
  for (size_t i = 0; i < dimension; ++i) B[dimension + na * i] = B[i + na * dimension] = -1;
  rhs[dimension] = -1;
  // SVD solve with threshold 0 (reference :650): pseudo-inverse over the non-zero singular values.
  std::vector<double> sv, U, V;
  dense::jacobi_svd(na, na, B, sv, U, V);
  std::vector<double> coeff(na, 0.0);
  for (size_t k = 0; k < na; ++k) {
    if (!(sv[k] > 0)) continue;
    double ub = 0;
    for (size_t i = 0; i < na; ++i) ub += U[i + na * k] * rhs[i];
    for (size_t i = 0; i < na; ++i) coeff[i] += V[i + na * k] * ub / sv[k];
  }
  solution.resize(dimension);
  for (size_t k = 0; k < dimension; ++k) {
    if (std::isnan(std::abs(coeff[k]))) throw std::overflow_error("NaN detected in DIIS submatrix solution");
    solution[k] = coeff[k];
  }
  (void)svdThreshold;
  (void)verbosity;
}

// Subspace linear equations (reference helper-implementation.h:553-617).  matrix: row-major
// nX x nX; rhs: the row-major nX x nroot EqnData::rhs block.  solution[k + nX*root].
//  * augmented_hessian == 0: H c = rhs by Householder QR (the reference's householderQr().solve);
//  * augmented_hessian > 0: for each root the lowest eigenpair of [[H, -a r], [-a r^T, 0]] with
//    metric diag(S, 1), c = v_head / (a v_last).  As in the reference, H is read column-major
//    (its transpose) and the rhs of root `root` as rhs[i + nX*root] in this branch.
inline void solve_LinearEquations(std::vector<double>& solution, std::vector<double>& eigenvalues,
                                  const std::vector<double>& matrix, const std::vector<double>& metric,
                                  const std::vector<double>& rhs, const size_t dimension, size_t nroot,
                                  double augmented_hessian, double svdThreshold, int verbosity) {
  dense::AlgebraScope clock_(dimension);
  const size_t nX = dimension;
  solution.assign(nX * nroot, 0.0);
  if (augmented_hessian > 0) {
    const size_t na = nX + 1;
    eigenvalues.resize(nroot);
    for (size_t root = 0; root < nroot; ++root) {
      std::vector<double> M(na * na, 0.0), Sa(na * na, 0.0);  // row-major for eigenproblem()
      for (size_t i = 0; i < nX; ++i)
        for (size_t j = 0; j < nX; ++j) {
          M[i * na + j] = matrix[j * nX + i];   // Eigen::Map column-major view of the row-major H
          Sa[i + na * j] = metric[i + nX * j];  // metric read column-major, as eigenproblem() does
        }
      for (size_t i = 0; i < nX; ++i) M[i * na + nX] = M[nX * na + i] = -augmented_hessian * rhs[i + nX * root];
      Sa[nX + na * nX] = 1;
      std::vector<double> evec, eval;
      eigenproblem(evec, eval, M, Sa, na, false, svdThreshold, verbosity, true);
      if (eval.empty()) throw std::runtime_error("solve_LinearEquations: empty augmented-Hessian eigenproblem");
      size_t imax = 0;
      for (size_t i = 0; i < eval.size(); ++i)
        if (eval[i] < eval[imax]) imax = i;
      eigenvalues[root] = eval[imax];
      const double last = evec[nX + na * imax];
      for (size_t k = 0; k < nX; ++k) solution[k + nX * root] = evec[k + na * imax] / (augmented_hessian * last);
    }
  } else {
    std::vector<double> A(nX * nX), B(nX * nroot);
    for (size_t i = 0; i < nX; ++i) {
      for (size_t j = 0; j < nX; ++j) A[i + nX * j] = matrix[i * nX + j];
      for (size_t r = 0; r < nroot; ++r) B[i + nX * r] = rhs[i * nroot + r];
    }
    householder_qr_solve(nX, A, B, nroot);
    for (size_t r = 0; r < nroot; ++r)
      for (size_t k = 0; k < nX; ++k) solution[k + nX * r] = B[k + nX * r];
  }
}

}  // namespace molpro::linalg::itsolv
