// 4-parameter interpolation of a function along a line from values and first derivatives at two
// points (reference itsolv/Interpolate.h:13-57, Interpolate.cpp:19-186): the "cubic" interpolant,
// OptimizeBFGS's line-search model, and the "morse" interpolant
// L0 + (k / 2a^2) (1 - exp(-a (y - y0)))^2, fitted to the two points by DIIS from the cubic's
// minimum (interpolate_morse.h, included at the end of solvers.h where the DIIS solver is defined).
#pragma once
#include <algorithm>
#include <cmath>
#include <ostream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace molpro::linalg::itsolv {

class Interpolate {
 public:
  struct point {
    double x;
    double f = std::nan("unset");
    double f1 = std::nan("unset");
    double f2 = std::nan("unset");
  };

  // reference Interpolate.cpp:55-100; an unknown interpolant throws std::runtime_error
  explicit Interpolate(point p0, point p1, std::string interpolant = "cubic", int verbosity = 0)
      : m_p0(p0), m_p1(p1), m_interpolant(std::move(interpolant)), m_parameters(4) {
    if (m_interpolant == "cubic") {
      // c0 + c1 (x - xbar) + c2 (x - xbar)^2 + c3 (x - xbar)^3, xbar = (x0 + x1) / 2 (reference :61-73)
      const double dx = m_p1.x - m_p0.x;
      const double fs = m_p1.f + m_p0.f, fd = m_p1.f - m_p0.f;
      const double gs = m_p1.f1 + m_p0.f1, gd = m_p1.f1 - m_p0.f1;
      m_parameters[0] = 0.5 * fs - 0.125 * gd * dx;
      m_parameters[1] = -0.25 * gs + 1.5 * fd / dx;
      m_parameters[2] = 0.5 * gd / dx;
      m_parameters[3] = (-2 * fd + gs * dx) / std::pow(dx, 3);
    } else if (m_interpolant == "morse") {
      // parameters L0, k, a, y0; starting guess from the cubic's minimum (reference :74-97)
      const Interpolate cubic(p0, p1, "cubic", 0);
      const point m = cubic(cubic.minimize(p0.x, p1.x).x);
      std::vector<double> guess{m.f, m.f2, -3 * cubic.m_parameters[3] / m.f2, m.x};
      m_parameters = fit_morse(m_p0, m_p1, std::move(guess), verbosity);
    } else {
      throw std::runtime_error("Unknown interpolant: " + m_interpolant);
    }
  }

  static std::vector<std::string> interpolants() { return {"cubic", "morse"}; }

  // value, first and second derivative of L0 + (k/2)((1 - exp(-a(y - y0)))/a)^2 (reference :19-28)
  static point morse(double y, const std::vector<double>& p) {
    const double e = std::exp(-p[2] * (y - p[3]));
    point r{y};
    r.f = p[0] + (p[1] / 2) * std::pow((1 - e) / p[2], 2);
    r.f1 = (p[1] / p[2]) * e * (1 - e);
    r.f2 = -p[1] * (1 - 2 * e);
    return r;
  }

  point operator()(double x) const {
    if (m_interpolant == "morse") return morse(x, m_parameters);
    const double t = x - 0.5 * (m_p1.x + m_p0.x);
    const auto& c = m_parameters;
    return point{x, c[0] + t * (c[1] + t * (c[2] + t * c[3])), c[1] + t * (2 * c[2] + 3 * t * c[3]),
                 2 * c[2] + 6 * t * c[3]};
  }

  // Stationary points of the cubic, the lower one (reference :127-146); NaN x when none is real.
  point minimize_cubic() const {
    if (m_interpolant != "cubic") throw std::logic_error("minimize_cubic called with non-cubic interpolant");
    const double c = m_parameters[1], b = 2 * m_parameters[2], a = 3 * m_parameters[3];
    const double disc = b * b / (4 * a * a) - c / a;
    if (std::isnan(disc) || disc < 0) return {std::nan("unset")};
    const double xbar = 0.5 * (m_p1.x + m_p0.x);
    const point pm = (*this)(xbar - b / (2 * a) + std::sqrt(disc));
    const point pp = (*this)(xbar - b / (2 * a) - std::sqrt(disc));
    return pm.f < pp.f ? pm : pp;
  }

  // Minimum within [xa, xb] (reference :148-186).  analytic and cubic: the cubic's own minimum (the
  // bounds are not used; OptimizeBFGS's path).  Otherwise: bracket a sign change of f1 on a grid of
  // bracket_grid intervals (doubled up to max_bracket_grid), then regula falsi on f1 to the last
  // representable bit; with no bracket, the lower end point.
  point minimize(double xa, double xb, size_t bracket_grid = 100, size_t max_bracket_grid = 100000,
                 bool analytic = true) const {
    if (xa > xb) std::swap(xa, xb);
    if (analytic && m_interpolant == "cubic") return minimize_cubic();
    for (size_t ngrid = bracket_grid; ngrid < std::max(bracket_grid, max_bracket_grid) + 1; ngrid *= 2) {
      const double step = (xb - xa) / ngrid;
      point lo = (*this)(xa);
      point p0 = (*this)(xa).f > (*this)(xb).f ? lo : (*this)(xb);
      point p1 = p0;
      for (size_t i = 0; i < ngrid; i++) {
        point hi = (*this)(lo.x + step);
        if (std::min(hi.f, lo.f) < p0.f && lo.f1 <= 0 && hi.f1 >= 0) {
          p1 = hi;
          p0 = lo;
        }
        std::swap(lo, hi);
      }
      if (p0.f1 < 0 && p1.f1 > 0) {
        point pnew = p1;
        const double tolerance = (std::nextafter(pnew.x, pnew.x + 1) - pnew.x) * 2;
        while (std::abs(p0.x - pnew.x) > tolerance) {
          pnew = (*this)((p1.x * p0.f1 - p0.x * p1.f1) / (p0.f1 - p1.f1));
          if (pnew.f1 * p0.f1 < 0) std::swap(p0, p1);
          std::swap(p0, pnew);
        }
        return p0;
      }
    }
    return (*this)(xa).f > (*this)(xb).f ? (*this)(xb) : (*this)(xa);
  }

  const std::vector<double>& parameters() const { return m_parameters; }
  const std::string& interpolant() const { return m_interpolant; }

  friend std::ostream& operator<<(std::ostream& os, const Interpolate& i) {
    for (double p : i.m_parameters) os << " " << p;
    return os;
  }

 private:
  // Defined in interpolate_morse.h (needs NonLinearEquationsDIIS).
  static inline std::vector<double> fit_morse(const point& p0, const point& p1, std::vector<double> guess, int verbosity);

  point m_p0, m_p1;
  std::string m_interpolant;
  std::vector<double> m_parameters;
};

inline bool operator==(const Interpolate::point& l, const Interpolate::point& r) {
  return l.x == r.x && l.f == r.f && l.f1 == r.f1;
}
inline std::ostream& operator<<(std::ostream& os, const Interpolate::point& p) {
  return os << "x=" << p.x << ", value=" << p.f << ", gradient=" << p.f1 << ", curvature=" << p.f2;
}

}  // namespace molpro::linalg::itsolv
