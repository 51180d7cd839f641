// Cubic interpolation of a function along a line from values and first derivatives at two points,
// the line-search model of OptimizeBFGS (reference itsolv/Interpolate.h:15-61,
// Interpolate.cpp:55-170; only the "cubic" interpolant, which is the one OptimizeBFGS builds).
#pragma once
#include <cmath>
#include <stdexcept>
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

  // c0 + c1 (x - xbar) + c2 (x - xbar)^2 + c3 (x - xbar)^3, xbar = (x0 + x1) / 2 (reference :61-73)
  Interpolate(point p0, point p1) : m_p0(p0), m_p1(p1), m_parameters(4) {
    const double dx = m_p1.x - m_p0.x;
    const double fs = m_p1.f + m_p0.f, fd = m_p1.f - m_p0.f;
    const double gs = m_p1.f1 + m_p0.f1, gd = m_p1.f1 - m_p0.f1;
    m_parameters[0] = 0.5 * fs - 0.125 * gd * dx;
    m_parameters[1] = -0.25 * gs + 1.5 * fd / dx;
    m_parameters[2] = 0.5 * gd / dx;
    m_parameters[3] = (-2 * fd + gs * dx) / std::pow(dx, 3);
  }

  point operator()(double x) const {
    const double t = x - 0.5 * (m_p1.x + m_p0.x);
    const auto& c = m_parameters;
    return point{x, c[0] + t * (c[1] + t * (c[2] + t * c[3])), c[1] + t * (2 * c[2] + 3 * t * c[3]),
                 2 * c[2] + 6 * t * c[3]};
  }

  // Stationary points of the cubic, the lower one (reference :127-146); NaN x when none is real.
  point minimize_cubic() const {
    const double c = m_parameters[1], b = 2 * m_parameters[2], a = 3 * m_parameters[3];
    const double disc = b * b / (4 * a * a) - c / a;
    if (std::isnan(disc) || disc < 0) return {std::nan("unset")};
    const double xbar = 0.5 * (m_p1.x + m_p0.x);
    const point pm = (*this)(xbar - b / (2 * a) + std::sqrt(disc));
    const point pp = (*this)(xbar - b / (2 * a) - std::sqrt(disc));
    return pm.f < pp.f ? pm : pp;
  }

  // reference :148-186 with analytic = true: the cubic's own minimum (the bounds are not used).
  point minimize(double xa, double xb) const {
    (void)xa;
    (void)xb;
    return minimize_cubic();
  }

  const std::vector<double>& parameters() const { return m_parameters; }

 private:
  point m_p0, m_p1;
  std::vector<double> m_parameters;
};

}  // namespace molpro::linalg::itsolv
