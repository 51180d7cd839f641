#include <algorithm>
#include <cmath>
#include <complex>
#include <limits>
#include <list>
#include <numeric>
#include <stdexcept>
#include <vector>
#define molpro molpro_new
#include "itsolv_hbm/dense.h"
void new_sym(size_t n, const std::vector<double>& a, std::vector<double>& e, std::vector<double>& v) {
  molpro_new::linalg::itsolv::dense::sym_eigen(n, a, e, v);
}
void new_eig(size_t n, const std::vector<double>& h, const std::vector<double>& s, std::vector<double>& ev, std::vector<double>& val) {
  molpro_new::linalg::itsolv::eigenproblem(ev, val, h, s, n, true, 1e-14, 0, true);
}
