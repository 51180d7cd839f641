// Proposing the next expansion vectors (R space) from preconditioned residuals, and D-space
// management — the byte-dominant host algorithm of a Davidson iteration.
//
// Restated from the reference:
//   normalise                              itsolv/propose_rspace.h:17-28
//   dspace::construct_projected_solution   :39-57,  construct_projected_solutions_overlap :73-108
//   dspace::remove_null_norm_and_normalise :117-144, remove_null_projected_solutions     :158-179
//   dspace::construct_full_subspace_overlap :190-256
//   append_overlap_with_r :271-300,  limit_qspace_size :310-336,  construct_dspace :349-403
//   modified_gram_schmidt :421-466 (P, then Q, then D; stored |S_xx| as the norm)
//   redundant_parameters  :481-512,  propose_rspace :553-624
//   DSpaceResetter        itsolv/DSpaceResetter.h:14-145, construct_solutions itsolv/util.h:218-239
#pragma once
#include <algorithm>
#include <cmath>
#include <list>
#include <numeric>
#include <set>
#include <sstream>
#include <tuple>
#include <type_traits>
#include <vector>

#include "dense.h"
#include "subspace.h"

namespace molpro::linalg::itsolv::detail {

using subspace::Dimensions;
using subspace::EqnData;
using subspace::Matrix;

// <x_i, x_i> for every x in xs, registered on the handler's lazy handle (reference
// ArrayHandler.h:298-437) and evaluated together: device handlers fold the batch into one
// gemm_inner launch and one reduction (fused_dot); the reference's CPU handler evaluates the same
// dots one by one in order.
template <class R, class Refs>
std::vector<double> self_dots(const Refs& xs, array::ArrayHandler<R, R>& handler) {
  std::vector<double> d(xs.size(), 0.0);
  auto lazy = handler.lazy_handle();
  for (size_t i = 0; i < xs.size(); ++i) lazy.dot(xs[i].get(), xs[i].get(), d[i]);
  lazy.eval();
  return d;
}

// reference propose_rspace.h:17-28 (the norms first, as one batch: scaling one vector does not
// change another's norm)
template <class R>
void normalise(VecRef<R>& params, array::ArrayHandler<R, R>& handler, Logger& logger, double thresh = 1.0e-14) {
  const auto dots = self_dots(params, handler);
  for (size_t i = 0; i < params.size(); ++i) {
    const double nrm = std::sqrt(std::abs(dots[i]));
    if (nrm > thresh)
      handler.scal(1. / nrm, params[i]);
    else
      logger.msg("parameter's length is too small for normalisation, dot = " + Logger::scientific(nrm), Logger::Warn);
  }
}

namespace dspace {

// Columns [Q_delete | D] of the solutions.
inline Matrix<double> construct_projected_solution(const Matrix<double>& sol, const Dimensions& d,
                                                   const std::vector<int>& qdel) {
  const size_t nqd = qdel.size(), ns = sol.rows();
  Matrix<double> out({ns, nqd + d.nD});
  for (size_t i = 0; i < ns; ++i) {
    for (size_t j = 0; j < nqd; ++j) out(i, j) = sol(i, d.oQ + qdel[j]);
    for (size_t j = 0; j < d.nD; ++j) out(i, nqd + j) = sol(i, d.oD + j);
  }
  return out;
}

// Index in the current subspace of column c of a [Q_delete | D] coefficient block.
inline size_t proj_index(size_t c, const Dimensions& d, const std::vector<int>& qdel) {
  return c < qdel.size() ? d.oQ + size_t(qdel[c]) : d.oD + (c - qdel.size());
}

// <x_i, x_j> for x_i = sum_c proj(i, c) u_c, in the reference's summation order.
inline Matrix<double> construct_projected_solutions_overlap(const Matrix<double>& proj, const Matrix<double>& S,
                                                            const Dimensions& d, const std::vector<int>& qdel) {
  const size_t ns = proj.rows(), nqd = qdel.size();
  Matrix<double> ov({ns, ns});
  for (size_t i = 0; i < ns; ++i)
    for (size_t ii = 0; ii <= i; ++ii) {
      double s = 0;
      for (size_t j = 0; j < nqd; ++j) {
        for (size_t k = 0; k < nqd; ++k) s += proj(i, j) * proj(ii, k) * S(d.oQ + qdel[j], d.oQ + qdel[k]);
        for (size_t k = 0; k < d.nD; ++k) s += proj(i, j) * proj(ii, nqd + k) * S(d.oQ + qdel[j], d.oD + k);
      }
      for (size_t j = 0; j < d.nD; ++j) {
        for (size_t k = 0; k < d.nD; ++k) s += proj(i, nqd + j) * proj(ii, nqd + k) * S(d.oD + j, d.oD + k);
        for (size_t k = 0; k < nqd; ++k) s += proj(i, nqd + j) * proj(ii, k) * S(d.oD + j, d.oQ + qdel[k]);
      }
      ov(i, ii) = ov(ii, i) = s;
    }
  return ov;
}

inline void remove_null_norm_and_normalise(Matrix<double>& params, Matrix<double>& ov, double norm_thresh,
                                           Logger& logger) {
  const size_t ns = params.rows();
  std::vector<double> nrm(ns);
  for (size_t i = 0; i < ns; ++i) nrm[i] = std::sqrt(std::abs(ov(i, i)));
  for (size_t i = 0, j = 0; i < ns; ++i) {
    if (nrm[i] > norm_thresh) {
      params.row(j).scal(1. / nrm[i]);
      ov.col(j).scal(1. / nrm[i]);
      ov.row(j).scal(1. / nrm[i]);
      ++j;
    } else {
      params.remove_row(j);
      ov.remove_row_col(j, j);
      logger.msg("remove projected solution parameter i = " + std::to_string(i), Logger::Info);
    }
  }
}

// Rotates the projected solutions onto the eigenvectors of their overlap with eigenvalue >= thresh,
// smallest eigenvalue first.
inline Matrix<double> remove_null_projected_solutions(const Matrix<double>& proj, const Matrix<double>& ov,
                                                      double svd_thresh) {
  auto svds = svd_system(ov.rows(), ov.cols(), ov.data(), std::numeric_limits<double>::max(), true);
  svds.remove_if([&](const auto& s) { return s.value < svd_thresh; });
  svds.sort([](const auto& a, const auto& b) { return a.value < b.value; });
  const size_t nd = svds.size(), nx = proj.cols();
  Matrix<double> out({nd, nx});
  auto it = svds.begin();
  for (size_t i = 0; i < nd; ++i, ++it)
    for (size_t j = 0; j < ov.cols(); ++j)
      for (size_t k = 0; k < nx; ++k) out(i, k) += it->v[j] * proj(j, k);
  return out;
}

}  // namespace dspace

// Overlap of P+Q+D plus new parameters appended last (reference :271-300).
template <class R, class Q, class P>
Matrix<double> append_overlap_with_r(const Matrix<double>& overlap, const CVecRef<R>& params, const CVecRef<P>& pp,
                                     const CVecRef<Q>& qp, const CVecRef<Q>& dp, ArrayHandlers<R, Q, P>& h) {
  const size_t nP = pp.size(), nQ = qp.size(), nD = dp.size(), nN = params.size();
  const size_t oQ = nP, oD = oQ + nQ, oN = oD + nD, nX = oN + nN;
  auto ov = overlap;
  ov.resize({nX, nX});
  bool fused = false;
  if constexpr (std::is_same_v<R, Q>) {
    // the blocks whose rows are the new parameters as one batched overlap where the handler has it
    // (array::fused_overlap_rows): columns [params, Q params, D params]
    Matrix<double> g;
    using array::fused_overlap_rows;
    if (nN > 0 && fused_overlap_rows(h.rr(), params, std::vector<CVecRef<R>>{params, qp, dp}, g)) {
      fused = true;
      for (size_t i = 0; i < nN; ++i) {
        for (size_t j = 0; j <= i; ++j) ov(oN + i, oN + j) = ov(oN + j, oN + i) = g(i, j);
        for (size_t j = 0; j < nQ; ++j) ov(oN + i, oQ + j) = g(i, nN + j);
        for (size_t j = 0; j < nD; ++j) ov(oN + i, oD + j) = g(i, nN + nQ + j);
      }
    }
  }
  if (!fused) {
    ov.slice({oN, oN}, {nX, nX}) = subspace::util::overlap(params, h.rr());
    ov.slice({oN, oQ}, {nX, oQ + nQ}) = subspace::util::overlap(params, qp, h.rq());
    ov.slice({oN, oD}, {nX, oD + nD}) = subspace::util::overlap(params, dp, h.rq());
  }
  ov.slice({oN, 0}, {nX, nP}) = subspace::util::overlap(params, pp, h.rp());
  for (size_t i = 0; i < oN; ++i)
    for (size_t j = 0; j < nN; ++j) ov(i, oN + j) = ov(oN + j, i);
  return ov;
}

// Q indices to delete so that at most max_q remain: repeatedly the one whose largest |coefficient|
// over the solutions is smallest (reference :310-336).
inline std::vector<int> limit_qspace_size(const Dimensions& d, size_t max_q, const Matrix<double>& sol, Logger& log) {
  std::vector<int> del, idx(d.nQ);
  std::iota(idx.begin(), idx.end(), 0);
  while (idx.size() > max_q) {
    std::vector<double> contrib;
    for (int i : idx) {
      double mx = -1;
      for (size_t j = 0; j < sol.rows(); ++j) mx = std::max(mx, std::abs(sol(j, d.oQ + i)));
      contrib.push_back(mx);
    }
    const size_t k = size_t(std::min_element(contrib.begin(), contrib.end()) - contrib.begin());
    del.push_back(idx[k]);
    idx.erase(idx.begin() + k);
    log.msg("delete Q i = " + std::to_string(k), Logger::Info);
  }
  return del;
}

// Overlap of P + (Q without deletions) + nR new + projected solutions (reference :190-256).
inline Matrix<double> construct_full_subspace_overlap(const Matrix<double>& proj, const Dimensions& d,
                                                      const std::vector<int>& qdel, const Matrix<double>& S,
                                                      size_t nR) {
  const size_t nDnew = proj.rows(), nqd = qdel.size(), nQ = d.nQ - nqd;
  auto ov = S;
  for (size_t i = 0; i < d.nD; ++i) ov.remove_row_col(d.oD, d.oD);
  auto deleted = [&](size_t i) { return std::find(qdel.begin(), qdel.end(), int(i)) != qdel.end(); };
  for (size_t i = 0, j = 0; i < d.nQ; ++i) {
    if (deleted(i))
      ov.remove_row_col(d.oQ + j, d.oQ + j);
    else
      ++j;
  }
  const size_t oDnew = d.nP + nQ + nR;
  ov.resize({oDnew + nDnew, oDnew + nDnew});
  auto offdiag = [&](size_t i, size_t j, size_t jj) {
    for (size_t k = 0; k < nqd; ++k) ov(oDnew + i, j) += proj(i, k) * S(jj, d.oQ + qdel[k]);
    for (size_t k = 0; k < d.nD; ++k) ov(oDnew + i, j) += proj(i, nqd + k) * S(jj, d.oD + k);
    ov(j, oDnew + i) = ov(oDnew + i, j);
  };
  for (size_t i = 0; i < nDnew; ++i) {
    for (size_t j = 0; j < d.nP; ++j) offdiag(i, j, d.oP + j);
    for (size_t j = 0, jj = 0; j < d.nQ; ++j)
      if (!deleted(j)) offdiag(i, d.nP + jj++, d.oQ + j);
    for (size_t j = 0; j < nR; ++j) offdiag(i, d.nP + nQ + j, d.nX + j);
  }
  for (size_t i = 0; i < nDnew; ++i)
    for (size_t j = 0; j <= i; ++j) {
      for (size_t k = 0; k < nqd; ++k) {
        for (size_t l = 0; l < nqd; ++l)
          ov(oDnew + i, oDnew + j) += proj(i, k) * proj(j, l) * S(d.oQ + qdel[k], d.oQ + qdel[l]);
        for (size_t l = 0; l < d.nD; ++l)
          ov(oDnew + i, oDnew + j) += proj(i, k) * proj(j, nqd + l) * S(d.oQ + qdel[k], d.oD + l);
      }
      for (size_t k = 0; k < d.nD; ++k) {
        for (size_t l = 0; l < nqd; ++l)
          ov(oDnew + i, oDnew + j) += proj(i, nqd + k) * proj(j, l) * S(d.oD + k, d.oQ + qdel[l]);
        for (size_t l = 0; l < d.nD; ++l)
          ov(oDnew + i, oDnew + j) += proj(i, nqd + k) * proj(j, nqd + l) * S(d.oD + k, d.oD + l);
      }
      ov(oDnew + j, oDnew + i) = ov(oDnew + i, oDnew + j);
    }
  return ov;
}

// New D space: solutions projected onto Q_delete + D, stabilised, built with qq axpys (reference :349-403).
template <class R, class Q, class P>
std::tuple<std::vector<Q>, std::vector<Q>> construct_dspace(const Matrix<double>& sol, const subspace::XSpace<R, Q, P>& xs,
                                                            const std::vector<int>& qdel, double norm_thresh,
                                                            double svd_thresh, array::ArrayHandler<Q, Q>& h,
                                                            Logger& log) {
  const auto d = xs.dimensions();
  const auto& S = xs.data.at(EqnData::S);
  auto proj = dspace::construct_projected_solution(sol, d, qdel);
  auto ovp = dspace::construct_projected_solutions_overlap(proj, S, d, qdel);
  dspace::remove_null_norm_and_normalise(proj, ovp, norm_thresh, log);
  proj = dspace::remove_null_projected_solutions(proj, ovp, svd_thresh);
  ovp = dspace::construct_projected_solutions_overlap(proj, S, d, qdel);
  dspace::remove_null_norm_and_normalise(proj, ovp, norm_thresh, log);
  const size_t nD = proj.rows(), nqd = qdel.size();
  const auto qp = xs.cparamsq(), qa = xs.cactionsq(), dp = xs.cparamsd(), da = xs.cactionsd();
  std::vector<Q> newp, newa;
  // The reference's copy + fill(0) + axpy loops, or one write-only pass when the handler has it
  // (sources in the same order: Q vectors being deleted, then D).
  std::vector<const Q*> srcp, srca;
  for (size_t j = 0; j < nqd; ++j) srcp.push_back(&qp.at(qdel[j]).get()), srca.push_back(&qa.at(qdel[j]).get());
  for (size_t j = 0; j < d.nD; ++j) srcp.push_back(&dp.at(j).get()), srca.push_back(&da.at(j).get());
  using array::fused_new_combinations;
  bool fused = false;
  if (nD > 0 && !srcp.empty()) {
    Matrix<double> c(std::make_pair(nD, srcp.size()));
    for (size_t i = 0; i < nD; ++i)
      for (size_t j = 0; j < srcp.size(); ++j) c(i, j) = proj(i, j);
    fused = fused_new_combinations(h, c, srcp, newp) && fused_new_combinations(h, c, srca, newa);
  }
  const Q* proto = !qp.empty() ? &qp.front().get() : (!dp.empty() ? &dp.front().get() : nullptr);
  if (proto && !fused)
    for (size_t i = 0; i < nD; ++i) {
      newp.emplace_back(h.copy(*proto));
      newa.emplace_back(h.copy(*proto));
      h.fill(0, newp.back());
      h.fill(0, newa.back());
    }
  // The reference's axpy loops, registered per destination set on a lazy handle: every destination
  // receives its sources in increasing order, so a device handler applies each set as one
  // gemm_outer, bit for bit the axpy sequence (fused_axpy); params and actions are disjoint sets.
  if (!fused) {
    auto lp = h.lazy_handle();
    auto la = h.lazy_handle();
    for (size_t i = 0; i < nD; ++i) {
      for (size_t j = 0; j < nqd; ++j) {
        lp.axpy(proj(i, j), qp.at(qdel[j]).get(), newp.at(i));
        la.axpy(proj(i, j), qa.at(qdel[j]).get(), newa.at(i));
      }
      for (size_t j = 0; j < d.nD; ++j) {
        lp.axpy(proj(i, nqd + j), dp.at(j).get(), newp.at(i));
        la.axpy(proj(i, nqd + j), da.at(j).get(), newa.at(i));
      }
    }
    lp.eval();
    la.eval();
  }
  const auto dots = self_dots(wrap(newp), h);
  for (size_t i = 0; i < nD; ++i) {
    const double nrm = std::sqrt(std::abs(dots[i]));
    h.scal(1. / nrm, newp[i]);
    h.scal(1. / nrm, newa[i]);
  }
  return {std::move(newp), std::move(newa)};
}

// Sequential self-orthonormalisation of R; indices whose norm is below norm_thresh are returned
// as null (reference propose_rspace.h:450-465).
template <class R>
std::vector<int> orthonormalise_among(const VecRef<R>& rparams, double norm_thresh, array::ArrayHandler<R, R>& hr) {
  std::vector<int> null_params;
  using array::fused_orthonormalise;
  if (fused_orthonormalise(hr, rparams, norm_thresh, null_params)) return null_params;
  const size_t nR = rparams.size();
  for (size_t i = 0; i < nR; ++i) {
    const double nrm = std::sqrt(std::abs(hr.dot(rparams[i], rparams[i])));
    if (nrm > norm_thresh) {
      hr.scal(1. / nrm, rparams[i]);
      for (size_t j = i + 1; j < nR; ++j) {
        const double ov = hr.dot(rparams[i], rparams[j]);
        hr.axpy(-ov, rparams[i], rparams[j]);
      }
    } else {
      null_params.push_back(int(i));
    }
  }
  return null_params;
}

// Orthogonalise R against P, Q, D (in that order) and among themselves (reference :421-466).
template <class R, class Q, class P>
std::vector<int> modified_gram_schmidt(const VecRef<R>& rparams, const Matrix<double>& S, const Dimensions& d,
                                       const CVecRef<P>& pp, const CVecRef<Q>& qp, const CVecRef<Q>& dp,
                                       double norm_thresh, ArrayHandlers<R, Q, P>& h) {
  const size_t nR = rparams.size();
  auto orthogonalise = [&](const auto& xparams, auto& handler, size_t oX, size_t nX) {
    for (size_t i = 0; i < nX; ++i) {
      const double nrm = std::abs(S(oX + i, oX + i));
      if (nR == 0) continue;
      auto dots = handler.gemm_inner(cwrap(rparams), cwrap_arg(xparams.at(i).get()));
      Matrix<double> coeff({1, nR});
      for (size_t j = 0; j < nR; ++j) coeff(0, j) = -dots(j, 0) / nrm;
      handler.gemm_outer(coeff, cwrap_arg(xparams.at(i).get()), rparams);
    }
  };
  // P vectors with pairwise disjoint supports (solve()'s P space is unit vectors on distinct
  // indices): <R_j, p_i> reads R_j only where no earlier p_l updated it, and each element of R_j is
  // updated by at most one p_i, so one gemm_inner over all of P followed by one gemm_outer is the
  // sequential sweep bit for bit -- two sparse launches (one reduction) instead of two per p_i.
  auto disjoint = [&] {
    std::set<size_t> seen;
    for (const auto& p : pp)
      for (const auto& e : p.get())
        if (!seen.insert(e.first).second) return false;
    return true;
  };
  if (nR > 0 && pp.size() > 1 && disjoint()) {
    auto dots = h.rp().gemm_inner(cwrap(rparams), pp);
    Matrix<double> coeff({pp.size(), nR});
    for (size_t i = 0; i < pp.size(); ++i)
      for (size_t j = 0; j < nR; ++j) coeff(i, j) = -dots(j, i) / std::abs(S(d.oP + i, d.oP + i));
    h.rp().gemm_outer(coeff, pp, rparams);
  } else {
    orthogonalise(pp, h.rp(), d.oP, pp.size());
  }
  // Q then D: the same handler and the same call sequence as two orthogonalise() sweeps, except
  // that a handler with a fused form (array::fused_axpy_inner) merges each step's gemm_outer with
  // the next step's gemm_inner into one pass over R: R is read once per
  // vector instead of twice, with bit-identical R updates.
  std::vector<std::pair<const Q*, double>> qd;
  for (size_t i = 0; i < qp.size(); ++i) qd.emplace_back(&qp.at(i).get(), std::abs(S(d.oQ + i, d.oQ + i)));
  for (size_t i = 0; i < dp.size(); ++i) qd.emplace_back(&dp.at(i).get(), std::abs(S(d.oD + i, d.oD + i)));
  if (nR > 0 && !qd.empty()) {
    auto& hq = h.rq();
    std::vector<double> dots(nR);
    auto inner = [&](size_t i) {
      auto m = hq.gemm_inner(cwrap(rparams), cwrap_arg(*qd[i].first));
      for (size_t j = 0; j < nR; ++j) dots[j] = m(j, 0);
    };
    inner(0);
    for (size_t i = 0; i < qd.size(); ++i) {
      std::vector<double> c(nR);
      for (size_t j = 0; j < nR; ++j) c[j] = -dots[j] / qd[i].second;
      if (i + 1 < qd.size()) {
        using array::fused_axpy_inner;
        if (fused_axpy_inner(hq, c, *qd[i].first, rparams, *qd[i + 1].first, dots)) continue;
      }
      Matrix<double> coeff({1, nR});
      for (size_t j = 0; j < nR; ++j) coeff(0, j) = c[j];
      hq.gemm_outer(coeff, cwrap_arg(*qd[i].first), rparams);
      if (i + 1 < qd.size()) inner(i + 1);
    }
  }
  return orthonormalise_among(rparams, norm_thresh, h.rr());
}

// Option block_gram_schmidt (extension): the same projection as
// modified_gram_schmidt above, R_j <- R_j + sum_i c(i,j) x_i over x = P, Q, D in that order, with
// c(i,j) = -<R_j^(i-1), x_i> / |S_ii| and <R_j^(i-1), x_i> = <R_j, x_i> + sum_{l<i} c(l,j) S_li.
// <R_j, x_i> are the rows `rows` of `full` (append_overlap_with_r, already computed for the
// redundancy screen), so the coefficients come from a forward substitution on the host and R is
// updated by one gemm_outer per space instead of one gemm_inner + gemm_outer per x_i. Identical
// in exact arithmetic; the rounding differs from the sequential sweep.
template <class R, class Q, class P>
std::vector<int> block_gram_schmidt(const VecRef<R>& rparams, const Matrix<double>& full,
                                    const std::vector<size_t>& rows, const Dimensions& d, const CVecRef<P>& pp,
                                    const CVecRef<Q>& qp, const CVecRef<Q>& dp, double norm_thresh,
                                    ArrayHandlers<R, Q, P>& h) {
  const size_t nR = rparams.size(), nX = d.nX;
  if (nR > 0 && nX > 0) {
    Matrix<double> c({nX, nR});
    for (size_t j = 0; j < nR; ++j)
      for (size_t i = 0; i < nX; ++i) {
        double t = full(rows[j], i);
        for (size_t l = 0; l < i; ++l) t += c(l, j) * full(l, i);
        c(i, j) = -t / std::abs(full(i, i));
      }
    auto block = [&](size_t o, size_t n) {
      Matrix<double> a({n, nR});
      for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j < nR; ++j) a(i, j) = c(o + i, j);
      return a;
    };
    CVecRef<Q> qd(qp.begin(), qp.end());
    qd.insert(qd.end(), dp.begin(), dp.end());
    using array::fused_block_update;
    if (!fused_block_update(h.rp(), block(d.oP, d.nP), pp, block(d.oQ, d.nQ + d.nD), qd, rparams)) {
      if (d.nP) h.rp().gemm_outer(block(d.oP, d.nP), pp, rparams);
      if (d.nQ + d.nD) h.rq().gemm_outer(block(d.oQ, d.nQ + d.nD), qd, rparams);
    } else {  // the handler calls the one pass replaced
      h.rp().count_replaced(0, 0, d.nP ? 1 : 0);
      h.rq().count_replaced(0, 0, d.nQ + d.nD ? 1 : 0);
    }
  }
  return orthonormalise_among(rparams, norm_thresh, h.rr());
}

// Indices among the last nR parameters made redundant by near-null singular vectors (reference :481-512).
inline std::vector<int> redundant_parameters(const Matrix<double>& ov, size_t oR, size_t nR, double svd_thresh,
                                             Logger& log) {
  std::vector<int> red, ridx(nR);
  std::iota(ridx.begin(), ridx.end(), 0);
  // The screen acts on the eigenpairs with eigenvalue <= svd_thresh only.  When a Cholesky test proves
  // there are none, the decomposition would return an empty list: skip it (the same result; on a
  // well-conditioned overlap of dimension 64 it saves about 0.2 ms of host time per iteration).
  if (nR == 0 || (ov.rows() == ov.cols() && dense::eigenvalues_exceed(ov.rows(), ov.data(), svd_thresh))) return red;
  auto svds = svd_system(ov.rows(), ov.cols(), ov.data(), svd_thresh, true);
  for (const auto& s : svds) {
    if (ridx.empty()) break;
    std::vector<double> c;
    for (int i : ridx) c.push_back(std::abs(s.v.at(oR + i)));
    const size_t k = size_t(std::max_element(c.begin(), c.end()) - c.begin());
    red.push_back(ridx[k]);
    ridx.erase(ridx.begin() + k);
    log.msg("redundant parameter found, i = " + std::to_string(red.back()), Logger::Info);
  }
  return red;
}

using util::delete_parameters;

// Roots from `working_set` whose residual survived into `wparams` (reference :515-523).
template <class R>
std::vector<int> get_new_working_set(const std::vector<int>& working_set, const CVecRef<R>& params,
                                     const CVecRef<R>& wparams) {
  std::vector<int> out;
  for (auto i : find_ref(wparams, params)) out.push_back(working_set.at(i));
  return out;
}

// Solutions of `roots` built by axpy loops over P, Q, D (reference itsolv/util.h:218-239).
template <class R, class Q, class P>
void construct_solutions(const VecRef<R>& params, const std::vector<int>& roots, const Matrix<double>& sol,
                         const CVecRef<P>& pp, const CVecRef<Q>& qp, const CVecRef<Q>& dp, size_t oP, size_t oQ,
                         size_t oD, array::ArrayHandler<R, R>& hrr, array::ArrayHandler<R, P>& hrp,
                         array::ArrayHandler<R, Q>& hrq) {
  for (size_t i = 0; i < roots.size(); ++i) hrr.fill(0, params.at(i));
  for (size_t i = 0; i < roots.size(); ++i) {
    const auto root = roots[i];
    for (size_t j = 0; j < pp.size(); ++j) hrp.axpy(sol(root, oP + j), pp.at(j), params.at(i));
    for (size_t j = 0; j < qp.size(); ++j) hrq.axpy(sol(root, oQ + j), qp.at(j), params.at(i));
    for (size_t j = 0; j < dp.size(); ++j) hrq.axpy(sol(root, oD + j), dp.at(j), params.at(i));
  }
}

// Removes the Q parameters contributing least to any solution until nQ <= max_q (reference
// DSpaceResetter.h:13-23); XS: anything with dimensions() and eraseq(i).
template <class XS>
void resize_qspace(XS& xs, const Matrix<double>& solutions, size_t max_q, Logger& log) {
  log.msg("resize_qspace()", Logger::Trace);
  auto del = limit_qspace_size(xs.dimensions(), max_q, solutions, log);
  std::sort(del.begin(), del.end(), std::greater<int>());
  for (int i : del) xs.eraseq(size_t(i));
}

// Q indices with the largest overlap with each R parameter, descending (reference DSpaceResetter.h:32-54).
template <class R, class Q>
std::vector<int> max_overlap_with_R(const CVecRef<R>& rparams, const CVecRef<Q>& qparams,
                                    array::ArrayHandler<R, Q>& handler) {
  auto ov = subspace::util::overlap(rparams, qparams, handler);
  std::vector<int> qidx(qparams.size()), out;
  std::iota(qidx.begin(), qidx.end(), 0);
  for (size_t i = 0; i < rparams.size() && !qidx.empty(); ++i) {
    std::vector<double> o;
    for (int j : qidx) o.push_back(std::abs(ov(i, j)));
    const size_t k = size_t(std::max_element(o.begin(), o.end()) - o.begin());
    out.push_back(qidx[k]);
    qidx.erase(qidx.begin() + k);
  }
  std::sort(out.begin(), out.end(), std::greater<int>());
  return out;
}

// Every n_reset iterations turns the current solutions into Q vectors and clears D
// (reference DSpaceResetter.h:69-146).
template <class Q>
class DSpaceResetter {
 public:
  bool do_reset(size_t iter, const Dimensions& d) const {
    return ((iter + 1) % size_t(m_nreset) == 0 && d.nD > 0) || !m_solutions.empty();
  }
  void set_nreset(size_t n) { m_nreset = int(n); }
  int get_nreset() const { return m_nreset; }
  void set_max_Qsize(size_t n) { m_max_q = int(n); }
  int get_max_Qsize() const { return m_max_q; }

  template <class R, class P>
  std::vector<int> run(const VecRef<R>& rparams, subspace::XSpace<R, Q, P>& xs, const Matrix<double>& sol,
                       double norm_thresh, double svd_thresh, ArrayHandlers<R, Q, P>& h, Logger& log) {
    log.msg("DSpaceResetter::run()", Logger::Trace);
    if (m_solutions.empty() && !rparams.empty()) {
      const auto d = xs.dimensions();
      const auto& S = xs.data.at(EqnData::S);
      std::vector<int> qall(d.nQ);
      std::iota(qall.begin(), qall.end(), 0);
      auto proj = dspace::construct_projected_solution(sol, d, qall);
      auto ovp = dspace::construct_projected_solutions_overlap(proj, S, d, qall);
      dspace::remove_null_norm_and_normalise(proj, ovp, norm_thresh, log);
      proj = dspace::remove_null_projected_solutions(proj, ovp, svd_thresh);
      ovp = dspace::construct_projected_solutions_overlap(proj, S, d, qall);
      dspace::remove_null_norm_and_normalise(proj, ovp, norm_thresh, log);
      const size_t nC = proj.rows();
      for (size_t i = 0; i < nC; ++i) {
        m_solutions.emplace_back(h.qr().copy(rparams.front().get()));
        h.qr().fill(0, m_solutions.back());
      }
      std::vector<int> roots(nC);
      std::iota(roots.begin(), roots.end(), 0);
      construct_solutions(wrap(m_solutions.begin(), m_solutions.end()), roots, proj, CVecRef<P>{}, xs.cparamsq(),
                          xs.cparamsd(), 0, 0, d.nQ, h.qq(), h.qp(), h.qq());
      VecRef<Q> none_p, none_a;
      xs.update_dspace(none_p, none_a);
    }
    const size_t nR = std::min(rparams.size(), m_solutions.size());
    for (size_t i = 0; i < nR; ++i) {
      h.rq().copy(rparams[i], m_solutions.front());
      m_solutions.pop_front();
    }
    const auto wparams = cwrap(rparams.begin(), rparams.begin() + nR);
    for (int i : max_overlap_with_R(wparams, xs.cparamsq(), h.rq())) xs.eraseq(size_t(i));
    if (xs.dimensions().nQ + nR > size_t(m_max_q))
      resize_qspace(xs, sol, size_t(m_max_q) > nR ? size_t(m_max_q) - nR : 0, log);
    std::vector<int> ws(nR);
    std::iota(ws.begin(), ws.end(), 0);
    return ws;
  }

 private:
  int m_nreset = std::numeric_limits<int>::max();
  int m_max_q = std::numeric_limits<int>::max();
  std::list<Q> m_solutions;
};

}  // namespace molpro::linalg::itsolv::detail
