// The subspace: P (sparse vectors), Q (history: parameter + action pairs) and D (stabilised solution
// projections), and the equation data S, H, rhs in the order P | Q | D.
//
// Semantics restated from the reference's subspace layer:
//   Dimensions                    itsolv/subspace/Dimensions.h:4-17
//   util::overlap (gemm / pairwise lower-triangle dots)   subspace/util.h:22-62
//   xspace::update_qspace_data    subspace/XSpace.h:30-83   (new Q rows/cols of S and H)
//   update_dspace_*_data          subspace/XSpace.h:86-148
//   XSpace                        subspace/XSpace.h:151-312
//   QSpace::update                subspace/QSpace.h:76-116  (new vectors are PREPENDED to Q)
//   PSpace, DSpace                subspace/PSpace.h, DSpace.h
// Every vector operation goes through the ArrayHandlers bundle; the host only touches the small
// matrices.
#pragma once
#include <list>
#include <map>
#include <memory>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "common.h"

namespace molpro::linalg::itsolv::subspace {

struct Dimensions {
  Dimensions() = default;
  Dimensions(size_t np, size_t nq, size_t nd) : nP(np), nQ(nq), nD(nd), nX(np + nq + nd), oP(0), oQ(np), oD(np + nq) {}
  size_t nP = 0, nQ = 0, nD = 0, nX = 0;
  size_t oP = 0, oQ = 0, oD = 0;
  size_t nRHS = 0;
};

enum class EqnData { H, S, rhs, value };
using SubspaceData = std::map<EqnData, Matrix<double>>;

template <EqnData... Kinds>
SubspaceData null_data() {
  SubspaceData d;
  (d.emplace(Kinds, Matrix<double>{}), ...);
  return d;
}

namespace util {

// Overlap matrix between two sets through a handler whose (left, right) types are (R, Q) or the
// reverse; the reversed case runs gemm_inner(right, left) and transposes (subspace/util.h:33-41).
template <class L, class Rt, class Z, class W>
Matrix<double> overlap(const CVecRef<L>& left, const CVecRef<Rt>& right, array::ArrayHandler<Z, W>& handler) {
  if constexpr (std::is_same_v<L, Z> && std::is_same_v<Rt, W>) {
    return handler.gemm_inner(left, right);
  } else {
    static_assert(std::is_same_v<L, W> && std::is_same_v<Rt, Z>, "handler does not match the vector types");
    auto t = handler.gemm_inner(right, left);
    Matrix<double> m({left.size(), right.size()});
    transpose_copy(m, t);
    return m;
  }
}

// Symmetric overlap of one set by pairwise dots over the lower triangle (subspace/util.h:55-62),
// or by one batched gemm_inner where the handlers support it (array::batched_symmetric_overlap).
template <class R>
Matrix<double> overlap(const CVecRef<R>& params, array::ArrayHandler<R, R>& handler) {
  Matrix<double> m({params.size(), params.size()});
  if constexpr (array::batched_symmetric_overlap<R>::value) {
    if (params.empty()) return m;
    auto g = handler.gemm_inner(params, params);
    for (size_t i = 0; i < m.rows(); ++i)
      for (size_t j = 0; j <= i; ++j) m(i, j) = m(j, i) = g(i, j);
    return m;
  }
  for (size_t i = 0; i < m.rows(); ++i)
    for (size_t j = 0; j <= i; ++j) m(i, j) = m(j, i) = handler.dot(params[i], params[j]);
  return m;
}

}  // namespace util

template <class R, class P>
class PSpace {
 public:
  void update(const CVecRef<P>& params, array::ArrayHandler<P, P>& handler) {
    for (const auto& p : params) m_params.emplace_back(handler.copy(p));
  }
  CVecRef<P> cparams() const { return cwrap(m_params); }
  VecRef<P> params() { return wrap(m_params); }
  size_t size() const { return m_params.size(); }
  void erase(size_t i) { m_params.erase(m_params.begin() + i); }

 private:
  std::vector<P> m_params;
};

template <class R, class Q, class P>
class QSpace {
 public:
  QSpace(std::shared_ptr<ArrayHandlers<R, Q, P>> h, std::shared_ptr<Logger> log)
      : m_handlers(std::move(h)), m_logger(std::move(log)) {}

  // Prepends copies of (params, actions) and splices the new blocks qq, qx, xq into `data`.
  void update(const CVecRef<R>& params, const CVecRef<R>& actions, const SubspaceData& qq, const SubspaceData& qx,
              const SubspaceData& xq, const Dimensions& dims, SubspaceData& data) {
    auto pos = m_items.begin();
    for (size_t i = 0; i < params.size(); ++i)
      m_items.insert(pos, Item{std::make_unique<Q>(m_handlers->qr().copy(params[i])),
                               std::make_unique<Q>(m_handlers->qr().copy(actions[i]))});
    const size_t nn = params.size(), nx = dims.nX, oq = dims.oQ, nxn = nx + nn;
    for (auto d : {EqnData::H, EqnData::S}) {
      const auto& old = data[d];
      Matrix<double> m({nxn, nxn});
      // Map an old index to its new position: P unchanged, Q and D shifted by nn.
      auto pos_of = [&](size_t i) { return i < oq ? i : i + nn; };
      for (size_t i = 0; i < nx; ++i)
        for (size_t j = 0; j < nx; ++j) m(pos_of(i), pos_of(j)) = old(i, j);
      const auto& bqq = qq.at(d);
      const auto& bqx = qx.at(d);
      const auto& bxq = xq.at(d);
      for (size_t i = 0; i < nn; ++i)
        for (size_t j = 0; j < nn; ++j) m(oq + i, oq + j) = bqq(i, j);
      for (size_t i = 0; i < nn; ++i)
        for (size_t j = 0; j < nx; ++j) m(oq + i, pos_of(j)) = bqx(i, j);
      for (size_t i = 0; i < nx; ++i)
        for (size_t j = 0; j < nn; ++j) m(pos_of(i), oq + j) = bxq(i, j);
      data[d] = std::move(m);
    }
    const auto& rq = qq.at(EqnData::rhs);
    if (!rq.empty()) {
      const auto& old = data[EqnData::rhs];
      Matrix<double> m({nxn, dims.nRHS});
      for (size_t i = 0; i < nx; ++i)
        for (size_t j = 0; j < dims.nRHS; ++j) m(i < oq ? i : i + nn, j) = old(i, j);
      for (size_t i = 0; i < nn; ++i)
        for (size_t j = 0; j < dims.nRHS; ++j) m(oq + i, j) = rq(i, j);
      data[EqnData::rhs] = std::move(m);
    }
    if (m_logger->data_dump) {
      m_logger->msg("S = " + as_string(data.at(EqnData::S)), Logger::Info);
      m_logger->msg("H = " + as_string(data.at(EqnData::H)), Logger::Info);
    }
  }

  void erase(size_t i) { m_items.erase(std::next(m_items.begin(), i)); }
  size_t size() const { return m_items.size(); }
  VecRef<Q> params() {
    VecRef<Q> r;
    for (auto& it : m_items) r.emplace_back(*it.param);
    return r;
  }
  VecRef<Q> actions() {
    VecRef<Q> r;
    for (auto& it : m_items) r.emplace_back(*it.action);
    return r;
  }
  CVecRef<Q> cparams() const {
    CVecRef<Q> r;
    for (auto& it : m_items) r.emplace_back(*it.param);
    return r;
  }
  CVecRef<Q> cactions() const {
    CVecRef<Q> r;
    for (auto& it : m_items) r.emplace_back(*it.action);
    return r;
  }

 private:
  struct Item {
    std::unique_ptr<Q> param;
    std::unique_ptr<Q> action;
  };
  std::shared_ptr<ArrayHandlers<R, Q, P>> m_handlers;
  std::shared_ptr<Logger> m_logger;
  std::list<Item> m_items;  // newest first
};

template <class Q>
class DSpace {
 public:
  // Clears the D space and moves params / actions in.
  void update(VecRef<Q>& params, VecRef<Q>& actions) {
    m_params.clear();
    m_actions.clear();
    for (size_t i = 0; i < params.size(); ++i) {
      m_params.emplace_back(std::move(params[i].get()));
      m_actions.emplace_back(std::move(actions[i].get()));
    }
  }
  void erase(size_t i) {
    m_params.erase(m_params.begin() + i);
    m_actions.erase(m_actions.begin() + i);
  }
  size_t size() const { return m_params.size(); }
  VecRef<Q> params() { return wrap(m_params); }
  VecRef<Q> actions() { return wrap(m_actions); }
  CVecRef<Q> cparams() const { return cwrap(m_params); }
  CVecRef<Q> cactions() const { return cwrap(m_actions); }

 private:
  std::vector<Q> m_params, m_actions;
};

// New rows / columns of the equation data for new parameters (reference XSpace.h:14-27).
struct NewData {
  NewData(size_t nnew, size_t nx, size_t nrhs) {
    for (auto d : {EqnData::H, EqnData::S}) {
      qq[d] = Matrix<double>({nnew, nnew});
      qx[d] = Matrix<double>({nnew, nx});
      xq[d] = Matrix<double>({nx, nnew});
    }
    qq[EqnData::rhs] = Matrix<double>({nnew, nrhs});
  }
  SubspaceData qq, qx, xq;
};

// The full subspace and its equation data (reference XSpace.h:151-312).
template <class R, class Q, class P>
class XSpace {
 public:
  XSpace(std::shared_ptr<ArrayHandlers<R, Q, P>> h, std::shared_ptr<Logger> log)
      : qspace(h, log), m_handlers(std::move(h)), m_logger(std::move(log)) {
    data = null_data<EqnData::H, EqnData::S, EqnData::rhs>();
  }

  SubspaceData data;

  const Dimensions& dimensions() const { return m_dim; }
  size_t size() const { return m_dim.nX; }
  void set_hermiticity(bool h) { m_hermitian = h; }
  bool get_hermiticity() const { return m_hermitian; }
  void set_action_action() { m_action_dot_action = true; }

  void update_qspace(const CVecRef<R>& params, const CVecRef<R>& actions) {
    m_logger->msg("XSpace::update_qspace", Logger::Trace);
    auto nd = new_qspace_data(params, actions);
    qspace.update(params, actions, nd.qq, nd.qx, nd.xq, m_dim, data);
    update_dimensions();
  }

  // Replaces the D space and recomputes its blocks of S and H (reference XSpace.h:174-187).
  void update_dspace(VecRef<Q>& params, VecRef<Q>& actions) {
    dspace.update(params, actions);
    update_dimensions();
    for (auto e : {EqnData::H, EqnData::S}) data[e].resize({m_dim.nX, m_dim.nX});
    auto& hqq = m_handlers->qq();
    auto& hqp = m_handlers->qp();
    const auto pp = cparamsp();
    const auto qp = cparamsq(), qa = cactionsq(), dp = cparamsd(), da = cactionsd();
    const auto& d = m_dim;
    // overlap blocks
    {
      auto sdd = util::overlap(dp, hqq);
      auto sdp = util::overlap(dp, pp, hqp);
      auto sdq = util::overlap(dp, qp, hqq);
      auto& S = data[EqnData::S];
      S.slice({d.oD, d.oD}, {d.oD + d.nD, d.oD + d.nD}) = sdd;
      S.slice({d.oD, d.oP}, {d.oD + d.nD, d.oP + d.nP}) = sdp;
      S.slice({d.oD, d.oQ}, {d.oD + d.nD, d.oQ + d.nQ}) = sdq;
      transpose_copy(S.slice({d.oP, d.oD}, {d.oP + d.nP, d.oD + d.nD}), sdp);
      transpose_copy(S.slice({d.oQ, d.oD}, {d.oQ + d.nQ, d.oD + d.nD}), sdq);
    }
    // action blocks
    {
      auto hdd = util::overlap(dp, da, hqq);
      auto hpd = util::overlap(pp, da, hqp);
      auto hqd = util::overlap(qp, da, hqq);
      auto hdq = util::overlap(dp, qa, hqq);
      auto& H = data[EqnData::H];
      H.slice({d.oD, d.oD}, {d.oD + d.nD, d.oD + d.nD}) = hdd;
      H.slice({d.oP, d.oD}, {d.oP + d.nP, d.oD + d.nD}) = hpd;
      H.slice({d.oQ, d.oD}, {d.oQ + d.nQ, d.oD + d.nD}) = hqd;
      H.slice({d.oD, d.oQ}, {d.oD + d.nD, d.oQ + d.nQ}) = hdq;
      transpose_copy(H.slice({d.oD, d.oP}, {d.oD + d.nD, d.oP + d.nP}), hpd);
    }
    data[EqnData::rhs].resize({m_dim.nX, m_dim.nRHS});
    if (m_dim.nRHS) {
      auto rd = util::overlap(dp, rhs(), hqq);
      data[EqnData::rhs].slice({d.oD, 0}, {d.oD + d.nD, d.nRHS}) = rd;
    }
  }

  // P space on an empty subspace, hermitian only (reference XSpace.h:191-205).
  void update_pspace(const CVecRef<P>& params, const std::vector<double>& pp_action_matrix) {
    if (m_dim.nX != 0) throw std::logic_error("P space can only be added to an empty subspace");
    if (!m_hermitian) throw std::runtime_error("P space can only be used with hermitian kernels");
    pspace.update(params, m_handlers->pp());
    update_dimensions();
    const size_t np = m_dim.nP;
    update_rhs_with_pspace();
    data[EqnData::S] = util::overlap(params, m_handlers->pp());
    data[EqnData::H] = Matrix<double>({np, np});
    for (size_t i = 0, ij = 0; i < np; ++i)
      for (size_t j = 0; j < np; ++j, ++ij) data[EqnData::H](i, j) = pp_action_matrix.at(ij);
  }

  void add_rhs_equations(const CVecRef<R>& rhs_) {
    for (const auto& r : rhs_) m_rhs.emplace_back(m_handlers->qr().copy(r));
    for (const auto& r : rhs_) {
      const double d = std::abs(m_handlers->rr().dot(r, r));
      if (d == 0) throw std::runtime_error("RHS vector cannot be zero");
      m_rhs_norm.push_back(std::sqrt(d));
    }
    update_dimensions();
    update_rhs_with_pspace();
  }
  CVecRef<Q> rhs() const { return cwrap(m_rhs); }
  const std::vector<double>& rhs_norm() const { return m_rhs_norm; }

  void eraseq(size_t i) {
    qspace.erase(i);
    remove_data(m_dim.oQ + i);
    update_dimensions();
  }
  void erasep(size_t i) {
    pspace.erase(i);
    remove_data(m_dim.oP + i);
    update_dimensions();
  }
  void erased(size_t i) {
    dspace.erase(i);
    remove_data(m_dim.oD + i);
    update_dimensions();
  }

  VecRef<P> paramsp() { return pspace.params(); }
  VecRef<Q> paramsq() { return qspace.params(); }
  VecRef<Q> actionsq() { return qspace.actions(); }
  VecRef<Q> paramsd() { return dspace.params(); }
  VecRef<Q> actionsd() { return dspace.actions(); }
  CVecRef<P> cparamsp() const { return pspace.cparams(); }
  CVecRef<Q> cparamsq() const { return qspace.cparams(); }
  CVecRef<Q> cactionsq() const { return qspace.cactions(); }
  CVecRef<Q> cparamsd() const { return dspace.cparams(); }
  CVecRef<Q> cactionsd() const { return dspace.cactions(); }

  PSpace<R, P> pspace;
  QSpace<R, Q, P> qspace;
  DSpace<Q> dspace;

 private:
  // reference xspace::update_qspace_data (XSpace.h:30-83)
  NewData new_qspace_data(const CVecRef<R>& params, const CVecRef<R>& actions) {
    auto& h = *m_handlers;
    const auto& d = m_dim;
    const size_t nn = params.size();
    NewData nd(nn, d.nX, m_rhs.size());
    auto& qq = nd.qq;
    auto& qx = nd.qx;
    auto& xq = nd.xq;
    const auto pp = cparamsp();
    const auto qp = cparamsq(), qa = cactionsq(), dp = cparamsd(), da = cactionsd();
    const auto& lhs_h = m_action_dot_action ? actions : params;
    bool fused = false;
    // S(R, P) and H(P, R) as one sparse inner product over [params, actions] (one launch, one
    // reduction; each element is the same sum over its P vector's entries either way), queued ahead of
    // the dense rows where the handler can (array::queued_overlap): the wait for those covers it
    std::function<Matrix<double>()> p_rows;
    CVecRef<R> both;
    if constexpr (array::batched_symmetric_overlap<R>::value) {
      if (m_hermitian && d.nP > 0 && nn > 0) {
        both.assign(params.begin(), params.end());
        both.insert(both.end(), actions.begin(), actions.end());
        using array::queued_overlap;
        p_rows = queued_overlap(h.rp(), both, pp);
      }
    }
    if constexpr (std::is_same_v<R, Q>) {
      // every block whose rows are the new parameters, as one batched overlap where the handler has
      // it: columns [params, actions, Q params, Q actions, D params, D actions, rhs]
      Matrix<double> g;
      using array::fused_overlap_rows;
      if (!m_action_dot_action && nn > 0 &&
          fused_overlap_rows(h.rr(), params, std::vector<CVecRef<R>>{params, actions, qp, qa, dp, da, rhs()}, g)) {
        fused = true;
        const size_t cA = nn, cQ = 2 * nn, cQA = cQ + d.nQ, cD = cQA + d.nQ, cDA = cD + d.nD, cR = cDA + d.nD;
        for (size_t i = 0; i < nn; ++i) {
          for (size_t j = 0; j <= i; ++j) qq[EqnData::S](i, j) = qq[EqnData::S](j, i) = g(i, j);
          for (size_t j = 0; j < nn; ++j) qq[EqnData::H](i, j) = g(i, cA + j);
          for (size_t j = 0; j < d.nQ; ++j) {
            qx[EqnData::S](i, d.oQ + j) = g(i, cQ + j);
            qx[EqnData::H](i, d.oQ + j) = g(i, cQA + j);
          }
          for (size_t j = 0; j < d.nD; ++j) {
            qx[EqnData::S](i, d.oD + j) = g(i, cD + j);
            qx[EqnData::H](i, d.oD + j) = g(i, cDA + j);
          }
          for (size_t j = 0; j < m_rhs.size(); ++j) qq[EqnData::rhs](i, j) = g(i, cR + j);
        }
      }
      // action . action (DIIS): the S rows from the parameters, the H rows from the actions -- two
      // batched overlaps: [params, Q params, D params, rhs] and [actions, Q actions, D actions]
      Matrix<double> ga;
      if (m_action_dot_action && nn > 0 &&
          fused_overlap_rows(h.rr(), params, std::vector<CVecRef<R>>{params, qp, dp, rhs()}, g) &&
          fused_overlap_rows(h.rr(), actions, std::vector<CVecRef<R>>{actions, qa, da}, ga)) {
        fused = true;
        const size_t cQ = nn, cD = cQ + d.nQ, cR = cD + d.nD;
        for (size_t i = 0; i < nn; ++i) {
          for (size_t j = 0; j <= i; ++j) {
            qq[EqnData::S](i, j) = qq[EqnData::S](j, i) = g(i, j);
            qq[EqnData::H](i, j) = qq[EqnData::H](j, i) = ga(i, j);
          }
          for (size_t j = 0; j < d.nQ; ++j) {
            qx[EqnData::S](i, d.oQ + j) = g(i, cQ + j);
            qx[EqnData::H](i, d.oQ + j) = ga(i, nn + j);
          }
          for (size_t j = 0; j < d.nD; ++j) {
            qx[EqnData::S](i, d.oD + j) = g(i, cD + j);
            qx[EqnData::H](i, d.oD + j) = ga(i, nn + d.nQ + j);
          }
          for (size_t j = 0; j < m_rhs.size(); ++j) qq[EqnData::rhs](i, j) = g(i, cR + j);
        }
      }
    }
    if (!fused) {
      qq[EqnData::S] = util::overlap(params, h.rr());
      qx[EqnData::S].slice({0, d.oQ}, {nn, d.oQ + d.nQ}) = util::overlap(params, qp, h.rq());
      qx[EqnData::S].slice({0, d.oD}, {nn, d.oD + d.nD}) = util::overlap(params, dp, h.rq());
      qq[EqnData::H] = m_action_dot_action ? util::overlap(actions, h.rr()) : util::overlap(params, actions, h.rr());
      qx[EqnData::H].slice({0, d.oQ}, {nn, d.oQ + d.nQ}) = util::overlap(lhs_h, qa, h.rq());
      qx[EqnData::H].slice({0, d.oD}, {nn, d.oD + d.nD}) = util::overlap(lhs_h, da, h.rq());
      qq[EqnData::rhs] = util::overlap(params, rhs(), h.rq());
    }
    bool p_rows_done = false;
    if constexpr (array::batched_symmetric_overlap<R>::value) {
      if (!both.empty()) {
        const auto g = p_rows ? p_rows() : util::overlap(both, pp, h.rp());
        for (size_t i = 0; i < nn; ++i)
          for (size_t j = 0; j < d.nP; ++j) {
            qx[EqnData::S](i, d.oP + j) = g(i, j);
            xq[EqnData::H](d.oP + j, i) = g(nn + i, j);
          }
        p_rows_done = true;
      }
    }
    if (!p_rows_done) qx[EqnData::S].slice({0, d.oP}, {nn, d.oP + d.nP}) = util::overlap(params, pp, h.rp());
    if (m_hermitian) {
      if (!p_rows_done) xq[EqnData::H].slice({d.oP, 0}, {d.oP + d.nP, nn}) = util::overlap(pp, actions, h.rp());
      transpose_copy(xq[EqnData::H].slice({d.oQ, 0}, {d.oQ + d.nQ, nn}), qx[EqnData::H].slice({0, d.oQ}, {nn, d.oQ + d.nQ}));
      transpose_copy(xq[EqnData::H].slice({d.oD, 0}, {d.oD + d.nD, nn}), qx[EqnData::H].slice({0, d.oD}, {nn, d.oD + d.nD}));
      transpose_copy(qx[EqnData::H].slice({0, d.oP}, {nn, d.oP + d.nP}), xq[EqnData::H].slice({d.oP, 0}, {d.oP + d.nP, nn}));
    } else {
      xq[EqnData::H].slice({d.oQ, 0}, {d.oQ + d.nQ, nn}) = util::overlap(qp, actions, h.rq());
      xq[EqnData::H].slice({d.oD, 0}, {d.oD + d.nD, nn}) = util::overlap(dp, actions, h.rq());
    }
    transpose_copy(xq[EqnData::S].slice({d.oP, 0}, {d.oP + d.nP, nn}), qx[EqnData::S].slice({0, d.oP}, {nn, d.oP + d.nP}));
    transpose_copy(xq[EqnData::S].slice({d.oQ, 0}, {d.oQ + d.nQ, nn}), qx[EqnData::S].slice({0, d.oQ}, {nn, d.oQ + d.nQ}));
    transpose_copy(xq[EqnData::S].slice({d.oD, 0}, {d.oD + d.nD, nn}), qx[EqnData::S].slice({0, d.oD}, {nn, d.oD + d.nD}));
    if (m_logger->data_dump) {
      m_logger->msg("Sqq = " + as_string(qq[EqnData::S]), Logger::Info);
      m_logger->msg("Hqq = " + as_string(qq[EqnData::H]), Logger::Info);
    }
    return nd;
  }

  void update_dimensions() {
    m_dim = Dimensions(pspace.size(), qspace.size(), dspace.size());
    m_dim.nRHS = m_rhs.size();
  }
  void update_rhs_with_pspace() {
    data[EqnData::rhs].resize({m_dim.nP, m_dim.nRHS});
    if (m_dim.nP && m_dim.nRHS) data[EqnData::rhs] = util::overlap(cparamsp(), rhs(), m_handlers->qp());
  }
  void remove_data(size_t i) {
    for (auto e : {EqnData::H, EqnData::S}) data[e].remove_row_col(i, i);
    if (data.count(EqnData::rhs) && !data[EqnData::rhs].empty()) data[EqnData::rhs].remove_row(i);
    if (data.count(EqnData::value) && !data[EqnData::value].empty()) data[EqnData::value].remove_row(i);
  }

  std::shared_ptr<ArrayHandlers<R, Q, P>> m_handlers;
  std::shared_ptr<Logger> m_logger;
  Dimensions m_dim;
  std::vector<Q> m_rhs;
  std::vector<double> m_rhs_norm;
  bool m_hermitian = false;
  bool m_action_dot_action = false;
};

}  // namespace molpro::linalg::itsolv::subspace
