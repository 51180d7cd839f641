// The handler bundle injected into a solver: ArrayHandlers<R, Q, P> with rr, qq, pp, rq, rp, qr, qp
// (reference itsolv/ArrayHandlers.h:24-112), built as
//   ArrayHandlers<R, Q, P>::create().rr(h1).qq(h2)...build()
// Handlers not given default to DefaultHandlers<R, Q, P>, which a vector-type header specialises
// (hbm_handlers.h for HBM vectors; the oracle for std::vector<double>).
#pragma once
#include <map>
#include <memory>
#include <stdexcept>

#include "array_handler.h"

namespace molpro::linalg::itsolv {

template <class T, class S>
struct DefaultHandler {
  static std::shared_ptr<array::ArrayHandler<T, S>> make() { return nullptr; }
};

template <typename R, typename Q = R, typename P = std::map<size_t, typename R::value_type>>
class ArrayHandlers {
  template <class T, class S>
  using H = std::shared_ptr<array::ArrayHandler<T, S>>;

 public:
  class Builder {
   public:
    template <class T, class S>
    class Slot {
     public:
      explicit Slot(Builder* b) : b_(b) {}
      Builder& operator()(const H<T, S>& h) {
        h_ = h;
        return *b_;
      }
      H<T, S> get() const {
        auto h = h_ ? h_ : DefaultHandler<T, S>::make();
        if (!h) throw std::logic_error("ArrayHandlers: no handler given and no default for this type pair");
        return h;
      }

     private:
      Builder* b_;
      H<T, S> h_;
    };
    Builder() : rr(this), qq(this), pp(this), rq(this), rp(this), qr(this), qp(this) {}
    Builder(const Builder&) = delete;
    ArrayHandlers build() { return ArrayHandlers(rr.get(), qq.get(), pp.get(), rq.get(), rp.get(), qr.get(), qp.get()); }
    std::shared_ptr<ArrayHandlers> build_shared() { return std::make_shared<ArrayHandlers>(build()); }
    Slot<R, R> rr;
    Slot<Q, Q> qq;
    Slot<P, P> pp;
    Slot<R, Q> rq;
    Slot<R, P> rp;
    Slot<Q, R> qr;
    Slot<Q, P> qp;
  };

  ArrayHandlers(H<R, R> rr, H<Q, Q> qq, H<P, P> pp, H<R, Q> rq, H<R, P> rp, H<Q, R> qr, H<Q, P> qp)
      : m_rr(rr), m_qq(qq), m_pp(pp), m_rq(rq), m_rp(rp), m_qr(qr), m_qp(qp) {}
  ArrayHandlers() : ArrayHandlers(Builder{}.build()) {}

  static Builder create() { return {}; }

  auto& rr() { return *m_rr; }
  auto& qq() { return *m_qq; }
  auto& pp() { return *m_pp; }
  auto& rq() { return *m_rq; }
  auto& qr() { return *m_qr; }
  auto& rp() { return *m_rp; }
  auto& qp() { return *m_qp; }

 private:
  H<R, R> m_rr;
  H<Q, Q> m_qq;
  H<P, P> m_pp;
  H<R, Q> m_rq;
  H<R, P> m_rp;
  H<Q, R> m_qr;
  H<Q, P> m_qp;
};

}  // namespace molpro::linalg::itsolv
