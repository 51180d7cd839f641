// Containers of references to vectors, as the reference's itsolv/wrap.h passes them
// (VecRef<R> = std::vector<std::reference_wrapper<R>>; wrap / cwrap / wrap_arg / find_ref).
#pragma once
#include <functional>
#include <iterator>
#include <memory>
#include <vector>

namespace molpro::linalg::itsolv {

template <class R>
using VecRef = std::vector<std::reference_wrapper<R>>;
template <class R>
using CVecRef = std::vector<std::reference_wrapper<const R>>;

template <class R>
VecRef<R> wrap(std::vector<R>& v) {
  return VecRef<R>(v.begin(), v.end());
}
template <class R>
CVecRef<R> wrap(const std::vector<R>& v) {
  return CVecRef<R>(v.begin(), v.end());
}
template <class R>
CVecRef<R> cwrap(const std::vector<R>& v) {
  return CVecRef<R>(v.begin(), v.end());
}
template <class R>
CVecRef<R> cwrap(const VecRef<R>& v) {
  return CVecRef<R>(v.begin(), v.end());
}
template <class R>
CVecRef<R> cwrap(const CVecRef<R>& v) {
  return v;
}
namespace detail {
template <class T>
struct unref {
  using type = T;
  static T& get(T& x) { return x; }
};
template <class T>
struct unref<std::reference_wrapper<T>> {
  using type = T;
  static T& get(const std::reference_wrapper<T>& x) { return x.get(); }
};
}  // namespace detail

// From an iterator range over objects or over reference_wrappers.
template <class It>
auto wrap(It b, It e) {
  using V = std::remove_const_t<typename std::iterator_traits<It>::value_type>;
  using U = std::remove_const_t<typename detail::unref<V>::type>;
  VecRef<U> r;
  for (; b != e; ++b) r.emplace_back(const_cast<U&>(detail::unref<V>::get(const_cast<V&>(*b))));
  return r;
}
template <class It>
auto cwrap(It b, It e) {
  using V = std::remove_const_t<typename std::iterator_traits<It>::value_type>;
  using U = std::remove_const_t<typename detail::unref<V>::type>;
  CVecRef<U> r;
  for (; b != e; ++b) r.emplace_back(static_cast<const U&>(detail::unref<V>::get(const_cast<V&>(*b))));
  return r;
}
template <class R>
VecRef<R> wrap_arg(R& x) {
  return VecRef<R>{std::ref(x)};
}
template <class R>
CVecRef<R> cwrap_arg(const R& x) {
  return CVecRef<R>{std::cref(x)};
}
template <class R>
VecRef<R> const_cast_wrap(const CVecRef<R>& v) {
  VecRef<R> r;
  for (auto& x : v) r.emplace_back(const_cast<R&>(x.get()));
  return r;
}

// Indices in `params` of the objects referenced by `wparams` (identity by address).
template <class R, class S>
std::vector<size_t> find_ref(const CVecRef<R>& wparams, const CVecRef<S>& params) {
  std::vector<size_t> out;
  for (auto& w : wparams)
    for (size_t i = 0; i < params.size(); ++i)
      if (std::addressof(params[i].get()) == std::addressof(w.get())) {
        out.push_back(i);
        break;
      }
  return out;
}

}  // namespace molpro::linalg::itsolv
