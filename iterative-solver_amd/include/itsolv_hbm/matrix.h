// Row-major dense matrix for subspace quantities (S, H, rhs, solution coefficients).
//
// Interface restated from the reference's itsolv::subspace::Matrix (itsolv/subspace/Matrix.h:27-278):
// row-major storage (:23, :59), rectangular slices assignable from slices / matrices, resize that
// keeps the overlapping top-left block (:126-139), remove_row / remove_col (:142-163) and
// transpose_copy (:280-286).  These matrices hold at most a few hundred rows and live on the host.
#pragma once
#include <algorithm>
#include <cassert>
#include <cstddef>
#include <iomanip>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace molpro::linalg::itsolv::subspace {

template <typename T>
class Matrix {
 public:
  using value_type = T;
  using index_type = size_t;
  using coord_type = std::pair<size_t, size_t>;

  // View of a rectangular block [r0, r1) x [c0, c1) of a matrix.
  class Slice {
   public:
    Slice(Matrix& m, coord_type ul, coord_type br) : m_(&m), r0_(ul.first), c0_(ul.second), r1_(br.first), c1_(br.second) {
      if (r0_ > r1_ || c0_ > c1_) throw std::runtime_error("Matrix slice: corners out of order");
      if (r1_ > m.rows() || c1_ > m.cols()) throw std::runtime_error("Matrix slice: out of range");
    }
    Slice(const Slice&) = delete;
    Slice(Slice&&) noexcept = default;

    size_t rows() const { return r1_ - r0_; }
    size_t cols() const { return c1_ - c0_; }
    coord_type dimensions() const { return {rows(), cols()}; }
    T& operator()(size_t i, size_t j) { return (*m_)(r0_ + i, c0_ + j); }
    T operator()(size_t i, size_t j) const { return (*m_)(r0_ + i, c0_ + j); }

    template <class Src>
    Slice& assign(const Src& src) {
      if (src.rows() != rows() || src.cols() != cols())
        throw std::runtime_error("Matrix slice assignment: dimensions differ");
      // Copy through a buffer so that overlapping source and destination blocks are safe.
      std::vector<T> buf(rows() * cols());
      for (size_t i = 0; i < rows(); ++i)
        for (size_t j = 0; j < cols(); ++j) buf[i * cols() + j] = src(i, j);
      for (size_t i = 0; i < rows(); ++i)
        for (size_t j = 0; j < cols(); ++j) (*this)(i, j) = buf[i * cols() + j];
      return *this;
    }
    Slice& operator=(const Slice& s) { return assign(s); }
    Slice& operator=(Slice&& s) { return assign(s); }
    Slice& operator=(const Matrix& m) { return assign(m); }
    Slice& operator=(const typename Matrix::CSlice& s) { return assign(s); }

    Slice& scal(T a) {
      for (size_t i = 0; i < rows(); ++i)
        for (size_t j = 0; j < cols(); ++j) (*this)(i, j) *= a;
      return *this;
    }
    Slice& fill(T a) {
      for (size_t i = 0; i < rows(); ++i)
        for (size_t j = 0; j < cols(); ++j) (*this)(i, j) = a;
      return *this;
    }
    template <class Src>
    Slice& axpy(T a, const Src& x) {
      if (x.rows() != rows() || x.cols() != cols()) throw std::runtime_error("Matrix slice axpy: dimensions differ");
      for (size_t i = 0; i < rows(); ++i)
        for (size_t j = 0; j < cols(); ++j) (*this)(i, j) += a * x(i, j);
      return *this;
    }

   private:
    Matrix* m_;
    size_t r0_, c0_, r1_, c1_;
  };

  class CSlice {
   public:
    CSlice(const Matrix& m, coord_type ul, coord_type br) : s_(const_cast<Matrix&>(m), ul, br) {}
    size_t rows() const { return s_.rows(); }
    size_t cols() const { return s_.cols(); }
    coord_type dimensions() const { return s_.dimensions(); }
    T operator()(size_t i, size_t j) const { return s_(i, j); }

   private:
    Slice s_;
  };

  Matrix() = default;
  explicit Matrix(coord_type dims) : rows_(dims.first), cols_(dims.second), buf_(dims.first * dims.second) {}
  Matrix(std::vector<T>&& data, coord_type dims) : rows_(dims.first), cols_(dims.second), buf_(std::move(data)) {
    if (buf_.size() != size()) throw std::runtime_error("Matrix: data buffer of the wrong size");
  }
  Matrix(const std::vector<T>& data, coord_type dims) : rows_(dims.first), cols_(dims.second), buf_(data) {
    if (buf_.size() != size()) throw std::runtime_error("Matrix: data buffer of the wrong size");
  }

  T& operator()(size_t i, size_t j) { return buf_[i * cols_ + j]; }
  T operator()(size_t i, size_t j) const { return buf_[i * cols_ + j]; }
  const std::vector<T>& data() const& { return buf_; }
  std::vector<T>&& data() && {
    rows_ = cols_ = 0;
    return std::move(buf_);
  }
  T* raw() { return buf_.data(); }

  size_t rows() const { return rows_; }
  size_t cols() const { return cols_; }
  size_t size() const { return rows_ * cols_; }
  bool empty() const { return size() == 0; }
  coord_type dimensions() const { return {rows_, cols_}; }
  void fill(T v) { std::fill(buf_.begin(), buf_.end(), v); }
  void clear() { resize({0, 0}); }
  //! Row-major index -> (row, column) (reference Matrix.h:80-86).
  coord_type to_coord(size_t ind) const {
    if (ind >= size()) throw std::out_of_range("Matrix::to_coord: index is larger than size");
    return {ind / cols_, ind % cols_};
  }

  Slice slice(coord_type ul, coord_type br) { return Slice(*this, ul, br); }
  Slice slice() { return slice({0, 0}, dimensions()); }
  CSlice slice(coord_type ul, coord_type br) const { return CSlice(*this, ul, br); }
  CSlice slice() const { return slice({0, 0}, dimensions()); }
  Slice row(size_t i) { return slice({i, 0}, {i + 1, cols_}); }
  CSlice row(size_t i) const { return slice({i, 0}, {i + 1, cols_}); }
  Slice col(size_t j) { return slice({0, j}, {rows_, j + 1}); }
  CSlice col(size_t j) const { return slice({0, j}, {rows_, j + 1}); }

  // New shape; the common top-left block keeps its values, new elements are zero.
  void resize(const coord_type& dims) {
    if (dims == dimensions()) return;
    std::vector<T> nb(dims.first * dims.second, T(0));
    const size_t rr = std::min(rows_, dims.first), cc = std::min(cols_, dims.second);
    for (size_t i = 0; i < rr; ++i)
      for (size_t j = 0; j < cc; ++j) nb[i * dims.second + j] = buf_[i * cols_ + j];
    buf_.swap(nb);
    rows_ = dims.first;
    cols_ = dims.second;
  }

  void remove_row(size_t r) {
    if (r >= rows_) throw std::runtime_error("Matrix::remove_row: out of range");
    buf_.erase(buf_.begin() + r * cols_, buf_.begin() + (r + 1) * cols_);
    --rows_;
  }

  void remove_col(size_t c) {
    if (c >= cols_) throw std::runtime_error("Matrix::remove_col: out of range");
    std::vector<T> nb;
    nb.reserve(rows_ * (cols_ - 1));
    for (size_t i = 0; i < rows_; ++i)
      for (size_t j = 0; j < cols_; ++j)
        if (j != c) nb.push_back(buf_[i * cols_ + j]);
    buf_.swap(nb);
    --cols_;
  }

  void remove_row_col(size_t r, size_t c) {
    remove_col(c);
    remove_row(r);
  }

 private:
  size_t rows_ = 0, cols_ = 0;
  std::vector<T> buf_;
};

// ml = transpose(mr)
template <class ML, class MR>
void transpose_copy(ML&& ml, const MR& mr) {
  assert(ml.rows() == mr.cols() && ml.cols() == mr.rows());
  for (size_t i = 0; i < ml.rows(); ++i)
    for (size_t j = 0; j < ml.cols(); ++j) ml(i, j) = mr(j, i);
}

template <class Mat>
std::string as_string(const Mat& m, int precision = 6) {
  std::ostringstream s;
  s << std::setprecision(precision) << "[";
  for (size_t i = 0; i < m.rows(); ++i) {
    s << (i ? ",\n [" : "[");
    for (size_t j = 0; j < m.cols(); ++j) s << (j ? ", " : "") << m(i, j);
    s << "]";
  }
  s << "]";
  return s.str();
}

}  // namespace molpro::linalg::itsolv::subspace
