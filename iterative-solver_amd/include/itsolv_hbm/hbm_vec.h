// HBM-resident vectors: the R / Q container type of the MI355X handlers, on libsubspace_hip.so alone.
//
// This header depends on nothing but the C ABI (include/subspace_hip.h) and the standard library,
// so it can be included beside either ArrayHandler base: the restated one
// (itsolv_hbm/array_handler.h, used by this package's solvers) or the reference's own
// molpro/linalg/array/ArrayHandler.h (itsolv_hbm/reference_handler.h, the drop-in).
//
// hbm::Vec is one rank's contiguous shard [offset, offset + local_size) of a global vector of length
// size(), distributed as the reference's make_distribution_spread_remainder (reference
// array/util/Distribution.h:99-109; DistrArraySpan.cpp:35-37).  It owns its HBM block (unlike
// DistrArraySpan, whose copies alias, reference DistrArraySpan.cpp:47-51), is movable and
// deep-copyable, and value_type is double (the reference's README.md:103 requirements on R and Q).
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "subspace_hip.h"

namespace molpro::linalg::hbm {

//! The P-space vector type: the reference's sparse map of index -> coefficient.
using SparseP = std::map<size_t, double>;

// C-ABI status -> the reference's exception types: size mismatch -> SizeError (the handler's
// util::ArrayHandlerError, reference ArrayHandler.h:25-27), alphas dimension mismatch ->
// std::out_of_range (reference util/gemm.h:66-71), unsupported operation -> std::logic_error
// (reference ArrayHandlerDistrSparse.h:26-28), anything else -> std::runtime_error.
template <class SizeError = std::length_error>
void check_status(int status, const char* what) {
  if (status == SSP_OK) return;
  std::string msg = std::string(what) + ": " + ssp_last_error();
  switch (status) {
    case SSP_ERR_SIZE: throw SizeError(msg);
    case SSP_ERR_RANGE: throw std::out_of_range(msg);
    case SSP_ERR_UNSUPPORTED: throw std::logic_error(msg);
    default: throw std::runtime_error(msg);
  }
}

// One process's device: the ssp context (HIP stream, HBM arena, optional RCCL communicator).
class Device {
 public:
  explicit Device(int device) { check_status(ssp_ctx_create(device, &m_ctx), "ssp_ctx_create"); }
  // Wraps a context owned by the caller (borrowed = true: not destroyed here).
  Device(ssp_ctx* ctx, bool borrowed) : m_ctx(ctx), m_owned(!borrowed) {
    if (!ctx) throw std::invalid_argument("hbm::Device: null ssp_ctx");
  }
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;
  virtual ~Device() {
    if (m_owned) ssp_ctx_destroy(m_ctx);
  }
  void attach_comm(int nranks, int rank, const char* unique_id) {
    check_status(ssp_ctx_attach_comm(m_ctx, nranks, rank, unique_id), "ssp_ctx_attach_comm");
  }
  ssp_ctx* ctx() const { return m_ctx; }
  int rank() const { return ssp_ctx_rank(m_ctx); }
  int nranks() const { return ssp_ctx_nranks(m_ctx); }
  // Shard of a global length n owned by this rank.
  std::pair<size_t, size_t> shard(size_t n) const {
    size_t offset = 0, length = 0;
    check_status(ssp_shard_range(n, nranks(), rank(), &offset, &length), "ssp_shard_range");
    return {offset, length};
  }

 private:
  ssp_ctx* m_ctx = nullptr;
  bool m_owned = true;
};

// Storage is shared copy-on-write.  The reference's solvers copy R vectors into new Q vectors
// (QSpace.h:80-84), the preconditioner's diagonals into params[0] (IterativeSolverTemplate.h:391)
// and the new working set into params (propose_rspace.h:617-619), and then overwrite the source or
// the copy with a write-only kernel (construct_solution, the action) -- so a copy shares the
// source's HBM block and costs no bytes.  Access is explicit about what a kernel does with the
// storage:
//   data()     const, for operands that are only read;
//   data_rw()  for read-modify-write destinations: a block still shared is first copied (exactly
//              the bytes the eager copy would have moved);
//   data_wo()  for destinations a kernel writes in full without reading: a shared block is
//              replaced by a fresh one, nothing is copied.
// The shared block outlives every holder's kernels: blocks return to the context's arena, whose
// reuse is ordered on the context's one stream.
//
// A scal is deferred: the vector's value is its block times a pending scale s (scale_by, the
// handlers' scal), which the next kernel that reads the vector applies as it loads each element --
// x_i * s is the one rounding the reference's scal loop stores (ArrayHandlerIterable.h:46-50), so the
// kernel sees bit for bit the values an eager scal would have left -- instead of a separate pass
// that reads and writes the vector (16 bytes per element).  Kernels that take scales read through
// data_deferred() / data_rw_deferred() (the *_scaled entry points of include/subspace_hip.h); every
// other access (data(), data_rw()) first stores the scaled values (materialize()), so a caller that
// knows nothing of the scale sees the eager result.  data_wo() drops the scale with the contents.
//
// A fill is deferred the same way (fill_deferred, the handlers' fill): the vector's value is the fill
// value everywhere, whatever its block holds, until an access needs the block -- data(), data_rw(),
// data_deferred() and data_rw_deferred() first store it (one fill pass, into a fresh block when the
// block is shared), while data_wo() drops it with the contents.  The runners' zero-initialised
// vectors (the reference's test drivers' std::vector<double>(n)) that the action or the initial guess
// then overwrites in full therefore cost no pass.
//
// A kernel that has just formed a vector's self-dot as a by-product (the last pass of the block
// self-orthonormalisation forms the Gram matrix of the vectors it stores) records it
// (set_known_norm2); the handlers' batched dots return it instead of reading the vector again, until
// any access that may change the value (data_rw, data_wo, the deferred forms, a scal or a fill).
class Vec {
  struct Block {
    std::shared_ptr<Device> dev;
    double* p = nullptr;
    Block(std::shared_ptr<Device> d, size_t n) : dev(std::move(d)) { check_status(ssp_alloc(dev->ctx(), n, &p), "ssp_alloc"); }
    Block(const Block&) = delete;
    Block& operator=(const Block&) = delete;
    ~Block() {
      if (p) ssp_free(dev->ctx(), p);
    }
  };

 public:
  using value_type = double;

  Vec() = default;
  Vec(std::shared_ptr<Device> dev, size_t n_global) : m_dev(std::move(dev)), m_size(n_global) {
    auto [off, n] = m_dev->shard(n_global);
    m_offset = off;
    m_local = n;
    m_block = std::make_shared<Block>(m_dev, m_local);
  }
  //! A copy: shares the storage until either side writes (see above).
  Vec(const Vec& o) = default;
  Vec(Vec&& o) noexcept { swap(o); }
  // A vector of the same length and distribution whose contents are not initialised (for
  // destinations that a kernel writes without reading).
  Vec alloc_like() const { return Vec(m_dev, m_size); }
  Vec& operator=(const Vec& o) = default;
  Vec& operator=(Vec&& o) noexcept {
    Vec t(std::move(o));
    swap(t);
    return *this;
  }
  ~Vec() = default;
  void swap(Vec& o) noexcept {
    std::swap(m_dev, o.m_dev);
    std::swap(m_block, o.m_block);
    std::swap(m_scale, o.m_scale);
    std::swap(m_fill_pending, o.m_fill_pending);
    std::swap(m_fill_value, o.m_fill_value);
    std::swap(m_norm2_known, o.m_norm2_known);
    std::swap(m_norm2, o.m_norm2);
    std::swap(m_size, o.m_size);
    std::swap(m_local, o.m_local);
    std::swap(m_offset, o.m_offset);
  }
  //! Becomes a copy of o (o's distribution): shares o's storage.
  void assign_shared(const Vec& o) {
    if (this != &o) *this = o;
  }

  size_t size() const { return m_size; }
  size_t local_size() const { return m_local; }
  size_t offset() const { return m_offset; }
  //! Read-only operand, scale applied (stored) first.
  const double* data() const {
    materialize();
    return m_block ? m_block->p : nullptr;
  }
  //! Read-modify-write destination, scale applied first; the block is this vector's alone.
  double* data_rw() {
    m_norm2_known = false;
    materialize();
    detach(true);
    return m_block ? m_block->p : nullptr;
  }
  //! Destination written in full without being read: contents, scale and pending fill are dropped.
  double* data_wo() {
    m_norm2_known = false;
    m_scale = 1.0;
    m_fill_pending = false;
    detach(false);
    return m_block ? m_block->p : nullptr;
  }
  //! The handlers' fill: x = alpha everywhere, deferred until an access needs the block (see above).
  void fill_deferred(double alpha) {
    m_norm2_known = false;
    m_scale = 1.0;
    m_fill_pending = true;
    m_fill_value = alpha;
  }
  //! The pending scale: the vector's value is scale() * (the block's contents).
  double scale() const { return m_scale; }
  //! Read-only operand of a kernel that multiplies each element by scale() as it loads it.
  const double* data_deferred() const {
    materialize_fill();
    return m_block ? m_block->p : nullptr;
  }
  //! Read-modify-write destination of a kernel that multiplies each element it reads by *s (set to
  //! the pending scale here) and stores the result in full; call scale_applied() once that kernel
  //! has been issued successfully (on an error the vector keeps its value: block and scale).
  double* data_rw_deferred(double* s) {
    m_norm2_known = false;
    materialize_fill();
    detach(true);
    *s = m_scale;
    return m_block ? m_block->p : nullptr;
  }
  //! The pending scale has been written into the block by a *_scaled kernel (data_rw_deferred).
  void scale_applied() { m_scale = 1.0; }
  //! The handlers' scal: x *= a, deferred to the next kernel that reads x (see above).  A second
  //! scal before any kernel has applied the first stores the first (two roundings, as the reference).
  void scale_by(double a) {
    m_norm2_known = false;
    materialize();
    m_scale = a;
  }
  //! Stores the pending scale into the block (one scal pass, or a scaled copy into a fresh block
  //! when the block is shared); a no-op when the scale is 1.
  void materialize() const {
    materialize_fill();
    if (m_scale == 1.0 || !m_block) return;
    if (m_block.use_count() > 1) {
      auto fresh = std::make_shared<Block>(m_dev, m_local);
      check_status(ssp_scal_copy(ctx(), m_scale, fresh->p, m_block->p, m_local), "ssp_scal_copy");
      m_block = std::move(fresh);
    } else {
      check_status(ssp_scal(ctx(), m_scale, m_block->p, m_local), "ssp_scal");
    }
    m_scale = 1.0;
  }
  //! Stores a pending fill into the block (into a fresh block when the block is shared: the other
  //! holders keep their values).  The scale is 1 while a fill is pending.
  void materialize_fill() const {
    if (!m_fill_pending || !m_block) return;
    if (m_block.use_count() > 1) m_block = std::make_shared<Block>(m_dev, m_local);
    check_status(ssp_fill(ctx(), m_fill_value, m_block->p, m_local), "ssp_fill");
    m_fill_pending = false;
  }
  bool fill_pending() const { return m_fill_pending; }
  //! The vector's self-dot as formed by the kernel that just wrote it (see above).
  void set_known_norm2(double v) {
    m_norm2 = v;
    m_norm2_known = true;
  }
  bool known_norm2(double* v) const {
    if (m_norm2_known) *v = m_norm2;
    return m_norm2_known;
  }
  //! Whether another Vec holds the same storage.
  bool shares_storage() const { return m_block && m_block.use_count() > 1; }
  ssp_ctx* ctx() const { return m_dev->ctx(); }
  const std::shared_ptr<Device>& device() const { return m_dev; }
  bool compatible(const Vec& o) const { return m_size == o.m_size && m_offset == o.m_offset && m_local == o.m_local; }

  std::vector<double> local_values() const {
    std::vector<double> v(m_local);
    check_status(ssp_download(ctx(), v.data(), data(), m_local), "ssp_download");
    return v;
  }
  void set_local_values(const std::vector<double>& v) {
    if (v.size() != m_local) throw std::invalid_argument("Vec::set_local_values: wrong length");
    check_status(ssp_upload(ctx(), data_wo(), v.data(), m_local), "ssp_upload");
  }

 private:
  void detach(bool keep_values) {
    if (!m_block || m_block.use_count() <= 1) return;
    auto fresh = std::make_shared<Block>(m_dev, m_local);
    if (keep_values) check_status(ssp_copy(ctx(), fresh->p, m_block->p, m_local), "ssp_copy");
    m_block = std::move(fresh);
  }

  std::shared_ptr<Device> m_dev;
  mutable std::shared_ptr<Block> m_block;  // mutable: materialize() on a const operand
  size_t m_size = 0, m_local = 0, m_offset = 0;
  mutable double m_scale = 1.0;
  mutable bool m_fill_pending = false;
  double m_fill_value = 0.0;
  bool m_norm2_known = false;
  double m_norm2 = 0.0;
};

}  // namespace molpro::linalg::hbm
