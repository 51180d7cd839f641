// Dense x sparse (R x P) operations.  P vectors are std::map<size_t,double> in the reference, almost
// always single unit vectors chosen by select (reference itsolv/IterativeSolverTemplate.h:340-368).
//
// Reference: ArrayHandlerIterableSparse.h:35-58, util/gemm.h:207-253, DistrArray.cpp:419-465.  The
// host keeps the entries that fall inside this rank's shard [offset, offset+n) (the reference's
// lower_bound/upper_bound), uploads (local index, value) arrays, and each output is accumulated by
// one lane in the reference's entry order, so the per-rank results are bitwise those of the
// reference loop; cross-rank sums are RCCL allreduces.
#include <algorithm>
#include <cstring>
#include <map>
#include <vector>

#include "ssp_internal.h"

// Products are rounded before the add, as in the reference's `tot += x[i] * v` (no FMA contraction),
// so each rank's sparse result is bitwise the reference loop's.
#pragma clang fp contract(off)

namespace {

using ssp::kBlock;

__global__ void k_scatter(double* __restrict__ x, const unsigned long long* __restrict__ li,
                          const double* __restrict__ v, size_t nnz, double alpha, int add) {
  for (size_t e = size_t(blockIdx.x) * blockDim.x + threadIdx.x; e < nnz; e += size_t(gridDim.x) * blockDim.x) {
    if (add)
      x[li[e]] += alpha * v[e];
    else
      x[li[e]] = v[e];
  }
}

// Few local entries (the P vectors are mostly unit vectors, IterativeSolverTemplate.h:340-368): the
// entries travel in the kernel argument block, so the op needs no staging copy and no second launch.
constexpr int kInlineEntries = 64;
struct ScatterInline {
  double* x;
  double alpha;
  int add;
  int nnz;
  unsigned long long li[kInlineEntries];
  double v[kInlineEntries];
};

__global__ void k_scatter_inline(const ScatterInline a) {
  const int e = int(threadIdx.x);
  if (e >= a.nnz) return;
  if (a.add)
    a.x[a.li[e]] += a.alpha * a.v[e];
  else
    a.x[a.li[e]] = a.v[e];
}

// The same for up to 16 destinations at once (ssp_sparse_axpy_batch): entry e goes to x[dst[e]]; up to
// 256 entries with 32-bit local indices (a P-space action's terms: 16 P vectors x 8 roots = 128).
constexpr int kBatchEntries = 256;
struct ScatterBatchInline {
  double* x[16];
  int nnz;
  unsigned char dst[kBatchEntries];
  unsigned li[kBatchEntries];
  double v[kBatchEntries];
};
static_assert(sizeof(ScatterBatchInline) <= 4000, "kernel argument block too large");

__global__ void k_scatter_batch_inline(const ScatterBatchInline a) {
  const int e = int(threadIdx.x);
  if (e >= a.nnz) return;
  a.x[a.dst[e]][a.li[e]] += a.v[e];
}

// out[i*k + j] = sum over entries e of p_j (in order) of x_i[li_e] * v_e.
struct SparseInnerArgs {
  const double* x[64];
  double xs[64];  // deferred scales (sc = 1)
  int sc;
  int m;
  int k;
  const unsigned long long* ptr;  // k+1 offsets into li/v (local entries only)
  const unsigned long long* li;
  const double* v;
  double* out;
};
// The same with k <= 32 vectors of at most kInlineEntries local entries in all carried inline.
struct SparseInnerInline {
  const double* x[64];
  double xs[64];
  int sc;
  int m;
  int k;
  unsigned short ptr[33];
  unsigned long long li[kInlineEntries];
  double v[kInlineEntries];
  double* out;
};
static_assert(sizeof(SparseInnerInline) + sizeof(ssp::FoldTail) <= 4000, "kernel argument block too large");

template <class A>
__device__ __forceinline__ double sparse_inner_value(const A& a, const unsigned long long* li, const double* v, int o) {
  const int i = o / a.k, j = o % a.k;
  double s = 0;
  const double xs = a.xs[i];
  for (unsigned long long e = a.ptr[j]; e < a.ptr[j + 1]; ++e) {
    const double xv = a.sc ? a.x[i][li[e]] * xs : a.x[i][li[e]];
    s += xv * v[e];
  }
  return s;
}

__global__ void k_sparse_inner(const SparseInnerArgs a) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o < a.m * a.k) a.out[o] = sparse_inner_value(a, a.li, a.v, o);
}

// Inline entries; with tail.host (one launch, no communicator) the last workgroup to arrive also
// publishes all m x k results to coherent host memory and sets the sequence flag -- the hand-off of
// ssp::fold_tail (write-through stores, vmcnt(0) drain, agent-scope arrival, sc1 loads; checked in
// the emitted assembly by tests/test_fold_tail_isa.py), so no publish kernel follows.
__global__ void k_sparse_inner_inline(const SparseInnerInline a, const ssp::FoldTail tail) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  const int nout = a.m * a.k;
  if (!tail.host) {
    if (o < nout) a.out[o] = sparse_inner_value(a, a.li, a.v, o);
    return;
  }
  if (o < nout) ssp::store_partial(a.out + o, sparse_inner_value(a, a.li, a.v, o));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's result has completed
  __syncthreads();
  unsigned* top = tail.counter + ssp::kFoldLine * ssp::kFoldShards;
  __shared__ unsigned s_last;
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the loads are sc1
  for (int q = int(threadIdx.x); q < nout; q += int(blockDim.x))
    __hip_atomic_store(tail.host + q, __hip_atomic_load(a.out + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's results have reached host memory
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(tail.flag, tail.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// yy[j][li_e] += alpha(i,j) * v_e for sources i in order, then entries in order; one lane per
// destination, so colliding indices accumulate in the reference's order.
struct SparseOuterArgs {
  double* y[64];
  int m;
  int k;
  const unsigned long long* ptr;
  const unsigned long long* li;
  const double* v;
  const double* alpha;  // k x m row-major (device)
};

__global__ void k_sparse_outer(const SparseOuterArgs a) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.m) return;
  for (int i = 0; i < a.k; ++i) {
    const double al = a.alpha[size_t(i) * a.m + j];
    for (unsigned long long e = a.ptr[i]; e < a.ptr[i + 1]; ++e) a.y[j][a.li[e]] += al * a.v[e];
  }
}

// construct_solution fix-up at the indices the P vectors touch: the dense pass (ssp_gemm_outer_set)
// summed Q and D from zero there, the reference sums P first.  One lane per (index, destination)
// recomputes the reference's sequence: v = 0; v += alpha(i,j) * p_i[idx] for P vectors i and their
// entries in order (no contraction); then v = fma(beta(s,j), x_s[idx], v) for the dense sources s in
// order, the arithmetic of k_gemm_outer.
// rmw (ssp_block_update): the destinations are read -- v starts from the value saved before the
// dense pass times the destination's deferred scale instead of 0.  xs: the dense sources' deferred
// scales (null: 1).
struct ConstructFixArgs {
  const double* saved;             // rmw: [u * m + j] = yy[j][uidx[u]] before the dense pass
  const double* ys;                // rmw: m destination scales
  const double* xs;                // k source scales or null
  int rmw;
  int exact;                       // the reference's arithmetic (kernels_exact.hip): no fma below
  const unsigned long long* uidx;  // distinct local indices touched by P
  size_t nu;
  int m;
  int kp;
  int k;
  const unsigned long long* ptr;   // kp+1 offsets into li/v
  const unsigned long long* li;
  const double* v;
  int entries;                     // ptr[kp]
  const double* palpha;            // kp x m
  const double* alpha;             // k x m
  const double* const* x;          // k dense sources
  double* const* y;                // m destinations
};

// The operand arrays the lanes of a fix-up read in sequence (P offsets, entries, coefficients, source
// pointers) are staged in LDS first: one round of parallel loads instead of a chain of dependent
// global loads per P entry (17.8 -> ~6 us a launch at the C4 shard).  Larger operands read global.
constexpr int kFixEntries = 512, kFixP = 64, kFixPalpha = 1024, kFixSrc = 128;
__global__ __launch_bounds__(256) void k_construct_fixup(const ConstructFixArgs a) {
  __shared__ unsigned long long s_ptr[kFixP + 1];
  __shared__ unsigned long long s_li[kFixEntries];
  __shared__ double s_v[kFixEntries];
  __shared__ double s_pal[kFixPalpha];
  __shared__ const double* s_x[kFixSrc];
  const bool staged = a.kp <= kFixP && a.entries <= kFixEntries && size_t(a.kp) * a.m <= kFixPalpha && a.k <= kFixSrc;
  if (staged) {
    for (int q = int(threadIdx.x); q <= a.kp; q += int(blockDim.x)) s_ptr[q] = a.ptr[q];
    for (int q = int(threadIdx.x); q < a.entries; q += int(blockDim.x)) {
      s_li[q] = a.li[q];
      s_v[q] = a.v[q];
    }
    for (int q = int(threadIdx.x); q < a.kp * a.m; q += int(blockDim.x)) s_pal[q] = a.palpha[q];
    for (int q = int(threadIdx.x); q < a.k; q += int(blockDim.x)) s_x[q] = a.x[q];
    __syncthreads();
  }
  const unsigned long long* ptr = staged ? s_ptr : a.ptr;
  const unsigned long long* li = staged ? s_li : a.li;
  const double* pv = staged ? s_v : a.v;
  const double* pal = staged ? s_pal : a.palpha;
  const double* const* xsrc = staged ? s_x : a.x;
  const size_t t = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= a.nu * size_t(a.m)) return;
  const size_t u = t / a.m;
  const int j = int(t % a.m);
  const unsigned long long g = a.uidx[u];
  double v = 0;
  if (a.rmw) v = a.saved[t] * a.ys[j];  // t = u * m + j
  for (int i = 0; i < a.kp; ++i) {
    const double al = pal[size_t(i) * a.m + j];
    for (unsigned long long e = ptr[i]; e < ptr[i + 1]; ++e)
      if (li[e] == g) v += al * pv[e];
  }
  // the dense sources in groups of 32: the group's loads are issued together (unconditionally: the
  // index is clamped, so no branch splits them), then the chain of adds.  x * 1 is x exactly.
  constexpr int G = 32;
  for (int s0 = 0; s0 < a.k; s0 += G) {
    double xv[G], al[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int s = min(s0 + u, a.k - 1);
      xv[u] = xsrc[s][g];
      al[u] = a.alpha[size_t(s) * a.m + j];
    }
    if (a.xs) {
#pragma unroll
      for (int u = 0; u < G; ++u) xv[u] *= a.xs[min(s0 + u, a.k - 1)];
    }
#pragma unroll
    for (int u = 0; u < G; ++u)
      if (s0 + u < a.k) v = a.exact ? v + al[u] * xv[u] : fma(al[u], xv[u], v);
  }
  a.y[j][g] = v;
}

// saved[u * m + j] = yy[j][uidx[u]] (ssp_block_update: the P-touched values before the dense pass)
__global__ void k_gather_touched(const unsigned long long* uidx, size_t nu, int m, double* const* y, double* saved) {
  const size_t t = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= nu * size_t(m)) return;
  saved[t] = y[t % m][uidx[t / m]];
}

// Local entries of one sparse vector: indices in [offset, offset+n), converted to local indices.
void filter_local(const size_t* idx, const double* val, size_t nnz, size_t n, size_t offset,
                  std::vector<unsigned long long>& li, std::vector<double>& lv) {
  for (size_t e = 0; e < nnz; ++e) {
    if (idx[e] >= offset && idx[e] < offset + n) {
      li.push_back(idx[e] - offset);
      lv.push_back(val[e]);
    }
  }
}

int upload_entries(ssp_ctx* ctx, const std::vector<unsigned long long>& ptr, const std::vector<unsigned long long>& li,
                   const std::vector<double>& lv, unsigned long long** dptr, unsigned long long** dli, double** dv) {
  void* p;
  SSP_TRY(ssp::upload_small(ctx, ptr.data(), ptr.size() * sizeof(unsigned long long), &p));
  *dptr = static_cast<unsigned long long*>(p);
  SSP_TRY(ssp::upload_small(ctx, li.data(), li.size() * sizeof(unsigned long long), &p));
  *dli = static_cast<unsigned long long*>(p);
  SSP_TRY(ssp::upload_small(ctx, lv.data(), lv.size() * sizeof(double), &p));
  *dv = static_cast<double*>(p);
  return SSP_OK;
}

int launch_scatter_inline(ssp_ctx* ctx, double* x, const std::vector<unsigned long long>& li,
                          const std::vector<double>& lv, double alpha, int add) {
  ScatterInline a{};
  a.x = x;
  a.alpha = alpha;
  a.add = add;
  a.nnz = int(li.size());
  for (size_t e = 0; e < li.size(); ++e) {
    a.li[e] = li[e];
    a.v[e] = lv[e];
  }
  SSP_LAUNCH(k_scatter_inline, dim3(1), dim3(kInlineEntries), 0, ctx->stream, a);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int check_entries(const size_t* idx, const double* val, size_t nnz, const char* what) {
  if (nnz && (!idx || !val)) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": null entries");
  return SSP_OK;
}

// Local entries of k sparse vectors (CSR ptr/idx/val) inside this rank's shard [offset, offset+n):
// lptr[j]..lptr[j+1] index li/lv for vector j.
int sparse_local_entries(const size_t* ptr, const size_t* idx, const double* val, int k, size_t n, size_t offset,
                         std::vector<unsigned long long>& lptr, std::vector<unsigned long long>& li,
                         std::vector<double>& lv) {
  lptr.assign(1, 0);
  for (int j = 0; j < k; ++j) {
    SSP_TRY(check_entries(idx + ptr[j], val + ptr[j], ptr[j + 1] - ptr[j], "ssp_gemm_inner_sparse"));
    filter_local(idx + ptr[j], val + ptr[j], ptr[j + 1] - ptr[j], n, offset, li, lv);
    lptr.push_back(li.size());
  }
  return SSP_OK;
}

// k <= 32 sparse vectors with at most kInlineEntries local entries in all: the entries travel in the
// kernel arguments, one launch per 64 dense vectors, results to out_dev (and, with tail.host, published
// by the last workgroup).
int launch_sparse_inline(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, int k,
                         const std::vector<unsigned long long>& lptr, const std::vector<unsigned long long>& li,
                         const std::vector<double>& lv, double* out_dev, const ssp::FoldTail& tail) {
  ssp::LedgerScope ls(ctx, "gemm_inner_sparse", 16.0 * li.size() * m);
  for (int i0 = 0; i0 < m; i0 += 64) {
    SparseInnerInline a{};
    a.m = std::min(64, m - i0);
    a.k = k;
    for (int i = 0; i < a.m; ++i) {
      a.x[i] = xx[i0 + i];
      a.xs[i] = xs ? xs[i0 + i] : 1.0;
      if (a.xs[i] != 1.0) a.sc = 1;
    }
    for (int j = 0; j <= k; ++j) a.ptr[j] = (unsigned short)lptr[size_t(j)];
    for (size_t e = 0; e < li.size(); ++e) {
      a.li[e] = li[e];
      a.v[e] = lv[e];
    }
    a.out = out_dev + size_t(i0) * k;
    const int outs = a.m * a.k;
    SSP_LAUNCH(k_sparse_inner_inline, dim3((outs + kBlock - 1) / kBlock), dim3(kBlock), 0, ctx->stream, a, tail);
    SSP_TRY_HIP(hipGetLastError());
  }
  return SSP_OK;
}

}  // namespace

extern "C" {

int ssp_sparse_copy(ssp_ctx* ctx, double* x, size_t n, size_t offset, const size_t* idx, const double* val,
                    size_t nnz) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(check_entries(idx, val, nnz, "ssp_sparse_copy"));
  SSP_TRY(ssp_fill(ctx, 0.0, x, n));
  std::vector<unsigned long long> li;
  std::vector<double> lv;
  filter_local(idx, val, nnz, n, offset, li, lv);
  if (li.empty()) return SSP_OK;
  if (li.size() <= size_t(kInlineEntries)) {
    ssp::LedgerScope ls(ctx, "sparse_copy", 16.0 * li.size());
    return launch_scatter_inline(ctx, x, li, lv, 1.0, 0);
  }
  std::vector<unsigned long long> ptr{0, li.size()};
  unsigned long long *dptr, *dli;
  double* dv;
  SSP_TRY(upload_entries(ctx, ptr, li, lv, &dptr, &dli, &dv));
  ssp::LedgerScope ls(ctx, "sparse_copy", 16.0 * li.size());
  const unsigned grid = unsigned(std::min<size_t>((li.size() + kBlock - 1) / kBlock, 1024));
  SSP_TRY(ssp::flush_uploads(ctx));
  SSP_LAUNCH(k_scatter, dim3(grid), dim3(kBlock), 0, ctx->stream, x, dli, dv, li.size(), 1.0, 0);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int ssp_sparse_axpy(ssp_ctx* ctx, double alpha, const size_t* idx, const double* val, size_t nnz, double* x,
                    size_t n, size_t offset) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(check_entries(idx, val, nnz, "ssp_sparse_axpy"));
  std::vector<unsigned long long> li;
  std::vector<double> lv;
  filter_local(idx, val, nnz, n, offset, li, lv);
  if (li.empty()) return SSP_OK;
  if (!x) return ssp::set_error(SSP_ERR_ARG, "ssp_sparse_axpy: null vector");
  if (li.size() <= size_t(kInlineEntries)) {
    ssp::LedgerScope ls(ctx, "sparse_axpy", 24.0 * li.size());
    return launch_scatter_inline(ctx, x, li, lv, alpha, 1);
  }
  std::vector<unsigned long long> ptr{0, li.size()};
  unsigned long long *dptr, *dli;
  double* dv;
  SSP_TRY(upload_entries(ctx, ptr, li, lv, &dptr, &dli, &dv));
  ssp::LedgerScope ls(ctx, "sparse_axpy", 24.0 * li.size());
  // Distinct map keys never collide, so entries can be applied in parallel.
  const unsigned grid = unsigned(std::min<size_t>((li.size() + kBlock - 1) / kBlock, 1024));
  SSP_TRY(ssp::flush_uploads(ctx));
  SSP_LAUNCH(k_scatter, dim3(grid), dim3(kBlock), 0, ctx->stream, x, dli, dv, li.size(), alpha, 1);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int ssp_sparse_axpy_batch(ssp_ctx* ctx, int nvec, const size_t* ptr, const size_t* idx, const double* val,
                          double* const* xx, size_t n, size_t offset) {
  SSP_CHECK_CTX(ctx);
  if (nvec < 0 || (nvec > 0 && (!ptr || !xx))) return ssp::set_error(SSP_ERR_ARG, "ssp_sparse_axpy_batch: bad arguments");
  ScatterBatchInline a{};
  bool inl = nvec <= 16;
  for (int k = 0; k < nvec && inl; ++k) {
    SSP_TRY(check_entries(idx + ptr[k], val + ptr[k], ptr[k + 1] - ptr[k], "ssp_sparse_axpy_batch"));
    std::vector<unsigned long long> li;
    std::vector<double> lv;
    filter_local(idx + ptr[k], val + ptr[k], ptr[k + 1] - ptr[k], n, offset, li, lv);
    if (li.empty()) continue;
    if (!xx[k]) return ssp::set_error(SSP_ERR_ARG, "ssp_sparse_axpy_batch: null vector");
    if (a.nnz + li.size() > size_t(kBatchEntries) || n > 0xffffffffull) {
      inl = false;
      break;
    }
    a.x[k] = xx[k];
    for (size_t e = 0; e < li.size(); ++e) {
      a.dst[a.nnz] = static_cast<unsigned char>(k);
      a.li[a.nnz] = static_cast<unsigned>(li[e]);
      a.v[a.nnz++] = lv[e];
    }
  }
  if (!inl) {  // more entries than one argument block carries: one launch per vector
    for (int k = 0; k < nvec; ++k) {
      const size_t b = ptr[k], e = ptr[k + 1];
      std::vector<size_t> sorted(idx + b, idx + e);
      std::sort(sorted.begin(), sorted.end());
      if (std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end()) {
        SSP_TRY(ssp_sparse_axpy(ctx, 1.0, idx + b, val + b, e - b, xx[k], n, offset));
      } else {  // a repeated index: the entries one at a time, in order
        for (size_t q = b; q < e; ++q) SSP_TRY(ssp_sparse_axpy(ctx, 1.0, idx + q, val + q, 1, xx[k], n, offset));
      }
    }
    return SSP_OK;
  }
  if (a.nnz == 0) return SSP_OK;
  ssp::LedgerScope ls(ctx, "sparse_axpy", 24.0 * a.nnz);
  // One vector's slice may hold an index more than once (a P-space action concatenates the entries of
  // all P vectors, which may share indices).  Entry e's generation is the number of earlier entries
  // with its (vector, index); each generation is one launch, in order, so no two lanes of a launch add
  // to one element and every element takes its adds in entry order -- ssp_sparse_axpy's per vector.
  std::vector<int> gen(size_t(a.nnz), 0);
  int ngen = 1;
  {
    std::map<std::pair<int, unsigned>, int> seen;
    for (int e = 0; e < a.nnz; ++e) {
      gen[size_t(e)] = seen[{a.dst[e], a.li[e]}]++;
      ngen = std::max(ngen, gen[size_t(e)] + 1);
    }
  }
  for (int g = 0; g < ngen; ++g) {
    ScatterBatchInline b = a;
    if (ngen > 1) {
      b.nnz = 0;
      for (int e = 0; e < a.nnz; ++e)
        if (gen[size_t(e)] == g) {
          b.dst[b.nnz] = a.dst[e];
          b.li[b.nnz] = a.li[e];
          b.v[b.nnz++] = a.v[e];
        }
    }
    SSP_LAUNCH(k_scatter_batch_inline, dim3(1), dim3(kBatchEntries), 0, ctx->stream, b);
    SSP_TRY_HIP(hipGetLastError());
  }
  return SSP_OK;
}

int ssp_gemm_inner_sparse(ssp_ctx* ctx, const double* const* xx, int m, size_t n, size_t offset, const size_t* ptr,
                          const size_t* idx, const double* val, int k, double* out) {
  return ssp_gemm_inner_sparse_scaled(ctx, xx, nullptr, m, n, offset, ptr, idx, val, k, out);
}

int ssp_gemm_inner_sparse_scaled(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, size_t n,
                                 size_t offset, const size_t* ptr, const size_t* idx, const double* val, int k,
                                 double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 0 || k < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner_sparse: negative dimension");
  if (m == 0 || k == 0) return SSP_OK;
  if (!out || !ptr || (m > 0 && !xx)) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner_sparse: null argument");
  std::vector<unsigned long long> lptr, li;
  std::vector<double> lv;
  SSP_TRY(sparse_local_entries(ptr, idx, val, k, n, offset, lptr, li, lv));
  const size_t total = size_t(m) * k;
  SSP_TRY(ssp::ensure_result(ctx, total));
  if (k <= 32 && li.size() <= size_t(kInlineEntries)) {
    // One launch (m <= 64) publishes its results itself; more launches leave them for reduce_fetch.
    const bool one = m <= 64;
    ssp::FoldTail tail{};
    if (one) SSP_TRY(ssp::fold_begin(ctx, int(total), &tail));
    SSP_TRY(launch_sparse_inline(ctx, xx, xs, m, k, lptr, li, lv, ctx->result_dev, tail));
    return one ? ssp::fold_finish(ctx, tail, out) : ssp::reduce_fetch(ctx, out, total);
  }
  unsigned long long *dptr, *dli;
  double* dv;
  SSP_TRY(upload_entries(ctx, lptr, li, lv, &dptr, &dli, &dv));
  {
    ssp::LedgerScope ls(ctx, "gemm_inner_sparse", 16.0 * li.size() * m);
    for (int i0 = 0; i0 < m; i0 += 64) {
      SparseInnerArgs a{};
      a.m = std::min(64, m - i0);
      a.k = k;
      for (int i = 0; i < a.m; ++i) {
        a.x[i] = xx[i0 + i];
        a.xs[i] = xs ? xs[i0 + i] : 1.0;
        if (a.xs[i] != 1.0) a.sc = 1;
      }
      a.ptr = dptr;
      a.li = dli;
      a.v = dv;
      a.out = ctx->result_dev + size_t(i0) * k;
      const int outs = a.m * a.k;
      SSP_TRY(ssp::flush_uploads(ctx));
      SSP_LAUNCH(k_sparse_inner, dim3((outs + kBlock - 1) / kBlock), dim3(kBlock), 0, ctx->stream, a);
      SSP_TRY_HIP(hipGetLastError());
    }
  }
  return ssp::reduce_fetch(ctx, out, total);
}

int ssp_gemm_inner_sparse_begin(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, size_t n,
                                size_t offset, const size_t* ptr, const size_t* idx, const double* val, int k) {
  SSP_CHECK_CTX(ctx);
  ctx->async_pending = false;  // an uncollected result is discarded (its launch precedes this one's)
  if (m < 0 || k < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner_sparse_begin: negative dimension");
  const size_t total = size_t(m) * size_t(k);
  if (total == 0) {
    ctx->async_n = 0;
    ctx->async_launched = false;
    ctx->async_pending = true;
    return SSP_OK;
  }
  if (!ptr || !xx) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner_sparse_begin: null argument");
  std::vector<unsigned long long> lptr, li;
  std::vector<double> lv;
  SSP_TRY(sparse_local_entries(ptr, idx, val, k, n, offset, lptr, li, lv));
  if (m <= 64 && k <= 32 && li.size() <= size_t(kInlineEntries) && !ssp::comm_attached(ctx)) {
    // One inline launch publishing to the pending buffers.  Stream order finishes it before anything
    // queued after it, so by the time a later reduction's flag is seen these results are in host
    // memory too, and _end finds its flag already set.
    SSP_TRY(ssp::ensure_async(ctx));
    ssp::FoldTail tail{};
    tail.counter = ctx->fold_counter;
    tail.nout = int(total);
    tail.flag = ctx->async_flag;
    tail.host = ctx->async_host;
    tail.seq = ++ctx->async_seq;
    SSP_TRY(launch_sparse_inline(ctx, xx, xs, m, k, lptr, li, lv, ctx->async_dev, tail));
    ctx->async_launched = true;
  } else {  // with ranks (a collective) or beyond the inline limits: computed now, delivered by _end
    ctx->async_sync.resize(total);
    SSP_TRY(ssp_gemm_inner_sparse_scaled(ctx, xx, xs, m, n, offset, ptr, idx, val, k, ctx->async_sync.data()));
    ctx->async_launched = false;
  }
  ctx->async_n = total;
  ctx->async_pending = true;
  return SSP_OK;
}

int ssp_gemm_inner_sparse_end(ssp_ctx* ctx, double* out) {
  SSP_CHECK_CTX(ctx);
  if (!ctx->async_pending) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner_sparse_end: nothing pending");
  ctx->async_pending = false;
  if (ctx->async_n == 0) return SSP_OK;
  if (!out) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner_sparse_end: null argument");
  if (!ctx->async_launched) {
    std::memcpy(out, ctx->async_sync.data(), ctx->async_n * sizeof(double));
    return SSP_OK;
  }
  bool seen = true;
  SSP_TRY(ssp::wait_flag(ctx, ctx->async_seq, &seen, "ssp_gemm_inner_sparse_end", ctx->async_flag));
  if (!seen)
    SSP_TRY_HIP(hipMemcpy(ctx->async_host, ctx->async_dev, ctx->async_n * sizeof(double), hipMemcpyDeviceToHost));
  std::memcpy(out, ctx->async_host, ctx->async_n * sizeof(double));
  return SSP_OK;
}

int ssp_sparse_dot(ssp_ctx* ctx, const double* x, size_t n, size_t offset, const size_t* idx, const double* val,
                   size_t nnz, double* out) {
  const size_t ptr[2] = {0, nnz};
  const double* xx[1] = {x};
  return ssp_gemm_inner_sparse(ctx, xx, 1, n, offset, ptr, idx, val, 1, out);
}

int ssp_gemm_outer_sparse(ssp_ctx* ctx, const double* alphas, const size_t* ptr, const size_t* idx,
                          const double* val, int k, double* const* yy, int m, size_t n, size_t offset) {
  SSP_CHECK_CTX(ctx);
  if (m < 0 || k < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer_sparse: negative dimension");
  if (m == 0 || k == 0 || n == 0) return SSP_OK;
  if (!alphas || !ptr || !yy) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer_sparse: null argument");
  std::vector<unsigned long long> lptr{0}, li;
  std::vector<double> lv;
  for (int i = 0; i < k; ++i) {
    SSP_TRY(check_entries(idx + ptr[i], val + ptr[i], ptr[i + 1] - ptr[i], "ssp_gemm_outer_sparse"));
    filter_local(idx + ptr[i], val + ptr[i], ptr[i + 1] - ptr[i], n, offset, li, lv);
    lptr.push_back(li.size());
  }
  if (li.empty()) return SSP_OK;
  unsigned long long *dptr, *dli;
  double* dv;
  SSP_TRY(upload_entries(ctx, lptr, li, lv, &dptr, &dli, &dv));
  ssp::LedgerScope ls(ctx, "gemm_outer_sparse", 24.0 * li.size() * m);
  for (int j0 = 0; j0 < m; j0 += 64) {
    SparseOuterArgs a{};
    a.m = std::min(64, m - j0);
    a.k = k;
    for (int j = 0; j < a.m; ++j) a.y[j] = yy[j0 + j];
    std::vector<double> al(size_t(k) * a.m);
    for (int i = 0; i < k; ++i)
      for (int j = 0; j < a.m; ++j) al[size_t(i) * a.m + j] = alphas[size_t(i) * m + j0 + j];
    void* dal;
    SSP_TRY(ssp::upload_small(ctx, al.data(), al.size() * sizeof(double), &dal));
    a.alpha = static_cast<const double*>(dal);
    a.ptr = dptr;
    a.li = dli;
    a.v = dv;
    SSP_TRY(ssp::flush_uploads(ctx));
    SSP_LAUNCH(k_sparse_outer, dim3(1), dim3(64), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
  }
  return SSP_OK;
}

}  // extern "C"

namespace {
// construct_solution (rmw = false: destinations written without being read) and the block update
// (rmw = true: yy[j] = ys[j] yy[j] + P + dense): the dense pass over every element, then the fix-up
// that recomputes the indices the P vectors touch in the reference's order (P first).
int solution_impl(ssp_ctx* ctx, const double* palphas, const size_t* ptr, const size_t* idx, const double* val,
                  int kp, const double* alphas, const double* const* xx, const double* xs, int k, double* const* yy,
                  const double* ys, int m, size_t n, size_t offset, bool rmw, const char* what) {
  SSP_CHECK_CTX(ctx);
  if (m < 0 || k < 0 || kp < 0) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": negative dimension");
  if (m == 0) return SSP_OK;
  if (kp > 0 && (!palphas || !ptr)) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": null P argument");
  std::vector<unsigned long long> lptr{0}, li;
  std::vector<double> lv;
  for (int i = 0; i < kp && n > 0; ++i) {
    SSP_TRY(check_entries(idx + ptr[i], val + ptr[i], ptr[i + 1] - ptr[i], what));
    filter_local(idx + ptr[i], val + ptr[i], ptr[i + 1] - ptr[i], n, offset, li, lv);
    lptr.push_back(li.size());
  }
  std::vector<unsigned long long> uidx(li);
  std::sort(uidx.begin(), uidx.end());
  uidx.erase(std::unique(uidx.begin(), uidx.end()), uidx.end());
  void* p;
  double* const* ydev = nullptr;
  const double* saved = nullptr;
  if (rmw && !uidx.empty()) {  // the values the dense pass is about to overwrite at the P indices
    SSP_TRY(ssp::upload_small(ctx, yy, size_t(m) * sizeof(double*), &p));
    ydev = static_cast<double* const*>(p);
    SSP_TRY(ssp::upload_small(ctx, uidx.data(), uidx.size() * sizeof(unsigned long long), &p));
    const size_t cnt = uidx.size() * size_t(m);
    SSP_TRY(ssp::ensure_partial(ctx, cnt));
    SSP_TRY(ssp::flush_uploads(ctx));
    SSP_LAUNCH(k_gather_touched, dim3(unsigned((cnt + 255) / 256)), dim3(256), 0, ctx->stream,
                       static_cast<const unsigned long long*>(p), uidx.size(), m, ydev, ctx->partial);
    SSP_TRY_HIP(hipGetLastError());
    saved = ctx->partial;  // nothing below resizes the partials workspace before the fix-up reads it
  }
  if (rmw)
    SSP_TRY(ssp_gemm_outer_scaled(ctx, alphas, xx, xs, k, yy, ys, m, n));
  else
    SSP_TRY(ssp_gemm_outer_set_scaled(ctx, alphas, xx, xs, k, yy, m, n));
  if (uidx.empty()) return SSP_OK;
  ConstructFixArgs a{};
  unsigned long long *dptr, *dli;
  double* dv;
  SSP_TRY(upload_entries(ctx, lptr, li, lv, &dptr, &dli, &dv));
  a.ptr = dptr;
  a.li = dli;
  a.v = dv;
  a.entries = int(li.size());
  SSP_TRY(ssp::upload_small(ctx, uidx.data(), uidx.size() * sizeof(unsigned long long), &p));
  a.uidx = static_cast<const unsigned long long*>(p);
  SSP_TRY(ssp::upload_small(ctx, palphas, size_t(kp) * m * sizeof(double), &p));
  a.palpha = static_cast<const double*>(p);
  if (k > 0) {
    SSP_TRY(ssp::upload_small(ctx, alphas, size_t(k) * m * sizeof(double), &p));
    a.alpha = static_cast<const double*>(p);
    SSP_TRY(ssp::upload_small(ctx, xx, size_t(k) * sizeof(double*), &p));
    a.x = static_cast<const double* const*>(p);
    if (xs) {
      SSP_TRY(ssp::upload_small(ctx, xs, size_t(k) * sizeof(double), &p));
      a.xs = static_cast<const double*>(p);
    }
  }
  if (!ydev) {
    SSP_TRY(ssp::upload_small(ctx, yy, size_t(m) * sizeof(double*), &p));
    ydev = static_cast<double* const*>(p);
  }
  a.y = ydev;
  if (rmw) {
    std::vector<double> one(size_t(m), 1.0);
    SSP_TRY(ssp::upload_small(ctx, ys ? ys : one.data(), size_t(m) * sizeof(double), &p));
    a.ys = static_cast<const double*>(p);
    a.saved = saved;
    a.rmw = 1;
  }
  a.nu = uidx.size();
  a.exact = ssp::exact_mode(ctx, n) ? 1 : 0;
  a.m = m;
  a.kp = kp;
  a.k = k;
  ssp::LedgerScope ls(ctx, rmw ? "block_update_sparse" : "construct_solution_sparse",
                      8.0 * a.nu * m * (2.0 + k + (rmw ? 1.0 : 0.0)));
  const size_t threads = a.nu * size_t(m);
  SSP_TRY(ssp::flush_uploads(ctx));
  SSP_LAUNCH(k_construct_fixup, dim3(unsigned((threads + 255) / 256)), dim3(256), 0, ctx->stream, a);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}
}  // namespace

extern "C" {

int ssp_construct_solution(ssp_ctx* ctx, const double* palphas, const size_t* ptr, const size_t* idx,
                           const double* val, int kp, const double* alphas, const double* const* xx, int k,
                           double* const* yy, int m, size_t n, size_t offset) {
  return solution_impl(ctx, palphas, ptr, idx, val, kp, alphas, xx, nullptr, k, yy, nullptr, m, n, offset, false,
                       "ssp_construct_solution");
}

int ssp_construct_solution_scaled(ssp_ctx* ctx, const double* palphas, const size_t* ptr, const size_t* idx,
                                  const double* val, int kp, const double* alphas, const double* const* xx,
                                  const double* xs, int k, double* const* yy, int m, size_t n, size_t offset) {
  return solution_impl(ctx, palphas, ptr, idx, val, kp, alphas, xx, xs, k, yy, nullptr, m, n, offset, false,
                       "ssp_construct_solution_scaled");
}

int ssp_block_update(ssp_ctx* ctx, const double* palphas, const size_t* ptr, const size_t* idx, const double* val,
                     int kp, const double* alphas, const double* const* xx, const double* xs, int k, double* const* yy,
                     const double* ys, int m, size_t n, size_t offset) {
  return solution_impl(ctx, palphas, ptr, idx, val, kp, alphas, xx, xs, k, yy, ys, m, n, offset, true,
                       "ssp_block_update");
}

}  // extern "C"
