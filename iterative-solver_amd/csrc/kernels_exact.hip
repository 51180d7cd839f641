// The reference's own arithmetic for short vectors (ssp_ctx_set_exact_max / SSP_EXACT_MAX, default
// 2048 local elements): every reduction a sequential sum in index order and every multiply-add
// rounded twice, exactly the reference's ArrayHandlerIterable loops (std::inner_product,
// ArrayHandlerIterable.h:76-82; y = alpha * x + y, :65-74) and its pairwise gemm_inner_default /
// gemm_outer_default (util/gemm.h:257-279).  A solve on such vectors is then the reference CPU path bit
// for bit (on one rank; on several, the reference's distributed build: rank-local sums added in rank
// order by the peer-memory and host transports).  The short vectors are the reference's own test
// problems (its matrices have 4 to 1000 rows): there every kernel is latency-bound, while the parallel
// kernels' other -- equally valid -- summation order and fused multiply-adds let last-bit differences
// decide knife-edge steps of those tests.  The cost is the chain of dependent adds, ≈ 7 ns per element
// on gfx950 (tools/exact_cost.py): 2048 elements add ≈ 14 µs to a reduction, about a bandwidth
// kernel's whole launch-and-fetch time; at 16384 a dot takes 131 µs against 14 µs, so longer vectors
// default to the bandwidth kernels (the knob raises the limit; tests/test_exact_gpu.py runs to 16384).
#include <algorithm>
#include <vector>

#include "ssp_internal.h"

// Products rounded before they are added, as in the reference's x86-64 build.
#pragma clang fp contract(off)

namespace {

using ssp::kBlock;

// Operands ride in the argument block when there are at most kInl of each (no staging copy).
constexpr int kInl = 64;
struct ExactInnerArgs {
  const double* const* x;  // m vectors (device array of pointers; null: inline below)
  const double* const* y;  // k vectors
  const double* xs;        // m deferred scales
  const double* ys;        // k deferred scales
  const double* xi[kInl];
  const double* yi[kInl];
  double xsi[kInl], ysi[kInl];
  int m, k;
  int pairs;               // 1: out[j] = <x_j, y_j> (m == k); 0: out[i * k + j] = <x_i, y_j>
  size_t n;
  double* out;             // device
  ssp::FoldTail tail;      // tail.host: the last workgroup publishes every output to the host
};

// s + buf[0] + buf[1] + ... + buf[len-1], added in that order.  The chain of dependent adds is the
// cost; the LDS reads are issued 16 values ahead of the adds that consume them, so their latency
// (≈ 50 cycles) hides behind the previous 16 adds.
__device__ __forceinline__ double add_in_order(const double* buf, int len, double s) {
  const double2* b2 = reinterpret_cast<const double2*>(buf);
  int t = 0;
  if (len >= 16) {
    double2 cur[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) cur[u] = b2[u];
    for (t = 16; t + 16 <= len; t += 16) {
      double2 nxt[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) nxt[u] = b2[t / 2 + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s = s + cur[u].x;
        s = s + cur[u].y;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) cur[u] = nxt[u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s = s + cur[u].x;
      s = s + cur[u].y;
    }
  }
  for (; t < len; ++t) s = s + buf[t];
  return s;
}

// One workgroup per output: the sequential std::inner_product of the (stored-equivalent) operands.
// Waves 1..3 form the products of the next chunk in LDS (each product rounded alone, whichever lane
// forms it) while lane 0 of wave 0 adds the current chunk in index order (double-buffered chunks).
constexpr int kExactChunk = 2048;
__global__ __launch_bounds__(kBlock) void k_exact_inner(const ExactInnerArgs a) {
  __shared__ __attribute__((aligned(16))) double prod[2][kExactChunk];
  const int o = int(blockIdx.x);
  const int i = a.pairs ? o : o / a.k, j = a.pairs ? o : o % a.k;
  const double* x = a.x ? a.x[i] : a.xi[i];
  const double* y = a.x ? a.y[j] : a.yi[j];
  const double xs = a.x ? a.xs[i] : a.xsi[i], ys = a.x ? a.ys[j] : a.ysi[j];
  const int fill_lane = int(threadIdx.x) - 64, fill_lanes = kBlock - 64;
  const int nchunk = int((a.n + kExactChunk - 1) / kExactChunk);
  auto fill = [&](int c) {
    const size_t c0 = size_t(c) * kExactChunk;
    const int len = int(a.n - c0 < size_t(kExactChunk) ? a.n - c0 : size_t(kExactChunk));
    // 4 elements' loads in flight per lane before the products are formed
    for (int t0 = fill_lane; t0 < len; t0 += 4 * fill_lanes) {
      double xv[4], yv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * fill_lanes;
        if (t < len) {
          xv[u] = x[c0 + t];
          yv[u] = y[c0 + t];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * fill_lanes;
        if (t < len) prod[c & 1][t] = (xv[u] * xs) * (yv[u] * ys);
      }
    }
  };
  if (fill_lane >= 0) fill(0);
  __syncthreads();
  double s = 0;
  for (int c = 0; c < nchunk; ++c) {
    if (fill_lane >= 0) {
      if (c + 1 < nchunk) fill(c + 1);
    } else if (threadIdx.x == 0) {
      const size_t c0 = size_t(c) * kExactChunk;
      const int len = int(a.n - c0 < size_t(kExactChunk) ? a.n - c0 : size_t(kExactChunk));
      s = add_in_order(prod[c & 1], len, s);
    }
    __syncthreads();
  }
  if (!a.tail.host) {  // a communicator is attached: the results stay on the device for the exchange
    if (threadIdx.x == 0) a.out[o] = s;
    return;
  }
  // One rank: each workgroup hands its output over write-through (the hand-off of ssp::fold_tail,
  // checked in the emitted assembly by tests/test_fold_tail_isa.py), and the last to arrive publishes
  // all of them into coherent host memory, then the sequence flag -- no second kernel, no copy.
  const int nout = a.pairs ? a.m : a.m * a.k;
  unsigned* top = a.tail.counter + ssp::kFoldLine * ssp::kFoldShards;
  __shared__ unsigned s_last;
  if (threadIdx.x == 0) {
    ssp::store_partial(a.out + o, s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == unsigned(nout) - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the loads are sc1
  for (int q = int(threadIdx.x); q < nout; q += kBlock)
    __hip_atomic_store(a.tail.host + q, __hip_atomic_load(a.out + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's results have reached host memory
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.tail.flag, a.tail.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static_assert(sizeof(ExactInnerArgs) <= 4000, "kernel argument block too large");

// Inline operands: at most kOutSrc sources, kOutDst destinations and kOutAl coefficients.
constexpr int kOutSrc = 32, kOutDst = 16, kOutAl = 128;
struct ExactOuterArgs {
  const double* const* x;  // k sources (device array; null: inline below)
  double* const* y;        // m destinations
  const double* xs;        // k source scales
  const double* ys;        // m destination scales (applied to the values read)
  const double* alpha;     // alpha[i * m + j]
  const double* xi[kOutSrc];
  double* yi[kOutDst];
  double xsi[kOutSrc], ysi[kOutDst], ali[kOutAl];
  int m, k, set;
  size_t n;
};
static_assert(sizeof(ExactOuterArgs) <= 4000, "kernel argument block too large");

// One thread per (element, destination): y_j[e] = y_j[e] + alpha(i, j) x_i[e] for i = 0..k-1 in order,
// each product rounded -- the pairwise axpy loop of gemm_outer_default, element by element.
__global__ __launch_bounds__(kBlock) void k_exact_outer(const ExactOuterArgs a) {
  const size_t total = a.n * size_t(a.m);
  for (size_t t = size_t(blockIdx.x) * kBlock + threadIdx.x; t < total; t += size_t(gridDim.x) * kBlock) {
    const int j = int(t / a.n);
    const size_t e = t % a.n;
    if (a.x) {
      double v = a.set ? 0.0 : a.y[j][e] * a.ys[j];
      for (int i = 0; i < a.k; ++i) v = v + a.alpha[size_t(i) * a.m + j] * (a.x[i][e] * a.xs[i]);
      a.y[j][e] = v;
    } else {
      double v = a.set ? 0.0 : a.yi[j][e] * a.ysi[j];
      for (int i = 0; i < a.k; ++i) v = v + a.ali[i * a.m + j] * (a.xi[i][e] * a.xsi[i]);
      a.yi[j][e] = v;
    }
  }
}

template <class T>
int stage(ssp_ctx* ctx, const T* host, size_t count, const T** dev) {
  void* p;
  SSP_TRY(ssp::upload_small(ctx, host, count * sizeof(T), &p));
  *dev = static_cast<const T*>(p);
  return SSP_OK;
}

}  // namespace

namespace ssp {

bool exact_mode(const ssp_ctx* ctx, size_t n) { return n > 0 && n <= ctx->exact_max; }

int exact_inner(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, const double* const* yy,
                const double* ys, int k, size_t n, bool pairs, const FoldTail& tail) {
  const int nout = pairs ? m : m * k;
  SSP_TRY(ensure_result(ctx, size_t(nout)));
  if (nout == 0) return SSP_OK;
  std::vector<double> one(size_t(std::max(m, k)), 1.0);
  ExactInnerArgs a{};
  if (m <= kInl && k <= kInl) {
    for (int i = 0; i < m; ++i) {
      a.xi[i] = xx[i];
      a.xsi[i] = xs ? xs[i] : 1.0;
    }
    for (int j = 0; j < k; ++j) {
      a.yi[j] = yy[j];
      a.ysi[j] = ys ? ys[j] : 1.0;
    }
  } else {
    SSP_TRY(stage(ctx, xx, size_t(m), &a.x));
    SSP_TRY(stage(ctx, yy, size_t(k), &a.y));
    SSP_TRY(stage(ctx, xs ? xs : one.data(), size_t(m), &a.xs));
    SSP_TRY(stage(ctx, ys ? ys : one.data(), size_t(k), &a.ys));
  }
  a.m = m;
  a.k = k;
  a.pairs = pairs ? 1 : 0;
  a.n = n;
  a.out = ctx->result_dev;
  a.tail = tail;
  SSP_TRY(flush_uploads(ctx));
  SSP_LAUNCH(k_exact_inner, dim3(unsigned(nout)), dim3(kBlock), 0, ctx->stream, a);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int exact_outer(ssp_ctx* ctx, const double* alphas, const double* const* xx, const double* xs, int k,
                double* const* yy, const double* ys, int m, size_t n, bool set) {
  if (m == 0 || n == 0) return SSP_OK;
  ExactOuterArgs a{};
  if (k <= kOutSrc && m <= kOutDst && k * m <= kOutAl) {
    for (int i = 0; i < k; ++i) {
      a.xi[i] = xx[i];
      a.xsi[i] = xs ? xs[i] : 1.0;
    }
    for (int j = 0; j < m; ++j) {
      a.yi[j] = yy[j];
      a.ysi[j] = ys && !set ? ys[j] : 1.0;
    }
    for (int q = 0; q < k * m; ++q) a.ali[q] = alphas[q];
    a.m = m;
    a.k = k;
    a.set = set ? 1 : 0;
    a.n = n;
    const size_t total = n * size_t(m);
    const unsigned grid = unsigned(std::min<size_t>((total + kBlock - 1) / kBlock, size_t(ctx->num_cus) * 4));
    SSP_LAUNCH(k_exact_outer, dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
    return SSP_OK;
  }
  std::vector<double> one(size_t(std::max(m, k)), 1.0);
  std::vector<double> al(size_t(std::max(1, k * m)), 0.0);
  if (k > 0) std::copy(alphas, alphas + size_t(k) * m, al.begin());
  std::vector<const double*> xp(size_t(std::max(k, 1)), nullptr);
  for (int i = 0; i < k; ++i) xp[size_t(i)] = xx[i];
  SSP_TRY(stage(ctx, xp.data(), xp.size(), &a.x));
  void* py;
  SSP_TRY(upload_small(ctx, yy, size_t(m) * sizeof(double*), &py));
  a.y = static_cast<double* const*>(py);
  SSP_TRY(stage(ctx, xs && k > 0 ? xs : one.data(), size_t(std::max(k, 1)), &a.xs));
  SSP_TRY(stage(ctx, ys && !set ? ys : one.data(), size_t(m), &a.ys));
  SSP_TRY(stage(ctx, al.data(), al.size(), &a.alpha));
  a.m = m;
  a.k = k;
  a.set = set ? 1 : 0;
  a.n = n;
  SSP_TRY(flush_uploads(ctx));
  const size_t total = n * size_t(m);
  const unsigned grid = unsigned(std::min<size_t>((total + kBlock - 1) / kBlock, size_t(ctx->num_cus) * 4));
  SSP_LAUNCH(k_exact_outer, dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

}  // namespace ssp

extern "C" {

int ssp_ctx_set_exact_max(ssp_ctx* ctx, size_t n) {
  SSP_CHECK_CTX(ctx);
  ctx->exact_max = n;
  return SSP_OK;
}

}  // extern "C"
