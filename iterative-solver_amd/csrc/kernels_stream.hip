// Streaming kernels: fill / scal / copy / axpy / dot / precondition.
//
// Reference loops (single-threaded std::fill / transform / inner_product):
//   ArrayHandlerIterable.h:46-82, DistrArray.cpp:43-138, itsolv/IterativeSolver.h:34-55.
// Each is HBM-bound (<= 0.25 flop/B).  Layout: 16-byte (double2) accesses per lane, nontemporal.
// Two access shapes (tools/mb_glds.hip mode a, profiles/r1/mb_stream_shapes.txt):
//   stride  4 double2 per lane spaced a whole grid apart, 64 workgroups per CU (fill; and
//           axpy/scal/copy below kWinMin elements, where the vectors are largely cache-resident);
//   window  each wave owns kWinU consecutive KiB of every vector per visit: dot always (5.6-6.0 ->
//           6.7-6.9 TB/s at N = 1e8, 5.6 -> 5.8 at the C4 shard), axpy/scal/copy from kWinMin
//           elements (axpy 5.1-5.3 -> 5.8 TB/s at N = 1e8).
// Reductions are deterministic: one partial per workgroup in a fixed grid (a function of N and the
// CU count), then a fixed-order fold (by the last workgroup to finish for small results,
// ssp::fold_tail; else the k_reduce_partials pass).
#include <algorithm>

#include "ssp_internal.h"

namespace {

using ssp::kBlock;

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
__device__ __forceinline__ void st2(double* p, double2 v) { *reinterpret_cast<double2*>(p) = v; }
// Deferred scal (include/subspace_hip.h): v * s is the one rounding an eager scal would have stored.
template <bool SC>
__device__ __forceinline__ double2 sc2(double2 v, double s) {
  return SC ? make_double2(v.x * s, v.y * s) : v;
}
template <bool SC>
__device__ __forceinline__ double sc1(double v, double s) {
  return SC ? v * s : v;
}

// Window shape: a wave covers kWinU x 64 consecutive double2 (kWinU KiB) of each vector per visit.
constexpr int kWinU = 8;
constexpr size_t kWinMin = size_t(1) << 24;  // elementwise ops switch to windows from 128 MiB vectors
constexpr int kDotU = 4;


// Sum over the 256 threads of a workgroup; result valid in thread 0.  Fixed order.
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double wsum[kBlock / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) wsum[wave] = v;
  __syncthreads();
  double s = 0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += wsum[w];
  }
  return s;
}

__global__ __launch_bounds__(kBlock) void k_fill(double* __restrict__ x, size_t n, double alpha) {
  const size_t n2 = n >> 1;
  const size_t stride = size_t(gridDim.x) * kBlock;
  const double2 v = make_double2(alpha, alpha);
  for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < n2; i += stride) st2(x + 2 * i, v);
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) x[n - 1] = alpha;
}

__global__ __launch_bounds__(kBlock) void k_scal(double* __restrict__ x, size_t n, double alpha) {
  using ssp::ld2nt;
  using ssp::st2nt;
  const size_t n2 = n >> 1;
  const size_t stride = size_t(gridDim.x) * kBlock;
  size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    double2 a0 = ld2nt(x + 2 * i), a1 = ld2nt(x + 2 * (i + stride)), a2 = ld2nt(x + 2 * (i + 2 * stride)),
            a3 = ld2nt(x + 2 * (i + 3 * stride));
    st2nt(x + 2 * i, make_double2(a0.x * alpha, a0.y * alpha));
    st2nt(x + 2 * (i + stride), make_double2(a1.x * alpha, a1.y * alpha));
    st2nt(x + 2 * (i + 2 * stride), make_double2(a2.x * alpha, a2.y * alpha));
    st2nt(x + 2 * (i + 3 * stride), make_double2(a3.x * alpha, a3.y * alpha));
  }
  for (; i < n2; i += stride) {
    double2 a = ld2(x + 2 * i);
    st2(x + 2 * i, make_double2(a.x * alpha, a.y * alpha));
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) x[n - 1] *= alpha;
}

// x = y (SC: x = alpha * y, the stored form of a scaled vector, ssp_scal_copy).
template <bool SC>
__global__ __launch_bounds__(kBlock) void k_copy(double* __restrict__ x, const double* __restrict__ y, size_t n,
                                                 double alpha) {
  using ssp::ld2nt;
  using ssp::st2nt;
  const size_t n2 = n >> 1;
  const size_t stride = size_t(gridDim.x) * kBlock;
  size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    double2 a0 = ld2nt(y + 2 * i), a1 = ld2nt(y + 2 * (i + stride)), a2 = ld2nt(y + 2 * (i + 2 * stride)),
            a3 = ld2nt(y + 2 * (i + 3 * stride));
    st2nt(x + 2 * i, sc2<SC>(a0, alpha));
    st2nt(x + 2 * (i + stride), sc2<SC>(a1, alpha));
    st2nt(x + 2 * (i + 2 * stride), sc2<SC>(a2, alpha));
    st2nt(x + 2 * (i + 3 * stride), sc2<SC>(a3, alpha));
  }
  for (; i < n2; i += stride) st2(x + 2 * i, sc2<SC>(ld2(y + 2 * i), alpha));
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) x[n - 1] = sc1<SC>(y[n - 1], alpha);
}

// y += alpha * x, element order as std::transform(y, x): y + alpha*x (one fma rounding).
// SC: operands with deferred scales, y = (y*ys) + alpha*(x*xs) with the same single fma.
template <bool SC>
__global__ __launch_bounds__(kBlock) void k_axpy(const double* __restrict__ x, double* __restrict__ y, size_t n,
                                                 double alpha, double xs, double ys) {
  const size_t n2 = n >> 1;
  const size_t stride = size_t(gridDim.x) * kBlock;
  size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    using ssp::ld2nt;
    using ssp::st2nt;
    double2 xv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) xv[u] = sc2<SC>(ld2nt(x + 2 * (i + u * stride)), xs);
#pragma unroll
    for (int u = 0; u < 4; ++u) yv[u] = sc2<SC>(ld2nt(y + 2 * (i + u * stride)), ys);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      st2nt(y + 2 * (i + u * stride), make_double2(fma(alpha, xv[u].x, yv[u].x), fma(alpha, xv[u].y, yv[u].y)));
  }
  for (; i < n2; i += stride) {
    double2 a = sc2<SC>(ld2(x + 2 * i), xs), b = sc2<SC>(ld2(y + 2 * i), ys);
    st2(y + 2 * i, make_double2(fma(alpha, a.x, b.x), fma(alpha, a.y, b.y)));
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
    y[n - 1] = fma(alpha, sc1<SC>(x[n - 1], xs), sc1<SC>(y[n - 1], ys));
}

__global__ __launch_bounds__(kBlock) void k_scal_win(double* __restrict__ x, size_t n, double alpha) {
  using ssp::ld2nt;
  using ssp::st2nt;
  ssp::for_windows<kWinU>(
      n,
      [&](size_t p0) {
        double2 v[kWinU];
#pragma unroll
        for (int u = 0; u < kWinU; ++u) v[u] = ld2nt(x + 2 * (p0 + 64 * u));
#pragma unroll
        for (int u = 0; u < kWinU; ++u) st2nt(x + 2 * (p0 + 64 * u), make_double2(v[u].x * alpha, v[u].y * alpha));
      },
      [&](size_t i) {
        const double2 a = ld2(x + 2 * i);
        st2(x + 2 * i, make_double2(a.x * alpha, a.y * alpha));
      },
      [&](size_t e) { x[e] *= alpha; });
}

template <bool SC>
__global__ __launch_bounds__(kBlock) void k_copy_win(double* __restrict__ x, const double* __restrict__ y, size_t n,
                                                     double alpha) {
  using ssp::ld2nt;
  using ssp::st2nt;
  ssp::for_windows<kWinU>(
      n,
      [&](size_t p0) {
        double2 v[kWinU];
#pragma unroll
        for (int u = 0; u < kWinU; ++u) v[u] = ld2nt(y + 2 * (p0 + 64 * u));
#pragma unroll
        for (int u = 0; u < kWinU; ++u) st2nt(x + 2 * (p0 + 64 * u), sc2<SC>(v[u], alpha));
      },
      [&](size_t i) { st2(x + 2 * i, sc2<SC>(ld2(y + 2 * i), alpha)); },
      [&](size_t e) { x[e] = sc1<SC>(y[e], alpha); });
}

// y += alpha * x in the window shape; the same single fma per element as k_axpy.
template <bool SC>
__global__ __launch_bounds__(kBlock) void k_axpy_win(const double* __restrict__ x, double* __restrict__ y, size_t n,
                                                     double alpha, double xs, double ys) {
  using ssp::ld2nt;
  using ssp::st2nt;
  ssp::for_windows<kWinU>(
      n,
      [&](size_t p0) {
        double2 xv[kWinU], yv[kWinU];
#pragma unroll
        for (int u = 0; u < kWinU; ++u) xv[u] = sc2<SC>(ld2nt(x + 2 * (p0 + 64 * u)), xs);
#pragma unroll
        for (int u = 0; u < kWinU; ++u) yv[u] = sc2<SC>(ld2nt(y + 2 * (p0 + 64 * u)), ys);
#pragma unroll
        for (int u = 0; u < kWinU; ++u)
          st2nt(y + 2 * (p0 + 64 * u), make_double2(fma(alpha, xv[u].x, yv[u].x), fma(alpha, xv[u].y, yv[u].y)));
      },
      [&](size_t i) {
        const double2 a = sc2<SC>(ld2(x + 2 * i), xs), b = sc2<SC>(ld2(y + 2 * i), ys);
        st2(y + 2 * i, make_double2(fma(alpha, a.x, b.x), fma(alpha, a.y, b.y)));
      },
      [&](size_t e) { y[e] = fma(alpha, sc1<SC>(x[e], xs), sc1<SC>(y[e], ys)); });
}

// SAME: x == y (norms), one load stream.  Window shape (kDotU KiB per vector per wave visit),
// 4 accumulators per lane (window position u into accumulator u % 4), then the positions past the
// last whole window and the odd element into accumulator 0.
template <bool SAME, bool SC>
__global__ __launch_bounds__(kBlock) void k_dot_partial(const double* __restrict__ x, const double* __restrict__ y,
                                                        size_t n, double* __restrict__ partial,
                                                        const ssp::FoldTail tail, double xs, double ys) {
  using ssp::ld2nt;
  double acc[4] = {0, 0, 0, 0};
  ssp::for_windows<kDotU>(
      n,
      [&](size_t p0) {
        double2 xv[kDotU], yv[kDotU];
#pragma unroll
        for (int u = 0; u < kDotU; ++u) xv[u] = sc2<SC>(ld2nt(x + 2 * (p0 + 64 * u)), xs);
#pragma unroll
        for (int u = 0; u < kDotU; ++u) yv[u] = SAME ? xv[u] : sc2<SC>(ld2nt(y + 2 * (p0 + 64 * u)), ys);
#pragma unroll
        for (int u = 0; u < kDotU; ++u) {
          acc[u & 3] = fma(xv[u].x, yv[u].x, acc[u & 3]);
          acc[u & 3] = fma(xv[u].y, yv[u].y, acc[u & 3]);
        }
      },
      [&](size_t i) {
        const double2 a = sc2<SC>(ld2(x + 2 * i), xs);
        const double2 b = SAME ? a : sc2<SC>(ld2(y + 2 * i), ys);
        acc[0] = fma(a.x, b.x, acc[0]);
        acc[0] = fma(a.y, b.y, acc[0]);
      },
      [&](size_t e) {
        const double a = sc1<SC>(x[e], xs);
        acc[0] = fma(a, SAME ? a : sc1<SC>(y[e], ys), acc[0]);
      });
  const double s0 = acc[0], s1 = acc[1], s2 = acc[2], s3 = acc[3];
  double s = block_sum((s0 + s1) + (s2 + s3));
  if (threadIdx.x == 0) ssp::store_partial(partial + blockIdx.x, s);
  ssp::fold_tail(partial, tail);
}

// out[(row0+r)*ldo + col0+c] = sum_b partial[b*rows*cols + r*cols + c]; one workgroup per output.
__global__ __launch_bounds__(kBlock) void k_reduce_partials(const double* __restrict__ partial, int nblocks, int rows,
                                                            int cols, double* __restrict__ out, int ldo, int row0,
                                                            int col0) {
  const int o = blockIdx.x;
  const int r = o / cols, c = o % cols;
  const size_t stride = size_t(rows) * cols;
  double s = 0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock) s += partial[size_t(b) * stride + o];
  s = block_sum(s);
  if (threadIdx.x == 0) out[size_t(row0 + r) * ldo + col0 + c] = s;
}

// The same pass publishing straight to the coherent host result buffer (one rank, no exchange), in
// place of k_reduce_partials + the k_publish copy behind it: each workgroup stores its sum to host
// memory (system scope) and, in the call's last pass (`flag` set), drains the store before its arrival
// (two-level counter, as ssp::fold_tail's); the last arriver sets the flag.  The earlier passes of a
// call completed before this one started (stream order), so their stores are in memory by then.  The
// sums are k_reduce_partials' (same order, same tree).
__global__ __launch_bounds__(kBlock) void k_reduce_publish(const double* __restrict__ partial, int nblocks, int rows,
                                                           int cols, double* host, int ldo, int row0, int col0,
                                                           unsigned* counter, unsigned long long* flag,
                                                           unsigned long long seq) {
  const int o = blockIdx.x;
  const int r = o / cols, c = o % cols;
  const size_t stride = size_t(rows) * cols;
  double s = 0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock) s += partial[size_t(b) * stride + o];
  s = block_sum(s);
  if (threadIdx.x == 0) {
    __hip_atomic_store(host + size_t(row0 + r) * ldo + col0 + c, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (flag) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sum has reached host memory
      const unsigned G = gridDim.x, sh = blockIdx.x & (ssp::kFoldShards - 1);
      const unsigned nsh = G < ssp::kFoldShards ? G : ssp::kFoldShards;
      const unsigned in_sh = (G - sh + ssp::kFoldShards - 1) / ssp::kFoldShards;
      unsigned* cs = counter + ssp::kFoldLine * sh;
      if (__hip_atomic_fetch_add(cs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_sh - 1) {
        __hip_atomic_store(cs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned* top = counter + ssp::kFoldLine * ssp::kFoldShards;
        if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1) {
          __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
}

struct PrecArgs {
  double* a[ssp::kPrecVec];
  double shift[ssp::kPrecVec];
  const double* d;
  int nvec;
  size_t n;
};

// a[v][i] = a[v][i] / ((d[i] - shift[v]) + 1e-15): reference itsolv/IterativeSolver.h:52-53.
__global__ __launch_bounds__(kBlock) void k_precondition(const PrecArgs p) {
  using ssp::ld2nt;
  using ssp::st2nt;
  constexpr int U = 4;
  ssp::for_windows<U>(
      p.n,
      [&](size_t p0) {
        double2 dv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) dv[u] = ld2nt(p.d + 2 * (p0 + 64 * u));
        for (int v = 0; v < p.nvec; ++v) {
          double2 av[U];
#pragma unroll
          for (int u = 0; u < U; ++u) av[u] = ld2nt(p.a[v] + 2 * (p0 + 64 * u));
#pragma unroll
          for (int u = 0; u < U; ++u) {
            av[u].x = av[u].x / (dv[u].x - p.shift[v] + 1e-15);
            av[u].y = av[u].y / (dv[u].y - p.shift[v] + 1e-15);
            st2nt(p.a[v] + 2 * (p0 + 64 * u), av[u]);
          }
        }
      },
      [&](size_t i) {
        const double2 dv = ld2(p.d + 2 * i);
        for (int v = 0; v < p.nvec; ++v) {
          double2 av = ld2(p.a[v] + 2 * i);
          av.x = av.x / (dv.x - p.shift[v] + 1e-15);
          av.y = av.y / (dv.y - p.shift[v] + 1e-15);
          st2(p.a[v] + 2 * i, av);
        }
      },
      [&](size_t j) {
        for (int v = 0; v < p.nvec; ++v) p.a[v][j] = p.a[v][j] / (p.d[j] - p.shift[v] + 1e-15);
      });
}

int check_vec(const void* p, size_t n, const char* what) {
  if (n == 0) return SSP_OK;
  if (!p) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": null vector");
  if (!ssp::aligned16(p)) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": vector not 16-byte aligned");
  return SSP_OK;
}

}  // namespace

namespace ssp {
int launch_reduce_partials(ssp_ctx* ctx, const double* partial, int nblocks, int rows, int cols, double* out, int ldo,
                           int row0, int col0, const FoldTail* pub, bool last) {
  if (rows * cols == 0) return SSP_OK;
  if (pub && pub->host) {
    SSP_LAUNCH(k_reduce_publish, dim3(rows * cols), dim3(kBlock), 0, ctx->stream, partial, nblocks, rows, cols,
               pub->host, ldo, row0, col0, pub->counter, last ? pub->flag : nullptr, pub->seq);
    SSP_TRY_HIP(hipGetLastError());
    return SSP_OK;
  }
  SSP_LAUNCH(k_reduce_partials, dim3(rows * cols), dim3(kBlock), 0, ctx->stream, partial, nblocks, rows, cols,
                     out, ldo, row0, col0);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}
}  // namespace ssp

extern "C" {

int ssp_fill(ssp_ctx* ctx, double alpha, double* x, size_t n) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(check_vec(x, n, "ssp_fill"));
  if (n == 0) return SSP_OK;
  ssp::LedgerScope ls(ctx, "fill", 8.0 * n);
  SSP_LAUNCH(k_fill, dim3(ssp::stream_grid(ctx, n / 2 + 1, 1, 64)), dim3(kBlock), 0, ctx->stream, x, n, alpha);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int ssp_scal(ssp_ctx* ctx, double alpha, double* x, size_t n) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(check_vec(x, n, "ssp_scal"));
  if (n == 0) return SSP_OK;
  ssp::LedgerScope ls(ctx, "scal", 16.0 * n);
  if (n >= kWinMin)
    SSP_LAUNCH(k_scal_win, dim3(ssp::win_grid(ctx, n, kWinU, 16)), dim3(kBlock), 0, ctx->stream, x, n, alpha);
  else
    SSP_LAUNCH(k_scal, dim3(ssp::stream_grid(ctx, n / 2 + 1, 4, 64)), dim3(kBlock), 0, ctx->stream, x, n, alpha);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

}  // extern "C"

namespace {
int copy_impl(ssp_ctx* ctx, double alpha, double* x, const double* y, size_t n, bool scaled, const char* what) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(check_vec(x, n, what));
  SSP_TRY(check_vec(y, n, what));
  if (n == 0 || (x == y && !scaled)) return SSP_OK;
  if (x == y) return ssp_scal(ctx, alpha, x, n);
  ssp::LedgerScope ls(ctx, scaled ? "scal_copy" : "copy", 16.0 * n);
  if (n >= kWinMin) {
    const dim3 g(ssp::win_grid(ctx, n, kWinU, 16));
    if (scaled) SSP_LAUNCH(k_copy_win<true>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha);
    else SSP_LAUNCH(k_copy_win<false>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha);
  } else {
    const dim3 g(ssp::stream_grid(ctx, n / 2 + 1, 4, 64));
    if (scaled) SSP_LAUNCH(k_copy<true>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha);
    else SSP_LAUNCH(k_copy<false>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha);
  }
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int axpy_impl(ssp_ctx* ctx, double alpha, const double* x, double xs, double* y, double ys, size_t n,
              const char* what) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(check_vec(x, n, what));
  SSP_TRY(check_vec(y, n, what));
  if (n == 0) return SSP_OK;
  const bool sc = xs != 1.0 || ys != 1.0;
  ssp::LedgerScope ls(ctx, "axpy", 24.0 * n);
  if (ssp::exact_mode(ctx, n)) return ssp::exact_outer(ctx, &alpha, &x, &xs, 1, &y, &ys, 1, n, false);
  if (n >= kWinMin) {
    const dim3 g(ssp::win_grid(ctx, n, kWinU, 16));
    if (sc) SSP_LAUNCH(k_axpy_win<true>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha, xs, ys);
    else SSP_LAUNCH(k_axpy_win<false>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha, xs, ys);
  } else {
    const dim3 g(ssp::stream_grid(ctx, n / 2 + 1, 4, 64));
    if (sc) SSP_LAUNCH(k_axpy<true>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha, xs, ys);
    else SSP_LAUNCH(k_axpy<false>, g, dim3(kBlock), 0, ctx->stream, x, y, n, alpha, xs, ys);
  }
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int dot_impl(ssp_ctx* ctx, const double* x, double xs, const double* y, double ys, size_t n, double* out,
             const char* what) {
  SSP_CHECK_CTX(ctx);
  if (!out) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": null out");
  SSP_TRY(check_vec(x, n, what));
  SSP_TRY(check_vec(y, n, what));
  if (n == 0) {
    SSP_TRY(ssp::ensure_result(ctx, 1));
    SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, sizeof(double), ctx->stream));
    return ssp::reduce_fetch(ctx, out, 1);
  }
  if (ssp::exact_mode(ctx, n)) {
    ssp::FoldTail tail{};
    SSP_TRY(ssp::fold_begin(ctx, 1, &tail));
    {
      ssp::LedgerScope ls(ctx, "dot", (x == y && xs == ys ? 8.0 : 16.0) * n);
      SSP_TRY(ssp::exact_inner(ctx, &x, &xs, 1, &y, &ys, 1, n, false, tail));
    }
    return ssp::fold_finish(ctx, tail, out);
  }
  const unsigned grid = ssp::win_grid(ctx, n, kDotU, 8);
  SSP_TRY(ssp::ensure_partial(ctx, grid));
  ssp::FoldTail tail{};
  SSP_TRY(ssp::fold_begin(ctx, 1, &tail));
  {
    const bool same = x == y && xs == ys, sc = xs != 1.0 || ys != 1.0;
    ssp::LedgerScope ls(ctx, "dot", (same ? 8.0 : 16.0) * n);
    const dim3 g(grid);
    double* part = ctx->partial;
    if (same && sc) SSP_LAUNCH((k_dot_partial<true, true>), g, dim3(kBlock), 0, ctx->stream, x, y, n, part, tail, xs, ys);
    else if (same) SSP_LAUNCH((k_dot_partial<true, false>), g, dim3(kBlock), 0, ctx->stream, x, y, n, part, tail, xs, ys);
    else if (sc) SSP_LAUNCH((k_dot_partial<false, true>), g, dim3(kBlock), 0, ctx->stream, x, y, n, part, tail, xs, ys);
    else SSP_LAUNCH((k_dot_partial<false, false>), g, dim3(kBlock), 0, ctx->stream, x, y, n, part, tail, xs, ys);
    SSP_TRY_HIP(hipGetLastError());
  }
  return ssp::fold_finish(ctx, tail, out);
}
}  // namespace

extern "C" {

int ssp_copy(ssp_ctx* ctx, double* x, const double* y, size_t n) { return copy_impl(ctx, 1.0, x, y, n, false, "ssp_copy"); }

int ssp_scal_copy(ssp_ctx* ctx, double alpha, double* x, const double* y, size_t n) {
  return copy_impl(ctx, alpha, x, y, n, true, "ssp_scal_copy");
}

int ssp_axpy(ssp_ctx* ctx, double alpha, const double* x, double* y, size_t n) {
  return axpy_impl(ctx, alpha, x, 1.0, y, 1.0, n, "ssp_axpy");
}

int ssp_axpy_scaled(ssp_ctx* ctx, double alpha, const double* x, double xs, double* y, double ys, size_t n) {
  return axpy_impl(ctx, alpha, x, xs, y, ys, n, "ssp_axpy_scaled");
}

int ssp_dot(ssp_ctx* ctx, const double* x, const double* y, size_t n, double* out) {
  return dot_impl(ctx, x, 1.0, y, 1.0, n, out, "ssp_dot");
}

int ssp_dot_scaled(ssp_ctx* ctx, const double* x, double xs, const double* y, double ys, size_t n, double* out) {
  return dot_impl(ctx, x, xs, y, ys, n, out, "ssp_dot_scaled");
}

int ssp_precondition(ssp_ctx* ctx, double* const* a, int nvec, const double* d, const double* shift, size_t n) {
  SSP_CHECK_CTX(ctx);
  if (nvec < 0 || (nvec > 0 && (!a || !shift))) return ssp::set_error(SSP_ERR_ARG, "ssp_precondition: bad vectors");
  if (n == 0 || nvec == 0) return SSP_OK;
  SSP_TRY(check_vec(d, n, "ssp_precondition"));
  ssp::LedgerScope ls(ctx, "precondition", 8.0 * n * (1 + 2 * nvec));
  for (int v0 = 0; v0 < nvec; v0 += ssp::kPrecVec) {
    PrecArgs p{};
    p.nvec = std::min(ssp::kPrecVec, nvec - v0);
    for (int v = 0; v < p.nvec; ++v) {
      SSP_TRY(check_vec(a[v0 + v], n, "ssp_precondition"));
      p.a[v] = a[v0 + v];
      p.shift[v] = shift[v0 + v];
    }
    p.d = d;
    p.n = n;
    SSP_LAUNCH(k_precondition, dim3(ssp::win_grid(ctx, n, 4, 8)), dim3(kBlock), 0, ctx->stream, p);
    SSP_TRY_HIP(hipGetLastError());
  }
  return SSP_OK;
}

}  // extern "C"
