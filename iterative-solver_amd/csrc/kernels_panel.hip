// Tall-skinny panel kernels: gemm_inner (m x k overlaps) and gemm_outer (k sources -> m destinations).
//
// Reference: util/gemm.h:257-279 computes both pairwise (handler.dot / handler.axpy per pair), so a
// 8 x 48 gemm_inner streams 2*8*48 vectors and a 48 -> 8 gemm_outer streams 3*8*48 vectors.  Here
// every vector of the panel is read from HBM exactly once per call:
//   gemm_inner  bytes = 8 N (m + k)       gemm_outer  bytes = 8 N (k + 2 m)
//
// gemm_inner runs on the f64 matrix cores (v_mfma_f64_16x16x4_f64).  The contraction index of the
// MFMA is the vector index n, so one wave instruction consumes 4 (x 2 registers) elements of 16 x
// vectors and 16 y vectors.  Lane l (c = l & 15, q = l >> 4) loads 16 B of vector c at element
// base + 2q: for a fixed vector the four q-lanes read one contiguous 64 B segment.  The two doubles
// of that load feed two MFMAs, so the contraction order within a 8-element chunk is permuted — the
// result is the same sum in a different rounding order.  Accumulators: one 16x16 f64 tile (4
// doubles per lane) per 16 columns.  Per-wave partial tiles are summed through LDS to one partial
// per workgroup, then summed over workgroups in a fixed order (ssp::launch_reduce_partials), so the
// result is bitwise reproducible run to run and identical on every rank after the RCCL allreduce.
#include <algorithm>
#include <vector>

#include "ssp_internal.h"

namespace {

using ssp::kBlock;
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
__device__ __forceinline__ void st2(double* p, double2 v) { *reinterpret_cast<double2*>(p) = v; }

struct InnerArgs {
  const double* x[ssp::kInnerRows];
  const double* y[ssp::kInnerCols];
  int m;
  int k;
  size_t n;
  double* partial;  // [gridDim.x][m][k]
};

// NT: column tiles of 16 (k <= 16*NT); U: 8-element chunks per wave per iteration.
template <int NT, int U>
__global__ __launch_bounds__(kBlock) void k_gemm_inner(const InnerArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  const double* xp = c < a.m ? a.x[c] : nullptr;
  const double* yp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) yp[t] = (16 * t + c < a.k) ? a.y[16 * t + c] : nullptr;

  f64x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f64x4{0, 0, 0, 0};

  const size_t gw = size_t(blockIdx.x) * (kBlock / 64) + wave;
  const size_t nw = size_t(gridDim.x) * (kBlock / 64);
  const size_t chunk = 8 * U;
  const size_t nchunks = a.n / chunk;
  const double2 z2 = make_double2(0, 0);
  for (size_t ch = gw; ch < nchunks; ch += nw) {
    const size_t base = ch * chunk + 2 * q;
    double2 xv[U];
    double2 yv[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = xp ? ld2(xp + base + 8 * u) : z2;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) yv[u][t] = yp[t] ? ld2(yp[t] + base + 8 * u) : z2;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[u].x, yv[u][t].x, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[u].y, yv[u][t].y, acc[t], 0, 0, 0);
      }
  }
  // Remainder [nchunks*chunk, n): 8-element sub-chunks spread over the waves, guarded loads.
  for (size_t s = nchunks * chunk + gw * 8; s < a.n; s += nw * 8) {
    const size_t i0 = s + 2 * q, i1 = i0 + 1;
    const double x0 = (xp && i0 < a.n) ? xp[i0] : 0.0;
    const double x1 = (xp && i1 < a.n) ? xp[i1] : 0.0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const double y0 = (yp[t] && i0 < a.n) ? yp[t][i0] : 0.0;
      const double y1 = (yp[t] && i1 < a.n) ? yp[t][i1] : 0.0;
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, y0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, y1, acc[t], 0, 0, 0);
    }
  }

  // Workgroup reduction of the 4 waves' tiles.  f64 16x16x4 C layout: register r of lane l holds
  // C[row = (l >> 4) + 4 r][col = l & 15].
  __shared__ double red[kBlock / 64][NT * 4][64];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][t * 4 + r][lane] = acc[t][r];
  __syncthreads();
  const size_t mk = size_t(a.m) * a.k;
  double* out = a.partial + size_t(blockIdx.x) * mk;
  for (int s = threadIdx.x; s < NT * 4 * 64; s += kBlock) {
    const int tr = s >> 6, ln = s & 63;
    const int t = tr >> 2, r = tr & 3;
    const int row = (ln >> 4) + 4 * r, col = 16 * t + (ln & 15);
    if (row < a.m && col < a.k) {
      double v = red[0][tr][ln];
#pragma unroll
      for (int w = 1; w < kBlock / 64; ++w) v += red[w][tr][ln];
      out[size_t(row) * a.k + col] = v;
    }
  }
}

struct OuterArgs {
  const double* x[ssp::kOuterSrc];
  double* y[ssp::kOuterDst];
  int k;
  int m;
  size_t n;
  double alpha[ssp::kOuterAlpha];  // alpha[i*m + j]
};
static_assert(sizeof(OuterArgs) <= 4000, "kernel argument block too large");

// yy[j] += sum_i alpha(i,j) xx[i]: for each destination the sources are added in order i = 0..k-1,
// as the reference's pairwise axpy loop does (util/gemm.h:259-264).
template <int M>
__global__ __launch_bounds__(kBlock) void k_gemm_outer(const OuterArgs a) {
  const size_t n2 = a.n >> 1;
  const size_t stride = size_t(gridDim.x) * kBlock;
  for (size_t p = size_t(blockIdx.x) * kBlock + threadIdx.x; p < n2; p += stride) {
    double2 acc[M];
#pragma unroll
    for (int j = 0; j < M; ++j)
      if (j < a.m) acc[j] = ld2(a.y[j] + 2 * p);
    int i = 0;
    for (; i + 4 <= a.k; i += 4) {
      const double2 x0 = ld2(a.x[i] + 2 * p), x1 = ld2(a.x[i + 1] + 2 * p), x2 = ld2(a.x[i + 2] + 2 * p),
                    x3 = ld2(a.x[i + 3] + 2 * p);
#pragma unroll
      for (int j = 0; j < M; ++j) {
        if (j < a.m) {
          const double a0 = a.alpha[i * a.m + j], a1 = a.alpha[(i + 1) * a.m + j], a2 = a.alpha[(i + 2) * a.m + j],
                       a3 = a.alpha[(i + 3) * a.m + j];
          acc[j].x = fma(a0, x0.x, acc[j].x);
          acc[j].y = fma(a0, x0.y, acc[j].y);
          acc[j].x = fma(a1, x1.x, acc[j].x);
          acc[j].y = fma(a1, x1.y, acc[j].y);
          acc[j].x = fma(a2, x2.x, acc[j].x);
          acc[j].y = fma(a2, x2.y, acc[j].y);
          acc[j].x = fma(a3, x3.x, acc[j].x);
          acc[j].y = fma(a3, x3.y, acc[j].y);
        }
      }
    }
    for (; i < a.k; ++i) {
      const double2 xv = ld2(a.x[i] + 2 * p);
#pragma unroll
      for (int j = 0; j < M; ++j) {
        if (j < a.m) {
          const double al = a.alpha[i * a.m + j];
          acc[j].x = fma(al, xv.x, acc[j].x);
          acc[j].y = fma(al, xv.y, acc[j].y);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < M; ++j)
      if (j < a.m) st2(a.y[j] + 2 * p, acc[j]);
  }
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x < a.m) {
    const size_t e = a.n - 1;
    const int j = threadIdx.x;
    double v = a.y[j][e];
    for (int i = 0; i < a.k; ++i) v = fma(a.alpha[i * a.m + j], a.x[i][e], v);
    a.y[j][e] = v;
  }
}

int check_ptrs(const double* const* v, int count, size_t n, const char* what) {
  if (count > 0 && !v) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": null vector list");
  if (n == 0) return SSP_OK;
  for (int i = 0; i < count; ++i) {
    if (!v[i]) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": null vector");
    if (!ssp::aligned16(v[i])) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": vector not 16-byte aligned");
  }
  return SSP_OK;
}

// Number of workgroups for a gemm_inner launch: enough to give every CU 4 workgroups (16 waves)
// when n allows, otherwise one wave per 8U-element chunk.
unsigned inner_grid(const ssp_ctx* ctx, size_t n, int U) {
  const size_t chunks = n / (8 * U) + 1;
  size_t blocks = (chunks + 3) / 4;
  const size_t cap = size_t(ctx->num_cus) * 4;
  return unsigned(std::max<size_t>(1, std::min(blocks, cap)));
}

template <int NT>
void launch_inner_nt(ssp_ctx* ctx, unsigned grid, const InnerArgs& a) {
  constexpr int U = NT <= 2 ? 4 : 2;
  hipLaunchKernelGGL((k_gemm_inner<NT, U>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
}

int launch_inner(ssp_ctx* ctx, const InnerArgs& a, unsigned grid, int nt) {
  switch (nt) {
    case 1: launch_inner_nt<1>(ctx, grid, a); break;
    case 2: launch_inner_nt<2>(ctx, grid, a); break;
    case 3: launch_inner_nt<3>(ctx, grid, a); break;
    default: launch_inner_nt<4>(ctx, grid, a); break;
  }
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int launch_outer(ssp_ctx* ctx, const OuterArgs& a) {
  const unsigned grid = ssp::stream_grid(ctx, a.n / 2 + 1, 1);
  if (a.m <= 1)
    hipLaunchKernelGGL((k_gemm_outer<1>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else if (a.m <= 2)
    hipLaunchKernelGGL((k_gemm_outer<2>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else if (a.m <= 4)
    hipLaunchKernelGGL((k_gemm_outer<4>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else if (a.m <= 8)
    hipLaunchKernelGGL((k_gemm_outer<8>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else
    hipLaunchKernelGGL((k_gemm_outer<16>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

}  // namespace

extern "C" {

int ssp_gemm_inner(ssp_ctx* ctx, const double* const* xx, int m, const double* const* yy, int k, size_t n,
                   double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 0 || k < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner: negative dimension");
  if (m * k > 0 && !out) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner: null out");
  if (m == 0 || k == 0) return SSP_OK;
  SSP_TRY(check_ptrs(xx, m, n, "ssp_gemm_inner"));
  SSP_TRY(check_ptrs(yy, k, n, "ssp_gemm_inner"));
  // Put the shorter side on the MFMA rows (padded to 16), the longer on the columns.
  const bool swap = m > k;
  const double* const* rows = swap ? yy : xx;
  const double* const* cols = swap ? xx : yy;
  const int R = swap ? k : m, C = swap ? m : k;
  const size_t total = size_t(R) * C;
  SSP_TRY(ssp::ensure_result(ctx, total));
  if (n == 0) {
    SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, total * sizeof(double), ctx->stream));
  } else {
    // Algorithmic bytes: every DISTINCT vector of the panel read once (8 N (m + k) when disjoint).
    std::vector<const double*> distinct(xx, xx + m);
    distinct.insert(distinct.end(), yy, yy + k);
    std::sort(distinct.begin(), distinct.end());
    const double nvec = double(std::unique(distinct.begin(), distinct.end()) - distinct.begin());
    ssp::LedgerScope ls(ctx, "gemm_inner", 8.0 * n * nvec);
    for (int r0 = 0; r0 < R; r0 += ssp::kInnerRows) {
      for (int c0 = 0; c0 < C; c0 += ssp::kInnerCols) {
        InnerArgs a{};
        a.m = std::min(ssp::kInnerRows, R - r0);
        a.k = std::min(ssp::kInnerCols, C - c0);
        a.n = n;
        for (int i = 0; i < a.m; ++i) a.x[i] = rows[r0 + i];
        for (int j = 0; j < a.k; ++j) a.y[j] = cols[c0 + j];
        const int nt = (a.k + 15) / 16;
        const unsigned grid = inner_grid(ctx, n, nt <= 2 ? 4 : 2);
        SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * a.m * a.k));
        a.partial = ctx->partial;
        SSP_TRY(launch_inner(ctx, a, grid, nt));
        SSP_TRY(ssp::launch_reduce_partials(ctx, ctx->partial, int(grid), a.m, a.k, ctx->result_dev, C, r0, c0));
      }
    }
  }
  SSP_TRY(ssp::allreduce_dev(ctx, ctx->result_dev, total));
  if (!swap) return ssp::fetch_result(ctx, out, total);
  std::vector<double> t(total);
  SSP_TRY(ssp::fetch_result(ctx, t.data(), total));
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) out[size_t(i) * k + j] = t[size_t(j) * m + i];
  return SSP_OK;
}

int ssp_gemm_outer(ssp_ctx* ctx, const double* alphas, const double* const* xx, int k, double* const* yy, int m,
                   size_t n) {
  SSP_CHECK_CTX(ctx);
  if (m < 0 || k < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer: negative dimension");
  if (m == 0 || k == 0 || n == 0) return SSP_OK;
  if (!alphas) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer: null alphas");
  SSP_TRY(check_ptrs(xx, k, n, "ssp_gemm_outer"));
  SSP_TRY(check_ptrs(const_cast<const double* const*>(yy), m, n, "ssp_gemm_outer"));
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < k; ++i)
      if (yy[j] == xx[i]) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer: a destination aliases a source");
  // Destinations are independent; sources are applied in increasing order, in groups that fit
  // the kernel argument block, so each destination sees the reference's summation order.
  ssp::LedgerScope ls(ctx, "gemm_outer", 8.0 * n * (k + 2.0 * m));
  for (int j0 = 0; j0 < m; j0 += ssp::kOuterDst) {
    const int mm = std::min(ssp::kOuterDst, m - j0);
    const int kmax = std::max(1, std::min(ssp::kOuterSrc, ssp::kOuterAlpha / mm));
    for (int i0 = 0; i0 < k; i0 += kmax) {
      OuterArgs a{};
      a.m = mm;
      a.k = std::min(kmax, k - i0);
      a.n = n;
      for (int i = 0; i < a.k; ++i) a.x[i] = xx[i0 + i];
      for (int j = 0; j < mm; ++j) a.y[j] = yy[j0 + j];
      for (int i = 0; i < a.k; ++i)
        for (int j = 0; j < mm; ++j) a.alpha[i * mm + j] = alphas[size_t(i0 + i) * m + j0 + j];
      SSP_TRY(launch_outer(ctx, a));
    }
  }
  return SSP_OK;
}

}  // extern "C"
