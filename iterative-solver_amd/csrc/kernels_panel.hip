// Tall-skinny panel kernels: gemm_inner (m x k overlaps) and gemm_outer (k sources -> m destinations).
//
// Reference: util/gemm.h:257-279 computes both pairwise (handler.dot / handler.axpy per pair), so a
// 8 x 48 gemm_inner streams 2*8*48 vectors and a 48 -> 8 gemm_outer streams 3*8*48 vectors.  Here
// every vector of the panel is read from HBM exactly once per call:
//   gemm_inner  bytes = 8 N (m + k)       gemm_outer  bytes = 8 N (k + 2 m)
//
// gemm_inner runs on the f64 matrix cores with the 4-block v_mfma_f64_4x4x4_f64 (measured lane map,
// tools/mfma_probe.hip):  lane l = 16k + 4b + i holds A_b[i][k] and B_b[k][i];  C_b[i][j] sits in
// lane 16i + 4b + j.  Rows / columns are groups of 4 vectors; the contraction (MFMA k and block b)
// runs over the vector index n.  The 16 lanes that hold one vector (same l & 3) load 16 B each at
// position p = l >> 2, i.e. 256 contiguous bytes per vector per load instruction (4 vectors per
// 1 KiB wave load), which streams at the HBM read rate (6.0-6.2 TB/s measured for 8 x 48 at N = 1e8,
// against 3.7 TB/s for the 16x16x4 layout, whose 16 x 64 B segments per load halve the load-path
// efficiency).  The two doubles of each 16 B load feed two MFMAs, so the summation order within a
// 32-element chunk is a fixed permutation.  Block partials are folded with two lane shuffles, waves
// through LDS, workgroups by a fixed-order second pass (ssp::launch_reduce_partials): bitwise
// reproducible, and identical on every rank after the RCCL allreduce.
#include <algorithm>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <vector>

#include "ssp_internal.h"

namespace {

using ssp::kBlock;

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
// Deferred scal (include/subspace_hip.h *_scaled): v * s is the one rounding an eager scal stores.
template <bool SC>
__device__ __forceinline__ double2 sc2(double2 v, double s) {
  return SC ? make_double2(v.x * s, v.y * s) : v;
}
template <bool SC>
__device__ __forceinline__ double sc1(double v, double s) {
  return SC ? v * s : v;
}

struct InnerArgs {
  const double* x[ssp::kInnerRows];  // rows: MG groups of 4
  const double* y[ssp::kInnerCols];  // columns: NG groups of 4
  double xs[ssp::kInnerRows];        // SC: deferred scales of the rows / columns
  double ys[ssp::kInnerCols];
  int m;
  int k;
  size_t n;
  double* partial;     // [gridDim.x][m][k]
  ssp::FoldTail tail;  // row kernel only: fused fold when tail.counter is set
};

// SYM: xx == yy (a symmetric overlap, MG == NG): each vector is loaded once and used as both
// operands of the MFMA.  SC: operands with deferred scales (each loaded element times its vector's
// scale before the MFMA).
// PIPE: the loads of the wave's next chunk are issued before the MFMAs of the current one (two
// register stages), so a wave keeps a chunk of every vector in flight while its matrix cores work.
// The chunks are accumulated in the same order (ch, ch + nw, ch + 2 nw, ...), so the results are
// bit-identical to the one-stage loop.  Operand lanes of absent vectors (4 g + r >= m) read their
// group's first vector -- the same addresses as that lane-group's valid lanes in the same load
// instruction, so no extra traffic -- and only feed accumulator rows / columns that are never
// stored (C[i][j] of the 4x4x4 MFMA depends on row i of A and column j of B alone).  Whole absent
// groups (4 g >= m: the instantiated NG above the panel's) skip their loads by a wave-uniform branch
// (re-reading one fixed line instead made every wave of the chip hit one L2 channel: 8 x 40 ran 6 %
// slower).  No load carries an exec-mask guard.
// PRE: the panel's first 4 MG columns are its rows (y[j] == x[j], ys[j] == xs[j] for j < m, columns
// m .. 4 MG - 1 padding whose results are dropped): those column groups take the row groups'
// registers instead of loading the same vectors again -- the batched overlap rows of the subspace
// update ([params, actions, Q, ...] against params) read each vector once.
template <int MG, int NG, bool SYM = false, bool SC = false, bool PIPE = false, bool PRE = false>
__global__ __launch_bounds__(kBlock) void k_gemm_inner(const InnerArgs a) {
  static_assert(!SYM || MG == NG, "symmetric panel needs square groups");
  static_assert(!PRE || (!SYM && NG >= MG), "column prefix needs at least the row groups");
  constexpr auto own = [](int h) { return SYM || (PRE && h < MG); };  // column group h = row group h
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 3, p = lane >> 2;
  const double* xp[MG];
  const double* yp[NG];
  double xsc[MG], ysc[NG];
  bool xok[MG], yok[NG];  // this lane's vector exists (remainder loop)
#pragma unroll
  for (int g = 0; g < MG; ++g) {
    xok[g] = 4 * g + r < a.m;
    xp[g] = xok[g] ? a.x[4 * g + r] : a.x[4 * g < a.m ? 4 * g : 0];
    xsc[g] = (SC && xok[g]) ? a.xs[4 * g + r] : 1.0;
  }
#pragma unroll
  for (int h = 0; h < NG; ++h) {
    yok[h] = 4 * h + r < a.k;
    yp[h] = yok[h] ? a.y[4 * h + r] : a.y[4 * h < a.k ? 4 * h : 0];
    ysc[h] = (SC && yok[h]) ? a.ys[4 * h + r] : 1.0;
  }
  double acc[MG][NG];
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) acc[g][h] = 0;

  // wave-uniform loop control in scalar registers
  const size_t gw = size_t(__builtin_amdgcn_readfirstlane(int(blockIdx.x * (kBlock / 64) + wave)));
  const size_t nw = size_t(gridDim.x) * (kBlock / 64);
  const size_t nchunks = a.n / 32;
  const double2 z2 = make_double2(0, 0);
  const auto load = [&](size_t ch, double2(&xv)[MG], double2(&yv)[NG]) {
    const size_t e = ch * 32 + 2 * p;
#pragma unroll
    for (int g = 0; g < MG; ++g) xv[g] = 4 * g < a.m ? ssp::ld2nt(xp[g] + e) : z2;
#pragma unroll
    for (int h = 0; h < NG; ++h) yv[h] = own(h) ? xv[h] : (4 * h < a.k ? ssp::ld2nt(yp[h] + e) : z2);
  };
  const auto mac = [&](double2(&xv)[MG], double2(&yv)[NG]) {
    // scales after every load of the chunk is in flight
    if constexpr (SC) {
#pragma unroll
      for (int g = 0; g < MG; ++g) xv[g] = sc2<SC>(xv[g], xsc[g]);
#pragma unroll
      for (int h = 0; h < NG; ++h) yv[h] = own(h) ? xv[h] : sc2<SC>(yv[h], ysc[h]);
    }
#pragma unroll
    for (int g = 0; g < MG; ++g)
#pragma unroll
      for (int h = 0; h < NG; ++h) {
        acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(xv[g].x, yv[h].x, acc[g][h], 0, 0, 0);
        acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(xv[g].y, yv[h].y, acc[g][h], 0, 0, 0);
      }
  };
  if constexpr (PIPE) {
    double2 xa[MG], ya[NG], xb[MG], yb[NG];
    size_t ch = gw;
    if (ch < nchunks) load(ch, xa, ya);
    for (;;) {
      if (ch + nw >= nchunks) {
        if (ch < nchunks) mac(xa, ya);
        break;
      }
      load(ch + nw, xb, yb);
      mac(xa, ya);
      ch += nw;
      if (ch + nw >= nchunks) {
        mac(xb, yb);
        break;
      }
      load(ch + nw, xa, ya);
      mac(xb, yb);
      ch += nw;
    }
  } else {
    for (size_t ch = gw; ch < nchunks; ch += nw) {
      double2 xv[MG], yv[NG];
      load(ch, xv, yv);
      mac(xv, yv);
    }
  }
  // Remainder [32 * nchunks, n): 32-element chunks spread over the waves, guarded element loads.
  for (size_t s = nchunks * 32 + gw * 32; s < a.n; s += nw * 32) {
    const size_t i0 = s + 2 * p, i1 = i0 + 1;
    double x0[MG], x1[MG];
#pragma unroll
    for (int g = 0; g < MG; ++g) {
      x0[g] = (xok[g] && i0 < a.n) ? sc1<SC>(xp[g][i0], xsc[g]) : 0.0;
      x1[g] = (xok[g] && i1 < a.n) ? sc1<SC>(xp[g][i1], xsc[g]) : 0.0;
    }
#pragma unroll
    for (int h = 0; h < NG; ++h) {
      const double y0 = own(h) ? x0[h] : ((yok[h] && i0 < a.n) ? sc1<SC>(yp[h][i0], ysc[h]) : 0.0);
      const double y1 = own(h) ? x1[h] : ((yok[h] && i1 < a.n) ? sc1<SC>(yp[h][i1], ysc[h]) : 0.0);
#pragma unroll
      for (int g = 0; g < MG; ++g) {
        acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(x0[g], y0, acc[g][h], 0, 0, 0);
        acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(x1[g], y1, acc[g][h], 0, 0, 0);
      }
    }
  }

  // Fold the 4 blocks (lane bits 2-3), then the 4 waves through LDS.
  __shared__ double red[kBlock / 64][MG * NG][16];
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) {
      double v = acc[g][h];
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if ((lane & 12) == 0) red[wave][g * NG + h][(lane >> 4) * 4 + (lane & 3)] = v;
    }
  __syncthreads();
  const size_t mk = size_t(a.m) * a.k;
  double* out = a.partial + size_t(blockIdx.x) * mk;
  for (int s = threadIdx.x; s < MG * NG * 16; s += kBlock) {
    const int gh = s >> 4, e = s & 15;
    const int row = 4 * (gh / NG) + (e >> 2), col = 4 * (gh % NG) + (e & 3);
    if (row < a.m && col < a.k) {
      double v = red[0][gh][e];
#pragma unroll
      for (int w = 1; w < kBlock / 64; ++w) v += red[w][gh][e];
      out[size_t(row) * a.k + col] = v;
    }
  }
}

// Panels of 1 x 1 and 1 x 2 (or 2 x 1) vectors: with only one or two MFMA operand rows live, the
// 4x4x4 layout leaves 3/4 of the lanes idle on loads (tools/shapes_bench.py: 1 x 1 at 3.4 TB/s),
// so these run on the VALU with every lane streaming 16 B per vector.  Two shapes:
//   k_gemm_inner_row_win  (default) each wave owns 4 consecutive KiB of every vector per visit, the
//                         shape of k_dot_partial;
//   k_gemm_inner_row      4 grid-strided positions in flight (round 2's shape, kept for the A/B:
//                         SSP_ROW_SHAPE=stride, tools/row_shape_ab.py).
// Round 2 kept the stride shape because the window order moved an ill-conditioned DIIS case (n = 1e5,
// rank 2, rho = 0.01, singular to rounding from its sixth step) from 15 to 30 iterations; with C5's
// well-posed instance (tests/golden/traces.json C5_*) the shape is decided by bandwidth
// (DESIGN.md section 4), and that case is held to its converged solution only.
template <int K, bool SC = false>
__global__ __launch_bounds__(kBlock) void k_gemm_inner_row(const InnerArgs a) {
  using ssp::ld2nt;
  const size_t n2 = a.n >> 1, stride = size_t(gridDim.x) * kBlock;
  double acc[K][2] = {};
  const bool same = K == 1 && a.y[0] == a.x[0] && (!SC || a.ys[0] == a.xs[0]);  // a norm: one load stream
  const double xs = SC ? a.xs[0] : 1.0;
  double ys[K];
#pragma unroll
  for (int j = 0; j < K; ++j) ys[j] = SC ? a.ys[j] : 1.0;
  size_t p = size_t(blockIdx.x) * kBlock + threadIdx.x;
  for (; p + 3 * stride < n2; p += 4 * stride) {
    double2 xv[4], yv[K][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) xv[u] = sc2<SC>(ld2nt(a.x[0] + 2 * (p + u * stride)), xs);
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) yv[j][u] = same ? xv[u] : sc2<SC>(ld2nt(a.y[j] + 2 * (p + u * stride)), ys[j]);
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc[j][u & 1] = fma(xv[u].x, yv[j][u].x, acc[j][u & 1]);
        acc[j][u & 1] = fma(xv[u].y, yv[j][u].y, acc[j][u & 1]);
      }
  }
  for (; p < n2; p += stride) {
    const double2 xv = sc2<SC>(ld2(a.x[0] + 2 * p), xs);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const double2 yv = sc2<SC>(ld2(a.y[j] + 2 * p), ys[j]);
      acc[j][0] = fma(xv.x, yv.x, acc[j][0]);
      acc[j][0] = fma(xv.y, yv.y, acc[j][0]);
    }
  }
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
#pragma unroll
    for (int j = 0; j < K; ++j)
      acc[j][0] = fma(sc1<SC>(a.x[0][a.n - 1], xs), sc1<SC>(a.y[j][a.n - 1], ys[j]), acc[j][0]);
  __shared__ double red[kBlock / 64][K];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double v = acc[j][0] + acc[j][1];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave][j] = v;
  }
  __syncthreads();
  if (int(threadIdx.x) < K) {
    double v = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) v += red[w][threadIdx.x];
    ssp::store_partial(a.partial + size_t(blockIdx.x) * K + threadIdx.x, v);
  }
  if (a.tail.counter) ssp::fold_tail<K>(a.partial, a.tail);
}

template <int K, bool SC = false>
__global__ __launch_bounds__(kBlock) void k_gemm_inner_row_win(const InnerArgs a) {
  using ssp::ld2nt;
  constexpr int U = 4;  // 4 KiB of each vector per wave visit
  double acc[K][2] = {};
  const bool same = K == 1 && a.y[0] == a.x[0] && (!SC || a.ys[0] == a.xs[0]);  // a norm: one load stream
  const double xs = SC ? a.xs[0] : 1.0;
  double ys[K];
#pragma unroll
  for (int j = 0; j < K; ++j) ys[j] = SC ? a.ys[j] : 1.0;
  ssp::for_windows<U>(
      a.n,
      [&](size_t p0) {
        double2 xv[U], yv[K][U];
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = ld2nt(a.x[0] + 2 * (p0 + 64 * u));
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
          for (int u = 0; u < U; ++u) yv[j][u] = same ? xv[u] : ld2nt(a.y[j] + 2 * (p0 + 64 * u));
        if constexpr (SC) {
#pragma unroll
          for (int u = 0; u < U; ++u) xv[u] = sc2<SC>(xv[u], xs);
#pragma unroll
          for (int j = 0; j < K; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) yv[j][u] = same ? xv[u] : sc2<SC>(yv[j][u], ys[j]);
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[j][u & 1] = fma(xv[u].x, yv[j][u].x, acc[j][u & 1]);
            acc[j][u & 1] = fma(xv[u].y, yv[j][u].y, acc[j][u & 1]);
          }
      },
      [&](size_t p) {
        const double2 xv = sc2<SC>(ld2(a.x[0] + 2 * p), xs);
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const double2 yv = sc2<SC>(ld2(a.y[j] + 2 * p), ys[j]);
          acc[j][0] = fma(xv.x, yv.x, acc[j][0]);
          acc[j][0] = fma(xv.y, yv.y, acc[j][0]);
        }
      },
      [&](size_t e) {
#pragma unroll
        for (int j = 0; j < K; ++j) acc[j][0] = fma(sc1<SC>(a.x[0][e], xs), sc1<SC>(a.y[j][e], ys[j]), acc[j][0]);
      });
  __shared__ double red[kBlock / 64][K];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double v = acc[j][0] + acc[j][1];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave][j] = v;
  }
  __syncthreads();
  if (int(threadIdx.x) < K) {
    double v = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) v += red[w][threadIdx.x];
    ssp::store_partial(a.partial + size_t(blockIdx.x) * K + threadIdx.x, v);
  }
  if (a.tail.counter) ssp::fold_tail<K>(a.partial, a.tail);
}

struct OuterArgs {
  const double* x[ssp::kOuterSrc];
  double* y[ssp::kOuterDst];
  int k;
  int m;
  int set;  // 1: yy[j] = sum (destinations not read: fill(0) + gemm_outer in one pass)
  size_t n;
  const double* alpha_dev;         // k*m > kOuterAlpha: alpha[i*m + j] in device memory
  const double* scale_dev;         // SC: deferred scales, sources [0, k) then destinations [k, k + m)
  double alpha[ssp::kOuterAlpha];  // alpha[i*m + j] in the argument block
};
static_assert(sizeof(OuterArgs) <= 4000, "kernel argument block too large");

// yy[j] += sum_i alpha(i,j) xx[i]: for each destination the sources are added in order i = 0..k-1,
// as the reference's pairwise axpy loop does (util/gemm.h:259-264).  Each wave owns windows of
// kOuterWin consecutive double2 positions (64 lanes x 16 B x kOuterWin contiguous bytes per vector)
// and loads 4 sources x kOuterWin positions before the fmas; sources and destinations are streamed
// once, with nontemporal accesses (tools/mb_stream.hip: 5.35 TB/s against 4.8 for one position per
// lane and plain accesses).
constexpr int kOuterWin = 4;

// SET (a.set = 1) is a separate instantiation: the write-only construct_solution form shows under its
// own name in rocprofv3 statistics, so its launches are not averaged with the read-modify-write ones.
// SC: sources and (read-modify-write) destinations with deferred scales, applied as each element is
// loaded (include/subspace_hip.h ssp_gemm_outer_scaled).
template <int M, bool DEV, bool SET, bool SC = false>
__global__ __launch_bounds__(kBlock) void k_gemm_outer(const OuterArgs a) {
  using ssp::ld2nt;
  using ssp::st2nt;
  // Device-resident alphas are read through the constant address space (scalar loads, as the
  // argument block's are): they are uniform across the wave and read-only in the kernel.
  using cdouble = const __attribute__((address_space(4))) double;
  const auto alpha = [&](int idx) { return DEV ? ((cdouble*)a.alpha_dev)[idx] : a.alpha[idx]; };
  const auto scale = [&](int idx) { return SC ? ((cdouble*)a.scale_dev)[idx] : 1.0; };
  constexpr int U = M > 8 ? 2 : kOuterWin;  // 16 destinations: 2 windows keep 2 waves per SIMD
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  const size_t nw = size_t(gridDim.x) * (kBlock / 64);
  const size_t n2 = a.n >> 1, win = 64 * U;
  const double2 z2 = make_double2(0, 0);
  for (size_t c = gw; c * win < n2; c += nw) {
    const size_t p0 = c * win + lane;
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ok[u] = p0 + 64 * u < n2;
    double2 acc[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) acc[u][j] = (j < a.m && ok[u] && !SET) ? ld2nt(a.y[j] + 2 * (p0 + 64 * u)) : z2;
    if constexpr (SC && !SET) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < M; ++j)
          if (j < a.m) acc[u][j] = sc2<SC>(acc[u][j], scale(a.k + j));  // only a.k + a.m scales exist
    }
    int i = 0;
    for (; i + 4 <= a.k; i += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ok[u] ? ld2nt(a.x[i + b] + 2 * (p0 + 64 * u)) : z2;
      if constexpr (SC) {
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int u = 0; u < U; ++u) xv[b][u] = sc2<SC>(xv[b][u], scale(i + b));
      }
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            const double al = alpha((i + b) * a.m + j);
#pragma unroll
            for (int u = 0; u < U; ++u) {
              acc[u][j].x = fma(al, xv[b][u].x, acc[u][j].x);
              acc[u][j].y = fma(al, xv[b][u].y, acc[u][j].y);
            }
          }
        }
    }
    for (; i < a.k; ++i) {
      double2 xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u] = ok[u] ? ld2nt(a.x[i] + 2 * (p0 + 64 * u)) : z2;
      if constexpr (SC) {
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = sc2<SC>(xv[u], scale(i));
      }
#pragma unroll
      for (int j = 0; j < M; ++j) {
        if (j < a.m) {
          const double al = alpha(i * a.m + j);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(al, xv[u].x, acc[u][j].x);
            acc[u][j].y = fma(al, xv[u].y, acc[u][j].y);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (ok[u])
#pragma unroll
        for (int j = 0; j < M; ++j)
          if (j < a.m) st2nt(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
  }
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x < a.m) {
    const size_t e = a.n - 1;
    const int j = threadIdx.x;
    double v = SET ? 0.0 : sc1<SC>(a.y[j][e], scale(a.k + j));
    for (int i = 0; i < a.k; ++i) v = fma(alpha(i * a.m + j), sc1<SC>(a.x[i][e], scale(i)), v);
    a.y[j][e] = v;
  }
}

// Fused MGS step: y_j += c_j x (the same fma as a one-source gemm_outer),
// then the updated y_j dotted with z, in one pass: R is read and written once instead of being read
// again by the next gemm_inner.  Bytes 8N(2 + 2m).
struct AxpyInnerArgs {
  const double* x;
  const double* z;
  double* y[ssp::kOuterDst];
  double c[ssp::kOuterDst];
  int m;
  size_t n;
  double* partial;     // [gridDim.x][m]
  ssp::FoldTail tail;  // fused fold when tail.counter is set
};

// Window shape (ssp::for_windows, kFusedU KiB per vector per wave visit): x and z are loaded once per
// window, then each destination is read, updated, stored and dotted with z.
constexpr int kFusedU = 4;

template <int M>
__global__ __launch_bounds__(kBlock) void k_axpy_inner(const AxpyInnerArgs a) {
  using ssp::ld2nt;
  using ssp::st2nt;
  double acc[M];
#pragma unroll
  for (int j = 0; j < M; ++j) acc[j] = 0;
  ssp::for_windows<kFusedU>(
      a.n,
      [&](size_t p0) {
        double2 xv[kFusedU], zv[kFusedU];
#pragma unroll
        for (int u = 0; u < kFusedU; ++u) xv[u] = ld2nt(a.x + 2 * (p0 + 64 * u));
#pragma unroll
        for (int u = 0; u < kFusedU; ++u) zv[u] = ld2nt(a.z + 2 * (p0 + 64 * u));
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 y[kFusedU];
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) y[u] = ld2nt(a.y[j] + 2 * (p0 + 64 * u));
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) {
              y[u].x = fma(a.c[j], xv[u].x, y[u].x);
              y[u].y = fma(a.c[j], xv[u].y, y[u].y);
              st2nt(a.y[j] + 2 * (p0 + 64 * u), y[u]);
              acc[j] = fma(y[u].x, zv[u].x, acc[j]);
              acc[j] = fma(y[u].y, zv[u].y, acc[j]);
            }
          }
        }
      },
      [&](size_t p) {
        const double2 xv = ld2(a.x + 2 * p), zv = ld2(a.z + 2 * p);
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 y = ld2(a.y[j] + 2 * p);
            y.x = fma(a.c[j], xv.x, y.x);
            y.y = fma(a.c[j], xv.y, y.y);
            *reinterpret_cast<double2*>(a.y[j] + 2 * p) = y;
            acc[j] = fma(y.x, zv.x, acc[j]);
            acc[j] = fma(y.y, zv.y, acc[j]);
          }
        }
      },
      [&](size_t e) {
        for (int j = 0; j < a.m; ++j) {
          const double y = fma(a.c[j], a.x[e], a.y[j][e]);
          a.y[j][e] = y;
          acc[j] = fma(y, a.z[e], acc[j]);
        }
      });
  __shared__ double red[kBlock / 64][M];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    double v = acc[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave][j] = v;
  }
  __syncthreads();
  if (int(threadIdx.x) < a.m) {
    double s = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
    ssp::store_partial(a.partial + size_t(blockIdx.x) * a.m + threadIdx.x, s);
  }
  if (a.tail.counter) ssp::fold_tail<(M < 8 ? M : 8)>(a.partial, a.tail);
}

// Per-block sums of acc[0..M) over the block's waves into partial[block][m].
template <int M>
__device__ __forceinline__ void block_partials(const double (&acc)[M], int m, double* partial) {
  __shared__ double red[kBlock / 64][M];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    double v = acc[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave][j] = v;
  }
  __syncthreads();
  if (int(threadIdx.x) < m) {
    double s = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
    ssp::store_partial(partial + size_t(blockIdx.x) * m + threadIdx.x, s);
  }
}

// x *= alpha; acc_j += x_scaled * y_j.
struct ScalInnerArgs {
  double* x;
  const double* y[ssp::kOuterDst];
  double alpha;
  int m;
  size_t n;
  double* partial;     // [gridDim.x][m]
  ssp::FoldTail tail;  // fused fold when tail.counter is set
};

template <int M>
__global__ __launch_bounds__(kBlock) void k_scal_inner(const ScalInnerArgs a) {
  using ssp::ld2nt;
  using ssp::st2nt;
  double acc[M];
#pragma unroll
  for (int j = 0; j < M; ++j) acc[j] = 0;
  ssp::for_windows<kFusedU>(
      a.n,
      [&](size_t p0) {
        double2 xv[kFusedU];
#pragma unroll
        for (int u = 0; u < kFusedU; ++u) xv[u] = ld2nt(a.x + 2 * (p0 + 64 * u));
#pragma unroll
        for (int u = 0; u < kFusedU; ++u) {
          xv[u].x *= a.alpha;
          xv[u].y *= a.alpha;
          st2nt(a.x + 2 * (p0 + 64 * u), xv[u]);
        }
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 y[kFusedU];
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) y[u] = ld2nt(a.y[j] + 2 * (p0 + 64 * u));
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) {
              acc[j] = fma(xv[u].x, y[u].x, acc[j]);
              acc[j] = fma(xv[u].y, y[u].y, acc[j]);
            }
          }
        }
      },
      [&](size_t p) {
        double2 xv = ld2(a.x + 2 * p);
        xv.x *= a.alpha;
        xv.y *= a.alpha;
        *reinterpret_cast<double2*>(a.x + 2 * p) = xv;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            const double2 y = ld2(a.y[j] + 2 * p);
            acc[j] = fma(xv.x, y.x, acc[j]);
            acc[j] = fma(xv.y, y.y, acc[j]);
          }
        }
      },
      [&](size_t e) {
        const double xs = a.x[e] * a.alpha;
        a.x[e] = xs;
        for (int j = 0; j < a.m; ++j) acc[j] = fma(xs, a.y[j][e], acc[j]);
      });
  block_partials<M>(acc, a.m, a.partial);
  if (a.tail.counter) ssp::fold_tail<(M < 8 ? M : 8)>(a.partial, a.tail);
}

// y_j += c_j x; acc += y_0_new^2.
template <int M>
__global__ __launch_bounds__(kBlock) void k_axpy_norm(const AxpyInnerArgs a) {
  using ssp::ld2nt;
  using ssp::st2nt;
  double acc[1] = {0};
  ssp::for_windows<kFusedU>(
      a.n,
      [&](size_t p0) {
        double2 xv[kFusedU];
#pragma unroll
        for (int u = 0; u < kFusedU; ++u) xv[u] = ld2nt(a.x + 2 * (p0 + 64 * u));
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 y[kFusedU];
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) y[u] = ld2nt(a.y[j] + 2 * (p0 + 64 * u));
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) {
              y[u].x = fma(a.c[j], xv[u].x, y[u].x);
              y[u].y = fma(a.c[j], xv[u].y, y[u].y);
              st2nt(a.y[j] + 2 * (p0 + 64 * u), y[u]);
              if (j == 0) {
                acc[0] = fma(y[u].x, y[u].x, acc[0]);
                acc[0] = fma(y[u].y, y[u].y, acc[0]);
              }
            }
          }
        }
      },
      [&](size_t p) {
        const double2 xv = ld2(a.x + 2 * p);
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 y = ld2(a.y[j] + 2 * p);
            y.x = fma(a.c[j], xv.x, y.x);
            y.y = fma(a.c[j], xv.y, y.y);
            *reinterpret_cast<double2*>(a.y[j] + 2 * p) = y;
            if (j == 0) {
              acc[0] = fma(y.x, y.x, acc[0]);
              acc[0] = fma(y.y, y.y, acc[0]);
            }
          }
        }
      },
      [&](size_t e) {
        for (int j = 0; j < a.m; ++j) {
          const double y = fma(a.c[j], a.x[e], a.y[j][e]);
          a.y[j][e] = y;
          if (j == 0) acc[0] = fma(y, y, acc[0]);
        }
      });
  block_partials<1>(acc, 1, a.partial);
  if (a.tail.counter) ssp::fold_tail(a.partial, a.tail);
}

// One pass per step of the self-orthonormalisation: x_s = x * xs (the scal's one rounding, stored
// when store_x), y_j += c_j x_s, then the Gram row of the next vector, acc_j += y_0_new * y_j_new.
struct AxpyGramArgs {
  double* x;
  double* y[ssp::kOuterDst];
  double c[ssp::kOuterDst];
  double xs;
  int store_x;
  int m;
  size_t n;
  double* partial;     // [gridDim.x][m]
  ssp::FoldTail tail;  // fused fold when tail.counter is set
};

template <int M>
__global__ __launch_bounds__(kBlock) void k_axpy_gram(const AxpyGramArgs a) {
  using ssp::ld2nt;
  using ssp::st2nt;
  double acc[M];
#pragma unroll
  for (int j = 0; j < M; ++j) acc[j] = 0;
  ssp::for_windows<kFusedU>(
      a.n,
      [&](size_t p0) {
        double2 xv[kFusedU], y0[kFusedU];
#pragma unroll
        for (int u = 0; u < kFusedU; ++u) xv[u] = ld2nt(a.x + 2 * (p0 + 64 * u));
#pragma unroll
        for (int u = 0; u < kFusedU; ++u) {
          xv[u].x *= a.xs;
          xv[u].y *= a.xs;
        }
        if (a.store_x) {
#pragma unroll
          for (int u = 0; u < kFusedU; ++u) st2nt(a.x + 2 * (p0 + 64 * u), xv[u]);
        }
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 y[kFusedU];
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) y[u] = ld2nt(a.y[j] + 2 * (p0 + 64 * u));
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) {
              y[u].x = fma(a.c[j], xv[u].x, y[u].x);
              y[u].y = fma(a.c[j], xv[u].y, y[u].y);
              st2nt(a.y[j] + 2 * (p0 + 64 * u), y[u]);
              if (j == 0) y0[u] = y[u];
              acc[j] = fma(y0[u].x, y[u].x, acc[j]);
              acc[j] = fma(y0[u].y, y[u].y, acc[j]);
            }
          }
        }
      },
      [&](size_t p) {
        double2 xv = ld2(a.x + 2 * p);
        xv.x *= a.xs;
        xv.y *= a.xs;
        if (a.store_x) *reinterpret_cast<double2*>(a.x + 2 * p) = xv;
        double2 y0 = make_double2(0, 0);
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 y = ld2(a.y[j] + 2 * p);
            y.x = fma(a.c[j], xv.x, y.x);
            y.y = fma(a.c[j], xv.y, y.y);
            *reinterpret_cast<double2*>(a.y[j] + 2 * p) = y;
            if (j == 0) y0 = y;
            acc[j] = fma(y0.x, y.x, acc[j]);
            acc[j] = fma(y0.y, y.y, acc[j]);
          }
        }
      },
      [&](size_t e) {
        const double xe = a.x[e] * a.xs;
        if (a.store_x) a.x[e] = xe;
        double y0 = 0;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            const double y = fma(a.c[j], xe, a.y[j][e]);
            a.y[j][e] = y;
            if (j == 0) y0 = y;
            acc[j] = fma(y0, y, acc[j]);
          }
        }
      });
  block_partials<M>(acc, a.m, a.partial);
  if (a.tail.counter) ssp::fold_tail<(M < 8 ? M : 8)>(a.partial, a.tail);
}

// Block transform in place (the block self-orthonormalisation of the new R vectors,
// itsolv_hbm/hbm_handlers.h fused_orthonormalise): x_j <- sum_{i<m} t(i,j) (s_i x_i), every output of a
// position formed from that position's loaded inputs before any is stored, so the destinations are
// the sources.  FMA: the sum by fused multiply-adds in order i = 0..m-1; without, each product rounded
// before its add (the short-vector arithmetic).  GRAM: the M(M+1)/2 dots <x_a', x_b'> (a <= b, row by
// row) of the stored outputs, folded per launch.
struct TransformArgs {
  double* x[ssp::kOuterDst];
  double s[ssp::kOuterDst];                     // deferred input scales
  double t[ssp::kOuterDst * ssp::kOuterDst];    // transposed: t[j * m + i] = t(i, j)
  int m;
  size_t n;
  double* partial;     // [gridDim.x][M (M + 1) / 2]
  ssp::FoldTail tail;  // GRAM: fused fold
};
static_assert(sizeof(TransformArgs) <= 4000, "kernel argument block too large");

template <bool FMA>
__device__ __forceinline__ double tmul(double t, double x, double acc) {
#pragma clang fp contract(off)
  if constexpr (FMA) return fma(t, x, acc);
  return acc + t * x;  // the product rounded before the add
}

// Coefficient column j (t(0..M-1, j), contiguous in the transposed layout), read from the kernel-argument
// segment where it is used.  The 64 coefficients of an 8-vector transform are more than the SGPR file
// holds beside the pointers; left to itself the compiler keeps them in VGPR lanes and re-reads every one
// with two v_readlane per fma (2576 readlanes in the 8-vector window loop, against 256 fmas).  The empty
// asm makes the segment pointer opaque at each column, so the column is fetched by s_load_dwordx16 right
// before its fmas (kept in SGPRs, used as scalar operands) and dies after them: no readlanes, 385 instead
// of 2957 instructions per window loop.  TransformArgs is the kernel's only argument (offset 0).
typedef const __attribute__((address_space(4))) double* kernarg_dp;
template <int M>
__device__ __forceinline__ kernarg_dp transform_column(int j) {
  kernarg_dp tp = (kernarg_dp)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() +
                               offsetof(TransformArgs, t));
  asm volatile("" : "+s"(tp));
  return tp + j * M;
}

// M = m exactly (instantiated for m = 1..8): no per-vector branch in the streaming loop.  DOTS: 0 none,
// 1 the M self-dots <x_j', x_j'> (accumulated as each output is formed), 2 the M(M+1)/2 pair dots.
// WIDE: twice the window for M > 4 -- more bytes in flight per lane at two waves per SIMD instead of
// three.  Used for the self-dot instance (DOTS = 1; SSP_TRANSFORM_WIDE=0 turns it off, per context):
// on the same vectors 4989 -> 5276 GB/s at 1.25e7 elements and 5285 -> 5626 at 1e8, while the Gram
// instance lost (5147 -> 5028, 5511 -> 5074; profiles/r6/ab_transform_wide/).
template <int M, int DOTS, bool FMA, bool WIDE = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WIDE ? 2 : 3))) void k_transform(const TransformArgs a) {
  using ssp::ld2nt;
  using ssp::st2nt;
  constexpr bool GRAM = DOTS == 2, NORM = DOTS == 1;
  constexpr int NP = M * (M + 1) / 2;
  constexpr int NA = GRAM ? NP : (NORM ? M : 1);
  // GRAM keeps every output of the window for the pair dots
  constexpr int U = GRAM ? (WIDE ? 2 : 1) : (M <= 4 ? 4 : (WIDE ? 4 : 2));
  double acc[NA];
#pragma unroll
  for (int q = 0; q < NA; ++q) acc[q] = 0;
  auto pairs = [&](const double (&y)[M]) {
    if constexpr (GRAM) {
      int q = 0;
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = i; j < M; ++j) {
          acc[q] = fma(y[i], y[j], acc[q]);
          ++q;
        }
    }
  };
  // Output j of every position of the window is formed and stored with column j's coefficients, then
  // column j + 1 (the GRAM instance keeps the window's outputs for the pair dots).
  ssp::for_windows<U>(
      a.n,
      [&](size_t p0) {
        double2 xv[U][M];
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int u = 0; u < U; ++u) xv[u][i] = sc2<true>(ld2nt(a.x[i] + 2 * (p0 + 64 * u)), a.s[i]);
        double ylo[U][M], yhi[U][M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const kernarg_dp tc = transform_column<M>(j);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            double vl = 0, vh = 0;
#pragma unroll
            for (int i = 0; i < M; ++i) {
              vl = tmul<FMA>(tc[i], xv[u][i].x, vl);
              vh = tmul<FMA>(tc[i], xv[u][i].y, vh);
            }
            st2nt(a.x[j] + 2 * (p0 + 64 * u), make_double2(vl, vh));
            ylo[u][j] = vl;
            yhi[u][j] = vh;
            if constexpr (NORM) {
              acc[j] = fma(vl, vl, acc[j]);
              acc[j] = fma(vh, vh, acc[j]);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          pairs(ylo[u]);
          pairs(yhi[u]);
        }
      },
      [&](size_t p) {
        double2 xv[M];
#pragma unroll
        for (int i = 0; i < M; ++i) xv[i] = sc2<true>(ld2(a.x[i] + 2 * p), a.s[i]);
        double ylo[M], yhi[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const kernarg_dp tc = transform_column<M>(j);
          double vl = 0, vh = 0;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            vl = tmul<FMA>(tc[i], xv[i].x, vl);
            vh = tmul<FMA>(tc[i], xv[i].y, vh);
          }
          *reinterpret_cast<double2*>(a.x[j] + 2 * p) = make_double2(vl, vh);
          ylo[j] = vl;
          yhi[j] = vh;
          if constexpr (NORM) {
            acc[j] = fma(vl, vl, acc[j]);
            acc[j] = fma(vh, vh, acc[j]);
          }
        }
        pairs(ylo);
        pairs(yhi);
      },
      [&](size_t e) {
        double x1[M], y1[M];
#pragma unroll
        for (int i = 0; i < M; ++i) x1[i] = a.x[i][e] * a.s[i];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const kernarg_dp tc = transform_column<M>(j);
          double v = 0;
#pragma unroll
          for (int i = 0; i < M; ++i) v = tmul<FMA>(tc[i], x1[i], v);
          a.x[j][e] = v;
          y1[j] = v;
          if constexpr (NORM) acc[j] = fma(v, v, acc[j]);
        }
        pairs(y1);
      });
  if constexpr (GRAM) {
    block_partials<NP>(acc, NP, a.partial);
    // one load trip per 8 outputs (M >= 7: up to 2048 workgroups; else up to 1024, launch_transform)
    if (a.tail.counter) ssp::fold_tail<(NP < 8 ? NP : 8), (M >= 7 ? 8 : 4)>(a.partial, a.tail);
  } else if constexpr (NORM) {
    block_partials<M>(acc, M, a.partial);
    if (a.tail.counter) ssp::fold_tail<M, 4>(a.partial, a.tail);  // two trips at 2048 workgroups
  }
}

// The fused-Gram instance runs one resident round of workgroups (its occupancy per CU, at most 4):
// each workgroup streams an equal share, and the last arriver folds the few partials in one load
// trip per 8 outputs (fold_tail<8, 4>) -- with 8 workgroups per CU the fold of the 36 dots took
// 20 dependent trips, 70 us of a 340 us launch at the C4 shard.
template <int M>
unsigned gram_grid(ssp_ctx* ctx, size_t n) {
  // resident workgroups per CU of k_transform<M, 2, true> (thread-safe one-time initialisation)
  static const int per_cu = [] {
    if (const char* e = std::getenv("SSP_GRAM_WG_PER_CU")) return std::max(1, std::min(8, std::atoi(e)));  // A/B
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_transform<M, 2, true>, kBlock, 0) != hipSuccess || occ < 1)
      occ = 2;
    return occ < 4 ? occ : 4;
  }();
  return ssp::win_grid(ctx, n, 1, unsigned(per_cu));
}

template <int M>
void launch_transform_m(ssp_ctx* ctx, unsigned grid, const TransformArgs& a, int dots, bool exact, bool pass) {
  const dim3 b(kBlock);
  if constexpr (M > 4) {
    if (ctx->transform_wide && !exact && dots == 1) {
      SSP_LAUNCH((k_transform<M, 1, true, true>), dim3(grid), b, 0, ctx->stream, a);
      return;
    }
  }
  if (exact) SSP_LAUNCH((k_transform<M, 0, false>), dim3(grid), b, 0, ctx->stream, a);
  else if (dots == 2)
    SSP_LAUNCH((k_transform<M, 2, true>), dim3(pass ? grid : gram_grid<M>(ctx, a.n)), b, 0, ctx->stream, a);
  else if (dots == 1) SSP_LAUNCH((k_transform<M, 1, true>), dim3(grid), b, 0, ctx->stream, a);
  else SSP_LAUNCH((k_transform<M, 0, true>), dim3(grid), b, 0, ctx->stream, a);
}

// The pair dots of the fused-Gram transform: by a reduce pass after the kernel (full streaming grid,
// one workgroup per dot) unless SSP_GRAM_FOLD=kernel (the last arriver folds them, one resident round
// of workgroups: gram_grid).  A/B switch, read once.
bool gram_reduce_pass() {
  static const bool v = [] {
    const char* e = std::getenv("SSP_GRAM_FOLD");
    return !(e && std::string(e) == "kernel");
  }();
  return v;
}

void launch_transform(ssp_ctx* ctx, int m, unsigned grid, const TransformArgs& a, int dots, bool exact, bool pass) {
  switch (m) {
    case 1: return launch_transform_m<1>(ctx, grid, a, dots, exact, pass);
    case 2: return launch_transform_m<2>(ctx, grid, a, dots, exact, pass);
    case 3: return launch_transform_m<3>(ctx, grid, a, dots, exact, pass);
    case 4: return launch_transform_m<4>(ctx, grid, a, dots, exact, pass);
    case 5: return launch_transform_m<5>(ctx, grid, a, dots, exact, pass);
    case 6: return launch_transform_m<6>(ctx, grid, a, dots, exact, pass);
    case 7: return launch_transform_m<7>(ctx, grid, a, dots, exact, pass);
    default: return launch_transform_m<8>(ctx, grid, a, dots, exact, pass);
  }
}

// The Davidson preconditioner with the self-dots of its outputs (precondition_default, reference
// IterativeSolver.h:52-53, followed by the normalisation of the new R vectors, propose_rspace.h:17-28):
// a_v <- a_v / ((d - shift_v) + 1e-15), element for element k_precondition's operations, and
// acc_v += a_v'^2 in the same pass.  M vectors per launch (compile-time bound, nvec <= M).
struct PrecNormArgs {
  double* a[ssp::kOuterDst];
  double shift[ssp::kOuterDst];
  const double* d;
  int nvec;
  size_t n;
  double* partial;     // [gridDim.x][nvec]
  ssp::FoldTail tail;  // fused fold when tail.counter is set
};

template <int M>
__global__ __launch_bounds__(kBlock) void k_precondition_norms(const PrecNormArgs p) {
  using ssp::ld2nt;
  using ssp::st2nt;
  constexpr int U = 4;
  double acc[M];
#pragma unroll
  for (int v = 0; v < M; ++v) acc[v] = 0;
  ssp::for_windows<U>(
      p.n,
      [&](size_t p0) {
        double2 dv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) dv[u] = ld2nt(p.d + 2 * (p0 + 64 * u));
#pragma unroll
        for (int v = 0; v < M; ++v) {
          if (v < p.nvec) {
            double2 av[U];
#pragma unroll
            for (int u = 0; u < U; ++u) av[u] = ld2nt(p.a[v] + 2 * (p0 + 64 * u));
#pragma unroll
            for (int u = 0; u < U; ++u) {
              av[u].x = av[u].x / (dv[u].x - p.shift[v] + 1e-15);
              av[u].y = av[u].y / (dv[u].y - p.shift[v] + 1e-15);
              st2nt(p.a[v] + 2 * (p0 + 64 * u), av[u]);
              acc[v] = fma(av[u].x, av[u].x, acc[v]);
              acc[v] = fma(av[u].y, av[u].y, acc[v]);
            }
          }
        }
      },
      [&](size_t i) {
        const double2 dv = ld2(p.d + 2 * i);
#pragma unroll
        for (int v = 0; v < M; ++v) {
          if (v < p.nvec) {
            double2 av = ld2(p.a[v] + 2 * i);
            av.x = av.x / (dv.x - p.shift[v] + 1e-15);
            av.y = av.y / (dv.y - p.shift[v] + 1e-15);
            *reinterpret_cast<double2*>(p.a[v] + 2 * i) = av;
            acc[v] = fma(av.x, av.x, acc[v]);
            acc[v] = fma(av.y, av.y, acc[v]);
          }
        }
      },
      [&](size_t j) {
#pragma unroll
        for (int v = 0; v < M; ++v) {
          if (v < p.nvec) {
            const double a = p.a[v][j] / (p.d[j] - p.shift[v] + 1e-15);
            p.a[v][j] = a;
            acc[v] = fma(a, a, acc[v]);
          }
        }
      });
  block_partials<M>(acc, p.nvec, p.partial);
  if (p.tail.counter) ssp::fold_tail<(M < 8 ? M : 8)>(p.partial, p.tail);
}

// Residuals and their norms in one pass (construct_residual + update_errors, reference
// LinearEigensystemDavidson.h:186-192 and IterativeSolverTemplate.h:95-102): y_j = y_j s^y_j +
// c_j (x_j s^x_j) -- ssp_axpy_scaled's fma, element for element -- then acc_j += y_j^2.
struct AxpyPairsArgs {
  const double* x[ssp::kOuterDst];
  double* y[ssp::kOuterDst];
  double c[ssp::kOuterDst];
  double xs[ssp::kOuterDst];
  double ys[ssp::kOuterDst];
  int m;
  size_t n;
  double* partial;     // [gridDim.x][m]
  ssp::FoldTail tail;  // fused fold when tail.counter is set
};

template <int M>
__global__ __launch_bounds__(kBlock) void k_axpy_pairs_norm(const AxpyPairsArgs a) {
  using ssp::ld2nt;
  using ssp::st2nt;
  double acc[M];
#pragma unroll
  for (int j = 0; j < M; ++j) acc[j] = 0;
  ssp::for_windows<kFusedU>(
      a.n,
      [&](size_t p0) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            double2 xv[kFusedU], yv[kFusedU];
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) xv[u] = sc2<true>(ld2nt(a.x[j] + 2 * (p0 + 64 * u)), a.xs[j]);
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) yv[u] = sc2<true>(ld2nt(a.y[j] + 2 * (p0 + 64 * u)), a.ys[j]);
#pragma unroll
            for (int u = 0; u < kFusedU; ++u) {
              const double2 r = make_double2(fma(a.c[j], xv[u].x, yv[u].x), fma(a.c[j], xv[u].y, yv[u].y));
              st2nt(a.y[j] + 2 * (p0 + 64 * u), r);
              acc[j] = fma(r.x, r.x, acc[j]);
              acc[j] = fma(r.y, r.y, acc[j]);
            }
          }
        }
      },
      [&](size_t p) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            const double2 xv = sc2<true>(ld2(a.x[j] + 2 * p), a.xs[j]), yv = sc2<true>(ld2(a.y[j] + 2 * p), a.ys[j]);
            const double2 r = make_double2(fma(a.c[j], xv.x, yv.x), fma(a.c[j], xv.y, yv.y));
            *reinterpret_cast<double2*>(a.y[j] + 2 * p) = r;
            acc[j] = fma(r.x, r.x, acc[j]);
            acc[j] = fma(r.y, r.y, acc[j]);
          }
        }
      },
      [&](size_t e) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j < a.m) {
            const double r = fma(a.c[j], sc1<true>(a.x[j][e], a.xs[j]), sc1<true>(a.y[j][e], a.ys[j]));
            a.y[j][e] = r;
            acc[j] = fma(r, r, acc[j]);
          }
        }
      });
  block_partials<M>(acc, a.m, a.partial);
  if (a.tail.counter) ssp::fold_tail<(M < 8 ? M : 8)>(a.partial, a.tail);
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

// Column groups per launch for MG row groups (accumulator registers: MG * NG doubles per lane):
// 16 (64 columns, the launch maximum) for every row-group count, so one launch reads every vector
// once (tools/mb_inner.hip: 16 x 64 at 5.9 TB/s in one launch against 4.3 TB/s in three).
constexpr int ng_max(int) { return 16; }

// Workgroups per gemm_inner launch: 4 per CU (16 waves) when n allows, else one wave per chunk.
// 8 per CU measures the same (tools/ab_inner.py, profiles/r1/ab_inner.txt); the nontemporal loads
// of the main loop gain 3 % over plain ones on the same vectors, with bit-identical results.
unsigned inner_grid(const ssp_ctx* ctx, size_t n) {
  const size_t chunks = n / 32 + 1;
  const size_t blocks = (chunks + 3) / 4;
  const size_t cap = size_t(ctx->num_cus) * size_t(ctx->inner_per_cu);
  return unsigned(std::max<size_t>(1, std::min(blocks, cap)));
}

// Two-stage loads (k_gemm_inner PIPE) for the small panels (at most 8 accumulator tiles, and the
// symmetric ones), whose second register stage still leaves >= 2 waves per SIMD.  SSP_INNER_PIPE:
// 0 off, 1 (default) small panels, 2 also up to 16 tiles (A/B knob, read once).
int inner_pipe_level() {
  static const int v = [] {
    const char* e = std::getenv("SSP_INNER_PIPE");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}
template <int MG, int NG, bool SYM, bool SC>
constexpr int inner_pipe_min_level() {
  return (SYM || MG * NG <= 8) ? 1 : (MG * NG <= 16 ? 2 : 99);
}

template <int MG, int NG, bool SC, bool PRE>
void launch_inner_tp(ssp_ctx* ctx, unsigned grid, const InnerArgs& a) {
  if constexpr (inner_pipe_min_level<MG, NG, false, SC>() < 99) {
    if (inner_pipe_level() >= inner_pipe_min_level<MG, NG, false, SC>()) {
      SSP_LAUNCH((k_gemm_inner<MG, NG, false, SC, true, PRE>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
      return;
    }
  }
  SSP_LAUNCH((k_gemm_inner<MG, NG, false, SC, false, PRE>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
}

// pre: the column-prefix form (k_gemm_inner PRE), instantiated for MG <= 2 (up to 8 rows, the
// solvers' working sets)
template <int MG, int NG, bool SC>
void launch_inner_t(ssp_ctx* ctx, unsigned grid, const InnerArgs& a, bool pre) {
  if constexpr (MG <= 2 && NG >= MG) {
    if (pre) return launch_inner_tp<MG, NG, SC, true>(ctx, grid, a);
  }
  launch_inner_tp<MG, NG, SC, false>(ctx, grid, a);
}

// Smallest instantiated NG >= need (need <= ng_max(MG)).
template <int MG, bool SC>
int launch_inner_mg(ssp_ctx* ctx, unsigned grid, const InnerArgs& a, int need, bool pre) {
  if (need <= 1) launch_inner_t<MG, 1, SC>(ctx, grid, a, pre);
  else if (need <= 2) launch_inner_t<MG, 2, SC>(ctx, grid, a, pre);
  else if (need <= 3) launch_inner_t<MG, 3, SC>(ctx, grid, a, pre);
  else if (need <= 4) launch_inner_t<MG, 4, SC>(ctx, grid, a, pre);
  else if (need <= 6) launch_inner_t<MG, 6, SC>(ctx, grid, a, pre);
  else if constexpr (ng_max(MG) >= 8) {
    if (need <= 8) launch_inner_t<MG, 8, SC>(ctx, grid, a, pre);
    else if constexpr (ng_max(MG) >= 12) {
      if (need <= 12) launch_inner_t<MG, 12, SC>(ctx, grid, a, pre);
      else if constexpr (ng_max(MG) >= 16) launch_inner_t<MG, 16, SC>(ctx, grid, a, pre);
    }
  }
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

template <int G, bool SC>
void launch_inner_sym_g(ssp_ctx* ctx, const InnerArgs& a, unsigned grid) {
  if (inner_pipe_level() >= 1)
    SSP_LAUNCH((k_gemm_inner<G, G, true, SC, true>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else
    SSP_LAUNCH((k_gemm_inner<G, G, true, SC>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
}

template <bool SC>
int launch_inner_sym_t(ssp_ctx* ctx, const InnerArgs& a, unsigned grid) {
  switch ((a.m + 3) / 4) {
    case 1: launch_inner_sym_g<1, SC>(ctx, a, grid); break;
    case 2: launch_inner_sym_g<2, SC>(ctx, a, grid); break;
    case 3: launch_inner_sym_g<3, SC>(ctx, a, grid); break;
    default: launch_inner_sym_g<4, SC>(ctx, a, grid); break;
  }
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int launch_inner_sym(ssp_ctx* ctx, const InnerArgs& a, unsigned grid, bool sc) {
  return sc ? launch_inner_sym_t<true>(ctx, a, grid) : launch_inner_sym_t<false>(ctx, a, grid);
}

template <bool SC>
int launch_inner_sc(ssp_ctx* ctx, const InnerArgs& a, unsigned grid, bool pre) {
  const int mg = (a.m + 3) / 4, need = (a.k + 3) / 4;
  switch (mg) {
    case 1: return launch_inner_mg<1, SC>(ctx, grid, a, need, pre);
    case 2: return launch_inner_mg<2, SC>(ctx, grid, a, need, pre);
    case 3: return launch_inner_mg<3, SC>(ctx, grid, a, need, false);
    default: return launch_inner_mg<4, SC>(ctx, grid, a, need, false);
  }
}

int launch_inner(ssp_ctx* ctx, const InnerArgs& a, unsigned grid, bool sc, bool pre = false) {
  return sc ? launch_inner_sc<true>(ctx, a, grid, pre) : launch_inner_sc<false>(ctx, a, grid, pre);
}

template <bool DEV, bool SET, bool SC>
void launch_outer_t(ssp_ctx* ctx, unsigned grid, const OuterArgs& a) {
  if (a.m <= 1)
    SSP_LAUNCH((k_gemm_outer<1, DEV, SET, SC>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else if (a.m <= 2)
    SSP_LAUNCH((k_gemm_outer<2, DEV, SET, SC>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else if (a.m <= 4)
    SSP_LAUNCH((k_gemm_outer<4, DEV, SET, SC>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else if (a.m <= 8)
    SSP_LAUNCH((k_gemm_outer<8, DEV, SET, SC>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
  else
    SSP_LAUNCH((k_gemm_outer<16, DEV, SET, SC>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
}

template <bool SC>
void launch_outer_sc(ssp_ctx* ctx, unsigned grid, const OuterArgs& a) {
  if (a.alpha_dev)
    a.set ? launch_outer_t<true, true, SC>(ctx, grid, a) : launch_outer_t<true, false, SC>(ctx, grid, a);
  else
    a.set ? launch_outer_t<false, true, SC>(ctx, grid, a) : launch_outer_t<false, false, SC>(ctx, grid, a);
}

int launch_outer(ssp_ctx* ctx, const OuterArgs& a) {
  // workgroups per CU of the launch: ctx->outer_per_cu (SSP_OUTER_WG_PER_CU at context creation)
  const unsigned grid = ssp::stream_grid(ctx, a.n / 2 + 1, kOuterWin, unsigned(ctx->outer_per_cu));
  a.scale_dev ? launch_outer_sc<true>(ctx, grid, a) : launch_outer_sc<false>(ctx, grid, a);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

// SSP_LEDGER_DETAIL tags: the kernel instance and the panel's shape
int ng_inst(int need) { return need <= 4 ? need : need <= 6 ? 6 : need <= 8 ? 8 : need <= 12 ? 12 : 16; }
std::string shape_tag(const char* kind, int a, int b, int c, int d, bool sc) {
  char t[96];
  std::snprintf(t, sizeof(t), "%s<%d,%d> %dx%d%s", kind, a, b, c, d, sc ? " sc" : "");
  return t;
}

bool any_scaled(const double* s, int n) {
  for (int i = 0; s && i < n; ++i)
    if (s[i] != 1.0) return true;
  return false;
}

}  // namespace

extern "C" {

int ssp_gemm_inner(ssp_ctx* ctx, const double* const* xx, int m, const double* const* yy, int k, size_t n,
                   double* out) {
  return ssp_gemm_inner_scaled(ctx, xx, nullptr, m, yy, nullptr, k, n, out);
}

int ssp_gemm_inner_scaled(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, const double* const* yy,
                          const double* ys, int k, size_t n, double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 0 || k < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner: negative dimension");
  if (m * k > 0 && !out) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_inner: null out");
  if (m == 0 || k == 0) return SSP_OK;
  SSP_TRY(check_ptrs(xx, m, n, "ssp_gemm_inner"));
  SSP_TRY(check_ptrs(yy, k, n, "ssp_gemm_inner"));
  // Put the shorter side on the MFMA rows (groups of 4, at most 16 per launch), the longer on the columns.
  const bool swap = m > k;
  const double* const* rows = swap ? yy : xx;
  const double* const* cols = swap ? xx : yy;
  const int R = swap ? k : m, C = swap ? m : k;
  // deferred scales (null: all 1), following the swap
  std::vector<double> rs(size_t(R), 1.0), cs(size_t(C), 1.0);
  for (int i = 0; i < m; ++i) (swap ? cs : rs)[size_t(i)] = xs ? xs[i] : 1.0;
  for (int j = 0; j < k; ++j) (swap ? rs : cs)[size_t(j)] = ys ? ys[j] : 1.0;
  const bool sc = any_scaled(rs.data(), R) || any_scaled(cs.data(), C);
  // Column prefix (k_gemm_inner PRE): when the first R columns are the rows themselves (the batched
  // overlap rows [params, actions, Q, ...] against params), the panel takes them from the row
  // registers.  The columns are laid out with 4 ceil(R / 4) - R padding columns after that prefix
  // (computed, never read back), in every branch below, so that every rank reduces the same count
  // whichever branch its shard length takes.
  int pad = -1;
  if (R <= 8 && C > R && !(R == 1 && C <= 2)) {
    bool pre = true;
    for (int i = 0; pre && i < R; ++i) pre = cols[i] == rows[i] && cs[size_t(i)] == rs[size_t(i)];
    if (pre) pad = 4 * ((R + 3) / 4) - R;
  }
  std::vector<const double*> cols_pad;
  if (pad >= 0) {
    cols_pad.assign(cols, cols + R);
    cols_pad.insert(cols_pad.end(), size_t(pad), rows[0]);
    cols_pad.insert(cols_pad.end(), cols + R, cols + C);
    cs.insert(cs.begin() + R, size_t(pad), 1.0);
    cols = cols_pad.data();
  }
  const int C2 = pad >= 0 ? C + pad : C;  // columns as launched and reduced
  const size_t total = size_t(R) * C2;
  ssp::FoldTail tail{};
  if (ssp::exact_mode(ctx, n)) {
    // The reference's sequential dots (each the same number whichever operand is the row), in the
    // R x C layout of the bandwidth kernels below: with a communicator attached the ranks' results are
    // summed element for element, and a rank whose shard is one element longer may take the other
    // branch (shards of spread_remainder differ by one; ssp_ctx_set_exact_max).
    SSP_TRY(ssp::fold_begin(ctx, int(total), &tail));
    std::vector<const double*> distinct(xx, xx + m);
    distinct.insert(distinct.end(), yy, yy + k);
    std::sort(distinct.begin(), distinct.end());
    const double nvec = double(std::unique(distinct.begin(), distinct.end()) - distinct.begin());
    ssp::LedgerScope ls(ctx, "gemm_inner", 8.0 * n * nvec);
    SSP_TRY(ssp::exact_inner(ctx, rows, rs.data(), R, cols, cs.data(), C2, n, false, tail));
  } else {
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
      // 1 x 1 and 1 x 2 panels (rows = the shorter side): VALU row kernel.
      if (R == 1 && C <= 2) {
        InnerArgs a{};
        a.m = 1;
        a.k = C;
        a.n = n;
        a.x[0] = rows[0];
        a.xs[0] = rs[0];
        for (int j = 0; j < C; ++j) {
          a.y[j] = cols[j];
          a.ys[j] = cs[size_t(j)];
        }
        const bool stride = ctx->row_stride;
        const unsigned grid = stride ? ssp::stream_grid(ctx, n / 2 + 1, 4) : ssp::win_grid(ctx, n, 4, 8);
        SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * C));
        a.partial = ctx->partial;
        SSP_TRY(ssp::fold_begin(ctx, C, &tail));
        a.tail = tail;
        const dim3 g(grid), b(kBlock);
        if (stride) {
          if (C == 1 && sc) SSP_LAUNCH((k_gemm_inner_row<1, true>), g, b, 0, ctx->stream, a);
          else if (C == 1) SSP_LAUNCH((k_gemm_inner_row<1>), g, b, 0, ctx->stream, a);
          else if (sc) SSP_LAUNCH((k_gemm_inner_row<2, true>), g, b, 0, ctx->stream, a);
          else SSP_LAUNCH((k_gemm_inner_row<2>), g, b, 0, ctx->stream, a);
        } else {
          if (C == 1 && sc) SSP_LAUNCH((k_gemm_inner_row_win<1, true>), g, b, 0, ctx->stream, a);
          else if (C == 1) SSP_LAUNCH((k_gemm_inner_row_win<1>), g, b, 0, ctx->stream, a);
          else if (sc) SSP_LAUNCH((k_gemm_inner_row_win<2, true>), g, b, 0, ctx->stream, a);
          else SSP_LAUNCH((k_gemm_inner_row_win<2>), g, b, 0, ctx->stream, a);
        }
        SSP_TRY_HIP(hipGetLastError());
      }
      // A symmetric overlap <xx_i, xx_j> of up to 16 vectors: one panel that loads each vector once.
      bool sym = m == k && m <= ssp::kInnerRows && !(R == 1 && C <= 2);
      for (int i = 0; sym && i < m; ++i) sym = xx[i] == yy[i] && rs[size_t(i)] == cs[size_t(i)];
      // MFMA panels: with one rank the reduce passes publish to the host themselves (fold_begin's host
      // tail; with a communicator it names result_dev and fold_finish exchanges as reduce_fetch did)
      if (!(R == 1 && C <= 2)) SSP_TRY(ssp::fold_begin(ctx, int(total), &tail));
      if (sym) {
        InnerArgs a{};
        a.m = a.k = m;
        a.n = n;
        for (int i = 0; i < m; ++i) {
          a.x[i] = a.y[i] = xx[i];
          a.xs[i] = a.ys[i] = rs[size_t(i)];
        }
        const unsigned grid = inner_grid(ctx, n);
        SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * m * m));
        a.partial = ctx->partial;
        ls.detail(shape_tag("sym", (m + 3) / 4, (m + 3) / 4, m, m, sc));
        SSP_TRY(launch_inner_sym(ctx, a, grid, sc));
        SSP_TRY(ssp::launch_reduce_partials(ctx, ctx->partial, int(grid), m, m, ctx->result_dev, m, 0, 0, &tail, true));
      }
      for (int r0 = 0; !sym && !(R == 1 && C <= 2) && r0 < R; r0 += ssp::kInnerRows) {
        const int mr = std::min(ssp::kInnerRows, R - r0);
        const int cols_per_launch = 4 * ng_max((mr + 3) / 4);
        for (int c0 = 0; c0 < C2; c0 += cols_per_launch) {
          InnerArgs a{};
          a.m = mr;
          a.k = std::min(cols_per_launch, C2 - c0);
          a.n = n;
          for (int i = 0; i < a.m; ++i) {
            a.x[i] = rows[r0 + i];
            a.xs[i] = rs[size_t(r0 + i)];
          }
          for (int j = 0; j < a.k; ++j) {
            a.y[j] = cols[c0 + j];
            a.ys[j] = cs[size_t(c0 + j)];
          }
          const bool sc_launch = any_scaled(a.xs, a.m) || any_scaled(a.ys, a.k);
          const unsigned grid = inner_grid(ctx, n);
          SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * a.m * a.k));
          a.partial = ctx->partial;
          const bool pre = pad >= 0 && c0 == 0;
          if (r0 == 0 && c0 == 0)
            ls.detail(shape_tag(pre ? "mfma-pre" : "mfma", (a.m + 3) / 4, ng_inst((a.k + 3) / 4), a.m, a.k, sc_launch));
          SSP_TRY(launch_inner(ctx, a, grid, sc_launch, pre));
          const bool last = r0 + ssp::kInnerRows >= R && c0 + cols_per_launch >= C2;
          SSP_TRY(ssp::launch_reduce_partials(ctx, ctx->partial, int(grid), a.m, a.k, ctx->result_dev, C2, r0, c0, &tail,
                                              last));
        }
      }
    }
  }
  std::vector<double> t(swap || pad >= 0 ? total : 0);
  double* dst = swap || pad >= 0 ? t.data() : out;
  if (tail.counter) {
    SSP_TRY(ssp::fold_finish(ctx, tail, dst));
  } else {
    SSP_TRY(ssp::reduce_fetch(ctx, dst, total));
  }
  if (pad >= 0) {  // drop the padding columns: R x C2 -> R x C (row-major)
    for (int i = 0; i < R; ++i)
      for (int j = 0; j < C; ++j) t[size_t(i) * C + j] = t[size_t(i) * C2 + (j < R ? j : j + pad)];
    if (!swap) {
      std::copy(t.begin(), t.begin() + long(size_t(R) * C), out);
      return SSP_OK;
    }
  }
  if (!swap) return SSP_OK;
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) out[size_t(i) * k + j] = t[size_t(j) * m + i];
  return SSP_OK;
}

}  // extern "C"

namespace {
int gemm_outer_impl(ssp_ctx* ctx, const double* alphas, const double* const* xx, const double* xs, int k,
                    double* const* yy, const double* ys, int m, size_t n, bool set) {
  SSP_CHECK_CTX(ctx);
  if (m < 0 || k < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer: negative dimension");
  if (set && k == 0) {
    for (int j = 0; j < m; ++j) SSP_TRY(ssp_fill(ctx, 0.0, yy[j], n));
    return SSP_OK;
  }
  if (m == 0 || n == 0) return SSP_OK;
  if (k == 0) {  // no sources: the destinations' deferred scales still have to be stored
    for (int j = 0; j < m; ++j)
      if (!set && ys && ys[j] != 1.0) SSP_TRY(ssp_scal(ctx, ys[j], yy[j], n));
    return SSP_OK;
  }
  if (!alphas) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer: null alphas");
  SSP_TRY(check_ptrs(xx, k, n, "ssp_gemm_outer"));
  SSP_TRY(check_ptrs(const_cast<const double* const*>(yy), m, n, "ssp_gemm_outer"));
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < k; ++i)
      if (yy[j] == xx[i]) return ssp::set_error(SSP_ERR_ARG, "ssp_gemm_outer: a destination aliases a source");
  // Destinations are independent; sources are applied in increasing order, in groups that fit
  // the kernel argument block, so each destination sees the reference's summation order.
  ssp::LedgerScope ls(ctx, set ? "gemm_outer_set" : "gemm_outer", 8.0 * n * (k + (set ? 1.0 : 2.0) * m));
  if (ssp::exact_mode(ctx, n)) return ssp::exact_outer(ctx, alphas, xx, xs, k, yy, ys, m, n, set);
  for (int j0 = 0; j0 < m; j0 += ssp::kOuterDst) {
    const int mm = std::min(ssp::kOuterDst, m - j0);
    // Up to kOuterSrc sources per launch; their alphas ride in the argument block when they fit,
    // else in device memory (one upload), so every destination is read and written once per
    // kOuterSrc sources.
    for (int i0 = 0; i0 < k; i0 += ssp::kOuterSrc) {
      OuterArgs a{};
      a.m = mm;
      a.k = std::min(ssp::kOuterSrc, k - i0);
      a.set = (set && i0 == 0) ? 1 : 0;
      a.n = n;
      for (int i = 0; i < a.k; ++i) a.x[i] = xx[i0 + i];
      for (int j = 0; j < mm; ++j) a.y[j] = yy[j0 + j];
      // deferred scales: every source's; the destinations' on their first read only (i0 == 0)
      std::vector<double> scl(size_t(a.k + mm), 1.0);
      for (int i = 0; i < a.k; ++i) scl[size_t(i)] = xs ? xs[i0 + i] : 1.0;
      for (int j = 0; j < mm; ++j) scl[size_t(a.k + j)] = (ys && i0 == 0 && !set) ? ys[j0 + j] : 1.0;
      if (any_scaled(scl.data(), int(scl.size()))) {
        void* ps;
        SSP_TRY(ssp::upload_small(ctx, scl.data(), scl.size() * sizeof(double), &ps));
        a.scale_dev = static_cast<const double*>(ps);
      }
      const bool dev = a.k * mm > ssp::kOuterAlpha;
      std::vector<double> block(dev ? size_t(a.k) * mm : 0);
      double* dst = dev ? block.data() : a.alpha;
      for (int i = 0; i < a.k; ++i)
        for (int j = 0; j < mm; ++j) dst[i * mm + j] = alphas[size_t(i0 + i) * m + j0 + j];
      if (dev) {
        void* p;
        SSP_TRY(ssp::upload_small(ctx, block.data(), block.size() * sizeof(double), &p));
        a.alpha_dev = static_cast<const double*>(p);
      }
      SSP_TRY(ssp::flush_uploads(ctx));
      if (j0 == 0 && i0 == 0) {
        const int mi = a.m <= 1 ? 1 : a.m <= 2 ? 2 : a.m <= 4 ? 4 : a.m <= 8 ? 8 : 16;
        ls.detail(shape_tag(dev ? "dev" : "arg", mi, a.set, a.k, mm, a.scale_dev != nullptr));
      }
      SSP_TRY(launch_outer(ctx, a));
    }
  }
  return SSP_OK;
}
}  // namespace

extern "C" {

int ssp_gemm_outer(ssp_ctx* ctx, const double* alphas, const double* const* xx, int k, double* const* yy, int m,
                   size_t n) {
  return gemm_outer_impl(ctx, alphas, xx, nullptr, k, yy, nullptr, m, n, false);
}

int ssp_gemm_outer_set(ssp_ctx* ctx, const double* alphas, const double* const* xx, int k, double* const* yy, int m,
                       size_t n) {
  return gemm_outer_impl(ctx, alphas, xx, nullptr, k, yy, nullptr, m, n, true);
}

int ssp_gemm_outer_scaled(ssp_ctx* ctx, const double* alphas, const double* const* xx, const double* xs, int k,
                          double* const* yy, const double* ys, int m, size_t n) {
  return gemm_outer_impl(ctx, alphas, xx, xs, k, yy, ys, m, n, false);
}

int ssp_gemm_outer_set_scaled(ssp_ctx* ctx, const double* alphas, const double* const* xx, const double* xs, int k,
                              double* const* yy, int m, size_t n) {
  return gemm_outer_impl(ctx, alphas, xx, xs, k, yy, nullptr, m, n, true);
}

int ssp_scal_inner(ssp_ctx* ctx, double alpha, double* x, const double* const* yy, int m, size_t n, double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_scal_inner: negative dimension");
  if (m > 0 && !out) return ssp::set_error(SSP_ERR_ARG, "ssp_scal_inner: null out");
  SSP_TRY(check_ptrs(const_cast<const double* const*>(&x), 1, n, "ssp_scal_inner"));
  SSP_TRY(check_ptrs(yy, m, n, "ssp_scal_inner"));
  for (int j = 0; j < m; ++j)
    if (yy[j] == x) return ssp::set_error(SSP_ERR_ARG, "ssp_scal_inner: a vector of yy aliases x");
  // no dots, more than one launch, or the reference's arithmetic (short vectors): the unfused pair
  if (m == 0 || m > ssp::kOuterDst || ssp::exact_mode(ctx, n)) {
    SSP_TRY(ssp_scal(ctx, alpha, x, n));
    return m == 0 ? SSP_OK : ssp_gemm_inner(ctx, const_cast<const double* const*>(&x), 1, yy, m, n, out);
  }
  SSP_TRY(ssp::ensure_result(ctx, size_t(m)));
  ssp::FoldTail tail{};
  if (n == 0) {
    SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, size_t(m) * sizeof(double), ctx->stream));
  } else {
    SSP_TRY(ssp::fold_begin(ctx, m, &tail));
    ssp::LedgerScope ls(ctx, "scal_inner", 8.0 * n * (2.0 + m));
    const unsigned grid = ssp::win_grid(ctx, n, kFusedU, unsigned(ctx->fused_per_cu));
    ScalInnerArgs a{};
    a.x = x;
    a.alpha = alpha;
    a.m = m;
    a.n = n;
    for (int j = 0; j < m; ++j) a.y[j] = yy[j];
    SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * m));
    a.partial = ctx->partial;
    a.tail = tail;
    if (m <= 1)
      SSP_LAUNCH((k_scal_inner<1>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 4)
      SSP_LAUNCH((k_scal_inner<4>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 8)
      SSP_LAUNCH((k_scal_inner<8>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else
      SSP_LAUNCH((k_scal_inner<16>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
  }
  if (tail.counter) return ssp::fold_finish(ctx, tail, out);
  return ssp::reduce_fetch(ctx, out, size_t(m));
}

int ssp_axpy_norm(ssp_ctx* ctx, const double* c, const double* x, double* const* yy, int m, size_t n, double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 1) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_norm: needs at least one destination");
  if (!c || !out) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_norm: null coefficients or out");
  SSP_TRY(check_ptrs(&x, 1, n, "ssp_axpy_norm"));
  SSP_TRY(check_ptrs(const_cast<const double* const*>(yy), m, n, "ssp_axpy_norm"));
  for (int j = 0; j < m; ++j)
    if (yy[j] == x) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_norm: a destination aliases x");
  if (m > ssp::kOuterDst || ssp::exact_mode(ctx, n)) {  // more than one launch / short vectors: the unfused pair
    std::vector<double> alpha(c, c + m);
    SSP_TRY(ssp_gemm_outer(ctx, alpha.data(), &x, 1, yy, m, n));
    return ssp_dot(ctx, yy[0], yy[0], n, out);
  }
  SSP_TRY(ssp::ensure_result(ctx, 1));
  ssp::FoldTail tail{};
  if (n == 0) {
    SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, sizeof(double), ctx->stream));
  } else {
    SSP_TRY(ssp::fold_begin(ctx, 1, &tail));
    ssp::LedgerScope ls(ctx, "axpy_norm", 8.0 * n * (1.0 + 2.0 * m));
    const unsigned grid = ssp::win_grid(ctx, n, kFusedU, unsigned(ctx->fused_per_cu));
    AxpyInnerArgs a{};
    a.x = x;
    a.m = m;
    a.n = n;
    for (int j = 0; j < m; ++j) {
      a.y[j] = yy[j];
      a.c[j] = c[j];
    }
    SSP_TRY(ssp::ensure_partial(ctx, size_t(grid)));
    a.partial = ctx->partial;
    a.tail = tail;
    if (m <= 1)
      SSP_LAUNCH((k_axpy_norm<1>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 4)
      SSP_LAUNCH((k_axpy_norm<4>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 8)
      SSP_LAUNCH((k_axpy_norm<8>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else
      SSP_LAUNCH((k_axpy_norm<16>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
  }
  if (tail.counter) return ssp::fold_finish(ctx, tail, out);
  return ssp::reduce_fetch(ctx, out, 1);
}

int ssp_axpy_gram(ssp_ctx* ctx, const double* c, double* x, double xs, int store_x, double* const* yy, int m,
                  size_t n, double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 1) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_gram: needs at least one destination");
  if (!c || !out) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_gram: null coefficients or out");
  SSP_TRY(check_ptrs(const_cast<const double* const*>(&x), 1, n, "ssp_axpy_gram"));
  SSP_TRY(check_ptrs(const_cast<const double* const*>(yy), m, n, "ssp_axpy_gram"));
  for (int j = 0; j < m; ++j) {
    if (yy[j] == x) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_gram: a destination aliases x");
    for (int i = 0; i < j; ++i)
      if (yy[i] == yy[j]) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_gram: repeated destination");
  }
  if (m > ssp::kOuterDst || ssp::exact_mode(ctx, n)) {  // more than one launch / short vectors: unfused
    const double* xp = x;
    SSP_TRY(ssp_gemm_outer_scaled(ctx, c, &xp, &xs, 1, yy, nullptr, m, n));
    if (store_x && xs != 1.0) SSP_TRY(ssp_scal(ctx, xs, x, n));
    const double* y0 = yy[0];
    return ssp_gemm_inner(ctx, &y0, 1, const_cast<const double* const*>(yy), m, n, out);
  }
  SSP_TRY(ssp::ensure_result(ctx, size_t(m)));
  ssp::FoldTail tail{};
  if (n == 0) {
    SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, size_t(m) * sizeof(double), ctx->stream));
  } else {
    SSP_TRY(ssp::fold_begin(ctx, m, &tail));
    const bool st = store_x && xs != 1.0;
    ssp::LedgerScope ls(ctx, "axpy_gram", 8.0 * n * ((st ? 2.0 : 1.0) + 2.0 * m));
    const unsigned grid = ssp::win_grid(ctx, n, kFusedU, unsigned(ctx->fused_per_cu));
    AxpyGramArgs a{};
    a.x = x;
    a.xs = xs;
    a.store_x = st ? 1 : 0;
    a.m = m;
    a.n = n;
    for (int j = 0; j < m; ++j) {
      a.y[j] = yy[j];
      a.c[j] = c[j];
    }
    SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * m));
    a.partial = ctx->partial;
    a.tail = tail;
    if (m <= 1)
      SSP_LAUNCH((k_axpy_gram<1>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 4)
      SSP_LAUNCH((k_axpy_gram<4>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 8)
      SSP_LAUNCH((k_axpy_gram<8>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else
      SSP_LAUNCH((k_axpy_gram<16>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
  }
  if (tail.counter) return ssp::fold_finish(ctx, tail, out);
  return ssp::reduce_fetch(ctx, out, size_t(m));
}

int ssp_axpy_pairs_norm(ssp_ctx* ctx, const double* c, const double* const* xx, const double* xs, double* const* yy,
                        const double* ys, int m, size_t n, double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_pairs_norm: negative dimension");
  if (m == 0) return SSP_OK;
  if (!c || !out) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_pairs_norm: null coefficients or out");
  SSP_TRY(check_ptrs(xx, m, n, "ssp_axpy_pairs_norm"));
  SSP_TRY(check_ptrs(const_cast<const double* const*>(yy), m, n, "ssp_axpy_pairs_norm"));
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < m; ++i)
      if (yy[j] == xx[i] || (i < j && yy[i] == yy[j]))
        return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_pairs_norm: a destination aliases another operand");
  if (ssp::exact_mode(ctx, n)) {  // short vectors: the reference's arithmetic, one reduction
    ssp::FoldTail tail{};
    SSP_TRY(ssp::fold_begin(ctx, m, &tail));
    {
      ssp::LedgerScope ls(ctx, "axpy_pairs_norm", 24.0 * n * m);
      for (int j = 0; j < m; ++j)
        SSP_TRY(ssp::exact_outer(ctx, c + j, xx + j, xs ? xs + j : nullptr, 1, yy + j, ys ? ys + j : nullptr, 1, n, false));
      SSP_TRY(ssp::exact_inner(ctx, const_cast<const double* const*>(yy), nullptr, m,
                               const_cast<const double* const*>(yy), nullptr, m, n, true, tail));
    }
    return ssp::fold_finish(ctx, tail, out);
  }
  if (m > ssp::kOuterDst) {  // more than one launch: the unfused sequence, same values
    for (int j = 0; j < m; ++j)
      SSP_TRY(ssp_axpy_scaled(ctx, c[j], xx[j], xs ? xs[j] : 1.0, yy[j], ys ? ys[j] : 1.0, n));
    for (int j = 0; j < m; ++j) SSP_TRY(ssp_dot(ctx, yy[j], yy[j], n, out + j));
    return SSP_OK;
  }
  SSP_TRY(ssp::ensure_result(ctx, size_t(m)));
  ssp::FoldTail tail{};
  if (n == 0) {
    SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, size_t(m) * sizeof(double), ctx->stream));
  } else {
    SSP_TRY(ssp::fold_begin(ctx, m, &tail));
    ssp::LedgerScope ls(ctx, "axpy_pairs_norm", 24.0 * n * m);
    const unsigned grid = ssp::win_grid(ctx, n, kFusedU, unsigned(ctx->fused_per_cu));
    AxpyPairsArgs a{};
    a.m = m;
    a.n = n;
    for (int j = 0; j < m; ++j) {
      a.x[j] = xx[j];
      a.y[j] = yy[j];
      a.c[j] = c[j];
      a.xs[j] = xs ? xs[j] : 1.0;
      a.ys[j] = ys ? ys[j] : 1.0;
    }
    SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * m));
    a.partial = ctx->partial;
    a.tail = tail;
    if (m <= 1)
      SSP_LAUNCH((k_axpy_pairs_norm<1>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 4)
      SSP_LAUNCH((k_axpy_pairs_norm<4>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (m <= 8)
      SSP_LAUNCH((k_axpy_pairs_norm<8>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else
      SSP_LAUNCH((k_axpy_pairs_norm<16>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
  }
  if (tail.counter) return ssp::fold_finish(ctx, tail, out);
  return ssp::reduce_fetch(ctx, out, size_t(m));
}

int ssp_axpy_inner(ssp_ctx* ctx, const double* c, const double* x, double* const* yy, int m, const double* z, size_t n,
                   double* out) {
  SSP_CHECK_CTX(ctx);
  if (m < 0) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_inner: negative dimension");
  if (m == 0) return SSP_OK;
  if (!c || !out) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_inner: null coefficients or out");
  SSP_TRY(check_ptrs(&x, 1, n, "ssp_axpy_inner"));
  SSP_TRY(check_ptrs(&z, 1, n, "ssp_axpy_inner"));
  SSP_TRY(check_ptrs(const_cast<const double* const*>(yy), m, n, "ssp_axpy_inner"));
  for (int j = 0; j < m; ++j)
    if (yy[j] == x || yy[j] == z) return ssp::set_error(SSP_ERR_ARG, "ssp_axpy_inner: a destination aliases x or z");
  if (ssp::exact_mode(ctx, n)) {  // short vectors: the reference's arithmetic, one reduction
    ssp::FoldTail tail{};
    SSP_TRY(ssp::fold_begin(ctx, m, &tail));
    {
      ssp::LedgerScope ls(ctx, "axpy_inner", 8.0 * n * (2.0 + 2.0 * m));
      SSP_TRY(ssp::exact_outer(ctx, c, &x, nullptr, 1, yy, nullptr, m, n, false));
      SSP_TRY(ssp::exact_inner(ctx, const_cast<const double* const*>(yy), nullptr, m, &z, nullptr, 1, n, false, tail));
    }
    return ssp::fold_finish(ctx, tail, out);
  }
  SSP_TRY(ssp::ensure_result(ctx, size_t(m)));
  ssp::FoldTail tail{};
  if (n == 0) {
    SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, size_t(m) * sizeof(double), ctx->stream));
  } else {
    if (m <= ssp::kOuterDst) SSP_TRY(ssp::fold_begin(ctx, m, &tail));  // one launch: fused fold
    ssp::LedgerScope ls(ctx, "axpy_inner", 8.0 * n * (2.0 + 2.0 * m));
    const unsigned grid = ssp::win_grid(ctx, n, kFusedU, unsigned(ctx->fused_per_cu));
    for (int j0 = 0; j0 < m; j0 += ssp::kOuterDst) {
      AxpyInnerArgs a{};
      a.m = std::min(ssp::kOuterDst, m - j0);
      a.n = n;
      a.x = x;
      a.z = z;
      for (int j = 0; j < a.m; ++j) {
        a.y[j] = yy[j0 + j];
        a.c[j] = c[j0 + j];
      }
      SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * a.m));
      a.partial = ctx->partial;
      a.tail = tail;
      if (a.m <= 1)
        SSP_LAUNCH((k_axpy_inner<1>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
      else if (a.m <= 4)
        SSP_LAUNCH((k_axpy_inner<4>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
      else if (a.m <= 8)
        SSP_LAUNCH((k_axpy_inner<8>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
      else
        SSP_LAUNCH((k_axpy_inner<16>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
      SSP_TRY_HIP(hipGetLastError());
      if (!tail.counter)
        SSP_TRY(ssp::launch_reduce_partials(ctx, ctx->partial, int(grid), 1, a.m, ctx->result_dev, m, 0, j0));
    }
  }
  if (tail.counter) return ssp::fold_finish(ctx, tail, out);
  return ssp::reduce_fetch(ctx, out, size_t(m));
}

}  // extern "C"

namespace {
// ssp_transform_gram / ssp_transform_norms: dots 2 = the Gram matrix into out (m x m), 1 = the self-dots
// into out (m), 0 = none.
int transform_impl(ssp_ctx* ctx, const double* t, double* const* xx, const double* xs, int m, size_t n, int dots,
                   double* out, const char* what) {
  SSP_CHECK_CTX(ctx);
  if (m < 1 || m > 8) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": 1 <= m <= 8");
  if (!t) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": null t");
  SSP_TRY(check_ptrs(const_cast<const double* const*>(xx), m, n, what));
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < j; ++i)
      if (xx[i] == xx[j]) return ssp::set_error(SSP_ERR_ARG, std::string(what) + ": repeated vector");
  const bool exact = ssp::exact_mode(ctx, n);
  TransformArgs a{};
  a.m = m;
  a.n = n;
  for (int i = 0; i < m; ++i) {
    a.x[i] = xx[i];
    a.s[i] = xs ? xs[i] : 1.0;
  }
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) a.t[j * m + i] = t[i * m + j];  // transposed: column j contiguous
  const int nd = dots == 2 ? m * (m + 1) / 2 : (dots == 1 ? m : 0);
  // the fused dots only from the bandwidth kernel; short vectors take the reference's sequential dots
  const int fused = (dots > 0 && !exact && n > 0) ? dots : 0;
  ssp::FoldTail tail{};
  if (n > 0) {
    ssp::LedgerScope ls(ctx, dots ? "transform_gram" : "transform", 16.0 * n * m);
    const bool wide = ctx->transform_wide && m > 4 && fused == 1;  // k_transform's WIDE instance
    const unsigned grid = ssp::win_grid(ctx, n, fused == 2 ? 1 : (m <= 4 ? 4 : (wide ? 4 : 2)),
                                        unsigned(ctx->fused_per_cu));
    const bool pass = fused == 2 && gram_reduce_pass();
    if (fused) {
      SSP_TRY(ssp::fold_begin(ctx, nd, &tail));
      SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * nd));
      a.partial = ctx->partial;
      if (!pass) a.tail = tail;  // else the kernel leaves its partials to the reduce pass below
    }
    ls.detail(shape_tag("transform", m, fused, m, m, xs != nullptr));
    launch_transform(ctx, m, grid, a, fused, exact, pass);
    SSP_TRY_HIP(hipGetLastError());
    if (pass)  // one workgroup per pair dot, publishing to the host (as the gemm_inner panels)
      SSP_TRY(ssp::launch_reduce_partials(ctx, ctx->partial, int(grid), 1, nd, ctx->result_dev, nd, 0, 0, &tail, true));
  }
  if (!dots) return SSP_OK;
  if (!fused) {
    // Short (or empty) vectors: the dots of the stored outputs as the reference's sequential dots
    // (each the number ssp_gemm_inner's short path gives), reduced in the fused kernel's layout -- the
    // nd pair dots (a <= b) or the m self-dots -- so that a rank whose shard takes this branch posts
    // the same collective as a rank on the bandwidth kernel (shards of spread_remainder differ by one
    // element and may straddle exact_max; a rank may hold none).
    std::vector<const double*> ra, rb;
    for (int i = 0; i < m; ++i)
      for (int j = i; j < (dots == 2 ? m : i + 1); ++j) {
        ra.push_back(xx[i]);
        rb.push_back(xx[j]);
      }
    SSP_TRY(ssp::fold_begin(ctx, nd, &tail));
    {
      ssp::LedgerScope ls(ctx, "gemm_inner", 8.0 * n * m);
      SSP_TRY(ssp::exact_inner(ctx, ra.data(), nullptr, nd, rb.data(), nullptr, nd, n, true, tail));
    }
  }
  if (dots == 1) return ssp::fold_finish(ctx, tail, out);
  std::vector<double> pr(static_cast<size_t>(nd));
  SSP_TRY(ssp::fold_finish(ctx, tail, pr.data()));
  for (int i = 0, q = 0; i < m; ++i)
    for (int j = i; j < m; ++j, ++q) out[size_t(i) * m + j] = out[size_t(j) * m + i] = pr[size_t(q)];
  return SSP_OK;
}
}  // namespace

extern "C" {

int ssp_transform_gram(ssp_ctx* ctx, const double* t, double* const* xx, const double* xs, int m, size_t n,
                       double* gram) {
  return transform_impl(ctx, t, xx, xs, m, n, gram ? 2 : 0, gram, "ssp_transform_gram");
}

int ssp_transform_norms(ssp_ctx* ctx, const double* t, double* const* xx, const double* xs, int m, size_t n,
                        double* norms2) {
  if (!norms2) return ssp::set_error(SSP_ERR_ARG, "ssp_transform_norms: null norms2");
  return transform_impl(ctx, t, xx, xs, m, n, 1, norms2, "ssp_transform_norms");
}

int ssp_precondition_norms(ssp_ctx* ctx, double* const* a, int nvec, const double* d, const double* shift, size_t n,
                           double* norms2) {
  SSP_CHECK_CTX(ctx);
  if (nvec < 0 || nvec > 8 || (nvec > 0 && (!a || !shift || !norms2)))
    return ssp::set_error(SSP_ERR_ARG, "ssp_precondition_norms: bad vectors (0 <= nvec <= 8)");
  if (nvec == 0) return SSP_OK;
  // short (or empty) vectors: the reference's arithmetic for the dots (sequential sums, the numbers
  // gemm_inner's short path gives), reduced as the bandwidth pass's nvec self-dots are (one collective
  // of nvec values whichever branch a rank's shard takes)
  if (n == 0 || ssp::exact_mode(ctx, n)) {
    SSP_TRY(ssp_precondition(ctx, a, nvec, d, shift, n));
    std::vector<const double*> c(a, a + nvec);
    ssp::FoldTail tail{};
    SSP_TRY(ssp::fold_begin(ctx, nvec, &tail));
    {
      ssp::LedgerScope ls(ctx, "gemm_inner", 8.0 * n * nvec);
      SSP_TRY(ssp::exact_inner(ctx, c.data(), nullptr, nvec, c.data(), nullptr, nvec, n, true, tail));
    }
    return ssp::fold_finish(ctx, tail, norms2);
  }
  SSP_TRY(check_ptrs(&d, 1, n, "ssp_precondition_norms"));
  SSP_TRY(check_ptrs(const_cast<const double* const*>(a), nvec, n, "ssp_precondition_norms"));
  PrecNormArgs p{};
  p.nvec = nvec;
  for (int v = 0; v < nvec; ++v) {
    p.a[v] = a[v];
    p.shift[v] = shift[v];
  }
  p.d = d;
  p.n = n;
  ssp::FoldTail tail{};
  {
    ssp::LedgerScope ls(ctx, "precondition", 8.0 * n * (1 + 2 * nvec));
    const unsigned grid = ssp::win_grid(ctx, n, 4, unsigned(ctx->fused_per_cu));
    SSP_TRY(ssp::fold_begin(ctx, nvec, &tail));
    SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * nvec));
    p.partial = ctx->partial;
    p.tail = tail;
    if (nvec <= 4) SSP_LAUNCH(k_precondition_norms<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    else SSP_LAUNCH(k_precondition_norms<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    SSP_TRY_HIP(hipGetLastError());
  }
  return ssp::fold_finish(ctx, tail, norms2);
}

}  // extern "C"
