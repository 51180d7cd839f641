// Synthetic problem generator for tests and benchmarks (not a reference hot-path operation).
//
// H = diag(d) + rho * sum_{l < rank} u_l u_l^T, g = global index; u_0 = 1 (the matrix of
// reference test/itsolv/test_rayleigh_quotient.cpp:37-42 for rank 1) and u_l(g) = +/-1 from
// splitmix64 for l > 0.  d_g = 1 + g (SSPX_DIAG_LINEAR, the Davidson configurations) or
// d_g = 1 + 2 frac(g phi1) (SSPX_DIAG_BOUNDED, the C5 DIIS instance; its preconditioner diagonal is
// d_g (1 + alpha (2 frac(g phi2) - 1)), itsolv_hbm/problems.h).  Applying H costs one rank x nvec
// reduction (+ allreduce) and one stream.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "ssp_internal.h"

namespace {

using ssp::kBlock;
constexpr int kMaxVec = 16;
constexpr int kMaxRank = 16;
constexpr int kSynthU = 2;  // window of the apply kernel: kSynthU x 64 pairs of each vector per wave visit

__host__ __device__ inline unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Stream key for (seed, stream): the per-element hash is splitmix64(key ^ g).
inline unsigned long long stream_key(unsigned long long seed, unsigned long long stream) {
  return splitmix64(seed ^ (stream * 0xD1B54A32D192ED03ull));
}

// Bit l of the mask is set when u_l(g) = -1 (u_0 = 1 always).  The masks are computed once per
// (seed, rank, shard) into a 2-byte-per-element table (sspx_synthetic_action's cache in the context),
// so the action kernels stream x, y and the table instead of evaluating rank - 1 splitmix64 hashes
// (two 64-bit multiplies each) per element and pass: 3.3 TB/s with the hashes inline, the table adds
// 2 B per element to the 16-24 B per element and vector the kernels move.
template <int R>
__device__ __forceinline__ unsigned sign_mask(const unsigned long long (&key)[16], unsigned long long g) {
  unsigned m = 0;
#pragma unroll
  for (int l = 1; l < R; ++l) m |= unsigned(splitmix64(key[l] ^ g) & 1ull) << l;
  return m;
}

__device__ __forceinline__ double flip(unsigned mask, int l, double v) { return ((mask >> l) & 1u) ? -v : v; }

// The diagonal families, bit-identical to itsolv_hbm/problems.h SyntheticSpec::d / ::diagonal (the
// same IEEE operations in the same order, contraction off).
constexpr double kPhi1 = 0x1.3c6ef372fe950p-1;
constexpr double kPhi2 = 0x1.827f5352054c6p-1;
__device__ __forceinline__ double frac_phi(unsigned long long g, double phi) {
#pragma clang fp contract(off)
  const double f = double(g) * phi;
  return f - floor(f);
}
__device__ __forceinline__ double synth_d(int kind, unsigned long long g) {
#pragma clang fp contract(off)
  return kind == SSPX_DIAG_BOUNDED ? 1.0 + 2.0 * frac_phi(g, kPhi1) : 1.0 + double(g);
}

struct SynthArgs {
  const double* x[kMaxVec];
  double xs[kMaxVec];  // deferred scales of the parameters (1: none); x * xs is the eager scal's value
  double* y[kMaxVec];
  unsigned long long key[kMaxRank];
  const unsigned short* mask;  // [n] sign masks of this shard
  int nvec;
  int rank;
  int diag_kind;
  size_t n;
  size_t offset;
  double rho;
  double* partial;      // [grid][nvec*rank]
  const double* coeff;  // [nvec*rank] global u_l . x_v
  int exact;            // the reference's arithmetic (ssp_ctx_set_exact_max): products rounded alone
};

template <int R>
__global__ __launch_bounds__(kBlock) void k_synth_mask(const SynthArgs a, unsigned short* mask) {
  const size_t stride = size_t(gridDim.x) * kBlock;
  for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
    mask[i] = (unsigned short)sign_mask<R>(a.key, a.offset + i);
}

__device__ __forceinline__ double block_sum(double v, double* wsum) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) wsum[wave] = v;
  __syncthreads();
  double s = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < kBlock / 64; ++w) s += wsum[w];
  return s;
}

// Element pairs: 16 B of each vector and 4 B of the mask table per lane and visit (the tail element
// of an odd-length shard is folded in by the thread that owns pair n/2).
__device__ __forceinline__ double2 ld2nt(const double* p) { return ssp::ld2nt(p); }

// Per-block partial sums of u_l . x_v for the NV vectors v0 .. v0+NV-1 (R x NV accumulators per
// thread).  NV is a compile-time count, so every vector's loads of a visit are issued together, and two
// visits (i, i + stride) are in flight per lane; each accumulator still adds its terms in the order
// i, i + stride, i + 2 stride, ...
template <int R, int NV>
__device__ __forceinline__ void coeff_visit(double (&s)[NV][R], unsigned mm, const double2 (&xv)[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int l = 0; l < R; ++l) s[v][l] += flip(mm, l, xv[v].x) + flip(mm >> 16, l, xv[v].y);
}

// G > 0: the launch holds gridDim.x / G consecutive vector groups of NV, G workgroups each (one
// launch for a whole action); workgroup b of group q works as workgroup b of a G-workgroup launch for
// vectors v0 + q NV .. -- the same visits and partial sums, so the same numbers.  G = 0: one group.
template <int R, int NV>
__global__ __launch_bounds__(kBlock) void k_synth_coeff(const SynthArgs a, int v0, unsigned G) {
  __shared__ double wsum[kBlock / 64];
  const unsigned nb = G ? G : gridDim.x, bid = G ? blockIdx.x % G : blockIdx.x;
  if (G) v0 += int(blockIdx.x / G) * NV;
  const size_t stride = size_t(nb) * kBlock, n2 = a.n >> 1;
  const unsigned* mask2 = reinterpret_cast<const unsigned*>(a.mask);
  const double* xp[NV];
  double xs[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    xp[v] = a.x[v0 + v];
    xs[v] = a.xs[v0 + v];
  }
  double s[NV][R];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int l = 0; l < R; ++l) s[v][l] = 0;
  size_t i = size_t(bid) * kBlock + threadIdx.x;
  for (; i + stride < n2; i += 2 * stride) {
    const unsigned m0 = mask2[i], m1 = mask2[i + stride];
    double2 x0[NV], x1[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      x0[v] = ld2nt(xp[v] + 2 * i);
      x1[v] = ld2nt(xp[v] + 2 * (i + stride));
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      x0[v].x *= xs[v];
      x0[v].y *= xs[v];
      x1[v].x *= xs[v];
      x1[v].y *= xs[v];
    }
    coeff_visit<R, NV>(s, m0, x0);
    coeff_visit<R, NV>(s, m1, x1);
  }
  if (i < n2) {
    const unsigned m0 = mask2[i];
    double2 x0[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      x0[v] = ld2nt(xp[v] + 2 * i);
      x0[v].x *= xs[v];
      x0[v].y *= xs[v];
    }
    coeff_visit<R, NV>(s, m0, x0);
  }
  if ((a.n & 1) && bid == 0 && threadIdx.x == 0) {
    const unsigned mm = a.mask[a.n - 1];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int l = 0; l < R; ++l) s[v][l] += flip(mm, l, xp[v][a.n - 1] * xs[v]);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int l = 0; l < R; ++l) {
      const double t = block_sum(s[v][l], wsum);
      if (threadIdx.x == 0) a.partial[size_t(bid) * a.nvec * R + (v0 + v) * R + l] = t;
    }
  }
}

// Short vectors (ssp_ctx_set_exact_max): the coefficients as sequential sums in index order, as the
// host restatement's loop.  One workgroup per vector: waves 1..3 stage the next chunk of scaled
// values and sign masks in LDS while lanes l < R of wave 0 add the current chunk for coefficient l in
// order (double-buffered; the LDS reads run 8 values ahead of the adds).  out[v * R + l], v < nvec.
template <int R>
__global__ __launch_bounds__(kBlock) void k_synth_coeff_exact(const SynthArgs a, double* out) {
  constexpr int kChunk = 2048;
  __shared__ __attribute__((aligned(16))) double xv[2][kChunk];
  __shared__ __attribute__((aligned(16))) unsigned short mk[2][kChunk];
  const int v = int(blockIdx.x), l = int(threadIdx.x);
  const int fill_lane = int(threadIdx.x) - 64, fill_lanes = kBlock - 64;
  const int nchunk = int((a.n + kChunk - 1) / kChunk);
  auto fill = [&](int c) {
    const size_t c0 = size_t(c) * kChunk;
    const int len = int(a.n - c0 < size_t(kChunk) ? a.n - c0 : size_t(kChunk));
    const double* x = a.x[v];
    const double xs = a.xs[v];
    for (int t0 = fill_lane; t0 < len; t0 += 4 * fill_lanes) {  // 4 elements' loads in flight per lane
      double x4[4];
      unsigned short m4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * fill_lanes;
        if (t < len) {
          x4[u] = x[c0 + t];
          m4[u] = a.mask[c0 + t];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * fill_lanes;
        if (t < len) {
          xv[c & 1][t] = x4[u] * xs;
          mk[c & 1][t] = m4[u];
        }
      }
    }
  };
  if (fill_lane >= 0) fill(0);
  __syncthreads();
  double s = 0;
  for (int c = 0; c < nchunk; ++c) {
    if (fill_lane >= 0) {
      if (c + 1 < nchunk) fill(c + 1);
    } else if (l < R) {
      const size_t c0 = size_t(c) * kChunk;
      const int len = int(a.n - c0 < size_t(kChunk) ? a.n - c0 : size_t(kChunk));
      const double* xb = xv[c & 1];
      const unsigned short* mb = mk[c & 1];
      int t = 0;
      for (; t + 8 <= len; t += 8) {
        double x8[8];
        unsigned short m8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          x8[u] = xb[t + u];
          m8[u] = mb[t + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) s = s + flip(m8[u], l, x8[u]);
      }
      for (; t < len; ++t) s = s + flip(mb[t], l, xb[t]);
    }
    __syncthreads();
  }
  if (l < R) out[v * R + l] = s;
}

// d x + rho s and y + rho s with every product rounded alone (the reference's arithmetic).
__device__ __forceinline__ double mul_add_mul(double a, double b, double c, double d) {
#pragma clang fp contract(off)
  return a * b + c * d;
}
__device__ __forceinline__ double add_mul(double y, double c, double d) {
#pragma clang fp contract(off)
  return y + c * d;
}

template <int R>
__device__ __forceinline__ double lowrank(unsigned mm, const double (&c)[R]) {
  double s = 0;
#pragma unroll
  for (int l = 0; l < R; ++l) s += flip(mm, l, c[l]);
  return s;
}

// The low-rank sums of every sign pattern (R <= 8: 2^R patterns), built by each workgroup before it
// streams: tab[v][m] = lowrank<R>(m, coeff of vector v0 + v), the same function of the same operands,
// so a lookup is bit for bit the inline sum.  The inline form costs 2R VALU operations (mask-bit test,
// conditional sign, add) per element and vector -- at rank 8 and 4 vectors ~500 VALU instructions per
// wave visit of 8.4 KiB, a VALU issue ceiling near the HBM rate -- against one LDS read.  The P-space
// update (ADD: no diagonal term, half the VALU work per byte) keeps the inline sums: building the table
// in each of its up to 4096 workgroups cost more than it saved (C4 shard 2.27 -> 2.38 ms per solve).
constexpr int kTabRank = 8;
template <int R, int NV, bool ON = true>
struct LowrankTab {
  static constexpr bool kOn = ON && R <= kTabRank;
  static constexpr int kSize = kOn ? (1 << R) : 1;
  double* t;  // [NV][kSize] in LDS
  __device__ __forceinline__ double operator()(int v, unsigned mm, const double (&c)[R]) const {
    if constexpr (kOn) return t[v * kSize + (mm & unsigned(kSize - 1))];
    return lowrank<R>(mm, c);
  }
};
template <int R, int NV, bool ON>
__device__ __forceinline__ LowrankTab<R, NV, ON> build_tab(const SynthArgs& a, int v0) {
  using T = LowrankTab<R, NV, ON>;
  __shared__ double tab[NV * T::kSize];
  if constexpr (T::kOn) {
    for (int i = int(threadIdx.x); i < NV * T::kSize; i += kBlock) {
      const int v = i / T::kSize;
      double c[R];
#pragma unroll
      for (int l = 0; l < R; ++l) c[l] = a.coeff[(v0 + v) * R + l];
      tab[i] = lowrank<R>(unsigned(i % T::kSize), c);
    }
    __syncthreads();
  }
  return T{tab};
}

// y_v = d x_v + rho sum_l u_l coeff[v][l]   (ADD = false)
// y_v += rho sum_l u_l coeff[v][l]          (ADD = true, the P-space low-rank term)
// for the NV vectors v0 .. v0+NV-1, coefficients in registers, in the window shape of the streaming
// kernels (ssp::for_windows: each wave owns U x 64 consecutive pairs of every vector per visit, all of
// the visit's masks and operands loaded before its stores).  Element for element the same operations
// as one pair at a time.
// EX: the reference's arithmetic (short vectors, kernels_exact.hip): products rounded alone.
// G > 0: gridDim.x / G vector groups of NV in one launch, G workgroups each (as k_synth_coeff).
template <int R, bool ADD, int NV, bool EX>
__global__ __launch_bounds__(kBlock) void k_synth_apply(const SynthArgs a, int v0, unsigned G) {
  constexpr int U = kSynthU;
  const unsigned nb = G ? G : gridDim.x, bid = G ? blockIdx.x % G : blockIdx.x;
  if (G) v0 += int(blockIdx.x / G) * NV;
  const unsigned* mask2 = reinterpret_cast<const unsigned*>(a.mask);
  const LowrankTab<R, NV, !ADD> tab = build_tab<R, NV, !ADD>(a, v0);
  double c[NV][R];
  const double* xp[NV];
  double* yp[NV];
  double xs[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int l = 0; l < R; ++l) c[v][l] = tab.kOn ? 0.0 : a.coeff[(v0 + v) * R + l];
    xp[v] = ADD ? a.y[v0 + v] : a.x[v0 + v];
    yp[v] = a.y[v0 + v];
    xs[v] = ADD ? 1.0 : a.xs[v0 + v];
  }
  // y at pair i from its mask and operands
  auto pair = [&](size_t i, unsigned mm, const double2 (&in)[NV]) {
    const size_t g = a.offset + 2 * i;
    const double d0 = synth_d(a.diag_kind, g), d1 = synth_d(a.diag_kind, g + 1);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const double s0 = tab(v, mm, c[v]), s1 = tab(v, mm >> 16, c[v]);
      double2 out;
      if (ADD) {
        const double2 y = in[v];
        out = EX ? make_double2(add_mul(y.x, a.rho, s0), add_mul(y.y, a.rho, s1))
                 : make_double2(fma(a.rho, s0, y.x), fma(a.rho, s1, y.y));
      } else {
        const double2 x = in[v];
        out = EX ? make_double2(mul_add_mul(d0, x.x * xs[v], a.rho, s0), mul_add_mul(d1, x.y * xs[v], a.rho, s1))
                 : make_double2(fma(d0, x.x * xs[v], a.rho * s0), fma(d1, x.y * xs[v], a.rho * s1));
      }
      ssp::st2nt(yp[v] + 2 * i, out);
    }
  };
  ssp::for_windows_in<U>(
      a.n, bid, nb,
      [&](size_t p0) {
        unsigned mm[U];
        double2 in[U][NV];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          mm[u] = mask2[p0 + 64 * u];
#pragma unroll
          for (int v = 0; v < NV; ++v) in[u][v] = ld2nt(xp[v] + 2 * (p0 + 64 * u));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) pair(p0 + 64 * u, mm[u], in[u]);
      },
      [&](size_t i) {
        double2 in[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) in[v] = ld2nt(xp[v] + 2 * i);
        pair(i, mask2[i], in);
      },
      [&](size_t e) {
        const unsigned mm = a.mask[e];
        const double d = synth_d(a.diag_kind, a.offset + e);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const double s = tab(v, mm, c[v]);
          if (EX)
            yp[v][e] = ADD ? add_mul(yp[v][e], a.rho, s) : mul_add_mul(d, xp[v][e] * xs[v], a.rho, s);
          else
            yp[v][e] = ADD ? fma(a.rho, s, yp[v][e]) : fma(d, xp[v][e] * xs[v], a.rho * s);
        }
      });
}

// The same, grid-strided one pair per lane and visit (SSP_SYNTH_SHAPE=stride, the A/B of the window shape).
// for the NV vectors v0 .. v0+NV-1, coefficients in registers.  The next visit's mask and operands
// are loaded before this visit's stores are issued: vector-memory operations retire in order on
// gfx9, so a load issued after a store cannot be waited for without waiting for the store.
// EX: the reference's arithmetic (short vectors, kernels_exact.hip): products rounded alone.
template <int R, bool ADD, int NV, bool EX>
__global__ __launch_bounds__(kBlock) void k_synth_apply_pipe(const SynthArgs a, int v0) {
  const size_t stride = size_t(gridDim.x) * kBlock, n2 = a.n >> 1;
  const unsigned* mask2 = reinterpret_cast<const unsigned*>(a.mask);
  const LowrankTab<R, NV, !ADD> tab = build_tab<R, NV, !ADD>(a, v0);
  double c[NV][R];
  const double* xp[NV];
  double* yp[NV];
  double xs[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int l = 0; l < R; ++l) c[v][l] = tab.kOn ? 0.0 : a.coeff[(v0 + v) * R + l];
    xp[v] = ADD ? a.y[v0 + v] : a.x[v0 + v];
    yp[v] = a.y[v0 + v];
    xs[v] = ADD ? 1.0 : a.xs[v0 + v];
  }
  size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n2) {
    unsigned mm = mask2[i];
    double2 in[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) in[v] = ld2nt(xp[v] + 2 * i);
    for (; i < n2; i += stride) {
      const size_t ip = i + stride < n2 ? i + stride : i;  // the next visit (or this one again)
      const unsigned mnext = mask2[ip];
      double2 nxt[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) nxt[v] = ld2nt(xp[v] + 2 * ip);
      const size_t g = a.offset + 2 * i;
      const double d0 = synth_d(a.diag_kind, g), d1 = synth_d(a.diag_kind, g + 1);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const double s0 = tab(v, mm, c[v]), s1 = tab(v, mm >> 16, c[v]);
        double2 out;
        if (ADD) {
          const double2 y = in[v];
          out = EX ? make_double2(add_mul(y.x, a.rho, s0), add_mul(y.y, a.rho, s1))
                   : make_double2(fma(a.rho, s0, y.x), fma(a.rho, s1, y.y));
        } else {
          const double2 x = in[v];
          out = EX ? make_double2(mul_add_mul(d0, x.x * xs[v], a.rho, s0), mul_add_mul(d1, x.y * xs[v], a.rho, s1))
                   : make_double2(fma(d0, x.x * xs[v], a.rho * s0), fma(d1, x.y * xs[v], a.rho * s1));
        }
        ssp::st2nt(yp[v] + 2 * i, out);
      }
      mm = mnext;
#pragma unroll
      for (int v = 0; v < NV; ++v) in[v] = nxt[v];
    }
  }
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const size_t e = a.n - 1;
    const unsigned mm = a.mask[e];
    const double d = synth_d(a.diag_kind, a.offset + e);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const double s = tab(v, mm, c[v]);
      if (EX)
        yp[v][e] = ADD ? add_mul(yp[v][e], a.rho, s) : mul_add_mul(d, xp[v][e] * xs[v], a.rho, s);
      else
        yp[v][e] = ADD ? fma(a.rho, s, yp[v][e]) : fma(d, xp[v][e] * xs[v], a.rho * s);
    }
  }
}

// Vectors in groups of NV = 4 (2 from rank 9 on, where R x NV accumulators would crowd the
// registers), one launch per group; the last group's NV is the remainder.
template <int R>
constexpr int coeff_group() {
  return R > 8 ? 2 : 4;
}

// merge: the full groups of a.nvec in one launch (grid workgroups per group), when there are several
// and no partial one.
template <int R>
void launch_coeff(unsigned grid, hipStream_t st, const SynthArgs& a, bool merge) {
  constexpr int G = coeff_group<R>();
  if (merge && a.nvec > G && a.nvec % G == 0) {
    SSP_LAUNCH((k_synth_coeff<R, G>), dim3(grid * unsigned(a.nvec / G)), dim3(kBlock), 0, st, a, 0, grid);
    return;
  }
  for (int v0 = 0; v0 < a.nvec; v0 += G) {
    const int nv = std::min(G, a.nvec - v0);
    if (nv == 4) SSP_LAUNCH((k_synth_coeff<R, (G >= 4 ? 4 : 1)>), dim3(grid), dim3(kBlock), 0, st, a, v0, 0u);
    else if (nv == 3) SSP_LAUNCH((k_synth_coeff<R, (G >= 4 ? 3 : 1)>), dim3(grid), dim3(kBlock), 0, st, a, v0, 0u);
    else if (nv == 2) SSP_LAUNCH((k_synth_coeff<R, 2>), dim3(grid), dim3(kBlock), 0, st, a, v0, 0u);
    else SSP_LAUNCH((k_synth_coeff<R, 1>), dim3(grid), dim3(kBlock), 0, st, a, v0, 0u);
  }
}

#define SSP_RANK_CASES(F) \
  F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(8) F(9) F(10) F(11) F(12) F(13) F(14) F(15) F(16)

void synth_coeff(unsigned grid, hipStream_t st, const SynthArgs& a, bool merge) {
  switch (a.rank) {
#define F(r) \
  case r:    \
    launch_coeff<r>(grid, st, a, merge); \
    break;
    SSP_RANK_CASES(F)
#undef F
  }
}

void synth_coeff_exact(hipStream_t st, const SynthArgs& a, double* out) {
  switch (a.rank) {
#define F(r)                                                                                          \
  case r:                                                                                             \
    SSP_LAUNCH((k_synth_coeff_exact<r>), dim3(unsigned(a.nvec)), dim3(kBlock), 0, st, a, out); \
    break;
    SSP_RANK_CASES(F)
#undef F
  }
}

template <int R, bool ADD, bool EX, bool WIN>
void launch_apply_ex(const ssp_ctx* ctx, hipStream_t st, const SynthArgs& a) {
  constexpr int G = coeff_group<R>();
  const unsigned grid = WIN ? ssp::win_grid(ctx, a.n, kSynthU, 16) : ssp::stream_grid(ctx, a.n, 1);
  if (WIN && !EX && ctx->synth_merge && a.nvec > G && a.nvec % G == 0) {  // the full groups in one launch
    SSP_LAUNCH((k_synth_apply<R, ADD, G, EX>), dim3(grid * unsigned(a.nvec / G)), dim3(kBlock), 0, st, a, 0, grid);
    return;
  }
  for (int v0 = 0; v0 < a.nvec; v0 += G) {
    const int nv = std::min(G, a.nvec - v0);
#define SSP_APPLY(NV)                                                                                       \
  if (WIN) SSP_LAUNCH((k_synth_apply<R, ADD, NV, EX>), dim3(grid), dim3(kBlock), 0, st, a, v0, 0u); \
  else SSP_LAUNCH((k_synth_apply_pipe<R, ADD, NV, EX>), dim3(grid), dim3(kBlock), 0, st, a, v0);
    if (nv == 4) { SSP_APPLY((G >= 4 ? 4 : 1)) }
    else if (nv == 3) { SSP_APPLY((G >= 4 ? 3 : 1)) }
    else if (nv == 2) { SSP_APPLY(2) }
    else { SSP_APPLY(1) }
#undef SSP_APPLY
  }
}

// Shape (tools/gpu_r4n.sh, profiles/r4/synth_shape_ab/): the window shape moves the P-space low-rank
// update (ADD) at every size measured (C3's 1e8: 18.6-18.8 against 19.9-22.3 ms per solve; C4's shard:
// 2.26 against 2.34-2.59 ms) and the action from 2^24 elements (C3: 24.9 against 25.4-28.2 ms), while
// at C4's shard the action's grid-strided pipelined form is ahead (3.33-3.40 against 3.61 ms: the
// window kernel holds 256 registers per lane).  SSP_SYNTH_SHAPE=stride forces the strided form.
// Round 5: with the action's low-rank sums tabulated (R <= kTabRank) the window kernel is no longer
// register-bound, and it leads at the C4 shard too (3.19 against 3.31-3.41 ms per solve, alternating
// processes, profiles/r5/ab_ledger_timing/): the window shape for every size there.
template <int R, bool ADD>
void launch_apply(const ssp_ctx* ctx, hipStream_t st, const SynthArgs& a) {
  const bool win = ctx->synth_window ||
                   (!ctx->synth_stride && (ADD || R <= kTabRank || a.n >= (size_t(1) << 24)));
  if (a.exact) win ? launch_apply_ex<R, ADD, true, true>(ctx, st, a) : launch_apply_ex<R, ADD, true, false>(ctx, st, a);
  else win ? launch_apply_ex<R, ADD, false, true>(ctx, st, a) : launch_apply_ex<R, ADD, false, false>(ctx, st, a);
}

template <bool ADD>
void synth_apply(const ssp_ctx* ctx, hipStream_t st, const SynthArgs& a) {
  switch (a.rank) {
#define F(r)                           \
  case r:                              \
    launch_apply<r, ADD>(ctx, st, a); \
    break;
    SSP_RANK_CASES(F)
#undef F
  }
}

void synth_mask_kernel(unsigned grid, hipStream_t st, const SynthArgs& a, unsigned short* mask) {
  switch (a.rank) {
#define F(r)                                                                                \
  case r:                                                                                   \
    SSP_LAUNCH((k_synth_mask<r>), dim3(grid), dim3(kBlock), 0, st, a, mask); \
    break;
    SSP_RANK_CASES(F)
#undef F
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// The shard's sign-mask table for (seed, rank, offset, n), built on first use (one hash pass).
int ensure_mask(ssp_ctx* ctx, SynthArgs& a, unsigned long long seed) {
  if (ctx->synth_mask && ctx->synth_mask_n == a.n && ctx->synth_mask_offset == a.offset &&
      ctx->synth_mask_seed == seed && ctx->synth_mask_rank == a.rank) {
    a.mask = ctx->synth_mask;
    return SSP_OK;
  }
  if (ctx->synth_mask) {
    SSP_TRY(ssp::sync_stream(ctx, "synthetic mask"));
    SSP_TRY_HIP(hipFree(ctx->synth_mask));
    ctx->synth_mask = nullptr;
  }
  // +1 element: the pair loads of an odd-length shard stay inside the table
  SSP_TRY_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->synth_mask), (a.n + 2) * sizeof(unsigned short)));
  ctx->synth_mask_n = a.n;
  ctx->synth_mask_offset = a.offset;
  ctx->synth_mask_seed = seed;
  ctx->synth_mask_rank = a.rank;
  if (a.n > 0) {
    synth_mask_kernel(ssp::stream_grid(ctx, a.n, 1), ctx->stream, a, ctx->synth_mask);
    SSP_TRY_HIP(hipGetLastError());
  }
  a.mask = ctx->synth_mask;
  return SSP_OK;
}

__global__ __launch_bounds__(kBlock) void k_synth_diag(double* d, size_t n, size_t offset, double rho, int rank,
                                                      int kind, double alpha) {
#pragma clang fp contract(off)
  const size_t stride = size_t(gridDim.x) * kBlock;
  for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    const unsigned long long g = offset + i;
    if (kind == SSPX_DIAG_BOUNDED) {
      const double t = 2.0 * frac_phi(g, kPhi2) - 1.0;
      const double s = alpha * t;
      d[i] = synth_d(kind, g) * (1.0 + s);
    } else {
      d[i] = 1.0 + double(g) + rank * rho;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_fill_random(double* x, size_t n, size_t offset, unsigned long long key) {
  const size_t stride = size_t(gridDim.x) * kBlock;
  for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    const unsigned long long h = splitmix64(key ^ (offset + i));
    x[i] = double(h >> 11) * (2.0 / 9007199254740992.0) - 1.0;
  }
}

struct DenseArgs {
  const double* a;
  size_t ng;
  const double* x[kMaxVec];
  double* y[kMaxVec];
  int nvec;
  size_t n;
  size_t offset;
};

// The fixture problems' H x: row sums in column order with every product rounded alone (the
// reference's test drivers' loop on x86-64), so that the parity fixtures see the same actions.
__global__ void k_dense_action(const DenseArgs p) {
#pragma clang fp contract(off)
  const size_t r = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= p.n) return;
  const double* row = p.a + (p.offset + r) * p.ng;
  for (int v = 0; v < p.nvec; ++v) {
    double s = 0;
    for (size_t j = 0; j < p.ng; ++j) s += row[j] * p.x[v][j];
    p.y[v][r] = s;
  }
}

}  // namespace

extern "C" {

int sspx_synth_action(ssp_ctx* ctx, const sspx_synth* spec, const double* const* xx, double* const* yy, int nvec,
                      size_t n, size_t offset) {
  return sspx_synth_action_scaled(ctx, spec, xx, nullptr, yy, nvec, n, offset);
}

int sspx_synth_action_scaled(ssp_ctx* ctx, const sspx_synth* spec, const double* const* xx, const double* xs,
                             double* const* yy, int nvec, size_t n, size_t offset) {
  SSP_CHECK_CTX(ctx);
  if (!spec) return ssp::set_error(SSP_ERR_ARG, "sspx_synth_action: null spec");
  const int rank = spec->rank;
  const unsigned long long seed = spec->seed;
  if (rank < 1 || rank > kMaxRank) return ssp::set_error(SSP_ERR_ARG, "sspx_synth_action: rank out of [1,16]");
  if (spec->diag_kind != SSPX_DIAG_LINEAR && spec->diag_kind != SSPX_DIAG_BOUNDED)
    return ssp::set_error(SSP_ERR_ARG, "sspx_synth_action: unknown diag_kind");
  if (nvec < 0) return ssp::set_error(SSP_ERR_ARG, "sspx_synth_action: nvec < 0");
  for (int v = 0; v < nvec; ++v)
    if (!aligned16(xx[v]) || !aligned16(yy[v]))
      return ssp::set_error(SSP_ERR_ARG, "sspx_synth_action: vectors must be 16-byte aligned");
  // x read twice (coefficients, then apply) and y written: 24 N per vector (the 2 B per element
  // sign table is not counted).
  ssp::LedgerScope ls(ctx, "action(synthetic)", 24.0 * n * nvec);
  for (int v0 = 0; v0 < nvec; v0 += kMaxVec) {
    SynthArgs a{};
    a.nvec = std::min(kMaxVec, nvec - v0);
    a.rank = rank;
    a.diag_kind = spec->diag_kind;
    a.n = n;
    a.offset = offset;
    a.rho = spec->rho;
    for (int v = 0; v < a.nvec; ++v) {
      a.x[v] = xx[v0 + v];
      a.xs[v] = xs ? xs[v0 + v] : 1.0;
      a.y[v] = yy[v0 + v];
    }
    for (int l = 0; l < rank; ++l) a.key[l] = stream_key(seed, 1000 + l);
    SSP_TRY(ensure_mask(ctx, a, seed));
    const int nc = a.nvec * rank;
    const unsigned grid = std::min<unsigned>(ssp::stream_grid(ctx, n, 4), 1024);
    SSP_TRY(ssp::ensure_partial(ctx, size_t(grid) * nc));
    SSP_TRY(ssp::ensure_result(ctx, nc));
    a.partial = ctx->partial;
    a.exact = ssp::exact_mode(ctx, n) ? 1 : 0;
    if (a.exact) {
      synth_coeff_exact(ctx->stream, a, ctx->result_dev);
      SSP_TRY_HIP(hipGetLastError());
    } else if (n > 0) {
      synth_coeff(grid, ctx->stream, a, ctx->synth_merge);
      SSP_TRY_HIP(hipGetLastError());
      SSP_TRY(ssp::launch_reduce_partials(ctx, ctx->partial, int(grid), 1, nc, ctx->result_dev, nc, 0, 0));
    } else {
      SSP_TRY_HIP(hipMemsetAsync(ctx->result_dev, 0, nc * sizeof(double), ctx->stream));
    }
    SSP_TRY(ssp::allreduce_dev(ctx, ctx->result_dev, nc));
    // The coefficients are consumed on the device straight from the result staging buffer: the next
    // reduction that rewrites it is queued after the apply kernel on the same stream.
    a.coeff = ctx->result_dev;
    if (n > 0) {
      synth_apply<false>(ctx, ctx->stream, a);
      SSP_TRY_HIP(hipGetLastError());
    }
  }
  return SSP_OK;
}

int sspx_synth_add_lowrank(ssp_ctx* ctx, const sspx_synth* spec, double* const* yy, int nvec, size_t n,
                           size_t offset, const double* w) {
  SSP_CHECK_CTX(ctx);
  if (!spec) return ssp::set_error(SSP_ERR_ARG, "sspx_synth_add_lowrank: null spec");
  const int rank = spec->rank;
  if (rank < 1 || rank > kMaxRank) return ssp::set_error(SSP_ERR_ARG, "sspx_synth_add_lowrank: rank out of [1,16]");
  if (n == 0 || nvec <= 0) return SSP_OK;
  for (int v = 0; v < nvec; ++v)
    if (!aligned16(yy[v])) return ssp::set_error(SSP_ERR_ARG, "sspx_synth_add_lowrank: vectors must be 16-byte aligned");
  ssp::LedgerScope ls(ctx, "p_action(synthetic)", 16.0 * n * nvec);
  for (int v0 = 0; v0 < nvec; v0 += kMaxVec) {
    SynthArgs a{};
    a.nvec = std::min(kMaxVec, nvec - v0);
    a.rank = rank;
    a.diag_kind = spec->diag_kind;
    a.n = n;
    a.offset = offset;
    a.rho = spec->rho;
    for (int v = 0; v < a.nvec; ++v) a.y[v] = yy[v0 + v];
    for (int l = 0; l < rank; ++l) a.key[l] = stream_key(spec->seed, 1000 + l);
    SSP_TRY(ensure_mask(ctx, a, spec->seed));
    void* coeff;
    SSP_TRY(ssp::upload_small(ctx, w + size_t(v0) * rank, size_t(a.nvec) * rank * sizeof(double), &coeff));
    a.coeff = static_cast<const double*>(coeff);
    a.exact = ssp::exact_mode(ctx, n) ? 1 : 0;
    SSP_TRY(ssp::flush_uploads(ctx));
    synth_apply<true>(ctx, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
  }
  return SSP_OK;
}

int sspx_synth_diagonal(ssp_ctx* ctx, const sspx_synth* spec, double* d, size_t n, size_t offset) {
  SSP_CHECK_CTX(ctx);
  if (!spec) return ssp::set_error(SSP_ERR_ARG, "sspx_synth_diagonal: null spec");
  if (n == 0) return SSP_OK;
  SSP_LAUNCH(k_synth_diag, dim3(ssp::stream_grid(ctx, n, 1)), dim3(kBlock), 0, ctx->stream, d, n, offset,
                     spec->rho, spec->rank, spec->diag_kind, spec->alpha);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

// The SSPX_DIAG_LINEAR entry points of round 1 (d_g = 1 + g).
int sspx_synthetic_action(ssp_ctx* ctx, const double* const* xx, double* const* yy, int nvec, size_t n, size_t offset,
                          double rho, int rank, unsigned long long seed) {
  const sspx_synth s{rho, rank, seed, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return sspx_synth_action(ctx, &s, xx, yy, nvec, n, offset);
}

int sspx_synthetic_add_lowrank(ssp_ctx* ctx, double* const* yy, int nvec, size_t n, size_t offset, double rho,
                               int rank, unsigned long long seed, const double* w) {
  const sspx_synth s{rho, rank, seed, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return sspx_synth_add_lowrank(ctx, &s, yy, nvec, n, offset, w);
}

int sspx_synthetic_diagonal(ssp_ctx* ctx, double* d, size_t n, size_t offset, double rho, int rank) {
  const sspx_synth s{rho, rank, 0, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return sspx_synth_diagonal(ctx, &s, d, n, offset);
}

int sspx_fill_random(ssp_ctx* ctx, double* x, size_t n, size_t offset, unsigned long long seed,
                     unsigned long long vec) {
  SSP_CHECK_CTX(ctx);
  if (n == 0) return SSP_OK;
  SSP_LAUNCH(k_fill_random, dim3(ssp::stream_grid(ctx, n, 1)), dim3(kBlock), 0, ctx->stream, x, n, offset,
                     stream_key(seed, vec));
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int sspx_dense_action(ssp_ctx* ctx, const double* a, size_t n_global, const double* const* xx, double* const* yy,
                      int nvec, size_t n, size_t offset) {
  SSP_CHECK_CTX(ctx);
  if (offset + n > n_global) return ssp::set_error(SSP_ERR_ARG, "sspx_dense_action: rows out of range");
  for (int v0 = 0; v0 < nvec; v0 += kMaxVec) {
    DenseArgs p{};
    p.a = a;
    p.ng = n_global;
    p.nvec = std::min(kMaxVec, nvec - v0);
    for (int v = 0; v < p.nvec; ++v) {
      p.x[v] = xx[v0 + v];
      p.y[v] = yy[v0 + v];
    }
    p.n = n;
    p.offset = offset;
    if (n > 0) {
      SSP_LAUNCH(k_dense_action, dim3(unsigned((n + 127) / 128)), dim3(128), 0, ctx->stream, p);
      SSP_TRY_HIP(hipGetLastError());
    }
  }
  return SSP_OK;
}

}  // extern "C"
