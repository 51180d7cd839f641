// Read path: register loads against LDS-DMA (global_load_lds_dwordx4) for the panel kernels'
// many-vector streams at N = 1e8 (development tool, not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_glds.hip -o tools/mb_glds
// Run:   tools/mb_glds [n=1e8] [s = read-pattern sweep | p = placement: default vs contiguous allocations | o = gemm_outer destination split, ow = wider windows | a = axpy/dot/fill access shapes]
//
// The question: MI355X_MICROARCH.md's ldsdma-fill row reads 6.5-6.8 TB/s chip-wide with nt LDS-DMA,
// against 6.3-6.4 TB/s for register loads (profiles/r1/mb_read_patterns.txt).  Does a 56-vector
// read (gemm_inner 8x48's stream set) or gemm_outer 48->8's sources gain from LDS-DMA?
//   reg   one wave per window of 1 KiB per vector, 4 vectors per load group, nt register loads
//   glds  each wave streams its pieces (1 KiB of one vector) through a private LDS ring, D pieces
//         in flight (counted vmcnt), consumes each piece with one ds_read_b128 per lane
//   oglds gemm_outer 48 -> 8 with the sources through the LDS ring, destinations in registers
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <functional>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld2nt(const double* p) {
  const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st2nt(double* p, double2 v) {
  d2v w = {v.x, v.y};
  __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(p));
}

struct Args {
  const double* x[64];
  double* y[16];
  size_t n;
  double alpha[384];
};

template <bool NT>
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

__device__ __forceinline__ double2 lds_rd(const char* p) {
  const d2v v = *reinterpret_cast<const d2v*>(p);
  return make_double2(v.x, v.y);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Register path: waves own 1 KiB x U windows, NV vectors in groups of B.
template <int U, int B = 4>
__global__ __launch_bounds__(256) void k_reg(const Args a, int nv, double* out) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t n2 = a.n >> 1, win = 64 * U;
  double s = 0;
  for (size_t c = gw; (c + 1) * win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
    for (int v = 0; v < nv; v += B) {
      double2 xv[B][U];
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ld2nt(a.x[v + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) s += xv[b][u].x + xv[b][u].y;
    }
  }
  if (s == 12345.678) out[0] = s;  // keep the loads
}

// gemm_inner's lane layout: lane l loads 16 B of vector 4g + (l & 3) at slot l >> 2, so one load
// instruction covers 4 vectors x 256 B.  A wave visit covers U consecutive 256 B chunks per vector
// (U x 256 B contiguous per vector), the 14 groups of 4 vectors one after the other.
template <int U>
__global__ __launch_bounds__(256) void k_quad(const Args a, int nv, double* out) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t win = 32 * U;  // elements per vector per visit
  double s = 0;
  for (size_t c = gw; (c + 1) * win <= a.n; c += nw) {
    const size_t e0 = c * win + 2 * (lane >> 2);
    for (int g = 0; g < nv / 4; ++g) {
      const double* x = a.x[4 * g + (lane & 3)];
      double2 xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u] = ld2nt(x + e0 + 32 * u);
#pragma unroll
      for (int u = 0; u < U; ++u) s += xv[u].x + xv[u].y;
    }
  }
  if (s == 12345.678) out[0] = s;
}

// Issue cursor of a wave's piece stream: piece = (window c, vector v), vectors fastest; slots
// advance round-robin through the ring.  Incremental (no 64-bit divisions in the loop).
template <int R, bool NT>
struct Cursor {
  const double* const* x;
  int nv, v = 0, slot = 0;
  size_t c, nw;
  unsigned base;
  __device__ __forceinline__ void issue(int lane) {
    glds16<NT>(x[v] + 2 * (c * 64 + lane), __builtin_amdgcn_readfirstlane(base + unsigned(slot) * 1024u));
    if (++v == nv) {
      v = 0;
      c += nw;
    }
    if (++slot == R) slot = 0;
  }
};

// LDS-DMA path: one wave per workgroup, private ring of R slots x 1 KiB, D pieces in flight.
template <int R, int D, bool NT>
__global__ __launch_bounds__(64) void k_glds(const Args a, int nv, double* out) {
  static_assert(R >= D + 1, "ring too small");
  __shared__ __attribute__((aligned(1024))) char ring[R * 1024];
  const int lane = threadIdx.x;
  const size_t gw = blockIdx.x, nw = gridDim.x;
  const size_t nwin = (a.n >> 1) / 64;  // whole 1 KiB windows
  const size_t mine = gw < nwin ? (nwin - gw + nw - 1) / nw : 0;
  const size_t T = mine * nv;
  Cursor<R, NT> cur{a.x, nv};
  cur.c = gw;
  cur.nw = nw;
  cur.base = static_cast<unsigned>(reinterpret_cast<uintptr_t>(ring));
  double s = 0;
  size_t t = 0;
  for (; t < D && t < T; ++t) cur.issue(lane);
  int rs = 0;
  for (t = 0; t + D < T; ++t) {
    wait_vm<D - 1>();
    const double2 v = lds_rd(ring + rs * 1024 + lane * 16);
    if (++rs == R) rs = 0;
    s += v.x + v.y;
    cur.issue(lane);
  }
  wait_vm<0>();
  for (; t < T; ++t) {
    const double2 v = lds_rd(ring + rs * 1024 + lane * 16);
    if (++rs == R) rs = 0;
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

// gemm_outer 48 -> 8 with sources through the LDS ring.  Per wave: windows of 1 KiB per vector
// (64 lanes x 16 B); destinations loaded to registers, the 48 sources stream through the ring
// D pieces ahead (the ring runs across window boundaries), destinations stored nt.  The
// destination loads are younger than the D glds in flight, so the first vmcnt(D-1) of a window
// retires them too (in-order counter).
template <int R, int D, bool NT>
__global__ __launch_bounds__(64) void k_oglds(const Args a) {
  constexpr int K = 48, M = 8;
  static_assert(R >= D + 1, "ring too small");
  __shared__ __attribute__((aligned(1024))) char ring[R * 1024];
  const int lane = threadIdx.x;
  const size_t gw = blockIdx.x, nw = gridDim.x;
  const size_t nwin = (a.n >> 1) / 64;
  const size_t mine = gw < nwin ? (nwin - gw + nw - 1) / nw : 0;
  const size_t T = mine * K;
  Cursor<R, NT> cur{a.x, K};
  cur.c = gw;
  cur.nw = nw;
  cur.base = static_cast<unsigned>(reinterpret_cast<uintptr_t>(ring));
  for (size_t t = 0; t < D && t < T; ++t) cur.issue(lane);
  size_t t = 0;
  int rs = 0;
  for (size_t w = 0; w < mine; ++w) {
    const size_t p = (gw + w * nw) * 64 + lane;
    double2 acc[M];
#pragma unroll
    for (int j = 0; j < M; ++j) acc[j] = ld2nt(a.y[j] + 2 * p);
    wait_vm<D - 1>();  // (conservative) the window's destinations
#pragma unroll 4
    for (int i = 0; i < K; ++i, ++t) {
      if (t + D < T)
        wait_vm<D - 1>();
      else
        wait_vm<0>();
      const double2 xv = lds_rd(ring + rs * 1024 + lane * 16);
      if (++rs == R) rs = 0;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        acc[j].x = fma(a.alpha[i * M + j], xv.x, acc[j].x);
        acc[j].y = fma(a.alpha[i * M + j], xv.y, acc[j].y);
      }
      if (t + D < T) cur.issue(lane);
    }
#pragma unroll
    for (int j = 0; j < M; ++j) st2nt(a.y[j] + 2 * p, acc[j]);
  }
}

// Library-form gemm_outer 48 -> 8 (U = 4 windows of 1 KiB per vector per wave, 4 sources per group).
__global__ __launch_bounds__(256) void k_outer_reg(const Args a);

// Wider windows: U KiB per vector per wave visit, B sources per load group (U = 8 needs the 512
// VGPRs of one wave per SIMD).
template <int U, int B>
__global__ __launch_bounds__(256) void k_outer_wide(const Args a) {
  constexpr int K = 48, M = 8;
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t n2 = a.n >> 1, win = 64 * U;
  for (size_t c = gw; (c + 1) * win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
    double2 acc[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) acc[u][j] = ld2nt(a.y[j] + 2 * (p0 + 64 * u));
    for (int i = 0; i < K; i += B) {
      double2 xv[B][U];
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ld2nt(a.x[i + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(a.alpha[(i + b) * M + j], xv[b][u].x, acc[u][j].x);
            acc[u][j].y = fma(a.alpha[(i + b) * M + j], xv[b][u].y, acc[u][j].y);
          }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) st2nt(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
  }
}

__global__ __launch_bounds__(256) void k_outer_reg(const Args a) {
  constexpr int K = 48, M = 8, U = 4;
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t n2 = a.n >> 1, win = 64 * U;
  for (size_t c = gw; (c + 1) * win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
    double2 acc[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) acc[u][j] = ld2nt(a.y[j] + 2 * (p0 + 64 * u));
    for (int i = 0; i < K; i += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ld2nt(a.x[i + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(a.alpha[(i + b) * M + j], xv[b][u].x, acc[u][j].x);
            acc[u][j].y = fma(a.alpha[(i + b) * M + j], xv[b][u].y, acc[u][j].y);
          }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) st2nt(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
  }
}

// Destinations split over the waves of a workgroup: the G = 8 / MW waves of a group share one 4 KiB
// window and each applies all 48 sources to its MW destinations (the sources' second and later
// reads of a window are meant to hit the CU's L1 / the XCD's L2).  Fewer accumulator registers per
// wave: more waves in flight per SIMD.
template <int MW>
__global__ __launch_bounds__(256) void k_outer_split(const Args a) {
  constexpr int K = 48, U = 4, G = 8 / MW, WPB = 4 / G;  // windows per block
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j0 = (wave % G) * MW;
  const size_t gw = size_t(blockIdx.x) * WPB + wave / G, nw = size_t(gridDim.x) * WPB;
  const size_t n2 = a.n >> 1, win = 64 * U;
  for (size_t c = gw; (c + 1) * win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
    double2 acc[U][MW];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < MW; ++j) acc[u][j] = ld2nt(a.y[j0 + j] + 2 * (p0 + 64 * u));
    for (int i = 0; i < K; i += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = *reinterpret_cast<const double2*>(a.x[i + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < MW; ++j)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(a.alpha[(i + b) * 8 + j0 + j], xv[b][u].x, acc[u][j].x);
            acc[u][j].y = fma(a.alpha[(i + b) * 8 + j0 + j], xv[b][u].y, acc[u][j].y);
          }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < MW; ++j) st2nt(a.y[j0 + j] + 2 * (p0 + 64 * u), acc[u][j]);
  }
}

// Streaming kernels, two access shapes: "stride" (the library's k_axpy: 4 double2 per lane spaced a
// whole grid apart) and "win" (each wave owns U consecutive KiB of every vector per visit).
__global__ __launch_bounds__(256) void k_axpy_stride(const double* __restrict__ x, double* __restrict__ y, size_t n,
                                                     double alpha) {
  const size_t n2 = n >> 1, stride = size_t(gridDim.x) * 256;
  size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    double2 x0 = ld2nt(x + 2 * i), x1 = ld2nt(x + 2 * (i + stride)), x2 = ld2nt(x + 2 * (i + 2 * stride)),
            x3 = ld2nt(x + 2 * (i + 3 * stride));
    double2 y0 = ld2nt(y + 2 * i), y1 = ld2nt(y + 2 * (i + stride)), y2 = ld2nt(y + 2 * (i + 2 * stride)),
            y3 = ld2nt(y + 2 * (i + 3 * stride));
    st2nt(y + 2 * i, make_double2(fma(alpha, x0.x, y0.x), fma(alpha, x0.y, y0.y)));
    st2nt(y + 2 * (i + stride), make_double2(fma(alpha, x1.x, y1.x), fma(alpha, x1.y, y1.y)));
    st2nt(y + 2 * (i + 2 * stride), make_double2(fma(alpha, x2.x, y2.x), fma(alpha, x2.y, y2.y)));
    st2nt(y + 2 * (i + 3 * stride), make_double2(fma(alpha, x3.x, y3.x), fma(alpha, x3.y, y3.y)));
  }
  for (; i < n2; i += stride) {
    double2 a = ld2nt(x + 2 * i), b = ld2nt(y + 2 * i);
    st2nt(y + 2 * i, make_double2(fma(alpha, a.x, b.x), fma(alpha, a.y, b.y)));
  }
}

template <int U>
__global__ __launch_bounds__(256) void k_axpy_win(const double* __restrict__ x, double* __restrict__ y, size_t n,
                                                  double alpha) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t n2 = n >> 1, win = 64 * U;
  for (size_t c = gw; (c + 1) * win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
    double2 xv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = ld2nt(x + 2 * (p0 + 64 * u));
#pragma unroll
    for (int u = 0; u < U; ++u) yv[u] = ld2nt(y + 2 * (p0 + 64 * u));
#pragma unroll
    for (int u = 0; u < U; ++u)
      st2nt(y + 2 * (p0 + 64 * u), make_double2(fma(alpha, xv[u].x, yv[u].x), fma(alpha, xv[u].y, yv[u].y)));
  }
}

template <int U>
__global__ __launch_bounds__(256) void k_dot_win(const double* __restrict__ x, size_t n, double* out) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t n2 = n >> 1, win = 64 * U;
  double s = 0;
  for (size_t c = gw; (c + 1) * win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
    double2 xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = ld2nt(x + 2 * (p0 + 64 * u));
#pragma unroll
    for (int u = 0; u < U; ++u) s = fma(xv[u].x, xv[u].x, fma(xv[u].y, xv[u].y, s));
  }
  if (s == 12345.678) out[0] = s;
}

__global__ __launch_bounds__(256) void k_dot_stride(const double* __restrict__ x, size_t n, double* out) {
  const size_t n2 = n >> 1, stride = size_t(gridDim.x) * 256;
  size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    double2 x0 = ld2nt(x + 2 * i), x1 = ld2nt(x + 2 * (i + stride)), x2 = ld2nt(x + 2 * (i + 2 * stride)),
            x3 = ld2nt(x + 2 * (i + 3 * stride));
    s0 = fma(x0.x, x0.x, fma(x0.y, x0.y, s0));
    s1 = fma(x1.x, x1.x, fma(x1.y, x1.y, s1));
    s2 = fma(x2.x, x2.x, fma(x2.y, x2.y, s2));
    s3 = fma(x3.x, x3.x, fma(x3.y, x3.y, s3));
  }
  const double s = (s0 + s1) + (s2 + s3);
  if (s == 12345.678) out[0] = s;
}

template <int U>
__global__ __launch_bounds__(256) void k_fill_win(double* __restrict__ x, size_t n, double alpha) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t n2 = n >> 1, win = 64 * U;
  for (size_t c = gw; (c + 1) * win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
#pragma unroll
    for (int u = 0; u < U; ++u) *reinterpret_cast<double2*>(x + 2 * (p0 + 64 * u)) = make_double2(alpha, alpha);
  }
}

__global__ __launch_bounds__(256) void k_fill_stride(double* __restrict__ x, size_t n, double alpha) {
  const size_t n2 = n >> 1, stride = size_t(gridDim.x) * 256;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n2; i += stride)
    *reinterpret_cast<double2*>(x + 2 * i) = make_double2(alpha, alpha);
}

__global__ void k_init(double* x, size_t n, unsigned seed) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    x[i] = double((i * 2654435761u + seed) % 1000) * 1e-3 - 0.5;
}

float timeit(const std::function<void()>& f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? size_t(atof(argv[1])) : 100000000;
  if (n % 128) {
    printf("n must be a multiple of 128\n");
    return 1;
  }
  constexpr int NV = 56;
  double* vec[NV];
  for (int i = 0; i < NV; ++i) {
    CK(hipMalloc((void**)&vec[i], n * 8));
    hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, vec[i], n, unsigned(i));
  }
  CK(hipDeviceSynchronize());
  double* out;
  CK(hipMalloc((void**)&out, 64));
  Args a{};
  a.n = n;
  for (int i = 0; i < NV; ++i) a.x[i] = vec[i];
  Args o{};  // gemm_outer: sources vec[8..55], destinations vec[0..7]
  o.n = n;
  for (int i = 0; i < 48; ++i) o.x[i] = vec[8 + i];
  for (int j = 0; j < 8; ++j) o.y[j] = vec[j];
  for (int i = 0; i < 384; ++i) o.alpha[i] = 1e-6 * (i % 17);
  auto rep = [&](const char* name, int g, float ms, double bytes) {
    printf("%-26s g=%-6d %8.3f ms  %7.1f GB/s\n", name, g, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
  const int reps = 7;
  const double rb = 8.0 * n * NV, ob = 8.0 * n * (48 + 16);
  if (argc > 2 && argv[2][0] == 'a') {
    // Streaming ops (axpy, self-dot, fill) on 100 MB / 800 MB vectors, stride vs window shapes.
    for (size_t nn : {n / 8, n}) {
      char nm[64];
      const double ab = 24.0 * nn, db = 8.0 * nn, fb = 8.0 * nn;
      for (int set = 0; set < 2; ++set) {
        double* xv = vec[2 * set];
        double* yv = vec[2 * set + 1];
        for (int g : {2048, 8192, 16384}) {
          snprintf(nm, 64, "n=%.3g axpy stride", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL(k_axpy_stride, dim3(g), dim3(256), 0, 0, xv, yv, nn, 1e-9); }, reps), ab);
        }
        for (int g : {1024, 2048, 4096}) {
          snprintf(nm, 64, "n=%.3g axpy win U4", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_axpy_win<4>), dim3(g), dim3(256), 0, 0, xv, yv, nn, 1e-9); }, reps), ab);
          snprintf(nm, 64, "n=%.3g axpy win U8", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_axpy_win<8>), dim3(g), dim3(256), 0, 0, xv, yv, nn, 1e-9); }, reps), ab);
        }
        for (int g : {1024, 2048}) {
          snprintf(nm, 64, "n=%.3g dot stride", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL(k_dot_stride, dim3(g), dim3(256), 0, 0, xv, nn, out); }, reps), db);
          snprintf(nm, 64, "n=%.3g dot win U4", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_dot_win<4>), dim3(g), dim3(256), 0, 0, xv, nn, out); }, reps), db);
          snprintf(nm, 64, "n=%.3g dot win U8", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_dot_win<8>), dim3(g), dim3(256), 0, 0, xv, nn, out); }, reps), db);
        }
        for (int g : {4096, 16384}) {
          snprintf(nm, 64, "n=%.3g fill stride", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL(k_fill_stride, dim3(g), dim3(256), 0, 0, yv, nn, 0.5); }, reps), fb);
        }
        for (int g : {1024, 2048, 4096}) {
          snprintf(nm, 64, "n=%.3g fill win U4", double(nn));
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_fill_win<4>), dim3(g), dim3(256), 0, 0, yv, nn, 0.5); }, reps), fb);
        }
      }
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'o') {
    // gemm_outer 48 -> 8: library form against destination-split forms, over fresh vector sets.
    for (int set = 0; set < 4; ++set) {
      if (set) {
        for (int i = 0; i < NV; ++i) CK(hipFree(vec[i]));
        for (int i = 0; i < NV; ++i) {
          CK(hipMalloc((void**)&vec[i], n * 8));
          hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, vec[i], n, unsigned(i));
        }
        CK(hipDeviceSynchronize());
        for (int i = 0; i < 48; ++i) o.x[i] = vec[8 + i];
        for (int j = 0; j < 8; ++j) o.y[j] = vec[j];
      }
      printf("-- set %d\n", set);
      for (int g : {1024, 2048}) {
        rep("outer reg U4 (library)", g, timeit([&] { hipLaunchKernelGGL(k_outer_reg, dim3(g), dim3(256), 0, 0, o); }, reps), ob);
        if (argv[2][1] == 'w') {
          rep("outer wide U6 B4", g, timeit([&] { hipLaunchKernelGGL((k_outer_wide<6, 4>), dim3(g), dim3(256), 0, 0, o); }, reps), ob);
          rep("outer wide U8 B2", g, timeit([&] { hipLaunchKernelGGL((k_outer_wide<8, 2>), dim3(g), dim3(256), 0, 0, o); }, reps), ob);
          rep("outer wide U8 B4", g, timeit([&] { hipLaunchKernelGGL((k_outer_wide<8, 4>), dim3(g), dim3(256), 0, 0, o); }, reps), ob);
          rep("outer wide U4 B2", g, timeit([&] { hipLaunchKernelGGL((k_outer_wide<4, 2>), dim3(g), dim3(256), 0, 0, o); }, reps), ob);
          continue;
        }
        rep("outer split 4 dst/wave", g, timeit([&] { hipLaunchKernelGGL((k_outer_split<4>), dim3(g), dim3(256), 0, 0, o); }, reps), ob);
        rep("outer split 2 dst/wave", g, timeit([&] { hipLaunchKernelGGL((k_outer_split<2>), dim3(g), dim3(256), 0, 0, o); }, reps), ob);
      }
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'p') {
    // Placement: the same kernels over freshly allocated vector sets, default hipMalloc against
    // hipExtMallocWithFlags(hipDeviceMallocContiguous), alternating.
    for (int i = 0; i < NV; ++i) CK(hipFree(vec[i]));
    for (int set = 0; set < 8; ++set) {
      const bool contig = set & 1;
      bool ok = true;
      for (int i = 0; i < NV; ++i) {
        hipError_t e = contig ? hipExtMallocWithFlags((void**)&vec[i], n * 8, hipDeviceMallocContiguous)
                              : hipMalloc((void**)&vec[i], n * 8);
        if (e != hipSuccess) {
          printf("set %d: allocation %d failed: %s\n", set, i, hipGetErrorString(e));
          for (int j = 0; j < i; ++j) CK(hipFree(vec[j]));
          ok = false;
          break;
        }
        hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, vec[i], n, unsigned(i));
      }
      (void)hipGetLastError();
      if (!ok) continue;
      CK(hipDeviceSynchronize());
      for (int i = 0; i < NV; ++i) a.x[i] = vec[i];
      for (int i = 0; i < 48; ++i) o.x[i] = vec[8 + i];
      for (int j = 0; j < 8; ++j) o.y[j] = vec[j];
      char nm[64];
      snprintf(nm, 64, "set %d %s outer", set, contig ? "contig " : "default");
      rep(nm, 2048, timeit([&] { hipLaunchKernelGGL(k_outer_reg, dim3(2048), dim3(256), 0, 0, o); }, reps), ob);
      snprintf(nm, 64, "set %d %s read56", set, contig ? "contig " : "default");
      rep(nm, 2048, timeit([&] { hipLaunchKernelGGL((k_reg<4, 4>), dim3(2048), dim3(256), 0, 0, a, NV, out); }, reps), rb);
      snprintf(nm, 64, "set %d %s quad", set, contig ? "contig " : "default");
      rep(nm, 2048, timeit([&] { hipLaunchKernelGGL((k_quad<1>), dim3(2048), dim3(256), 0, 0, a, NV, out); }, reps), rb);
      for (int i = 0; i < NV; ++i) CK(hipFree(vec[i]));
    }
    return 0;
  }
  const bool sweep = argc > 2 && argv[2][0] == 's';
  for (int round = 0; round < 2; ++round) {
    if (sweep) {
      for (int g : {1024, 2048}) {
        rep("read56 reg U1 B4", g, timeit([&] { hipLaunchKernelGGL((k_reg<1, 4>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 reg U2 B4", g, timeit([&] { hipLaunchKernelGGL((k_reg<2, 4>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 reg U4 B4", g, timeit([&] { hipLaunchKernelGGL((k_reg<4, 4>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 reg U8 B2", g, timeit([&] { hipLaunchKernelGGL((k_reg<8, 2>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 reg U8 B4", g, timeit([&] { hipLaunchKernelGGL((k_reg<8, 4>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 reg U4 B8", g, timeit([&] { hipLaunchKernelGGL((k_reg<4, 8>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 reg U16 B1", g, timeit([&] { hipLaunchKernelGGL((k_reg<16, 1>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 quad U1", g, timeit([&] { hipLaunchKernelGGL((k_quad<1>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 quad U4", g, timeit([&] { hipLaunchKernelGGL((k_quad<4>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 quad U8", g, timeit([&] { hipLaunchKernelGGL((k_quad<8>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
        rep("read56 quad U16", g, timeit([&] { hipLaunchKernelGGL((k_quad<16>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
      }
      continue;
    }
    for (int g : {1024, 2048}) rep("read56 reg U1", g, timeit([&] { hipLaunchKernelGGL((k_reg<1>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
    for (int g : {1024, 2048}) rep("read56 reg U4", g, timeit([&] { hipLaunchKernelGGL((k_reg<4>), dim3(g), dim3(256), 0, 0, a, NV, out); }, reps), rb);
    // one wave per workgroup: 256 CUs x {4, 8, 16} waves
    for (int g : {1024, 2048, 4096}) {
      rep("read56 glds R10 D8 nt", g, timeit([&] { hipLaunchKernelGGL((k_glds<10, 8, true>), dim3(g), dim3(64), 0, 0, a, NV, out); }, reps), rb);
      rep("read56 glds R10 D8", g, timeit([&] { hipLaunchKernelGGL((k_glds<10, 8, false>), dim3(g), dim3(64), 0, 0, a, NV, out); }, reps), rb);
      rep("read56 glds R18 D16 nt", g, timeit([&] { hipLaunchKernelGGL((k_glds<18, 16, true>), dim3(g), dim3(64), 0, 0, a, NV, out); }, reps), rb);
      rep("read56 glds R34 D32 nt", g, timeit([&] { hipLaunchKernelGGL((k_glds<34, 32, true>), dim3(g), dim3(64), 0, 0, a, NV, out); }, reps), rb);
    }
    for (int g : {1024, 2048}) rep("outer reg U4 (library)", g, timeit([&] { hipLaunchKernelGGL(k_outer_reg, dim3(g), dim3(256), 0, 0, o); }, reps), ob);
    for (int g : {1024, 2048, 4096}) {
      rep("outer glds R18 D16 nt", g, timeit([&] { hipLaunchKernelGGL((k_oglds<18, 16, true>), dim3(g), dim3(64), 0, 0, o); }, reps), ob);
      rep("outer glds R34 D32 nt", g, timeit([&] { hipLaunchKernelGGL((k_oglds<34, 32, true>), dim3(g), dim3(64), 0, 0, o); }, reps), ob);
    }
  }
  return 0;
}
