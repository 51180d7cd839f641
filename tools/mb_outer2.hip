// gemm_outer (48 -> 8, N = 1e8) work-distribution and pipelining variants against read / copy
// ceilings measured in the same process (development tool, not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_outer2.hip -o tools/mb_outer2
// Run:   tools/mb_outer2 [n=1e8]
//
// Variants (all: 4 sources x U windows of 64 lanes x 16 B per load group, nontemporal access,
// sources applied in order i = 0..k-1 as the library kernel does):
//   stride  grid-stride wave windows (the library's k_gemm_outer<8>)
//   contig  each wave owns one contiguous run of windows
//   xcd     blocks remapped so each XCD (blockIdx % 8) sweeps its own contiguous eighth of N,
//           grid-stride inside the eighth
//   pipe    stride + explicit double buffering of the next 4-source group
//   set     stride without reading the destinations (the fused construct_solution form)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr int M = 8, K = 48;
struct OArgs {
  const double* x[64];
  double* y[16];
  size_t n;
  double alpha[384];
};

// One window: destinations loaded (unless SET), K sources in groups of 4, stores.
template <int U, bool SET, bool PIPE>
__device__ __forceinline__ void window(const OArgs& a, size_t p0) {
  double2 acc[U][M];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < M; ++j) acc[u][j] = SET ? make_double2(0, 0) : ld2nt(a.y[j] + 2 * (p0 + 64 * u));
  if constexpr (!PIPE) {
#pragma unroll 1
    for (int i = 0; i < K; i += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ld2nt(a.x[i + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const double al = a.alpha[(i + b) * M + j];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(al, xv[b][u].x, acc[u][j].x);
            acc[u][j].y = fma(al, xv[b][u].y, acc[u][j].y);
          }
        }
    }
  } else {
    double2 cur[4][U], nxt[4][U];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int u = 0; u < U; ++u) cur[b][u] = ld2nt(a.x[b] + 2 * (p0 + 64 * u));
#pragma unroll 1
    for (int i = 0; i < K; i += 4) {
      if (i + 4 < K) {
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int u = 0; u < U; ++u) nxt[b][u] = ld2nt(a.x[i + 4 + b] + 2 * (p0 + 64 * u));
      }
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const double al = a.alpha[(i + b) * M + j];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(al, cur[b][u].x, acc[u][j].x);
            acc[u][j].y = fma(al, cur[b][u].y, acc[u][j].y);
          }
        }
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) cur[b][u] = nxt[b][u];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < M; ++j) st2nt(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
}

// n2 is a multiple of 64 * U * waves in every run below (no tails).
template <int U, bool SET, bool PIPE>
__global__ __launch_bounds__(256) void k_stride(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t nwin = (a.n >> 1) / (64 * U);
  for (size_t c = gw; c < nwin; c += nw) window<U, SET, PIPE>(a, c * 64 * U + lane);
}

template <int U>
__global__ __launch_bounds__(256) void k_contig(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t nwin = (a.n >> 1) / (64 * U);
  const size_t per = (nwin + nw - 1) / nw, c0 = gw * per, c1 = std::min(nwin, c0 + per);
  for (size_t c = c0; c < c1; ++c) window<U, false, false>(a, c * 64 * U + lane);
}

template <int U>
__global__ __launch_bounds__(256) void k_xcd(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const unsigned xcd = blockIdx.x & 7, bx = blockIdx.x >> 3, nbx = gridDim.x >> 3;
  const size_t nwin = (a.n >> 1) / (64 * U);
  const size_t per = (nwin + 7) / 8, c0 = xcd * per, c1 = std::min(nwin, c0 + per);
  const size_t gw = size_t(bx) * 4 + (threadIdx.x >> 6), nw = size_t(nbx) * 4;
  for (size_t c = c0 + gw; c < c1; c += nw) window<U, false, false>(a, c * 64 * U + lane);
}

__global__ __launch_bounds__(256) void k_read(const OArgs a, int nv, double* out) {
  const size_t n2 = a.n >> 1, stride = size_t(gridDim.x) * 256;
  double s = 0;
  for (size_t p = size_t(blockIdx.x) * 256 + threadIdx.x; p < n2; p += stride)
    for (int v = 0; v < nv; ++v) {
      const double2 x = ld2nt(a.x[v] + 2 * p);
      s += x.x + x.y;
    }
  if (s == 12345.678) out[0] = s;
}


// Read-pattern probes: R (1 position per lane, vectors in order), RW (U positions per lane, 4 sources x U
// loads in flight), with OCC-limiting dynamic LDS when asked.
template <int U, int B>
__global__ __launch_bounds__(256) void k_readw(const OArgs a, int nv, double* out) {
  extern __shared__ double pad[];
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t nwin = (a.n >> 1) / (64 * U);
  double s = 0;
  for (size_t c = gw; c < nwin; c += nw) {
    const size_t p0 = c * 64 * U + lane;
    for (int v = 0; v < nv; v += B) {
      double2 xv[B][U];
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ld2nt(a.x[v + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) s += xv[b][u].x * xv[b][u].y;
    }
  }
  if (s == 12345.678) out[0] = s + pad[0];
}


// Read:write mix probe: R vectors read, W vectors written per position (values: sums of the reads),
// U positions per lane, all loads of a window before the stores; NT stores or plain.
template <int R, int W, int U, bool NTS>
__global__ __launch_bounds__(256) void k_mix(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t nwin = (a.n >> 1) / (64 * U);
  for (size_t c = gw; c < nwin; c += nw) {
    const size_t p0 = c * 64 * U + lane;
    double2 s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = make_double2(0, 0);
#pragma unroll
    for (int v = 0; v < R; v += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ld2nt(a.x[v + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          s[u].x += xv[b][u].x;
          s[u].y += xv[b][u].y;
        }
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double2 o = make_double2(s[u].x * (w + 1), s[u].y);
        if (NTS) st2nt(a.y[w] + 2 * (p0 + 64 * u), o);
        else *reinterpret_cast<double2*>(a.y[w] + 2 * (p0 + 64 * u)) = o;
      }
  }
}

__global__ __launch_bounds__(256) void k_copy(const double* x, double* y, size_t n) {
  const size_t n2 = n >> 1, stride = size_t(gridDim.x) * 256 * 4;
  for (size_t p = size_t(blockIdx.x) * 1024 + threadIdx.x; p < n2; p += stride) {
    double2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p + 256 * u < n2 ? ld2nt(x + 2 * (p + 256 * u)) : make_double2(0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (p + 256 * u < n2) st2nt(y + 2 * (p + 256 * u), v[u]);
  }
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
  double* vec[64];
  for (int i = 0; i < M + K; ++i) {
    CK(hipMalloc((void**)&vec[i], n * 8));
    CK(hipMemset(vec[i], 0, n * 8));
  }
  double* out;
  CK(hipMalloc((void**)&out, 64));
  OArgs a{};
  a.n = n;
  for (int i = 0; i < K; ++i) a.x[i] = vec[M + i];
  for (int j = 0; j < M; ++j) a.y[j] = vec[j];
  for (int i = 0; i < K * M; ++i) a.alpha[i] = 1e-3 * (i % 17);
  const double ob = 8.0 * n * (K + 2 * M), sb = 8.0 * n * (K + M);
  auto rep = [&](const char* name, int g, float ms, double bytes) {
    printf("%-22s g=%-6d %8.3f ms  %7.1f GB/s\n", name, g, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
  const int reps = 7;
  for (int i = K; i < 56; ++i) a.x[i] = vec[i - K];  // 56 read vectors: the 48 sources + the 8 destinations
  if (argc > 2 && argv[2][0] == 'm') {
    for (int round = 0; round < 2; ++round)
      for (int g : {1024, 2048}) {
        rep("mix 56r 8w U4 nt", g, timeit([&] { hipLaunchKernelGGL((k_mix<56, 8, 4, true>), dim3(g), dim3(256), 0, 0, a); }, reps), 8.0 * n * 64);
        rep("mix 56r 8w U4 plain", g, timeit([&] { hipLaunchKernelGGL((k_mix<56, 8, 4, false>), dim3(g), dim3(256), 0, 0, a); }, reps), 8.0 * n * 64);
        rep("mix 56r 8w U1 nt", g, timeit([&] { hipLaunchKernelGGL((k_mix<56, 8, 1, true>), dim3(g), dim3(256), 0, 0, a); }, reps), 8.0 * n * 64);
        rep("mix 48r 8w U4 nt", g, timeit([&] { hipLaunchKernelGGL((k_mix<48, 8, 4, true>), dim3(g), dim3(256), 0, 0, a); }, reps), 8.0 * n * 56);
        rep("mix 8r 1w U4 nt", g, timeit([&] { hipLaunchKernelGGL((k_mix<8, 1, 4, true>), dim3(g), dim3(256), 0, 0, a); }, reps), 8.0 * n * 9);
        rep("mix 4r 4w U4 nt", g, timeit([&] { hipLaunchKernelGGL((k_mix<4, 4, 4, true>), dim3(g), dim3(256), 0, 0, a); }, reps), 8.0 * n * 8);
        rep("mix 4r 1w U4 nt", g, timeit([&] { hipLaunchKernelGGL((k_mix<4, 1, 4, true>), dim3(g), dim3(256), 0, 0, a); }, reps), 8.0 * n * 5);
        rep("stride U4 (outer)", g, timeit([&] { hipLaunchKernelGGL((k_stride<4, false, false>), dim3(g), dim3(256), 0, 0, a); }, reps), ob);
      }
    return 0;
  }
  if (argc > 2) {
    for (int round = 0; round < 2; ++round) {
      for (int nv : {48, 56}) {
        char nm[64];
        for (int g : {1024, 2048, 4096}) {
          snprintf(nm, 64, "read%d U1", nv);
          rep(nm, g, timeit([&] { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, a, nv, out); }, reps), 8.0 * n * nv);
          snprintf(nm, 64, "readw%d U1 B4", nv);
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_readw<1, 4>), dim3(g), dim3(256), 0, 0, a, nv, out); }, reps), 8.0 * n * nv);
          snprintf(nm, 64, "readw%d U4 B4", nv);
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_readw<4, 4>), dim3(g), dim3(256), 0, 0, a, nv, out); }, reps), 8.0 * n * nv);
          snprintf(nm, 64, "readw%d U4 B4 occ2", nv);
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_readw<4, 4>), dim3(g), dim3(256), 64 << 10, 0, a, nv, out); }, reps), 8.0 * n * nv);
          snprintf(nm, 64, "readw%d U2 B8", nv);
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_readw<2, 8>), dim3(g), dim3(256), 0, 0, a, nv, out); }, reps), 8.0 * n * nv);
          snprintf(nm, 64, "readw%d U1 B8 occ2", nv);
          rep(nm, g, timeit([&] { hipLaunchKernelGGL((k_readw<1, 8>), dim3(g), dim3(256), 64 << 10, 0, a, nv, out); }, reps), 8.0 * n * nv);
        }
      }
    }
    return 0;
  }
  for (int round = 0; round < 2; ++round) {
    for (int g : {512, 1024, 2048, 4096}) {
      rep("stride U4", g, timeit([&] { hipLaunchKernelGGL((k_stride<4, false, false>), dim3(g), dim3(256), 0, 0, a); }, reps), ob);
      rep("stride U2", g, timeit([&] { hipLaunchKernelGGL((k_stride<2, false, false>), dim3(g), dim3(256), 0, 0, a); }, reps), ob);
      rep("pipe U2", g, timeit([&] { hipLaunchKernelGGL((k_stride<2, false, true>), dim3(g), dim3(256), 0, 0, a); }, reps), ob);
      rep("contig U4", g, timeit([&] { hipLaunchKernelGGL((k_contig<4>), dim3(g), dim3(256), 0, 0, a); }, reps), ob);
      rep("xcd U4", g, timeit([&] { hipLaunchKernelGGL((k_xcd<4>), dim3(g), dim3(256), 0, 0, a); }, reps), ob);
      rep("set U4", g, timeit([&] { hipLaunchKernelGGL((k_stride<4, true, false>), dim3(g), dim3(256), 0, 0, a); }, reps), sb);
    }
    rep("read 48 vectors", 2048, timeit([&] { hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, 0, a, 48, out); }, reps), 8.0 * n * 48);
    rep("copy", 4096, timeit([&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, vec[M], vec[0], n); }, reps), 16.0 * n);
  }
  return 0;
}
