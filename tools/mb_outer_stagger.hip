// gemm_outer (48 -> 8, N = 1e8) and the 56-vector read against the start offset of each vector
// within its allocation (development tool, not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_outer_stagger.hip -o tools/mb_outer_stagger
// Run:   tools/mb_outer_stagger [n=1e8] [sets=3]
//
// Every large vector is its own hipMalloc (as the library's arena does); vector v of a set starts
// v * S bytes into its allocation.  S = 0 is the library's layout.  The earlier slab experiment
// (profiles/r1/mb_outer_slab_stagger.txt) staggered by whole MiB only; this one probes sub-2-MiB
// offsets, which change the low address bits of the 64 streams a wave window touches together.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr int M = 8, K = 48, U = 4, BLOCK = 256;
struct OArgs {
  const double* x[K];
  double* y[M];
  size_t n;
  double alpha[K * M];
};

__global__ __launch_bounds__(BLOCK) void k_outer(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * (BLOCK / 64) + (threadIdx.x >> 6);
  const size_t nw = size_t(gridDim.x) * (BLOCK / 64);
  const size_t n2 = a.n >> 1, win = 64 * U;
  for (size_t c = gw; c * win + win <= n2; c += nw) {
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
        for (int j = 0; j < M; ++j) {
          const double al = a.alpha[(i + b) * M + j];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(al, xv[b][u].x, acc[u][j].x);
            acc[u][j].y = fma(al, xv[b][u].y, acc[u][j].y);
          }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) st2nt(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
  }
}

struct RArgs {
  const double* x[K + M];
  size_t n;
  double* out;
};

__global__ __launch_bounds__(BLOCK) void k_read(const RArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * (BLOCK / 64) + (threadIdx.x >> 6);
  const size_t nw = size_t(gridDim.x) * (BLOCK / 64);
  const size_t n2 = a.n >> 1, win = 64 * U;
  double s = 0;
  for (size_t c = gw; c * win + win <= n2; c += nw) {
    const size_t p0 = c * win + lane;
    for (int i = 0; i < K + M; i += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ld2nt(a.x[i + b] + 2 * (p0 + 64 * u));
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) s += xv[b][u].x * xv[b][u].y;
    }
  }
  if (s == 12345.678) a.out[0] = s;  // keeps the loads
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? size_t(atof(argv[1])) : size_t(1e8);
  const int sets = argc > 2 ? atoi(argv[2]) : 3;
  const size_t bytes = n * 8;
  const size_t strides[] = {0, 256, 4096, 4096 + 256, 65536 + 4096, 262144 + 4096, 1048576 + 4096};
  const size_t pad = 64 * (1048576 + 4096) + 4096;
  double* out;
  CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 2048;
  for (int set = 0; set < sets; ++set) {
    std::vector<char*> base(K + M);
    for (auto& b : base) {
      CK(hipMalloc(&b, bytes + pad));
      CK(hipMemset(b, 0, bytes + pad));
    }
    for (size_t st : strides) {
      OArgs oa{};
      RArgs ra{};
      for (int v = 0; v < K + M; ++v) {
        double* p = reinterpret_cast<double*>(base[v] + v * st);
        if (v < K) oa.x[v] = p; else oa.y[v - K] = p;
        ra.x[v] = p;
      }
      oa.n = ra.n = n;
      for (int i = 0; i < K * M; ++i) oa.alpha[i] = 1e-3 * (i % 7);
      ra.out = out;
      float best_o = 1e30f, best_r = 1e30f, med[2][5];
      for (int rep = 0; rep < 5; ++rep) {
        float ms;
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_outer, dim3(grid), dim3(BLOCK), 0, 0, oa);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        med[0][rep] = ms;
        best_o = std::min(best_o, ms);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(BLOCK), 0, 0, ra);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        med[1][rep] = ms;
        best_r = std::min(best_r, ms);
      }
      std::sort(med[0], med[0] + 5);
      std::sort(med[1], med[1] + 5);
      const double ob = 8.0 * n * (K + 2 * M), rb = 8.0 * n * (K + M);
      printf("set %d stagger %8zu B  outer %7.3f ms %7.1f GB/s   read56 %7.3f ms %7.1f GB/s\n", set, st, med[0][2],
             ob / med[0][2] / 1e6, med[1][2], rb / med[1][2] / 1e6);
      fflush(stdout);
    }
    for (auto b : base) CK(hipFree(b));
  }
  return 0;
}
