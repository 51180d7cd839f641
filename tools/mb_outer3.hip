// gemm_outer (48 -> 8, N = 1e8, read-modify-write) cache-policy and scheduling variants, round 3
// (development tool, not part of the library).  Variants of the library's window shape (4 sources x
// U = 4 windows of 64 lanes x 16 B per load group, sources applied in order):
//   DL  destination loads   0 nontemporal (library) | 1 plain (lines stay in L2 for the store)
//   ST  stores              0 nontemporal (library) | 1 plain (L2 write-back)
//   SL  source loads        0 nontemporal (library) | 1 plain
//   SY  1: the 4 waves of a workgroup (adjacent windows, 16 KiB contiguous per vector) step through
//       the source groups in lockstep (a barrier per group)
// plus grid sizes (the library launches 8 workgroups per CU; 2 are resident at 200 VGPRs).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_outer3.hip -o tools/mb_outer3
// Run:   tools/mb_outer3 [n=1e8]
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
template <int NT>
__device__ __forceinline__ double2 ld2(const double* p) {
  if constexpr (NT == 0) {
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
  } else {
    return *reinterpret_cast<const double2*>(p);
  }
}
template <int NT>
__device__ __forceinline__ void st2(double* p, double2 v) {
  if constexpr (NT == 0) {
    d2v w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(p));
  } else {
    *reinterpret_cast<double2*>(p) = v;
  }
}

constexpr int M = 8, K = 48, U = 4;
struct OArgs {
  const double* x[48];
  double* y[8];
  size_t n;
  double alpha[384];
};

template <int DL, int ST, int SL, int SY>
__global__ __launch_bounds__(256) void k_outer(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t nwin = (a.n >> 1) / (64 * U);
  // SY: every wave of the workgroup runs the same number of windows (barriers stay matched)
  const size_t rounds = (nwin + nw - 1) / nw;
  for (size_t r = 0; r < rounds; ++r) {
    const size_t c = gw + r * nw;
    const bool live = c < nwin;
    if (!SY && !live) break;
    const size_t p0 = (live ? c : 0) * 64 * U + lane;
    double2 acc[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) acc[u][j] = live ? ld2<DL>(a.y[j] + 2 * (p0 + 64 * u)) : make_double2(0, 0);
#pragma unroll 1
    for (int i = 0; i < K; i += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = live ? ld2<SL>(a.x[i + b] + 2 * (p0 + 64 * u)) : make_double2(0, 0);
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
      if constexpr (SY) __syncthreads();
    }
    if (live)
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < M; ++j) st2<ST>(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
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
  double* vec[56];
  for (int i = 0; i < M + K; ++i) {
    CK(hipMalloc((void**)&vec[i], n * 8));
    CK(hipMemset(vec[i], 0, n * 8));
  }
  OArgs a{};
  a.n = n;
  for (int i = 0; i < K; ++i) a.x[i] = vec[M + i];
  for (int j = 0; j < M; ++j) a.y[j] = vec[j];
  for (int i = 0; i < K * M; ++i) a.alpha[i] = 1e-3 * (i % 17);
  const double bytes = 8.0 * n * (K + 2 * M);
  const int reps = 7;
  auto rep = [&](const char* name, int g, float ms) {
    printf("%-34s g=%-5d %8.3f ms  %7.1f GB/s\n", name, g, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
#define RUN(name, DL, ST, SL, SY, g) \
  rep(name, g, timeit([&] { hipLaunchKernelGGL((k_outer<DL, ST, SL, SY>), dim3(g), dim3(256), 0, 0, a); }, reps))
  for (int round = 0; round < 3; ++round) {
    for (int g : {512, 2048}) {
      RUN("library (nt/nt/nt)", 0, 0, 0, 0, g);
      RUN("dest load plain, store plain", 1, 1, 0, 0, g);
      RUN("dest load plain, store nt", 1, 0, 0, 0, g);
      RUN("dest load nt, store plain", 0, 1, 0, 0, g);
      RUN("sources plain", 0, 0, 1, 0, g);
      RUN("lockstep groups (barrier)", 0, 0, 0, 1, g);
      RUN("lockstep, dest/store plain", 1, 1, 0, 1, g);
    }
  }
  return 0;
}
