// Static vs dynamic window assignment for the streaming panel kernels at one C4 shard's length
// (development tool, not part of the library).  The kernel is the library's write-only gemm_outer
// shape (construct_solution: K sources -> M = 8 destinations, 4 sources x U = 4 windows of 64 lanes x
// 16 B per load group, sources applied in order, nontemporal accesses), with the windows handed out
//   S   statically: wave w takes windows w, w + W, w + 2W, ... (the library's grid stride)
//   Dt  dynamically: each wave takes t windows at a time from a launch-wide atomic ticket counter
//       (lane 0 fetches the next ticket while the current windows stream), so waves on faster CUs / XCDs
//       take more of the vector and the launch ends when the last window does.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_dyn.hip -o tools/mb_dyn
// Run:   tools/mb_dyn [reps=20]
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
__device__ __forceinline__ double2 ld2(const double* p) {
  const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st2(double* p, double2 v) {
  d2v w = {v.x, v.y};
  __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(p));
}

constexpr int M = 8, U = 4, KMAX = 64;
struct OArgs {
  const double* x[KMAX];
  double* y[M];
  int k;
  size_t n;
  unsigned* ticket;
  double alpha[KMAX * M];
};

__device__ __forceinline__ void window(const OArgs& a, size_t c, int lane, size_t n2) {
  constexpr size_t win = 64 * U;
  const size_t p0 = c * win + lane;
  bool ok[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ok[u] = p0 + 64 * u < n2;
  double2 acc[U][M];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < M; ++j) acc[u][j] = make_double2(0, 0);
  for (int i = 0; i + 4 <= a.k; i += 4) {
    double2 xv[4][U];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int u = 0; u < U; ++u) xv[b][u] = ok[u] ? ld2(a.x[i + b] + 2 * (p0 + 64 * u)) : make_double2(0, 0);
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
    if (ok[u])
#pragma unroll
      for (int j = 0; j < M; ++j) st2(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
}

template <int T>  // T = 0: static; T > 0: dynamic, T windows per ticket
__global__ __launch_bounds__(256) void k_outer(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t n2 = a.n >> 1, nwin = (n2 + 64 * U - 1) / (64 * U);
  if constexpr (T == 0) {
    const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
    for (size_t c = gw; c < nwin; c += nw) window(a, c, lane, n2);
  } else {
    unsigned t = 0;
    if (lane == 0) t = atomicAdd(a.ticket, 1u);
    t = __builtin_amdgcn_readfirstlane(t);
    while (size_t(t) * T < nwin) {
      unsigned next = 0;
      if (lane == 0) next = atomicAdd(a.ticket, 1u);  // in flight while the windows stream
      for (int q = 0; q < T; ++q) {
        const size_t c = size_t(t) * T + q;
        if (c < nwin) window(a, c, lane, n2);
      }
      t = __builtin_amdgcn_readfirstlane(next);
    }
  }
}

template <int T>
float run(const OArgs& a, int grid, int reps, hipStream_t s) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipMemsetAsync(a.ticket, 0, 4, s));
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(k_outer<T>, dim3(grid), dim3(256), 0, s, a);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 2) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const size_t nmax = 100000000;
  const int K = 48;
  std::vector<double*> buf(K + M);
  for (auto& b : buf) {
    CK(hipMalloc(&b, nmax * sizeof(double)));
    CK(hipMemset(b, 0, nmax * sizeof(double)));
  }
  unsigned* ticket;
  CK(hipMalloc(&ticket, 64));
  printf("n        k  variant  grid   median_ms  GB/s\n");
  for (size_t n : {size_t(12500000), size_t(100000000)}) {
    for (int k : {8, 48}) {
      OArgs a{};
      for (int i = 0; i < k; ++i) a.x[i] = buf[i];
      for (int j = 0; j < M; ++j) a.y[j] = buf[K + j];
      a.k = k;
      a.n = n;
      a.ticket = ticket;
      for (int q = 0; q < k * M; ++q) a.alpha[q] = 1e-3 * (q % 7);
      const double bytes = 8.0 * n * (k + M);
      for (int per_cu : {4, 8}) {
        const int grid = cus * per_cu;
        const float s0 = run<0>(a, grid, reps, s);
        const float d1 = run<1>(a, grid, reps, s);
        const float d2 = run<2>(a, grid, reps, s);
        printf("%-9zu %2d  S   %6d  %9.4f  %7.1f\n", n, k, grid, s0, bytes / s0 / 1e6);
        printf("%-9zu %2d  D1  %6d  %9.4f  %7.1f\n", n, k, grid, d1, bytes / d1 / 1e6);
        printf("%-9zu %2d  D2  %6d  %9.4f  %7.1f\n", n, k, grid, d2, bytes / d2 / 1e6);
      }
    }
  }
  return 0;
}
