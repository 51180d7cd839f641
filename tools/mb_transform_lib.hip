// The library's ssp_transform_gram against the microbenchmark kernel of tools/mb_transform.hip on the
// SAME buffers in one process (development tool): separates the kernel code from the vectors' placement.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/mb_transform_lib.hip
//          -L iterative-solver_amd/lib -lsubspace_hip -Wl,-rpath,'$ORIGIN/../iterative-solver_amd/lib'
//          -o tools/mb_transform_lib
// Run:   tools/mb_transform_lib [reps=10]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "subspace_hip.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)
#define SK(x)                                                               \
  do {                                                                      \
    if ((x) != 0) {                                                         \
      printf("ssp error %s at %s:%d\n", ssp_last_error(), __FILE__, __LINE__); \
      exit(1);                                                              \
    }                                                                       \
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

constexpr int M = 8, NP = 36;
struct TArgs {
  double* x[M];
  double t[M * M];
  size_t n;
  double* partial;
};

template <int GRAM, int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_t(const TArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  double acc[GRAM ? NP : 1];
#pragma unroll
  for (int q = 0; q < (GRAM ? NP : 1); ++q) acc[q] = 0;
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
  const size_t win = 64 * U, nwin = (a.n / 2) / win;
  for (size_t c = gw; c < nwin; c += nw) {
    const size_t p0 = c * win + lane;
    double2 xv[U][M];
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u][i] = ld2(a.x[i] + 2 * (p0 + 64 * u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double ylo[M], yhi[M];
#pragma unroll
      for (int j = 0; j < M; ++j) {
        double vl = 0, vh = 0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          vl = fma(a.t[i * M + j], xv[u][i].x, vl);
          vh = fma(a.t[i * M + j], xv[u][i].y, vh);
        }
        ylo[j] = vl;
        yhi[j] = vh;
        st2(a.x[j] + 2 * (p0 + 64 * u), make_double2(vl, vh));
      }
      pairs(ylo);
      pairs(yhi);
    }
  }
  if constexpr (GRAM) {
#pragma unroll
    for (int q = 0; q < NP; ++q)
      if (acc[q] == 12345.678) a.partial[q] = acc[q];
  }
}

static float timed(hipStream_t s, int reps, const std::function<void()>& f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(e0, s));
    f();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 2) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  ssp_ctx* ctx = nullptr;
  SK(ssp_ctx_create(0, &ctx));
  hipStream_t s = static_cast<hipStream_t>(ssp_ctx_stream(ctx));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  double* partial;
  CK(hipMalloc(&partial, 4096));
  double tm[M * M];
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < M; ++j) tm[i * M + j] = i == j ? 1.0 : (i < j ? 1e-9 : 0.0);
  for (size_t n : {size_t(100000000), size_t(12500000)}) {
    for (int alloc_kind = 0; alloc_kind < 2; ++alloc_kind) {  // 0: ssp_alloc, 1: hipMalloc interleaved with spares
      std::vector<double*> x(M), spare;
      for (int i = 0; i < M; ++i) {
        if (alloc_kind == 0) {
          SK(ssp_alloc(ctx, n, &x[i]));
        } else {
          CK(hipMalloc(&x[i], n * sizeof(double)));
          double* sp;
          CK(hipMalloc(&sp, n * sizeof(double)));
          spare.push_back(sp);
        }
        CK(hipMemsetAsync(x[i], 0x3f, n * sizeof(double), s));
      }
      CK(hipStreamSynchronize(s));
      TArgs a{};
      for (int i = 0; i < M; ++i) a.x[i] = x[i];
      for (int q = 0; q < M * M; ++q) a.t[q] = tm[q];
      a.n = n;
      a.partial = partial;
      const double gb = 16.0 * M * n / 1e9;
      double gram[M * M];
      const char* an = alloc_kind ? "hipMalloc+spare" : "ssp_alloc";
      auto line = [&](const char* what, float ms) {
        printf("%-10zu %-16s %-26s %8.4f ms %7.1f GB/s\n", n, an, what, ms, gb / ms * 1e3);
      };
      for (int per_cu : {8}) {
        const int g = cus * per_cu;
        line("mb plain U2", timed(s, reps, [&] { hipLaunchKernelGGL((k_t<0, 2>), dim3(g), dim3(256), 0, s, a); }));
        line("lib transform", timed(s, reps, [&] { SK(ssp_transform_gram(ctx, tm, x.data(), nullptr, M, n, nullptr)); }));
        line("mb gram U1", timed(s, reps, [&] { hipLaunchKernelGGL((k_t<1, 1>), dim3(g), dim3(256), 0, s, a); }));
        line("lib transform_gram", timed(s, reps, [&] { SK(ssp_transform_gram(ctx, tm, x.data(), nullptr, M, n, gram)); }));
        line("mb plain U2 (again)", timed(s, reps, [&] { hipLaunchKernelGGL((k_t<0, 2>), dim3(g), dim3(256), 0, s, a); }));
        line("lib transform (again)", timed(s, reps, [&] { SK(ssp_transform_gram(ctx, tm, x.data(), nullptr, M, n, nullptr)); }));
      }
      for (int i = 0; i < M; ++i) {
        if (alloc_kind == 0) SK(ssp_free(ctx, x[i]));
        else CK(hipFree(x[i]));
      }
      for (double* p : spare) CK(hipFree(p));
      SK(ssp_release_cached(ctx));
    }
  }
  SK(ssp_ctx_destroy(ctx));
  return 0;
}
