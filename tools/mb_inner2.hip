// gemm_inner (8 x 48, N = 1e8) load-pattern variants of the library's 4x4x4 f64 MFMA kernel
// (development tool, not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_inner2.hip -o tools/mb_inner2
// Run:   tools/mb_inner2 [n=1e8] [p = placement sets, library form vs burst forms]
//   NT  nontemporal loads (the library kernel uses plain loads)
//   U   consecutive 32-element chunks per wave iteration (U x 256 B contiguous per vector)
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
template <bool NT>
__device__ __forceinline__ double2 ld(const double* p) {
  if constexpr (NT) {
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
  } else {
    return *reinterpret_cast<const double2*>(p);
  }
}

struct Args {
  const double* x[16];
  const double* y[64];
  int m, k;
  size_t n;
  double* partial;  // [gridDim.x]
};

template <int MG, int NG, bool NT, int U>
__global__ __launch_bounds__(256) void k_inner(const Args a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 3, p = lane >> 2;
  const double* xp[MG];
  const double* yp[NG];
#pragma unroll
  for (int g = 0; g < MG; ++g) xp[g] = a.x[4 * g + r];
#pragma unroll
  for (int h = 0; h < NG; ++h) yp[h] = a.y[4 * h + r];
  double acc[MG][NG];
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) acc[g][h] = 0;
  const size_t gw = size_t(blockIdx.x) * 4 + wave, nw = size_t(gridDim.x) * 4;
  const size_t nsuper = a.n / (32 * U);  // n is a multiple of 32 U here
  for (size_t ch = gw; ch < nsuper; ch += nw) {
    double2 xv[U][MG], yv[U][NG];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t e = (ch * U + u) * 32 + 2 * p;
#pragma unroll
      for (int g = 0; g < MG; ++g) xv[u][g] = ld<NT>(xp[g] + e);
#pragma unroll
      for (int h = 0; h < NG; ++h) yv[u][h] = ld<NT>(yp[h] + e);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int g = 0; g < MG; ++g)
#pragma unroll
        for (int h = 0; h < NG; ++h) {
          acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(xv[u][g].x, yv[u][h].x, acc[g][h], 0, 0, 0);
          acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(xv[u][g].y, yv[u][h].y, acc[g][h], 0, 0, 0);
        }
  }
  // Per-block folded sums (enough to check the variants agree).
  double s = 0;
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) s += acc[g][h];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < 256; ++i) t += red[i];
    a.partial[blockIdx.x] = t;
  }
}

// Burst form: a wave visit covers U consecutive 32-element chunks (U x 256 B contiguous per vector);
// the row groups' U chunks are loaded first and held, then each column group's U chunks are loaded
// back to back and contracted against the held rows (the 4 vectors of a group: 4 x U x 256 B per burst).
template <int MG, int NG, int U>
__global__ __launch_bounds__(256, 2) void k_burst(const Args a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 3, p = lane >> 2;
  const double* xp[MG];
  const double* yp[NG];
#pragma unroll
  for (int g = 0; g < MG; ++g) xp[g] = a.x[4 * g + r];
#pragma unroll
  for (int h = 0; h < NG; ++h) yp[h] = a.y[4 * h + r];
  double acc[MG][NG];
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) acc[g][h] = 0;
  const size_t gw = size_t(blockIdx.x) * 4 + wave, nw = size_t(gridDim.x) * 4;
  const size_t nsuper = a.n / (32 * U);
  for (size_t ch = gw; ch < nsuper; ch += nw) {
    const size_t e0 = ch * U * 32 + 2 * p;
    double2 xv[MG][U];
#pragma unroll
    for (int g = 0; g < MG; ++g)
#pragma unroll
      for (int u = 0; u < U; ++u) xv[g][u] = ld<true>(xp[g] + e0 + 32 * u);
#pragma unroll
    for (int h = 0; h < NG; ++h) {
      double2 yv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) yv[u] = ld<true>(yp[h] + e0 + 32 * u);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int g = 0; g < MG; ++g) {
          acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(xv[g][u].x, yv[u].x, acc[g][h], 0, 0, 0);
          acc[g][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(xv[g][u].y, yv[u].y, acc[g][h], 0, 0, 0);
        }
    }
  }
  double s = 0;
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) s += acc[g][h];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < 256; ++i) t += red[i];
    a.partial[blockIdx.x] = t;
  }
}

float timeit(const std::function<void()>& f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
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

__global__ void k_init(double* v, size_t n, unsigned seed) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    v[i] = double(z >> 11) * 0x1.0p-53 - 0.5;
  }
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? size_t(atof(argv[1])) : 100000000;
  const int m = 8, k = 48;
  const int gmax = 2048;
  if (n % 128) {
    printf("n must be a multiple of 128\n");
    return 1;
  }
  std::vector<double*> vec(m + k);
  for (int i = 0; i < m + k; ++i) {
    CK(hipMalloc((void**)&vec[i], n * 8));
    hipLaunchKernelGGL(k_init, dim3(2048), dim3(256), 0, 0, vec[i], n, unsigned(i));
  }
  double* partial = nullptr;
  CK(hipMalloc((void**)&partial, gmax * sizeof(double)));
  CK(hipDeviceSynchronize());
  Args a{};
  a.m = m;
  a.k = k;
  a.n = n;
  a.partial = partial;
  for (int i = 0; i < m; ++i) a.x[i] = vec[i];
  for (int j = 0; j < k; ++j) a.y[j] = vec[m + j];
  const double bytes = 8.0 * n * (m + k);
  auto check = [&](int g) {
    std::vector<double> h(g);
    CK(hipMemcpy(h.data(), partial, g * sizeof(double), hipMemcpyDeviceToHost));
    double s = 0;
    for (double v : h) s += v;
    return s;
  };
  auto run = [&](const char* name, int g, const std::function<void()>& f) {
    if (g > gmax) return;
    f();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const float ms = timeit(f, 7);
    printf("%-22s g=%-6d %8.3f ms  %7.1f GB/s  sum %.10e\n", name, g, ms, bytes / ms / 1e6, check(g));
    fflush(stdout);
  };
  if (argc > 2 && argv[2][0] == 'p') {
    // Placement: library form (nt U1) against the burst forms over freshly allocated vector sets.
    for (int set = 0; set < 4; ++set) {
      if (set) {
        for (int i = 0; i < m + k; ++i) CK(hipFree(vec[i]));
        for (int i = 0; i < m + k; ++i) {
          CK(hipMalloc((void**)&vec[i], n * 8));
          hipLaunchKernelGGL(k_init, dim3(2048), dim3(256), 0, 0, vec[i], n, unsigned(i));
        }
        CK(hipDeviceSynchronize());
        for (int i = 0; i < m; ++i) a.x[i] = vec[i];
        for (int j = 0; j < k; ++j) a.y[j] = vec[m + j];
      }
      printf("-- set %d\n", set);
      for (int g : {1024, 2048}) {
        run("lib nt U1", g, [&] { hipLaunchKernelGGL((k_inner<2, 12, true, 1>), dim3(g), dim3(256), 0, 0, a); });
        run("burst U4", g, [&] { hipLaunchKernelGGL((k_burst<2, 12, 4>), dim3(g), dim3(256), 0, 0, a); });
        run("burst U8", g, [&] { hipLaunchKernelGGL((k_burst<2, 12, 8>), dim3(g), dim3(256), 0, 0, a); });
        run("burst U16", g, [&] { hipLaunchKernelGGL((k_burst<2, 12, 16>), dim3(g), dim3(256), 0, 0, a); });
      }
    }
    return 0;
  }
  for (int round = 0; round < 2; ++round)
    for (int g : {512, 1024, 2048}) {
      run("lib (plain, U1)", g, [&] { hipLaunchKernelGGL((k_inner<2, 12, false, 1>), dim3(g), dim3(256), 0, 0, a); });
      run("nt U1", g, [&] { hipLaunchKernelGGL((k_inner<2, 12, true, 1>), dim3(g), dim3(256), 0, 0, a); });
      run("plain U2", g, [&] { hipLaunchKernelGGL((k_inner<2, 12, false, 2>), dim3(g), dim3(256), 0, 0, a); });
      run("nt U2", g, [&] { hipLaunchKernelGGL((k_inner<2, 12, true, 2>), dim3(g), dim3(256), 0, 0, a); });
      run("nt U4", g, [&] { hipLaunchKernelGGL((k_inner<2, 12, true, 4>), dim3(g), dim3(256), 0, 0, a); });
    }
  return 0;
}
