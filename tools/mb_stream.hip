// Microbenchmark for the streaming kernels (gemm_outer, fill, axpy, dot) against plain read / copy
// references at N = 1e8 (development tool, not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_stream.hip -o /tmp/mb_stream
// Run:   /tmp/mb_stream [n=1e8] [m=8] [k=48]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
__device__ __forceinline__ void st2(double* p, double2 v) { *reinterpret_cast<double2*>(p) = v; }
typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld2nt(const double* p) {
  const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st2nt(double* p, double2 v) {
  d2v w = {v.x, v.y};
  __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(p));
}

struct OArgs {
  const double* x[64];
  double* y[16];
  int k, m;
  size_t n;
  double alpha[384];
};

// o0: library kernel as of r1 (runtime k, 4 sources per step).
template <int M>
__global__ __launch_bounds__(256) void k_o0(const OArgs a) {
  const size_t n2 = a.n >> 1, stride = size_t(gridDim.x) * 256;
  for (size_t p = size_t(blockIdx.x) * 256 + threadIdx.x; p < n2; p += stride) {
    double2 acc[M];
#pragma unroll
    for (int j = 0; j < M; ++j) acc[j] = ld2(a.y[j] + 2 * p);
    for (int i = 0; i + 4 <= a.k; i += 4) {
      const double2 x0 = ld2(a.x[i] + 2 * p), x1 = ld2(a.x[i + 1] + 2 * p), x2 = ld2(a.x[i + 2] + 2 * p),
                    x3 = ld2(a.x[i + 3] + 2 * p);
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const double a0 = a.alpha[i * M + j], a1 = a.alpha[(i + 1) * M + j], a2 = a.alpha[(i + 2) * M + j],
                     a3 = a.alpha[(i + 3) * M + j];
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
#pragma unroll
    for (int j = 0; j < M; ++j) st2(a.y[j] + 2 * p, acc[j]);
  }
}

// o1: batches of B sources loaded together (more loads in flight); NT = nontemporal loads/stores.
template <int M, int B, bool NT>
__global__ __launch_bounds__(256) void k_o1(const OArgs a) {
  const size_t n2 = a.n >> 1, stride = size_t(gridDim.x) * 256;
  for (size_t p = size_t(blockIdx.x) * 256 + threadIdx.x; p < n2; p += stride) {
    double2 acc[M];
#pragma unroll
    for (int j = 0; j < M; ++j) acc[j] = NT ? ld2nt(a.y[j] + 2 * p) : ld2(a.y[j] + 2 * p);
    for (int i = 0; i < a.k; i += B) {
      double2 xv[B];
#pragma unroll
      for (int b = 0; b < B; ++b) xv[b] = NT ? ld2nt(a.x[i + b] + 2 * p) : ld2(a.x[i + b] + 2 * p);
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const double al = a.alpha[(i + b) * M + j];
          acc[j].x = fma(al, xv[b].x, acc[j].x);
          acc[j].y = fma(al, xv[b].y, acc[j].y);
        }
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
      if (NT) st2nt(a.y[j] + 2 * p, acc[j]);
      else st2(a.y[j] + 2 * p, acc[j]);
    }
  }
}

// o2: U positions per thread per iteration (p, p + 64 within the wave's 2U KiB window).
template <int M, int B, int U, bool NTX = false, bool NTY = false>
__global__ __launch_bounds__(256) void k_o2(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
  const size_t n2 = a.n >> 1, chunk = 64 * U;
  for (size_t c = gw; c * chunk < n2; c += nw) {
    const size_t p0 = c * chunk + lane;
    double2 acc[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) acc[u][j] = (p0 + 64 * u < n2) ? ld2(a.y[j] + 2 * (p0 + 64 * u)) : make_double2(0, 0);
    for (int i = 0; i < a.k; i += B) {
      double2 xv[U][B];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int b = 0; b < B; ++b)
          xv[u][b] = (p0 + 64 * u < n2) ? (NTX ? ld2nt(a.x[i + b] + 2 * (p0 + 64 * u)) : ld2(a.x[i + b] + 2 * (p0 + 64 * u)))
                                        : make_double2(0, 0);
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const double al = a.alpha[(i + b) * M + j];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][j].x = fma(al, xv[u][b].x, acc[u][j].x);
            acc[u][j].y = fma(al, xv[u][b].y, acc[u][j].y);
          }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (p0 + 64 * u < n2)
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (NTY) st2nt(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
          else st2(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
        }
  }
}

// o3: library design (4 sources x U windows) with selectable nontemporal loads of y, and block size BS.
template <int M, int U, bool NTYL, int BS>
__global__ __launch_bounds__(BS) void k_o3(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * (BS / 64) + (threadIdx.x >> 6), nw = size_t(gridDim.x) * (BS / 64);
  const size_t n2 = a.n >> 1, win = 64 * U;
  for (size_t c = gw; c * win < n2; c += nw) {
    const size_t p0 = c * win + lane;
    double2 acc[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < M; ++j) acc[u][j] = NTYL ? ld2nt(a.y[j] + 2 * (p0 + 64 * u)) : ld2(a.y[j] + 2 * (p0 + 64 * u));
    for (int i = 0; i + 4 <= a.k; i += 4) {
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

// o4: guarded windows (every load tested against n2), runtime destination count -- the r1 library form.
template <int M, int U>
__global__ __launch_bounds__(256) void k_o4(const OArgs a) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = size_t(gridDim.x) * 4;
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
      for (int j = 0; j < M; ++j) acc[u][j] = (j < a.m && ok[u]) ? ld2nt(a.y[j] + 2 * (p0 + 64 * u)) : z2;
    for (int i = 0; i + 4 <= a.k; i += 4) {
      double2 xv[4][U];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) xv[b][u] = ok[u] ? ld2nt(a.x[i + b] + 2 * (p0 + 64 * u)) : z2;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j = 0; j < M; ++j)
          if (j < a.m) {
            const double al = a.alpha[(i + b) * a.m + j];
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
        for (int j = 0; j < M; ++j)
          if (j < a.m) st2nt(a.y[j] + 2 * (p0 + 64 * u), acc[u][j]);
  }
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void k_fill(double* y, size_t n, double v) {
  const size_t n2 = n >> 1, stride = size_t(gridDim.x) * 256;
  const double2 vv = make_double2(v, v);
  size_t p = size_t(blockIdx.x) * 256 + threadIdx.x;
  for (; p + (U - 1) * stride < n2; p += U * stride)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) st2nt(y + 2 * (p + u * stride), vv);
      else st2(y + 2 * (p + u * stride), vv);
    }
  for (; p < n2; p += stride) st2(y + 2 * p, vv);
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void k_axpy(const double* x, double* y, size_t n, double al) {
  const size_t n2 = n >> 1, stride = size_t(gridDim.x) * 256;
  size_t p = size_t(blockIdx.x) * 256 + threadIdx.x;
  for (; p + (U - 1) * stride < n2; p += U * stride) {
    double2 xv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xv[u] = NT ? ld2nt(x + 2 * (p + u * stride)) : ld2(x + 2 * (p + u * stride));
      yv[u] = NT ? ld2nt(y + 2 * (p + u * stride)) : ld2(y + 2 * (p + u * stride));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      yv[u].x = fma(al, xv[u].x, yv[u].x);
      yv[u].y = fma(al, xv[u].y, yv[u].y);
      if (NT) st2nt(y + 2 * (p + u * stride), yv[u]);
      else st2(y + 2 * (p + u * stride), yv[u]);
    }
  }
  for (; p < n2; p += stride) {
    double2 xv = ld2(x + 2 * p), yv = ld2(y + 2 * p);
    yv.x = fma(al, xv.x, yv.x);
    yv.y = fma(al, xv.y, yv.y);
    st2(y + 2 * p, yv);
  }
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void k_dot(const double* x, size_t n, double* out) {
  const size_t n2 = n >> 1, stride = size_t(gridDim.x) * 256;
  size_t p = size_t(blockIdx.x) * 256 + threadIdx.x;
  double s = 0;
  for (; p + (U - 1) * stride < n2; p += U * stride) {
    double2 xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = NT ? ld2nt(x + 2 * (p + u * stride)) : ld2(x + 2 * (p + u * stride));
#pragma unroll
    for (int u = 0; u < U; ++u) s = fma(xv[u].y, xv[u].y, fma(xv[u].x, xv[u].x, s));
  }
  for (; p < n2; p += stride) {
    double2 xv = ld2(x + 2 * p);
    s = fma(xv.y, xv.y, fma(xv.x, xv.x, s));
  }
  out[size_t(blockIdx.x) * 256 + threadIdx.x] = s;
}

float timeit(const std::function<void()>& f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? size_t(atof(argv[1])) : 100000000;
  const int m = 8, k = 48;
  double* vec[64];
  for (int i = 0; i < m + k; ++i) {
    CK(hipMalloc((void**)&vec[i], n * 8));
    CK(hipMemset(vec[i], 0, n * 8));
  }
  double* partial;
  CK(hipMalloc((void**)&partial, 65536 * 256 * 8));
  OArgs a{};
  a.k = k;
  a.m = m;
  a.n = n;
  for (int i = 0; i < k; ++i) a.x[i] = vec[m + i];
  for (int j = 0; j < m; ++j) a.y[j] = vec[j];
  for (int i = 0; i < k * m; ++i) a.alpha[i] = 1e-3 * (i % 17);
  const double obytes = 8.0 * n * (k + 2 * m), vb = 8.0 * n;
  auto rep = [&](const char* name, int g, float ms, double bytes) {
    printf("%-26s g=%-6d %8.3f ms  %7.1f GB/s\n", name, g, ms, bytes / ms / 1e6);
  };
  // Placement: one slab per trial, vector i at i * (pitch + stagger) for large staggers.
  const size_t MB2 = size_t(2) << 20;
  const size_t pitch = ((n * 8 + MB2 - 1) / MB2) * MB2;
  const size_t staggers[] = {0, MB2, 3 * MB2, 7 * MB2, 15 * MB2, 31 * MB2, 63 * MB2, 127 * MB2};
  for (int rep_i = 0; rep_i < 2; ++rep_i)
    for (size_t st : staggers) {
      const size_t step = pitch + st;
      char* base = nullptr;
      CK(hipMalloc((void**)&base, step * (m + k)));
      CK(hipMemset(base, 0, step * (m + k)));
      for (int j = 0; j < m; ++j) a.y[j] = reinterpret_cast<double*>(base + j * step);
      for (int i = 0; i < k; ++i) a.x[i] = reinterpret_cast<double*>(base + (m + i) * step);
      char name[64];
      snprintf(name, sizeof name, "slab stagger %zu MB", st >> 20);
      rep(name, 1024, timeit([&] { hipLaunchKernelGGL((k_o4<8, 4>), dim3(1024), dim3(256), 0, 0, a); }, 4), obytes);
      CK(hipFree(base));
    }
  return 0;
}
