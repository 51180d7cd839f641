// Microbenchmark for gemm_inner kernel variants (development tool, not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_inner.hip -o /tmp/mb_inner
// Run:   /tmp/mb_inner [n=1e8] [m=8] [k=48]
#include <hip/hip_runtime.h>

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

typedef double f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }

struct Args {
  const double* x[16];
  const double* y[64];
  int m, k;
  size_t n;
  double* partial;
};

// V0: current library kernel (MFMA, lane-strided 16B loads)
template <int NT, int U, bool MFMA>
__global__ __launch_bounds__(256) void k_v0(const Args a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  const double* xp = c < a.m ? a.x[c] : nullptr;
  const double* yp[NT];
  for (int t = 0; t < NT; ++t) yp[t] = (16 * t + c < a.k) ? a.y[16 * t + c] : nullptr;
  f64x4 acc[NT];
  for (int t = 0; t < NT; ++t) acc[t] = f64x4{0, 0, 0, 0};
  const size_t gw = size_t(blockIdx.x) * 4 + wave, nw = size_t(gridDim.x) * 4;
  const size_t chunk = 8 * U, nchunks = a.n / chunk;
  const double2 z2 = make_double2(0, 0);
  for (size_t ch = gw; ch < nchunks; ch += nw) {
    const size_t base = ch * chunk + 2 * q;
    double2 xv[U], yv[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = xp ? ld2(xp + base + 8 * u) : z2;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) yv[u][t] = yp[t] ? ld2(yp[t] + base + 8 * u) : z2;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (MFMA) {
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[u].x, yv[u][t].x, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[u].y, yv[u][t].y, acc[t], 0, 0, 0);
        } else {
          acc[t][0] = fma(xv[u].x, yv[u][t].x, acc[t][0]);
          acc[t][1] = fma(xv[u].y, yv[u][t].y, acc[t][1]);
        }
      }
  }
  double s = 0;
  for (int t = 0; t < NT; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  a.partial[size_t(blockIdx.x) * 256 + threadIdx.x] = s;
}

// Streaming read of m+k vectors, fully coalesced 16B per lane, sum (bandwidth reference).
__global__ __launch_bounds__(256) void k_read(const Args a) {
  const size_t n2 = a.n / 2, stride = size_t(gridDim.x) * 256;
  double s = 0;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n2; i += stride) {
    double2 v[16];
    int j = 0;
    for (int v0 = 0; v0 < a.m + a.k; v0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int vi = v0 + u;
        const double* p = vi < a.m ? a.x[vi] : (vi - a.m < a.k ? a.y[vi - a.m] : nullptr);
        v[u] = p ? ld2(p + 2 * i) : make_double2(0, 0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u].x * v[u].y;
    }
    (void)j;
  }
  a.partial[size_t(blockIdx.x) * 256 + threadIdx.x] = s;
}

// V2: LDS-staged.  Each wave loads a coalesced 128-element (1 KiB) block of ONE vector per
// instruction into LDS ([vec][128] doubles), then reads it back in MFMA layout.
template <int NT>
__global__ __launch_bounds__(256) void k_v2(const Args a) {
  constexpr int TILE = 128;  // elements per vector per stage
  __shared__ double lds[16 + 16 * NT][TILE + 2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  const int nv = 16 + 16 * NT;
  f64x4 acc[NT];
  for (int t = 0; t < NT; ++t) acc[t] = f64x4{0, 0, 0, 0};
  const size_t ntiles = a.n / TILE;
  for (size_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const size_t base = tile * TILE;
    // load: vectors distributed over waves; each lane 16B (2 doubles) -> 128 doubles per wave-instr
    for (int v = wave; v < nv; v += 4) {
      const double* p = v < 16 ? (v < a.m ? a.x[v] : nullptr) : ((v - 16) < a.k ? a.y[v - 16] : nullptr);
      double2 d = p ? ld2(p + base + 2 * lane) : make_double2(0, 0);
      lds[v][2 * lane] = d.x;
      lds[v][2 * lane + 1] = d.y;
    }
    __syncthreads();
    // each wave takes 32 of the 128 elements: 8 MFMA k-steps of 4
    for (int s = 0; s < 8; ++s) {
      const int e = wave * 32 + s * 4 + q;
      const double xa = lds[c][e];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, lds[16 + 16 * t + c][e], acc[t], 0, 0, 0);
    }
    __syncthreads();
  }
  double s = 0;
  for (int t = 0; t < NT; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  a.partial[size_t(blockIdx.x) * 256 + threadIdx.x] = s;
}

// V3: v_mfma_f64_4x4x4f64 (4 blocks).  Lane l = 16k + 4b + i holds A_b[i][k] / B_b[k][j] (j = i),
// C lane 16i + 4b + j holds C_b[i][j].  Rows/cols = groups of 4 vectors; the 16 lanes of one
// vector load 16 B each at position p = l >> 2: 256 contiguous bytes per vector per instruction.
template <int MG, int NG, int U>
__global__ __launch_bounds__(256) void k_v3(const Args a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 3, p = lane >> 2;
  const double* xp[MG];
  const double* yp[NG];
#pragma unroll
  for (int g = 0; g < MG; ++g) xp[g] = (4 * g + r < a.m) ? a.x[4 * g + r] : nullptr;
#pragma unroll
  for (int h = 0; h < NG; ++h) yp[h] = (4 * h + r < a.k) ? a.y[4 * h + r] : nullptr;
  double acc[MG][NG];
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) acc[g][h] = 0;
  const size_t gw = size_t(blockIdx.x) * 4 + wave, nw = size_t(gridDim.x) * 4;
  const size_t chunk = 32 * U, nchunks = a.n / chunk;
  const double2 z2 = make_double2(0, 0);
  for (size_t ch = gw; ch < nchunks; ch += nw) {
    const size_t base = ch * chunk + 2 * p;
    double2 xv[U][MG], yv[U][NG];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int g = 0; g < MG; ++g) xv[u][g] = xp[g] ? ld2(xp[g] + base + 32 * u) : z2;
#pragma unroll
      for (int h = 0; h < NG; ++h) yv[u][h] = yp[h] ? ld2(yp[h] + base + 32 * u) : z2;
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
  double s = 0;
#pragma unroll
  for (int g = 0; g < MG; ++g)
#pragma unroll
    for (int h = 0; h < NG; ++h) s += acc[g][h];
  a.partial[size_t(blockIdx.x) * 256 + threadIdx.x] = s;
}

template <class F>
float timeit(F f, int reps) {
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
  size_t n = argc > 1 ? size_t(atof(argv[1])) : 100000000;
  int m = argc > 2 ? atoi(argv[2]) : 8;
  int k = argc > 3 ? atoi(argv[3]) : 48;
  Args a{};
  a.m = m;
  a.k = k;
  a.n = n;
  for (int i = 0; i < m; ++i) CK(hipMalloc((void**)&a.x[i], n * 8));
  for (int j = 0; j < k; ++j) CK(hipMalloc((void**)&a.y[j], n * 8));
  for (int i = 0; i < m; ++i) CK(hipMemset((void*)a.x[i], 0, n * 8));
  for (int j = 0; j < k; ++j) CK(hipMemset((void*)a.y[j], 0, n * 8));
  CK(hipMalloc(&a.partial, 8192 * 256 * 8));
  const double bytes = 8.0 * n * (m + k);
  auto report = [&](const char* name, float ms) { printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6); };
  if (m == 16 && k == 64) {
    // 16 x 64: one launch with 16 column groups vs the library's three (6 + 6 + 4 groups)
    for (int rep = 0; rep < 2; ++rep)
      for (int grid : {1024, 2048}) {
        char nm[64];
        snprintf(nm, 64, "v3 MG4 NG16 1 launch g=%d", grid);
        report(nm, timeit([&] { hipLaunchKernelGGL((k_v3<4, 16, 1>), dim3(grid), dim3(256), 0, 0, a); }, 5));
        snprintf(nm, 64, "v3 MG4 NG8 2 launches g=%d", grid);
        report(nm, timeit([&] {
                 Args b = a;
                 for (int h = 0; h < 2; ++h) {
                   b.k = 32;
                   for (int j = 0; j < 32; ++j) b.y[j] = a.y[32 * h + j];
                   hipLaunchKernelGGL((k_v3<4, 8, 1>), dim3(grid), dim3(256), 0, 0, b);
                 }
               }, 5));
        snprintf(nm, 64, "v3 MG4 NG6 3 launches g=%d", grid);
        report(nm, timeit([&] {
                 Args b = a;
                 const int c0[3] = {0, 24, 48}, kk[3] = {24, 24, 16};
                 for (int h = 0; h < 3; ++h) {
                   b.k = kk[h];
                   for (int j = 0; j < kk[h]; ++j) b.y[j] = a.y[c0[h] + j];
                   if (h < 2) hipLaunchKernelGGL((k_v3<4, 6, 1>), dim3(grid), dim3(256), 0, 0, b);
                   else hipLaunchKernelGGL((k_v3<4, 4, 1>), dim3(grid), dim3(256), 0, 0, b);
                 }
               }, 5));
      }
    return 0;
  }
  for (int grid : {512, 1024, 2048}) {
    char nm[64];
    snprintf(nm, 64, "read g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a); }, 5));
  }
  for (int grid : {512, 1024, 2048}) {
    char nm[64];
    snprintf(nm, 64, "v3 4x4x4 MG2 NG12 U1 g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_v3<2, 12, 1>), dim3(grid), dim3(256), 0, 0, a); }, 5));
    snprintf(nm, 64, "v3 4x4x4 MG2 NG12 U2 g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_v3<2, 12, 2>), dim3(grid), dim3(256), 0, 0, a); }, 5));
  }
  for (int grid : {1024, 2048}) {
    char nm[64];
    snprintf(nm, 64, "v0 mfma NT3 U2 g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_v0<3, 2, true>), dim3(grid), dim3(256), 0, 0, a); }, 5));
    snprintf(nm, 64, "v0 mfma NT3 U4 g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_v0<3, 4, true>), dim3(grid), dim3(256), 0, 0, a); }, 5));
    snprintf(nm, 64, "v0 mfma NT3 U1 g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_v0<3, 1, true>), dim3(grid), dim3(256), 0, 0, a); }, 5));
    snprintf(nm, 64, "v0 valu NT3 U2 g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_v0<3, 2, false>), dim3(grid), dim3(256), 0, 0, a); }, 5));
    snprintf(nm, 64, "v2 lds NT3 g=%d", grid);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_v2<3>), dim3(grid), dim3(256), 0, 0, a); }, 5));
  }
  return 0;
}
