// Host-visible latency of one small reduction's completion paths (development tool).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sync_probe.hip -o tools/sync_probe
// Run:   tools/sync_probe [spin|yield|block|auto]
//   sync     kernel, hipStreamSynchronize
//   memcpy   kernel writes device result, hipMemcpyAsync D2H into pinned memory, hipStreamSynchronize
//   2k+copy  two kernels (partials + fold), hipMemcpyAsync, hipStreamSynchronize (the library's path)
//   hostw    kernel writes the result straight into pinned host memory, hipStreamSynchronize
//   flag     kernel writes result + sequence flag (system-scope release) into pinned memory, the host
//            polls the flag (no runtime wait)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void k_sum(const double* x, int n, double* out) {
  __shared__ double s[256];
  double v = 0;
  for (int i = threadIdx.x; i < n; i += 256) v += x[i];
  s[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < 256; ++i) t += s[i];
    out[0] = t;
  }
}

__global__ void k_sum_flag(const double* x, int n, double* out, unsigned long long* flag, unsigned long long seq) {
  __shared__ double s[256];
  double v = 0;
  for (int i = threadIdx.x; i < n; i += 256) v += x[i];
  s[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < 256; ++i) t += s[i];
    out[0] = t;
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

double us_per(const std::function<void()>& f, int reps) {
  for (int i = 0; i < 50; ++i) f();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) f();
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "auto";
  unsigned flags = hipDeviceScheduleAuto;
  if (!strcmp(mode, "spin")) flags = hipDeviceScheduleSpin;
  if (!strcmp(mode, "yield")) flags = hipDeviceScheduleYield;
  if (!strcmp(mode, "block")) flags = hipDeviceScheduleBlockingSync;
  CK(hipSetDeviceFlags(flags));
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int n = 1024;
  double *x, *dres;
  CK(hipMalloc((void**)&x, n * sizeof(double)));
  CK(hipMemset(x, 0, n * sizeof(double)));
  CK(hipMalloc((void**)&dres, 64));
  double* hres;
  CK(hipHostMalloc((void**)&hres, 64, hipHostMallocDefault));
  unsigned long long* flag;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocDefault));
  *flag = 0;
  unsigned long long seq = 0;
  const int reps = 3000;
  double sink = 0;
  printf("mode %s\n", mode);
  printf("  launch only (async)  %7.2f us\n", us_per([&] { hipLaunchKernelGGL(k_sum, 1, 256, 0, st, x, n, dres); }, reps));
  CK(hipStreamSynchronize(st));
  printf("  sync                 %7.2f us\n", us_per([&] {
           hipLaunchKernelGGL(k_sum, 1, 256, 0, st, x, n, dres);
           (void)hipStreamSynchronize(st);
         }, reps));
  printf("  memcpy               %7.2f us\n", us_per([&] {
           hipLaunchKernelGGL(k_sum, 1, 256, 0, st, x, n, dres);
           (void)hipMemcpyAsync(hres, dres, 8, hipMemcpyDeviceToHost, st);
           (void)hipStreamSynchronize(st);
           sink += hres[0];
         }, reps));
  printf("  2k+copy              %7.2f us\n", us_per([&] {
           hipLaunchKernelGGL(k_sum, 1, 256, 0, st, x, n, dres + 1);
           hipLaunchKernelGGL(k_sum, 1, 256, 0, st, dres + 1, 1, dres);
           (void)hipMemcpyAsync(hres, dres, 8, hipMemcpyDeviceToHost, st);
           (void)hipStreamSynchronize(st);
           sink += hres[0];
         }, reps));
  printf("  hostw                %7.2f us\n", us_per([&] {
           hipLaunchKernelGGL(k_sum, 1, 256, 0, st, x, n, hres);
           (void)hipStreamSynchronize(st);
           sink += hres[0];
         }, reps));
  bool timeout = false;
  printf("  flag                 %7.2f us\n", us_per([&] {
           if (timeout) return;
           ++seq;
           hipLaunchKernelGGL(k_sum_flag, 1, 256, 0, st, x, n, hres, flag, seq);
           const auto t0 = std::chrono::steady_clock::now();
           while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
             if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
               timeout = true;
               break;
             }
           }
           sink += hres[0];
         }, reps));
  CK(hipStreamSynchronize(st));
  if (timeout) printf("  flag: TIMEOUT (flag never seen)\n");
  printf("sink %g\n", sink);
  return 0;
}
