// Probes the lane layout of v_mfma_f64_4x4x4f64 (development tool).
// For every lane L: A = e_L, B = (lane+1) -> which C lanes receive which B value tells (block,row,k).
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(int L, int which, double* out) {
  const int l = threadIdx.x;
  double a, b;
  if (which == 0) {  // A = e_L, B = lane id + 1
    a = (l == L) ? 1.0 : 0.0;
    b = l + 1.0;
  } else {  // B = e_L, A = lane id + 1
    b = (l == L) ? 1.0 : 0.0;
    a = l + 1.0;
  }
  double c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[l] = c;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 64 * sizeof(double));
  double h[64];
  for (int which = 0; which < 2; ++which) {
    printf("%s\n", which == 0 ? "A=e_L: C lanes receiving B value (B lane = value-1)" : "B=e_L: C lanes receiving A value");
    for (int L = 0; L < 64; ++L) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, L, which, d);
      (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("L=%2d:", L);
      for (int l = 0; l < 64; ++l)
        if (h[l] != 0) printf(" C%d<-%d", l, int(h[l]) - 1);
      printf("\n");
    }
  }
  return 0;
}
