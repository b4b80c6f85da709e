// operand/result layout of v_mfma_f64_4x4x4f64 (4 blocks) and v_mfma_f64_16x16x4f64
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k4(double *out) {  // out[t][l]: test t < 64: A = unit at lane t, B = 1000+l
  const int l = threadIdx.x;
  for (int t = 0; t < 128; ++t) {
    double a, b;
    if (t < 64) { a = (l == t) ? 1.0 : 0.0; b = 1000 + l; }
    else { b = (l == t - 64) ? 1.0 : 0.0; a = 1000 + l; }
    double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[t * 64 + l] = d;
  }
}
int main() {
  double *d; hipMalloc(&d, 128 * 64 * 8);
  hipLaunchKernelGGL(k4, dim3(1), dim3(64), 0, 0, d);
  double h[128 * 64];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int t = 0; t < 128; ++t) {
    printf("%s%2d:", t < 64 ? "A" : "B", t % 64);
    for (int l = 0; l < 64; ++l) if (h[t * 64 + l] != 0) printf(" %d=%g", l, h[t * 64 + l] - 1000);
    printf("\n");
  }
  return 0;
}
