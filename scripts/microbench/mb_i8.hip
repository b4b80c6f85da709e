// microbenchmark (r4): int8 MFMA rate on gfx950 and whether it co-issues with VALU work of
// another wave on the same SIMD (the f64 MFMA does not, profiles/r2_microbench.txt) -- the
// question behind an exact integer split of the assembly's fp32 products
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// role: 0 = i8 mfma 16x16x64, 1 = fp32 fma valu, 2 = f64 fma valu, 3 = idle, 5 = int valu,
//       6 = f64 mfma 16x16x4
template <int ROLE>
__device__ void work(int iters, double *out, float seed) {
  const int lane = threadIdx.x & 63;
  if constexpr (ROLE == 0) {
    i32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    i32x4 x = {lane, lane * 3, lane * 5, lane * 7}, y = {lane + 1, lane * 2, 9, lane};
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(y, y, a3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
  } else if constexpr (ROLE == 6) {
    f64x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    double x = seed + lane, y = seed * 2 - lane;
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
  } else if constexpr (ROLE == 1) {
    float a[8];
    for (int j = 0; j < 8; ++j) a[j] = seed + j + lane;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = __builtin_fmaf(a[j], 0.999f, 1e-3f);
    float s = 0;
    for (int j = 0; j < 8; ++j) s += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  } else if constexpr (ROLE == 2) {
    double a[8];
    for (int j = 0; j < 8; ++j) a[j] = seed + j + lane;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = __builtin_fma(a[j], 0.999, 1e-3);
    double s = 0;
    for (int j = 0; j < 8; ++j) s += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  } else if constexpr (ROLE == 5) {
    unsigned a[8];
    for (int j = 0; j < 8; ++j) a[j] = (unsigned)(seed) + j + lane;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] * 2654435761u + 12345u;
    unsigned s = 0;
    for (int j = 0; j < 8; ++j) s ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

template <int A, int B>
__global__ void __launch_bounds__(512) kern(int itA, int itB, double *out, float seed) {
  const int w = threadIdx.x >> 6;
  if (w < (blockDim.x >> 7)) work<A>(itA, out, seed);
  else work<B>(itB, out, seed);
}

template <int A, int B>
float run(int itA, int itB, double *out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kern<A, B>), dim3(256), dim3(512), 0, 0, itA, itB, out, 1.0f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((kern<A, B>), dim3(256), dim3(512), 0, 0, itA, itB, out, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double *out; hipMalloc(&out, 256 * 512 * 8);
  const int it = 20000;
  float t;
#define R(A, B, ia, ib, name) t = run<A, B>(ia, ib, out); printf("%-44s %8.3f ms\n", name, t);
  R(0, 3, 4 * it, 0, "i8 mfma 16x16x64 alone (320k/wave)");
  R(0, 0, 4 * it, 4 * it, "i8 mfma x2 waves/SIMD");
  R(6, 3, it, 0, "f64 mfma 16x16x4 alone (80k/wave)");
  R(1, 3, 4 * it, 0, "fp32 fma alone");
  R(2, 3, it, 0, "f64 fma alone");
  R(5, 3, 4 * it, 0, "int mad alone");
  R(0, 1, 4 * it, 4 * it, "i8 mfma + fp32 fma (other wave)");
  R(0, 5, 4 * it, 4 * it, "i8 mfma + int mad (other wave)");
  R(0, 2, 4 * it, it, "i8 mfma + f64 fma (other wave)");
  R(0, 6, 4 * it, it, "i8 mfma + f64 mfma (other wave)");
  return 0;
}
