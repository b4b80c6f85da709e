// microbenchmarks: f64 MFMA rates and MFMA/VALU co-issue on gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef double f64x1 __attribute__((ext_vector_type(1)));

// role: 0 = f64 mfma 16x16x4, 1 = fp32 fma valu, 2 = f64 fma valu, 3 = idle, 4 = mfma f64 4x4x4, 5 = int valu
template <int ROLE>
__device__ void work(int iters, double *out, float seed) {
  const int lane = threadIdx.x & 63;
  if constexpr (ROLE == 0) {
    f64x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    double x = seed + lane, y = seed * 2 - lane;
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
  } else if constexpr (ROLE == 4) {
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    double x = seed + lane, y = seed * 2 - lane;
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_4x4x4f64(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f64_4x4x4f64(y, y, a3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
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

// block of 64*W threads; waves w < W/2 do role A, others role B (waves are dealt to SIMDs
// round-robin, so with W = 8: waves 0-3 on SIMD 0-3 with role A, waves 4-7 pair with them)
template <int A, int B>
__global__ void __launch_bounds__(512) kern(int itA, int itB, double *out, float seed) {
  const int w = threadIdx.x >> 6;
  if (w < (blockDim.x >> 7)) work<A>(itA, out, seed);
  else work<B>(itB, out, seed);
}

template <int A, int B>
float run(int W, int itA, int itB, double *out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kern<A, B>), dim3(256), dim3(64 * W), 0, 0, itA, itB, out, 1.0f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((kern<A, B>), dim3(256), dim3(64 * W), 0, 0, itA, itB, out, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double *out; hipMalloc(&out, 256 * 512 * 8);
  const int it = 20000;
  // per SIMD: W=8 -> 2 waves per SIMD; roles A (waves 0-3) and B (waves 4-7)
  // cycles per instruction estimate: time * clk / (iters*4) per wave on its SIMD
  float t;
#define R(A, B, ia, ib, name) t = run<A, B>(8, ia, ib, out); printf("%-40s %8.3f ms\n", name, t);
  R(0, 3, it, 0, "mfma16 f64 alone (1 wave/SIMD)");
  R(0, 0, it, it, "mfma16 f64 x2 waves/SIMD");
  R(4, 3, it, 0, "mfma4x4 f64 alone");
  R(4, 4, it, it, "mfma4x4 f64 x2");
  R(1, 3, 4 * it, 0, "fp32 fma alone (8 chains x4)");
  R(2, 3, it, 0, "f64 fma alone");
  R(5, 3, 4 * it, 0, "int mad alone");
  R(0, 1, it, 4 * it, "mfma16 + fp32 fma");
  R(0, 2, it, it, "mfma16 + f64 fma");
  R(0, 5, it, 4 * it, "mfma16 + int mad");
  R(1, 1, 4 * it, 4 * it, "fp32 + fp32");
  R(2, 2, it, it, "f64 + f64");
  return 0;
}
