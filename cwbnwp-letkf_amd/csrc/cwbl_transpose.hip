// cwbl_transpose.hip — device side of the member <-> column transposes around the core
// (module_mpi_util.f90:71-358, 445-580).
//
// The reference moves each variable between "member layout" (rank m holds member m's whole
// field, global(nx,ny,nz)) and "column layout" (every rank holds its cyclic columns for all
// members, var(loc_nx,loc_ny,nz,0:k-1)) with mpi_alltoallv, packing and unpacking on the host.
// Here the exchange is RCCL point-to-point over xGMI (cwbl/transpose.py); these kernels are
// the packing on either side, done in HBM:
//   pack_columns_kernel    letkf_scatter_grid send side (:224-258): global -> per-rank chunks
//   unpack_columns_kernel  letkf_gather_grid receive side (:326-350): chunks -> global
//   vcoord_mean_kernel     letkf_scatter_vcoord (:491-505): member mean of PH / g, destagger
//   member_sum_kernel, scale_kernel   write_mean (module_grid.f90:744-840): the rank-local
//                          member sum ahead of the one reduce, and the root's sscal
// All three are HBM bound byte moves (no arithmetic worth a matrix core): one thread per
// element of the global field, so the global side is read or written fully coalesced and
// the chunk side is px interleaved contiguous streams per wavefront.
#include "../../include/cwb_letkf_core.h"
#include "cwbl_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace cwbl {

namespace {

// columns of a cyclic (block 1) split of n over p ranks owned by rank coordinate id
__host__ __device__ inline int cyc_count(int n, int id, int p) {
  return id < n ? (n - id + p - 1) / p : 0;
}

}  // namespace

void make_decomp(Decomp &d, int nx, int ny, int nz, int px, int py) {
  d.nx = nx; d.ny = ny; d.nz = nz; d.px = px; d.py = py;
  int acc = 0;
  for (int a = 0; a < px; ++a) { d.cols_before[a] = acc; acc += cyc_count(nx, a, px); }
  acc = 0;
  for (int b = 0; b < py; ++b) { d.rows_before[b] = acc; acc += cyc_count(ny, b, py); }
}

// Element (x, y, z) of global(nx,ny,nz) goes to its position in the rank-major chunk buffer
// (line_pos).  One block row per (y, z) line of the field (blockIdx.y = y, blockIdx.z = z), threads along
// x: the row's rank-grid row and offsets are block-uniform, and a thread does one 32-bit
// division (x by px) instead of the 64-bit element decomposition (r4: the kernels were
// integer-division bound at ~0.7 TB/s).
constexpr int kPackThreads = 128;
__device__ inline long long line_pos(const Decomp &d, int x, int y, int z) {
  const int idy = y % d.py, j = y / d.py;   // block-uniform
  const int lny = cyc_count(d.ny, idy, d.py);
  const int i = x / d.px, idx = x - i * d.px;
  const int lnx = cyc_count(d.nx, idx, d.px);
  const long long base = (long long)d.nz * ((long long)d.rows_before[idy] * d.nx +
                                            (long long)lny * d.cols_before[idx]);
  return base + i + (long long)lnx * (j + (long long)lny * z);
}

__global__ void __launch_bounds__(kPackThreads)
pack_columns_kernel(const float *__restrict__ global, Decomp d, float *__restrict__ send) {
  const int x = blockIdx.x * kPackThreads + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= d.nx) return;
  send[line_pos(d, x, y, z)] = global[((long long)z * d.ny + y) * d.nx + x];
}

__global__ void __launch_bounds__(kPackThreads)
unpack_columns_kernel(const float *__restrict__ recv, Decomp d, float *__restrict__ global) {
  const int x = blockIdx.x * kPackThreads + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= d.nx) return;
  global[((long long)z * d.ny + y) * d.nx + x] = recv[line_pos(d, x, y, z)];
}

// tmp3d = sgemv('n', n2d*nz_ph, k, 1.0/(g*k), ph, ., x = 1, 0.0) in the reference BLAS
// order (y = 0; y += (alpha*x(j)) * A(:,j) for j = 1..k), then (:500-505)
//   stagger 1: alt = tmp3d;  stagger 0: alt = (tmp3d(:,:,2:nz_ph) + tmp3d(:,:,1:nz)) * 0.5
__device__ inline float member_mean(const float *__restrict__ ph, long long stride, int k,
                                    float alpha, long long at) {
  float y = 0.0f;
  for (int m = 0; m < k; ++m) y = y + alpha * ph[at + m * stride];
  return y;
}

__global__ void __launch_bounds__(256)
vcoord_mean_kernel(const float *__restrict__ ph, long long n2d, int nz_ph, int k, int stagger,
                   float alpha, float *__restrict__ alt) {
  const int nz_out = stagger == 1 ? nz_ph : nz_ph - 1;
  const long long stride = n2d * nz_ph;  // member stride of ph(n2d, nz_ph, 0:k-1)
  const long long n = n2d * nz_out;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n;
       e += (long long)gridDim.x * 256) {
    if (stagger == 1) {
      alt[e] = member_mean(ph, stride, k, alpha, e);
    } else {
      const float lo = member_mean(ph, stride, k, alpha, e);
      const float hi = member_mean(ph, stride, k, alpha, e + n2d);
      alt[e] = (hi + lo) * 0.5f;
    }
  }
}

// write_mean's member sum (module_grid.f90:744-822, the rank-local part): fp32, member order
__global__ void __launch_bounds__(256)
member_sum_kernel(const float *__restrict__ f, long long n, int nm, float *__restrict__ out) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n;
       e += (long long)gridDim.x * 256) {
    float s = 0.0f;
    for (int m = 0; m < nm; ++m) s = s + f[e + (long long)m * n];
    out[e] = s;
  }
}

// sscal (module_grid.f90:827-...)
__global__ void __launch_bounds__(256)
scale_kernel(float *__restrict__ x, long long n, float alpha) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n;
       e += (long long)gridDim.x * 256)
    x[e] = alpha * x[e];
}

static dim3 grid_for(long long n) {
  const long long b = (n + 255) / 256;
  return dim3((unsigned)std::min<long long>(std::max<long long>(b, 1), 1 << 20));
}

hipError_t launch_pack_columns(hipStream_t s, const float *global, const Decomp &d,
                               float *send) {
  const long long n = (long long)d.nx * d.ny * d.nz;
  if (n == 0) return hipSuccess;
  if (d.ny > 65535 || d.nz > 65535) return hipErrorInvalidValue;
  const dim3 grid((d.nx + kPackThreads - 1) / kPackThreads, d.ny, d.nz);
  hipLaunchKernelGGL(pack_columns_kernel, grid, dim3(kPackThreads), 0, s, global, d, send);
  return hipGetLastError();
}

hipError_t launch_unpack_columns(hipStream_t s, const float *recv, const Decomp &d,
                                 float *global) {
  const long long n = (long long)d.nx * d.ny * d.nz;
  if (n == 0) return hipSuccess;
  if (d.ny > 65535 || d.nz > 65535) return hipErrorInvalidValue;
  const dim3 grid((d.nx + kPackThreads - 1) / kPackThreads, d.ny, d.nz);
  hipLaunchKernelGGL(unpack_columns_kernel, grid, dim3(kPackThreads), 0, s, recv, d, global);
  return hipGetLastError();
}

hipError_t launch_vcoord_mean(hipStream_t s, const float *ph, long long n2d, int nz_ph, int k,
                              int stagger, float alpha, float *alt) {
  const long long n = n2d * (stagger == 1 ? nz_ph : nz_ph - 1);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(vcoord_mean_kernel, grid_for(n), dim3(256), 0, s, ph, n2d, nz_ph, k,
                     stagger, alpha, alt);
  return hipGetLastError();
}

hipError_t launch_member_sum(hipStream_t s, const float *fields, long long n, int nm,
                             float *out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(member_sum_kernel, grid_for(n), dim3(256), 0, s, fields, n, nm, out);
  return hipGetLastError();
}

hipError_t launch_scale(hipStream_t s, float *x, long long n, float alpha) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scale_kernel, grid_for(n), dim3(256), 0, s, x, n, alpha);
  return hipGetLastError();
}

}  // namespace cwbl
