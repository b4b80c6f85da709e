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
#include <cstdint>

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
// (line_pos).  One wavefront per (y, z) line of one member's field (r5: the line index and
// the member come from the block, four lines per 256-thread block, so there is no 65535 limit
// on ny or nz), each lane moving four consecutive x: the global side is one 16-B access per
// lane where the line is 16-B aligned (nx % 4 == 0 and an aligned field), the chunk side four
// 4-B accesses that a wavefront writes as px contiguous runs.  The row's rank-grid row and
// offsets are wave-uniform; a lane does one 32-bit division (x by px) per element.
constexpr int kPackThreads = 256, kPackLines = kPackThreads / 64;
struct LineMap {  // the chunk-side offsets of one (y, z) line
  long long row_base;  // nz * rows_before[idy] * nx: the chunks of rank-grid row idy
  int lny, off_j;      // loc_ny of row idy; j + lny * z
};
__device__ inline LineMap line_map(const Decomp &d, int y, int z) {
  const int idy = y % d.py, j = y / d.py;
  LineMap m;
  m.lny = cyc_count(d.ny, idy, d.py);
  m.row_base = (long long)d.nz * d.rows_before[idy] * d.nx;
  m.off_j = j + m.lny * z;
  return m;
}
__device__ inline long long chunk_pos(const Decomp &d, const LineMap &m, int x) {
  const int i = x / d.px, idx = x - i * d.px;
  const int lnx = cyc_count(d.nx, idx, d.px);
  return m.row_base + (long long)d.nz * m.lny * d.cols_before[idx] + i +
         (long long)lnx * m.off_j;
}

// DIR 0: pack (global -> chunks), 1: unpack (chunks -> global); VEC: 16-B global accesses;
// PXV: the chunk side of a lane's four x as one float4 (px = 1: x0..x0+3 are consecutive in
// one chunk), two float2 (px = 2: x0, x0+2 and x0+1, x0+3 pair up in the two chunks) or four
// floats (px >= 3: each store instruction of a wave writes 64 consecutive floats of one chunk)
template <int DIR, bool VEC, int PXV>
__global__ void __launch_bounds__(kPackThreads)
transpose_columns_kernel(const float *__restrict__ src, long long sstride, Decomp d,
                         float *__restrict__ dst, long long dstride, long long nlines) {
  const long long line = (long long)blockIdx.x * kPackLines + (threadIdx.x >> 6);
  if (line >= nlines) return;
  const int lane = threadIdx.x & 63;
  const int y = (int)(line % d.ny), z = (int)(line / d.ny);
  const LineMap m = line_map(d, y, z);
  const float *__restrict__ s = src + (long long)blockIdx.y * sstride;
  float *__restrict__ t = dst + (long long)blockIdx.y * dstride;
  const long long gline = line * d.nx;  // global offset of the line
  for (int x0 = 4 * lane; x0 < d.nx; x0 += 256) {
    if (VEC && x0 + 3 < d.nx) {
      float4 v;
      if (DIR == 1) {
        if constexpr (PXV == 1) {
          v = *reinterpret_cast<const float4 *>(s + chunk_pos(d, m, x0));
        } else if constexpr (PXV == 2) {
          const float2 a = *reinterpret_cast<const float2 *>(s + chunk_pos(d, m, x0));
          const float2 b = *reinterpret_cast<const float2 *>(s + chunk_pos(d, m, x0 + 1));
          v = make_float4(a.x, b.x, a.y, b.y);
        } else {
          v.x = s[chunk_pos(d, m, x0)];
          v.y = s[chunk_pos(d, m, x0 + 1)];
          v.z = s[chunk_pos(d, m, x0 + 2)];
          v.w = s[chunk_pos(d, m, x0 + 3)];
        }
        *reinterpret_cast<float4 *>(t + gline + x0) = v;
      } else {
        v = *reinterpret_cast<const float4 *>(s + gline + x0);
        if constexpr (PXV == 1) {
          *reinterpret_cast<float4 *>(t + chunk_pos(d, m, x0)) = v;
        } else if constexpr (PXV == 2) {
          *reinterpret_cast<float2 *>(t + chunk_pos(d, m, x0)) = make_float2(v.x, v.z);
          *reinterpret_cast<float2 *>(t + chunk_pos(d, m, x0 + 1)) = make_float2(v.y, v.w);
        } else {
          t[chunk_pos(d, m, x0)] = v.x;
          t[chunk_pos(d, m, x0 + 1)] = v.y;
          t[chunk_pos(d, m, x0 + 2)] = v.z;
          t[chunk_pos(d, m, x0 + 3)] = v.w;
        }
      }
    } else {
      const int n = min(4, d.nx - x0);
      for (int e = 0; e < n; ++e) {
        if (DIR == 0) t[chunk_pos(d, m, x0 + e)] = s[gline + x0 + e];
        else t[gline + x0 + e] = s[chunk_pos(d, m, x0 + e)];
      }
    }
  }
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

// nm member fields: member i at src + i * sstride, dst + i * dstride (elements)
hipError_t launch_transpose_columns(hipStream_t s, bool unpack, const float *src,
                                    long long sstride, int nm, const Decomp &d, float *dst,
                                    long long dstride) {
  const long long nlines = (long long)d.ny * d.nz;
  if (nlines == 0 || d.nx == 0 || nm <= 0) return hipSuccess;
  if (nm > 65535) return hipErrorInvalidValue;
  const long long nb = (nlines + kPackLines - 1) / kPackLines;
  if (nb >= (1LL << 31)) return hipErrorInvalidValue;
  // the global side is 16-B aligned line by line when nx % 4 == 0, its base is 16-B aligned
  // and so is every member's (stride % 4 == 0)
  const float *g = unpack ? dst : src;
  const long long gs = unpack ? dstride : sstride;
  const bool vec = d.nx % 4 == 0 && (reinterpret_cast<uintptr_t>(g) & 15) == 0 &&
                   (nm == 1 || gs % 4 == 0);
  // the chunk side as float4 / float2: px = 1 or 2 and every chunk offset a multiple of 4
  // (nx % 4 == 0 makes every chunk's extents and line offsets multiples of 4 / 2 alike) and
  // every member of the chunk buffer aligned
  const float *ck = unpack ? src : dst;
  const long long cs = unpack ? sstride : dstride;
  const bool cal = vec && (reinterpret_cast<uintptr_t>(ck) & 15) == 0 && (nm == 1 || cs % 4 == 0);
  const int pxv = cal && d.px == 1 ? 1 : cal && d.px == 2 ? 2 : 0;
  const dim3 grid((unsigned)nb, (unsigned)nm);
#define CWBL_TRANSPOSE_LAUNCH(DIR, VEC, PXV)                                                   \
  hipLaunchKernelGGL((transpose_columns_kernel<DIR, VEC, PXV>), grid, dim3(kPackThreads), 0, s, \
                     src, sstride, d, dst, dstride, nlines)
  if (!vec) {
    if (!unpack) CWBL_TRANSPOSE_LAUNCH(0, false, 0);
    else CWBL_TRANSPOSE_LAUNCH(1, false, 0);
  } else if (!unpack) {
    if (pxv == 1) CWBL_TRANSPOSE_LAUNCH(0, true, 1);
    else if (pxv == 2) CWBL_TRANSPOSE_LAUNCH(0, true, 2);
    else CWBL_TRANSPOSE_LAUNCH(0, true, 0);
  } else {
    if (pxv == 1) CWBL_TRANSPOSE_LAUNCH(1, true, 1);
    else if (pxv == 2) CWBL_TRANSPOSE_LAUNCH(1, true, 2);
    else CWBL_TRANSPOSE_LAUNCH(1, true, 0);
  }
#undef CWBL_TRANSPOSE_LAUNCH
  return hipGetLastError();
}

hipError_t launch_pack_columns(hipStream_t s, const float *global, const Decomp &d,
                               float *send) {
  return launch_transpose_columns(s, false, global, 0, 1, d, send, 0);
}

hipError_t launch_unpack_columns(hipStream_t s, const float *recv, const Decomp &d,
                                 float *global) {
  return launch_transpose_columns(s, true, recv, 0, 1, d, global, 0);
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
