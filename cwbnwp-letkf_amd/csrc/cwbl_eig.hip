// cwbl_eig.hip — eigenvalues of A = (k-1)/infl I + Yb Yb^T for the eigenvalue output of
// cwbl_solve_batch, at every k the library supports.
//
// letkf_solve's inverse_matrix takes the eigendecomposition of A with dsyevd('v','l')
// (module_eigen.f90:48-49), whose eigenvalues come back in ascending order.  The tq kernels
// (cwbl_tq.hip, cwbl_tq_big.hip) already reduce A to the tridiagonal T = Q^T A Q with
// Householder reflectors (dsytd2 order) before their quadrature, so the spectrum is T's: in
// assembled mode they write d_i and c(i, i+1) of every point, and this kernel finds T's
// eigenvalues by bisection on the Sturm count (the LDL^T inertia of T - x I, as LAPACK's
// dstebz does), one thread per eigenvalue, every thread converging to fp64 resolution.
// Eigenvalue i is the i-th smallest, so the output is ascending by construction.  The
// padding rows of T (k < KP) are decoupled unit rows (c(k-1, k) = 0 exactly) and are not
// read.  A is SPD with lambda >= inflat, so the bisection's relative accuracy is that of the
// reduction: |d lambda| <~ k eps ||A||.
#include "cwbl_internal.h"

#include <cfloat>

namespace cwbl {

constexpr int kEigThreads = 128;  // >= the largest k (CWBL_MAX_MEMBERS)

__global__ void __launch_bounds__(kEigThreads)
tridiag_eigvals_kernel(int kp, int k, int npts, const double *__restrict__ tri,
                       double *__restrict__ evals) {
  __shared__ double d[kEigThreads], e2[kEigThreads], ea[kEigThreads];
  const int p = blockIdx.x, tid = threadIdx.x;
  if (p >= npts) return;
  const double *t = tri + (long long)p * 2 * kp;
  if (tid < k) {
    d[tid] = t[tid];
    const double e = tid + 1 < k ? t[kp + tid] : 0.0;  // c(i, i+1); none past row k-1
    e2[tid] = e * e;
    ea[tid] = fabs(e);
  }
  __syncthreads();
  if (tid >= k) return;
  // Gershgorin interval and the pivot floor (dstebz: pivmin = safmin * max(1, max e^2))
  double gl = d[0], gu = d[0], emax2 = 0.0;
  for (int j = 0; j < k; ++j) {
    const double r = (j > 0 ? ea[j - 1] : 0.0) + ea[j];
    gl = fmin(gl, d[j] - r);
    gu = fmax(gu, d[j] + r);
    emax2 = fmax(emax2, e2[j]);
  }
  const double pivmin = DBL_MIN * fmax(1.0, emax2);
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double fudge = 2.0 * DBL_EPSILON * tnorm * k + 2.0 * pivmin;
  double lo = gl - fudge, hi = gu + fudge;
  // number of eigenvalues of T below x: negative pivots of T - x I = L D L^T
  auto count = [&](double x) {
    int n = 0;
    double q = d[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    n += q < 0.0;
    for (int j = 1; j < k; ++j) {
      q = (d[j] - x) - e2[j - 1] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      n += q < 0.0;
    }
    return n;
  };
  // lambda_tid is the smallest x with count(x) > tid: keep count(lo) <= tid < count(hi)
  for (int it = 0; it < 256; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (!(mid > lo && mid < hi)) break;  // the interval is one ulp wide
    if (hi - lo <= 2.0 * DBL_EPSILON * fmax(fabs(lo), fabs(hi)) + pivmin) break;
    if (count(mid) > tid) hi = mid;
    else lo = mid;
  }
  evals[(long long)p * k + tid] = 0.5 * (lo + hi);
}

hipError_t launch_tridiag_eigvals(hipStream_t s, int kp, int k, int npts, const double *tri,
                                  double *evals) {
  if (npts <= 0) return hipSuccess;
  if (k < 1 || k > kEigThreads || kp < k || !tri || !evals) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tridiag_eigvals_kernel, dim3(npts), dim3(kEigThreads), 0, s, kp, k, npts,
                     tri, evals);
  return hipGetLastError();
}

}  // namespace cwbl
