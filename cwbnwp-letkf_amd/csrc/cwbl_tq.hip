// cwbl_tq.hip — solve_tq_kernel<KP>: the per-point LETKF solve without an explicit
// eigendecomposition.
//
// letkf_solve (module_letkf_core.f90:598-700) forms A = (k-1)/infl I + Yb Yb^T, takes its
// eigendecomposition A = V L V^T (dsyevd, module_eigen.f90:37-108) and uses it for two
// products:
//     wbar = V L^-1 V^T (Yb d)            (Pa Yb^T R^-1 d, :650-660)
//     W    = V sqrt((k-1) L^-1) V^T       (symmetric square root of (k-1) Pa, :661-670)
// and the analysis of member m is xb_mean + wbar . x' + (W x')_m  (:671-679).  Only these
// two matrix functions of A are needed, applied to two vectors, so this kernel computes
// them as such:
//   1. A is assembled exactly as in the Jacobi kernel (fp64, 4x4 register blocks) and moved
//      into registers, one row of A per lane.
//   2. Householder tridiagonalisation A = Q T Q^T (dsytd2 order), applied on the fly to
//      b1 = Yb d and x' (u1 = Q^T b1, u2 = Q^T x').  Rows stay in VGPRs; per step only the
//      pivot row, v and w cross lanes (LDS broadcasts + DPP reductions).
//   3. wbar . x' = b1^T A^-1 x' = u1^T T^-1 u2, and A^-1/2 x' = Q T^-1/2 u2 with
//          T^-1/2 = sum_j  omega_j (T + sigma_j I)^-1
//      the elliptic-substitution midpoint rule for (2/pi) int_0^inf (t^2 + T)^-1 dt on the
//      spectrum bound [m, M] = [(k-1)/infl, trace A] (Hale, Higham & Trefethen 2008), 31
//      nodes for the decade of M/m (tables built on the host, cwbl_abi.hip).  Each node is
//      one shifted SPD tridiagonal solve, done as a twisted (top/bottom) factorisation by a
//      lane pair: lanes n and n+32 solve node n; pair 31 solves T^-1 u2 exactly.
//   4. Q is applied back to T^-1/2 u2 (the stored reflectors, last first).
// Every step is fp64; the fp32 inputs and the fp32 RTPP/RTPS epilogue follow the
// reference's operation order as in the Jacobi kernel.  Results agree with the
// eigendecomposition path to the rounding of fp64 (the rule's relative error is below
// 1e-13 up to M/m = 1e8), well inside the parity tolerance.
#include "cwbl_device.h"

namespace cwbl {

constexpr int kTqChunk = 32;  // columns staged per round (LDS budget: ~11 KB per wave)

template <int KP>
struct TqSmem {
  static constexpr int NB = KP / 4;
  static constexpr int PLD = 4 * NB + 4;  // pb row pitch: 2*PLD = 8*odd dwords, so the 8 block
                                          // rows of a half wave hit disjoint bank octets
  union {
    ColumnChunk<KP, kTqChunk> ch;
    struct {
      double hv[KP * (KP - 1) / 2];       // Householder vectors, packed (v_j: k-1-j entries)
      union {
        double pb[NB][PLD];               // A v partials: pb[R][4c+r] = block (R,c), row r
        // T and the transformed vectors, twice: [0] in row order, [1] mirrored (row KP-1-t),
        // so that the top and bottom lanes of a twisted solve read at the same offsets
        struct {
          double md[2][KP];               // diagonal
          double mc[2][KP];               // coupling to the previous (mirrored) row
          double mu1[2][KP], mu2[2][KP];  // Q^T b1, Q^T x'
        } t;
      } x;
    } h;
  } u;
  double col[KP];                         // pivot column of the current step
  double vb[KP], wb[KP];                  // v and w of the current step (zero above the pivot)
  double td[KP], te[KP];                  // T: diagonal, sub-diagonal (te[i] couples i, i+1)
  double y[KP];                           // T^-1/2 u2
  double tau[KP];                         // Householder scalars
  float xb[KP], xa[KP];
  double scal[4];
  float fscal[4];
};

template <int KP, bool ASSEMBLED>
__global__ void __launch_bounds__(64)
solve_tq_kernel(const TreeDesc *__restrict__ trees, SolveConsts c, SlabDev slab, long long g0,
                int npts, const int *__restrict__ nbr_cnt, const int *__restrict__ nbr_idx,
                const float *__restrict__ nbr_r2, const long long *__restrict__ col_off,
                const float *__restrict__ yo_in, const float *__restrict__ yb_in,
                const float *__restrict__ xb_in, float *__restrict__ xa_out,
                int2 *__restrict__ info) {
  static_assert(KP % 8 == 0 && KP <= 64, "KP");
  constexpr int H = KP / 2;
  constexpr int NBL = AsmLayout<KP>::NBL, NBLK = AsmLayout<KP>::NBLK;
  __shared__ TqSmem<KP> sm;

  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int lane = threadIdx.x;
  const int k = c.k;

  long long P = 0;  // var index of member 0
  if constexpr (!ASSEMBLED) {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long r = g / slab.ix_lim;
    const int j = (int)(r % slab.iy_lim);
    const int kz = (int)(r / slab.iy_lim);
    P = i + (long long)slab.nx * (j + (long long)slab.ny * kz);
    if (lane < KP) sm.xb[lane] = lane < k ? slab.var[P + slab.L * lane] : 0.0f;
  } else {
    if (lane < KP) sm.xb[lane] = lane < k ? xb_in[(long long)gi * k + lane] : 0.0f;
  }

  int bi[NBL], bj[NBL];
  block_of_lane<KP>(lane, bi, bj);
  double acc[NBL][16];
  double b1acc;
  int ptot;
  assemble_point<KP, kTqChunk, ASSEMBLED>(sm.u.ch, trees, c, gi, lane, nbr_cnt, nbr_idx,
                                          nbr_r2, col_off, yo_in, yb_in, bi, bj, acc, b1acc,
                                          ptot);

  if (ptot == 0) {  // no accepted observation: var left unchanged (:220, :226)
    if (lane == 0 && info) info[gi] = make_int2(0, 0);
    if constexpr (ASSEMBLED) {
      if (lane < k) xa_out[(long long)gi * k + lane] = sm.xb[lane];
    }
    return;
  }

  if (c.debug_stop == 1) {  // timing ablation: keep the assembly live, skip the rest
    if (lane == 0 && info) info[gi] = make_int2(ptot, (int)(acc[0][0] + b1acc));
    return;
  }
  // ---- A = inflat*I + Yb Yb^T, kept in the assembly's 4x4 register blocks ---------------
  const double inflat_r8 = (double)c.inflat;
#pragma unroll
  for (int it = 0; it < NBL; ++it) {
    if (lane + 64 * it < NBLK && bi[it] == bj[it]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = 4 * bi[it] + r;
        acc[it][5 * r] = ii < k ? acc[it][5 * r] + inflat_r8 : 1.0;
      }
    }
  }
  if (lane == 0) {  // xb_mean = sum(xb) * nmember_inv in fp32 (:671)
    float s = 0.0f;
    for (int mm = 0; mm < k; ++mm) s = s + sm.xb[mm];
    sm.scal[0] = (double)(s * c.nmember_inv);
  }
  if (lane < KP) {  // padding of T: decoupled unit rows
    sm.td[lane] = 1.0;
    sm.te[lane] = 0.0;
    sm.tau[lane] = 0.0;
  }
  __syncthreads();
  const double xb_mean = sm.scal[0];
  double ux = (lane < k) ? (double)sm.xb[lane] - xb_mean : 0.0;  // x', becomes Q^T x'
  double ub = (lane < KP) ? b1acc : 0.0;                          // Yb d, becomes Q^T b1

  // ---- Householder tridiagonalisation (lower, dsytd2 order) ------------------------------
  // Lane L keeps its lower 4x4 blocks (bi, bj) of A.  Per step j: the blocks of block
  // column j/4 publish column j; lane i < KP forms v_i; every block adds its row and
  // (transposed) column partial of A v into pb; lane i sums row i of pb; A -= v w^T + w v^T
  // block by block.
  double trace = 0.0;
  for (int j = 0; j < k; ++j) {
    const int J = j >> 2, qj = j & 3;
#pragma unroll
    for (int it = 0; it < NBL; ++it) {
      if (lane + 64 * it < NBLK && bj[it] == J) {
        double cv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cv[r] = qj == 0 ? acc[it][4 * r] : qj == 1 ? acc[it][4 * r + 1]
                : qj == 2 ? acc[it][4 * r + 2] : acc[it][4 * r + 3];
        *reinterpret_cast<double2 *>(&sm.col[4 * bi[it]]) = make_double2(cv[0], cv[1]);
        *reinterpret_cast<double2 *>(&sm.col[4 * bi[it] + 2]) = make_double2(cv[2], cv[3]);
      }
    }
    __syncthreads();
    const double dj = sm.col[j];
    trace += dj;
    if (lane == 0) sm.td[j] = dj;
    if (j >= k - 2) {  // trailing 2x2 block: already tridiagonal
      if (j == k - 2 && lane == 0) sm.te[j] = sm.col[j + 1];
      continue;
    }
    const double x = (lane > j + 1 && lane < k) ? sm.col[lane] : 0.0;
    const double alpha = sm.col[j + 1];
    const double xn2 = wave_sum_dpp(x * x);
    double tau = 0.0, beta = alpha, scal = 0.0;
    if (xn2 > 0.0) {  // dlarfg
      beta = -copysign(sqrt(fma(alpha, alpha, xn2)), alpha);
      tau = (beta - alpha) / beta;
      scal = 1.0 / (alpha - beta);
    }
    if (lane == 0) {
      sm.te[j] = beta;
      sm.tau[j] = tau;
    }
    if (tau == 0.0) continue;  // H_j = I (uniform)
    const double v = lane == j + 1 ? 1.0 : x * scal;
    const int off = j * (k - 1) - j * (j - 1) / 2;  // packed start of v_j
    if (lane < KP) sm.vb[lane] = v;
    if (lane > j && lane < k) sm.u.h.hv[off + lane - (j + 1)] = v;
    __syncthreads();
    // partials of A v
    double vi[NBL][4], vj[NBL][4];
#pragma unroll
    for (int it = 0; it < NBL; ++it) {
      if (lane + 64 * it < NBLK) {
        const double2 a0 = *reinterpret_cast<const double2 *>(&sm.vb[4 * bi[it]]);
        const double2 a1 = *reinterpret_cast<const double2 *>(&sm.vb[4 * bi[it] + 2]);
        const double2 b0 = *reinterpret_cast<const double2 *>(&sm.vb[4 * bj[it]]);
        const double2 b1 = *reinterpret_cast<const double2 *>(&sm.vb[4 * bj[it] + 2]);
        vi[it][0] = a0.x; vi[it][1] = a0.y; vi[it][2] = a1.x; vi[it][3] = a1.y;
        vj[it][0] = b0.x; vj[it][1] = b0.y; vj[it][2] = b1.x; vj[it][3] = b1.y;
        double pr[4], pc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pr[r] = acc[it][4 * r] * vj[it][0];
#pragma unroll
          for (int q = 1; q < 4; ++q) pr[r] = fma(acc[it][4 * r + q], vj[it][q], pr[r]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pc[q] = acc[it][q] * vi[it][0];
#pragma unroll
          for (int r = 1; r < 4; ++r) pc[q] = fma(acc[it][4 * r + q], vi[it][r], pc[q]);
        }
        double *dst = &sm.u.h.x.pb[bi[it]][4 * bj[it]];
        *reinterpret_cast<double2 *>(dst) = make_double2(pr[0], pr[1]);
        *reinterpret_cast<double2 *>(dst + 2) = make_double2(pr[2], pr[3]);
        if (bi[it] != bj[it]) {
          double *dt = &sm.u.h.x.pb[bj[it]][4 * bi[it]];
          *reinterpret_cast<double2 *>(dt) = make_double2(pc[0], pc[1]);
          *reinterpret_cast<double2 *>(dt + 2) = make_double2(pc[2], pc[3]);
        }
      }
    }
    __syncthreads();
    double pp = 0.0;
    if (lane < KP) {
      const double *prow = &sm.u.h.x.pb[lane >> 2][lane & 3];
#pragma unroll
      for (int cb = 0; cb < TqSmem<KP>::NB; ++cb) pp += prow[4 * cb];
    }
    const double p = (lane > j && lane < k) ? tau * pp : 0.0;
    const double s1 = wave_sum_dpp(p * v);
    const double s2 = wave_sum_dpp(v * ux);
    const double s3 = wave_sum_dpp(v * ub);
    const double w = fma(-0.5 * tau * s1, v, p);  // w = p - (tau/2)(p.v) v
    ux = fma(-tau * s2, v, ux);
    ub = fma(-tau * s3, v, ub);
    if (lane < KP) sm.wb[lane] = w;
    __syncthreads();
    // A <- A - v w^T - w v^T (rows and columns <= j are untouched: v, w vanish there)
#pragma unroll
    for (int it = 0; it < NBL; ++it) {
      if (lane + 64 * it < NBLK) {
        const double2 a0 = *reinterpret_cast<const double2 *>(&sm.wb[4 * bi[it]]);
        const double2 a1 = *reinterpret_cast<const double2 *>(&sm.wb[4 * bi[it] + 2]);
        const double2 b0 = *reinterpret_cast<const double2 *>(&sm.wb[4 * bj[it]]);
        const double2 b1 = *reinterpret_cast<const double2 *>(&sm.wb[4 * bj[it] + 2]);
        const double wi[4] = {a0.x, a0.y, a1.x, a1.y};
        const double wj[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[it][4 * r + q] =
                fma(-vi[it][r], wj[q], fma(-wi[r], vj[it][q], acc[it][4 * r + q]));
      }
    }
  }
  __syncthreads();
  if (lane < KP) {  // T and Q^T b1, Q^T x' in row order and mirrored
    const double di = sm.td[lane];
    const double cprev = lane >= 1 ? sm.te[lane - 1] : 0.0;  // couples lane-1, lane
    const double cmir = sm.te[KP - 1 - lane];                // couples KP-1-lane, KP-lane
    sm.u.h.x.t.md[0][lane] = di;
    sm.u.h.x.t.md[1][KP - 1 - lane] = di;
    sm.u.h.x.t.mc[0][lane] = cprev;
    sm.u.h.x.t.mc[1][lane] = cmir;
    sm.u.h.x.t.mu1[0][lane] = ub;
    sm.u.h.x.t.mu1[1][KP - 1 - lane] = ub;
    sm.u.h.x.t.mu2[0][lane] = ux;
    sm.u.h.x.t.mu2[1][KP - 1 - lane] = ux;
  }
  __syncthreads();

  if (c.debug_stop == 2) {
    if (lane == 0 && info) info[gi] = make_int2(ptot, (int)(trace + ux + ub));
    return;
  }
  // ---- T^-1/2 u2 by quadrature, u1^T T^-1 u2 exactly --------------------------------------
  // spectrum of A within [m, M]: m = inflat (A - inflat I = Yb Yb^T >= 0), M = trace(A)
  const double m = inflat_r8;
  const double ratio = trace / m - (double)(k - 1);  // lam_max <= trace - (k-1) m
  int level = 1;
  double dec = 10.0;
  while (level < kQuadLevels && dec < ratio) {
    dec *= 10.0;
    ++level;
  }
  const int node = lane & 31, side = lane >> 5;
  double sigma = 0.0, omega = 0.0;
  if (node < kQuadNodes) {
    const double2 tw = c.quad[(level - 1) * 32 + node];
    sigma = m * tw.x;
    omega = sqrt(m) * tw.y;
  }
  const auto &tt = sm.u.h.x.t;
  const double *dd = tt.md[side], *cc = tt.mc[side], *uu = tt.mu2[side], *u1 = tt.mu1[side];
  double rd[H], g[H];
  double dl = dd[0] + sigma;
  g[0] = uu[0];
  rd[0] = rcp64(dl);
#pragma unroll
  for (int t = 1; t < H; ++t) {
    const double ct = cc[t];
    const double l = ct * rd[t - 1];
    dl = fma(-l, ct, dd[t] + sigma);
    g[t] = fma(-l, g[t - 1], uu[t]);
    rd[t] = rcp64(dl);
  }
  // meeting rows H-1 (top) and H (bottom): 2x2 solve with the partner lane's pivot
  const double cm = tt.mc[0][H];
  const double dlo = __shfl_xor(dl, 32, 64), go = __shfl_xor(g[H - 1], 32, 64);
  double xv = (g[H - 1] * dlo - cm * go) / fma(dl, dlo, -cm * cm);
  double dot = u1[H - 1] * xv;  // node 31: u1 . T^-1 u2
  {
    const double ys = half_sum_dpp(omega * xv);
    if (node == 0) sm.y[side ? H : H - 1] = ys;
  }
#pragma unroll
  for (int t = H - 2; t >= 0; --t) {
    xv = (g[t] - cc[t + 1] * xv) * rd[t];
    dot = fma(u1[t], xv, dot);
    const double ys = half_sum_dpp(omega * xv);
    if (node == 0) sm.y[side ? KP - 1 - t : t] = ys;
  }
  const double d = readlane_f64(dot, 31) + readlane_f64(dot, 63);  // wbar . x'
  __syncthreads();

  if (c.debug_stop == 3) {
    if (lane == 0 && info) info[gi] = make_int2(ptot, (int)d);
    return;
  }
  // ---- back-transform: y <- Q y = H_0 H_1 ... H_{k-3} y -----------------------------------
  double yl = lane < KP ? sm.y[lane] : 0.0;
  for (int j = k - 3; j >= 0; --j) {
    const double tj = sm.tau[j];
    if (tj == 0.0) continue;
    const int off = j * (k - 1) - j * (j - 1) / 2;
    const double vj = (lane > j && lane < k) ? sm.u.h.hv[off + lane - (j + 1)] : 0.0;
    const double s = wave_sum_dpp(vj * yl);
    yl = fma(-tj * s, vj, yl);
  }
  const double sk = sqrt((double)(k - 1));
  if (lane < KP) sm.xa[lane] = (float)(xb_mean + (d + sk * yl));  // xa = wbar (:675-679)
  __syncthreads();

  // ---- RTPP / RTPS (:684-698), fp32 in the reference's order -------------------------
  if (c.use_rtpp || c.use_rtps) {
    if (lane == 0) {
      float s = 0.0f;
      for (int mm = 0; mm < k; ++mm) s = s + sm.xa[mm];
      sm.fscal[0] = s * c.nmember_inv;  // xa_mean
    }
    __syncthreads();
    const float xa_mean = sm.fscal[0];
    const double xpl = lane < k ? (double)sm.xb[lane] - xb_mean : 0.0;
    float xap = 0.0f;
    if (lane < k) {
      xap = sm.xa[lane] - xa_mean;
      if (c.use_rtpp)
        xap = (float)((double)((1.0f - c.rtpp_alpha) * xap) + (double)c.rtpp_alpha * xpl);
    }
    if (c.use_rtps) {
      __syncthreads();
      if (lane < k) sm.xa[lane] = xap;  // stage xa_prime
      __syncthreads();
      if (lane == 0) {
        double d8 = 0.0;
        for (int mm = 0; mm < k; ++mm) {
          const double xp = (double)sm.xb[mm] - xb_mean;
          d8 = d8 + xp * xp;
        }
        const float xb_std = (float)d8;
        float xa_std = 0.0f;
        for (int mm = 0; mm < k; ++mm) xa_std = xa_std + sm.xa[mm] * sm.xa[mm];
        sm.fscal[1] = c.rtps_alpha * sqrtf(xb_std / xa_std) - c.rtps_alpha + 1.0f;
      }
      __syncthreads();
      xap = xap * sm.fscal[1];
    }
    if (lane < k) sm.xa[lane] = xa_mean + xap;
    __syncthreads();
  }

  if (lane < k) {
    if constexpr (ASSEMBLED) xa_out[(long long)gi * k + lane] = sm.xa[lane];
    else slab.var[P + slab.L * lane] = sm.xa[lane];
  }
  // info.y: decade of the quadrature rule (negative when M/m exceeds the last table)
  if (lane == 0 && info) info[gi] = make_int2(ptot, ratio > dec ? -level : level);
}

template <int KP>
static hipError_t launch_tq_kp(hipStream_t s, bool assembled, const TreeDesc *trees,
                               SolveConsts c, SlabDev slab, long long g0, int npts,
                               const int *nbr_cnt, const int *nbr_idx, const float *nbr_r2,
                               const long long *col_off, const float *yo, const float *yb,
                               const float *xb, float *xa, int2 *info) {
  if (assembled)
    hipLaunchKernelGGL((solve_tq_kernel<KP, true>), dim3(npts), dim3(64), 0, s, trees, c, slab,
                       g0, npts, nbr_cnt, nbr_idx, nbr_r2, col_off, yo, yb, xb, xa, info);
  else
    hipLaunchKernelGGL((solve_tq_kernel<KP, false>), dim3(npts), dim3(64), 0, s, trees, c,
                       slab, g0, npts, nbr_cnt, nbr_idx, nbr_r2, col_off, yo, yb, xb, xa, info);
  return hipGetLastError();
}

hipError_t launch_solve_tq(hipStream_t s, int kp, bool assembled, const TreeDesc *trees,
                           SolveConsts c, SlabDev slab, long long g0, int npts,
                           const int *nbr_cnt, const int *nbr_idx, const float *nbr_r2,
                           const long long *col_off, const float *yo, const float *yb,
                           const float *xb, float *xa, int2 *info) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr) return hipErrorInvalidValue;
#define CWBL_TQ_CASE(K)                                                                      \
  case K:                                                                                    \
    return launch_tq_kp<K>(s, assembled, trees, c, slab, g0, npts, nbr_cnt, nbr_idx, nbr_r2, \
                           col_off, yo, yb, xb, xa, info);
  switch (kp) {
    CWBL_TQ_CASE(8)
    CWBL_TQ_CASE(16)
    CWBL_TQ_CASE(24)
    CWBL_TQ_CASE(32)
    CWBL_TQ_CASE(40)
    CWBL_TQ_CASE(48)
    CWBL_TQ_CASE(56)
    CWBL_TQ_CASE(64)
    default:
      return hipErrorInvalidValue;
  }
#undef CWBL_TQ_CASE
}

}  // namespace cwbl
