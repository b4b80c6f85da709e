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

#include <type_traits>

namespace cwbl {

// Assembly of Yb Yb^T: fp64 FMAs on the lower 4x4 blocks from columns staged in LDS as
// fp64 (16 per round), or on the matrix cores (v_mfma_f64_16x16x4 on 16x16 tiles of
// [Yb; yo], 32 float columns per round).  On gfx950 the FP64 matrix and vector rates are
// equal and the two do not co-issue; the tiles waste 44% of their products at KP = 40, so
// the block form is faster.  The MFMA form is kept for comparison (kTqMfmaAssembly).
constexpr bool kTqMfmaAssembly = true;
constexpr int kTqChunk = kTqMfmaAssembly ? 32 : 16;  // columns staged per round
using TqStage = std::conditional_t<kTqMfmaAssembly, float, double>;

// LDS of one point (KP = 40: 9.4 KB, so 16 waves fit a CU).  The big union is reused by
// phase: staged columns -> half of A -> {Householder vectors + A v partials}, then
// {Householder vectors + Q^T b1, Q^T x', T^-1/2 u2}.  The A v partials of step j only need
// block rows >= j/4 and sit at the top of the region, above the Householder vectors
// written so far.
template <int KP>
struct TqSmem {
  static constexpr int NB = KP / 4;
  static constexpr int PLD = 4 * NB + 4;  // pb row pitch: 2*PLD = 8*odd dwords, so the 8 block
                                          // rows of a half wave hit disjoint bank octets
  // Trailing phase: from step J0T on, the remaining kTail x kTail matrix is held as 2x2
  // blocks (NB2*(NB2+1)/2 = 55 <= 64 lanes), 4x fewer FMAs per lane than 4x4 blocks.
  static constexpr int kTail = 20;
  // (KP = 40 only: with more than one 4x4 block per lane the two phases' live ranges spill)
  static constexpr int J0T = KP == 40 ? KP - kTail : KP;  // first step of the 2x2 phase
  static constexpr int NB2 = kTail / 2;
  static constexpr int NBLK2 = NB2 * (NB2 + 1) / 2;
  static constexpr int PLD2 = 2 * NB2 + 2;  // 2x2-phase partials pitch (>= the packed tail)
  static_assert(NB2 * PLD2 >= kTail * (kTail + 1) / 2 && NBLK2 <= 64, "tail layout");
  static constexpr int NHV = KP * (KP - 1) / 2;  // packed Householder vectors at k = KP
  static constexpr int hv_off(int j) { return j * (KP - 1) - j * (j - 1) / 2; }
  static constexpr int cap() {  // region size: vectors so far + partials of the live rows
    int m = NHV + KP;
    for (int j = 0; j + 2 < KP; ++j) {
      const int need = hv_off(j + 1) + (j < J0T ? (NB - j / 4) * PLD
                                                : (NB2 - (j - J0T) / 2) * PLD2);
      m = need > m ? need : m;
    }
    if (J0T < KP) {  // the packed tail at the switch (in the 2x2 partials' place)
      const int need = hv_off(J0T) + NB2 * PLD2;
      m = need > m ? need : m;
    }
    return m;
  }
  static constexpr int REG = cap();
  static constexpr int pb_base(int J) { return REG - (NB - J) * PLD; }
  static constexpr int pb2_base(int J2) { return REG - (NB2 - J2) * PLD2; }
  union {
    ColumnChunk<KP, kTqChunk, TqStage, kTqMfmaAssembly ? MfmaLayout<KP>::PITCH : KP,
                kTqMfmaAssembly && MfmaLayout<KP>::SWZ, kTqMfmaAssembly && MfmaLayout<KP>::XSW> ch;
    double ah[KP / 2][KP + 2];            // half of A on its way from MFMA tiles to blocks
    double reg[REG];                      // hv[0, NHV) | y after the loop | pb
  } u;
  double col[KP];                         // pivot column of the current step
  double vb[KP];                          // v of the current step (zero above the pivot)
  double wb[KP];                          // w of the current step; Yb d before the loop
  // row i of T and the transformed vectors, one 32-B record per row so that a shifted solve
  // reads a row with one address; record KP only holds c(KP-1,KP) = 0
  double tq[KP + 1][4];                   // d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
  double tau[KP];                         // Householder scalars
};

// waves per SIMD the register allocation is held to (VGPR budget 512 / waves)
template <int KP>
struct TqOccupancy {
  static constexpr int kWaves = KP <= 40 ? 4 : KP <= 48 ? 3 : 2;
};

// ws (assembled mode, nullable): T of every point (d, then c(i, i+1); 2 KP words) for the
// eigenvalue output of cwbl_solve_batch (launch_tridiag_eigvals).
template <int KP, bool ASSEMBLED>
__global__ void __launch_bounds__(64, TqOccupancy<KP>::kWaves)
solve_tq_kernel(const TreeDesc *__restrict__ trees, SolveConsts c, SlabDev slab, long long g0,
                int npts, const int *__restrict__ nbr_cnt, const int *__restrict__ nbr_idx,
                const long long *__restrict__ col_off,
                const float *__restrict__ yo_in, const float *__restrict__ yb_in,
                const float *__restrict__ xb_in, float *__restrict__ xa_out,
                int2 *__restrict__ info, double *__restrict__ ws = nullptr) {
  static_assert(KP % 8 == 0 && KP <= 64, "KP");
  constexpr int H = KP / 2;
  constexpr int NBL = AsmLayout<KP>::NBL, NBLK = AsmLayout<KP>::NBLK;
  using SM = TqSmem<KP>;
  __shared__ SM sm;

  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int lane = threadIdx.x;
  const int k = c.k;

  long long P = 0;  // var index of member 0
  float3 pt = make_float3(0.0f, 0.0f, 0.0f);  // the point's projected x, y and altitude
  float xbl = 0.0f;                            // background of member `lane`
  if constexpr (!ASSEMBLED) {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long r = g / slab.ix_lim;
    const int j = (int)(r % slab.iy_lim);
    const int kz = (int)(r / slab.iy_lim);
    P = i + (long long)slab.nx * (j + (long long)slab.ny * kz);
    if (lane < k) xbl = slab.var[P + slab.L * lane];
    slab_point(slab, g, pt.x, pt.y, pt.z);
  } else {
    if (lane < k) xbl = xb_in[(long long)gi * k + lane];
  }

  int bi[NBL], bj[NBL];
  block_of_lane<KP>(lane, bi, bj);
  double acc[NBL][16];
  double b1acc;
  int ptot;
  if constexpr (!kTqMfmaAssembly) {
    assemble_point<KP, kTqChunk, ASSEMBLED, 64, TqStage>(sm.u.ch, trees, c, gi, lane, nbr_cnt,
                                                         nbr_idx, pt, col_off, yo_in, yb_in,
                                                         bi, bj, acc, b1acc, ptot);
    if (ptot == 0) {  // no accepted observation: var left unchanged (:220, :226)
      if (lane == 0 && info) info[gi] = make_int2(0, 0);
      if constexpr (ASSEMBLED) {
        if (lane < k) xa_out[(long long)gi * k + lane] = xbl;
      }
      return;
    }
    if (CWBL_DBG_STOP(c) == 1) {  // timing ablation: keep the assembly live, skip the rest
      if (lane == 0 && info) info[gi] = make_int2(ptot, (int)(acc[0][0] + b1acc));
      return;
    }
  } else {
    f64x4 tile[MfmaLayout<KP>::NTL];
    assemble_point_mfma<KP, kTqChunk, ASSEMBLED>(sm.u.ch, trees, c, gi, lane, nbr_cnt, nbr_idx,
                                                 pt, col_off, yo_in, yb_in, tile, b1acc, ptot);
    if (ptot == 0) {
      if (lane == 0 && info) info[gi] = make_int2(0, 0);
      if constexpr (ASSEMBLED) {
        if (lane < k) xa_out[(long long)gi * k + lane] = xbl;
        if (ws && lane < KP) {  // T = A = inflat I (no observation)
          ws[(long long)gi * 2 * KP + lane] = lane < k ? (double)c.inflat : 1.0;
          ws[(long long)gi * 2 * KP + KP + lane] = 0.0;
        }
      }
      return;
    }
    if (CWBL_DBG_STOP(c) == 1) {
      double t = b1acc;
#pragma unroll
      for (int q = 0; q < MfmaLayout<KP>::NTL; ++q) t += tile[q][0] + tile[q][3];
      if (lane == 0 && info) info[gi] = make_int2(ptot, (int)t);
      return;
    }
    // MFMA tiles -> LDS (two row halves) -> 4x4 register blocks
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      int t = 0;
#pragma unroll
      for (int I = 0; I < MfmaLayout<KP>::NT; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J, ++t) {
          const int col = 16 * J + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * I + (lane >> 4) + 4 * r;
            if (row / H == half && row < KP && col < KP) sm.u.ah[row - half * H][col] = tile[t][r];
            if (MfmaLayout<KP>::YO_ROW && half == 0 && row == KP && col < KP)
              sm.wb[col] = tile[t][r];  // row KP of Y' Y'^T = Yb d
          }
        }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < NBL; ++it) {
        if (lane + 64 * it < NBLK && (4 * bi[it]) / H == half) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double *src = &sm.u.ah[4 * bi[it] + r - half * H][4 * bj[it]];
            const double2 x0 = *reinterpret_cast<const double2 *>(src);
            const double2 x1 = *reinterpret_cast<const double2 *>(src + 2);
            acc[it][4 * r] = x0.x; acc[it][4 * r + 1] = x0.y;
            acc[it][4 * r + 2] = x1.x; acc[it][4 * r + 3] = x1.y;
          }
        }
      }
      __syncthreads();
    }
    if (MfmaLayout<KP>::YO_ROW && lane < KP) b1acc = sm.wb[lane];
  }
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
  if (lane < KP) {  // padding of T: decoupled unit rows
    sm.tq[lane][0] = 1.0;
    sm.tq[lane][1] = 0.0;
    sm.tau[lane] = 0.0;
  }
  if (lane == 0) sm.tq[KP][1] = 0.0;
  __syncthreads();
  double xb_mean;
  {  // xb_mean = sum(xb) * nmember_inv in fp32 (:671), sequential like the reference
    float s = 0.0f;
    for (int mm = 0; mm < k; ++mm)
      s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xbl), mm));
    xb_mean = (double)(s * c.nmember_inv);
  }
  double ux = (lane < k) ? (double)xbl - xb_mean : 0.0;  // x', becomes Q^T x'
  double ub = (lane < KP) ? b1acc : 0.0;                          // Yb d, becomes Q^T b1

  // ---- Householder tridiagonalisation (lower, dsytd2 order) ------------------------------
  // Lane L keeps its lower 4x4 blocks (bi, bj) of A; from step J0T on (KP >= 40) the
  // trailing kTail x kTail matrix is re-dealt as 2x2 blocks (bi2, bj2), one per lane.  Per
  // step j: the blocks of the pivot's block column publish column j; lane i < KP forms v_i;
  // every block adds its row and (transposed) column partial of A v into pb; lane i sums row
  // i of pb; A -= v w^T + w v^T block by block.
  constexpr int J0T = SM::J0T, NB2 = SM::NB2, PLD2 = SM::PLD2;
  int bi2 = 0, bj2 = 0;  // this lane's block of the 2x2 phase (lane < NBLK2)
  while ((bi2 + 1) * (bi2 + 2) / 2 <= lane) ++bi2;
  bj2 = lane - bi2 * (bi2 + 1) / 2;
  const bool tail_lane = lane < SM::NBLK2;
  double trace = 0.0;
  auto ld4 = [](const double *p, double (&o)[4]) {
    const double2 a0 = *reinterpret_cast<const double2 *>(p);
    const double2 a1 = *reinterpret_cast<const double2 *>(p + 2);
    o[0] = a0.x; o[1] = a0.y; o[2] = a1.x; o[3] = a1.y;
  };
  // One step of either phase.  The phases run as separate loops so that each keeps its own
  // register assignment (one loop with a run-time phase test copies the blocks between
  // registers every step).  The blocks are reached through the capture at NBL = 1 and
  // through the parameter otherwise: the other way round, the compiler keeps them in scratch.
  auto step = [&](const int j, auto phase, auto q, double (&Ap)[NBL][16])
                  __attribute__((always_inline)) {
    constexpr bool ph2 = decltype(phase)::value;
    constexpr int qj = decltype(q)::value, q2 = qj;  // column within the block: constant
    double (&A)[NBL][16] = *[&]() {
      if constexpr (NBL == 1) return &acc; else return &Ap;
    }();
    const int J = j >> 2;
    const int J2 = (j - J0T) >> 1;
    if constexpr (ph2) {
      if (j == J0T) {  // re-deal the tail: 4x4 blocks -> packed lower triangle -> 2x2 blocks
        double *tri = &sm.u.reg[J0T < KP ? SM::pb2_base(0) : 0];
        constexpr int JB = J0T / 4;
#pragma unroll
        for (int it = 0; it < NBL; ++it) {
          if (lane + 64 * it < NBLK && bi[it] >= JB && bj[it] >= JB) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int a = 4 * (bi[it] - JB) + r, b = 4 * (bj[it] - JB) + q;
                if (a >= b) tri[a * (a + 1) / 2 + b] = A[it][4 * r + q];
              }
          }
        }
        __syncthreads();
        if (tail_lane) {
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int a = 2 * bi2 + r, b = 2 * bj2 + q;
              A[0][2 * r + q] = a >= b ? tri[a * (a + 1) / 2 + b] : tri[b * (b + 1) / 2 + a];
            }
        }
        __syncthreads();
      }
    }
    if constexpr (!ph2) {
#pragma unroll
      for (int it = 0; it < NBL; ++it) {
        if (lane + 64 * it < NBLK && bj[it] == J) {  // publish column j
          *reinterpret_cast<double2 *>(&sm.col[4 * bi[it]]) =
              make_double2(A[it][qj], A[it][4 + qj]);
          *reinterpret_cast<double2 *>(&sm.col[4 * bi[it] + 2]) =
              make_double2(A[it][8 + qj], A[it][12 + qj]);
        }
      }
    } else if (tail_lane && bj2 == J2) {  // publish column j (2x2 phase)
      const double c0 = A[0][q2 & 1], c1 = A[0][2 + (q2 & 1)];
      *reinterpret_cast<double2 *>(&sm.col[J0T + 2 * bi2]) = make_double2(c0, c1);
    }
    __syncthreads();
    const double dj = sm.col[j];
    trace += dj;
    if (lane == 0) sm.tq[j][0] = dj;
    if (j >= k - 2) {  // trailing 2x2 block: already tridiagonal
      if (j == k - 2 && lane == 0) {
        sm.tq[j + 1][1] = sm.col[j + 1];
      }
      return;
    }
    const double x = (lane > j + 1 && lane < k) ? sm.col[lane] : 0.0;
    const double alpha = sm.col[j + 1];
    // x.x, x.ux, x.ub in one pass: v = x * scal + e_{j+1} gives v.u = scal (x.u) + u_{j+1}
    double xn2 = x * x, xux = x * ux, xub = x * ub, pad = 0.0;
    wave_sum4_dpp(xn2, xux, xub, pad);
    double tau = 0.0, beta = alpha, scal = 0.0;
    if (xn2 > 0.0) {  // dlarfg, with fp64 rcp/rsq refined to ~1 ulp
      const double a2 = fma(alpha, alpha, xn2);
      const double r = rsq64(a2);             // 1/|beta|
      beta = -copysign(a2 * r, alpha);
      tau = (beta - alpha) * -copysign(r, alpha);  // (beta - alpha) / beta
      scal = rcp64(alpha - beta);
    }
    if (lane == 0) {
      sm.tq[j + 1][1] = beta;
      sm.tau[j] = tau;
    }
    if (tau == 0.0) return;  // H_j = I (uniform)
    // v_i = x_i * scal (i > j+1), v_{j+1} = 1, 0 elsewhere
    const double v = lane == j + 1 ? 1.0 : x * scal;
    if (lane < KP) sm.vb[lane] = v;
    if (lane > j && lane < k) sm.u.reg[SM::hv_off(0) + j * (k - 1) - j * (j - 1) / 2 + lane - (j + 1)] = v;
    const double s2 = fma(scal, xux, readlane_f64(ux, j + 1));  // v . ux
    const double s3 = fma(scal, xub, readlane_f64(ub, j + 1));  // v . ub
    ux = fma(-tau * s2, v, ux);
    ub = fma(-tau * s3, v, ub);
    __syncthreads();
    // partials of A v (block rows >= J only: v vanishes above)
    double s1p = 0.0;  // this lane's share of v^T A v
    double pp = 0.0;
    if constexpr (!ph2) {
      double *pb = &sm.u.reg[SM::pb_base(J)] - J * SM::PLD;  // pb[R * PLD + col], R >= J
#pragma unroll
      for (int it = 0; it < NBL; ++it) {
        if (lane + 64 * it < NBLK && bi[it] >= J) {
          double vi[4], vj[4];
          ld4(&sm.vb[4 * bi[it]], vi);
          ld4(&sm.vb[4 * bj[it]], vj);
          double pr[4], pc[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pr[r] = A[it][4 * r] * vj[0];
#pragma unroll
            for (int q = 1; q < 4; ++q) pr[r] = fma(A[it][4 * r + q], vj[q], pr[r]);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            pc[q] = A[it][q] * vi[0];
#pragma unroll
            for (int r = 1; r < 4; ++r) pc[q] = fma(A[it][4 * r + q], vi[r], pc[q]);
          }
          double sp = vi[0] * pr[0];
#pragma unroll
          for (int r = 1; r < 4; ++r) sp = fma(vi[r], pr[r], sp);
          double *dst = pb + bi[it] * SM::PLD + 4 * bj[it];
          *reinterpret_cast<double2 *>(dst) = make_double2(pr[0], pr[1]);
          *reinterpret_cast<double2 *>(dst + 2) = make_double2(pr[2], pr[3]);
          if (bi[it] != bj[it]) {
            if (bj[it] >= J) {
              double *dt = pb + bj[it] * SM::PLD + 4 * bi[it];
              *reinterpret_cast<double2 *>(dt) = make_double2(pc[0], pc[1]);
              *reinterpret_cast<double2 *>(dt + 2) = make_double2(pc[2], pc[3]);
            }
            sp = sp + sp;  // the transposed block contributes v_j^T B^T v_i = v_i^T B v_j
          }
          s1p += sp;
        }
      }
      const double s1 = tau * wave_sum_dpp(s1p);  // p . v with p = tau A v
      __syncthreads();
      if (lane < KP && lane > j) {
        const double *prow = pb + (lane >> 2) * SM::PLD + (lane & 3);
        pp = prow[0];
#pragma unroll
        for (int cb = 1; cb < SM::NB; ++cb) pp += prow[4 * cb];
      }
      s1p = s1;
    } else {
      double *pb = &sm.u.reg[SM::pb2_base(J2)] - J2 * PLD2;  // pb[R * PLD2 + col], R >= J2
      if (tail_lane && bi2 >= J2) {
        const double2 vi = *reinterpret_cast<const double2 *>(&sm.vb[J0T + 2 * bi2]);
        const double2 vj = *reinterpret_cast<const double2 *>(&sm.vb[J0T + 2 * bj2]);
        const double pr0 = fma(A[0][1], vj.y, A[0][0] * vj.x);
        const double pr1 = fma(A[0][3], vj.y, A[0][2] * vj.x);
        double sp = fma(vi.y, pr1, vi.x * pr0);
        *reinterpret_cast<double2 *>(pb + bi2 * PLD2 + 2 * bj2) = make_double2(pr0, pr1);
        if (bi2 != bj2) {
          if (bj2 >= J2) {
            const double pc0 = fma(A[0][2], vi.y, A[0][0] * vi.x);
            const double pc1 = fma(A[0][3], vi.y, A[0][1] * vi.x);
            *reinterpret_cast<double2 *>(pb + bj2 * PLD2 + 2 * bi2) = make_double2(pc0, pc1);
          }
          sp = sp + sp;
        }
        s1p = sp;
      }
      const double s1 = tau * wave_sum_dpp(s1p);
      __syncthreads();
      if (lane < KP && lane > j) {
        const double *prow = pb + ((lane - J0T) >> 1) * PLD2 + ((lane - J0T) & 1);
        pp = prow[0];
#pragma unroll
        for (int cb = 1; cb < NB2; ++cb) pp += prow[2 * cb];
      }
      s1p = s1;
    }
    const double s1 = s1p;
    const double p = (lane > j && lane < k) ? tau * pp : 0.0;
    const double w = fma(-0.5 * tau * s1, v, p);  // w = p - (tau/2)(p.v) v
    if (lane < KP) sm.wb[lane] = w;
    __syncthreads();
    // A <- A - v w^T - w v^T (rows and columns <= j are untouched: v, w vanish there)
    if constexpr (!ph2) {
#pragma unroll
      for (int it = 0; it < NBL; ++it) {
        if (lane + 64 * it < NBLK && bi[it] >= J) {
          double vi[4], vj[4], wi[4], wj[4];
          ld4(&sm.vb[4 * bi[it]], vi);
          ld4(&sm.vb[4 * bj[it]], vj);
          ld4(&sm.wb[4 * bi[it]], wi);
          ld4(&sm.wb[4 * bj[it]], wj);
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              A[it][4 * r + q] = fma(-vi[r], wj[q], fma(-wi[r], vj[q], A[it][4 * r + q]));
        }
      }
    } else if (tail_lane && bi2 >= J2) {
      const double2 vi = *reinterpret_cast<const double2 *>(&sm.vb[J0T + 2 * bi2]);
      const double2 vj = *reinterpret_cast<const double2 *>(&sm.vb[J0T + 2 * bj2]);
      const double2 wi = *reinterpret_cast<const double2 *>(&sm.wb[J0T + 2 * bi2]);
      const double2 wj = *reinterpret_cast<const double2 *>(&sm.wb[J0T + 2 * bj2]);
      A[0][0] = fma(-vi.x, wj.x, fma(-wi.x, vj.x, A[0][0]));
      A[0][1] = fma(-vi.x, wj.y, fma(-wi.x, vj.y, A[0][1]));
      A[0][2] = fma(-vi.y, wj.x, fma(-wi.y, vj.x, A[0][2]));
      A[0][3] = fma(-vi.y, wj.y, fma(-wi.y, vj.y, A[0][3]));
    }
  };
  // unrolled by the block width, so that the pivot column's registers are known statically
  using std::false_type, std::true_type, std::integral_constant;
  const int jend1 = k < J0T ? k : J0T;
  for (int j = 0; j < jend1; j += 4) {
    step(j, false_type{}, integral_constant<int, 0>{}, acc);
    if (j + 1 < jend1) step(j + 1, false_type{}, integral_constant<int, 1>{}, acc);
    if (j + 2 < jend1) step(j + 2, false_type{}, integral_constant<int, 2>{}, acc);
    if (j + 3 < jend1) step(j + 3, false_type{}, integral_constant<int, 3>{}, acc);
  }
  if constexpr (J0T < KP) {
    static_assert(J0T % 2 == 0, "2x2 phase alignment");
    for (int j = J0T; j < k; j += 2) {
      step(j, true_type{}, integral_constant<int, 0>{}, acc);
      if (j + 1 < k) step(j + 1, true_type{}, integral_constant<int, 1>{}, acc);
    }
  }
  // after the Householder vectors (the partials are dead): per side, in walk order, the
  // quadrature sum (Ym) and node 31's exact solve (Zm)
  double *Ym = &sm.u.reg[SM::NHV], *Zm = Ym + KP;
  if (lane < KP) {
    sm.tq[lane][2] = ub;
    sm.tq[lane][3] = ux;
  }
  __syncthreads();
  if constexpr (ASSEMBLED) {  // T for the eigenvalue output (cwbl_solve_batch)
    if (ws && lane < KP) {
      ws[(long long)gi * 2 * KP + lane] = sm.tq[lane][0];           // d_i
      ws[(long long)gi * 2 * KP + KP + lane] = sm.tq[lane + 1][1];  // c(i, i+1)
    }
  }

  if (CWBL_DBG_STOP(c) == 2) {
    if (lane == 0 && info) info[gi] = make_int2(ptot, (int)(trace + ux + ub));
    return;
  }
  // ---- T^-1/2 u2 by quadrature, u1^T T^-1 u2 exactly --------------------------------------
  // spectrum of A within [m, M]: m = inflat (A - inflat I = Yb Yb^T >= 0),
  // M = trace(A) - (k-1) m (the other k-1 eigenvalues are >= m)
  const double m = inflat_r8;
  const double ratio = trace / m - (double)(k - 1);
  int level = 1;
  double dec = 10.0;
  while (level < kQuadLevels && dec < ratio) {
    dec *= 10.0;
    ++level;
  }
  const int node = lane & 31, side = lane >> 5;
  // one pass of 31 nodes (+ the exact solve on node 31) up to level kQuadLevels31, a second
  // pass with nodes 31..62 of the 63-node rule above (quad_passes; wave-uniform)
  const int npass = quad_passes(level);
  const double2 *rule = quad_rule(c.quad_r, npass == 1 ? 4 : 8, level);
  // lane side 0 walks rows 0, 1, .. H-1; side 1 walks rows KP-1, KP-2, .. H (mirrored).
  // Forward elimination towards the middle keeps, per row, h_t = g_t / dl_t and
  // m_t = c_{t+1} / dl_t, so that back substitution is x_t = h_t - m_t x_{t+1}.
  // byte offsets into sm.tq: row t of the walk at q0 + dirb t (opaque_after, cwbl_device.h)
  const unsigned q0 = side ? (KP - 1) * 32u : 0u, dirb = side ? (unsigned)-32 : 32u;
  // coupling with the previous mirrored row: c(i-1,i) / c(i,i+1)
  const unsigned csb = side ? 40u : 8u;
  double *ym = Ym + side * H, *zm = Zm + side * H;
  for (int pass = 0; pass < npass; ++pass) {
    const bool exact = pass == 0 && node == 31;
    double sigma = 0.0, omega = 0.0;
    if (!exact) {
      const double2 tw = rule[31 * pass + node];
      sigma = m * tw.x;
      omega = sqrt(m) * tw.y;
    }
    double hh[H], mm[H];
    double dl = lds_at(sm.tq, q0) + sigma;
    double gt = lds_at(sm.tq, q0 + 24);
    double rdl = rcp64(dl);
#pragma unroll
    for (int t = 1; t < H; ++t) {
      const unsigned o = opaque_after(q0, dl) + dirb * (unsigned)t;
      const double ct = lds_at(sm.tq, o + csb);
      const double l = ct * rdl;
      hh[t - 1] = gt * rdl;
      mm[t - 1] = l;  // = c_t / dl_{t-1}
      asm volatile("" : "+v"(hh[t - 1]));  // materialise now: g_{t-1} and 1/dl_{t-1} die here
      dl = fma(-l, ct, lds_at(sm.tq, o) + sigma);
      gt = fma(-l, gt, lds_at(sm.tq, o + 24));
      rdl = rcp64(dl);
      __builtin_amdgcn_sched_barrier(0);  // keep the recurrence in order: bounded live ranges
    }
    // meeting rows H-1 (top) and H (bottom): 2x2 solve with the partner lane's pivot
    const double cm = sm.tq[H][1];
    const double dlo = __shfl_xor(dl, 32, 64), go = __shfl_xor(gt, 32, 64);
    double xv = (gt * dlo - cm * go) / fma(dl, dlo, -cm * cm);
    {
      const double ys = half_sum_dpp(omega * xv);
      if (node == 0) ym[H - 1] = pass ? ym[H - 1] + ys : ys;
      if (exact) zm[H - 1] = xv;
    }
#pragma unroll
    for (int t = H - 2; t >= 0; --t) {
      xv = fma(-mm[t], xv, hh[t]);
      const double ys = half_sum_dpp(omega * xv);
      if (node == 0) ym[t] = pass ? ym[t] + ys : ys;
      if (exact) zm[t] = xv;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();
  const int wi = lane < H ? lane : H + (KP - 1 - lane);  // walk slot of row `lane`
  const double zl = lane < KP ? Zm[wi] : 0.0;
  double yl = lane < KP ? Ym[wi] : 0.0;
  const double d = wave_sum_dpp(lane < KP ? sm.tq[lane][2] * zl : 0.0);  // u1 . T^-1 u2

  if (CWBL_DBG_STOP(c) == 3) {
    if (lane == 0 && info) info[gi] = make_int2(ptot, (int)d);
    return;
  }
  // ---- back-transform: y <- Q y = H_0 H_1 ... H_{k-3} y, two reflectors per reduction ----
  // H_{j-1} H_j y: a = v_j.y, b = v_{j-1}.y, c = v_{j-1}.v_j (one 4-value reduction), then
  // y -= tau_j a v_j and y -= tau_{j-1} (b - tau_j a c) v_{j-1}.
  auto hvec = [&](int j) {
    const int off = j * (k - 1) - j * (j - 1) / 2;
    return (lane > j && lane < k) ? sm.u.reg[off + lane - (j + 1)] : 0.0;
  };
  int j = k - 3;
  for (; j >= 1; j -= 2) {
    const double t1 = sm.tau[j], t0 = sm.tau[j - 1];
    // a reflector with tau = 0 was never stored (H = I): use a zero vector
    const double v1 = t1 == 0.0 ? 0.0 : hvec(j), v0 = t0 == 0.0 ? 0.0 : hvec(j - 1);
    double a1 = v1 * yl, b0 = v0 * yl, c01 = v0 * v1, pad = 0.0;
    wave_sum4_dpp(a1, b0, c01, pad);
    yl = fma(-t1 * a1, v1, yl);
    yl = fma(-t0 * fma(-t1 * a1, c01, b0), v0, yl);
  }
  if (j == 0 && sm.tau[0] != 0.0) {
    const double v0 = hvec(0);
    const double s0 = wave_sum_dpp(v0 * yl);
    yl = fma(-sm.tau[0] * s0, v0, yl);
  }
  const double sk = sqrt((double)(k - 1));
  // analysis of member `lane` (xa = wbar, :675-679); fp32 from here on, in registers
  float xal = lane < KP ? (float)(xb_mean + (d + sk * yl)) : 0.0f;

  // ---- RTPP / RTPS (:684-698), fp32 in the reference's order -------------------------
  // the reference's sequential sums run on wave-uniform values read lane by lane
  auto seq_sum = [&](float x) {
    float s = 0.0f;
    for (int mm = 0; mm < k; ++mm) s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), mm));
    return s;
  };
  if (c.use_rtpp || c.use_rtps) {
    const float xa_mean = seq_sum(xal) * c.nmember_inv;
    const double xpl = lane < k ? (double)xbl - xb_mean : 0.0;
    float xap = 0.0f;
    if (lane < k) {
      xap = xal - xa_mean;
      if (c.use_rtpp)
        xap = (float)((double)((1.0f - c.rtpp_alpha) * xap) + (double)c.rtpp_alpha * xpl);
    }
    if (c.use_rtps) {
      double d8 = 0.0;
      for (int mm = 0; mm < k; ++mm) {
        const double xp = readlane_f64(xpl, mm);
        d8 = d8 + xp * xp;
      }
      const float xb_std = (float)d8;
      const float xa_std = seq_sum(xap * xap);
      xap = xap * (c.rtps_alpha * sqrtf(xb_std / xa_std) - c.rtps_alpha + 1.0f);
    }
    xal = xa_mean + xap;
  }

  if (lane < k) {
    if constexpr (ASSEMBLED) xa_out[(long long)gi * k + lane] = xal;
    else slab.var[P + slab.L * lane] = xal;
  }
  // info.y: decade of the quadrature rule (negative when M/m exceeds the last table)
  if (lane == 0 && info) info[gi] = make_int2(ptot, ratio > dec ? -level : level);
}

// Stage + assemble only (the default KP = 40 split), one point per wavefront, into the record
// (AsmRecord): A = inflat I + Yb Yb^T packed lower (inflat on the live diagonal, 1 on the
// padding's: decoupled unit rows, as solve_tq_kernel's blocks) and b1 = Yb d.
//
// The product of the staged rows Y' = [Yb (rows 0..39); yo (row 40)] is covered with
//   three v_mfma_f64_16x16x4 tiles  (A rows x B cols; C/D lane: col = lane & 15, row =
//                                    (lane >> 4) + 4 reg)
//     T0 = {yo, 1..15} x {0..15}      yo . Yb(0..15) = b1(0..15) and A(1..15, 0..15) lower
//     T1 = {16..31}    x {0..15}      A(16..31, 0..15)
//     T2 = {yo, 17..31} x {16..31}    b1(16..31) and A(17..31, 16..31) lower
//   four v_mfma_f64_4x4x4_4b strips  rows 32..35 / 36..39 (broadcast over the 4 blocks) x
//                                    tile column J's own 16x16 operand (J = 0, 1): A(32..39,
//                                    0..31); result lane 16 i + 4 b + j = (32 + 4 r + i,
//                                    16 J + 4 b + j)
//   one 4x4x4_4b corner             four blocks (rows x cols) 32..35 x {yo,32,33,34},
//                                    36..39 x {yo,35,36,37}, 36..39 x {32,33,34,38} and
//                                    {35,39,0,16} x {35,39,0,16}: A(32..39, 32..39) lower,
//                                    b1(32..39) and the diagonals A(0,0), A(16,16) that the
//                                    yo rows of T0 and T2 displaced
// = 3 x 64 + 5 x 16 = 272 matrix-pipe cycles per 4 columns for the 860 needed entries (215
// cycles of work; 1.27x), against 336 for the 48 x 48 tiling with a yo strip (1.56x).  (r4,
// measured and dropped: a cover of one 16x16 tile and ten 4x4x4_4b, 224 cycles, 1.04x, whose
// extra operands cost more VALU issue than the matrix cycles it saves, 2-5% slower:
// profiles/r4m_record_cover_ab.txt.)  Every
// entry is one fp64 FMA chain over the columns in staging order, like the reference's
// dsyrk/dgemv (products of fp32 values are exact in fp64).
// The record kernel's fp64 side rows of a staged chunk (see assemble_record_kernel): per
// column rows 32..39, yo, row 0, row 16 (and one pad word: columns 96 B apart)
struct RecordStripRows {
  double d[kTqChunk][12];
};
struct RecordSide {
  static constexpr bool kPad = false;  // the chunk's rows past 31 (but yo) are never read
  RecordStripRows &s;
  __device__ __forceinline__ void stage(int half, int sl, const f32x4 (&g)[kTq4KP / 8], float w) {
    double *d = s.d[sl];
    if (half) {  // rows 32..39 (this lane stages rows 20..39)
      d[0] = (double)(g[3].x * w); d[1] = (double)(g[3].y * w);
      d[2] = (double)(g[3].z * w); d[3] = (double)(g[3].w * w);
      d[4] = (double)(g[4].x * w); d[5] = (double)(g[4].y * w);
      d[6] = (double)(g[4].z * w); d[7] = (double)(g[4].w * w);
    } else {  // rows 0 and 16 (rows 0..19)
      d[9] = (double)(g[0].x * w);
      d[10] = (double)(g[4].x * w);
    }
  }
  __device__ __forceinline__ void yo(int sl, float y) { s.d[sl][8] = (double)y; }
};

template <int WAVES>
__global__ void __launch_bounds__(64, WAVES)
assemble_record_kernel(const TreeDesc *__restrict__ trees, SolveConsts c, SlabDev slab,
                       long long g0, int npts, const int *__restrict__ nbr_cnt,
                       const int *__restrict__ nbr_idx, int2 *__restrict__ info,
                       double *__restrict__ ws) {
  constexpr int KP = kTq4KP, PITCH = 48, YO = KP;
  static_assert(KP == 40 && MfmaLayout<KP>::PITCH == PITCH, "the cover is laid out for KP = 40");
  using HO = AsmRecord<KP>;
  __shared__ ColumnChunk<KP, kTqChunk, float, PITCH, true> ch;  // shifted columns (SWZ)
  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int lane = threadIdx.x, kk = lane >> 4, m = lane & 15;
  float3 pt;
  slab_point(slab, g0 + gi, pt.x, pt.y, pt.z);
  // corner operands of this lane (m = 4 b + i for the A rows, 4 b + j for the B columns):
  // entry i of a 16-entry byte table held as two 64-bit literals (a shift and a mask, not 16
  // compares and selects per lookup)
  struct Tab16 {
    unsigned long long lo, hi;
    __device__ __forceinline__ int operator[](int i) const {
      return (int)(((i < 8 ? lo : hi) >> (8 * (i & 7))) & 0xffull);
    }
  };
  constexpr Tab16 kRowA = {0x2726252423222120ull, 0x1000272327262524ull};  // 32..39 36..39 35 39 0 16
  constexpr Tab16 kColB = {0x2524232822212028ull, 0x1000272326222120ull};  // yo 32..34 yo 35..37 32..34 38 35 39 0 16
  // rows of the strips and the corner in the fp64 side rows (RecordStripRows): 32..39 ->
  // 0..7, yo -> 8, row 0 -> 9, row 16 -> 10
  constexpr Tab16 kRowD = {0x0706050403020100ull, 0x0a09070307060504ull};
  constexpr Tab16 kColD = {0x0504030802010008ull, 0x0a09070306020100ull};
  const int ia = kRowD[m], ib = kColD[m];
  // A rows of the diagonal tiles: yo in place of rows 0 and 16 (read from the staged yo row,
  // not selected after the conversion: 2 reads instead of 4 v_cndmask per group)
  const int r0 = m == 0 ? YO : m, r1 = m == 0 ? YO : 16 + m;
  // The strip and corner operands (rows 32..39, yo, 0, 16: four of a lane's eight per group,
  // each shared by 4 to 16 lanes) are also staged as fp64, converted once per value by the
  // staging lane instead of once per reading lane: 4 fewer v_cvt_f64_f32 per lane and group
  // (8 groups per chunk) for 11 per chunk at staging.  Columns 96 B apart: the 32 lanes of a
  // half wave (columns 4 g + kk, kk in {0, 1} or {2, 3}) read 24 distinct dwords each.
  __shared__ RecordStripRows sr;
  f64x4 t0 = {0.0, 0.0, 0.0, 0.0}, t1 = t0, t2 = t0;
  double st[4] = {0.0, 0.0, 0.0, 0.0}, cn = 0.0;
  const int ptot = stage_columns_pair<KP, kTqChunk, PITCH>(
      ch, trees, c, gi, lane, nbr_cnt, nbr_idx, pt, [&](int nsl) {
        // column s = 4 g + kk of the chunk is k-slot kk of group g; staged columns past nsl
        // are zero.  The group loop is unrolled with a static double buffer: group g + 1's
        // operands are read before group g's MFMAs.
        float f[2][4];
        double e[2][4];
        const float *c0 = ch.col(kk);  // column 4 g + kk at c0 + g GSTRIDE
        const double *d0 = sr.d[kk];   // its side rows at d0 + 48 g
        auto load = [&](int b, int g) {
          const float *col = c0 + g * ch.GSTRIDE;
          f[b][0] = col[m];
          f[b][1] = col[16 + m];
          f[b][2] = col[r0];
          f[b][3] = col[r1];
          const double *dc = d0 + 48 * g;
          e[b][0] = dc[m & 3];
          e[b][1] = dc[4 + (m & 3)];
          e[b][2] = dc[ia];
          e[b][3] = dc[ib];
        };
        const int nl = CWBL_DBG_STOP(c) == 11 ? 0 : nsl;
        if (nl > 0) load(0, 0);
#pragma unroll
        for (int g = 0; g < kTqChunk / 4; ++g) {
          if (4 * g >= nl) break;  // nsl is wave-uniform
          const int b = g & 1;
          const double o0 = (double)f[b][0], o1 = (double)f[b][1];
          const double a0 = (double)f[b][2], a1 = (double)f[b][3];
          const double s0 = e[b][0], s1 = e[b][1];
          const double ca = e[b][2], cbv = e[b][3];
          if (g + 1 < kTqChunk / 4 && 4 * (g + 1) < nl) load(b ^ 1, g + 1);
          t0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, o0, t0, 0, 0, 0);
          t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(o1, o0, t1, 0, 0, 0);
          t2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, o1, t2, 0, 0, 0);
          st[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(s0, o0, st[0], 0, 0, 0);
          st[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(s1, o0, st[1], 0, 0, 0);
          st[2] = __builtin_amdgcn_mfma_f64_4x4x4f64(s0, o1, st[2], 0, 0, 0);
          st[3] = __builtin_amdgcn_mfma_f64_4x4x4f64(s1, o1, st[3], 0, 0, 0);
          cn = __builtin_amdgcn_mfma_f64_4x4x4f64(ca, cbv, cn, 0, 0, 0);
        }
      },
      RecordSide{sr});
  if (lane == 0) info[gi] = make_int2(ptot, 0);  // p = 0: the solve leaves var unchanged
  if (ptot == 0) return;
  if (CWBL_DBG_STOP(c) == 1) {  // timing ablation: keep the assembly live, skip the record
    const double t = t0[0] + t1[1] + t2[2] + st[0] + st[3] + cn;
    if (lane == 0) info[gi] = make_int2(ptot, (int)t);
    return;
  }
  const int k = c.k;
  const double inflat = (double)c.inflat;
  double *__restrict__ w = ws + (long long)gi * HO::WORDS;
  auto put = [&](int row, int col, double a) {  // packed lower; inflat on the live diagonal
    w[HO::TA + row * (row + 1) / 2 + col] = row != col ? a : row < k ? a + inflat : 1.0;
  };
  // The tiles' and strips' entries: A(kk + c, m + d) for a compile-time (c, d) is record word
  // TA + tri(kk + c) + m + d = TA + tri(kk) + m + c kk + tri(c) + d, i.e. one lane base, one
  // v_mad_u32_u24 (c kk) and an immediate.  On the diagonal (m == kk + c, c < 32) the value
  // is a + inflat on live rows and 1 on padding rows, whose a is +0: a + dd with dd = inflat
  // or 1, and a + 0 elsewhere (a is never -0: the sums start from +0), so no store selects.
  char *const wb = reinterpret_cast<char *>(w);
  const unsigned b8 = 8u * (unsigned)(HO::TA + ((kk * (kk + 1)) >> 1) + m);
  auto at = [&](int cc, int d) -> double & {
    return *reinterpret_cast<double *>(wb + (b8 + 8u * (unsigned)cc * (unsigned)kk) +
                                       8u * (unsigned)((cc * (cc + 1)) / 2 + d));
  };
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = kk + 4 * r;  // A-operand row index of the tiles
    if (r == 0 && kk == 0) {
      w[HO::U1 + m] = t0[r];        // yo . Yb(m)
      w[HO::U1 + 16 + m] = t2[r];   // yo . Yb(16 + m)
    } else if (m <= i) {
      const bool dg = m == i;
      at(4 * r, 0) = t0[r] + (dg ? inflat : 0.0);                           // rows 1..15 < k
      at(16 + 4 * r, 16) = t2[r] + (dg ? (16 + i < k ? inflat : 1.0) : 0.0);
    }
    at(16 + 4 * r, 0) = t1[r];
  }
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int J = 0; J < 2; ++J) at(32 + 4 * r, 16 * J) = st[2 * J + r];
  {  // corner: lane 16 i + 4 b + j = (row kRowA[4 b + i], col kColB[4 b + j])
    const int bb = (lane >> 2) & 3, i = kk, j = lane & 3;
    const int row = kRowA[4 * bb + i], col = kColB[4 * bb + j];
    if (col == YO) w[HO::U1 + row] = cn;
    else if (bb == 3 ? i == j : col <= row) put(row, col, cn);
  }
}


hipError_t launch_assemble_record(hipStream_t s, int kp, const TreeDesc *trees, SolveConsts c,
                                  SlabDev slab, long long g0, int npts, const int *nbr_cnt,
                                  const int *nbr_idx, int2 *info, double *ws) {
  if (npts <= 0) return hipSuccess;
  if (kp != kTq4KP) return hipErrorInvalidValue;
  hipLaunchKernelGGL((assemble_record_kernel<kRecordWaves>), dim3(npts), dim3(64), 0, s, trees,
                     c, slab, g0, npts, nbr_cnt, nbr_idx, info, ws);
  return hipGetLastError();
}

template <int KP>
static hipError_t launch_tq_kp(hipStream_t s, bool assembled, const TreeDesc *trees,
                               SolveConsts c, SlabDev slab, long long g0, int npts,
                               const int *nbr_cnt, const int *nbr_idx,
                               const long long *col_off, const float *yo, const float *yb,
                               const float *xb, float *xa, int2 *info, double *tri) {
  if (assembled)
    hipLaunchKernelGGL((solve_tq_kernel<KP, true>), dim3(npts), dim3(64), 0, s, trees, c, slab,
                       g0, npts, nbr_cnt, nbr_idx, col_off, yo, yb, xb, xa, info, tri);
  else
    hipLaunchKernelGGL((solve_tq_kernel<KP, false>), dim3(npts), dim3(64), 0, s, trees, c,
                       slab, g0, npts, nbr_cnt, nbr_idx, col_off, yo, yb, xb, xa, info);
  return hipGetLastError();
}

hipError_t launch_solve_tq(hipStream_t s, int kp, bool assembled, const TreeDesc *trees,
                           SolveConsts c, SlabDev slab, long long g0, int npts,
                           const int *nbr_cnt, const int *nbr_idx,
                           const long long *col_off, const float *yo, const float *yb,
                           const float *xb, float *xa, int2 *info, double *tri) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr || (tri && !assembled)) return hipErrorInvalidValue;
#define CWBL_TQ_CASE(K)                                                                      \
  case K:                                                                                    \
    return launch_tq_kp<K>(s, assembled, trees, c, slab, g0, npts, nbr_cnt, nbr_idx,         \
                           col_off, yo, yb, xb, xa, info, tri);
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
