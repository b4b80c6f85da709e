// cwbl_tq4.hip — solve_tq4_kernel<KP, J0>: the second half of the per-point LETKF solve
// (letkf_solve, module_letkf_core.f90:598-700) for four grid points per wavefront.
//
// solve_tq_kernel<KP, false, J0> (cwbl_tq.hip) stages the point's columns, assembles
// A = (k-1)/infl I + Yb Yb^T and b1 = Yb d on the matrix cores and runs the first J0 steps
// of the Householder tridiagonalisation A = Q T Q^T (dsytd2 order) on its 4x4 register
// blocks, one point per wavefront; it hands the trailing (KP-J0)^2 matrix, the J0
// reflectors, T so far and Q^T b1, Q^T x' over through the workspace (Tq4Handoff).  This
// kernel finishes the algorithm of solve_tq_kernel — the remaining steps, the T^-1/2
// quadrature and the T^-1 solve, the back-transform and the RTPP/RTPS epilogue in the
// reference's fp32 order — with a different mapping:
//
//   one 16-lane DPP row per point (q = lane / 16); lane l holds the FULL trailing rows
//   J0 + l and J0 + 16 + l (slots 0, 1) in registers, and the vectors' rows l < J0
//   (the prefix slot) for the back-transform and the epilogue.
//
// With one point per wavefront a step costs ~200 instructions of mostly fixed work (wave
// reductions, broadcasts, LDS round trips) per point.  Here every instruction serves four
// points, reductions span 16 lanes (4 DPP stages), broadcasts of v_c / w_c are one
// v_mov_b64 row_newbcast each, the pivot column is a static register of every row (no
// publish) and each reflector stays in the registers of the column it eliminated.  All
// loops over steps, slots and columns are compile-time (sfor), so register indices are
// static; with 32 trailing rows the matrix takes 128 VGPRs and two waves fit a SIMD.
#include "cwbl_device.h"

#include <utility>

namespace cwbl {

namespace {

template <int... Is, class F>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, Is...>, F &&f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>), in order
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
  sfor_impl(std::make_integer_sequence<int, N>{}, f);
}

// value of lane L of this lane's 16-lane row (DPP row_newbcast; one v_mov_b64 for fp64).
// bound_ctrl: every source lane is active, and without it the compiler first copies the
// unused "old" operand into the destination (one more v_mov_b64 per broadcast).
template <int L>
__device__ __forceinline__ double rbcast(double x) {
  return __longlong_as_double(
      __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(x), 0x150 + L, 0xf, 0xf, true));
}
template <int L>
__device__ __forceinline__ float rbcast(float x) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 + L, 0xf, 0xf, true));
}
// value of lane l ^ 8 of the row (row_ror:8)
__device__ __forceinline__ double ror8(double x) { return dpp_f64<0x128>(x); }

}  // namespace

template <int KP, int J0>
struct Tq4Smem {
  static constexpr int KT = KP - J0;
  static constexpr int NT = KT * (KT + 1) / 2;
  static constexpr int QLD = 9;  // 8 nodes per quadrature round (+1 against bank conflicts)
  union {
    double qx[4][KP][QLD];        // per round: omega_n x_n(row) of the 8 nodes
  } u;
  double tq[4][KP + 1][4];        // d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
  double tau[4][KP];
};

template <int KP, int J0>
__global__ void __launch_bounds__(64, 2)
solve_tq4_kernel(SolveConsts c, SlabDev slab, long long g0, int npts,
                 const double *__restrict__ ws, int2 *__restrict__ info) {
  using HO = Tq4Handoff<KP, J0>;
  constexpr int KT = HO::KT;          // trailing rows
  constexpr int NS = (KT + 15) / 16;  // trailing row slots per lane
  constexpr int NV = NS + 1;          // vector slots: 0 = rows l < J0, 1.. = trailing slots
  constexpr int H = KP / 2;           // rows walked by each side of a twisted solve
  static_assert(KT % 16 == 0 && J0 <= 16 && KP % 2 == 0, "tq4 layout");
  using SM = Tq4Smem<KP, J0>;
  __shared__ SM sm;

  const int lane = threadIdx.x, q = lane >> 4, l = lane & 15;
  const int gi = 4 * blockIdx.x + q;
  const bool valid = gi < npts;
  const int k = c.k;
  const int ptot = valid ? info[gi].x : 0;
  // hand-off words of this point: ws[wb + i] through an SGPR base and a 32-bit VGPR
  // offset (the host keeps a hand-off batch below 2^32 bytes)
  const unsigned wb = (unsigned)(valid ? gi : 0) * (unsigned)HO::WORDS;
  auto w = [&](int i) { return gld(ws, wb + (unsigned)i); };
  // global row of vector slot vs (rows that do not exist get KP + 1: never < k)
  auto vrow = [&](int vs) { return vs == 0 ? (l < J0 ? l : KP + 1) : J0 + l + 16 * (vs - 1); };

  // var index of member 0 (g = i + ix_lim (j + iy_lim kz); g < 2^32: var would exceed HBM first)
  long long P = 0;
  {
    const unsigned g = (unsigned)(g0 + (valid ? gi : 0));
    const unsigned ix = (unsigned)slab.ix_lim, iy = (unsigned)slab.iy_lim;
    const unsigned rr = g / ix, ii = g - rr * ix, kz = rr / iy, jj = rr - kz * iy;
    P = ii + (long long)slab.nx * (jj + (long long)slab.ny * kz);
  }

  // ---- trailing matrix: full rows from the packed hand-off (L2/MALL-resident) -----------
  double A[NS][KT];
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int t = l + 16 * r;
    sfor<KT>([&](auto cc) {
      constexpr int col = decltype(cc)::value;
      A[r][col] = w(col <= t ? t * (t + 1) / 2 + col : col * (col + 1) / 2 + t);
    });
  });

  double ux[NS], ub[NS];  // trailing rows of Q^T x' and Q^T b1
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int t = J0 + l + 16 * r;
    ux[r] = w(HO::U2 + t);
    ub[r] = w(HO::U1 + t);
  });
  // T rows < J0 (and c(J0-1, J0)) and the first reflectors' tau, from the hand-off
  {
    const int lj = l < J0 ? l : J0 - 1;  // lanes >= J0 repeat row J0-1 (same values)
    sm.tq[q][lj][0] = w(HO::D + lj);
    sm.tq[q][lj + 1][1] = w(HO::E + lj);
    sm.tq[q][lj][2] = w(HO::U1 + lj);
    sm.tq[q][lj][3] = w(HO::U2 + lj);
    sm.tau[q][lj] = w(HO::TAU + lj);
  }
  double trace = 0.0;  // sum of d_j, j < k
  sfor<J0>([&](auto jj) {
    constexpr int j = decltype(jj)::value;
    trace += j < k ? w(HO::D + j) : 0.0;
  });

  // ---- Householder steps J0 .. KP-3 on the trailing matrix (local column jl) --------------
  // Steps j >= k - 2 (k < KP) are exact no-ops: the padding rows and columns of A are the
  // identity, so x = 0 there, tau = 0 and beta = A(j+1,j); running them keeps the code
  // branch-free.
  sfor<KT>([&](auto jj) {
    constexpr int jl = decltype(jj)::value, j = J0 + jl;
    constexpr int RJ = jl / 16, LJ = jl % 16;
    const double dj = rbcast<LJ>(A[RJ][jl]);  // A(j,j): final diagonal of T
    trace += j < k ? dj : 0.0;
    if constexpr (jl + 2 < KT) {
      constexpr int J1 = jl + 1, R1 = J1 / 16, L1 = J1 % 16;
      const double alpha = rbcast<L1>(A[R1][jl]);
      double x[NS], xx = 0.0, xu = 0.0, xb = 0.0;
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        if constexpr (16 * r + 15 > J1) {
          const int i = J0 + l + 16 * r;
          x[r] = (i > j + 1 && i < k) ? A[r][jl] : 0.0;
          xx = fma(x[r], x[r], xx);
          xu = fma(x[r], ux[r], xu);
          xb = fma(x[r], ub[r], xb);
        } else {
          x[r] = 0.0;
        }
      });
      xx = row16_sum(xx);
      xu = row16_sum(xu);
      xb = row16_sum(xb);
      // dlarfg with fp64 rcp/rsq refined to ~1 ulp; H = I when x = 0 (tau = 0, v = e_j+1)
      const double a2 = fma(alpha, alpha, xx);
      const double rs = rsq64(a2);  // 1/|beta|
      const bool nz = xx > 0.0;
      const double bt = -copysign(a2 * rs, alpha);
      const double beta = nz ? bt : alpha;
      const double tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
      const double rab = rcp64(alpha - bt);
      const double scal = nz ? rab : 0.0;
      // every lane of the row writes the same value (no divergent branch in the step)
      sm.tq[q][j][0] = dj;
      sm.tq[q][j + 1][1] = beta;
      sm.tau[q][j] = tau;
      double v[NS];
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        const int t = l + 16 * r;
        const double xs = x[r] * scal;
        v[r] = t == J1 ? 1.0 : xs;
        if constexpr (16 * r + 15 > J1) A[r][jl] = xs;  // the reflector, rows > j + 1
      });
      const double s2 = fma(scal, xu, rbcast<L1>(ux[R1]));  // v . x'
      const double s3 = fma(scal, xb, rbcast<L1>(ub[R1]));  // v . b1
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        ux[r] = fma(-tau * s2, v[r], ux[r]);
        ub[r] = fma(-tau * s3, v[r], ub[r]);
      });
      // A v over the trailing columns (v vanishes at columns <= jl), column by column so
      // that one broadcast v_c is live at a time
      double p0[NS], p1[NS];
      sfor<NS>([&](auto rr) { p0[decltype(rr)::value] = p1[decltype(rr)::value] = 0.0; });
      sfor<KT - J1>([&](auto cc) {
        constexpr int col = J1 + decltype(cc)::value;
        const double vcol = rbcast<col % 16>(v[col / 16]);
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          if constexpr (16 * r + 15 > jl) {
            if constexpr ((col - J1) % 2 == 0) p0[r] = fma(A[r][col], vcol, p0[r]);
            else p1[r] = fma(A[r][col], vcol, p1[r]);
          }
        });
      });
      double pp[NS], sp = 0.0;
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        pp[r] = p0[r] + p1[r];
        if constexpr (16 * r + 15 > jl) sp = fma(v[r], pp[r], sp);  // rows <= j: v = 0
      });
      const double s1 = tau * row16_sum(sp);  // v^T (tau A v)
      double wv[NS];
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        const int t = l + 16 * r;
        wv[r] = t > jl ? fma(-0.5 * tau * s1, v[r], tau * pp[r]) : 0.0;
      });
      // A <- A - v w^T - w v^T on the trailing rows and columns
      sfor<KT - J1>([&](auto cc) {
        constexpr int col = J1 + decltype(cc)::value;
        const double vcol = rbcast<col % 16>(v[col / 16]);
        const double wcol = rbcast<col % 16>(wv[col / 16]);
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          if constexpr (16 * r + 15 > jl)
            A[r][col] = fma(-v[r], wcol, fma(-wv[r], vcol, A[r][col]));
        });
      });
    } else {  // the trailing 2x2: already tridiagonal (c(KP-2,KP-3) is step KP-3's beta)
      const double ej = rbcast<LJ>(A[RJ][jl - 1]);
      sm.tq[q][j][0] = dj;
      if constexpr (jl == KT - 1) sm.tq[q][j][1] = ej;
    }
  });
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int i = J0 + l + 16 * r;
    sm.tq[q][i][2] = ub[r];
    sm.tq[q][i][3] = ux[r];
  });
  if (l == 0) {
    sm.tq[q][0][1] = 0.0;
    sm.tq[q][KP][1] = 0.0;
  }
  __syncthreads();

  // ---- T^-1/2 u2 by quadrature, T^-1 u2 exactly --------------------------------------------
  // lambda^-1/2 = (2/pi) int_0^inf dt / (t^2 + lambda) with the elliptic substitution and
  // the midpoint rule on the spectrum bound [m, M] (solve_tq_kernel, cwbl_tq.hip): each node
  // is one shifted SPD tridiagonal solve, twisted: lane l & 7 is the node of the round,
  // side l >> 3 walks rows 0..H-1 (top) or KP-1..H (bottom); node 31 solves T^-1 u2.
  const double m = (double)c.inflat;
  const double ratio = trace / m - (double)(k - 1);
  int level = 1;
  double dec = 10.0;
  while (level < kQuadLevels && dec < ratio) {
    dec *= 10.0;
    ++level;
  }
  const int side = l >> 3, n8 = l & 7;
  const double(*T)[4] = sm.tq[q];
  const double *tq0 = &T[side ? KP - 1 : 0][0];
  const int dir = side ? -4 : 4;
  const int cs = side ? 5 : 1;  // coupling with the previous row of the walk
  double ys[NV], z[NV];
  sfor<NV>([&](auto vv) { ys[decltype(vv)::value] = 0.0; });
  for (int round = 0; round < 4; ++round) {
    const int node = 8 * round + n8;
    const double2 tw = c.quad[(level - 1) * 32 + min(node, kQuadNodes - 1)];
    const double sigma = node < kQuadNodes ? m * tw.x : 0.0;
    const double omega = node < kQuadNodes ? sqrt(m) * tw.y : 1.0;
    double hh[H], mm[H];
    double dl = tq0[0] + sigma, gt = tq0[3];
    double rdl = rcp64(dl);
    sfor<H - 1>([&](auto tt) {
      constexpr int t = decltype(tt)::value + 1;
      const double *qt = tq0 + dir * t;
      const double ct = qt[cs];
      const double lt = ct * rdl;
      hh[t - 1] = gt * rdl;
      mm[t - 1] = lt;
      dl = fma(-lt, ct, qt[0] + sigma);
      gt = fma(-lt, gt, qt[3]);
      rdl = rcp64(dl);
    });
    // rows H-1 (top) and H (bottom): 2x2 solve with the partner lane's pivot
    const double cm = T[H][1];
    const double dlo = ror8(dl), go = ror8(gt);
    double xv = (gt * dlo - cm * go) / fma(dl, dlo, -cm * cm);
    auto row_of = [&](int t) { return side ? KP - 1 - t : t; };
    sm.u.qx[q][row_of(H - 1)][n8] = omega * xv;
    sfor<H - 1>([&](auto tt) {
      constexpr int t = H - 2 - decltype(tt)::value;
      xv = fma(-mm[t], xv, hh[t]);
      sm.u.qx[q][row_of(t)][n8] = omega * xv;
    });
    __syncthreads();
    const bool last = round == 3;  // node 31 (slot 7 of the last round) is T^-1 u2
    sfor<NV>([&](auto vv) {
      constexpr int vs = decltype(vv)::value;
      const int i = vrow(vs);
      const double *row = sm.u.qx[q][i < KP ? i : 0];
      double s = 0.0;
      sfor<7>([&](auto nn) { s += row[decltype(nn)::value]; });
      const double r7 = row[7];
      s = last ? s : s + r7;
      ys[vs] += i < KP ? s : 0.0;
      if (last) z[vs] = i < KP ? r7 : 0.0;
    });
    __syncthreads();
  }
  double dpart = 0.0;  // u1 . T^-1 u2 = wbar . x'
  sfor<NV>([&](auto vv) {
    constexpr int vs = decltype(vv)::value;
    const int i = vrow(vs);
    double u1 = 0.0;
    if constexpr (vs == 0) {
      const double t = w(HO::U1 + (l < J0 ? l : 0));
      u1 = l < J0 ? t : 0.0;
    }
    else u1 = ub[vs - 1];
    dpart = i < KP ? fma(u1, z[vs], dpart) : dpart;
  });
  const double d = row16_sum(dpart);

  // ---- back-transform: y <- Q y = H_0 H_1 ... H_{KP-3} y ----------------------------------
  double y[NV];
  sfor<NV>([&](auto vv) { y[decltype(vv)::value] = ys[decltype(vv)::value]; });
  sfor<KT - 2>([&](auto jj) {  // this kernel's reflectors, registers of the column they cut
    constexpr int jl = KT - 3 - decltype(jj)::value, j = J0 + jl, J1 = jl + 1;
    const double tj = sm.tau[q][j];
    double vv[NS], a = 0.0;
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      if constexpr (16 * r + 15 >= J1) {
        const int t = l + 16 * r;
        vv[r] = t == J1 ? 1.0 : (t > J1 ? A[r][jl] : 0.0);
        a = fma(vv[r], y[r + 1], a);
      } else {
        vv[r] = 0.0;
      }
    });
    a = row16_sum(a);
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      if constexpr (16 * r + 15 >= J1) y[r + 1] = fma(-tj * a, vv[r], y[r + 1]);
    });
  });
  sfor<J0>([&](auto jj) {  // the hand-off's reflectors (rows j+1 .. KP-1, 0 elsewhere)
    constexpr int j = J0 - 1 - decltype(jj)::value;
    const double tj = sm.tau[q][j];
    double vv[NV], a = 0.0;
    sfor<NV>([&](auto vs_c) {
      constexpr int vs = decltype(vs_c)::value;
      const int i = vrow(vs);
      const double h = w(HO::HV + j * KP + (i < KP ? i : 0));  // branch-free load
      vv[vs] = i < KP ? h : 0.0;
      a = fma(vv[vs], y[vs], a);
    });
    a = row16_sum(a);
    sfor<NV>([&](auto vs_c) {
      constexpr int vs = decltype(vs_c)::value;
      y[vs] = fma(-tj * a, vv[vs], y[vs]);
    });
  });

  // ---- background of the point: member i = row i (loaded here, where it is used: loaded
  // early, the compiler keeps its 40 broadcasts live across the whole kernel) ------------
  float xbl[NV];
  sfor<NV>([&](auto vv) {
    constexpr int vs = decltype(vv)::value;
    const int i = vrow(vs);
    const bool mem = valid && i < k;
    const float xv = slab.var[P + slab.L * (mem ? i : 0)];  // branch-free: a valid address
    xbl[vs] = mem ? xv : 0.0f;
  });
  // fp32 sum over members in member order; member m is row m: prefix slot lane m (m < J0),
  // else trailing slot (m - J0) / 16, lane (m - J0) % 16
  auto seq_sum_f32 = [&](const float (&x)[NV]) {
    float s = 0.0f;
    sfor<KP>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      constexpr int vs = m < J0 ? 0 : 1 + (m - J0) / 16, ln = m < J0 ? m : (m - J0) % 16;
      const float b = rbcast<ln>(x[vs]);
      s = s + (m < k ? b : 0.0f);  // s + 0 = s: s is never -0
    });
    return s;
  };
  // sum(xb) * nmember_inv (:671)
  const double xb_mean = (double)(seq_sum_f32(xbl) * c.nmember_inv);
  // ---- analysis and RTPP / RTPS (:675-698), fp32 in the reference's order ----------------
  const double sk = sqrt((double)(k - 1));
  float xa[NV];
  sfor<NV>([&](auto vv) {
    constexpr int vs = decltype(vv)::value;
    xa[vs] = vrow(vs) < k ? (float)(xb_mean + (d + sk * y[vs])) : 0.0f;
  });
  if (c.use_rtpp || c.use_rtps) {
    const float xa_mean = seq_sum_f32(xa) * c.nmember_inv;
    double xpl[NV];
    float xap[NV];
    sfor<NV>([&](auto vv) {
      constexpr int vs = decltype(vv)::value;
      const bool mem = vrow(vs) < k;
      xpl[vs] = mem ? (double)xbl[vs] - xb_mean : 0.0;
      xap[vs] = 0.0f;
      if (mem) {
        xap[vs] = xa[vs] - xa_mean;
        if (c.use_rtpp)
          xap[vs] = (float)((double)((1.0f - c.rtpp_alpha) * xap[vs]) +
                            (double)c.rtpp_alpha * xpl[vs]);
      }
    });
    if (c.use_rtps) {
      double d8 = 0.0;
      sfor<KP>([&](auto mm) {
        constexpr int mb = decltype(mm)::value;
        constexpr int vs = mb < J0 ? 0 : 1 + (mb - J0) / 16, ln = mb < J0 ? mb : (mb - J0) % 16;
        const double xp = rbcast<ln>(xpl[vs]);  // 0 past member k-1
        d8 = d8 + xp * xp;
      });
      const float xb_std = (float)d8;
      float sq[NV];
      sfor<NV>([&](auto vv) {
        constexpr int vs = decltype(vv)::value;
        sq[vs] = xap[vs] * xap[vs];
      });
      const float xa_std = seq_sum_f32(sq);
      const float f = c.rtps_alpha * sqrtf(xb_std / xa_std) - c.rtps_alpha + 1.0f;
      sfor<NV>([&](auto vv) { xap[decltype(vv)::value] = xap[decltype(vv)::value] * f; });
    }
    sfor<NV>([&](auto vv) { xa[decltype(vv)::value] = xa_mean + xap[decltype(vv)::value]; });
  }
  if (valid && ptot > 0) {
    sfor<NV>([&](auto vv) {
      constexpr int vs = decltype(vv)::value;
      const int i = vrow(vs);
      if (i < k) slab.var[P + slab.L * i] = xa[vs];
    });
    // info.y: decade of the quadrature rule (negative when M/m exceeds the last table)
    if (l == 0) info[gi] = make_int2(ptot, ratio > dec ? -level : level);
  }
}

hipError_t launch_solve_tq4(hipStream_t s, int kp, SolveConsts c, SlabDev slab, long long g0,
                            int npts, const double *ws, int2 *info) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr || kp != kTq4KP) return hipErrorInvalidValue;
  hipLaunchKernelGGL((solve_tq4_kernel<kTq4KP, kTq4J0>), dim3((npts + 3) / 4), dim3(64), 0, s,
                     c, slab, g0, npts, ws, info);
  return hipGetLastError();
}

}  // namespace cwbl
