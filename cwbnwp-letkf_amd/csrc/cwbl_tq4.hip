// cwbl_tq4.hip — solve_tq4_kernel<KP>: the dense half of the per-point LETKF solve
// (letkf_solve, module_letkf_core.f90:598-700) for four grid points per wavefront.
//
// solve_tq_kernel<KP, false, true> (cwbl_tq.hip) stages the point's columns and assembles
// A = (k-1)/infl I + Yb Yb^T and b1 = Yb d on the matrix cores, then hands them over
// through the workspace (packed lower rows, fp64).  This kernel does the rest of the
// algorithm of solve_tq_kernel — Householder tridiagonalisation A = Q T Q^T (dsytd2 order)
// applied on the fly to b1 and x', the T^-1/2 quadrature and T^-1 solve, the back-transform
// and the RTPP/RTPS epilogue in the reference's fp32 order — with a different mapping:
//
//   one 16-lane DPP row per point (q = lane / 16), lane l holding the FULL rows
//   i = l, l + 16, l + 32 of A (slot r = i / 16) in registers.
//
// With one point per wavefront the tridiagonalisation costs ~40 steps x ~200 instructions
// of mostly fixed per-step work (wave reductions, broadcasts, LDS round trips) for 4/3 k^3
// useful flops.  Here every instruction serves four points, reductions span 16 lanes
// (4 DPP stages), broadcasts of v_c / w_c are one v_mov_b64 row_newbcast each, the pivot
// column is a static register of every row (no publish), and the Householder vectors are
// kept in the registers of the columns they eliminated.  All loops over steps, slots and
// columns are compile-time (sfor), so every register index is static.
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

// value of lane L of this lane's 16-lane row (DPP row_newbcast; one v_mov_b64 for fp64)
template <int L>
__device__ __forceinline__ double rbcast(double x) {
  return __longlong_as_double(
      __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(x), 0x150 + L, 0xf, 0xf, false));
}
template <int L>
__device__ __forceinline__ float rbcast(float x) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 + L, 0xf, 0xf, false));
}

// A double parked in two AGPRs: the Householder vectors wait there from their step to the
// back-transform, outside the arch VGPRs the trailing matrix needs.
struct AccF64 {
  int lo, hi;
};
__device__ __forceinline__ void acc_put(AccF64 &a, double x) {
  const long long b = __double_as_longlong(x);
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(a.lo) : "v"((int)b));
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(a.hi) : "v"((int)(b >> 32)));
}
__device__ __forceinline__ double acc_get(const AccF64 &a) {
  int lo, hi;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(lo) : "a"(a.lo));
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(hi) : "a"(a.hi));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

}  // namespace

template <int KP>
struct Tq4Smem {
  static constexpr int NA = KP * (KP + 1) / 2;  // packed lower triangle
  static constexpr int QLD = 17;                // node pitch of a quadrature row
  union {
    double a[4][NA];            // the four points' A on their way into registers
    double qx[4][KP][QLD];      // per round: omega_n x_n(row) of the 16 node lanes
  } u;
  double tq[4][KP + 1][4];      // d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
  double tau[4][KP];
};

template <int KP>
__global__ void __launch_bounds__(64, 1)
solve_tq4_kernel(SolveConsts c, SlabDev slab, long long g0, int npts,
                 const double *__restrict__ ws_a, const double *__restrict__ ws_b1,
                 int2 *__restrict__ info) {
  constexpr int NS = (KP + 15) / 16;  // row slots per lane
  using SM = Tq4Smem<KP>;
  constexpr int NA = SM::NA;
  __shared__ SM sm;

  const int lane = threadIdx.x, q = lane >> 4, l = lane & 15;
  const int wb = blockIdx.x;
  const int gi = 4 * wb + q;
  const bool valid = gi < npts;
  const int k = c.k;
  const int ptot = valid ? info[gi].x : 0;

  // ---- A of the four points: workspace -> LDS -> full rows in registers ---------------------
  {
    const int npt = min(4, npts - 4 * wb);
    const double2 *src = reinterpret_cast<const double2 *>(ws_a + (long long)4 * wb * NA);
    double2 *dst = reinterpret_cast<double2 *>(&sm.u.a[0][0]);
    const int n2 = npt * NA / 2;  // NA * npt is even for every KP used (KP % 8 == 0)
    for (int t = lane; t < n2; t += 64) dst[t] = src[t];
  }
  __syncthreads();
  double A[NS][KP];
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int i = l + 16 * r;
    sfor<KP>([&](auto cc) {
      constexpr int col = decltype(cc)::value;
      const int ic = i < KP ? i : 0;  // slot lanes past the last row read row 0, then zero it
      const double v = sm.u.a[q][col <= ic ? ic * (ic + 1) / 2 + col : col * (col + 1) / 2 + ic];
      A[r][col] = i < KP ? v : 0.0;
    });
  });
  __syncthreads();

  // ---- background of the point: member i = row i ------------------------------------------
  long long P = 0;
  if (valid) {
    const long long g = g0 + gi;
    const int ii = (int)(g % slab.ix_lim);
    const long long rr = g / slab.ix_lim;
    const int jj = (int)(rr % slab.iy_lim);
    const int kz = (int)(rr / slab.iy_lim);
    P = ii + (long long)slab.nx * (jj + (long long)slab.ny * kz);
  }
  float xbl[NS];
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int i = l + 16 * r;
    xbl[r] = (valid && i < k) ? slab.var[P + slab.L * i] : 0.0f;
  });
  // sum(xb) * nmember_inv in fp32, sequential in member order (:671)
  auto seq_sum_f32 = [&](const float (&x)[NS]) {
    float s = 0.0f;
    sfor<KP>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      const float b = rbcast<m % 16>(x[m / 16]);
      s = s + (m < k ? b : 0.0f);  // s + 0 = s: s is never -0
    });
    return s;
  };
  const double xb_mean = (double)(seq_sum_f32(xbl) * c.nmember_inv);
  double ux[NS], ub[NS];  // x' and b1, become Q^T x' and Q^T b1
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int i = l + 16 * r;
    ux[r] = i < k ? (double)xbl[r] - xb_mean : 0.0;
    ub[r] = (valid && i < KP) ? ws_b1[(long long)gi * KP + i] : 0.0;
  });

  // ---- Householder tridiagonalisation (lower, dsytd2 order) ------------------------------
  double trace = 0.0;
  AccF64 hv[NS][KP - 2];  // reflector j, rows > j + 1 of slot r (its unit entry is implicit)
  sfor<KP>([&](auto jj) {
    constexpr int j = decltype(jj)::value;
    constexpr int RJ = j / 16, LJ = j % 16;
    const double dj = rbcast<LJ>(A[RJ][j]);  // A(j,j): final diagonal of T
    trace += j < k ? dj : 0.0;
    // Steps j >= k - 2 (k < KP) are exact no-ops: the padding rows and columns of A are the
    // identity, so x = 0 there, tau = 0 and beta = A(j+1,j); running them keeps the code
    // branch-free.
    if constexpr (j + 2 < KP) {
      {
        constexpr int J1 = j + 1, R1 = J1 / 16, L1 = J1 % 16;
        const double alpha = rbcast<L1>(A[R1][j]);
        double x[NS], xx = 0.0, xu = 0.0, xb = 0.0;
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          if constexpr (16 * r + 15 > J1) {
            const int i = l + 16 * r;
            x[r] = (i > J1 && i < k) ? A[r][j] : 0.0;
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
        // dlarfg with fp64 rcp/rsq refined to ~1 ulp; H = I when x = 0 (tau = 0, v = e_J1)
        const double a2 = fma(alpha, alpha, xx);
        const double rs = rsq64(a2);  // 1/|beta|
        const bool nz = xx > 0.0;
        const double bt = -copysign(a2 * rs, alpha);
        const double beta = nz ? bt : alpha;
        const double tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
        const double scal = nz ? rcp64(alpha - bt) : 0.0;
        if (l == 0) {
          sm.tq[q][j][0] = dj;
          sm.tq[q][J1][1] = beta;
          sm.tau[q][j] = tau;
        }
        double v[NS];
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          const int i = l + 16 * r;
          const double xs = x[r] * scal;
          v[r] = i == J1 ? 1.0 : xs;
          if constexpr (16 * r + 15 > J1) acc_put(hv[r][j], xs);  // reflector, rows > J1
        });
        const double s2 = fma(scal, xu, rbcast<L1>(ux[R1]));  // v . x'
        const double s3 = fma(scal, xb, rbcast<L1>(ub[R1]));  // v . b1
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          ux[r] = fma(-tau * s2, v[r], ux[r]);
          ub[r] = fma(-tau * s3, v[r], ub[r]);
        });
        // A v over the trailing columns (v vanishes at columns <= j), column by column so
        // that only one broadcast v_c is live
        double p0[NS], p1[NS];
        sfor<NS>([&](auto rr) { p0[decltype(rr)::value] = p1[decltype(rr)::value] = 0.0; });
        sfor<KP - J1>([&](auto cc) {
          constexpr int col = J1 + decltype(cc)::value;
          const double vcol = rbcast<col % 16>(v[col / 16]);
          sfor<NS>([&](auto rr) {
            constexpr int r = decltype(rr)::value;
            if constexpr (16 * r + 15 > j) {
              if constexpr ((col - J1) % 2 == 0) p0[r] = fma(A[r][col], vcol, p0[r]);
              else p1[r] = fma(A[r][col], vcol, p1[r]);
            }
          });
        });
        double pp[NS], sp = 0.0;
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          pp[r] = p0[r] + p1[r];
          if constexpr (16 * r + 15 > j) sp = fma(v[r], pp[r], sp);  // rows <= j: v = 0
        });
        const double s1 = tau * row16_sum(sp);  // v^T (tau A v)
        double w[NS];
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          const int i = l + 16 * r;
          w[r] = i > j ? fma(-0.5 * tau * s1, v[r], tau * pp[r]) : 0.0;
        });
        // A <- A - v w^T - w v^T on the trailing rows and columns
        sfor<KP - J1>([&](auto cc) {
          constexpr int col = J1 + decltype(cc)::value;
          const double vcol = rbcast<col % 16>(v[col / 16]);
          const double wcol = rbcast<col % 16>(w[col / 16]);
          sfor<NS>([&](auto rr) {
            constexpr int r = decltype(rr)::value;
            if constexpr (16 * r + 15 > j)
              A[r][col] = fma(-v[r], wcol, fma(-w[r], vcol, A[r][col]));
          });
        });
      }
    } else {  // the trailing 2x2: already tridiagonal (c(KP-2,KP-3) is step KP-3's beta)
      const double ej = rbcast<LJ>(A[RJ][j - 1]);
      if (l == 0) {
        sm.tq[q][j][0] = dj;
        if constexpr (j == KP - 1) sm.tq[q][j][1] = ej;
      }
    }
  });
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int i = l + 16 * r;
    if (i < KP) {
      sm.tq[q][i][2] = ub[r];
      sm.tq[q][i][3] = ux[r];
    }
  });
  if (l == 0) {
    sm.tq[q][0][1] = 0.0;
    sm.tq[q][KP][1] = 0.0;
  }
  __syncthreads();

  // ---- T^-1/2 u2 by quadrature, T^-1 u2 exactly (cwbl_tq.hip) ---------------------------
  const double m = (double)c.inflat;
  const double ratio = trace / m - (double)(k - 1);
  int level = 1;
  double dec = 10.0;
  while (level < kQuadLevels && dec < ratio) {
    dec *= 10.0;
    ++level;
  }
  double ys[NS], z[NS];
  sfor<NS>([&](auto rr) { ys[decltype(rr)::value] = 0.0; });
  sfor<2>([&](auto rho_c) {
    constexpr int rho = decltype(rho_c)::value;
    const int node = 16 * rho + l;  // node 31: the exact solve (sigma = 0)
    const double2 tw = c.quad[(level - 1) * 32 + min(node, kQuadNodes - 1)];
    const double sigma = node < kQuadNodes ? m * tw.x : 0.0;
    const double omega = node < kQuadNodes ? sqrt(m) * tw.y : 1.0;
    // (T + sigma I) x = u2, forward elimination then back substitution (x_t = h_t - m_t x_t+1)
    const double(*T)[4] = sm.tq[q];
    double hh[KP], mm[KP];
    double dl = T[0][0] + sigma, gt = T[0][3];
    double rdl = rcp64(dl);
    sfor<KP - 1>([&](auto tt) {
      constexpr int t = decltype(tt)::value + 1;
      const double ct = T[t][1];
      const double lt = ct * rdl;
      hh[t - 1] = gt * rdl;
      mm[t - 1] = lt;
      dl = fma(-lt, ct, T[t][0] + sigma);
      gt = fma(-lt, gt, T[t][3]);
      rdl = rcp64(dl);
    });
    double xv = gt * rdl;
    sm.u.qx[q][KP - 1][l] = omega * xv;
    sfor<KP - 1>([&](auto tt) {
      constexpr int t = KP - 2 - decltype(tt)::value;
      xv = fma(-mm[t], xv, hh[t]);
      sm.u.qx[q][t][l] = omega * xv;
    });
    __syncthreads();
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      const int i = l + 16 * r;
      const double *row = sm.u.qx[q][i < KP ? i : 0];
      double s = 0.0;
      sfor<rho ? 15 : 16>([&](auto nn) { s += row[decltype(nn)::value]; });
      ys[r] += i < KP ? s : 0.0;
      if constexpr (rho == 1) z[r] = i < KP ? row[15] : 0.0;
    });
    __syncthreads();
  });
  double dpart = 0.0;
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    dpart = fma(ub[r], z[r], dpart);
  });
  const double d = row16_sum(dpart);  // u1 . T^-1 u2 = wbar . x'

  // ---- back-transform: y <- Q y = H_0 H_1 ... H_{k-3} y -----------------------------------
  double y[NS];
  sfor<NS>([&](auto rr) { y[decltype(rr)::value] = ys[decltype(rr)::value]; });
  sfor<KP - 2>([&](auto jj) {
    constexpr int j = KP - 3 - decltype(jj)::value;
    {  // j > k - 3: tau = 0, a no-op
      constexpr int J1 = j + 1;
      const double tj = sm.tau[q][j];
      double vv[NS], a = 0.0;
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        if constexpr (16 * r + 15 >= J1) {
          const int i = l + 16 * r;
          double h = 0.0;
          if constexpr (16 * r + 15 > J1) h = acc_get(hv[r][j]);
          vv[r] = i == J1 ? 1.0 : (i > J1 ? h : 0.0);
          a = fma(vv[r], y[r], a);
        } else {
          vv[r] = 0.0;
        }
      });
      a = row16_sum(a);
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        if constexpr (16 * r + 15 >= J1) y[r] = fma(-tj * a, vv[r], y[r]);
      });
    }
  });

  // ---- analysis and RTPP / RTPS (:675-698), fp32 in the reference's order ----------------
  const double sk = sqrt((double)(k - 1));
  float xa[NS];
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int i = l + 16 * r;
    xa[r] = i < k ? (float)(xb_mean + (d + sk * y[r])) : 0.0f;
  });
  if (c.use_rtpp || c.use_rtps) {
    const float xa_mean = seq_sum_f32(xa) * c.nmember_inv;
    double xpl[NS];
    float xap[NS];
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      const int i = l + 16 * r;
      xpl[r] = i < k ? (double)xbl[r] - xb_mean : 0.0;
      xap[r] = 0.0f;
      if (i < k) {
        xap[r] = xa[r] - xa_mean;
        if (c.use_rtpp)
          xap[r] = (float)((double)((1.0f - c.rtpp_alpha) * xap[r]) + (double)c.rtpp_alpha * xpl[r]);
      }
    });
    if (c.use_rtps) {
      double d8 = 0.0;
      sfor<KP>([&](auto mm) {
        constexpr int mb = decltype(mm)::value;
        const double xp = rbcast<mb % 16>(xpl[mb / 16]);  // 0 past member k-1
        d8 = d8 + xp * xp;
      });
      const float xb_std = (float)d8;
      float sq[NS];
      sfor<NS>([&](auto rr) { sq[decltype(rr)::value] = xap[decltype(rr)::value] * xap[decltype(rr)::value]; });
      const float xa_std = seq_sum_f32(sq);
      const float f = c.rtps_alpha * sqrtf(xb_std / xa_std) - c.rtps_alpha + 1.0f;
      sfor<NS>([&](auto rr) { xap[decltype(rr)::value] = xap[decltype(rr)::value] * f; });
    }
    sfor<NS>([&](auto rr) { xa[decltype(rr)::value] = xa_mean + xap[decltype(rr)::value]; });
  }
  if (valid && ptot > 0) {
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      const int i = l + 16 * r;
      if (i < k) slab.var[P + slab.L * i] = xa[r];
    });
    // info.y: decade of the quadrature rule (negative when M/m exceeds the last table)
    if (l == 0) info[gi] = make_int2(ptot, ratio > dec ? -level : level);
  }
}

hipError_t launch_solve_tq4(hipStream_t s, int kp, SolveConsts c, SlabDev slab, long long g0,
                            int npts, const double *ws_a, const double *ws_b1, int2 *info) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr) return hipErrorInvalidValue;
  const int blocks = (npts + 3) / 4;
  switch (kp) {
    case 40:
      hipLaunchKernelGGL((solve_tq4_kernel<40>), dim3(blocks), dim3(64), 0, s, c, slab, g0,
                         npts, ws_a, ws_b1, info);
      return hipGetLastError();
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace cwbl
