// cwbl_band_tail.hip — band_tail_kernel, stage 2 of the two-stage k = 128 solve (see
// cwbl_band.hip for the design): the bulge chase, Q2^T on b1 and x', the quadrature, the
// back-transform and the epilogue, one point per wavefront.
#include "cwbl_band.h"

namespace cwbl {

__constant__ ChasePlan cChase = kChase;

// ==== stage 2: chase, quadrature, back-transform, epilogue ===================================
struct BandTailSmem {
  static constexpr int ROWS = 142;  // 128 rows + padding: a task at row r <= 126 reaches row
                                    // r + 15; what lands past row 127 is never read as data
  static constexpr int UROWS = 136; // u rows r + e <= 133
  union {
    double band[ROWS * 16];  // the chase: A(i, i - d) at 16 i + d, d = 0..15
    double tq[129][4];       // then d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
    double y[128];           // then y for the back-transform
  } a;
  union {
    double u[2][UROWS];  // Q1^T b1, Q1^T x', then through the chase's reflectors
    struct {
      double Ym[128], Zm[128];  // quadrature sum / exact solve, walk order
    } q;
  } b;
};
// (8 blocks of one wavefront per CU: the chase is issue-bound at two waves per SIMD)
static_assert(8 * sizeof(BandTailSmem) <= 160 * 1024, "band tail LDS");

__global__ void __launch_bounds__(64, 2)
band_tail_kernel(SolveConsts c, SlabDev slab, long long g0, int npts, double *__restrict__ ws,
                 int2 *__restrict__ info) {
  constexpr int KP = 128, H = KP / 2;
  using HR = BandRec;
  __shared__ BandTailSmem sm;
  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int l = threadIdx.x;
  const int k = c.k;
  const int ptot = info[gi].x;
  if (ptot == 0) return;  // var unchanged
  double *__restrict__ rec = ws + (long long)gi * HR::WORDS;

  long long P = 0;
  {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long rr = g / slab.ix_lim;
    const int jj = (int)(rr % slab.iy_lim);
    const int kz = (int)(rr / slab.iy_lim);
    P = i + (long long)slab.nx * (jj + (long long)slab.ny * kz);
  }
  const bool mem0 = l < k, mem1 = 64 + l < k;
  const float xb0v = slab.var[P + slab.L * (mem0 ? l : 0)];
  const float xb1v = slab.var[P + slab.L * (mem1 ? 64 + l : 0)];
  const float xb0 = mem0 ? xb0v : 0.0f, xb1 = mem1 ? xb1v : 0.0f;

  // ---- the band into LDS (padding rows zero) -------------------------------------------------
  double *const band = sm.a.band;
  for (int e = l; e < BandTailSmem::ROWS * 16; e += 64) {
    const int i = e >> 4, d = e & 15;
    band[e] = i < 128 && d <= HR::B ? rec[HR::BAND + i * (HR::B + 1) + d] : 0.0;
  }
  for (int i = l; i < BandTailSmem::UROWS; i += 64) {
    sm.b.u[0][i] = i < 128 ? rec[HR::U1 + i] : 0.0;
    sm.b.u[1][i] = i < 128 ? rec[HR::U2 + i] : 0.0;
  }
  __syncthreads();

  // ---- the chase: rounds of up to two tasks (slot 0: even sweeps, slot 1: odd sweeps) ------
  // The reflector of a task (rows r .. r + L - 1) is v_e on lanes e = 0..7 of both 16-lane rows
  // of its slot.  Every lane holds one 8-vector X at the LDS words M r + C + off[e]:
  //   row 0, lanes 0-6:  the left block's column r - 7 + lo at rows r + e (16 r + 7 - lo + 17 e)
  //   row 0, lane 7:     u1 rows r + e
  //   row 0, lanes 8-15: the diagonal block's row r + b, both triangles
  //                      (16 r + 16 max(e, b) + |e - b|)
  //   row 1, lanes 0-7:  the bulge row r + 8 + lo (16 (r + 8 + lo) + 8 + lo - e)
  //   row 1, lanes 8-15: u2 rows r + e (eight identical copies)
  // One instruction stream for all: X -= al v + be w with (al, be) = (tau v^T X, 0) one-sided
  // and (w_b, v_b) two-sided (w = tau (D v) - 1/2 tau^2 (v^T D v) v).  Every lane stores all 8
  // entries back: what lies past row 127 (or is the identity's zero left of a sweep's first
  // task) is rewritten harmlessly (v_e = 0 there, values stay finite); an entry of the
  // diagonal block held twice (lanes 8 + b and 8 + e) takes the later store's rounding; the
  // annihilated column is written last.  A slot without a task this round repeats the other
  // slot's task (identical values to identical words).
  const int slot = l >> 5, rr = (l >> 4) & 1, lo = l & 15;
  const int e8 = lo & 7, b = lo - 8;
  const int U1 = (int)(sm.b.u[0] - band), U2 = (int)(sm.b.u[1] - band);
  int M, CO[8];  // words: M r + CO[e]
  {
    const bool rA = rr == 0 && lo < 7, rB = rr == 0 && lo >= 8, rC = rr == 1 && lo < 8;
    M = rA || rB || rC ? 16 : 1;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      CO[e] = rA ? 7 - lo + 17 * e
            : rB ? 16 * max(e, b) + (e > b ? e - b : b - e)
            : rC ? 136 + 17 * lo - e
            : (rr == 0 ? U1 : U2) + e;
  }
  const bool rV = rr == 0 && lo < 8;  // stores the reflector
  // each slot's sweep, its start round, first task index and task count: uniform values (both
  // slots, scalar loads of the plan), so no vector load keeps the round loop waiting on memory
  int jsS[2], stS[2], fjS[2], ntS[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    jsS[s] = s;
    stS[s] = cChase.start[s];
    fjS[s] = cChase.first[s];
    ntS[s] = cChase.ntask[s];
  }
  double *__restrict__ r2 = rec + HR::R2;
  for (int R = 0; R < cChase.rounds; ++R) {
    // per slot (uniform): task row, annihilated-column word, reflector index
    int rS[2], aS[2], qS[2];
    bool actS[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = R - stS[s];
      actS[s] = jsS[s] <= 125 && t >= 0 && t < ntS[s];
      rS[s] = jsS[s] + 1 + 8 * t;
      aS[s] = 16 * rS[s] + (t == 0 ? 1 : 8);
      qS[s] = fjS[s] + t;
    }
    if (actS[0] || actS[1]) {
      // a slot without a task repeats the other's
      const int sl = actS[slot] ? slot : slot ^ 1;
      const int r = sl ? rS[1] : rS[0];
      const int acol = (sl ? aS[1] : aS[0]) + 17 * e8;  // rows r + e8 of the annihilated column
      const int q = sl ? qS[1] : qS[0];
      double xe = band[acol];
      xe = r + e8 < 128 ? xe : 0.0;
      const double xx = rbcast<0>(rsum8(e8 >= 1 ? xe * xe : 0.0));
      const double alpha = rbcast<0>(xe);
      // this lane's vector (loaded while the reflector is formed)
      const int mr = M * r;
      double X[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) X[e] = band[mr + CO[e]];
      const double a2 = fma(alpha, alpha, xx);
      const double rs = rsq64(a2);
      const bool nz = xx > 0.0;
      const double bt = -copysign(a2 * rs, alpha);
      const double beta = nz ? bt : alpha;
      const double tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
      const double scal = nz ? rcp64(alpha - bt) : 0.0;
      double v = e8 == 0 ? 1.0 : xe * scal;  // v_e on lanes e of a row (lanes 8-15: unused)
      dpp_pin(v);
      double dot = 0.0, dot2 = 0.0;  // v^T X (two chains)
      sfor<8>([&](auto ee) {
        constexpr int e = decltype(ee)::value;
        if constexpr (e % 2 == 0) dot = fmac_row<e>(dot, v, X[e]);
        else dot2 = fmac_row<e>(dot2, v, X[e]);
      });
      dot += dot2;
      const double vb = ror8(v);  // v_b on lane 8 + b
      const double s1 = rsum8(vb * dot);
      double wB = tau * fma(-0.5 * tau, s1 * vb, dot);
      const bool twos = rr == 0 && lo >= 8;
      const double al = twos ? wB : tau * dot;
      const double be = twos ? vb : 0.0;
      dpp_pin(wB);
      sfor<8>([&](auto ee) {
        constexpr int e = decltype(ee)::value;
        X[e] = fnmac_row<8 + e>(fnmac_row<e>(X[e], v, al), wB, be);
      });
#pragma unroll
      for (int e = 0; e < 8; ++e) band[mr + CO[e]] = X[e];
      band[acol] = e8 == 0 ? beta : 0.0;
      if (rV) r2[q * 8 + lo] = lo == 0 ? tau : v;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // a slot whose sweep ends this round takes the next one
      if (jsS[s] <= 125 && R - stS[s] + 1 == ntS[s]) {
        fjS[s] += ntS[s] + chase_ntask(jsS[s] + 1);
        jsS[s] += 2;
        stS[s] = jsS[s] <= 125 ? cChase.start[jsS[s]] : 1 << 30;
        ntS[s] = chase_ntask(jsS[s]);
      }
    }
    __syncthreads();
  }
  if (CWBL_DBG_STOP(c) == 2) {  // timing ablation: the chase only
    rec[HR::BAND + l] = band[16 * l] + band[16 * (64 + l)] + sm.b.u[0][l] + sm.b.u[1][l];
    return;
  }
  // ---- T: d_i = A(i, i), c(i-1, i) = A(i, i-1) ------------------------------------------------
  double dA = band[16 * l], eA = band[16 * l + 1];
  double dB = band[16 * (64 + l)], eB = band[16 * (64 + l) + 1];
  __syncthreads();
  sm.a.tq[l][0] = dA;
  sm.a.tq[l][1] = l == 0 ? 0.0 : eA;
  sm.a.tq[64 + l][0] = dB;
  sm.a.tq[64 + l][1] = eB;
  if (l == 0) sm.a.tq[KP][1] = 0.0;
  // (Q2^T u1, Q2^T u2 were formed in the chase)
  sm.a.tq[l][2] = sm.b.u[0][l];
  sm.a.tq[64 + l][2] = sm.b.u[0][64 + l];
  sm.a.tq[l][3] = sm.b.u[1][l];
  sm.a.tq[64 + l][3] = sm.b.u[1][64 + l];
  __syncthreads();
  // trace of T (= trace of A) for the spectrum bound
  double trace = 0.0;
  {
    double tp = 0.0;
    if (l < k) tp += sm.a.tq[l][0];
    if (64 + l < k) tp += sm.a.tq[64 + l][0];
    trace = wave_sum_dpp(tp);
  }

  // ---- T^-1/2 u2 by quadrature, u1^T T^-1 u2 exactly (the tail kernel's rule) ----------------
  const double m = (double)c.inflat;
  const double ratio = trace / m - (double)(k - 1);
  int level = 1;
  double dec = 10.0;
  while (level < kQuadLevels && dec < ratio) {
    dec *= 10.0;
    ++level;
  }
  {
    const int node = l & 31, side = l >> 5;
    const int npass = quad_passes(level);
    const double2 *rule = quad_rule(c.quad_r, npass == 1 ? 4 : 8, level);
    for (int pass = 0; pass < npass; ++pass) {
      const bool exact = pass == 0 && node == 31;
      double sigma = 0.0, omega = 0.0;
      if (!exact) {
        const double2 tw = rule[31 * pass + node];
        sigma = m * tw.x;
        omega = sqrt(m) * tw.y;
      }
      const unsigned q0 = side ? (KP - 1) * 32u : 0u, dirb = side ? (unsigned)-32 : 32u;
      const unsigned csb = side ? 40u : 8u;
      auto fwd = [&](int t, double &dl, double &gt) {
        const unsigned o = opaque_after(q0, dl) + dirb * (unsigned)t;
        const double ct = lds_at(sm.a.tq, o + csb);
        const double lt = ct * rcp64(dl);
        dl = fma(-lt, ct, lds_at(sm.a.tq, o) + sigma);
        gt = fma(-lt, gt, lds_at(sm.a.tq, o + 24));
      };
      constexpr int S = 8, NS = H / S;
      double ckd[NS], ckg[NS];
      double dl = lds_at(sm.a.tq, q0) + sigma, gt = lds_at(sm.a.tq, q0 + 24);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        ckd[s] = dl;
        ckg[s] = gt;
#pragma unroll
        for (int t = S * s + 1; t < S * s + S; ++t) fwd(t, dl, gt);
        if (s + 1 < NS) fwd(S * s + S, dl, gt);
      }
      const double cm = sm.a.tq[H][1];
      const double dlo = __shfl_xor(dl, 32, 64), go = __shfl_xor(gt, 32, 64);
      double xv = (gt * dlo - cm * go) / fma(dl, dlo, -cm * cm);
      double *ym = sm.b.q.Ym + side * H, *zm = sm.b.q.Zm + side * H;
      for (int s = NS - 1; s >= 0; --s) {
        double hh[S], mmv[S];
        double d2 = ckd[s], g2 = ckg[s];
#pragma unroll
        for (int i = 0; i < S; ++i) {
          const int t = S * s + i;
          if (i > 0) fwd(t, d2, g2);
          const double rd = rcp64(d2);
          hh[i] = g2 * rd;
          mmv[i] = (t + 1 < H)
                       ? lds_at(sm.a.tq, opaque_after(q0, d2) + dirb * (unsigned)(t + 1) + csb) * rd
                       : 0.0;
        }
#pragma unroll
        for (int i = S - 1; i >= 0; --i) {
          const int t = S * s + i;
          if (t != H - 1) xv = fma(-mmv[i], xv, hh[i]);
          const double ys = half_sum_dpp(omega * xv);
          if (node == 0) ym[t] = pass ? ym[t] + ys : ys;
          if (exact) zm[t] = xv;
        }
      }
    }
  }
  __syncthreads();
  if (CWBL_DBG_STOP(c) == 3) {  // timing ablation: chase + quadrature
    rec[HR::BAND + l] = sm.b.q.Ym[l] + sm.b.q.Zm[l];
    return;
  }
  auto walk = [](int i) { return i < H ? i : H + (KP - 1 - i); };
  const double d = wave_sum_dpp(fma(sm.a.tq[l][2], sm.b.q.Zm[walk(l)],
                                    sm.a.tq[64 + l][2] * sm.b.q.Zm[walk(64 + l)]));
  double y0 = sm.b.q.Ym[walk(l)], y1 = sm.b.q.Ym[walk(64 + l)];
  __syncthreads();
  // ---- y <- Q1 Q2 y: the chase's reflectors sweep by sweep in reverse, then the panels -------
  sm.a.y[l] = y0;
  sm.a.y[64 + l] = y1;
  __syncthreads();
  {
    // sweeps in reverse; a sweep's reflectors act on disjoint rows, 8 per pass (lane: reflector
    // l >> 3, entry l & 7); the next pass's reflectors are loaded while this one runs
    // (the loads are unconditional, at a valid address, and masked at use: loads under a
    // branch would make the wait before the use cover the prefetch too)
    struct Pass {
      double tu, ve;  // raw: q[0], q[e]
      int row;        // -1: no entry
    };
    auto load_pass = [&](int j, int pass) {
      Pass d;
      const int tt = 8 * pass + (l >> 3), e = l & 7;
      const bool ok = j >= 0 && tt < chase_ntask(j);
      const int r = j + 1 + 8 * tt;
      const bool in = ok && e < min(8, 128 - r);
      const double *q = r2 + (ok ? cChase.first[max(j, 0)] + tt : 0) * 8;
      d.tu = q[0];
      d.ve = q[e];
      d.row = in ? r + e : -1;
      return d;
    };
    int j = 125, pass = 0;
    Pass cur = load_pass(j, pass);
    while (j >= 0) {
      int jn = j, pn = pass + 1;
      if (8 * pn >= chase_ntask(j)) {
        jn = j - 1;
        pn = 0;
      }
      const Pass nxt = load_pass(jn, pn);
      const bool in = cur.row >= 0;
      const double ve = in ? ((l & 7) == 0 ? 1.0 : cur.ve) : 0.0;
      const double yv = sm.a.y[in ? cur.row : 0];
      const double dd = rsum8(ve * yv);
      if (in) sm.a.y[cur.row] = fma(-cur.tu * dd, ve, yv);
      __syncthreads();
      cur = nxt;
      j = jn;
      pass = pn;
    }
  }
  y0 = sm.a.y[l];
  y1 = sm.a.y[64 + l];
  {
    // lane l: rows l and 64 + l of V_p (rows >= r0 only) and T_p[l >> 3][l & 7] (T upper, zeros
    // below); the next panel's loads are issued before this one's arithmetic (unconditional, at
    // valid addresses, masked at use)
    struct Panel {
      double Va[8], Vb[8], t;
    };
    auto load_panel = [&](int p) {
      Panel d;
      const int r0 = 8 * p + 8;
      const double *pv = rec + HR::pv(p);
      const int ia = max(l - r0, 0), ib = max(64 + l - r0, 0);
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        d.Va[a] = pv[ia * 8 + a];
        d.Vb[a] = pv[ib * 8 + a];
      }
      d.t = rec[HR::PT + 64 * p + l];
      return d;
    };
    Panel cur = load_panel(HR::NP - 1);
    for (int p = HR::NP - 1; p >= 0; --p) {
      const Panel nxt = load_panel(max(p - 1, 0));
      const int r0 = 8 * p + 8;
      const bool va = l >= r0, vb = 64 + l >= r0;
      double Va[8], Vbb[8], s[8];
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        Va[a] = va ? cur.Va[a] : 0.0;
        Vbb[a] = vb ? cur.Vb[a] : 0.0;
        s[a] = fma(Va[a], y0, Vbb[a] * y1);
      }
      wave_sum4_dpp(s[0], s[1], s[2], s[3]);
      wave_sum4_dpp(s[4], s[5], s[6], s[7]);
      // z = T s: lane (a, b) forms T[a][b] s_b, the 8 lanes of row a sum it
      double sb = s[0];
#pragma unroll
      for (int b = 1; b < 8; ++b) sb = (l & 7) == b ? s[b] : sb;
      const double zl = rsum8(cur.t * sb);
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const double za = readlane_f64(zl, 8 * a);
        y0 = fma(-Va[a], za, y0);
        y1 = fma(-Vbb[a], za, y1);
      }
      cur = nxt;
    }
  }

  // ---- analysis and RTPP / RTPS (:671-698), fp32 in the reference's order --------------------
  auto seq_sum_f32 = [&](float a0, float a1) {
    float s = 0.0f;
    for (int mm = 0; mm < 64; ++mm) s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a0), mm));
    for (int mm = 64; mm < k; ++mm) s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a1), mm - 64));
    return s;
  };
  const double xb_mean = (double)(seq_sum_f32(xb0, xb1) * c.nmember_inv);  // fp32 (:671)
  const double sk = sqrt((double)(k - 1));
  float xa0 = mem0 ? (float)(xb_mean + (d + sk * y0)) : 0.0f;
  float xa1 = mem1 ? (float)(xb_mean + (d + sk * y1)) : 0.0f;
  if (c.use_rtpp || c.use_rtps) {
    const float xa_mean = seq_sum_f32(xa0, xa1) * c.nmember_inv;
    const double xp0 = mem0 ? (double)xb0 - xb_mean : 0.0;
    const double xp1 = mem1 ? (double)xb1 - xb_mean : 0.0;
    float xap0 = mem0 ? xa0 - xa_mean : 0.0f;
    float xap1 = mem1 ? xa1 - xa_mean : 0.0f;
    if (c.use_rtpp) {
      if (mem0) xap0 = (float)((double)((1.0f - c.rtpp_alpha) * xap0) + (double)c.rtpp_alpha * xp0);
      if (mem1) xap1 = (float)((double)((1.0f - c.rtpp_alpha) * xap1) + (double)c.rtpp_alpha * xp1);
    }
    if (c.use_rtps) {
      double d8 = 0.0;
      for (int mm = 0; mm < 64; ++mm) {
        const double xp = readlane_f64(xp0, mm);
        d8 = d8 + xp * xp;
      }
      for (int mm = 64; mm < k; ++mm) {
        const double xp = readlane_f64(xp1, mm - 64);
        d8 = d8 + xp * xp;
      }
      const float xb_std = (float)d8;
      const float xa_std = seq_sum_f32(xap0 * xap0, xap1 * xap1);
      const float f = c.rtps_alpha * sqrtf(xb_std / xa_std) - c.rtps_alpha + 1.0f;
      xap0 = xap0 * f;
      xap1 = xap1 * f;
    }
    xa0 = xa_mean + xap0;
    xa1 = xa_mean + xap1;
  }
  if (mem0) slab.var[P + slab.L * l] = xa0;
  if (mem1) slab.var[P + slab.L * (64 + l)] = xa1;
  if (l == 0) info[gi] = make_int2(ptot, ratio > dec ? -level : level);
}

hipError_t launch_band_tail(hipStream_t s, SolveConsts c, SlabDev slab, long long g0, int npts,
                            double *ws, int2 *info) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr || c.kp != 128 || c.k <= 96) return hipErrorInvalidValue;
  hipLaunchKernelGGL(band_tail_kernel, dim3(npts), dim3(64), 0, s, c, slab, g0, npts, ws, info);
  return hipGetLastError();
}

}  // namespace cwbl
