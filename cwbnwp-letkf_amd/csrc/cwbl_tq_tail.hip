// cwbl_tq_tail.hip — solve_tqb_tail_kernel<KP, J0>: the second half of the per-point LETKF
// solve (letkf_solve, module_letkf_core.f90:598-700) for large ensembles (configs[3],
// k = 97..128), one grid point per wavefront.
//
// solve_tq_big_kernel<KP, false, J0> (cwbl_tq_big.hip) stages the point's columns, assembles
// A = (k-1)/infl I + Yb Yb^T and b1 = Yb d on the matrix cores and runs the first J0 steps of
// the Householder tridiagonalisation A = Q T Q^T (dsytd2 order) on 4x4 register blocks spread
// over a 256-thread workgroup; each of its steps is a chain of four barriers and LDS
// exchanges, so its cost per step is nearly fixed.  It hands the trailing KT x KT matrix,
// its J0 reflectors, T so far and Q^T b1, Q^T x' over through the workspace (BigHandoff).
// This kernel finishes the algorithm — the remaining steps, the T^-1/2 quadrature and the
// T^-1 solve, the back-transform and the RTPP/RTPS epilogue in the reference's fp32 order —
// inside one wavefront, with no barrier between lanes of different waves:
//
//   lane l holds the FULL trailing row J0 + l (KT = 64 doubles, static register indices)
//   and the vectors' rows l (prefix) and J0 + l (trailing).
//
// A step needs the pivot column per lane and the pivot row's entries as operands of every
// lane.  A is kept symmetric (both triangles are updated), so lane l's entry A(l, j) is the
// pivot row's entry l: each lane picks it from its registers, two v_permlane swaps per half
// copy the row into four row-replicated registers, and the matvec and the rank-2 update take
// x_c = A(j, c) and w_c as the row_newbcast operand of a fused v_fmac_f64_dpp — no LDS in the
// step.  Row j is never touched again by later steps (v and w vanish there), so it IS the
// Householder vector (v = scal x, 1 at row j + 1): each lane parks its entry in the record's
// scratch rows, where the back-transform reads it.  Columns are processed in groups of
// eight; the steps run in blocks by the group of column j + 1, so the groups left of it are
// skipped at compile time and the rest run without selects.
#include "cwbl_device.h"

#include <utility>

namespace cwbl {

namespace {


__device__ __forceinline__ float readlane_f32(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}

}  // namespace

template <int KP, int J0>
struct TailSmem {
  static constexpr int KT = KP - J0;
  double row[KT];         // a row of the trailing 2x2 block's step
  double tq[KP + 1][4];   // d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
  double tau[KP];
  double scl[KP];         // this kernel's reflectors: v = scl * x below row j + 1
  double Ym[KP], Zm[KP];  // quadrature sum / exact solve, walk order
};

// WPE: waves per SIMD the register budget is sized for (2: 256 VGPRs, 3: 168)
template <int KP, int J0, int WPE>
__global__ void __launch_bounds__(64, WPE)
solve_tqb_tail_kernel(SolveConsts c, SlabDev slab, long long g0, int npts,
                      double *__restrict__ ws, int2 *__restrict__ info) {
  using HO = BigHandoff<KP, J0>;
  constexpr int KT = HO::KT;  // trailing rows: one per lane
  constexpr int H = KP / 2;   // rows walked by each side of a twisted solve
  constexpr int NG = KT / 8;  // column groups
  static_assert(KT == 64 && J0 <= 64 && J0 % 4 == 0, "one trailing row per lane; prefix rows on lanes < J0");
  using SM = TailSmem<KP, J0>;
  __shared__ SM sm;

  // the hand-off kernel's XCD chunks, each from its end: the records it wrote last (still in
  // the MALL) are read first
  const int gi = xcd_remap_rev(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int l = threadIdx.x;
  const int k = c.k;
  const int ptot = info[gi].x;
  if (ptot == 0) return;  // no accepted observation: var unchanged (:220, :226)
  const auto *__restrict__ w = gptr(ws + (long long)gi * HO::WORDS);

  // background of the point (used by the epilogue; loaded first, the latency hides behind
  // the steps)
  long long P = 0;
  {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long rr = g / slab.ix_lim;
    const int jj = (int)(rr % slab.iy_lim);
    const int kz = (int)(rr / slab.iy_lim);
    P = i + (long long)slab.nx * (jj + (long long)slab.ny * kz);
  }
  const bool mem0 = l < J0;      // prefix row / member l exists (k > J0)
  const bool mem1 = J0 + l < k;  // member J0 + l exists
  const float xb0v = slab.var[P + slab.L * (mem0 ? l : 0)];  // branch-free: valid addresses
  const float xb1v = slab.var[P + slab.L * (mem1 ? J0 + l : 0)];
  const float xb0 = mem0 ? xb0v : 0.0f;
  const float xb1 = mem1 ? xb1v : 0.0f;

  // ---- hand-off: trailing rows (coalesced by column), T and the vectors' prefix ----------
  double A[KT];
  sfor<KT>([&](auto cc) {
    constexpr int col = decltype(cc)::value;
    A[col] = w[HO::TA + col * KT + l];
  });
  double u1t = w[HO::U1 + J0 + l], u2t = w[HO::U2 + J0 + l];  // trailing Q^T b1, Q^T x'
  if (mem0) {
    sm.tq[l][0] = w[HO::D + l];
    sm.tq[l + 1][1] = w[HO::E + l];
    sm.tq[l][2] = w[HO::U1 + l];
    sm.tq[l][3] = w[HO::U2 + l];
    sm.tau[l] = w[HO::TAU + l];
  }
  // trailing rows of T: decoupled unit rows until the steps write them (rows >= k stay so)
  sm.tq[J0 + l][0] = 1.0;
  sm.tq[J0 + l + 1][1] = 0.0;
  sm.tau[J0 + l] = 0.0;
  if (l == 0) sm.tq[0][1] = 0.0;
  __syncthreads();
  double trace = 0.0;  // d_0 + d_1 + ... in step order, as solve_tq_big_kernel sums it
  for (int j = 0; j < J0; ++j) trace += sm.tq[j][0];

  // lane jl's row -> sm.row (static register indices): the trailing 2x2 block's entries
  auto publish_row = [&](int jl) {
    __syncthreads();  // the previous readers of sm.row are done
    if (l == jl) {
      sfor<KT / 2>([&](auto cc) {
        constexpr int col = 2 * decltype(cc)::value;
        *reinterpret_cast<double2 *>(&sm.row[col]) = make_double2(A[col], A[col + 1]);
      });
    }
    __syncthreads();
  };
  // the record's scratch rows (BT): row jl of this kernel's steps, where the back-transform
  // finds it once the registers are released
  // (entries at or above the reflector's row j + 1 are neither stored nor loaded: rec_off)
  const auto rec = rec_rsrc(ws + (long long)gi * HO::WORDS, HO::WORDS);

  // ---- Householder steps j = J0 .. k-3 (local jl = j - J0) --------------------------------
  // A is symmetric, so lane l's entry A[jl] is the pivot row's entry l.  The pivot row and w
  // reach the lanes without LDS: rep4 copies them into four row-replicated registers (every
  // 16-lane row of R[g] holds entries 16g .. 16g+15) and the matvec and the rank-2 update take
  // entry c as the row_newbcast operand of a fused v_fmac_f64_dpp.  The steps run in blocks by
  // the group of column j + 1 (gb = (jl + 1) / 8, static): the 8-column groups left of it are
  // skipped at compile time, and the pivot column is picked from the block's eight registers
  // by value.  Column j + 1 and the columns left of it in its group need no selects: the
  // replicated row carries xt_{j+1} = alpha - beta and zeros left of it (A(:, c) xt_c and the
  // update then vanish there; w_c = 0 at c <= j as well).
  auto rep4 = [](double x, double (&R)[4]) {
    const int xl = (int)__double_as_longlong(x), xh = (int)(__double_as_longlong(x) >> 32);
    auto mk = [](int lo, int hi) {
      return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    };
    // rows (0, 1, 0, 1) and (2, 3, 2, 3), then each row of those over its pair
    const auto al = __builtin_amdgcn_permlane32_swap(xl, xl, false, false);
    const auto ah = __builtin_amdgcn_permlane32_swap(xh, xh, false, false);
    const auto bl = __builtin_amdgcn_permlane16_swap(al[0], al[0], false, false);
    const auto bh = __builtin_amdgcn_permlane16_swap(ah[0], ah[0], false, false);
    const auto cl = __builtin_amdgcn_permlane16_swap(al[1], al[1], false, false);
    const auto ch = __builtin_amdgcn_permlane16_swap(ah[1], ah[1], false, false);
    R[0] = mk(bl[0], bh[0]);
    R[1] = mk(bl[1], bh[1]);
    R[2] = mk(cl[0], ch[0]);
    R[3] = mk(cl[1], ch[1]);
    // a DPP source is not read within two wait states of its VALU write
    asm volatile("s_nop 1" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]));
  };
  const int nst = k - 2 - J0;  // k > J0 + 2 (launcher)
  auto step = [&](auto GB, int jl) {
    constexpr int gb = decltype(GB)::value;
    constexpr int jb = gb == 0 ? 0 : 8 * gb - 1;  // the block's first step
    const int j = J0 + jl, j1 = jl + 1;
    // A(J0 + l, j) = A[jl], picked by value: the candidates pass an empty asm, so that the
    // compiler cannot fold the selects of register-array loads into one load through a
    // selected address (which sends all of A to scratch memory)
    auto opq = [](double a) {
      asm("" : "+v"(a));
      return a;
    };
    double xr = opq(A[jb]);
    sfor<7>([&](auto ii) {
      constexpr int cc = jb + 1 + decltype(ii)::value;
      if constexpr (cc < KT) xr = jl == cc ? opq(A[cc]) : xr;
    });
    rec_st(rec, rec_off(l > j1, HO::BT + jl * KT + l), xr);
    const double dj = readlane_f64(xr, jl), alpha = readlane_f64(xr, j1);
    trace += dj;
    const double x = l > j1 ? xr : 0.0;
    double xx = x * x, xu = x * u2t, xb = x * u1t, z3 = 0.0;
    wave_sum4_dpp(xx, xu, xb, z3);
    // dlarfg with fp64 rcp/rsq refined to ~1 ulp; H = I when x = 0 (tau = 0, v = e_j+1)
    const double a2 = fma(alpha, alpha, xx);
    const double rs = rsq64(a2);  // 1/|beta|
    const bool nz = xx > 0.0;
    const double bt = -copysign(a2 * rs, alpha);
    const double beta = nz ? bt : alpha;
    const double tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
    const double rab = rcp64(alpha - bt);
    const double scal = nz ? rab : 0.0;
    if (l == 0) {
      sm.tq[j][0] = dj;
      sm.tq[j + 1][1] = beta;
      sm.tau[j] = tau;
      sm.scl[j] = scal;
    }
    const double v = l == j1 ? 1.0 : x * scal;
    const double s2 = fma(scal, xu, readlane_f64(u2t, j1));  // v . x'
    const double s3 = fma(scal, xb, readlane_f64(u1t, j1));  // v . b1
    u2t = fma(-tau * s2, v, u2t);
    u1t = fma(-tau * s3, v, u1t);
    // The uniform side of v: v_c = scal * xt_c with xt_c = x_c = A(j, c) below row j + 1 and
    // xt_{j+1} = alpha - beta = 1/scal (0 when H = I), so column j + 1 needs no special
    // case (v_{j+1} = scal (alpha - beta) is 1 to the last bit or so).
    const double amb = nz ? alpha - bt : 0.0;
    double R[4], W[4];
    rep4(l > j1 ? x : l == j1 ? amb : 0.0, R);
    // A v = scal * sum_{c >= j+1} A(:, c) xt_c (volatile forms, in this order)
    // (four chains, each chain's FMAs four instructions apart, past the DPP read-after-write
    // wait states; r6: eight chains cost eight zeroing moves and four adds more per step,
    // 4.45 against 4.38 ms per launch)
    double q[4] = {0.0, 0.0, 0.0, 0.0};
    sfor<KT - 8 * gb>([&](auto cc) {
      constexpr int col = 8 * gb + decltype(cc)::value;
      q[col % 4] = fmac_row_v<col % 16>(q[col % 4], R[col / 16], A[col]);
    });
    const double av = scal * ((q[0] + q[1]) + (q[2] + q[3]));  // (A v)_l
    const double s1 = tau * wave_sum_dpp(v * av);   // v^T (tau A v); v = 0 at rows <= j
    // (w is not zeroed on the eliminated rows: as in the hand-off kernel, it only moves their
    // own entries, which nothing reads again)
    const double wl = fma(-0.5 * tau * s1, v, tau * av);
    const double wsl = wl * scal;
    rep4(wl, W);
    // A <- A - w v^T - v w^T, a group's eight columns per pass (each column's second FMA
    // eight instructions after its first)
    sfor<NG - gb>([&](auto gg) {
      constexpr int c0 = 8 * (gb + decltype(gg)::value);
      sfor<8>([&](auto ii) {
        constexpr int col = c0 + decltype(ii)::value;
        A[col] = fnmac_row_v<col % 16>(A[col], R[col / 16], wsl);
      });
      sfor<8>([&](auto ii) {
        constexpr int col = c0 + decltype(ii)::value;
        A[col] = fnmac_row_v<col % 16>(A[col], W[col / 16], v);
      });
    });
  };
  // (timing ablation, debug builds: CWBL_DEBUG_TQ_STOP=2 with CWBL_DEBUG_TQ_STEPS = 64 + S runs
  // only this kernel's first S steps; the hand-off kernel's 64 all run)
  const int nrun = CWBL_DBG_STOP(c) == 2 && CWBL_DBG_STEPS(c) > 64 ? min(nst, CWBL_DBG_STEPS(c) - 64) : nst;
  sfor<NG>([&](auto GB) {  // block gb: steps jl = 8 gb - 1 .. 8 gb + 6 (column j + 1 in group gb)
    constexpr int gb = decltype(GB)::value;
    const int hi = min(8 * gb + 6, nrun - 1);
    for (int jl = gb == 0 ? 0 : 8 * gb - 1; jl <= hi; ++jl) step(GB, jl);
  });
  {  // the trailing 2x2 (rows k-2, k-1): already tridiagonal
    const int jl = nst;
    publish_row(jl);
    const double d0 = sm.row[jl], e1 = sm.row[jl + 1];
    publish_row(jl + 1);
    const double d1 = sm.row[jl + 1];
    trace += d0;
    trace += d1;
    if (l == 0) {
      sm.tq[k - 2][0] = d0;
      sm.tq[k - 1][1] = e1;
      sm.tq[k - 1][0] = d1;
    }
  }
  sm.tq[J0 + l][2] = u1t;
  sm.tq[J0 + l][3] = u2t;
  __syncthreads();
  if (CWBL_DBG_STOP(c) == 2) {  // timing ablation: stop after the tridiagonalisation
    if (l == 0) info[gi] = make_int2(ptot, (int)(trace + u1t + u2t));
    return;
  }

  // ---- T^-1/2 u2 by quadrature, u1^T T^-1 u2 exactly (solve_tq_big_kernel's rule) --------
  // lane = node (0..31) + 32 side: side 0 walks rows 0..H-1, side 1 rows KP-1..H; node 31
  // solves T^-1 u2.  The forward sweep is checkpointed every 8 rows and recomputed per
  // segment in the backward sweep.
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
    // one pass of 31 nodes (+ the exact solve on node 31) up to level kQuadLevels31, a
    // second pass with nodes 31..62 of the 63-node rule above (quad_passes; wave-uniform)
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
    // byte offsets into sm.tq: row t of the walk at q0 + dirb t (opaque_after, cwbl_device.h)
    const unsigned q0 = side ? (KP - 1) * 32u : 0u, dirb = side ? (unsigned)-32 : 32u;
    const unsigned csb = side ? 40u : 8u;  // coupling with the previous row of the walk
    auto fwd = [&](int t, double &dl, double &gt) {
      const unsigned o = opaque_after(q0, dl) + dirb * (unsigned)t;
      const double ct = lds_at(sm.tq, o + csb);
      const double lt = ct * rcp64(dl);
      dl = fma(-lt, ct, lds_at(sm.tq, o) + sigma);
      gt = fma(-lt, gt, lds_at(sm.tq, o + 24));
    };
    constexpr int S = 8, NS = H / S;
    double ckd[NS], ckg[NS];
    double dl = lds_at(sm.tq, q0) + sigma, gt = lds_at(sm.tq, q0 + 24);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      ckd[s] = dl;
      ckg[s] = gt;
#pragma unroll
      for (int t = S * s + 1; t < S * s + S; ++t) fwd(t, dl, gt);
      if (s + 1 < NS) fwd(S * s + S, dl, gt);
    }
    const double cm = sm.tq[H][1];  // meeting rows H-1 (top) and H (bottom)
    const double dlo = __shfl_xor(dl, 32, 64), go = __shfl_xor(gt, 32, 64);
    double xv = (gt * dlo - cm * go) / fma(dl, dlo, -cm * cm);
    double *ym = sm.Ym + side * H, *zm = sm.Zm + side * H;
    for (int s = NS - 1; s >= 0; --s) {
      double hh[S], mmv[S];
      double d2 = ckd[s], g2 = ckg[s];
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int t = S * s + i;
        if (i > 0) fwd(t, d2, g2);
        const double rd = rcp64(d2);
        hh[i] = g2 * rd;
        mmv[i] = (t + 1 < H)  // c_{t+1} / dl_t
                     ? lds_at(sm.tq, opaque_after(q0, d2) + dirb * (unsigned)(t + 1) + csb) * rd
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
    }  // pass
  }
  __syncthreads();
  // rows l (slot 0) and J0 + l (slot 1) in walk order: side 1 walks KP-1 .. H
  auto walk = [](int i) { return i < H ? i : H + (KP - 1 - i); };
  const int w0 = walk(mem0 ? l : 0), w1 = walk(J0 + l);
  double y0 = mem0 ? sm.Ym[w0] : 0.0, y1 = sm.Ym[w1];
  const double d = wave_sum_dpp(fma(mem0 ? sm.tq[l][2] : 0.0, sm.Zm[w0],
                                    sm.tq[J0 + l][2] * sm.Zm[w1]));
  if (CWBL_DBG_STOP(c) == 3) {  // timing ablation: stop after the quadrature
    if (l == 0) info[gi] = make_int2(ptot, (int)(d + y0 + y1));
    return;
  }

  // ---- back-transform y <- Q y = H_0 H_1 ... H_{k-3} y, four reflectors per reduction ------
  // For H_a H_{a+1} H_{a+2} H_{a+3} y (H_{a+3} first): v_q . y and v_q . v_p (q < p) in one
  // 10-value reduction, then y -= sum_q c_q v_q with c_3 = tau_3 v_3.y, c_2 = tau_2 (v_2.y -
  // c_3 v_2.v_3), ...  Lane slots: row l (v0, y0) and row J0 + l (v1, y1).
  auto apply4 = [&](const double (&v0)[4], const double (&v1)[4], const double (&ta)[4]) {
    double t[12];
    sfor<4>([&](auto qq) { t[qq] = fma(v0[qq], y0, v1[qq] * y1); });
    constexpr int P[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
    sfor<6>([&](auto ee) {
      constexpr int a = P[ee][0], b = P[ee][1];
      t[4 + ee] = fma(v0[a], v0[b], v1[a] * v1[b]);
    });
    t[10] = t[11] = 0.0;
    wave_sum4_dpp(t[0], t[1], t[2], t[3]);
    wave_sum4_dpp(t[4], t[5], t[6], t[7]);
    wave_sum4_dpp(t[8], t[9], t[10], t[11]);
    // t: d0..d3, G01 G02 G03 G12 G13 G23
    const double c3 = ta[3] * t[3];
    const double c2 = ta[2] * fma(-c3, t[9], t[2]);
    const double c1 = ta[1] * fma(-c3, t[8], fma(-c2, t[7], t[1]));
    const double c0 = ta[0] * fma(-c3, t[6], fma(-c2, t[5], fma(-c1, t[4], t[0])));
    y0 = fma(-c0, v0[0], fma(-c1, v0[1], fma(-c2, v0[2], fma(-c3, v0[3], y0))));
    y1 = fma(-c0, v1[0], fma(-c1, v1[1], fma(-c2, v1[2], fma(-c3, v1[3], y1))));
  };
  // The reflector rows come from the record in HBM (a sub-batch's records are far larger than
  // the caches): one group's loads take ~4 k cycles under load against ~350 cycles of apply4.
  // So the groups run as a static pipeline over a ring of register slots holding the raw
  // loaded rows only, group g + D's loads issued right after group g's rows are formed (no
  // register copies between iterations: the wait before a group covers only its own loads,
  // issued D groups earlier; tau, the scale and the unit entry are formed from LDS when the
  // group is applied).  (r6: a loop that copied the next group's registers into the current
  // ones made the compiler wait for every load at the end of each iteration — one memory
  // latency per group.)  Groups past the last reflector (k < KP) load nothing and apply
  // tau = 0.
  auto issue_tail = [&](int top, double (&x)[4]) {
    sfor<4>([&](auto qq) {
      const int jl = top - 3 + qq;  // < 0: padding (H = I)
      x[qq] = rec_ld(rec, rec_off(jl >= 0 && l > jl + 1, HO::BT + jl * KT + l));
    });
  };
  // (branch-free: a uniform `jl < 0 ?` select let the compiler branch around the use of the
  // loaded row and sink the load into the branch, with a wait for it right there)
  auto form_tail = [&](int top, const double (&x)[4], double (&v1)[4], double (&ta)[4]) {
    sfor<4>([&](auto qq) {
      const int jl = top - 3 + qq, jc = jl < 0 ? 0 : jl;
      const int j1 = jl + 1;
      const double pad = jl < 0 ? 0.0 : 1.0;  // padding group entries: H = I
      const double sc = sm.scl[J0 + jc];
      v1[qq] = pad * (l == j1 ? 1.0 : (l > j1 ? sc * x[qq] : 0.0));
      ta[qq] = pad * sm.tau[J0 + jc];
    });
  };
  auto issue_hand = [&](int top, double (&x0)[4], double (&x1)[4]) {
    sfor<4>([&](auto qq) {
      const int j = top - 3 + qq;
      // rows <= j hold zeros (not loaded); row j + 1 holds 1.0
      x0[qq] = rec_ld(rec, rec_off(mem0 && l > j, HO::HV + j * KP + l));
      x1[qq] = w[HO::HV + j * KP + J0 + l];
    });
  };
  {
    constexpr int NGT = (KT - 2 + 3) / 4;  // groups of this kernel's reflectors at k = KP
    constexpr int D = NGT < 8 ? NGT : 8;   // groups in flight (8 VGPRs each)
    const double zero4[4] = {0.0, 0.0, 0.0, 0.0};
    double rx[D][4];
    sfor<D>([&](auto G) { issue_tail(nst - 1 - 4 * decltype(G)::value, rx[decltype(G)::value]); });
    sfor<NGT>([&](auto G) {
      constexpr int g = decltype(G)::value, sl = g % D;
      double v1[4], ta[4];
      form_tail(nst - 1 - 4 * g, rx[sl], v1, ta);
      if constexpr (g + D < NGT) issue_tail(nst - 1 - 4 * (g + D), rx[sl]);
      apply4(zero4, v1, ta);
    });
  }
  {
    constexpr int NGH = J0 / 4;            // the hand-off's reflectors (rows > j)
    constexpr int D = NGH < 4 ? NGH : 4;   // (v0 and v1: 16 VGPRs each)
    double r0[D][4], r1[D][4];
    sfor<D>([&](auto G) {
      constexpr int g = decltype(G)::value;
      issue_hand(J0 - 1 - 4 * g, r0[g], r1[g]);
    });
    sfor<NGH>([&](auto G) {
      constexpr int g = decltype(G)::value, sl = g % D, top = J0 - 1 - 4 * g;
      double v0[4], v1[4], ta[4];
      sfor<4>([&](auto qq) {
        v0[qq] = r0[sl][qq];
        v1[qq] = r1[sl][qq];
        ta[qq] = sm.tau[top - 3 + decltype(qq)::value];
      });
      if constexpr (g + D < NGH) issue_hand(J0 - 1 - 4 * (g + D), r0[sl], r1[sl]);
      apply4(v0, v1, ta);
    });
  }

  // ---- analysis and RTPP / RTPS (:671-698), fp32 in the reference's order -----------------
  // sequential fp32 sum over members 0 .. k-1 (member m: slot m / J0, lane m % J0)
  auto seq_sum_f32 = [&](float a0, float a1) {
    float s = 0.0f;
    for (int mm = 0; mm < J0; ++mm) s = s + readlane_f32(a0, mm);
    for (int mm = J0; mm < k; ++mm) s = s + readlane_f32(a1, mm - J0);
    return s;
  };
  const double xb_mean = (double)(seq_sum_f32(xb0, xb1) * c.nmember_inv);  // fp32 (:671)
  const double sk = sqrt((double)(k - 1));
  float xa0 = (float)(xb_mean + (d + sk * y0));
  float xa1 = mem1 ? (float)(xb_mean + (d + sk * y1)) : 0.0f;
  if (c.use_rtpp || c.use_rtps) {
    const float xa_mean = seq_sum_f32(xa0, xa1) * c.nmember_inv;
    const double xp0 = (double)xb0 - xb_mean;
    const double xp1 = mem1 ? (double)xb1 - xb_mean : 0.0;
    float xap0 = xa0 - xa_mean;
    float xap1 = mem1 ? xa1 - xa_mean : 0.0f;
    if (c.use_rtpp) {
      xap0 = (float)((double)((1.0f - c.rtpp_alpha) * xap0) + (double)c.rtpp_alpha * xp0);
      if (mem1)
        xap1 = (float)((double)((1.0f - c.rtpp_alpha) * xap1) + (double)c.rtpp_alpha * xp1);
    }
    if (c.use_rtps) {
      double d8 = 0.0;
      for (int mm = 0; mm < J0; ++mm) {
        const double xp = readlane_f64(xp0, mm);
        d8 = d8 + xp * xp;
      }
      for (int mm = J0; mm < k; ++mm) {
        const double xp = readlane_f64(xp1, mm - J0);
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
  if (mem1) slab.var[P + slab.L * (J0 + l)] = xa1;
  // info.y: decade of the quadrature rule (negative when M/m exceeds the last table)
  if (l == 0) info[gi] = make_int2(ptot, ratio > dec ? -level : level);
}

hipError_t launch_solve_tqb_tail(hipStream_t s, int kp, SolveConsts c, SlabDev slab,
                                 long long g0, int npts, double *ws, int2 *info) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr || (kp != 96 && kp != 128) || c.k <= kp - 62) return hipErrorInvalidValue;
  // (KP = 128 at three waves per SIMD: 168 VGPRs, a few spills outside the step loop; 5.2 ms
  // per 77.6 k-point launch against 5.8 at two.  Loading the back-transform's reflectors three
  // groups ahead instead of one measured 5.8 ms.)
  if (kp == 128)
    hipLaunchKernelGGL((solve_tqb_tail_kernel<128, 64, 3>), dim3(npts), dim3(64), 0, s, c, slab,
                       g0, npts, ws, info);
  else
    hipLaunchKernelGGL((solve_tqb_tail_kernel<96, 32, 2>), dim3(npts), dim3(64), 0, s, c, slab,
                       g0, npts, ws, info);
  return hipGetLastError();
}

}  // namespace cwbl
