// cwbl_tq40.hip — solve_tq40_kernel<KP>: the per-point LETKF solve (letkf_solve,
// module_letkf_core.f90:598-700) from an assembled A, four grid points per wavefront.
//
// assemble_record_kernel (cwbl_tq.hip) stages the point's columns and forms
// A = (k-1)/infl I + Yb Yb^T and b1 = Yb d on the matrix cores, one point per wavefront,
// and writes them to the workspace (AsmRecord).  This kernel runs everything else of the
// algorithm of solve_tq_kernel — the Householder tridiagonalisation A = Q T Q^T (dsytd2
// order) applied on the fly to b1 and x', the T^-1/2 quadrature and the T^-1 solve, the
// back-transform and the RTPP/RTPS epilogue in the reference's fp32 order — with
//
//   one 16-lane DPP row per point (q = lane / 16); lane l holds the FULL rows J0 + l and
//   J0 + 16 + l of A (slots 0, 1; all KP columns) in registers, and lane l < J0 the
//   top-left J0 x J0 block's row l (the prefix block).
//
// Rows 0..J0-1 of A are never held as rows: their entries right of column J0-1 are the
// slots' columns 0..J0-1 (A is symmetric), which the slots' own rank-2 updates keep
// current.  So during the first J0 steps (phase 1):
//   - the pivot column j is register j of every slot row and of the prefix block;
//   - (A v)_i of a prefix row i is its prefix-block part plus the column sum
//     sum_c A(c, i) v_c over the slot rows (one 16-lane reduction per prefix row);
//   - the update of the slots covers columns j+1 .. KP-1, which includes the prefix rows'
//     entries right of the block; the block itself is updated on lanes < J0.
// After J0 steps the trailing (KP-J0)^2 matrix is held as 16-lane rows (phase 2).  Phase 1's
// reflectors go to LDS as they are formed; phase 2's stay in the registers of the column
// they eliminated.  Nothing is written to global memory but the analysis, and the kernel
// spills no registers (244 VGPRs, two waves per SIMD, 19.4 KB of LDS per wave).  Every loop
// over steps, slots and columns is compile-time (sfor), so all register indices are static.
#include "cwbl_device.h"

#include <utility>

namespace cwbl {

namespace {

// Rank-2 updates run in groups of kUG columns, each group's first products before its second
// ones, so no fused FMA reads the accumulator the one before it wrote (the compiler puts an
// s_nop between two inline-asm statements that share a register); the matvec keeps kNA
// partial sums per row (column c -> sum c % kNA).  r6 A/B of the alternatives:
// profiles/r6_tq40_ab.txt.
constexpr int kUG = 8;
constexpr int kNA = 2;
template <int NS>
__device__ __forceinline__ double acc_sum(const double (&pa)[kNA][NS], int r) {
  return pa[0][r] + pa[1][r];
}

// Sum over this lane's 16-lane row, the same value on every lane: two quad_perm stages (two
// v_mov_b32_dpp and a v_add_f64 each: gfx950 has no 64-bit quad_perm), then the four quad
// sums Q0 + Q4 + Q8 + Q12 as one row_newbcast move and three fused v_fmac_f64_dpp (x 1.0,
// one rounding each, as an add): 10 VALU instructions instead of row16_sum's 12.  The quad
// sum is read by DPP two or more wait states after its add (the move's own hazard nop).
__device__ __forceinline__ double rsum16(double v) {
  v += dpp_f64<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
  double s = rbcast<0>(v);
  s = fmac_row<4>(s, v, 1.0);
  s = fmac_row<8>(s, v, 1.0);
  return fmac_row<12>(s, v, 1.0);
}

// Three row sums, stage by stage: each stage's DPP reads come three instructions after the
// adds that feed them, so no wait states are needed between the stages (the same sums, the
// same rounding order as rsum16)
__device__ __forceinline__ void rsum16x3(double &a, double &b, double &c) {
  a += dpp_f64<0xB1>(a);
  b += dpp_f64<0xB1>(b);
  c += dpp_f64<0xB1>(c);
  a += dpp_f64<0x4E>(a);
  b += dpp_f64<0x4E>(b);
  c += dpp_f64<0x4E>(c);
  double sa = rbcast<0>(a), sb = rbcast<0>(b), sc = rbcast<0>(c);
  sa = fmac_row<4>(sa, a, 1.0);
  sb = fmac_row<4>(sb, b, 1.0);
  sc = fmac_row<4>(sc, c, 1.0);
  sa = fmac_row<8>(sa, a, 1.0);
  sb = fmac_row<8>(sb, b, 1.0);
  sc = fmac_row<8>(sc, c, 1.0);
  a = fmac_row<12>(sa, a, 1.0);
  b = fmac_row<12>(sb, b, 1.0);
  c = fmac_row<12>(sc, c, 1.0);
}

// N row sums stage by stage (rsum16x3's interleaving for the prefix rows' column sums; the
// same rounding order as rsum16)
template <int N>
__device__ __forceinline__ void rsum16xN(double (&a)[N]) {
  double s[N];
  sfor<N>([&](auto ii) { a[decltype(ii)::value] += dpp_f64<0xB1>(a[decltype(ii)::value]); });
  sfor<N>([&](auto ii) { a[decltype(ii)::value] += dpp_f64<0x4E>(a[decltype(ii)::value]); });
  sfor<N>([&](auto ii) { s[decltype(ii)::value] = rbcast<0>(a[decltype(ii)::value]); });
  sfor<N>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    s[i] = fmac_row<4>(s[i], a[i], 1.0);
  });
  sfor<N>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    s[i] = fmac_row<8>(s[i], a[i], 1.0);
  });
  sfor<N>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    a[i] = fmac_row<12>(s[i], a[i], 1.0);
  });
}

// STOP = 6 (a timing bound; wrong results): the matvec and rank-2 update skip the 16-column
// blocks right of a slot's rows (trailing column tc >= 16 (r + 1)), i.e. the products a
// lower-triangle layout would not form, with nothing put in their place: what such a layout
// could save at most, before the cross-lane exchange its transposed products need
template <int STOP>
constexpr bool upper_free(int r, int tc) { return STOP == 6 && tc >= 16 * (r + 1); }

}  // namespace

template <int KP>
struct Tq40Smem {
  double pv[4][kTq40J0][KP];  // phase 1's reflectors, column j by row (rows <= j + 1 unused)
  double qs[4][KP];           // per quadrature round: sum over the round's nodes of omega x(row)
  double qz[4][KP + 1];       // T^-1 u2 (slot 7 of the last round); [KP]: other lanes' dump
  double tq[4][KP + 1][4];    // d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
  double tau[4][KP];
};

// STOP > 0: timing-ablation instantiations (CWBL_DEBUG_TQ_STOP = 5: the record loads only,
// 4: after the first J0 steps, 2: after the tridiagonalisation, 3: after the quadrature; var
// is not written), so
// that the production kernel's code is not perturbed by the early exits
template <int KP, int STOP = 0>
__global__ void __launch_bounds__(64, 2)
solve_tq40_kernel(SolveConsts c, SlabDev slab, long long g0, int npts,
                  double *__restrict__ ws, int2 *__restrict__ info) {
  using HO = AsmRecord<KP>;
  constexpr int J0 = kTq40J0;         // steps with the prefix block (phase 1)
  constexpr int KT = KP - J0;         // slot rows J0 + l + 16 r
  constexpr int NS = KT / 16;         // row slots per lane
  constexpr int NV = NS + 1;          // vector slots: 0 = rows l < J0, 1.. = row slots
  constexpr int H = KP / 2;           // rows walked by each side of a twisted solve
  static_assert(KT % 16 == 0 && J0 <= 16 && J0 >= 2 && KP % 2 == 0, "tq40 layout");
  using SM = Tq40Smem<KP>;
  __shared__ SM sm;

  const int lane = threadIdx.x, q = lane >> 4, l = lane & 15;
  // Groups of four points, XCD by XCD like the assembly's points (xcd_remap), each XCD's chunk
  // from its end: the records written last, still in the MALL, are read first
  const int g4 = xcd_remap_rev(blockIdx.x, gridDim.x);
  const int gi = 4 * g4 + q;
  const bool valid = gi < npts;
  const int k = c.k;
  const int ptot = valid ? info[gi].x : 0;
  // record words of this point: SGPR base + 32-bit offset (the host keeps a batch's records
  // below 2^32 bytes).  A lane past the batch reads the spare record npts (the host
  // allocates npts + 1)
  const unsigned wb = (unsigned)(valid ? gi : npts) * (unsigned)HO::WORDS;
  auto w = [&](int i) { return gld(ws, wb + (unsigned)i); };
  auto apk = [](int r, int col) {  // packed lower index of A(r, col)
    return col <= r ? r * (r + 1) / 2 + col : col * (col + 1) / 2 + r;
  };
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

  // fp32 sum over members in member order; member m is row m: prefix slot lane m (m < J0),
  // else row slot (m - J0) / 16, lane (m - J0) % 16.  Every caller's x is +0 on the rows past
  // k, and s + 0 = s (s is never -0), so the rows past k need no mask and each term is one
  // v_add_f32 with a row_newbcast source.
  auto seq_sum_f32 = [&](const float (&x)[NV]) {
    float s = 0.0f;
    sfor<KP>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      constexpr int vs = m < J0 ? 0 : 1 + (m - J0) / 16, ln = m < J0 ? m : (m - J0) % 16;
      s = s + rbcast<ln>(x[vs]);
    });
    return s;
  };
  // ---- background of the point: member i = row i --------------------------------------------
  float xbl[NV];
  double xb_mean;
  {
    sfor<NV>([&](auto vv) {
      constexpr int vs = decltype(vv)::value;
      const int i = vrow(vs);
      const bool mem = valid && i < k;
      const float xv = slab.var[P + slab.L * (mem ? i : 0)];  // branch-free: a valid address
      xbl[vs] = mem ? xv : 0.0f;
    });
    // sum(xb) * nmember_inv (:671)
    xb_mean = (double)(seq_sum_f32(xbl) * c.nmember_inv);
  }

  // ---- A from the record ---------------------------------------------------------------------
  double A[NS][KP];  // slot rows, all columns
  double Pb[J0];     // prefix block row l (lanes >= J0 hold row 0's copy, never used)
  const int lp = l < J0 ? l : 0;
  const bool pre = l < J0;
  double uxP, ubP, ux[NS], ub[NS];
  // A(t, col) of row t = J0 + l + 16 r: packed word tri(t) + col where col <= t, tri(col) + t
  // above.  A column at or left of the slot's first row is in the lower part on every lane, one
  // right of its last row in the upper part: one lane base plus a compile-time offset each,
  // and only the columns inside the slot's row range pick per lane.  The loads go through a
  // buffer resource on the wave's four records (a lane past the batch reads the spare record
  // npts, at most three records on), so the compile-time part of each offset sits in the
  // instruction's offset fields instead of a per-load address computation.  (r6, measured and
  // dropped: staging the records through LDS with coalesced 16-byte loads — equal at best,
  // the per-lane gathers cost latency, not address throughput.)
  const __amdgpu_buffer_rsrc_t rs = rec_rsrc(ws + (size_t)(4 * g4) * HO::WORDS, 4 * HO::WORDS);
  const unsigned rq = (unsigned)(valid ? q : npts - 4 * g4) * (unsigned)HO::WORDS;
  auto rw = [&](unsigned vword, unsigned cword) {  // record word vword + cword (cword static)
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(8u * vword), (int)(8u * cword), 0);
    return __longlong_as_double(((long long)v[1] << 32) | (unsigned)v[0]);
  };
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    constexpr int T0 = J0 + 16 * r, T1 = T0 + 15;  // the slot's rows
    const int t = T0 + l;
    const unsigned lo = rq + (unsigned)(HO::TA + t * (t + 1) / 2), up = rq + (unsigned)(HO::TA + t);
    sfor<KP>([&](auto cc) {
      constexpr int col = decltype(cc)::value;
      constexpr unsigned tc = (unsigned)(col * (col + 1) / 2);
      if constexpr (col <= T0) A[r][col] = rw(lo, col);
      else if constexpr (col > T1) A[r][col] = rw(up, tc);
      else A[r][col] = rw(col <= t ? lo + col : up + tc, 0u);
    });
  });
  {
    const unsigned lo = rq + (unsigned)(HO::TA + lp * (lp + 1) / 2), up = rq + (unsigned)(HO::TA + lp);
    sfor<J0>([&](auto cc) {
      constexpr int col = decltype(cc)::value;
      Pb[col] = rw(col <= lp ? lo + col : up + (unsigned)(col * (col + 1) / 2), 0u);
    });
  }
  {
    const double b = w(HO::U1 + lp);
    ubP = pre ? b : 0.0;
  }
  // x' (fp64, :671-672) and b1 = Yb d; both become Q^T x', Q^T b1
  uxP = pre && l < k ? (double)xbl[0] - xb_mean : 0.0;
  sfor<NS>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    const int t = J0 + l + 16 * r;
    ub[r] = w(HO::U1 + t);
    ux[r] = t < k ? (double)xbl[r + 1] - xb_mean : 0.0;
  });

  if constexpr (STOP == 5) {  // timing ablation: the record loads only (kept live)
    double acc = uxP + ubP;
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      acc += ux[r] + ub[r];
      sfor<KP>([&](auto cc) { acc += A[r][decltype(cc)::value]; });
    });
    sfor<J0>([&](auto cc) { acc += Pb[decltype(cc)::value]; });
    if (valid && l == 0) info[gi] = make_int2(ptot, (int)acc);
    return;
  }
  // dlarfg with fp64 rcp/rsq refined to ~1 ulp; H = I when x = 0 (tau = 0, v = e_j+1)
  struct Refl {
    double beta, tau, scal;
  };
  auto dlarfg = [](double alpha, double xx) {
    const double a2 = fma(alpha, alpha, xx);
    const double rs = rsq64(a2);  // 1/|beta|
    const bool nz = xx > 0.0;
    const double bt = -copysign(a2 * rs, alpha);
    Refl h;
    h.beta = nz ? bt : alpha;
    h.tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
    const double rab = rcp64(alpha - bt);
    h.scal = nz ? rab : 0.0;
    return h;
  };

  // ---- phase 1: Householder steps 0 .. J0-1 with the prefix block -------------------------
  sfor<J0>([&](auto jj) {
    constexpr int j = decltype(jj)::value, J1 = j + 1;
    const double dj = rbcast<j>(Pb[j]);  // A(j,j): final diagonal of T
    // alpha = A(j+1, j): prefix row j+1, or slot 0 lane 0 (row J0) at the last step
    double alpha, u2a, u1a;
    if constexpr (J1 < J0) {
      alpha = rbcast<J1>(Pb[j]);
      u2a = rbcast<J1>(uxP);
      u1a = rbcast<J1>(ubP);
    } else {
      alpha = rbcast<0>(A[0][j]);
      u2a = rbcast<0>(ux[0]);
      u1a = rbcast<0>(ub[0]);
    }
    // x: column j below row j + 1 (rows < k)
    const double xP = (pre && l > J1 && l < k) ? Pb[j] : 0.0;
    double x[NS];
    double xx = xP * xP, xu = xP * uxP, xb = xP * ubP;
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      const int i = J0 + l + 16 * r;
      x[r] = (i > J1 && i < k) ? A[r][j] : 0.0;
      xx = fma(x[r], x[r], xx);
      xu = fma(x[r], ux[r], xu);
      xb = fma(x[r], ub[r], xb);
    });
    rsum16x3(xx, xu, xb);
    // x_c of column c, wave-uniform per row: prefix lane c (c < J0) or its slot lane; the
    // products with it are one fmac_row each (acc + x_c y)
    auto src_of = [&](auto cc, const double &vp, const double (&vs)[NS]) -> const double & {
      constexpr int col = decltype(cc)::value;
      if constexpr (col < J0) return vp;
      else return vs[(col - J0) / 16];
    };
    auto lane_of = [](int col) { return col < J0 ? col : (col - J0) % 16; };
    const Refl h = dlarfg(alpha, xx);
    // every lane of the row writes the same value (no divergent branch in the step)
    sm.tq[q][j][0] = dj;
    sm.tq[q][J1][1] = h.beta;
    sm.tau[q][j] = h.tau;
    const double tau = h.tau;
    // v: 1 at row j + 1, x * scal below; the reflector stays in column j's registers
    const double xsP = xP * h.scal;
    double vP = (pre && l == J1) ? 1.0 : xsP;
    double v[NS];
    // the reflector is final: it goes to LDS until the back-transform, and column j's
    // registers are dead from here on
    sm.pv[q][j][pre ? l : 0] = xsP;  // lanes >= J0: 0 into row 0, which no reflector uses
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      const double xs = x[r] * h.scal;
      if constexpr (J1 == J0 && r == 0) v[r] = l == 0 ? 1.0 : xs;
      else v[r] = xs;
      sm.pv[q][j][J0 + l + 16 * r] = xs;
    });
    const double s2 = fma(h.scal, xu, u2a);  // v . x'
    const double s3 = fma(h.scal, xb, u1a);  // v . b1
    uxP = fma(-tau * s2, vP, uxP);
    ubP = fma(-tau * s3, vP, ubP);
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      ux[r] = fma(-tau * s2, v[r], ux[r]);
      ub[r] = fma(-tau * s3, v[r], ub[r]);
    });
    dpp_pin(vP);
    sfor<NS>([&](auto rr) { dpp_pin(v[decltype(rr)::value]); });
    // A v: slot rows over columns j+1 .. KP-1; prefix rows = their block part + the column
    // sums over the slot rows (A(i, c) = A(c, i) for c >= J0)
    double pa[kNA][NS], pP = 0.0;
    sfor<kNA * NS>([&](auto ii) { pa[decltype(ii)::value / NS][decltype(ii)::value % NS] = 0.0; });
    sfor<KP - J1>([&](auto cc) {
      constexpr int col = J1 + decltype(cc)::value;
      constexpr int LC = lane_of(col);
      const double &vs = src_of(std::integral_constant<int, col>{}, vP, v);
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        constexpr int a = (col - J1) % kNA;
        if constexpr (!upper_free<STOP>(r, col - J0)) pa[a][r] = fmac_row<LC>(pa[a][r], vs, A[r][col]);
      });
      if constexpr (col < J0) pP = fmac_row<LC>(pP, vs, Pb[col]);
    });
    if constexpr (J1 < J0) {  // prefix rows j+1 .. J0-1: column sums of the slots
      // (in chunks of up to three: seven sums at once spill)
      constexpr int NC = J0 - J1, CH = 3;
      sfor<(NC + CH - 1) / CH>([&](auto kk) {
        constexpr int c0 = J1 + CH * decltype(kk)::value;
        constexpr int n = J0 - c0 < CH ? J0 - c0 : CH;
        double cs[n];
        sfor<n>([&](auto cc) {
          constexpr int col = c0 + decltype(cc)::value;
          double s = 0.0;
          sfor<NS>([&](auto rr) {
            constexpr int r = decltype(rr)::value;
            s = fma(A[r][col], v[r], s);
          });
          cs[decltype(cc)::value] = s;
        });
        rsum16xN(cs);
        sfor<n>([&](auto cc) {
          constexpr int col = c0 + decltype(cc)::value;
          pP += l == col ? cs[decltype(cc)::value] : 0.0;
        });
      });
    }
    double pp[NS];
    double sp = vP * pP;  // rows <= j: v = 0
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      pp[r] = acc_sum(pa, r);
      sp = fma(v[r], pp[r], sp);
    });
    const double s1 = tau * rsum16(sp);  // v^T (tau A v)
    // w on the rows <= j (and lanes >= J0) is not zeroed: it only updates those rows' own
    // entries, which nothing reads again (their w is never a broadcast source: the update
    // runs over columns > j)
    const double wP = fma(-0.5 * tau * s1, vP, tau * pP);
    double wv[NS];
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      wv[r] = fma(-0.5 * tau * s1, v[r], tau * pp[r]);
    });
    // A <- A - v w^T - w v^T: slot rows over columns j+1 .. KP-1, the prefix block over
    // columns j+1 .. J0-1.  (v is renamed first: otherwise the compiler reuses the matvec's
    // broadcasts and keeps all KP - j of them live across the reduction, which spills.)
    double wPp = wP;
    dpp_pin(wPp);
    sfor<NS>([&](auto rr) { dpp_pin(wv[decltype(rr)::value]); });
    // Columns go in pairs, each pair's first products before its second ones, so that no
    // fmac reads the accumulator the fmac just before it wrote (the compiler puts an s_nop
    // between two inline-asm statements that share a register)
    sfor<(KP - J1 + kUG - 1) / kUG>([&](auto pp) {
      constexpr int c0 = J1 + kUG * decltype(pp)::value;
      sfor<2>([&](auto hh) {  // hh = 0: A - wv v_c; hh = 1: - v w_c (the reference's order)
        constexpr int h = decltype(hh)::value;
        sfor<kUG>([&](auto ee) {
          constexpr int col = c0 + decltype(ee)::value;
          if constexpr (col < KP) {
            constexpr int LC = lane_of(col);
            const double &vs = src_of(std::integral_constant<int, col>{}, vP, v);
            const double &ws = src_of(std::integral_constant<int, col>{}, wPp, wv);
            sfor<NS>([&](auto rr) {
              constexpr int r = decltype(rr)::value;
              if constexpr (upper_free<STOP>(r, col - J0)) {
              } else if constexpr (h == 0) A[r][col] = fnmac_row<LC>(A[r][col], vs, wv[r]);
              else A[r][col] = fnmac_row<LC>(A[r][col], ws, v[r]);
            });
            if constexpr (col < J0) {
              if constexpr (h == 0) Pb[col] = fnmac_row<LC>(Pb[col], vs, wPp);
              else Pb[col] = fnmac_row<LC>(Pb[col], ws, vP);
            }
          }
        });
      });
    });
  });
  // a (one-wave) workgroup barrier: a fence the scheduler does not move phase 2 across
  __syncthreads();
  // the prefix rows of Q^T b1, Q^T x' are final (later reflectors vanish there)
  if (pre) {
    sm.tq[q][l][2] = ubP;
    sm.tq[q][l][3] = uxP;
  }

  if constexpr (STOP == 4) {  // timing ablation: phase 1 only
    if (valid && l == 0) info[gi] = make_int2(ptot, (int)(uxP + A[1][KP - 1]));
    return;
  }
  // ---- phase 2: steps J0 .. KP-3 on the trailing rows (solve_tq4_kernel's step) -----------
  // Steps j >= k - 2 (k < KP) are exact no-ops: the padding rows and columns of A are the
  // identity, so x = 0 there, tau = 0 and beta = A(j+1,j); running them keeps the code
  // branch-free.
  sfor<KT>([&](auto jj) {
    constexpr int jl = decltype(jj)::value, j = J0 + jl;
    constexpr int RJ = jl / 16, LJ = jl % 16;
    const double dj = rbcast<LJ>(A[RJ][j]);  // A(j,j): final diagonal of T
    if constexpr (jl + 2 < KT) {
      constexpr int J1 = jl + 1, R1 = J1 / 16, L1 = J1 % 16;
      const double alpha = rbcast<L1>(A[R1][j]);
      double x[NS], xx = 0.0, xu = 0.0, xb = 0.0;
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        if constexpr (16 * r + 15 > J1) {
          const int i = J0 + l + 16 * r;
          x[r] = (i > j + 1 && i < k) ? A[r][j] : 0.0;
          xx = fma(x[r], x[r], xx);
          xu = fma(x[r], ux[r], xu);
          xb = fma(x[r], ub[r], xb);
        } else {
          x[r] = 0.0;
        }
      });
      rsum16x3(xx, xu, xb);
      const Refl h = dlarfg(alpha, xx);
      const double tau = h.tau;
      sm.tq[q][j][0] = dj;
      sm.tq[q][j + 1][1] = h.beta;
      sm.tau[q][j] = tau;
      double v[NS];
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        const int t = l + 16 * r;
        const double xs = x[r] * h.scal;
        v[r] = t == J1 ? 1.0 : xs;
        if constexpr (16 * r + 15 > J1) A[r][j] = xs;  // the reflector, rows > j + 1
      });
      const double s2 = fma(h.scal, xu, rbcast<L1>(ux[R1]));  // v . x'
      const double s3 = fma(h.scal, xb, rbcast<L1>(ub[R1]));  // v . b1
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        ux[r] = fma(-tau * s2, v[r], ux[r]);
        ub[r] = fma(-tau * s3, v[r], ub[r]);
      });
      // A v over the trailing columns (v vanishes at columns <= j), column by column so
      // that one broadcast v_c is live at a time
      double pa[kNA][NS];
      sfor<kNA * NS>([&](auto ii) { pa[decltype(ii)::value / NS][decltype(ii)::value % NS] = 0.0; });
      sfor<NS>([&](auto rr) { dpp_pin(v[decltype(rr)::value]); });
      sfor<KT - J1>([&](auto cc) {
        constexpr int cl = J1 + decltype(cc)::value;
        sfor<NS>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          if constexpr (16 * r + 15 > jl && !upper_free<STOP>(r, cl)) {
            constexpr int a = (cl - J1) % kNA;
            pa[a][r] = fmac_row<cl % 16>(pa[a][r], v[cl / 16], A[r][J0 + cl]);
          }
        });
      });
      double pp[NS], sp = 0.0;
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        pp[r] = acc_sum(pa, r);
        if constexpr (16 * r + 15 > jl) sp = fma(v[r], pp[r], sp);  // rows <= j: v = 0
      });
      const double s1 = tau * rsum16(sp);  // v^T (tau A v)
      double wv[NS];
      sfor<NS>([&](auto rr) {
        constexpr int r = decltype(rr)::value;
        const int t = l + 16 * r;
        (void)t;  // rows <= j: as in phase 1
        wv[r] = fma(-0.5 * tau * s1, v[r], tau * pp[r]);
      });
      // A <- A - v w^T - w v^T on the trailing rows and columns
      sfor<NS>([&](auto rr) { dpp_pin(wv[decltype(rr)::value]); });
      // column pairs, first products before second ones (as in phase 1)
      sfor<(KT - J1 + kUG - 1) / kUG>([&](auto pp) {
        constexpr int c0 = J1 + kUG * decltype(pp)::value;
        sfor<2>([&](auto hh) {
          constexpr int h = decltype(hh)::value;
          sfor<kUG>([&](auto ee) {
            constexpr int cl = c0 + decltype(ee)::value;
            if constexpr (cl < KT) {
              sfor<NS>([&](auto rr) {
                constexpr int r = decltype(rr)::value;
                if constexpr (16 * r + 15 > jl && !upper_free<STOP>(r, cl)) {
                  if constexpr (h == 0)
                    A[r][J0 + cl] = fnmac_row<cl % 16>(A[r][J0 + cl], v[cl / 16], wv[r]);
                  else
                    A[r][J0 + cl] = fnmac_row<cl % 16>(A[r][J0 + cl], wv[cl / 16], v[r]);
                }
              });
            }
          });
        });
      });
    } else {  // the trailing 2x2: already tridiagonal (c(KP-2,KP-3) is step KP-3's beta)
      const double ej = rbcast<LJ>(A[RJ][j - 1]);
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
  // trace of T (= trace of A) over the members, from the diagonal in LDS: summed here, not
  // step by step, so that no step's d_j stays live to the end
  double trace;
  {
    double tp = 0.0;
    sfor<(KP + 15) / 16>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      const int i = l + 16 * r;
      if (16 * r + 15 < KP || i < KP) tp += i < k ? sm.tq[q][i < KP ? i : 0][0] : 0.0;
    });
    trace = rsum16(tp);
  }

  if constexpr (STOP == 2) {  // timing ablation: tridiagonalisation only
    if (valid && l == 0) info[gi] = make_int2(ptot, (int)(trace + ux[1]));
    return;
  }
  // ---- T^-1/2 u2 by quadrature, T^-1 u2 exactly --------------------------------------------
  // lambda^-1/2 = (2/pi) int_0^inf dt / (t^2 + lambda) with the elliptic substitution and
  // the midpoint rule on the spectrum bound [m, M] (solve_tq_kernel, cwbl_tq.hip): each node
  // is one shifted SPD tridiagonal solve, twisted: lane l & 7 is the node of the round,
  // side l >> 3 walks rows 0..H-1 (top) or KP-1..H (bottom); slot 7 of the last round solves
  // T^-1 u2.  Each row's sum over the round's 8 nodes is an 8-lane DPP reduction; its lane 0
  // hands it to the row's owner through LDS.
  const double m = (double)c.inflat;
  const double ratio = trace / m - (double)(k - 1);
  int level = 1;
  double dec = 10.0;
  while (level < kQuadLevels && dec < ratio) {
    dec *= 10.0;
    ++level;
  }
  // rounds of 8 nodes: the wave's largest need (quad_rounds) over its four points, with the
  // (8 R - 1)-node rule of each point's own level; slot 7 of the last round is T^-1 u2
  const int rp = quad_rounds(level);
  const int R = __ballot(rp == 8) ? 8 : __ballot(rp == 4) ? 4 : __ballot(rp == 3) ? 3 : 2;
  const int NQ = 8 * R - 1;  // (R is wave-uniform)
  const double2 *qtab = quad_rule(c.quad_r, R, level);
  const int side = l >> 3, n8 = l & 7;
  const double(*T)[4] = sm.tq[q];
  // LDS byte offsets, walked one row per step through a register the compiler cannot see
  // through (asm): computed addresses of every row would be loop-invariant, and hoisting
  // them out of the round loop holds ~40 VGPRs
  char *const smb = reinterpret_cast<char *>(&sm);
  auto lds = [&](unsigned off) { return *reinterpret_cast<const double *>(smb + off); };
  auto sts = [&](unsigned off, double v) { *reinterpret_cast<double *>(smb + off) = v; };
  const unsigned tq0 = (unsigned)(offsetof(SM, tq) + (size_t)q * sizeof(sm.tq[0])) +
                       (side ? (KP - 1) * 32u : 0u);   // row 0 of the walk
  const unsigned dirb = side ? (unsigned)-32 : 32u;   // next row of the walk
  const unsigned csb = side ? 40u : 8u;  // coupling with the previous row of the walk
  const unsigned qs0 = (unsigned)(offsetof(SM, qs) + (size_t)q * sizeof(sm.qs[0])) +
                       (side ? (KP - H) * 8u : (H - 1) * 8u);  // row H-1 of the walk
  const unsigned qz0 = (unsigned)(offsetof(SM, qz) + (size_t)q * sizeof(sm.qz[0]));
  const unsigned bdir = side ? 8u : (unsigned)-8;    // back-substitution: previous row
  double ys[NV], z[NV];
  sfor<NV>([&](auto vv) { ys[decltype(vv)::value] = 0.0; });
  for (int round = 0; round < R; ++round) {
    const int node = 8 * round + n8;
    const double2 tw = qtab[min(node, NQ - 1)];
    const double sigma = node < NQ ? m * tw.x : 0.0;
    const double omega = node < NQ ? sqrt(m) * tw.y : 1.0;
    double hh[H], mm[H];
    unsigned pw = tq0;
    double dl = lds(pw) + sigma, gt = lds(pw + 24);
    double rdl = rcp64(dl);
    sfor<H - 1>([&](auto tt) {
      constexpr int t = decltype(tt)::value + 1;
      pw += dirb;
      asm volatile("" : "+v"(pw) : "v"(dl));  // row t is read once d_{t-1} is known
      const double ct = lds(pw + csb);
      const double lt = ct * rdl;
      hh[t - 1] = gt * rdl;
      mm[t - 1] = lt;
      dl = fma(-lt, ct, lds(pw) + sigma);
      gt = fma(-lt, gt, lds(pw + 24));
      rdl = rcp64(dl);
    });
    // rows H-1 (top) and H (bottom): 2x2 solve with the partner lane's pivot
    const double cm = T[H][1];
    const double dlo = ror8(dl), go = ror8(gt);
    double xv = (gt * dlo - cm * go) / fma(dl, dlo, -cm * cm);
    const bool last = round == R - 1;
    const bool zlane = last && n8 == 7;  // T^-1 u2: not a node of the sum
    const double om = zlane ? 0.0 : omega;
    unsigned ps = qs0;                          // qs of the walk's current row
    unsigned pz = qz0 + (zlane ? qs0 - (unsigned)offsetof(SM, qs) - (unsigned)q * KP * 8u
                               : KP * 8u);     // qz of that row, or the dump word
    const unsigned zdir = zlane ? bdir : 0u;
    auto emit = [&](double x) {
      double s = om * x;
      s += dpp_f64<0xB1>(s);   // quad_perm [1,0,3,2]
      s += dpp_f64<0x4E>(s);   // quad_perm [2,3,0,1]
      s += dpp_f64<0x141>(s);  // row_half_mirror: the 8 lanes of the side
      // stores without branches: the side's 8 lanes store the same sum
      sts(ps, s);
      sts(pz, x);
    };
    emit(xv);
    sfor<H - 1>([&](auto tt) {
      constexpr int t = H - 2 - decltype(tt)::value;
      xv = fma(-mm[t], xv, hh[t]);
      ps += bdir;
      pz += zdir;
      asm volatile("" : "+v"(ps), "+v"(pz) : "v"(xv));
      emit(xv);
    });
    __syncthreads();
    sfor<NV>([&](auto vv) {
      constexpr int vs = decltype(vv)::value;
      const int i = vrow(vs);
      const int ic = i < KP ? i : 0;
      ys[vs] += i < KP ? sm.qs[q][ic] : 0.0;
      if (last) z[vs] = i < KP ? sm.qz[q][ic] : 0.0;
    });
    __syncthreads();
  }
  double dpart = 0.0;  // u1 . T^-1 u2 = wbar . x'
  sfor<NV>([&](auto vv) {
    constexpr int vs = decltype(vv)::value;
    const int i = vrow(vs);
    const double u1 = vs == 0 ? ubP : ub[vs > 0 ? vs - 1 : 0];
    dpart = i < KP ? fma(u1, z[vs], dpart) : dpart;
  });
  const double d = rsum16(dpart);
  if constexpr (STOP == 3) {  // timing ablation: up to the quadrature
    if (valid && l == 0) info[gi] = make_int2(ptot, (int)(d + ys[0] + ys[1] + ys[2]));
    return;
  }

  // ---- back-transform: y <- Q y = H_0 H_1 ... H_{KP-3} y ----------------------------------
  double y[NV];
  sfor<NV>([&](auto vv) { y[decltype(vv)::value] = ys[decltype(vv)::value]; });
  sfor<KT - 2>([&](auto jj) {  // phase 2's reflectors (rows > J0 only)
    constexpr int jl = KT - 3 - decltype(jj)::value, j = J0 + jl, J1 = jl + 1;
    const double tj = sm.tau[q][j];
    double vv[NS], a = 0.0;
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      if constexpr (16 * r + 15 >= J1) {
        const int t = l + 16 * r;
        // column j's registers hold x * scal, which is 0 on the rows <= j + 1 (x is), in the
        // slots that step j wrote (16 r + 15 > J1): the reflector is 1 at row j + 1 and the
        // register elsewhere
        if constexpr (16 * r + 15 > J1) vv[r] = t == J1 ? 1.0 : A[r][j];
        else vv[r] = t == J1 ? 1.0 : 0.0;
        a = fma(vv[r], y[r + 1], a);
      } else {
        vv[r] = 0.0;
      }
    });
    a = rsum16(a);
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      if constexpr (16 * r + 15 >= J1) y[r + 1] = fma(-tj * a, vv[r], y[r + 1]);
    });
  });
  sfor<J0>([&](auto jj) {  // phase 1's reflectors: prefix register j and slot column j
    constexpr int j = J0 - 1 - decltype(jj)::value, J1 = j + 1;
    const double tj = sm.tau[q][j];
    const double *pj = sm.pv[q][j];
    const double v0 = l == J1 ? 1.0 : (pre && l > J1) ? pj[lp] : 0.0;  // 0 at rows <= j + 1
    double vv[NS];
    double a = v0 * y[0];
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      const double pr = pj[J0 + l + 16 * r];
      if constexpr (J1 == J0 && r == 0) vv[r] = l == 0 ? 1.0 : pr;
      else vv[r] = pr;
      a = fma(vv[r], y[r + 1], a);
    });
    a = rsum16(a);
    y[0] = fma(-tj * a, v0, y[0]);
    sfor<NS>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      y[r + 1] = fma(-tj * a, vv[r], y[r + 1]);
    });
  });

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

hipError_t launch_solve_tq40(hipStream_t s, int kp, SolveConsts c, SlabDev slab, long long g0,
                             int npts, double *ws, int2 *info) {
  if (npts <= 0) return hipSuccess;
  if (c.quad_r == nullptr || kp != kTq4KP) return hipErrorInvalidValue;
  const dim3 grid((npts + 3) / 4);
#ifdef CWBL_DEBUG_KNOBS  // timing-ablation instantiations (make DEBUG_KNOBS=1)
  switch (c.debug_stop) {
    case 2: hipLaunchKernelGGL((solve_tq40_kernel<kTq4KP, 2>), grid, dim3(64), 0, s, c, slab, g0, npts, ws, info); return hipGetLastError();
    case 3: hipLaunchKernelGGL((solve_tq40_kernel<kTq4KP, 3>), grid, dim3(64), 0, s, c, slab, g0, npts, ws, info); return hipGetLastError();
    case 4: hipLaunchKernelGGL((solve_tq40_kernel<kTq4KP, 4>), grid, dim3(64), 0, s, c, slab, g0, npts, ws, info); return hipGetLastError();
    case 5: hipLaunchKernelGGL((solve_tq40_kernel<kTq4KP, 5>), grid, dim3(64), 0, s, c, slab, g0, npts, ws, info); return hipGetLastError();
    case 6: hipLaunchKernelGGL((solve_tq40_kernel<kTq4KP, 6>), grid, dim3(64), 0, s, c, slab, g0, npts, ws, info); return hipGetLastError();
    default: break;
  }
#endif
  hipLaunchKernelGGL((solve_tq40_kernel<kTq4KP>), grid, dim3(64), 0, s, c, slab, g0, npts, ws, info);
  return hipGetLastError();
}

}  // namespace cwbl
