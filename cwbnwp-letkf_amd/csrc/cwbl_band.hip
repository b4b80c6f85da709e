// cwbl_band.hip — the two-stage solve for large ensembles (configs[3], k = 97..128, KP = 128):
// letkf_solve (module_letkf_core.f90:598-700) with the eigendecomposition of
// A = (k-1)/infl I + Yb Yb^T (module_eigen.f90:48-56, dsyevd) replaced, as in every tq
// kernel, by an orthogonal reduction A = Q T Q^T to tridiagonal form and a quadrature for
// T^-1/2 — here in two stages, so that the reduction's sequential chain is short:
//
//   band_head_kernel (256 threads per point): stages the columns, assembles A and b1 = Yb d on
//     the matrix cores (v_mfma_f64_16x16x4_f64), and reduces A to a band of half-bandwidth
//     b = 8 with 15 panel block reflectors Q_p = I - V_p T_p V_p^T.  Wave w holds the 16x16
//     tiles of the two tile COLUMNS w and 7 - w of the full symmetric A in its accumulator
//     registers.  A panel (8 columns) is QR-factorised in place by the wave that holds it
//     (dgeqr2 order, DPP broadcasts inside a 16-lane row, no workgroup barrier), and the
//     two-sided trailing update A22 <- Q_p^T A22 Q_p = A22 - V Z^T - Z V^T,
//     W = A22 V T, Z = W - 1/2 V (T^T V^T W), runs on the matrix cores (the tiles are the
//     accumulators, V and Z the operands): three workgroup barriers per panel instead of five
//     per Householder step.  Q_p^T is applied to b1 and x' as the panels go.  The band, the
//     panels' V and T and Q1^T b1, Q1^T x' go to the workspace (BandRec).
//   band_tail_kernel (one wavefront per point): chases the band to tridiagonal form (1056
//     Householder reflectors of length <= 8, two sweeps in flight three tasks apart, each task
//     on 32 lanes: the reflector's left block, diagonal block, the bulge below it and Q2^T on
//     b1, x' as one instruction stream), the band in LDS (row i holds A(i, i-d), d = 0..15),
//     then the T^-1/2 quadrature of the tail kernel, the back-transform y <- Q1 Q2 y (chase
//     reflectors sweep by sweep, then the 15 panels) and the RTPP/RTPS epilogue in the
//     reference's fp32 order.
//
// On gfx950 this path is slower than the hand-off path (the FP64 matrix
// rate equals the vector rate, so the GEMM form buys no rate while doing twice dsytd2's flops,
// and the panel QR is a serial chain); it is CWBL_OPT_BIG_PATH = 2, not the default.
//
// The design is checked step for step by scripts/two_stage_b8.py (numpy; the same panels,
// schedule, storage bounds and application orders).  Padding rows (k < 128) are identity rows
// of A: their panel reflectors and chase reflectors are exact no-ops (tau = 0).
#include "cwbl_band.h"

namespace cwbl {

// ==== stage 1: assembly + band reduction ====================================================
constexpr int kBandChunk = 64;
struct BandHeadSmem {
  union {
    ColumnChunk<128, kBandChunk, float, 128, false, true> ch[2];  // staging (stage_columns_pipe)
    double mir[28][16 * 17];      // lower off-diagonal tiles, for the upper ones (transposed)
    struct {
      double V[2][128][8];        // panel reflectors, row rho - r0 (double buffer by panel)
      double Z[128][8];
      double M[4][64];            // per-wave partial V^T W
      double T[64];               // T[a * 8 + b]
      double u[2][128];           // Q^T b1, Q^T x' so far
    } s;
  } u;
  float parf;
  int ptot;
};

// the mirror slot of lower tile (J, I), J > I
__device__ __forceinline__ int mir_slot(int J, int I) { return J * (J - 1) / 2 + I; }

template <bool ASSEMBLED>
__global__ void __launch_bounds__(256, 2)
band_head_kernel(const TreeDesc *__restrict__ trees, SolveConsts c, SlabDev slab, long long g0,
                 int npts, const int *__restrict__ nbr_cnt, const int *__restrict__ nbr_idx,
                 int2 *__restrict__ info, double *__restrict__ ws) {
  constexpr int KP = 128, NT = 256;
  using HR = BandRec;
  __shared__ BandHeadSmem sm;
  static_assert(!ASSEMBLED, "slab path only");

  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k = c.k;
  const int m16 = lane & 15, kk = lane >> 4;  // C/D: column m16, rows kk + 4 r
  double *__restrict__ rec = ws + (long long)gi * HR::WORDS;

  long long P = 0;
  float3 pt = make_float3(0.0f, 0.0f, 0.0f);
  float xbl = 0.0f;  // background of member `tid`
  {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long r = g / slab.ix_lim;
    const int j = (int)(r % slab.iy_lim);
    const int kz = (int)(r / slab.iy_lim);
    P = i + (long long)slab.nx * (j + (long long)slab.ny * kz);
    if (tid < k) xbl = slab.var[P + slab.L * tid];
    slab_point(slab, g, pt.x, pt.y, pt.z);
  }

  // ---- matrix-core assembly: lower tiles (J, I), J >= I, of the wave's columns I0, I1 ------
  // tile9[t]: t < 8 - w: (J = w + t, I = w); t >= 8 - w: (J = 7 - w + t - (8 - w), I = 7 - w)
  const int I0 = wave, I1 = 7 - wave;
  constexpr int NTW = 9;
  f64x4 tile9[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) tile9[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  double b1p[4] = {0.0, 0.0, 0.0, 0.0};
  using CC = std::remove_reference_t<decltype(sm.u.ch[0])>;
  const int xk = CC::xr(kk);
  int offJx[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int J = t < 8 - wave ? wave + t : 7 - wave + (t - (8 - wave));
    offJx[t] = (16 * J + m16) ^ xk;
  }
  const int offB0 = (16 * I0 + m16) ^ xk, offB1 = (16 * I1 + m16) ^ xk;
  auto mfma_chunk = [&](int nsl, const CC &cb) {
    for (int s0 = 0; s0 < nsl; s0 += 4) {
      const float *ys = cb.yb[s0 + kk];
      const double b0 = (double)ys[offB0], bb1 = (double)ys[offB1];
#pragma unroll
      for (int t = 0; t < NTW; ++t)
        tile9[t] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)ys[offJx[t]],
                                                         t < 8 - wave ? b0 : bb1, tile9[t], 0, 0, 0);
    }
    // Yb d: eight columns per round, four chains (the staged columns past nsl are zeros)
    if (tid < KP) {
      const int nr = (nsl + 7) / 8;
      for (int r8 = 0; r8 < nr; ++r8) {
        const float4 o0 = *reinterpret_cast<const float4 *>(&cb.yo[8 * r8]);
        const float4 o1 = *reinterpret_cast<const float4 *>(&cb.yo[8 * r8 + 4]);
        const float o[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
        float y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = cb.at(8 * r8 + i, tid);
#pragma unroll
        for (int i = 0; i < 8; ++i) b1p[i & 3] = fma((double)y[i], (double)o[i], b1p[i & 3]);
      }
    }
  };
  int ptot = stage_columns_pipe<KP, kBandChunk, NT>(sm.u.ch, trees, c, gi, tid, nbr_cnt,
                                                    nbr_idx, pt, mfma_chunk);
  const double b1acc = (b1p[0] + b1p[1]) + (b1p[2] + b1p[3]);
  if (tid == 0) sm.ptot = ptot;  // counted by wave 0
  __syncthreads();
  ptot = sm.ptot;
  if (ptot == 0) {  // no accepted observation: var left unchanged (:220, :226)
    if (tid == 0) info[gi] = make_int2(0, 0);
    return;
  }
  // inflat on the diagonal (padding rows: 1), diagonal tiles t = 0 (I0) and t = 8 - w (I1)
  {
    const double inf = (double)c.inflat;
    auto diag = [&](f64x4 &tl, int I) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int a = kk + 4 * r;
        if (a == m16) tl[r] = 16 * I + a < k ? tl[r] + inf : 1.0;
      }
    };
    diag(tile9[0], I0);
    // (selects, not branches on t: see pick below)
    sfor<NTW - 1>([&](auto tt) {
      constexpr int t = decltype(tt)::value + 1;
      f64x4 d = tile9[t];
      diag(d, I1);
      const bool on = t == 8 - wave;
#pragma unroll
      for (int r = 0; r < 4; ++r) tile9[t][r] = on ? d[r] + 0.0 : tile9[t][r] + 0.0;
    });
  }

  // ---- the full symmetric A: upper tiles as transposes of the lower ones, through LDS -----
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int I = t < 8 - wave ? I0 : I1;
    const int J = t < 8 - wave ? wave + t : 7 - wave + (t - (8 - wave));
    if (J > I) {
      double *d = sm.u.mir[mir_slot(J, I)];
#pragma unroll
      for (int r = 0; r < 4; ++r) d[(kk + 4 * r) * 17 + m16] = tile9[t][r];
    }
  }
  __syncthreads();
  // tile[s * 8 + J] = A(rows 16J + kk + 4r, columns 16 I_s + m16), I_0 = w, I_1 = 7 - w
  // (value selects throughout: per-wave branches that each copy a different tile get merged
  // into one copy through a pointer phi, which moves the tiles to scratch memory)
  f64x4 tile[16];
  sfor<16>([&](auto tt) {
    constexpr int t = decltype(tt)::value, J = t & 7;
    const int I = t < 8 ? I0 : I1;
    // (J, I), J >= I, from tile9: slot 0 at t9 = J - w, slot 1 at t9 = J + 1
    f64x4 own;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (t < 8) {
        long long bits = 0;
        sfor<4>([&](auto WW) {
          constexpr int W = decltype(WW)::value;
          if constexpr (J >= W) bits |= __double_as_longlong(tile9[J - W][r]) & -(long long)(wave == W);
        });
        own[r] = __longlong_as_double(bits);
      } else {
        own[r] = tile9[J + 1][r];
      }
    }
    // (J, I) = (I, J)^T for J < I: element (a, b) of (J, I) is (b, a) of (I, J)
    const double *s = sm.u.mir[J < I ? mir_slot(I, J) : 0];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double mv = s[m16 * 17 + kk + 4 * r];
      tile[t][r] = J >= I ? own[r] + 0.0 : mv + 0.0;
    }
  });
  // x' and b1 (fp64); xb_mean in the reference's sequential fp32 order (:671)
  float xbm;
  {
    for (int w = 0; 64 * w < k; ++w) {
      if (wave == w) {
        float s = w == 0 ? 0.0f : sm.parf;
        const int n = min(64, k - 64 * w);
        for (int mm = 0; mm < n; ++mm)
          s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xbl), mm));
        if (lane == 0) sm.parf = s;
      }
      __syncthreads();
    }
    xbm = sm.parf;
  }
  __syncthreads();  // the mirror area is read; stage 1's buffers take it over
  const double xb_mean = (double)(xbm * c.nmember_inv);
  if (tid < KP) {
    sm.u.s.u[0][tid] = b1acc;
    sm.u.s.u[1][tid] = tid < k ? (double)xbl - xb_mean : 0.0;
  }

  if (CWBL_DBG_STOP(c) == 1) {  // timing ablation: assembly only (keeps the tiles live)
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < 16; ++t) acc += (tile[t][0] + tile[t][1]) + (tile[t][2] + tile[t][3]);
    rec[HR::BAND + tid] = acc;
    if (tid == 0) info[gi] = make_int2(ptot, 0);
    return;
  }
  // ---- stage 1: 15 panels of 8 columns -------------------------------------------------------
  // the band row i of the record: A(i, i - d), d = 0..8
  auto band_st = [&](int i, int d, double v) { rec[HR::BAND + i * (HR::B + 1) + d] = v; };
  for (int p = 0; p < HR::NP; ++p) {
    const int Q = p >> 1, h = p & 1, r0 = 8 * p + 8, q0 = Q + h;
    const int owner = Q < 4 ? Q : 7 - Q;
    double(*Vb)[8] = sm.u.s.V[p & 1];  // (double buffer: slower waves may still read the last V)
    // (no barrier here: T, Z and M of the previous panel were last read before its barrier B3,
    // and a wave reaches this panel's B1 only after its part of the previous update)
    if (wave == owner && CWBL_DBG_STOP(c) != 5) {  // (5: timing ablation without the QRs)
      // -- the panel QR, in place in tile column Q, columns 8H .. 8H + 7 -----------------------
      // The QR runs on slot 0's registers: a wave whose panel lies in its second tile column
      // swaps its two slots around it (the tile order of the rest is per slot, so only the QR
      // needs to know).
      const bool swp = Q != I0;
      auto swap_slots = [&]() {
        sfor<8>([&](auto JJ) {
          constexpr int J = decltype(JJ)::value;
          const f64x4 t0 = tile[J];
          tile[J] = tile[8 + J];
          tile[8 + J] = t0;
        });
      };
      if (swp) swap_slots();
      // tile (j, Q) of slot 0 by value: bit masks, not branches — branches that each touch a
      // different tile get merged into one access through a pointer phi, and that sends the
      // whole slot to scratch memory
      auto pick = [&](int j) {
        f64x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          long long bits = 0;
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            bits |= __double_as_longlong(tile[J][r]) & -(long long)(j == J);
          });
          o[r] = __longlong_as_double(bits);
        }
        return o;
      };
      auto qr = [&](auto H_) {
        constexpr int H = decltype(H_)::value;
        constexpr int C0 = 8 * H;
        // the pivot tile (q0, Q): the panel's rows r0 - 8 + 8H .. ; the QR changes only the
        // panel's columns, which no later step reads, so neither it nor the tiles below it are
        // written back
        f64x4 tq = pick(q0);
        // band: the diagonal block D_p (rows 8p + a, columns 8p + b, b <= a): tile (Q, Q),
        // rows C0 + a (kk + 4r), columns C0 + b (m16)
        {
          const f64x4 td = H == 0 ? tq : pick(Q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int a = kk + 4 * r - C0, bq = m16 - C0;
            if (a >= 0 && a < 8 && bq >= 0 && bq <= a) band_st(8 * p + a, a - bq, td[r]);
          }
        }
        // per lane of panel column c: its reflector's scal and beta (set in step c)
        double myscal = 0.0, mybeta = 0.0;
        sfor<8>([&](auto ii) {
          constexpr int i = decltype(ii)::value, CC_ = C0 + i;
          // pivot row rho = r0 + i: tile q0, row-in-tile 8 (1 - H) + i = kk + 4 r
          constexpr int PR = 8 * (1 - H) + i, GI = PR & 3, RI = PR >> 2;
          // x . x below the pivot, per lane for its own column, then over the 4 row groups
          double xx = 0.0, xx2 = 0.0;
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J > q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const double x = tile[J][r];
                if (r & 1) xx2 = fma(x, x, xx2);
                else xx = fma(x, x, xx);
              }
            }
          });
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double x = kk + 4 * r > PR ? tq[r] : 0.0;
            xx = fma(x, x, xx);
          }
          const double alpha = readlane_f64(tq[RI], 16 * GI + CC_);
          xx = swap_add_f64<32>(swap_add_f64<16>(xx + xx2));
          const double xxp = readlane_f64(xx, CC_);
          // dlarfg (rcp/rsq refined to ~1 ulp); H = I when x = 0
          const double a2 = fma(alpha, alpha, xxp);
          const double rs = rsq64(a2);
          const bool nz = xxp > 0.0;
          const double bt = -copysign(a2 * rs, alpha);
          const double beta = nz ? bt : alpha;
          const double tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
          const double scal = nz ? rcp64(alpha - bt) : 0.0;
          const double amb = nz ? alpha - bt : 0.0;  // xt at the pivot: v = scal xt
          if (m16 == CC_) {
            myscal = scal;
            mybeta = beta;
          }
          // S'_c = sum over rows >= rho of xt(row) A(row, c), xt = column CC_ from lane CC_ of
          // the row: 0 above the pivot, alpha - beta at it, x below.  Tiles past q0 with one
          // fused v_fmac_f64_dpp per register (volatile: the passes keep their order, and
          // each opens with two wait states after the last VALU write of a DPP source).
          double S = 0.0, S2 = 0.0;
          dpp_fence();
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J > q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                if (r & 1) S2 = fmac_row_v<CC_>(S2, tile[J][r], tile[J][r]);
                else S = fmac_row_v<CC_>(S, tile[J][r], tile[J][r]);
              }
            }
          });
          double Sq = 0.0;
          double xsq[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rr = kk + 4 * r;
            const double xb = rbcast<CC_>(tq[r]);
            xsq[r] = rr > PR ? xb : rr == PR ? amb : 0.0;
            Sq = fma(xsq[r], tq[r], Sq);
          }
          S = swap_add_f64<32>(swap_add_f64<16>((S + S2) + Sq));
          // v^T A(:, c) = scal S'_c.  Columns c > CC_ of the panel: A(:, c) -= tau v (v^T A(:,c))
          // = tau scal^2 S'_c xt; the earlier columns c < CC_ keep x_c = v_c / scal_c below
          // their pivots, so their S'_c give the Gram entries v_c^T v_i = scal_c scal S'_c.
          const bool upd = m16 > CC_ && m16 < C0 + 8;
          const double gam = upd ? tau * scal * scal * S : 0.0;
#pragma unroll
          for (int r = 0; r < 4; ++r) tq[r] = fma(-gam, xsq[r], tq[r]);
          dpp_fence();
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J > q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                tile[J][r] = fnmac_row_v<CC_>(tile[J][r], tile[J][r], gam);
            }
          });
          // T column i: T[i][i] = tau; T[j][i] = -tau sum_{k=j}^{i-1} T[j][k] t_k,
          // t_k = scal_k scal S'_{C0+k} (row group 0, lanes C0 + j)
          {
            const double tk = myscal * scal * S;
            double acc = 0.0;
            const int jl = m16 - C0;
            sfor<i>([&](auto kq) {
              constexpr int kq_ = decltype(kq)::value;
              const double tb = rbcast<C0 + kq_>(tk);
              if (jl >= 0 && jl <= kq_) acc = fma(sm.u.s.T[jl * 8 + kq_], tb, acc);
            });
            if (kk == 0 && jl >= 0 && jl < i) sm.u.s.T[jl * 8 + i] = -tau * acc;
            if (kk == 0 && jl == i) sm.u.s.T[i * 8 + i] = tau;
            if (kk == 0 && jl > i && jl < 8) sm.u.s.T[jl * 8 + i] = 0.0;
          }
        });
        // V (column c = m16 - C0: scal_c x below its pivot, 1 at it, 0 above) and the R entries
        // (rows r0 .. r0 + c - 1 as updated, beta_c at the pivot): the panel columns hold x_c
        // below their pivots (a step leaves its own column unchanged).  V rows r0 - 8 .. r0 - 1
        // (tile q0 above the panel when H = 0) land in V's unused rows 120..127.
        {
          const int cl = m16 - C0;
          const bool pc = cl >= 0 && cl < 8;
          const int prc = 8 * (1 - H) + cl;  // the column's pivot row within tile q0
#pragma unroll
          for (int r = 0; r < 4; ++r) {  // the pivot tile
            const int rr = kk + 4 * r, row = 16 * q0 + rr;
            const double x = tq[r];
            const double vv = rr > prc ? x * myscal : (rr == prc ? 1.0 : 0.0);
            if (pc) Vb[(row - r0) & 127][cl] = vv;
            if (pc && rr >= 8 * (1 - H) && rr <= prc)
              band_st(row, row - 8 * p - cl, rr == prc ? mybeta : x);
          }
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J > q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int row = 16 * J + kk + 4 * r;
                if (pc) Vb[row - r0][cl] = tile[J][r] * myscal;
              }
            }
          });
        }
      };
      if (h == 0) qr(std::integral_constant<int, 0>{});
      else qr(std::integral_constant<int, 1>{});
      if (swp) swap_slots();
      // V rows of the panel's top block above the diagonal and the rows of the trailing
      // columns are written above; the record gets V and T
      const int m = 128 - r0;
      double *pv = rec + HR::pv(p);
      for (int e = lane; e < 8 * m; e += 64) pv[e] = Vb[e >> 3][e & 7];
      rec[HR::PT + 64 * p + lane] = sm.u.s.T[lane];
      // u <- Q_p^T u = u - V T^T V^T u for u1, u2 (rows r0 .. 127: lane l, rows r0 + l, r0 + 64 + l)
      {
        double pa[8], pb[8];
        const int ra = lane, rb = lane + 64;
        const bool va = ra < m, vb = rb < m;
        const double ua0 = va ? sm.u.s.u[0][r0 + ra] : 0.0, ua1 = va ? sm.u.s.u[1][r0 + ra] : 0.0;
        const double ub0 = vb ? sm.u.s.u[0][r0 + rb] : 0.0, ub1 = vb ? sm.u.s.u[1][r0 + rb] : 0.0;
        double Va[8], Vbb[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          Va[a] = va ? Vb[ra][a] : 0.0;
          Vbb[a] = vb ? Vb[rb][a] : 0.0;
          pa[a] = fma(Va[a], ua0, Vbb[a] * ub0);
          pb[a] = fma(Va[a], ua1, Vbb[a] * ub1);
        }
        wave_sum4_dpp(pa[0], pa[1], pa[2], pa[3]);
        wave_sum4_dpp(pa[4], pa[5], pa[6], pa[7]);
        wave_sum4_dpp(pb[0], pb[1], pb[2], pb[3]);
        wave_sum4_dpp(pb[4], pb[5], pb[6], pb[7]);
        // y = T^T s (T upper): y_a = sum_{b <= a} T[b][a] s_b
        double ya[8], yb[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          double s0 = 0.0, s1 = 0.0;
#pragma unroll
          for (int b = 0; b <= a; ++b) {
            const double tba = sm.u.s.T[b * 8 + a];
            s0 = fma(tba, pa[b], s0);
            s1 = fma(tba, pb[b], s1);
          }
          ya[a] = s0;
          yb[a] = s1;
        }
        double na0 = ua0, na1 = ua1, nb0 = ub0, nb1 = ub1;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          na0 = fma(-Va[a], ya[a], na0);
          na1 = fma(-Va[a], yb[a], na1);
          nb0 = fma(-Vbb[a], ya[a], nb0);
          nb1 = fma(-Vbb[a], yb[a], nb1);
        }
        if (va) {
          sm.u.s.u[0][r0 + ra] = na0;
          sm.u.s.u[1][r0 + ra] = na1;
        }
        if (vb) {
          sm.u.s.u[0][r0 + rb] = nb0;
          sm.u.s.u[1][r0 + rb] = nb1;
        }
      }
    }
    __syncthreads();  // B1: V, T of the panel
    if (CWBL_DBG_STOP(c) == 6) continue;  // timing ablation: the QRs only

    // -- W(I) = (A22 V)(I) T for the wave's columns I >= q0 (rows < r0 masked) ------------------
    // V(J) in C/D layout (lane: row 16J + kk + 4r, column m16 < 8) is the B operand of the
    // tile (J, I) read as A^T: sum over J of A(J, I)^T V(J) = (A V)(I) (A symmetric)
    const bool act0 = I0 >= q0, act1 = I1 >= q0;
    auto vcd = [&](int J, int r) {
      const int row = 16 * J + kk + 4 * r;
      return m16 < 8 && row >= r0 ? Vb[row - r0][m16] : 0.0;
    };
    f64x4 W0 = {0.0, 0.0, 0.0, 0.0}, W1 = {0.0, 0.0, 0.0, 0.0};
    double V0c[4] = {0.0, 0.0, 0.0, 0.0}, V1c[4] = {0.0, 0.0, 0.0, 0.0};  // V(I0), V(I1) in C/D
    sfor<8>([&](auto JJ) {
      constexpr int J = decltype(JJ)::value;
      if (J >= q0) {
        double vj[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) vj[r] = vcd(J, r);
        if (J == I0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) V0c[r] = vj[r];
        }
        if (J == I1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) V1c[r] = vj[r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (act0) W0 = __builtin_amdgcn_mfma_f64_16x16x4f64(tile[J][r], vj[r], W0, 0, 0, 0);
          if (act1) W1 = __builtin_amdgcn_mfma_f64_16x16x4f64(tile[8 + J][r], vj[r], W1, 0, 0, 0);
        }
      }
    });
    // mask rows < r0, then W <- W T: W[row][c] = sum_{k <= c} W0[row][k] T[k][c] (lane c)
    double tcol[8];
#pragma unroll
    for (int kq = 0; kq < 8; ++kq) tcol[kq] = m16 < 8 ? sm.u.s.T[kq * 8 + m16] : 0.0;
    auto wt = [&](f64x4 &Wr, int I) {
      f64x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double wv = 16 * I + kk + 4 * r >= r0 ? Wr[r] : 0.0;
        double s = 0.0;
        sfor<8>([&](auto kq) {
          constexpr int kq_ = decltype(kq)::value;
          s = fma(rbcast<kq_>(wv), tcol[kq_], s);
        });
        o[r] = s;
      }
      Wr = o;
    };
    if (act0) wt(W0, I0);
    if (act1) wt(W1, I1);
    // M partial = V(I)^T W(I) on the matrix cores (V(I) in C/D layout is the A operand of V^T)
    {
      f64x4 Mp = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (act0) Mp = __builtin_amdgcn_mfma_f64_16x16x4f64(V0c[r], W0[r], Mp, 0, 0, 0);
        if (act1) Mp = __builtin_amdgcn_mfma_f64_16x16x4f64(V1c[r], W1[r], Mp, 0, 0, 0);
      }
      // M[a][b]: lane (kk, m16 = b), register r: a = kk + 4 r; a, b < 8
#pragma unroll
      for (int r = 0; r < 2; ++r)
        if (m16 < 8) sm.u.s.M[wave][(kk + 4 * r) * 8 + m16] = Mp[r];
    }
    __syncthreads();  // B2: the partial M of every wave
    // N = T^T M (lane c = m16 < 8: column c), Z(I) = W(I) - 1/2 V(I) N
    double ncol[8];
    {
      double mc[8];
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int ix = a * 8 + (m16 & 7);
        mc[a] = (sm.u.s.M[0][ix] + sm.u.s.M[1][ix]) + (sm.u.s.M[2][ix] + sm.u.s.M[3][ix]);
      }
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        double s = 0.0;
#pragma unroll
        for (int b = 0; b <= a; ++b) s = fma(sm.u.s.T[b * 8 + a], mc[b], s);
        ncol[a] = m16 < 8 ? s : 0.0;
      }
    }
    auto zst = [&](const f64x4 &Wr, const double (&Vc)[4], int I) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double s = 0.0;
        sfor<8>([&](auto aa) {
          constexpr int a = decltype(aa)::value;
          s = fma(rbcast<a>(Vc[r]), ncol[a], s);
        });
        const int row = 16 * I + kk + 4 * r;
        if (m16 < 8 && row >= r0) sm.u.s.Z[row - r0][m16] = fma(-0.5, s, Wr[r]);
      }
    };
    if (act0) zst(W0, V0c, I0);
    if (act1) zst(W1, V1c, I1);
    __syncthreads();  // B3: Z
    // -- A22 -= V Z^T + Z V^T on the tiles (J, I), J, I >= q0: K = 8 as two 4-slices ---------
    // A operand: lane (m16 = row in the tile, kk = k in the slice), B operand: lane (m16 =
    // column in the tile, kk)
    auto rowop = [&](const double(*X)[8], int J, int q) {
      const int row = 16 * J + m16;
      return row >= r0 ? X[row - r0][kk + 4 * q] : 0.0;
    };
    double vI0[2], zI0[2], vI1[2], zI1[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      vI0[q] = act0 ? rowop(Vb, I0, q) : 0.0;
      zI0[q] = act0 ? rowop(sm.u.s.Z, I0, q) : 0.0;
      vI1[q] = act1 ? rowop(Vb, I1, q) : 0.0;
      zI1[q] = act1 ? rowop(sm.u.s.Z, I1, q) : 0.0;
    }
    sfor<8>([&](auto JJ) {
      constexpr int J = decltype(JJ)::value;
      if (J >= q0) {
        double vJ[2], zJ[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          vJ[q] = -rowop(Vb, J, q);
          zJ[q] = -rowop(sm.u.s.Z, J, q);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (act0) {
            tile[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(vJ[q], zI0[q], tile[J], 0, 0, 0);
            tile[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(zJ[q], vI0[q], tile[J], 0, 0, 0);
          }
          if (act1) {
            tile[8 + J] = __builtin_amdgcn_mfma_f64_16x16x4f64(vJ[q], zI1[q], tile[8 + J], 0, 0, 0);
            tile[8 + J] = __builtin_amdgcn_mfma_f64_16x16x4f64(zJ[q], vI1[q], tile[8 + J], 0, 0, 0);
          }
        }
      }
    });
  }
  // the last diagonal block D_15: rows 120 + a, columns 120 + b (tile (7, 7), wave 0 slot 1)
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = kk + 4 * r - 8, b = m16 - 8;
      if (a >= 0 && b >= 0 && b <= a) band_st(120 + a, a - b, tile[15][r]);
    }
  }
  __syncthreads();
  if (tid < KP) {
    rec[HR::U1 + tid] = sm.u.s.u[0][tid];
    rec[HR::U2 + tid] = sm.u.s.u[1][tid];
  }
  if (tid == 0) info[gi] = make_int2(ptot, 0);
}

hipError_t launch_band_head(hipStream_t s, const TreeDesc *trees, SolveConsts c, SlabDev slab,
                            long long g0, int npts, const int *nbr_cnt, const int *nbr_idx,
                            int2 *info, double *ws) {
  if (npts <= 0) return hipSuccess;
  if (c.kp != 128 || c.k <= 96) return hipErrorInvalidValue;
  hipLaunchKernelGGL((band_head_kernel<false>), dim3(npts), dim3(256), 0, s, trees, c, slab, g0,
                     npts, nbr_cnt, nbr_idx, info, ws);
  return hipGetLastError();
}

size_t band_record_bytes() { return (size_t)BandRec::WORDS * sizeof(double); }

}  // namespace cwbl
