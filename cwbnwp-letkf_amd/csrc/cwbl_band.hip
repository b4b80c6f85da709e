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
//     on 32 lanes: the reflector's left block, diagonal block and the bulge below it as one
//     instruction stream), the band in LDS (16 KB: row i holds A(i, i-d), d = 0..15);
//     applies the chase's reflectors to Q1^T b1, Q1^T x' (a sweep's reflectors act on
//     disjoint rows: 8 at a time), runs the T^-1/2 quadrature of the tail kernel, the
//     back-transform y <- Q1 Q2 y (chase reflectors sweep by sweep, then the 15 panels) and
//     the RTPP/RTPS epilogue in the reference's fp32 order.
//
// The design is checked step for step by scripts/two_stage_b8.py (numpy; the same panels,
// schedule, storage bounds and application orders).  Padding rows (k < 128) are identity rows
// of A: their panel reflectors and chase reflectors are exact no-ops (tau = 0).
#include "cwbl_device.h"

#include <type_traits>
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

// value of lane L of this lane's 16-lane row (DPP row_newbcast, one v_mov_b64)
template <int L>
__device__ __forceinline__ double rbcast(double x) {
  return __longlong_as_double(
      __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(x), 0x150 + L, 0xf, 0xf, true));
}
// value of lane l ^ 8 of the row (row_ror:8)
__device__ __forceinline__ double ror8(double x) { return dpp_f64<0x128>(x); }
// sum over each 8-lane half of a 16-lane row (quad sums, then the half mirror)
__device__ __forceinline__ double rsum8(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  return v;
}

}  // namespace

// ---- the workspace record of one point ------------------------------------------------------
struct BandRec {
  static constexpr int N = 128, B = 8, NP = 15, NTASK = 1056;
  static constexpr int BAND = 0;                // [N][B+1]: A(i, i-d), d = 0..B
  static constexpr int U1 = BAND + N * (B + 1);   // Q1^T b1
  static constexpr int U2 = U1 + N;               // Q1^T x'
  static constexpr int PV = U2 + N;               // panel p: V (m_p x 8 row-major), m_p = 120-8p
  static constexpr int PT = PV + 8 * 960;         // panel p: T (8 x 8, upper)
  static constexpr int R2 = PT + NP * 64;         // chase reflector q: [q][0] tau, [q][e] v_e
  static constexpr int WORDS = R2 + NTASK * 8;
  __host__ __device__ static constexpr int pv(int p) { return PV + 8 * (120 * p - 4 * p * (p - 1)); }
};
static_assert(BandRec::pv(15) == BandRec::PT, "panel reflector offsets");

// the chase schedule (scripts/two_stage_b8.py: schedule): tasks of sweep j, their first index,
// and the round in which sweep j starts (two slots, sweep j+1 three tasks behind sweep j)
struct ChasePlan {
  short start[126], first[127], ntask[126];
  int rounds;
};
__host__ __device__ constexpr int chase_ntask(int j) { return j <= 125 ? (125 - j) / 8 + 1 : 0; }
__host__ __device__ constexpr ChasePlan make_chase_plan() {
  ChasePlan p{};
  int acc = 0, end = 0;
  for (int j = 0; j < 126; ++j) {
    int s = 0;
    if (j >= 1 && p.start[j - 1] + 3 > s) s = p.start[j - 1] + 3;
    if (j >= 2 && p.start[j - 2] + p.ntask[j - 2] > s) s = p.start[j - 2] + p.ntask[j - 2];
    p.start[j] = (short)s;
    p.ntask[j] = (short)chase_ntask(j);
    p.first[j] = (short)acc;
    acc += p.ntask[j];
    if (s + p.ntask[j] > end) end = s + p.ntask[j];
  }
  p.first[126] = (short)acc;
  p.rounds = end;
  return p;
}
constexpr ChasePlan kChase = make_chase_plan();
static_assert(kChase.first[126] == BandRec::NTASK && kChase.rounds == 586, "chase plan");
__constant__ ChasePlan cChase = kChase;

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
    // (the select keeps tile9's index static)
#pragma unroll
    for (int t = 1; t < NTW; ++t)
      if (t == 8 - wave) diag(tile9[t], I1);
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
  f64x4 tile[16];
  auto build = [&](auto W_) {
    constexpr int W = decltype(W_)::value;
    sfor<16>([&](auto tt) {
      constexpr int t = decltype(tt)::value;
      constexpr int I = t < 8 ? W : 7 - W, J = t & 7;
      if constexpr (J >= I) {
        constexpr int t9 = t < 8 ? J - W : (8 - W) + J - (7 - W);
        tile[t] = tile9[t9];
      } else {  // (J, I) = (I, J)^T: element (a, b) of (J, I) is (b, a) of (I, J)
        const double *s = sm.u.mir[mir_slot(I, J)];
#pragma unroll
        for (int r = 0; r < 4; ++r) tile[t][r] = s[m16 * 17 + kk + 4 * r];
      }
    });
  };
  switch (wave) {
    case 0: build(std::integral_constant<int, 0>{}); break;
    case 1: build(std::integral_constant<int, 1>{}); break;
    case 2: build(std::integral_constant<int, 2>{}); break;
    default: build(std::integral_constant<int, 3>{}); break;
  }
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

  // ---- stage 1: 15 panels of 8 columns -------------------------------------------------------
  // the band row i of the record: A(i, i - d), d = 0..8
  auto band_st = [&](int i, int d, double v) { rec[HR::BAND + i * (HR::B + 1) + d] = v; };
  for (int p = 0; p < HR::NP; ++p) {
    const int Q = p >> 1, h = p & 1, r0 = 8 * p + 8, q0 = Q + h;
    const int owner = Q < 4 ? Q : 7 - Q;
    double(*Vb)[8] = sm.u.s.V[p & 1];  // (double buffer: slower waves may still read the last V)
    // (no barrier here: T, Z and M of the previous panel were last read before its barrier B3,
    // and a wave reaches this panel's B1 only after its part of the previous update)
    if (wave == owner) {
      // -- the panel QR, in place in tile column Q (slot SL), columns 8H .. 8H + 7 --------------
      auto qr = [&](auto SL_, auto H_) {
        constexpr int SL = decltype(SL_)::value, H = decltype(H_)::value;
        constexpr int C0 = 8 * H;
        // band: the diagonal block D_p (rows 8p + a, columns 8p + b, b <= a): tile (Q, Q),
        // rows C0 + a (kk + 4r), columns C0 + b (m16)
        sfor<8>([&](auto JJ) {
          constexpr int J = decltype(JJ)::value;
          if (J == Q) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int a = kk + 4 * r - C0, b = m16 - C0;
              if (a >= 0 && a < 8 && b >= 0 && b <= a) band_st(8 * p + a, a - b, tile[SL * 8 + J][r]);
            }
          }
        });
        double myscal = 0.0;  // scal of this lane's column's reflector (lanes of the panel)
        sfor<8>([&](auto ii) {
          constexpr int i = decltype(ii)::value, CC_ = C0 + i;
          // pivot row rho = r0 + i: tile q0, row-in-tile 8 (1 - H) + i = kk + 4 r
          constexpr int PR = 8 * (1 - H) + i, GI = PR & 3, RI = PR >> 2;
          // x . x below the pivot, per lane for its own column, then over the 4 row groups
          double xx = 0.0, alpha = 0.0;
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J >= q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const double x = tile[SL * 8 + J][r];
                const bool below = J > q0 || kk + 4 * r > PR;
                xx = fma(below ? x : 0.0, below ? x : 0.0, xx);
              }
              if (J == q0) alpha = readlane_f64(tile[SL * 8 + J][RI], 16 * GI + CC_);
            }
          });
          xx = swap_add_f64<32>(swap_add_f64<16>(xx));
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
          if (m16 == CC_) myscal = scal;
          // S'_c = sum over rows >= rho of xt(row) A(row, c), xt = column CC_ from lane CC_
          // of the row (masked: 0 above the pivot, alpha - beta at it)
          double S = 0.0;
          auto xt_of = [&](int J, int r, double x) {
            const int rr = kk + 4 * r;
            return J > q0 ? x : (rr > PR ? x : rr == PR ? amb : 0.0);
          };
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J >= q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const double xs = xt_of(J, r, rbcast<CC_>(tile[SL * 8 + J][r]));
                S = fma(xs, tile[SL * 8 + J][r], S);
              }
            }
          });
          S = swap_add_f64<32>(swap_add_f64<16>(S));
          // v^T A(:, c) = scal S'_c.  Columns c > CC_ of the panel: A(:, c) -= tau v (v^T A(:,c))
          // = tau scal^2 S'_c xt; the earlier columns c < CC_ keep x_c = v_c / scal_c below
          // their pivots, so their S'_c give the Gram entries v_c^T v_i = scal_c scal S'_c.
          const bool upd = m16 > CC_ && m16 < C0 + 8;
          const double gam = upd ? tau * scal * scal * S : 0.0;
          // the R entries of column CC_ (rows r0 .. rho - 1 and beta at rho) and V column i,
          // before the update (which leaves column CC_ itself unchanged)
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J >= q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int rr = kk + 4 * r, row = 16 * J + rr;
                const double x = tile[SL * 8 + J][r];
                if (m16 == CC_ && row >= r0) {
                  if (J == q0 && rr <= PR)  // rows r0 .. rho of R
                    band_st(row, row - 8 * p - i, rr == PR ? beta : x);
                  Vb[row - r0][i] = J > q0 || rr > PR ? x * scal : rr == PR ? 1.0 : 0.0;
                }
              }
            }
          });
          sfor<8>([&](auto JJ) {
            constexpr int J = decltype(JJ)::value;
            if (J >= q0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const double xs = xt_of(J, r, rbcast<CC_>(tile[SL * 8 + J][r]));
                tile[SL * 8 + J][r] = fma(-gam, xs, tile[SL * 8 + J][r]);
              }
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
      };
      if (Q == I0) {
        if (h == 0) qr(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
        else qr(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
      } else {
        if (h == 0) qr(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
        else qr(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
      }
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

// ==== stage 2: chase, quadrature, back-transform, epilogue ===================================
struct BandTailSmem {
  union {
    double band[128][16];  // the chase: row i holds A(i, i - d), d = 0..15
    double tq[129][4];     // then d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
    double y[128];         // then y for the back-transform
  } a;
  union {
    double u[2][128];      // Q1^T b1, Q1^T x' through the chase's reflectors
    struct {
      double Ym[128], Zm[128];  // quadrature sum / exact solve, walk order
    } q;
  } b;
};

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

  // ---- the band into LDS --------------------------------------------------------------------
  for (int e = l; e < 128 * 16; e += 64) {
    const int i = e >> 4, d = e & 15;
    sm.a.band[i][d] = d <= HR::B ? rec[HR::BAND + i * (HR::B + 1) + d] : 0.0;
  }
  sm.b.u[0][l] = rec[HR::U1 + l];
  sm.b.u[0][64 + l] = rec[HR::U1 + 64 + l];
  sm.b.u[1][l] = rec[HR::U2 + l];
  sm.b.u[1][64 + l] = rec[HR::U2 + 64 + l];
  __syncthreads();

  // ---- the chase: rounds of up to two tasks (slot 0: even sweeps, slot 1: odd sweeps) ------
  // lanes of a slot: row 0 = lanes 0-7 left block (and the reflector), 8-15 diagonal block;
  // row 1 = lanes 0-7 the bulge rows below, 8-15 idle
  const int slot = l >> 5, rr = (l >> 4) & 1, lo = l & 15;
  const int e8 = lo & 7;
  const bool rA = rr == 0 && lo < 8, rB = rr == 0 && lo >= 8, rC = rr == 1 && lo < 8;
  int js = slot;  // this slot's current sweep
  double *__restrict__ r2 = rec + HR::R2;
  for (int R = 0; R < cChase.rounds; ++R) {
    const int st = js <= 125 ? cChase.start[js] : 1 << 30;
    const int t = R - st;
    const bool act = js <= 125 && t >= 0 && t < cChase.ntask[js];
    const int j = js <= 125 ? js : 0;
    const int r = j + 1 + 8 * (act ? t : 0);
    const int cc = (act && t > 0) ? r - 8 : j;  // the annihilated column
    const int L = min(8, 128 - r);              // reflector length (>= 2 for a task)
    // column entries x_e = A(r + e, cc) on lanes 0-7 of both rows
    double xe = 0.0;
    if (act && lo < 8 && e8 < L) xe = sm.a.band[r + e8][r + e8 - cc];
    const double sq = lo < 8 && e8 >= 1 ? xe * xe : 0.0;
    const double xx = rbcast<0>(rsum8(sq));
    const double alpha = rbcast<0>(xe);
    const double a2 = fma(alpha, alpha, xx);
    const double rs = rsq64(a2);
    const bool nz = xx > 0.0;
    const double bt = -copysign(a2 * rs, alpha);
    const double beta = nz ? bt : alpha;
    const double tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
    const double scal = nz ? rcp64(alpha - bt) : 0.0;
    const double v = lo < 8 ? (e8 == 0 ? 1.0 : xe * scal) : 0.0;  // v_e on lanes e of a row
    // this lane's 8-vector: A column (left block), A row (diagonal block, both triangles
    // from the lower storage), A row (bulge rows below)
    double X[8];
    int rowX = 0;  // the band row of the lane's vector (A, C: varies with e; B: r + b)
    const int b = lo - 8;
    const int colA = cc + 1 + lo;            // role A's column
    const bool vA = act && rA && t > 0 && lo < 7;
    const bool vB = act && rB && b < L;
    const int rowC = r + 8 + lo;
    const bool vC = act && rC && L == 8 && rowC < 128;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      double x = 0.0;
      if (e < L) {
        if (vA) x = sm.a.band[r + e][r + e - colA];
        else if (vB) x = e <= b ? sm.a.band[r + b][b - e] : sm.a.band[r + e][e - b];
        else if (vC) x = sm.a.band[rowC][8 + lo - e];
      }
      X[e] = x;
    }
    (void)rowX;
    // v^T X on every lane (v_e from lane e of the row)
    double dot = 0.0;
    sfor<8>([&](auto ee) {
      constexpr int e = decltype(ee)::value;
      dot = fma(rbcast<e>(v), X[e], dot);
    });
    // the diagonal block (lanes 8-15 of row 0): p = tau D v, w = p - 1/2 tau (v^T p) v
    const double vb = ror8(v);  // v_b on lane 8 + b
    const double s1 = rsum8(vb * dot);
    const double wB = tau * fma(-0.5 * tau, s1 * vb, dot);
    const double al = rB ? wB : tau * dot;
    const double be = rB ? vb : 0.0;
    // X -= al v + be w  (one-sided: tau (v^T X) v; two-sided: w_b v + v_b w)
    sfor<8>([&](auto ee) {
      constexpr int e = decltype(ee)::value;
      X[e] = fma(-al, rbcast<e>(v), X[e]);
      X[e] = fma(-be, rbcast<8 + e>(wB), X[e]);
    });
    // stores: the annihilated column, the blocks, the reflector
    if (act && rA && lo < L) sm.a.band[r + lo][r + lo - cc] = lo == 0 ? beta : 0.0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (e < L) {
        if (vA) sm.a.band[r + e][r + e - colA] = X[e];
        else if (vB && e <= b) sm.a.band[r + b][b - e] = X[e];
        else if (vC) sm.a.band[rowC][8 + lo - e] = X[e];
      }
    }
    if (act && rA) r2[(cChase.first[j] + t) * 8 + lo] = lo == 0 ? tau : (lo < L ? v : 0.0);
    if (act && t + 1 == cChase.ntask[js]) js += 2;
    __syncthreads();
  }
  // ---- T: d_i = A(i, i), c(i-1, i) = A(i, i-1) ------------------------------------------------
  double dA = sm.a.band[l][0], eA = sm.a.band[l][1];
  double dB = sm.a.band[64 + l][0], eB = sm.a.band[64 + l][1];
  __syncthreads();
  sm.a.tq[l][0] = dA;
  sm.a.tq[l][1] = l == 0 ? 0.0 : eA;
  sm.a.tq[64 + l][0] = dB;
  sm.a.tq[64 + l][1] = eB;
  if (l == 0) sm.a.tq[KP][1] = 0.0;
  // ---- Q2^T applied to u1, u2: sweep after sweep, a sweep's reflectors (disjoint rows) 8 at a
  // time: lane = reflector tt (l >> 3) + 8 pass, entry e = l & 7
  auto apply_sweep = [&](double *u0, double *u1v, int j, int pass, bool both) {
    const int tt = 8 * pass + (l >> 3), e = l & 7;
    const bool ok = tt < cChase.ntask[j];
    const int r = j + 1 + 8 * tt;
    const int L = min(8, 128 - r);
    const double *q = r2 + (ok ? cChase.first[j] + tt : 0) * 8;
    const double tu = ok ? q[0] : 0.0;
    const double ve = ok && e < L ? (e == 0 ? 1.0 : q[e]) : 0.0;
    const int row = ok && e < L ? r + e : 0;
    const double a0 = ve * u0[row];
    const double d0 = rsum8(a0);
    double d1 = 0.0;
    if (both) d1 = rsum8(ve * u1v[row]);
    __syncthreads();
    if (ok && e < L) {
      u0[row] = fma(-tu * d0, ve, u0[row]);
      if (both) u1v[row] = fma(-tu * d1, ve, u1v[row]);
    }
    __syncthreads();
  };
  for (int j = 0; j < 126; ++j)
    for (int pass = 0; 8 * pass < cChase.ntask[j]; ++pass)
      apply_sweep(sm.b.u[0], sm.b.u[1], j, pass, true);
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
  auto walk = [](int i) { return i < H ? i : H + (KP - 1 - i); };
  const double d = wave_sum_dpp(fma(sm.a.tq[l][2], sm.b.q.Zm[walk(l)],
                                    sm.a.tq[64 + l][2] * sm.b.q.Zm[walk(64 + l)]));
  double y0 = sm.b.q.Ym[walk(l)], y1 = sm.b.q.Ym[walk(64 + l)];
  __syncthreads();
  // ---- y <- Q1 Q2 y: the chase's reflectors sweep by sweep in reverse, then the panels -------
  sm.a.y[l] = y0;
  sm.a.y[64 + l] = y1;
  __syncthreads();
  for (int j = 125; j >= 0; --j)
    for (int pass = 0; 8 * pass < cChase.ntask[j]; ++pass)
      apply_sweep(sm.a.y, nullptr, j, pass, false);
  y0 = sm.a.y[l];
  y1 = sm.a.y[64 + l];
  for (int p = HR::NP - 1; p >= 0; --p) {
    const int r0 = 8 * p + 8, mrows = 128 - r0;
    const double *pv = rec + HR::pv(p);
    const double *pt = rec + HR::PT + 64 * p;
    // lane l: rows l and 64 + l (row index >= r0 only)
    const int ia = l - r0, ib = 64 + l - r0;
    const bool va = ia >= 0 && ia < mrows, vb = ib >= 0 && ib < mrows;
    double Va[8], Vbb[8], s[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      Va[a] = va ? pv[ia * 8 + a] : 0.0;
      Vbb[a] = vb ? pv[ib * 8 + a] : 0.0;
      s[a] = fma(Va[a], y0, Vbb[a] * y1);
    }
    wave_sum4_dpp(s[0], s[1], s[2], s[3]);
    wave_sum4_dpp(s[4], s[5], s[6], s[7]);
    double z[8];  // z = T s (T upper)
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      double acc = 0.0;
#pragma unroll
      for (int bq = a; bq < 8; ++bq) acc = fma(pt[a * 8 + bq], s[bq], acc);
      z[a] = acc;
    }
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      y0 = fma(-Va[a], z[a], y0);
      y1 = fma(-Vbb[a], z[a], y1);
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

hipError_t launch_band_head(hipStream_t s, const TreeDesc *trees, SolveConsts c, SlabDev slab,
                            long long g0, int npts, const int *nbr_cnt, const int *nbr_idx,
                            int2 *info, double *ws) {
  if (npts <= 0) return hipSuccess;
  if (c.kp != 128 || c.k <= 96) return hipErrorInvalidValue;
  hipLaunchKernelGGL((band_head_kernel<false>), dim3(npts), dim3(256), 0, s, trees, c, slab, g0,
                     npts, nbr_cnt, nbr_idx, info, ws);
  return hipGetLastError();
}

hipError_t launch_band_tail(hipStream_t s, SolveConsts c, SlabDev slab, long long g0, int npts,
                            double *ws, int2 *info) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr || c.kp != 128 || c.k <= 96) return hipErrorInvalidValue;
  hipLaunchKernelGGL(band_tail_kernel, dim3(npts), dim3(64), 0, s, c, slab, g0, npts, ws, info);
  return hipGetLastError();
}

size_t band_record_bytes() { return (size_t)BandRec::WORDS * sizeof(double); }

}  // namespace cwbl
