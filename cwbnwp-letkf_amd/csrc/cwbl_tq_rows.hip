// cwbl_tq_rows.hip — solve_tq_rows_kernel<128, 64>: the first half of the per-point LETKF
// solve (letkf_solve, module_letkf_core.f90:598-700) at k = 97..128 on the slab path: the
// column staging and the matrix-core assembly of A = (k-1)/infl I + Yb Yb^T and b1 = Yb d,
// then the first 64 steps of the Householder tridiagonalisation A = Q T Q^T (dsytd2 order,
// the reference's dsyevd reduction, module_eigen.f90:48-56), handed over through the
// workspace (BigHandoff<128, 64>) to solve_tqb_tail_kernel (cwbl_tq_tail.hip).
//
// One 256-thread workgroup per grid point, the matrix held in HALF ROWS: wave w holds row
// 64 (w / 2) + lane, the columns of half h = w % 2 (the 8-column groups 2 i + h: dead columns
// leave both halves at the same rate), both triangles (A is kept symmetric).  A step then
// needs no LDS traffic beyond three vectors:
//   - the pivot column (the waves of the half holding column j: each lane's own entry,
//     picked by value) goes to LDS with its norm partials (barrier A);
//   - every lane copies the 64 pivot-row entries of its half into four row-replicated
//     registers (four LDS reads) and runs the matvec as row_newbcast operands of fused
//     v_fmac_f64_dpp, as the tail kernel does; the half-row partials of A v and the partial
//     sums of v.Av, v.x', v.b1 go to LDS (barrier B);
//   - every lane forms w for its replicated columns from the two partials (no third
//     exchange) and runs the rank-2 update the same way.
// Two barriers per step (the 4x4-block kernel, solve_tq_big_kernel, needs four and moves its
// block partials and both vectors through LDS each step).  The steps run in compile-time
// blocks by the 8-column group of column j + 1, so the dead columns (c <= j) are skipped
// statically.
#include "cwbl_device.h"

#include <type_traits>

namespace cwbl {

namespace {

// (64-column chunks: a chunk's MFMA phase at two waves per SIMD then covers the next chunk's
// gathers; the staging shares its LDS with the 72 KB tile area, so they cost no occupancy)
constexpr int kRowsKP = 128, kRowsHS = 64, kRowsChunk = 64;

// element (i, jj) of a staged 16x16 tile: rows of 16 doubles, the column XOR-rotated by the
// row pair so that 16 lanes reading one column of a tile (rows i) hit 32 distinct banks
__device__ __forceinline__ int tile_at(int i, int jj) { return 16 * i + (jj ^ ((i >> 1) & 7)); }
// lower-triangle tile index of tile (I, J), I >= J
__device__ __forceinline__ int tile_index(int I, int J) { return I * (I + 1) / 2 + J; }
// the column of local column cc of half h: half h holds the 8-column groups 2 i + h, so the
// dead columns (c <= j) leave both halves at the same rate
__host__ __device__ constexpr int gcol(int h, int cc) { return 16 * (cc >> 3) + 8 * h + (cc & 7); }

}  // namespace

struct RowsSmem {
  union {
    ColumnChunk<kRowsKP, kRowsChunk, float, kRowsKP, false, true> ch[2];  // column staging
    double tl[36][256];  // the 36 lower 16x16 tiles of A (tile_at), for the half-row gather
  } u;
  double x[kRowsKP];        // pivot column j (raw); before the steps: x'
  double p[2][kRowsKP];     // (A v)_r partials over column halves; before the steps: b1
  double redA[2];           // x.x partials of the half-0 waves
  double redB[4][4];        // [wave]: v.Av, v.x', v.b1 partials
  double d[kRowsHS];        // d_j
  double e[kRowsHS + 1];    // c(j-1, j) = beta of step j-1
  double tau[kRowsHS];
  float parf;
  int ptot;
};

template <int KP, int HS>
__global__ void __launch_bounds__(256, 2)
solve_tq_rows_kernel(const TreeDesc *__restrict__ trees, SolveConsts c, SlabDev slab,
                     long long g0, int npts, const int *__restrict__ nbr_cnt,
                     const int *__restrict__ nbr_idx, int2 *__restrict__ info,
                     double *__restrict__ ws) {
  static_assert(KP == kRowsKP && HS == kRowsHS, "one instantiation: 128 rows, 64 steps");
  constexpr int NT = 256, NTW = 9;
  using HO = BigHandoff<KP, HS>;
  static_assert(sizeof(RowsSmem) <= 80 * 1024, "two workgroups per CU");
  __shared__ RowsSmem sm;

  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int tid = threadIdx.x, l = tid & 63, wave = tid >> 6;
  const int rb = wave >> 1, h = wave & 1;  // row block, column half
  const int r = 64 * rb + l;               // this lane's row
  const int k = c.k;

  long long P;
  float3 pt;
  {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long q = g / slab.ix_lim;
    const int jj = (int)(q % slab.iy_lim);
    const int kz = (int)(q / slab.iy_lim);
    P = i + (long long)slab.nx * (jj + (long long)slab.ny * kz);
    slab_point(slab, g, pt.x, pt.y, pt.z);
  }
  const float xbl = tid < k ? slab.var[P + slab.L * tid] : 0.0f;  // background of member tid

  // ---- matrix-core assembly: the 36 lower tiles, nine per wave (wave w: tile rows w and
  // 7 - w; its tile t is (w, t) for t <= w, (7 - w, t - w - 1) above).  A lane holds rows
  // kk + 4 q of column m of each tile.  b1 = Yb d on threads < 128 (row tid).
  using CC = std::remove_reference_t<decltype(sm.u.ch[0])>;
  f64x4 tile[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) tile[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  double b1p[4] = {0.0, 0.0, 0.0, 0.0};
  const int m = l & 15, kk = l >> 4;
  {
    // the rows of column 4 g + kk are XOR 16 for odd kk (ColumnChunk XSW)
    const int xk = CC::xr(kk);
    const int offAx = (16 * wave + m) ^ xk, offBx = (16 * (7 - wave) + m) ^ xk;
    int offJx[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) offJx[t] = (16 * (t <= wave ? t : t - wave - 1) + m) ^ xk;
    auto chunk = [&](int nsl, const CC &cb) {
      for (int s0 = 0; s0 < (CWBL_DBG_STOP(c) == 12 ? 0 : nsl); s0 += 4) {
        const float *ys = cb.yb[s0 + kk];
        const double a = (double)ys[offAx], b = (double)ys[offBx];
#pragma unroll
        for (int t = 0; t < NTW; ++t)
          tile[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(t <= wave ? a : b, (double)ys[offJx[t]],
                                                         tile[t], 0, 0, 0);
      }
      {  // Yb d: row tid % 128, the rounds of eight columns split between the two thread
         // halves (all four waves take a share), four chains
        const int nr = (nsl + 7) / 8;
        for (int r8 = tid >> 7; r8 < nr; r8 += 2) {
          const float4 o0 = *reinterpret_cast<const float4 *>(&cb.yo[8 * r8]);
          const float4 o1 = *reinterpret_cast<const float4 *>(&cb.yo[8 * r8 + 4]);
          const float o[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
          float y[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) y[i] = cb.at(8 * r8 + i, tid & 127);
#pragma unroll
          for (int i = 0; i < 8; ++i) b1p[i & 3] = fma((double)y[i], (double)o[i], b1p[i & 3]);
        }
      }
    };
    const int pt_ = stage_columns_pipe<KP, kRowsChunk, NT>(sm.u.ch, trees, c, gi, tid, nbr_cnt,
                                                            nbr_idx, pt, chunk);
    if (tid == 0) sm.ptot = pt_;  // counted by wave 0
  }
  const double b1acc = (b1p[0] + b1p[1]) + (b1p[2] + b1p[3]);
  __syncthreads();  // ptot; the staging area is free
  const int ptot = sm.ptot;
  if (ptot == 0) {  // no accepted observation: var left unchanged (:220, :226)
    if (tid == 0) info[gi] = make_int2(0, 0);
    return;
  }

  // ---- tiles -> LDS (all 36 at once), the diagonal inflated (padding rows: 1) ---------------
  const double inflat_r8 = (double)c.inflat;
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int I = t <= wave ? wave : 7 - wave, J = t <= wave ? t : t - wave - 1;
    double *dst = sm.u.tl[tile_index(I, J)];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = kk + 4 * q, row = 16 * I + i;
      double vv = tile[t][q];
      if (I == J && i == m) vv = row < k ? vv + inflat_r8 : 1.0;
      dst[tile_at(i, m)] = vv;
    }
  }
  // x' and b1 by row (rows 64..127 live in waves 2, 3 here, in threads 64..127 above)
  const float xb_mean_f = [&] {  // the reference's sequential fp32 member sum (:671)
    for (int w = 0; 64 * w < k; ++w) {
      if (wave == w) {
        float s = w == 0 ? 0.0f : sm.parf;
        const int n = min(64, k - 64 * w);
        for (int mm = 0; mm < n; ++mm)
          s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xbl), mm));
        if (l == 0) sm.parf = s;
      }
      __syncthreads();
    }
    return sm.parf * c.nmember_inv;
  }();
  const double xb_mean = (double)xb_mean_f;
  if (tid < KP) sm.x[tid] = tid < k ? (double)xbl - xb_mean : 0.0;
  sm.p[tid >> 7][tid & 127] = b1acc;  // the two halves' Yb d partials
  __syncthreads();
  double ux = sm.x[r], ub = sm.p[0][r] + sm.p[1][r];  // x', then Q^T x'; b1, then Q^T b1
  // half row: A[cc] = A(r, gcol(h, cc))
  double A[64];
  {
    const int I = r >> 4, i = r & 15;
    sfor<64>([&](auto CC_) {
      constexpr int cc = decltype(CC_)::value;
      const int col = gcol(h, cc), J = col >> 4, jj = col & 15;
      A[cc] = I >= J ? sm.u.tl[tile_index(I, J)][tile_at(i, jj)]
                     : sm.u.tl[tile_index(J, I)][tile_at(jj, i)];
    });
  }
  if (CWBL_DBG_STOP(c) == 1 || CWBL_DBG_STOP(c) >= 12) {  // timing ablation: assembly only
    double t = ux + ub;
#pragma unroll
    for (int cc = 0; cc < 64; ++cc) t += A[cc];
    if (tid == 0) info[gi] = make_int2(ptot, (int)t);
    return;
  }

  double *__restrict__ wo = ws + (long long)gi * HO::WORDS;
  const auto rec = rec_rsrc(wo, HO::WORDS);
  auto opq = [](double a) {  // (see the tail kernel: picks by value, no scratch)
    asm("" : "+v"(a));
    return a;
  };
  // four row-replicated registers: R[g] holds, in every 16-lane row, src[64 h + 16 g + 0..15]
  // (read from LDS); mask applies the pivot-row form xt_c
  auto pin4 = [](double (&R)[4]) {
    asm volatile("s_nop 1" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]));
  };

  // ---- Householder steps j = 0 .. 63 ----------------------------------------------------------
  // Phase A of step jn: column jn (in group gjn, held by half gjn & 1 as its local columns
  // 8 (gjn / 2) ..) and x.x below row jn + 1 to LDS.  It runs inside the previous step's
  // update, right after the group holding the column is updated, so its reductions overlap
  // the rest of the update (nobody reads x or redA between barrier B and the next barrier A).
  auto phase_a = [&](int jn, auto GJN) {
    constexpr int gjn = decltype(GJN)::value;
    double xr = 0.0;
    sfor<8>([&](auto ee) {
      constexpr int e = decltype(ee)::value, cc = 8 * (gjn >> 1) + e;
      xr = jn == 8 * gjn + e ? opq(A[cc]) : xr;
    });
    sm.x[r] = xr;
    const double xs = wave_sum_dpp(r > jn + 1 ? xr * xr : 0.0);
    if (l == 0) sm.redA[rb] = xs;
  };
  // Block GJ: the steps whose column j + 1 is in group gj (j = 8 gj - 1 .. 8 gj + 6); H: this
  // wave's half (static); c0: its first live local column in the block
  const int jend = CWBL_DBG_STEPS(c) > 0 ? min(HS, CWBL_DBG_STEPS(c)) : HS;  // (ablation)
  auto step = [&](const int j, auto GJ, auto H) {
    constexpr int gj = decltype(GJ)::value, hh = decltype(H)::value;
    constexpr int i0 = (gj - hh + 1) >> 1 > 0 ? (gj - hh + 1) >> 1 : 0, c0 = 8 * i0;
    constexpr bool half0 = hh == 0;
    const int j1 = j + 1;
    __syncthreads();  // barrier A: column j and its x.x are in LDS
    // phase B: the reflector, v, the replicated pivot row, the matvec
    const double xn2 = sm.redA[0] + sm.redA[1];
    const double dj = sm.x[j], alpha = sm.x[j1];
    const double a2 = fma(alpha, alpha, xn2);
    const double rs = rsq64(a2);  // 1/|beta|
    const bool nz = xn2 > 0.0;
    const double bt = -copysign(a2 * rs, alpha);
    const double beta = nz ? bt : alpha;
    const double tau = nz ? (bt - alpha) * -copysign(rs, alpha) : 0.0;
    const double rab = rcp64(alpha - bt);
    const double scal = nz ? rab : 0.0;
    const double amb = nz ? alpha - bt : 0.0;
    if (tid == 0) {
      sm.d[j] = dj;
      sm.e[j1] = beta;
      sm.tau[j] = tau;
    }
    const double xo = sm.x[r];
    const double v = r == j1 ? 1.0 : r > j1 ? xo * scal : 0.0;
    // reflector j, rows > j (1 at row j + 1; the tail kernel loads no row above)
    if constexpr (half0) rec_st(rec, rec_off(r > j, HO::HV + j * KP + r), v);
    double R[4];
    sfor<4>([&](auto G) {
      constexpr int g = decltype(G)::value;
      if constexpr (16 * g + 15 >= c0) {
        const int cc = gcol(hh, 16 * g + (l & 15));
        const double xc = sm.x[cc];
        R[g] = cc > j1 ? xc : cc == j1 ? amb : 0.0;
      } else {
        R[g] = 0.0;
      }
    });
    pin4(R);
    // four chains, each chain's FMAs four instructions apart (r6: eight chains cost eight
    // zeroing moves and four adds more per step, 21.60 against 21.45 ms per launch)
    double q[4] = {0.0, 0.0, 0.0, 0.0};
    sfor<64 - c0>([&](auto CC_) {
      constexpr int cc = c0 + decltype(CC_)::value;
      q[cc % 4] = fmac_row_v<cc % 16>(q[cc % 4], R[cc / 16], A[cc]);
    });
    const double ph = scal * ((q[0] + q[1]) + (q[2] + q[3]));
    sm.p[h][r] = ph;
    double s1 = v * ph, s2 = half0 ? v * ux : 0.0, s3 = half0 ? v * ub : 0.0, z = 0.0;
    wave_sum4_dpp(s1, s2, s3, z);
    if (l == 0) {
      sm.redB[wave][0] = s1;
      sm.redB[wave][1] = s2;
      sm.redB[wave][2] = s3;
    }
    __syncthreads();
    // phase C: w and the rank-2 update A <- A - w v^T - v w^T
    const double sv = (sm.redB[0][0] + sm.redB[1][0]) + (sm.redB[2][0] + sm.redB[3][0]);
    const double su = (sm.redB[0][1] + sm.redB[1][1]) + (sm.redB[2][1] + sm.redB[3][1]);
    const double sb = (sm.redB[0][2] + sm.redB[1][2]) + (sm.redB[2][2] + sm.redB[3][2]);
    const double s1t = tau * sv;  // v^T (tau A v)
    ux = fma(-tau * su, v, ux);
    ub = fma(-tau * sb, v, ub);
    const double hs = -0.5 * tau * s1t;
    // w is not zeroed on the eliminated rows and columns (r, c <= j): it only moves their own
    // entries, which nothing reads again (the matvec's R is zero there and the hand-off takes
    // columns past 63), by an orthogonal transform, so they stay bounded
    const double wl = fma(hs, v, tau * (sm.p[0][r] + sm.p[1][r]));
    const double wsl = wl * scal;
    double W[4];
    sfor<4>([&](auto G) {
      constexpr int g = decltype(G)::value;
      if constexpr (16 * g + 15 >= c0) {
        const int cc = gcol(hh, 16 * g + (l & 15));
        W[g] = fma(hs, scal * R[g], tau * (sm.p[0][cc] + sm.p[1][cc]));
      } else {
        W[g] = 0.0;
      }
    });
    pin4(W);
    sfor<(64 - c0) / 8>([&](auto GG) {
      constexpr int gg = decltype(GG)::value, cb = c0 + 8 * gg;
      sfor<8>([&](auto ii) {
        constexpr int cc = cb + decltype(ii)::value;
        A[cc] = fnmac_row_v<cc % 16>(A[cc], R[cc / 16], wsl);
      });
      sfor<8>([&](auto ii) {
        constexpr int cc = cb + decltype(ii)::value;
        A[cc] = fnmac_row_v<cc % 16>(A[cc], W[cc / 16], v);
      });
      // column j + 1 (group gj, the first live group of half gj & 1) is final: phase A of the
      // next step
      if constexpr (gg == 0 && hh == (gj & 1) && gj < 8) {
        if (j1 < jend) phase_a(j1, GJ);
      }
    });
  };
  if (h == 0) phase_a(0, std::integral_constant<int, 0>{});  // column 0: half 0, group 0
  auto run = [&](auto H) {
    sfor<9>([&](auto GJ) {  // j + 1 <= 64: groups 0 .. 8
      constexpr int gj = decltype(GJ)::value;
      for (int j = gj == 0 ? 0 : 8 * gj - 1; j <= min(8 * gj + 6, jend - 1); ++j) step(j, GJ, H);
    });
  };
  if (h == 0) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, 1>{});

  // ---- hand-off (BigHandoff): the trailing 64x64 (wave 3's half rows), Q^T b1, Q^T x', T ----
  if (rb == 1) {  // columns 64..127: local columns 32..63 of either half
    sfor<32>([&](auto CC_) {
      constexpr int cc = 32 + decltype(CC_)::value;
      wo[HO::TA + (gcol(h, cc) - 64) * HO::KT + l] = A[cc];  // (r, c) at c KT + r
    });
  }
  if (h == 0) {
    wo[HO::U1 + r] = ub;
    wo[HO::U2 + r] = ux;
  }
  __syncthreads();  // d, e, tau of the last steps
  if (tid < HS) {
    wo[HO::D + tid] = sm.d[tid];
    wo[HO::E + tid] = sm.e[tid + 1];
    wo[HO::TAU + tid] = sm.tau[tid];
  }
  if (tid == 0) info[gi] = make_int2(ptot, 0);
}

hipError_t launch_rows_handoff(hipStream_t s, const TreeDesc *trees, SolveConsts c, SlabDev slab,
                               long long g0, int npts, const int *nbr_cnt, const int *nbr_idx,
                               int2 *info, double *ws) {
  if (npts <= 0) return hipSuccess;
  if (c.k <= kRowsHS + 2 || c.k > kRowsKP) return hipErrorInvalidValue;
  hipLaunchKernelGGL((solve_tq_rows_kernel<kRowsKP, kRowsHS>), dim3(npts), dim3(256), 0, s, trees,
                     c, slab, g0, npts, nbr_cnt, nbr_idx, info, ws);
  return hipGetLastError();
}

}  // namespace cwbl
