// cwbl_tq_big.hip — solve_tq_big_kernel<KP>: the Householder + quadrature solve of
// cwbl_tq.hip for large ensembles (KP = 96, 128; configs[3] is k = 128), one 256-thread
// workgroup (4 waves) per grid point.
//
// Same algorithm as solve_tq_kernel (see there for the derivation and the reference lines);
// what changes with k:
//   - the k x k matrix lives in 4x4 register blocks spread over 256 threads (NBL blocks per
//     thread), assembled on the VALU (the MFMA tile set of Y'Y'^T would not fit in registers);
//   - reductions are wave reductions followed by a 4-entry exchange through LDS;
//   - the Householder vectors are kept in registers, in the entries of column j that the
//     tridiagonalisation no longer reads (rows > j+1 of block column j/4), and published
//     again for the back-transform;
//   - the shifted tridiagonal solves of the quadrature run on wave 0 (lane pairs, twisted
//     factorisation) with the forward sweep checkpointed every 8 rows and recomputed per
//     segment in the backward sweep, so a lane holds 64 rows in 64 VGPRs;
//   - the reference's sequential fp32 member sums run wave after wave.
#include "cwbl_device.h"

#include <type_traits>

namespace cwbl {

constexpr int kBigThreads = 256;
// columns staged per chunk: 64 at KP = 128 on the one-kernel path, so that a chunk's MFMA
// phase (two waves per SIMD) is long enough to cover the next chunk's gathers
// (stage_columns_pipe); 32 on the hand-off path, whose LDS then allows three workgroups per CU
template <int KP, int HS>
constexpr int kBigChunk = KP == 128 && HS == 0 ? 64 : 32;
// waves per SIMD the register budget is sized for: the hand-off kernels fit 168 VGPRs (three
// workgroups per CU); the one-kernel path keeps 256 for the back-transform's registers
template <int HS>
constexpr int kBigWaves = HS > 0 ? 3 : 1;

// thread -> 4x4 blocks of the lower block triangle for the tridiagonalisation's benefit.
// Blocks are numbered column-major over the triangle; block (bi, bj) is read and updated
// while the step's block column J <= bj, so contiguous runs retire together.  A thread's
// blocks come in 64-block slots, one per (wave, it):
//   - the last `it` is partial (lanes < NBLK - 256 (NBL-1) - 64 wave, the same lanes as
//     assemble_point's `tid + 256 it < NBLK`) and takes the first, shortest-lived blocks;
//   - the full slots, in ascending lifetime s_0 .. s_{F-1}, are dealt snake-wise (it 0:
//     wave w -> s_{F-1-w}, it 1: s_w, it 2: s_{F-5-w}), so every wave pairs a long-lived slot
//     with a short-lived one and no wave carries the trailing matrix alone.
// At k = 128 the heaviest wave runs 144 slot-steps of matvec + update instead of ~340 with
// the row-major numbering (whose first slot holds rows that live to the last step).
template <int KP>
__device__ __forceinline__ void big_block_of_lane(int tid, int (&bi)[AsmLayout<KP, 256>::NBL],
                                                  int (&bj)[AsmLayout<KP, 256>::NBL]) {
  using L = AsmLayout<KP, 256>;
  constexpr int NB = L::NB, NBL = L::NBL, F = 4 * (NBL - 1);
  constexpr int R = L::NBLK - 256 * (NBL - 1);  // blocks in the partial slots
  static_assert(NBL >= 1 && NBL <= 3 && R > 0, "slot plan");
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int it = 0; it < NBL; ++it) {
    int s;  // full-slot rank by lifetime
    if (it == 0) s = F - 1 - wave;
    else if (it == 1) s = wave;
    else s = F - 5 - wave;
    int b = it == NBL - 1 ? 64 * wave + lane : R + 64 * s + lane;
    if (b >= L::NBLK) b = L::NBLK - 1;  // invalid lane of a partial slot (never used)
    int cj = 0;
    while (b >= NB - cj) {  // column cj holds blocks bi = cj .. NB-1
      b -= NB - cj;
      ++cj;
    }
    bj[it] = cj;
    bi[it] = cj + b;
  }
}

// last block column of the partial slot NBL - 1 (blocks 0 .. R-1 in column-major order)
template <int KP>
constexpr int big_partial_last_column() {
  using L = AsmLayout<KP, 256>;
  int b = L::NBLK - 256 * (L::NBL - 1) - 1, cj = 0;
  while (b >= L::NB - cj) {
    b -= L::NB - cj;
    ++cj;
  }
  return cj;
}
static_assert(big_partial_last_column<128>() == 0 && big_partial_last_column<96>() == 1, "JP");

template <int KP, int CHK>
struct BigSmem {
  static constexpr int NB = KP / 4;
  static constexpr int PLD = 4 * NB + 4;  // 2*PLD = 8*odd dwords: conflict-free row sums
  union {
    // staged columns (two buffers: stage_columns_pipe); odd columns' rows XOR 16 at KP = 128
    ColumnChunk<KP, CHK, float, KP, false, KP == 128> ch[2];
    double pb[NB][PLD];                   // A v partials: pb[R][4c+r] = block (R,c), row r
  } u;
  double col[KP];                         // pivot column / reflector j (back-transform)
  double col2[KP];                        // reflector j-1 (back-transform)
  double vb[KP], wb[KP];                  // v and w of the current step; Yb d before
  double tq[KP + 1][4];                   // d_i, c(i-1,i), (Q^T b1)_i, (Q^T x')_i
  double Ym[KP], Zm[KP];                  // quadrature sum / exact solve, walk order
  double tau[KP];
  double red[2][4][4];                    // [buffer][wave][value] of the block reductions
  double red10[4][10];                    // [wave][value]: back-transform group reduction
  double pard;                            // sequential-sum partial handed wave to wave
  float parf;
  int ptot;
};

// HS > 0 (slab path, KP = kBigSplitKP): stop after HS Householder steps and hand the rest
// over through ws (BigHandoff<KP, HS>) to solve_tqb_tail_kernel.
template <int KP, bool ASSEMBLED, int HS = 0>
__global__ void __launch_bounds__(kBigThreads, kBigWaves<HS>)
solve_tq_big_kernel(const TreeDesc *__restrict__ trees, SolveConsts c, SlabDev slab,
                    long long g0, int npts, const int *__restrict__ nbr_cnt,
                    const int *__restrict__ nbr_idx, const long long *__restrict__ col_off,
                    const float *__restrict__ yo_in, const float *__restrict__ yb_in,
                    const float *__restrict__ xb_in, float *__restrict__ xa_out,
                    int2 *__restrict__ info, double *__restrict__ ws = nullptr) {
  constexpr int NT = kBigThreads;
  constexpr int H = KP / 2;
  using L = AsmLayout<KP, NT>;
  constexpr int NBL = L::NBL, NBLK = L::NBLK;
  constexpr int CHK = kBigChunk<KP, HS>;
  using SM = BigSmem<KP, CHK>;
  static_assert(KP % 8 == 0 && KP <= 2 * 64 && H % 8 == 0, "KP");
  __shared__ SM sm;

  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k = c.k;

  // ---- block reductions: 4 values, wave sums + exchange through LDS (one barrier) ---------
  int rbuf = 0;
  auto bsum4 = [&](double &a, double &b, double &cc, double &d) {
    wave_sum4_dpp(a, b, cc, d);
    double(*r)[4] = sm.red[rbuf];
    rbuf ^= 1;
    if (lane == 0) {
      r[wave][0] = a; r[wave][1] = b; r[wave][2] = cc; r[wave][3] = d;
    }
    __syncthreads();
    a = (r[0][0] + r[1][0]) + (r[2][0] + r[3][0]);
    b = (r[0][1] + r[1][1]) + (r[2][1] + r[3][1]);
    cc = (r[0][2] + r[1][2]) + (r[2][2] + r[3][2]);
    d = (r[0][3] + r[1][3]) + (r[2][3] + r[3][3]);
  };
  // the reference's sequential member-order sums (member m lives in thread m), wave by wave
  auto seq_sum_f32 = [&](float x) {
    for (int w = 0; 64 * w < k; ++w) {
      if (wave == w) {
        float s = w == 0 ? 0.0f : sm.parf;
        const int n = min(64, k - 64 * w);
        for (int m = 0; m < n; ++m)
          s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), m));
        if (lane == 0) sm.parf = s;
      }
      __syncthreads();
    }
    const float s = sm.parf;
    __syncthreads();
    return s;
  };
  auto seq_sumsq_f64 = [&](double x) {
    for (int w = 0; 64 * w < k; ++w) {
      if (wave == w) {
        double s = w == 0 ? 0.0 : sm.pard;
        const int n = min(64, k - 64 * w);
        for (int m = 0; m < n; ++m) {
          const double v = readlane_f64(x, m);
          s = s + v * v;
        }
        if (lane == 0) sm.pard = s;
      }
      __syncthreads();
    }
    const double s = sm.pard;
    __syncthreads();
    return s;
  };

  long long P = 0;
  float3 pt = make_float3(0.0f, 0.0f, 0.0f);
  float xbl = 0.0f;  // background of member `tid`
  if constexpr (!ASSEMBLED) {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long r = g / slab.ix_lim;
    const int j = (int)(r % slab.iy_lim);
    const int kz = (int)(r / slab.iy_lim);
    P = i + (long long)slab.nx * (j + (long long)slab.ny * kz);
    if (tid < k) xbl = slab.var[P + slab.L * tid];
    slab_point(slab, g, pt.x, pt.y, pt.z);
  } else {
    if (tid < k) xbl = xb_in[(long long)gi * k + tid];
  }

  int bi[NBL], bj[NBL];
  big_block_of_lane<KP>(tid, bi, bj);
  double acc[NBL][16];
  double b1acc;
  int ptot;
  if constexpr (KP == 128) {
    // Matrix-core assembly (v_mfma_f64_16x16x4_f64): the 36 lower 16x16 tiles of Yb Yb^T,
    // nine per wave: wave w owns tile rows w and 7-w (tiles (w, 0..w) and (7-w, 0..7-w)).
    // The VALU form reads two float4 of the chunk from LDS per 16 FMAs and is LDS-bound;
    // here a lane reads 11 floats per 4 columns for 9 MFMAs.  Then the tiles go through
    // LDS, 16 at a time, into the 4x4 register blocks of the tridiagonalisation.
    constexpr int NTW = 9;
    static_assert(sizeof(sm.u.pb) >= 16 * 256 * sizeof(double), "tile staging area");
    f64x4 tile[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) tile[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    double b1p[4] = {0.0, 0.0, 0.0, 0.0};
    const int m = lane & 15, kk = lane >> 4;
    const int offA = 16 * wave + m, offB = 16 * (7 - wave) + m;
    int offJ[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) offJ[t] = 16 * (t <= wave ? t : t - wave - 1) + m;
    // columns past nsl are staged as zeros (a multiple of 4 stays inside the chunk)
    // (debug_stop 12: staging only, timing ablation)
    // the rows of column 4 g + kk are XOR 16 for odd kk (ColumnChunk XSW): the lane's offsets
    // take it once
    using CC = std::remove_reference_t<decltype(sm.u.ch[0])>;
    const int xk = CC::xr(kk);
    const int offAx = offA ^ xk, offBx = offB ^ xk;
    int offJx[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) offJx[t] = offJ[t] ^ xk;
    auto mfma_chunk = [&](int nsl, const CC &cb) {
      // (software-pipelining the group loop, group g + 1's operand reads before group g's
      // MFMAs, measured no faster: 2.52 s per C4 variable either way)
      for (int s0 = 0; s0 < (CWBL_DBG_STOP(c) == 12 ? 0 : nsl); s0 += 4) {
        const float *ys = cb.yb[s0 + kk];
        const double a = (double)ys[offAx], b = (double)ys[offBx];
#pragma unroll
        for (int t = 0; t < NTW; ++t)
          tile[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(t <= wave ? a : b, (double)ys[offJx[t]],
                                                         tile[t], 0, 0, 0);
      }
      // Yb d (row KP of [Yb; yo] does not fit the tile padding): eight columns per round,
      // their LDS reads issued together, four chains (the staged columns past nsl are zeros)
      if (tid < KP) {
        constexpr int CH = CHK;
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
        static_assert(CH % 8 == 0, "Yb d rounds");
      }
    };
    if constexpr (!ASSEMBLED)
      ptot = stage_columns_pipe<KP, CHK, NT>(sm.u.ch, trees, c, gi, tid, nbr_cnt, nbr_idx,
                                                   pt, mfma_chunk);
    else
      ptot = stage_columns<KP, CHK, ASSEMBLED, NT>(
          sm.u.ch[0], trees, c, gi, tid, nbr_cnt, nbr_idx, pt, col_off, yo_in, yb_in,
          [&](int nsl) { mfma_chunk(nsl, sm.u.ch[0]); });
    b1acc = (b1p[0] + b1p[1]) + (b1p[2] + b1p[3]);
    // block (bi, bj) lies in tile (I, J) = (bi/4, bj/4), held by wave min(I, 7-I) as its
    // tile t = J (I <= 3) or 8 - I + J (I >= 4); staged in round t/4, slot 4 wave + t%4
    int rnd[NBL], off[NBL];
#pragma unroll
    for (int it = 0; it < NBL; ++it) {
      const int I = bi[it] >> 2, J = bj[it] >> 2;
      const int wI = I <= 3 ? I : 7 - I, t = I <= 3 ? J : 8 - I + J;
      rnd[it] = t >> 2;
      off[it] = (4 * wI + (t & 3)) * 256 + (4 * (bi[it] & 3)) * 16 + 4 * (bj[it] & 3);
    }  // (no zero fill: a slot is read only where tid + NT it < NBLK, and a fill would keep all
       // of acc live beside the tiles)
    double *tl = &sm.u.pb[0][0];
#pragma unroll
    for (int rd = 0; rd < 3; ++rd) {
      __syncthreads();  // the chunk / the previous round's readers are done
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int t = 4 * rd + tt;
        if (t < NTW) {
          double *dst = tl + (4 * wave + tt) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) dst[(kk + 4 * r) * 16 + m] = tile[t][r];
        }
      }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < NBL; ++it) {
        if (tid + NT * it < NBLK && rnd[it] == rd) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double *src = tl + off[it] + 16 * r;
            const double2 x0 = *reinterpret_cast<const double2 *>(src);
            const double2 x1 = *reinterpret_cast<const double2 *>(src + 2);
            acc[it][4 * r] = x0.x; acc[it][4 * r + 1] = x0.y;
            acc[it][4 * r + 2] = x1.x; acc[it][4 * r + 3] = x1.y;
          }
        }
      }
    }
  } else {
    assemble_point<KP, CHK, ASSEMBLED, NT>(sm.u.ch[0], trees, c, gi, tid, nbr_cnt, nbr_idx,
                                                 pt, col_off, yo_in, yb_in, bi, bj, acc, b1acc,
                                                 ptot);
  }
  if (tid == 0) sm.ptot = ptot;  // counted by wave 0
  __syncthreads();
  ptot = sm.ptot;
  if (ptot == 0) {  // no accepted observation: var left unchanged (:220, :226)
    if (tid == 0 && info) info[gi] = make_int2(0, 0);
    if constexpr (ASSEMBLED) {
      if (tid < k) xa_out[(long long)gi * k + tid] = xbl;
      if (ws && tid < KP) {  // T = A = inflat I (no observation)
        ws[(long long)gi * 2 * KP + tid] = tid < k ? (double)c.inflat : 1.0;
        ws[(long long)gi * 2 * KP + KP + tid] = 0.0;
      }
    }
    return;
  }

  if (CWBL_DBG_STOP(c) == 1 || CWBL_DBG_STOP(c) >= 12) {  // timing ablation: assembly only
    double t = b1acc;
#pragma unroll
    for (int it = 0; it < NBL; ++it)
      if (tid + NT * it < NBLK) t += acc[it][0] + acc[it][15];
    if (tid == 0 && info) info[gi] = make_int2(ptot, (int)t);
    return;
  }
  const double inflat_r8 = (double)c.inflat;
#pragma unroll
  for (int it = 0; it < NBL; ++it) {
    if (tid + NT * it < NBLK && bi[it] == bj[it]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = 4 * bi[it] + r;
        acc[it][5 * r] = ii < k ? acc[it][5 * r] + inflat_r8 : 1.0;
      }
    }
  }
  if (tid < KP) {  // padding of T: decoupled unit rows
    sm.tq[tid][0] = 1.0;
    sm.tq[tid][1] = 0.0;
    sm.tau[tid] = 0.0;
  }
  if (tid == 0) sm.tq[KP][1] = 0.0;
  const double xb_mean = (double)(seq_sum_f32(xbl) * c.nmember_inv);  // fp32 (:671)
  double ux = (tid < k) ? (double)xbl - xb_mean : 0.0;                 // x', then Q^T x'
  double ub = (tid < KP) ? b1acc : 0.0;                                // Yb d, then Q^T b1

  auto ld4 = [](const double *p, double (&o)[4]) {
    const double2 a0 = *reinterpret_cast<const double2 *>(p);
    const double2 a1 = *reinterpret_cast<const double2 *>(p + 2);
    o[0] = a0.x; o[1] = a0.y; o[2] = a1.x; o[3] = a1.y;
  };
  // The step's 4-value groups in LDS (v, w: group x = rows 4x..4x+3; the A v partials: block
  // row R) keep their two halves swapped when bit 3 of the group index is set (hsw), so that
  // the 16 lanes of a 16-B access, whose groups are mostly 16 consecutive ones (32 B apart),
  // hit all 64 banks once instead of half of them twice (r4: LDS bank conflicts were 82% of
  // the kernel's LDS-active cycles, profiles/r4n_c4_sq_counters.txt).  Element i of v or w
  // lives at i ^ (hsw(i >> 2) << 1).
  auto hsw = [](int x) { return (x >> 3) & 1; };
  auto ld4s = [](const double *p, int sw, double (&o)[4]) {  // logical half 0 at p + 2 sw
    const double2 a0 = *reinterpret_cast<const double2 *>(p + 2 * sw);
    const double2 a1 = *reinterpret_cast<const double2 *>(p + 2 - 2 * sw);
    o[0] = a0.x; o[1] = a0.y; o[2] = a1.x; o[3] = a1.y;
  };
  auto st4s = [](double *p, int sw, double a0, double a1, double a2, double a3) {
    *reinterpret_cast<double2 *>(p + 2 * sw) = make_double2(a0, a1);
    *reinterpret_cast<double2 *>(p + 2 - 2 * sw) = make_double2(a2, a3);
  };
  const int tsw = tid ^ (hsw(tid >> 2) << 1);  // this thread's element of v and w
  // column j of the lower block triangle -> dst (4 rows per block of block column j/4); the
  // column within the block is uniform, so a switch picks it (no per-value selects)
  auto pub4 = [](double *d, double a0, double a1, double a2, double a3) {
    *reinterpret_cast<double2 *>(d) = make_double2(a0, a1);
    *reinterpret_cast<double2 *>(d + 2) = make_double2(a2, a3);
  };
  // (QJ: the column within the block, static: the steps run four to a block column)
  auto publish = [&](int J_, auto QJ, auto NS, const int (&bI)[NBL], const int (&bJ)[NBL],
                     double *dst) {
    constexpr int q_ = decltype(QJ)::value;
#pragma unroll
    for (int it = 0; it < decltype(NS)::value; ++it) {
      if (tid + NT * it < NBLK && bJ[it] == J_) {
        const double *a_ = acc[it];
        pub4(&dst[4 * bI[it]], a_[q_], a_[4 + q_], a_[8 + q_], a_[12 + q_]);
      }
    }
  };

  // ---- Householder tridiagonalisation ----------------------------------------------------
  double trace = 0.0;
  static_assert(HS == 0 || (!ASSEMBLED && HS % 4 == 0 && HS + 4 <= KP), "hand-off step");
  // (k > HS + 2 on the split path: every hand-off step is a full step)
  // (debug_steps: timing ablation, the first steps only; the hand-off then carries a partial
  // reduction)
  const int jend = CWBL_DBG_STEPS(c) > 0 ? min(HS > 0 ? HS : k, CWBL_DBG_STEPS(c)) : HS > 0 ? HS : k;
  // NS: the slots a step visits (static).  The partial slot NBL - 1 holds only blocks of block
  // columns <= JP, so the steps past block column JP leave it out and its registers are free
  auto step = [&](const int j, auto QJ, auto NS) {
    constexpr int ns = decltype(NS)::value;
    // the slots' block indices through opaque registers: the LDS addresses formed from them
    // live for one step, not for the whole loop (hoisted, they did not fit 168 VGPRs)
    int bI[NBL], bJ[NBL];
#pragma unroll
    for (int it = 0; it < NBL; ++it) {
      bI[it] = opaque_int(bi[it]);
      bJ[it] = opaque_int(bj[it]);
    }
    constexpr int qj = decltype(QJ)::value;
    const int J = j >> 2;
    // The previous full step read col only before its three later barriers, so only the
    // step after the (barrier-free) trailing step k-2 needs one here.
    if (j >= k - 1) __syncthreads();
    publish(J, QJ, NS, bI, bJ, sm.col);
    // x.x (x = column j below row j + 1) from the owners' registers, reduced with the publish
    // barrier.  Rows >= k hold exact zeros in columns < k, so no row bound is needed.
    {
      double xs = 0.0;
#pragma unroll
      for (int it = 0; it < ns; ++it) {
        if (tid + NT * it < NBLK && bJ[it] == J) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {  // row 4 bI + r > j + 1
            const bool below = bI[it] > J + 1 || (bI[it] == J ? r > qj + 1 : r > qj - 3);
            const double a = acc[it][4 * r + qj];
            xs = below ? fma(a, a, xs) : xs;
          }
        }
      }
      xs = wave_sum_dpp(xs);
      if (lane == 0) sm.red[rbuf][wave][0] = xs;
    }
    __syncthreads();
    const double xn2 = (sm.red[rbuf][0][0] + sm.red[rbuf][1][0]) +
                       (sm.red[rbuf][2][0] + sm.red[rbuf][3][0]);
    rbuf ^= 1;
    const double dj = sm.col[j];
    trace += dj;
    if (tid == 0) sm.tq[j][0] = dj;
    if (j >= k - 2) {  // trailing 2x2 block: already tridiagonal
      if (j == k - 2 && tid == 0) sm.tq[j + 1][1] = sm.col[j + 1];
      return;
    }
    const double x = (tid > j + 1 && tid < k) ? sm.col[tid] : 0.0;
    const double alpha = sm.col[j + 1];
    double tau = 0.0, beta = alpha, scal = 0.0;
    if (xn2 > 0.0) {  // dlarfg, fp64 rcp/rsq refined to ~1 ulp
      const double a2 = fma(alpha, alpha, xn2);
      const double r = rsq64(a2);             // 1/|beta|
      beta = -copysign(a2 * r, alpha);
      tau = (beta - alpha) * -copysign(r, alpha);  // (beta - alpha) / beta
      scal = rcp64(alpha - beta);
    }
    if (tid == 0) {
      sm.tq[j + 1][1] = beta;
      sm.tau[j] = tau;
    }
    // tau = 0 (H_j = I) runs the step too, as an exact no-op (w = 0): dead blocks (bj < J)
    // are skipped below, and the row sums rely on every block's last live step
    // (j = 4 bj + 3, where v vanishes on its columns) leaving exact zeros in its A v partials.
    const double v = tid == j + 1 ? 1.0 : x * scal;
    if (tid < KP) sm.vb[tsw] = v;
    __syncthreads();
    double s1p = 0.0;
#pragma unroll
    for (int it = 0; it < ns; ++it) {
      if (tid + NT * it < NBLK && bJ[it] >= J) {
        double vi[4], vj[4];
        ld4s(&sm.vb[4 * bI[it]], hsw(bI[it]), vi);
        ld4s(&sm.vb[4 * bJ[it]], hsw(bJ[it]), vj);
        double pr[4], pc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pr[r] = acc[it][4 * r] * vj[0];
#pragma unroll
          for (int q = 1; q < 4; ++q) pr[r] = fma(acc[it][4 * r + q], vj[q], pr[r]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pc[q] = acc[it][q] * vi[0];
#pragma unroll
          for (int r = 1; r < 4; ++r) pc[q] = fma(acc[it][4 * r + q], vi[r], pc[q]);
        }
        double sp = vi[0] * pr[0];
#pragma unroll
        for (int r = 1; r < 4; ++r) sp = fma(vi[r], pr[r], sp);
        st4s(&sm.u.pb[bI[it]][4 * bJ[it]], hsw(bI[it]), pr[0], pr[1], pr[2], pr[3]);
        if (bI[it] != bJ[it]) {
          if (bJ[it] >= J)
            st4s(&sm.u.pb[bJ[it]][4 * bI[it]], hsw(bJ[it]), pc[0], pc[1], pc[2], pc[3]);
          sp = sp + sp;
        }
        s1p += sp;
      }
    }
    // v.A v, v.x', v.b1 in one reduction (its barrier also publishes pb)
    double s2 = v * ux, s3 = v * ub, z3 = 0.0;
    bsum4(s1p, s2, s3, z3);
    ux = fma(-tau * s2, v, ux);
    ub = fma(-tau * s3, v, ub);
    const double s1 = s1p * tau;  // p . v with p = tau A v
    double pp = 0.0;
    if (tid < KP && tid > j) {
      const double *prow = &sm.u.pb[tid >> 2][tsw & 3];
      // block columns < J hold exact zeros (dead blocks): start at the 8-column segment of J
      auto rsum = [&](auto C) {
        constexpr int c0 = decltype(C)::value;
        double t = 0.0;
#pragma unroll
        for (int cb = c0; cb < SM::NB; ++cb) t += prow[4 * cb];
        return t;
      };
      const int seg = J >> 3;
      if (seg >= 3 && SM::NB > 24) pp = rsum(std::integral_constant<int, (SM::NB > 24 ? 24 : 0)>{});
      else if (seg >= 2) pp = rsum(std::integral_constant<int, 16>{});
      else if (seg >= 1) pp = rsum(std::integral_constant<int, 8>{});
      else pp = rsum(std::integral_constant<int, 0>{});
    }
    const double p = (tid > j && tid < k) ? tau * pp : 0.0;
    const double w = fma(-0.5 * tau * s1, v, p);
    if (tid < KP) sm.wb[tsw] = w;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ns; ++it) {
      if (tid + NT * it < NBLK && bJ[it] >= J) {
        double vi[4], vj[4], wi[4], wj[4];
        ld4s(&sm.vb[4 * bI[it]], hsw(bI[it]), vi);
        ld4s(&sm.vb[4 * bJ[it]], hsw(bJ[it]), vj);
        ld4s(&sm.wb[4 * bI[it]], hsw(bI[it]), wi);
        ld4s(&sm.wb[4 * bJ[it]], hsw(bJ[it]), wj);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[it][4 * r + q] = fma(-vi[r], wj[q], fma(-wi[r], vj[q], acc[it][4 * r + q]));
        if (bJ[it] == J) {  // keep v_j in the entries of column j the steps no longer read
          const int r0 = j + 2 - 4 * bI[it];  // rows r >= r0 of the block
          auto keep = [&](auto Q) {
            constexpr int q = decltype(Q)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[it][4 * r + q] = r >= r0 ? vi[r] : acc[it][4 * r + q];
          };
          keep(QJ);
        }
      }
    }
  };
  auto block_column = [&](int j0, auto NS) {  // four steps per block column: qj static
    step(j0, std::integral_constant<int, 0>{}, NS);
    if (j0 + 1 < jend) step(j0 + 1, std::integral_constant<int, 1>{}, NS);
    if (j0 + 2 < jend) step(j0 + 2, std::integral_constant<int, 2>{}, NS);
    if (j0 + 3 < jend) step(j0 + 3, std::integral_constant<int, 3>{}, NS);
  };
  // hand-off (BigHandoff) of slot it's blocks: trailing blocks as the full matrix, the others
  // as reflector columns
  auto handoff_slot = [&](auto IT) {
    constexpr int it = decltype(IT)::value;
    using HO = BigHandoff<KP, (HS > 0 ? HS : 4)>;
    constexpr int KT = HO::KT, JB = HS / 4;
    double *__restrict__ w = ws + (long long)gi * HO::WORDS;
    {
      if (tid + NT * it < NBLK) {
        if (bj[it] >= JB) {  // trailing block: both triangles of the full KT x KT matrix
          const int a0 = 4 * (bi[it] - JB), b0 = 4 * (bj[it] - JB);
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // column b0 + q, rows a0 .. a0 + 3
            double *d = w + HO::TA + (b0 + q) * KT + a0;
            pub4(d, acc[it][q], acc[it][4 + q], acc[it][8 + q], acc[it][12 + q]);
          }
          if (bi[it] != bj[it]) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // column a0 + r, rows b0 .. b0 + 3
              double *d = w + HO::TA + (a0 + r) * KT + b0;
              pub4(d, acc[it][4 * r], acc[it][4 * r + 1], acc[it][4 * r + 2], acc[it][4 * r + 3]);
            }
          }
        } else {  // reflector columns j = 4 bj + q: v_j at rows > j (1 at row j + 1)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int j = 4 * bj[it] + q, a0 = 4 * bi[it];
            double e[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int a = a0 + r;
              e[r] = a == j + 1 ? 1.0 : a > j + 1 ? acc[it][4 * r + q] : 0.0;
            }
            pub4(w + HO::HV + j * KP + a0, e[0], e[1], e[2], e[3]);
          }
        }
      }
    }
  };
  constexpr int JP = big_partial_last_column<KP>();
  int j0 = 0;
  for (; j0 < jend && j0 < 4 * (JP + 1); j0 += 4) block_column(j0, std::integral_constant<int, NBL>{});
  // on the hand-off path the partial slot's blocks (reflector columns <= JP) go out now, so that
  // its registers are free for the remaining steps
  if constexpr (HS > 0) handoff_slot(std::integral_constant<int, NBL - 1>{});
  for (; j0 < jend; j0 += 4) block_column(j0, std::integral_constant<int, NBL - 1>{});
  if constexpr (HS > 0) {  // hand-off (BigHandoff) after HS steps
    using HO = BigHandoff<KP, HS>;
    static_assert(JP < HS / 4, "the partial slot holds reflector columns only");
    double *__restrict__ w = ws + (long long)gi * HO::WORDS;
    __syncthreads();  // T, tau of the last steps are in LDS
    sfor<NBL - 1>([&](auto IT) { handoff_slot(IT); });
    if (tid < KP) {
      w[HO::U1 + tid] = ub;
      w[HO::U2 + tid] = ux;
    }
    if (tid < HS) {
      w[HO::D + tid] = sm.tq[tid][0];
      w[HO::E + tid] = sm.tq[tid + 1][1];
      w[HO::TAU + tid] = sm.tau[tid];
    }
    if (tid == 0) info[gi] = make_int2(ptot, 0);
    return;
  }
  if (tid < KP) {
    sm.tq[tid][2] = ub;
    sm.tq[tid][3] = ux;
  }
  __syncthreads();
  if constexpr (ASSEMBLED && HS == 0) {  // T for the eigenvalue output (cwbl_solve_batch)
    if (ws && tid < KP) {
      ws[(long long)gi * 2 * KP + tid] = sm.tq[tid][0];           // d_i
      ws[(long long)gi * 2 * KP + KP + tid] = sm.tq[tid + 1][1];  // c(i, i+1)
    }
  }

  if (CWBL_DBG_STOP(c) == 2) {
    if (tid == 0 && info) info[gi] = make_int2(ptot, (int)(trace + ux + ub));
    return;
  }
  // ---- T^-1/2 u2 by quadrature (wave 0), u1^T T^-1 u2 exactly ----------------------------
  const double m = inflat_r8;
  const double ratio = trace / m - (double)(k - 1);
  int level = 1;
  double dec = 10.0;
  while (level < kQuadLevels && dec < ratio) {
    dec *= 10.0;
    ++level;
  }
  if (wave == 0) {
    const int node = lane & 31, side = lane >> 5;
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
    const unsigned csb = side ? 40u : 8u;  // coupling with the previous mirrored row
    // one row of the forward elimination (identical in both sweeps)
    auto fwd = [&](int t, double &dl, double &gt) {
      const unsigned o = opaque_after(q0, dl) + dirb * (unsigned)t;
      const double ct = lds_at(sm.tq, o + csb);
      const double l = ct * rcp64(dl);
      dl = fma(-l, ct, lds_at(sm.tq, o) + sigma);
      gt = fma(-l, gt, lds_at(sm.tq, o + 24));
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
    // meeting rows H-1 (top) and H (bottom)
    const double cm = sm.tq[H][1];
    const double dlo = __shfl_xor(dl, 32, 64), go = __shfl_xor(gt, 32, 64);
    double xv = (gt * dlo - cm * go) / fma(dl, dlo, -cm * cm);
    double *ym = sm.Ym + side * H, *zm = sm.Zm + side * H;
    for (int s = NS - 1; s >= 0; --s) {  // recompute the segment, then substitute back
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
  const int wi = tid < H ? tid : H + (KP - 1 - tid);
  const double zl = tid < KP ? sm.Zm[wi] : 0.0;
  double yl = tid < KP ? sm.Ym[wi] : 0.0;
  double dsum = tid < KP ? sm.tq[tid][2] * zl : 0.0, z5 = 0.0, z6 = 0.0, z7 = 0.0;
  bsum4(dsum, z5, z6, z7);
  const double d = dsum;  // wbar . x' = u1 . T^-1 u2
  if (CWBL_DBG_STOP(c) == 3) {
    if (tid == 0 && info) info[gi] = make_int2(ptot, (int)d);
    return;
  }

  // ---- back-transform y <- Q y = H_0 H_1 ... H_{k-3} y, four reflectors per reduction ------
  // The reflectors of block column J live in the owners' registers (blocks (bi, J)), so a
  // group of four is applied where it lies: the owners form v_q . y and v_q . v_p (q < p)
  // from their rows (one 10-value reduction), every thread turns them into the coefficients
  // of y -= sum_q c_q v_q (H_{4J+3} first), and the owners update their rows of y in LDS.
  // Two barriers per four reflectors, and no reflector is published.
  // First the register entries become exact reflector entries: 1 at row j+1, 0 at and above
  // the diagonal (T is already in sm.tq).
#pragma unroll
  for (int it = 0; it < NBL; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 4 * bi[it] + r, col = 4 * bj[it] + q;
        acc[it][4 * r + q] = row == col + 1 ? 1.0 : row > col + 1 ? acc[it][4 * r + q] : 0.0;
      }
  }
  double *ys = sm.col;
  if (tid < KP) ys[tid] = yl;
  for (int JJ = (k - 3) >> 2; JJ >= 0 && k >= 3; --JJ) {
    __syncthreads();  // y rows of the previous group are written
    double dq[4] = {0.0, 0.0, 0.0, 0.0}, g[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int it = 0; it < NBL; ++it) {
      if (tid + NT * it < NBLK && bj[it] == JJ) {
        double yr[4];
        ld4(&ys[4 * bi[it]], yr);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double *V = &acc[it][4 * r];
#pragma unroll
          for (int q = 0; q < 4; ++q) dq[q] = fma(V[q], yr[r], dq[q]);
          g[0] = fma(V[0], V[1], g[0]);
          g[1] = fma(V[0], V[2], g[1]);
          g[2] = fma(V[0], V[3], g[2]);
          g[3] = fma(V[1], V[2], g[3]);
          g[4] = fma(V[1], V[3], g[4]);
          g[5] = fma(V[2], V[3], g[5]);
        }
      }
    }
    double z0 = 0.0, z1 = 0.0;
    wave_sum4_dpp(dq[0], dq[1], dq[2], dq[3]);
    wave_sum4_dpp(g[0], g[1], g[2], g[3]);
    wave_sum4_dpp(g[4], g[5], z0, z1);
    if (lane == 0) {
      double *rw = sm.red10[wave];
      rw[0] = dq[0]; rw[1] = dq[1]; rw[2] = dq[2]; rw[3] = dq[3];
      rw[4] = g[0]; rw[5] = g[1]; rw[6] = g[2]; rw[7] = g[3]; rw[8] = g[4]; rw[9] = g[5];
    }
    __syncthreads();
    double t[10];
#pragma unroll
    for (int e = 0; e < 10; ++e)
      t[e] = (sm.red10[0][e] + sm.red10[1][e]) + (sm.red10[2][e] + sm.red10[3][e]);
    // t: d0..d3, G01 G02 G03 G12 G13 G23
    const double tau0 = sm.tau[4 * JJ], tau1 = sm.tau[4 * JJ + 1];
    const double tau2 = sm.tau[4 * JJ + 2], tau3 = sm.tau[4 * JJ + 3];
    const double c3 = tau3 * t[3];
    const double c2 = tau2 * fma(-c3, t[9], t[2]);
    const double c1 = tau1 * fma(-c3, t[8], fma(-c2, t[7], t[1]));
    const double c0 = tau0 * fma(-c3, t[6], fma(-c2, t[5], fma(-c1, t[4], t[0])));
#pragma unroll
    for (int it = 0; it < NBL; ++it) {
      if (tid + NT * it < NBLK && bj[it] == JJ) {
        double yr[4];
        ld4(&ys[4 * bi[it]], yr);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double *V = &acc[it][4 * r];
          yr[r] = fma(-c0, V[0], fma(-c1, V[1], fma(-c2, V[2], fma(-c3, V[3], yr[r]))));
        }
        *reinterpret_cast<double2 *>(&ys[4 * bi[it]]) = make_double2(yr[0], yr[1]);
        *reinterpret_cast<double2 *>(&ys[4 * bi[it] + 2]) = make_double2(yr[2], yr[3]);
      }
    }
  }
  __syncthreads();
  if (tid < KP) yl = ys[tid];
  const double sk = sqrt((double)(k - 1));
  float xal = tid < KP ? (float)(xb_mean + (d + sk * yl)) : 0.0f;

  // ---- RTPP / RTPS (:684-698), fp32 in the reference's order -------------------------
  if (c.use_rtpp || c.use_rtps) {
    const float xa_mean = seq_sum_f32(xal) * c.nmember_inv;
    const double xpl = tid < k ? (double)xbl - xb_mean : 0.0;
    float xap = 0.0f;
    if (tid < k) {
      xap = xal - xa_mean;
      if (c.use_rtpp)
        xap = (float)((double)((1.0f - c.rtpp_alpha) * xap) + (double)c.rtpp_alpha * xpl);
    }
    if (c.use_rtps) {
      const float xb_std = (float)seq_sumsq_f64(xpl);
      const float xa_std = seq_sum_f32(xap * xap);
      xap = xap * (c.rtps_alpha * sqrtf(xb_std / xa_std) - c.rtps_alpha + 1.0f);
    }
    xal = xa_mean + xap;
  }

  if (tid < k) {
    if constexpr (ASSEMBLED) xa_out[(long long)gi * k + tid] = xal;
    else slab.var[P + slab.L * tid] = xal;
  }
  if (tid == 0 && info) info[gi] = make_int2(ptot, ratio > dec ? -level : level);
}

template <int KP>
static hipError_t launch_big_kp(hipStream_t s, bool assembled, const TreeDesc *trees,
                                SolveConsts c, SlabDev slab, long long g0, int npts,
                                const int *nbr_cnt, const int *nbr_idx,
                                const long long *col_off, const float *yo, const float *yb,
                                const float *xb, float *xa, int2 *info, double *tri) {
  if (assembled)
    hipLaunchKernelGGL((solve_tq_big_kernel<KP, true>), dim3(npts), dim3(kBigThreads), 0, s,
                       trees, c, slab, g0, npts, nbr_cnt, nbr_idx, col_off, yo, yb, xb, xa,
                       info, tri);
  else
    hipLaunchKernelGGL((solve_tq_big_kernel<KP, false>), dim3(npts), dim3(kBigThreads), 0, s,
                       trees, c, slab, g0, npts, nbr_cnt, nbr_idx, col_off, yo, yb, xb, xa,
                       info);
  return hipGetLastError();
}

hipError_t launch_big_handoff(hipStream_t s, int kp, const TreeDesc *trees, SolveConsts c,
                              SlabDev slab, long long g0, int npts, const int *nbr_cnt,
                              const int *nbr_idx, int2 *info, double *ws) {
  if (npts <= 0) return hipSuccess;
  if ((kp != 96 && kp != 128) || c.k <= kp - 62) return hipErrorInvalidValue;
  // hand-off after kp - 64 steps: 64 trailing rows, one per tail lane.  KP = 128 runs the
  // half-row kernel (cwbl_tq_rows.hip): two barriers per step against this kernel's four
  if (kp == 128)
    return launch_rows_handoff(s, trees, c, slab, g0, npts, nbr_cnt, nbr_idx, info, ws);
  else
    hipLaunchKernelGGL((solve_tq_big_kernel<96, false, 32>), dim3(npts), dim3(kBigThreads), 0,
                       s, trees, c, slab, g0, npts, nbr_cnt, nbr_idx, nullptr, nullptr, nullptr,
                       nullptr, nullptr, info, ws);
  return hipGetLastError();
}

hipError_t launch_solve_tq_big(hipStream_t s, int kp, bool assembled, const TreeDesc *trees,
                               SolveConsts c, SlabDev slab, long long g0, int npts,
                               const int *nbr_cnt, const int *nbr_idx,
                               const long long *col_off, const float *yo, const float *yb,
                               const float *xb, float *xa, int2 *info, double *tri) {
  if (npts <= 0) return hipSuccess;
  if (c.quad == nullptr || (tri && !assembled)) return hipErrorInvalidValue;
  switch (kp) {
    case 96:
      return launch_big_kp<96>(s, assembled, trees, c, slab, g0, npts, nbr_cnt, nbr_idx,
                               col_off, yo, yb, xb, xa, info, tri);
    case 128:
      return launch_big_kp<128>(s, assembled, trees, c, slab, g0, npts, nbr_cnt, nbr_idx,
                                col_off, yo, yb, xb, xa, info, tri);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace cwbl
