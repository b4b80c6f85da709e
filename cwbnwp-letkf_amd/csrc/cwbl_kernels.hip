// cwbl_kernels.hip — gfx950 kernels of the LETKF analysis core.
//
//   obs_prep_kernel   per (observation, obs-variable): the point-independent half of
//                     letkf_yoyb (module_letkf_core.f90:429-437, 497-510): ensemble mean,
//                     perturbations, spread, error, QC and gross-error decision -> column table
//   search_kernel     one lane per grid point: get_lz -> kdtree2_r_nearest for every tree
//                     (module_localization.f90:188-331, module_kdtree2.f90:1118-1712), same
//                     neighbours in the same traversal order, truncated at max_lz_pts
//   solve_kernel<KP>  one wavefront per grid point: the point-dependent half of letkf_yoyb
//                     (localisation weight, :443-452) + letkf_solve (:598-700): fp64
//                     Yb Yb^T accumulation, parallel cyclic Jacobi eigensolver with A in LDS
//                     and the eigenvector rows in VGPRs, W^a / wbar^a applied matrix-free,
//                     RTPP/RTPS epilogue in the reference's fp32 operation order.
//
// Built with -ffp-contract=off: every fp32 expression is evaluated unfused, in the
// reference's order (amdflang x86-64 evaluates the Fortran that way; see oracle/).
// fp64 code uses explicit fma() where a fused result is wanted.
#include "cwbl_device.h"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace cwbl {

// ---------------------------------------------------------------------------------------
// obs_prep_kernel: one thread per column c = n*nvar + v of one obs type
// ---------------------------------------------------------------------------------------
struct PrepParams {
  float err_muti[5], err_rej[5];
  int is_assim[5];
};

__global__ void __launch_bounds__(256)
obs_prep_kernel(int k, int kp, int family, int type_id, int nvar, int nobs,
                const float *__restrict__ obs, const float *__restrict__ error,
                const float *__restrict__ hdxb, const int *__restrict__ qc, PrepParams pp,
                float norain, const int *__restrict__ slot_obs, float *__restrict__ col_bg,
                float *__restrict__ col_omm, float *__restrict__ col_err,
                uint8_t *__restrict__ col_ok) {
  // output column cs = slot*nvar + v (tree slot order); input column c = obs*nvar + v
  const long long cs = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long ncol = (long long)nobs * nvar;
  if (cs >= ncol) return;
  const int slot = (int)(cs / nvar), v = (int)(cs - (long long)slot * nvar);
  const int n = slot_obs ? slot_obs[slot] : slot;
  const long long c = (long long)n * nvar + v;
  const long long mstride = ncol;  // hdxb(nvar,nobs,0:k-1): member stride = nvar*nobs
  float *bg = col_bg + cs * kp;
  bool ok;
  float omm = 0.0f, err = 0.0f;
  if (family == 0) {
    ok = pp.is_assim[v] != 0;
    if (ok) {  // any(qc(k,idx,:) >= 0)   (:429)
      bool anyqc = false;
      for (int m = 0; m < k; ++m) anyqc |= qc[c + mstride * m] >= 0;
      ok = anyqc;
    }
  } else {
    ok = pp.is_assim[0] != 0;  // radar: hclr(ivar) > 0 (:487)
  }
  if (ok) {
    const float ninv = 1.0f / (float)k, n1inv = 1.0f / (float)(k - 1);
    float s = 0.0f;
    for (int m = 0; m < k; ++m) s = s + hdxb[c + mstride * m];          // sum(bg)
    const float mean = s * ninv;
    float d = 0.0f;
    for (int m = 0; m < k; ++m) {
      const float b = hdxb[c + mstride * m] - mean;
      bg[m] = b;
      d = d + b * b;                                                    // dot_product(bg,bg)
    }
    const float o = obs[c];
    omm = o - mean;
    const float std = sqrtf(d * n1inv);
    const float e = family == 0 ? error[c] * pp.err_muti[v] : pp.err_muti[0];
    const float rej = family == 0 ? pp.err_rej[v] : pp.err_rej[0];
    const bool gross = fabsf(omm) > sqrtf(std * std + e * e) * rej;
    if (family == 1 && type_id == 1) {  // dbz, :504-507
      if (gross && o != norain) ok = false;
      if (o == norain && mean == norain) ok = false;
    } else if (gross) {
      ok = false;
    }
    err = e;
  }
  for (int m = ok ? k : 0; m < kp; ++m) bg[m] = 0.0f;
  col_omm[cs] = omm;
  col_err[cs] = err;
  col_ok[cs] = ok ? 1 : 0;
}

hipError_t launch_obs_prep(hipStream_t s, int k, int kp, int family, int type_id, int nvar,
                           int nobs, const float *obs, const float *error, const float *hdxb,
                           const int *qc, const float err_muti[5], const float err_rej[5],
                           const int is_assim[5], float norain, const int *slot_obs,
                           float *col_bg, float *col_omm, float *col_err, uint8_t *col_ok) {
  PrepParams pp;
  for (int i = 0; i < 5; ++i) {
    pp.err_muti[i] = err_muti[i];
    pp.err_rej[i] = err_rej[i];
    pp.is_assim[i] = is_assim[i];
  }
  const long long ncol = (long long)nobs * nvar;
  if (ncol == 0) return hipSuccess;
  const unsigned grid = (unsigned)((ncol + 255) / 256);
  hipLaunchKernelGGL(obs_prep_kernel, dim3(grid), dim3(256), 0, s, k, kp, family, type_id,
                     nvar, nobs, obs, error, hdxb, qc, pp, norain, slot_obs, col_bg, col_omm,
                     col_err, col_ok);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// search_kernel: one lane per query point
// ---------------------------------------------------------------------------------------
constexpr int kStackDepth = kSearchStackDepth;

__device__ __forceinline__ float dis2_from_bnd(float x, float amin, float amax) {
  if (x > amax) return (x - amax) * (x - amax);
  if (x < amin) return (amin - x) * (amin - x);
  return 0.0f;
}

// kdtree2_r_nearest on one tree (fixed ball).  The recursion of search() (:1381-1457) is run
// with an explicit stack: because the ball never shrinks in the fixed-ball search, the
// decision to visit the farther child can be taken before descending the closer one, and
// LIFO order then reproduces the recursive visiting order exactly.
constexpr int kAhead = 4;  // bucket points loaded ahead of their tests
__device__ int search_tree(const TreeDesc &T, float q0, float q1, float q2, float r2,
                           int *out_idx, float *out_r2, int *stk, bool &overflow) {
  const TreeNode *__restrict__ nodes = T.nodes;
  const int dim = T.tree_dim;
  int count = 0, sp = 0, node = 0;
  overflow = false;
  // analysis lists: slots are buffered kListGroup at a time and stored as one 16-B write
  static_assert(kListGroup == 4, "int4 groups");
  int4 grp = make_int4(0, 0, 0, 0);
  auto flush = [&]() {
    if (!out_r2 && (count % kListGroup) != 0)
      *reinterpret_cast<int4 *>(out_idx + list_slot(count - count % kListGroup)) = grp;
  };
  // "while-while" traversal: a lane descends internal nodes until it reaches a bucket, and
  // the wave processes buckets together once every lane holds one (the if-if form ran the
  // bucket loop once per subset of lanes that happened to be at a leaf).  Each lane's own
  // visiting order, hence its result order, is unchanged.
  while (true) {
    TreeNode nd = nodes[node];
    while (nd.cut_dim >= 0) {
      const int cd = nd.cut_dim;
      const float qval = cd == 0 ? q0 : (cd == 1 ? q1 : q2);
      int closer, farther;
      float dis;
      if (qval < nd.cut_val) {
        closer = nd.left; farther = nd.right;
        dis = (nd.cut_val_right - qval) * (nd.cut_val_right - qval);
      } else {
        closer = nd.right; farther = nd.left;
        dis = (nd.cut_val_left - qval) * (nd.cut_val_left - qval);
      }
      bool far_ok = farther >= 0 && dis <= r2;
      if (far_ok) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (i >= dim || i == cd || !far_ok) continue;
          const float qi = i == 0 ? q0 : (i == 1 ? q1 : q2);
          dis = dis + dis2_from_bnd(qi, nd.lo[i], nd.hi[i]);
          if (dis > r2) far_ok = false;
        }
      }
      if (far_ok) stk[sp++ * 64] = farther;
      node = closer;
      nd = nodes[node];
    }
    // process_terminal_node_fixedball (:1654-1707): the bucket's points are loaded four at
    // a time ahead of the tests, so one round trip to memory covers four candidates; tests
    // and appends stay in index order
    for (int i0 = nd.l; i0 <= nd.u; i0 += kAhead) {
      float4 d[kAhead];
#pragma unroll
      for (int e = 0; e < kAhead; ++e)
        d[e] = T.rdata[min(i0 + e, nd.u)];
#pragma unroll
      for (int e = 0; e < kAhead; ++e) {
        const int i = i0 + e;
        const float dx = d[e].x - q0, dy = d[e].y - q1;
        float sd = dx * dx;
        sd = sd + dy * dy;
        if (dim == 3) {
          const float dz = d[e].z - q2;
          sd = sd + dz * dz;
        }
        if (i <= nd.u && sd <= r2) {
          if (count == T.max_lz) { overflow = true; flush(); return count; }
          if (out_r2) {  // cwbl_search: original obs index and distance
            out_idx[count] = T.ind[i];
            out_r2[count] = sd;
          } else {       // analysis: the tree slot (columns are stored in slot order)
            const int g = count % kListGroup;
            grp.x = g == 0 ? i : grp.x;
            grp.y = g == 1 ? i : grp.y;
            grp.z = g == 2 ? i : grp.z;
            grp.w = i;
            if (g == kListGroup - 1)
              *reinterpret_cast<int4 *>(out_idx + list_slot(count - g)) = grp;
          }
          ++count;
        }
      }
    }
    if (sp == 0) { flush(); return count; }
    node = stk[--sp * 64];
  }
}

struct SlabQuery {
  SlabDev s;
  long long g0;
  // thread li -> batch point gi (false: no point)
  __device__ bool map(int li, int npts, int &gi) const {
    gi = li;
    return li < npts;
  }
  __device__ void at(int gi, float &x, float &y, float &z) const {
    // (g < 2^32, as slab_point)
    const unsigned g = (unsigned)(g0 + gi), ix = (unsigned)s.ix_lim, iy = (unsigned)s.iy_lim;
    const unsigned r = g / ix, i = g - r * ix, kz = r / iy, j = r - kz * iy;
    x = s.x[i + (long long)s.nx * j];
    y = s.y[i + (long long)s.nx * j];
    z = s.alt[i + (long long)s.alt_nx * (j + (long long)s.alt_ny * kz)];
  }
};

struct ListQuery {
  const float *q;  // (3,nq)
  __device__ bool map(int li, int npts, int &gi) const {
    gi = li;
    return li < npts;
  }
  __device__ void at(int gi, float &x, float &y, float &z) const {
    x = q[3 * (long long)gi];
    y = q[3 * (long long)gi + 1];
    z = q[3 * (long long)gi + 2];
  }
};

// the batch points the binned search flagged (their lists would pass max_lz)
struct FlagQuery {
  SlabQuery sq;
  const int *cnt, *idx;
  __device__ bool map(int li, int, int &gi) const {
    if (li >= *cnt) return false;
    gi = idx[li];
    return true;
  }
  __device__ void at(int gi, float &x, float &y, float &z) const { sq.at(gi, x, y, z); }
};

template <class Q>
__global__ void __launch_bounds__(64)
search_kernel(const TreeDesc *__restrict__ trees, int ntrees, int list_cap, float r2, Q qs,
              int npts, int *__restrict__ nbr_cnt, int *__restrict__ nbr_idx,
              float *__restrict__ nbr_r2, DevStats *stats) {
  // traversal stacks, one column per lane; sized by the host to the deepest tree, so a
  // shallow tree leaves LDS for more resident waves (the search is latency bound)
  extern __shared__ int stk[];
  int gi;
  if (!qs.map(blockIdx.x * 64 + threadIdx.x, npts, gi)) return;
  float px, py, pz;
  qs.at(gi, px, py, pz);
  unsigned trunc = 0;
  for (int t = 0; t < ntrees; ++t) {
    const TreeDesc &T = trees[t];
    // get_lz normalisation (module_localization.f90:243-253)
    const float q0 = px * T.hclr_inv, q1 = py * T.hclr_inv;
    const float q2 = T.query3d ? pz * T.vclr_inv : 0.0f;
    // cwbl_search: one contiguous list per query; analysis: lists interleaved by wave
    // (list_index), so the 64 lanes of a wave write slot c of their lists side by side
    const long long base = nbr_r2 ? (long long)gi * list_cap + T.list_off
                                  : list_index(gi, list_cap, T.list_off);
    bool ovf = false;
    int cnt = 0;
    if (T.max_lz > 0)
      cnt = search_tree(T, q0, q1, q2, r2, nbr_idx + base, nbr_r2 ? nbr_r2 + base : nullptr,
                        stk + threadIdx.x, ovf);
    nbr_cnt[(long long)gi * ntrees + t] = cnt;
    trunc += ovf ? 1u : 0u;
  }
  if (trunc && stats) atomicAdd(&stats->lz_truncated, (unsigned long long)trunc);
}

static size_t stack_bytes(int depth) {
  return (size_t)std::min(std::max(depth, 1), kStackDepth) * 64 * sizeof(int);
}

hipError_t launch_search(hipStream_t s, const TreeDesc *trees, int ntrees, int depth,
                         int list_cap, float r2, SlabDev slab, long long g0, int npts,
                         int *nbr_cnt, int *nbr_idx, float *nbr_r2, DevStats *stats) {
  if (npts <= 0) return hipSuccess;
  SlabQuery q{slab, g0};
  hipLaunchKernelGGL(search_kernel<SlabQuery>, dim3((npts + 63) / 64), dim3(64),
                     stack_bytes(depth), s, trees,
                     ntrees, list_cap, r2, q, npts, nbr_cnt, nbr_idx, nbr_r2, stats);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// search_binned_kernel: one lane per grid point.  The fixed-radius sets of search_kernel
// (same normalisation, the same fp32 distance d - q in dimension order and d2 <= r2 test as
// process_terminal_node_fixedball, module_kdtree2.f90:1654-1707) from uniform bins: the
// cells of the ball's bounding box are, per (iy, iz), one contiguous run of points, so a
// lane streams through at most 5 x 5 runs instead of walking the tree (divergent, latency
// bound).  The sets are identical; the order is the bins', which only changes the order of
// the fp64 sums of the solve.  Where kdtree2's order decides WHICH points are kept (a list
// past max_lz, Q4) the point is flagged and search_kernel<FlagQuery> redoes it.
// ---------------------------------------------------------------------------------------
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int kBinAhead = 8;  // bin points loaded ahead of their tests
static_assert(kBinAhead <= kBinPad, "the look-ahead stays inside the bins' padding");
__global__ void __launch_bounds__(64)
search_binned_kernel(const TreeDesc *__restrict__ trees, int ntrees, int list_cap, float r2,
                     float rbox, SlabQuery qs, int npts, int *__restrict__ nbr_cnt,
                     int *__restrict__ nbr_idx, int *__restrict__ flag_cnt,
                     int *__restrict__ flag_idx) {
  // (r4, measured and dropped: an XCD-aware block order, a tie at C2 and C5; four lanes per
  // point, which cuts this kernel's time by 25% at C2 and 38% at C5 but, overlapped with the
  // assembly, costs the step 1-2% at C2 through its extra issue cycles: profiles/r4k_*)
  __shared__ __attribute__((aligned(16))) int sgrp[64][4];
  // blocks XCD chunk by chunk, each chunk from its end (xcd_remap_rev): the assembly reads the
  // lists chunk by chunk from each chunk's start, so the lists written last (in the MALL) are
  // read first
  const int gi = xcd_remap_rev(blockIdx.x, gridDim.x) * 64 + threadIdx.x;
  if (gi >= npts) return;
  float px, py, pz;
  qs.at(gi, px, py, pz);
  bool flagged = false;
  for (int t = 0; t < ntrees; ++t) {
    const TreeDesc &T = trees[t];
    const float q0 = px * T.hclr_inv, q1 = py * T.hclr_inv;  // get_lz (:243-253)
    const float q2 = T.query3d ? pz * T.vclr_inv : 0.0f;
    // this point's list: byte offset from nbr_idx (the list buffer stays below 2 GiB)
    const unsigned obase = 4u * (unsigned)list_index(gi, list_cap, T.list_off);
    int *grp = sgrp[threadIdx.x];  // this lane's group of 4 list slots
    const int dim = T.tree_dim, max_lz = T.max_lz;
    int count = 0;
    bool ovf = false;
    if (max_lz > 0) {
      // conservative cell range of [q - rbox, q + rbox] (clamped before the int conversion)
      // (the margin also covers the rounding of q -/+ rbox and of the cell arithmetic, which
      // grows with the coordinates' magnitude)
      auto margin = [&](float q, float b0) { return 2e-6f * (fabsf(q) + fabsf(b0)); };
      auto crange = [&](float q, float b0, int nb, int &a, int &b) {
        const float rq = rbox + margin(q, b0);
        const float lo = (q - rq - b0) * T.binv, hi = (q + rq - b0) * T.binv;
        a = (int)fminf(fmaxf(floorf(lo), 0.0f), (float)nb);
        b = (int)fminf(fmaxf(floorf(hi), -1.0f), (float)(nb - 1));
      };
      int ix0, ix1, iy0, iy1, iz0 = 0, iz1 = 0;
      crange(q0, T.bx0, T.nbx, ix0, ix1);
      crange(q1, T.by0, T.nby, iy0, iy1);
      if (dim == 3) crange(q2, T.bz0, T.nbz, iz0, iz1);
      if (ix0 > ix1) iy1 = iy0 - 1;  // the box misses the grid in x
      // distance from q to the slab of cell row/layer i along one axis, shrunk by a margin
      // (conservative against the fp32 cell assignment)
      const float h = 1.0f / T.binv, rb2 = rbox * rbox;
      auto gap = [&](float q, float b0, int i) {
        const float lo = b0 + (float)i * h, hi = lo + h;
        const float g = fmaxf(fmaxf(lo - q, q - hi), 0.0f);
        return fmaxf(g - 1e-3f * h - margin(q, b0), 0.0f);
      };
      for (int iz = iz0; iz <= iz1; ++iz) {
        const float gz = dim == 3 ? gap(q2, T.bz0, iz) : 0.0f;
        for (int iy = iy0; iy <= iy1; ++iy) {
          // the ball's x-extent over this row of cells
          const float gy = gap(q1, T.by0, iy);
          const float rem = rb2 - gy * gy - gz * gz;
          if (rem < 0.0f) continue;
          const float xh = sqrtf(rem) + margin(q0, T.bx0);
          const int jx0 = max(ix0, (int)fminf(fmaxf(floorf((q0 - xh - T.bx0) * T.binv), 0.0f),
                                               (float)T.nbx));
          const int jx1 = min(ix1, (int)fminf(fmaxf(floorf((q0 + xh - T.bx0) * T.binv), -1.0f),
                                               (float)(T.nbx - 1)));
          if (jx0 > jx1) continue;
          const int cb = (iz * T.nby + iy) * T.nbx;
          const int e = gld(T.bstart, (unsigned)(cb + jx1 + 1));
          // global loads at SGPR base + 32-bit offset; the points past e that a round reads
          // (at most kBinAhead - 1, never accepted) stay inside the array's padding
          const float *bx = reinterpret_cast<const float *>(T.bxyz);
          for (int i0 = gld(T.bstart, (unsigned)(cb + jx0)); i0 < e; i0 += kBinAhead) {
            f32x4 d[kBinAhead];
#pragma unroll
            for (int a = 0; a < kBinAhead; ++a) d[a] = gld4(bx, 4u * (unsigned)(i0 + a));
#pragma unroll
            for (int a = 0; a < kBinAhead; ++a) {
              const float dx = d[a].x - q0, dy = d[a].y - q1;
              float sd = dx * dx;
              sd = sd + dy * dy;
              if (dim == 3) {
                const float dz = d[a].z - q2;
                sd = sd + dz * dz;
              }
              // a hit goes to this lane's 4-slot group in LDS, a full group to the list as
              // one 16-B store; hits past max_lz are counted, not stored: count > max_lz is
              // the overflow (Q4)
              if (i0 + a < e && sd <= r2) {
                if (count < max_lz) {
                  grp[count & 3] = __float_as_int(d[a].w);
                  if ((count & 3) == 3)  // slot count - 3 = count & ~3 starts the group
                    gst(reinterpret_cast<i32x4 *>(nbr_idx), obase + 4u * list_slot(count & ~3),
                        *reinterpret_cast<const i32x4 *>(grp));
                }
                ++count;
              }
            }
            if (count > max_lz) break;
          }
          if (count > max_lz) break;
        }
        if (count > max_lz) break;
      }
      ovf = count > max_lz;
      count = min(count, max_lz);
      if (count & 3)  // the last, partial group (its slots past count are never read)
        gst(reinterpret_cast<i32x4 *>(nbr_idx), obase + 4u * list_slot(count & ~3),
            *reinterpret_cast<const i32x4 *>(grp));
    }
    nbr_cnt[(long long)gi * ntrees + t] = count;
    flagged = flagged || ovf;
  }
  if (flagged) flag_idx[atomicAdd(flag_cnt, 1)] = gi;
}

hipError_t launch_search_binned(hipStream_t s, const TreeDesc *trees, int ntrees, int list_cap,
                                float r2, float rbox, SlabDev slab, long long g0, int npts,
                                int *nbr_cnt, int *nbr_idx, int *flag_cnt, int *flag_idx) {
  if (npts <= 0) return hipSuccess;
  SlabQuery q{slab, g0};
  hipLaunchKernelGGL(search_binned_kernel, dim3((npts + 63) / 64), dim3(64), 0, s, trees,
                     ntrees, list_cap, r2, rbox, q, npts, nbr_cnt, nbr_idx, flag_cnt, flag_idx);
  return hipGetLastError();
}

hipError_t launch_search_flagged(hipStream_t s, const TreeDesc *trees, int ntrees, int depth,
                                 int list_cap, float r2, SlabDev slab, long long g0, int npts,
                                 const int *flag_cnt, const int *flag_idx, int *nbr_cnt,
                                 int *nbr_idx, DevStats *stats) {
  if (npts <= 0) return hipSuccess;
  FlagQuery q{SlabQuery{slab, g0}, flag_cnt, flag_idx};
  hipLaunchKernelGGL(search_kernel<FlagQuery>, dim3((npts + 63) / 64), dim3(64),
                     stack_bytes(depth), s, trees, ntrees, list_cap, r2, q, npts, nbr_cnt,
                     nbr_idx, (float *)nullptr, stats);
  return hipGetLastError();
}

hipError_t launch_search_single(hipStream_t s, const TreeDesc *tree, int depth, float r2,
                                int nq, const float *q_xyz, int max_lz, int *nfound, int *idx,
                                float *r2out) {
  if (nq <= 0) return hipSuccess;
  ListQuery q{q_xyz};
  hipLaunchKernelGGL(search_kernel<ListQuery>, dim3((nq + 63) / 64), dim3(64),
                     stack_bytes(depth), s, tree, 1,
                     max_lz, r2, q, nq, nfound, idx, r2out, (DevStats *)nullptr);
  return hipGetLastError();
}

// letkf_tune_q (module_letkf_core.f90:702-733) over the analysed region of var(nx,ny,nz,0:k-1),
// one thread per point.  Both member sums run in member order in fp32 (`sum(var)` and
// `sum(var, mask=var>0)`, :720); a point with no positive member gets ratio = 0/0 (or x/0),
// so its non-negative members become NaN (Q3, replicated).  HBM bound: 2 reads + 1 write of
// the k values, coalesced across threads (neighbouring points are adjacent in memory).
__global__ void __launch_bounds__(256)
tune_q_kernel(SlabDev s, int k, long long npts) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (g >= npts) return;
  const int i = (int)(g % s.ix_lim);
  const long long r = g / s.ix_lim;
  const int j = (int)(r % s.iy_lim);
  const int kz = (int)(r / s.iy_lim);
  float *__restrict__ v = s.var + i + (long long)s.nx * (j + (long long)s.ny * kz);
  float sum = 0.0f, sum_pos = 0.0f;
  for (int m = 0; m < k; ++m) {
    const float x = v[m * s.L];
    sum = sum + x;
    if (x > 0.0f) sum_pos = sum_pos + x;
  }
  const float ratio = sum / sum_pos;
  for (int m = 0; m < k; ++m) {
    const float x = v[m * s.L];
    v[m * s.L] = x < 0.0f ? 0.0f : ratio * x;  // where (var < 0) 0 elsewhere ratio*var
  }
}

hipError_t launch_tune_q(hipStream_t st, SlabDev s, int k) {
  const long long npts = (long long)s.ix_lim * s.iy_lim * s.nz;
  if (npts <= 0) return hipSuccess;
  hipLaunchKernelGGL(tune_q_kernel, dim3((unsigned)((npts + 255) / 256)), dim3(256), 0, st, s,
                     k, npts);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// solve_kernel<KP>: one wavefront (64 lanes) per grid point, members padded to KP
// ---------------------------------------------------------------------------------------
constexpr int kChunk = 32;      // columns staged per round (two lanes per column)


// Round-robin ("circle") tournament in slot form: slots (2i, 2i+1) form pair i; slot 0 is
// fixed and the other KP-1 slots rotate one ring position per step, so every pair of
// indices meets exactly once per KP-1 steps and the slot permutation is the identity again
// after a full sweep.
template <int KP>
struct Ring {
  static constexpr int R = KP - 1;
  // ring position of slot (slot != 0): tops 2i (i>=1) -> i-1, bottoms 2i+1 -> 2m-2-i
  __host__ __device__ static constexpr int pos(int slot) {
    return (slot & 1) ? (KP - 2 - (slot >> 1)) : ((slot >> 1) - 1);
  }
  __host__ __device__ static constexpr int slot_at(int p) {
    return p < KP / 2 - 1 ? 2 * (p + 1) : 2 * (KP - 2 - p) + 1;
  }
  // slot the content of `slot` moves to after a step
  __host__ __device__ static constexpr int next(int slot) {
    return slot == 0 ? 0 : slot_at(pos(slot) + 1 == R ? 0 : pos(slot) + 1);
  }
};


template <int KP>
struct SolveSmem {
  union {
    double A[KP + 1][KP + 2];  // work matrix (16-B aligned rows; last row = dummy
                               // target of padding writes) / eigenvectors at the end
    ColumnChunk<KP, kChunk> ch;
  } u;
  double cs[KP / 2][2];  // c, s per pair
  double b1[KP];         // Yb d (fp64)
  double xp[KP];         // x' = xb - xb_mean (fp64)
  double z1[KP], z2[KP];
  double lam[KP];
  float xb[KP], xa[KP];
  double scal[4];
  float fscal[4];
};



template <int KP, bool ASSEMBLED>
__global__ void __launch_bounds__(64)
solve_kernel(const TreeDesc *__restrict__ trees, SolveConsts c, SlabDev slab, long long g0,
             int npts, const int *__restrict__ nbr_cnt, const int *__restrict__ nbr_idx,
             const long long *__restrict__ col_off,
             const float *__restrict__ yo_in, const float *__restrict__ yb_in,
             const float *__restrict__ xb_in, float *__restrict__ xa_out,
             double *__restrict__ evals, int2 *__restrict__ info) {
  static_assert(KP % 8 == 0 && KP <= 64, "KP");
  constexpr int NP = KP / 2;                     // pairs per step
  constexpr int NPB = NP * (NP + 1) / 2;         // pair blocks (lower)
  constexpr int NPL = (NPB + 63) / 64;
  __shared__ SolveSmem<KP> sm;

  const int gi = xcd_remap(blockIdx.x, gridDim.x);
  if (gi >= npts) return;
  const int lane = threadIdx.x;
  const int k = c.k;

  long long P = 0;  // var index of member 0
  float3 pt = make_float3(0.0f, 0.0f, 0.0f);  // the point's projected x, y and altitude
  if constexpr (!ASSEMBLED) {
    const long long g = g0 + gi;
    const int i = (int)(g % slab.ix_lim);
    const long long r = g / slab.ix_lim;
    const int j = (int)(r % slab.iy_lim);
    const int kz = (int)(r / slab.iy_lim);
    P = i + (long long)slab.nx * (j + (long long)slab.ny * kz);
    if (lane < KP) sm.xb[lane] = lane < k ? slab.var[P + slab.L * lane] : 0.0f;
    slab_point(slab, g, pt.x, pt.y, pt.z);
  } else {
    if (lane < KP) sm.xb[lane] = lane < k ? xb_in[(long long)gi * k + lane] : 0.0f;
  }

  constexpr int NBL = AsmLayout<KP>::NBL, NBLK = AsmLayout<KP>::NBLK;
  int bi[NBL], bj[NBL];
  block_of_lane<KP>(lane, bi, bj);
  double acc[NBL][16];
  double b1acc;
  int ptot;
  assemble_point<KP, kChunk, ASSEMBLED>(sm.u.ch, trees, c, gi, lane, nbr_cnt, nbr_idx, pt,
                                        col_off, yo_in, yb_in, bi, bj, acc, b1acc, ptot);

  if (ptot == 0) {  // no accepted observation: var left unchanged (:220, :226)
    if (lane == 0 && info) info[gi] = make_int2(0, 0);
    if constexpr (ASSEMBLED) {
      if (lane < k) xa_out[(long long)gi * k + lane] = sm.xb[lane];
    }
    return;
  }

  // ---- A = inflat*I + Yb Yb^T (full symmetric, padded identity) ----------------------
  const double inflat_r8 = (double)c.inflat;
#pragma unroll
  for (int it = 0; it < NBL; ++it) {
    if (lane + 64 * it < NBLK) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ii = 4 * bi[it] + r, jj = 4 * bj[it] + q;
          double v = acc[it][4 * r + q];
          if (ii == jj) v = ii < k ? v + inflat_r8 : 1.0;
          sm.u.A[ii][jj] = v;
          sm.u.A[jj][ii] = v;
        }
    }
  }
  if (lane < KP) sm.b1[lane] = b1acc;
  if (lane == 0) {  // xb_mean = sum(xb) * nmember_inv in fp32 (:671)
    float s = 0.0f;
    for (int m = 0; m < k; ++m) s = s + sm.xb[m];
    sm.scal[0] = (double)(s * c.nmember_inv);
  }
  __syncthreads();
  const double xb_mean = sm.scal[0];
  if (lane < KP) sm.xp[lane] = lane < k ? (double)sm.xb[lane] - xb_mean : 0.0;

  // ---- parallel cyclic Jacobi ---------------------------------------------------------
  // Brent-Luk ordering in "slot" space: slots (2i, 2i+1) are pair i of every step and, after
  // a step, the content of slot s moves to Ring::next(s) (circle tournament, identity after
  // KP-1 steps).  Every lane owns fixed 2x2 blocks (P,Q), P >= Q, of the lower triangle in
  // slot space, held in registers; the step's permutation is a write of each element to its
  // new (static) LDS position and a read-back.  V (row `lane`) lives in VGPRs in slot order.
  constexpr int LD = KP + 2;
  double *M = &sm.u.A[0][0];
  double v[KP];
#pragma unroll
  for (int q = 0; q < KP; ++q) v[q] = lane == q ? 1.0 : 0.0;
  int bP[NPL], bQ[NPL], wad[NPL][4], rad[NPL];
  double e[NPL][4];
  constexpr int DUMMY = KP * LD;  // LDS element that absorbs writes of padding lanes
#pragma unroll
  for (int it = 0; it < NPL; ++it) {
    const int b = lane + 64 * it;
    const bool valid = b < NPB;
    int PP = 0, QQ = 0;
    if (b < NP) {
      PP = QQ = b;  // diagonal blocks first: lanes 0..NP-1 of it = 0
    } else if (valid) {
      const int bb = b - NP;
      int rr = 0;
      while ((rr + 1) * (rr + 2) / 2 <= bb) ++rr;
      PP = rr + 1;
      QQ = bb - rr * (rr + 1) / 2;
    }
    bP[it] = PP;
    bQ[it] = QQ;
    const int rs[4] = {2 * PP, 2 * PP, 2 * PP + 1, 2 * PP + 1};
    const int cl[4] = {2 * QQ, 2 * QQ + 1, 2 * QQ, 2 * QQ + 1};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int nr = Ring<KP>::next(rs[j]), nc = Ring<KP>::next(cl[j]);
      if (nr < nc) { const int t = nr; nr = nc; nc = t; }
      wad[it][j] = (!valid || (PP == QQ && j == 1)) ? DUMMY + j : nr * LD + nc;
    }
    rad[it] = 2 * PP * LD + 2 * QQ;
    const double2 r0 = *reinterpret_cast<const double2 *>(M + rad[it]);
    const double2 r1 = *reinterpret_cast<const double2 *>(M + rad[it] + LD);
    e[it][0] = r0.x; e[it][1] = PP == QQ ? r1.x : r0.y; e[it][2] = r1.x; e[it][3] = r1.y;
  }
  const bool diag_lane = lane < NP;  // owns diagonal block (lane,lane) as e[0]
  const double tol = 1e-14;   // rotate pair (p,q) iff |apq| > tol * sqrt(app*aqq)
  const double tol_q = 1e-8;  // quadratic convergence: a sweep that started below this ends ~1e-16
  int sweeps = 0;
  bool converged = false;
  for (int sweep = 0; sweep < c.max_sweeps; ++sweep) {
    bool rotated = false;
    double mrel = 0.0;
#pragma unroll 1
    for (int st = 0; st < KP - 1; ++st) {
      // rotation parameters from the diagonal blocks (lane P < NP owns block (P,P)),
      // computed branch-free on every lane and published by the diagonal lanes
      double d0, d3, cc = 1.0, ss = 0.0;
      bool rot = false;
      {
        const double app = e[0][0], aqq = e[0][3], apq = e[0][2];
        const double rel = fabs(apq) * rsq64(app * aqq);
        rot = diag_lane && apq != 0.0 && rel > tol;
        mrel = diag_lane && apq != 0.0 ? fmax(mrel, rel) : mrel;
        const double theta = (aqq - app) * rcp64(2.0 * apq);
        const double w = fma(theta, theta, 1.0);
        double t = fabs(theta) > 1e150 ? 0.5 * rcp64(fabs(theta))
                                       : rcp64(fabs(theta) + w * rsq64(w));
        t = theta < 0.0 ? -t : t;
        const double c0 = rsq64(fma(t, t, 1.0));
        cc = rot ? c0 : 1.0;
        ss = rot ? t * c0 : 0.0;
        const double tapq = rot ? t * apq : 0.0;
        d0 = app - tapq;
        d3 = aqq + tapq;
        rotated |= rot;
        if (diag_lane) {
          sm.cs[lane][0] = cc;
          sm.cs[lane][1] = ss;
        }
      }
      __syncthreads();
      // all blocks: rows rotated by pair P, columns by pair Q
#pragma unroll
      for (int it = 0; it < NPL; ++it) {
        const double2 p1 = *reinterpret_cast<const double2 *>(&sm.cs[bP[it]][0]);
        const double2 p2 = *reinterpret_cast<const double2 *>(&sm.cs[bQ[it]][0]);
        const double c1 = p1.x, s1 = p1.y, c2 = p2.x, s2 = p2.y;
        const double x = e[it][0], y = e[it][1], z = e[it][2], w = e[it][3];
        const double x1 = fma(c1, x, -s1 * z), z1 = fma(s1, x, c1 * z);
        const double y1 = fma(c1, y, -s1 * w), w1 = fma(s1, y, c1 * w);
        e[it][0] = fma(c2, x1, -s2 * y1);
        e[it][1] = fma(s2, x1, c2 * y1);
        e[it][2] = fma(c2, z1, -s2 * w1);
        e[it][3] = fma(s2, z1, c2 * w1);
      }
      // diagonal blocks take the exact Jacobi update (a'_pp = app - t apq, a'_pq = 0)
      e[0][0] = diag_lane ? d0 : e[0][0];
      e[0][3] = diag_lane ? d3 : e[0][3];
      e[0][1] = diag_lane && rot ? 0.0 : e[0][1];
      e[0][2] = diag_lane && rot ? 0.0 : e[0][2];
      // V <- V J on the slot pairs, then the ring advance of the slots
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const double2 pc = *reinterpret_cast<const double2 *>(&sm.cs[i][0]);
        const double vp = v[2 * i], vq = v[2 * i + 1];
        v[2 * i] = fma(pc.x, vp, -pc.y * vq);
        v[2 * i + 1] = fma(pc.y, vp, pc.x * vq);
      }
      {
        constexpr int R = KP - 1;
        const double last = v[Ring<KP>::slot_at(R - 1)];
#pragma unroll
        for (int p = R - 1; p >= 1; --p) v[Ring<KP>::slot_at(p)] = v[Ring<KP>::slot_at(p - 1)];
        v[Ring<KP>::slot_at(0)] = last;
      }
      // permute A: every element to its new slot position (lower triangle)
#pragma unroll
      for (int it = 0; it < NPL; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j) M[wad[it][j]] = e[it][j];
      __syncthreads();
#pragma unroll
      for (int it = 0; it < NPL; ++it) {
        const double2 r0 = *reinterpret_cast<const double2 *>(M + rad[it]);
        const double2 r1 = *reinterpret_cast<const double2 *>(M + rad[it] + LD);
        e[it][0] = r0.x;
        e[it][1] = (it == 0 && diag_lane) ? r1.x : r0.y;
        e[it][2] = r1.x;
        e[it][3] = r1.y;
      }
    }
    sweeps = sweep + 1;
    const bool any_rot = __any(rotated);
    double wm = mrel;
    for (int off = 32; off > 0; off >>= 1) wm = fmax(wm, __shfl_xor(wm, off, 64));
    if (!any_rot || wm < tol_q) { converged = true; break; }
  }

  // ---- apply the weights matrix-free ----------------------------------------------------
  // eigenvalues lam_j = A(j,j); V written to LDS (A no longer needed)
  if (lane < KP) sm.lam[lane] = sm.u.A[lane][lane];
  __syncthreads();
  if (lane < KP) {
#pragma unroll
    for (int q = 0; q < KP; ++q) sm.u.A[lane][q] = v[q];
  }
  __syncthreads();
  if (lane < KP) {
    double u1 = 0.0, u2 = 0.0;
    for (int r = 0; r < KP; ++r) {
      const double vr = sm.u.A[r][lane];
      u1 = fma(vr, sm.b1[r], u1);   // V^T (Yb d)
      u2 = fma(vr, sm.xp[r], u2);   // V^T x'
    }
    const double einv = 1.0 / sm.lam[lane];  // eval = 1/lambda (module_eigen.f90:52)
    sm.z1[lane] = u1 * einv;
    sm.z2[lane] = u2 * sqrt(einv);           // sqrt(eval) (module_eigen.f90:90)
  }
  __syncthreads();
  double wb = 0.0, sr = 0.0;  // wbar_r = (Pa Yb d)_r ; s_r = (Pa^{1/2} x')_r
#pragma unroll
  for (int q = 0; q < KP; q += 4) {
    // bounded groups: keeps the LDS loads of z1/z2 from all being hoisted at once
    const double2 a0 = *reinterpret_cast<const double2 *>(&sm.z1[q]);
    const double2 a1 = *reinterpret_cast<const double2 *>(&sm.z1[q + 2]);
    const double2 b0 = *reinterpret_cast<const double2 *>(&sm.z2[q]);
    const double2 b1 = *reinterpret_cast<const double2 *>(&sm.z2[q + 2]);
    wb = fma(v[q], a0.x, wb); wb = fma(v[q + 1], a0.y, wb);
    wb = fma(v[q + 2], a1.x, wb); wb = fma(v[q + 3], a1.y, wb);
    sr = fma(v[q], b0.x, sr); sr = fma(v[q + 1], b0.y, sr);
    sr = fma(v[q + 2], b1.x, sr); sr = fma(v[q + 3], b1.y, sr);
    __builtin_amdgcn_sched_barrier(0);
  }
  const double xpl = lane < KP ? sm.xp[lane] : 0.0;
  const double d = wave_sum_f64(lane < k ? wb * xpl : 0.0);  // sum_i wbar_i x'_i
  const double sk = sqrt((double)(k - 1));
  if (lane < KP) sm.xa[lane] = (float)(xb_mean + (d + sk * sr));  // xa = wbar (:675-679)
  __syncthreads();

  // ---- RTPP / RTPS (:684-698), fp32 in the reference's order -------------------------
  if (c.use_rtpp || c.use_rtps) {
    if (lane == 0) {
      float s = 0.0f;
      for (int m = 0; m < k; ++m) s = s + sm.xa[m];
      sm.fscal[0] = s * c.nmember_inv;  // xa_mean
    }
    __syncthreads();
    const float xa_mean = sm.fscal[0];
    float xap = 0.0f;
    if (lane < k) {
      xap = sm.xa[lane] - xa_mean;
      if (c.use_rtpp)
        xap = (float)((double)((1.0f - c.rtpp_alpha) * xap) + (double)c.rtpp_alpha * sm.xp[lane]);
    }
    if (c.use_rtps) {
      __syncthreads();
      if (lane < k) sm.xa[lane] = xap;  // stage xa_prime
      __syncthreads();
      if (lane == 0) {
        double d8 = 0.0;
        for (int m = 0; m < k; ++m) d8 = d8 + sm.xp[m] * sm.xp[m];
        const float xb_std = (float)d8;
        float xa_std = 0.0f;
        for (int m = 0; m < k; ++m) xa_std = xa_std + sm.xa[m] * sm.xa[m];
        sm.fscal[1] = c.rtps_alpha * sqrtf(xb_std / xa_std) - c.rtps_alpha + 1.0f;
      }
      __syncthreads();
      xap = xap * sm.fscal[1];
    }
    if (lane < k) sm.xa[lane] = xa_mean + xap;
    __syncthreads();
  }

  if (lane < k) {
    if constexpr (ASSEMBLED) xa_out[(long long)gi * k + lane] = sm.xa[lane];
    else slab.var[P + slab.L * lane] = sm.xa[lane];
  }
  if (lane == 0 && info) info[gi] = make_int2(ptot, converged ? sweeps : -sweeps);
  if (ASSEMBLED && evals != nullptr && lane < k) {
    // eigenvalues ascending (dsyevd order) over the k real indices
    const double lj = sm.lam[lane];
    int rank = 0;
    for (int i = 0; i < k; ++i) {
      const double li = sm.lam[i];
      rank += (li < lj || (li == lj && i < lane)) ? 1 : 0;
    }
    evals[(long long)gi * k + rank] = lj;
  }
}

template <int KP>
static hipError_t launch_solve_kp(hipStream_t s, bool assembled, const TreeDesc *trees,
                                  SolveConsts c, SlabDev slab, long long g0, int npts,
                                  const int *nbr_cnt, const int *nbr_idx,
                                  const long long *col_off, const float *yo, const float *yb,
                                  const float *xb, float *xa, double *evals, int2 *info) {
  if (assembled)
    hipLaunchKernelGGL((solve_kernel<KP, true>), dim3(npts), dim3(64), 0, s, trees, c, slab,
                       g0, npts, nbr_cnt, nbr_idx, col_off, yo, yb, xb, xa, evals, info);
  else
    hipLaunchKernelGGL((solve_kernel<KP, false>), dim3(npts), dim3(64), 0, s, trees, c, slab,
                       g0, npts, nbr_cnt, nbr_idx, col_off, yo, yb, xb, xa, evals, info);
  return hipGetLastError();
}

// KP <= 64: one wavefront per point (solve_tq_kernel, solve_kernel); 96 and 128: one
// 256-thread workgroup per point (solve_tq_big_kernel; no Jacobi eigenvalue path)
static const int kSupportedKP[] = {8, 16, 24, 32, 40, 48, 56, 64, 96, 128};

int supported_kp(int k) {
  for (int kp : kSupportedKP)
    if (k <= kp) return kp;
  return -1;
}

static hipError_t dispatch_solve(hipStream_t s, int kp, bool assembled, const TreeDesc *trees,
                                 SolveConsts c, SlabDev slab, long long g0, int npts,
                                 const int *nbr_cnt, const int *nbr_idx,
                                 const long long *col_off, const float *yo, const float *yb,
                                 const float *xb, float *xa, double *evals, int2 *info) {
  if (npts <= 0) return hipSuccess;
#define CWBL_KP_CASE(K)                                                                      \
  case K:                                                                                    \
    return launch_solve_kp<K>(s, assembled, trees, c, slab, g0, npts, nbr_cnt, nbr_idx,      \
                              col_off, yo, yb, xb, xa, evals, info);
  switch (kp) {
    CWBL_KP_CASE(8)
    CWBL_KP_CASE(16)
    CWBL_KP_CASE(24)
    CWBL_KP_CASE(32)
    CWBL_KP_CASE(40)
    CWBL_KP_CASE(48)
    CWBL_KP_CASE(56)
    CWBL_KP_CASE(64)
    default:
      return hipErrorInvalidValue;
  }
#undef CWBL_KP_CASE
}

hipError_t launch_solve_neighbors(hipStream_t s, int kp, const TreeDesc *trees,
                                  SolveConsts c, SlabDev slab, long long g0, int npts,
                                  const int *nbr_cnt, const int *nbr_idx,
                                  int2 *info) {
  return dispatch_solve(s, kp, false, trees, c, slab, g0, npts, nbr_cnt, nbr_idx, nullptr,
                        nullptr, nullptr, nullptr, nullptr, nullptr, info);
}

hipError_t launch_solve_assembled(hipStream_t s, int kp, SolveConsts c, int npts,
                                  const long long *col_off, const float *yo, const float *yb,
                                  const float *xb, float *xa, double *evals, int2 *info) {
  SlabDev none{};
  return dispatch_solve(s, kp, true, nullptr, c, none, 0, npts, nullptr, nullptr,
                        col_off, yo, yb, xb, xa, evals, info);
}

// per-batch reduction of the per-point info into DevStats: a grid-stride loop per block, a
// block reduction through LDS, and one atomic per counter per block
constexpr int kInfoThreads = 1024;
__global__ void __launch_bounds__(kInfoThreads)
reduce_info_kernel(const int2 *__restrict__ info, int n, DevStats *stats) {
  unsigned long long solved = 0, nobs = 0, noncv = 0, swsum = 0;
  unsigned int maxp = 0, maxsw = 0;
  for (int i = blockIdx.x * kInfoThreads + threadIdx.x; i < n; i += gridDim.x * kInfoThreads) {
    const int2 v = info[i];
    if (v.x > 0) {
      solved += 1;
      nobs += (unsigned long long)v.x;
      maxp = max(maxp, (unsigned)v.x);
      const int sw = v.y < 0 ? -v.y : v.y;
      maxsw = max(maxsw, (unsigned)sw);
      swsum += (unsigned long long)sw;
      noncv += v.y < 0 ? 1 : 0;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    solved += __shfl_xor(solved, off, 64);
    nobs += __shfl_xor(nobs, off, 64);
    noncv += __shfl_xor(noncv, off, 64);
    swsum += __shfl_xor(swsum, off, 64);
    maxp = max(maxp, (unsigned)__shfl_xor((int)maxp, off, 64));
    maxsw = max(maxsw, (unsigned)__shfl_xor((int)maxsw, off, 64));
  }
  constexpr int NW = kInfoThreads / 64;
  __shared__ unsigned long long red[4][NW];
  __shared__ unsigned int redm[2][NW];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = solved; red[1][w] = nobs; red[2][w] = noncv; red[3][w] = swsum;
    redm[0][w] = maxp; redm[1][w] = maxsw;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < NW; ++q) {
      solved += red[0][q]; nobs += red[1][q]; noncv += red[2][q]; swsum += red[3][q];
      maxp = max(maxp, redm[0][q]); maxsw = max(maxsw, redm[1][q]);
    }
    if (solved) atomicAdd(&stats->solved, solved);
    if (nobs) atomicAdd(&stats->nobs_sum, nobs);
    if (noncv) atomicAdd(&stats->nonconverged, noncv);
    if (swsum) atomicAdd(&stats->sweeps_sum, swsum);
    if (maxp) atomicMax(&stats->max_p, maxp);
    if (maxsw) atomicMax(&stats->max_sweeps, maxsw);
  }
}

hipError_t launch_reduce_info(hipStream_t s, const int2 *info, int n, DevStats *stats) {
  if (n <= 0) return hipSuccess;
  const int blocks = std::min(256, (n + kInfoThreads - 1) / kInfoThreads);
  hipLaunchKernelGGL(reduce_info_kernel, dim3(blocks), dim3(kInfoThreads), 0, s, info, n,
                     stats);
  return hipGetLastError();
}

}  // namespace cwbl
