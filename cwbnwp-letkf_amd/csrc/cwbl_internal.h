// cwbl_internal.h — data layouts shared by the host orchestration (cwbl_abi.hip),
// the host k-d tree builder (kdtree_build.cpp) and the HIP kernels (cwbl_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

namespace cwbl {

// One node of a flattened kdtree2 tree (module_kdtree2.f90:512-528).  64 bytes.
struct TreeNode {
  float cut_val, cut_val_left, cut_val_right;
  int   cut_dim;          // 0..2 for internal nodes, -1 for terminal (bucket) nodes
  float lo[3];            // node%box(:)%lower (final, union of children)
  float hi[3];            // node%box(:)%upper
  int   left, right;      // child node indices (-1 = null)
  int   l, u;             // inclusive range into the permuted data
  int   pad_[2];
};
static_assert(sizeof(TreeNode) == 64, "TreeNode layout");

// Host-side result of building one tree.
struct HostTree {
  int dim = 3;
  int n = 0;
  std::vector<TreeNode> nodes;     // root = 0
  std::vector<int>      ind;       // permutation (0-based obs index of rearranged slot)
  std::vector<float>    rdata;     // rearranged normalised coords, 4 floats per slot
};

// kdtree2_create(xyz(3,n), dim) with the reference's settings (bucket 12, exact median,
// rearranged data).  xyz3 is already normalised by hclr/vclr as in build_tree.
void build_kdtree(const float *xyz3, int n, int dim, HostTree &out);

// Per-tree descriptor handed to the kernels (device-resident array of these).
struct TreeDesc {
  const TreeNode *nodes;
  const float4   *rdata;      // rearranged normalised coords (x,y,z,0)
  const int      *ind;
  // column table of this type for the current variable, one column per (tree slot,
  // obs-var): column slot*nvar + v belongs to obs ind[slot]
  const float    *col_bg;     // [n*nvar][KP] fp32 bg = hdxb - mean, zero padded
  const float    *col_omm;    // [n*nvar] obs - mean
  const float    *col_err;    // [n*nvar] error * err_muti
  const uint8_t  *col_ok;     // [n*nvar] accepted (is_assim, qc, gross-error tests)
  float hclr_inv, vclr_inv;   // this type's own normalisation (get_lz)
  int   tree_dim;             // dimension the tree was built with
  int   query3d;              // this type queries in 3-D (own vclr > 0)
  int   nvar;
  int   max_lz;
  int   list_off;             // offset of this type inside a point's neighbour list
  int   q1_undef;
  // uniform bins over the same normalised coordinates (search_binned_kernel): cell
  // (ix, iy, iz) = floor((x - b0) * binv) per dimension, cells x-fastest; bxyz holds the
  // points cell by cell (tree-slot order within a cell) with the slot in .w (int bits),
  // bstart[c] .. bstart[c + 1] the points of cell c
  const float4 *bxyz;
  const int    *bstart;
  float bx0, by0, bz0, binv;
  int   nbx, nby, nbz;
};

// Host-side bins of one tree (build_bins, kdtree_build.cpp).
struct HostBins {
  float x0 = 0.0f, y0 = 0.0f, z0 = 0.0f, binv = 1.0f;
  int nbx = 1, nby = 1, nbz = 1;
  std::vector<float> xyzs;   // 4 floats per point: x, y, z, slot (int bits)
  std::vector<int> start;    // ncells + 1
};
// Bins of side ~r/2 (r: the search radius in normalised units) over a built tree's
// rearranged coordinates; dim 2 ignores z.  Capped at 2^22 cells.
void build_bins(const HostTree &t, int dim, float r, HostBins &out, int div = 2);

// Per-variable constants of the solve.
struct SolveConsts {
  int   k;
  int   kp;                   // padded member count of the kernel instantiation
  int   ntrees;
  int   list_cap;             // sum of max_lz over trees
  int   weight_function;
  int   use_rtpp, use_rtps;
  float inflat, rtpp_alpha, rtps_alpha;
  float nmember_inv;          // 1.0/k (module_param.f90:245)
  float r2;                   // gc1999**2
  int   max_sweeps;           // Jacobi sweep cap (CWBL_DEBUG_MAX_SWEEPS overrides; ablation only)
  const double2 *quad;        // = quad_r (non-null once the tables are built)
  const double2 *quad_r;      // [4][kQuadLevels][kQuadStride] (t2, w) of the x^-1/2 rules of
                              // 8 R - 1 nodes, R = 2, 3, 4, 8 (quad_rule)
  int   debug_stop;           // CWBL_DEBUG_TQ_STOP: 1 = after assembly, 2 = after
                              // tridiagonalisation, 3 = after quadrature, 4 = after the first
                              // kTq40J0 steps of solve_tq40_kernel (timing ablation only)
  int   debug_steps;          // CWBL_DEBUG_TQ_STEPS: > 0 runs only that many Householder steps
                              // in solve_tq_big_kernel (timing ablation only)
};
// The timing-ablation exits read debug_stop / debug_steps only in `make DEBUG_KNOBS=1`
// builds; in the release library they are the constant 0 and the branches compile away.
#ifdef CWBL_DEBUG_KNOBS
#define CWBL_DBG_STOP(c) ((c).debug_stop)
#define CWBL_DBG_STEPS(c) ((c).debug_steps)
#else
#define CWBL_DBG_STOP(c) 0
#define CWBL_DBG_STEPS(c) 0
#endif

// Inverse-square-root quadrature of the tq kernels (quad_tables.cpp): level L = 1..kQuadLevels
// covers spectrum bounds with max/min <= 10^L.  The one-wavefront kernels run kQuadNodes nodes
// per pass (64 lanes = 32 nodes x 2 sides, node 31 of the first pass the exact T^-1 solve):
// one pass (31 nodes) up to level kQuadLevels31, two (63 nodes) above; beyond 10^24 a point is
// counted non-converged.  Tables hold kQuadStride (t2, w) entries per level.
constexpr int kQuadNodes = 31;
constexpr int kQuadLevels = 24;
constexpr int kQuadLevels31 = 12;
constexpr int kQuadStride = 64;
void quad_table(int level, double2 *out64, int nodes = kQuadNodes);
// Rounds of 8 nodes (the last round's slot 7 is the exact T^-1 solve) solve_tq40_kernel runs
// at a level: the fewest whose (8 R - 1)-node rule stays within 1e-12 relative error where the
// 31-node rule does (levels 1..7), and the 31-node rule itself up to level 12, 63 nodes above
// (tests/test_quadrature.py: 15 nodes <= 2.1e-13 to level 3, 23 nodes <= 6.4e-14 to level 5).
// r6: 15 nodes at level 3 (C2: two thirds of the points, so nearly every wave of four) instead
// of 23 — one quadrature round fewer per wave; the error stays ~1e7 below the fp32 rounding of
// the analysis.
__host__ __device__ constexpr int quad_rounds(int level) {
  return level <= 3 ? 2 : level <= 5 ? 3 : level <= kQuadLevels31 ? 4 : 8;
}
// passes of the one-wavefront kernels' rule (31 nodes per pass + the exact solve)
__host__ __device__ constexpr int quad_passes(int level) { return level <= kQuadLevels31 ? 1 : 2; }
// the (8 R - 1)-node rule of a level, R = 2, 3, 4 or 8
__host__ __device__ inline const double2 *quad_rule(const double2 *quad_r, int R, int level) {
  return quad_r + ((size_t)(R == 8 ? 3 : R - 2) * kQuadLevels + (level - 1)) * kQuadStride;
}

// Point enumeration of a slab: g = i + ix_lim*(j + iy_lim*kz).
struct SlabDev {
  int nx, ny, nz, alt_nx, alt_ny, ix_lim, iy_lim;
  long long L;                // nx*ny*nz (member stride of var)
  const float *x, *y, *alt;
  float *var;
};

// Device-side counters (atomics) reported through cwbl_stats.
struct DevStats {
  unsigned long long solved, nobs_sum, lz_truncated, nonconverged, q1_undefined, sweeps_sum;
  unsigned int max_p, max_sweeps;
};

// Kernel launchers (cwbl_kernels.hip).
hipError_t launch_obs_prep(hipStream_t s, int k, int kp, int family, int type_id, int nvar,
                           int nobs, const float *obs, const float *error, const float *hdxb,
                           const int *qc, const float err_muti[5], const float err_rej[5],
                           const int is_assim[5], float norain, const int *slot_obs,
                           float *col_bg, float *col_omm, float *col_err, uint8_t *col_ok);

// Cyclic (block 1) column decomposition of letkf_local_info (module_mpi_util.f90:71-188) on a
// px x py rank grid: rank r = id_x + id_y*px owns x = id_x + i*px, y = id_y + j*py.
constexpr int kMaxRankDim = 64;
struct Decomp {
  int nx, ny, nz, px, py;
  int cols_before[kMaxRankDim];  // columns owned by rank coordinates a < id_x
  int rows_before[kMaxRankDim];  // rows owned by rank coordinates b < id_y
};
void make_decomp(Decomp &d, int nx, int ny, int nz, int px, int py);
hipError_t launch_pack_columns(hipStream_t s, const float *global, const Decomp &d,
                               float *send);
hipError_t launch_unpack_columns(hipStream_t s, const float *recv, const Decomp &d,
                                 float *global);
// nm member fields at once (member i at src + i sstride -> dst + i dstride, in elements)
hipError_t launch_transpose_columns(hipStream_t s, bool unpack, const float *src,
                                    long long sstride, int nm, const Decomp &d, float *dst,
                                    long long dstride);
hipError_t launch_vcoord_mean(hipStream_t s, const float *ph, long long n2d, int nz_ph, int k,
                              int stagger, float alpha, float *alt);
hipError_t launch_member_sum(hipStream_t s, const float *fields, long long n, int nm,
                             float *out);
hipError_t launch_scale(hipStream_t s, float *x, long long n, float alpha);

// letkf_tune_q over the analysed region of s.var (module_letkf_core.f90:702-733)
hipError_t launch_tune_q(hipStream_t st, SlabDev s, int k);

// depth: the deepest tree's level count (tree_depth), which sizes the traversal stacks
hipError_t launch_search(hipStream_t s, const TreeDesc *trees, int ntrees, int depth,
                         int list_cap, float r2, SlabDev slab, long long g0, int npts,
                         int *nbr_cnt, int *nbr_idx, float *nbr_r2, DevStats *stats);

// nbr_idx holds tree slots (search with nbr_r2 = nullptr); the solve recomputes r2
hipError_t launch_solve_neighbors(hipStream_t s, int kp, const TreeDesc *trees,
                                  SolveConsts c, SlabDev slab, long long g0, int npts,
                                  const int *nbr_cnt, const int *nbr_idx, int2 *info);

hipError_t launch_solve_assembled(hipStream_t s, int kp, SolveConsts c, int npts,
                                  const long long *col_off, const float *yo, const float *yb,
                                  const float *xb, float *xa, double *evals, int2 *info);

// Tridiagonalisation + quadrature solve (cwbl_tq.hip); same data contract as the two
// launchers above.  `tri` (assembled mode only): T of every point for launch_tridiag_eigvals.
hipError_t launch_solve_tq(hipStream_t s, int kp, bool assembled, const TreeDesc *trees,
                           SolveConsts c, SlabDev slab, long long g0, int npts,
                           const int *nbr_cnt, const int *nbr_idx,
                           const long long *col_off, const float *yo, const float *yb,
                           const float *xb, float *xa, int2 *info, double *tri = nullptr);

constexpr int kTq4KP = 40;  // KP of the split record path (k = 25..40)

// The default KP = 40 split: assemble_record_kernel (cwbl_tq.hip) only stages and assembles,
// one point per wavefront, and writes A = inflat I + Yb Yb^T (packed lower, the padding's
// diagonal 1) and b1 = Yb d; solve_tq40_kernel (cwbl_tq40.hip) runs the whole
// tridiagonalisation with four points per wavefront (the first kTq40J0 steps on full rows
// J0..KP-1 plus the prefix rows' top-left block, then 16-lane rows of the trailing 32 x 32
// matrix), solves and writes var in place.
constexpr int kTq40J0 = 8;
constexpr int kRecordWaves = 4;  // waves per SIMD of the record kernel (assemble_record_kernel)
template <int KP>
struct AsmRecord {
  static constexpr int TA = 0;                   // A(r, c), c <= r, at r (r + 1) / 2 + c
  static constexpr int U1 = KP * (KP + 1) / 2;   // b1 = Yb d (KP)
  static constexpr int WORDS = (U1 + KP + 1) / 2 * 2;
};
hipError_t launch_assemble_record(hipStream_t s, int kp, const TreeDesc *trees, SolveConsts c,
                                  SlabDev slab, long long g0, int npts, const int *nbr_cnt,
                                  const int *nbr_idx, int2 *info, double *ws);
hipError_t launch_solve_tq40(hipStream_t s, int kp, SolveConsts c, SlabDev slab, long long g0,
                             int npts, double *ws, int2 *info);

// Split form of the KP = 128 slab path (configs[3]: k = 97..128).  solve_tq_big_kernel<128,
// false, kBigJ0> assembles A and runs the first kBigJ0 Householder steps (4x4 register
// blocks over 256 threads, one point per workgroup), then hands the trailing
// (KP-J0)^2 matrix, its J0 reflectors, T so far and Q^T b1, Q^T x' over through the
// workspace (BigHandoff, info[gi] = (p, 0)); solve_tqb_tail_kernel (cwbl_tq_tail.hip)
// finishes with one point per wavefront, lane l holding the full trailing row J0 + l.
// (KP = 96, k = 65..96: the same with the hand-off after 32 steps)
constexpr int kBigSplitKP = 128;
constexpr int kBigJ0 = 64;
constexpr int big_split_j0(int kp) { return kp - 64; }
// fp64 words of one point's hand-off record
template <int KP, int J0>
struct BigHandoff {
  static constexpr int KT = KP - J0;        // trailing rows
  static constexpr int TA = 0;              // trailing A, full: (r, c) at TA + c*KT + r
  static constexpr int HV = TA + KT * KT;   // reflector j < J0 at HV + j*KP + row (rows > j)
  static constexpr int D = HV + J0 * KP;    // d_0 .. d_{J0-1}
  static constexpr int E = D + J0;          // c(j, j+1), j = 0..J0-1
  static constexpr int TAU = E + J0;        // tau_0 .. tau_{J0-1}
  static constexpr int U1 = TAU + J0;       // Q_J0^T b1 (KP)
  static constexpr int U2 = U1 + KP;        // Q_J0^T x' (KP)
  static constexpr int BT = U2 + KP;        // tail scratch: its reflector rows (KT x KT)
  static constexpr int WORDS = BT + KT * KT;
};
hipError_t launch_big_handoff(hipStream_t s, int kp, const TreeDesc *trees, SolveConsts c,
                              SlabDev slab, long long g0, int npts, const int *nbr_cnt,
                              const int *nbr_idx, int2 *info, double *ws);
// KP = 128: the half-row hand-off kernel (cwbl_tq_rows.hip), launched by launch_big_handoff
hipError_t launch_rows_handoff(hipStream_t s, const TreeDesc *trees, SolveConsts c, SlabDev slab,
                               long long g0, int npts, const int *nbr_cnt, const int *nbr_idx,
                               int2 *info, double *ws);
hipError_t launch_solve_tqb_tail(hipStream_t s, int kp, SolveConsts c, SlabDev slab,
                                 long long g0, int npts, double *ws, int2 *info);

// KP = 96, 128: one 256-thread workgroup per point (cwbl_tq_big.hip)
hipError_t launch_solve_tq_big(hipStream_t s, int kp, bool assembled, const TreeDesc *trees,
                               SolveConsts c, SlabDev slab, long long g0, int npts,
                               const int *nbr_cnt, const int *nbr_idx,
                               const long long *col_off, const float *yo, const float *yb,
                               const float *xb, float *xa, int2 *info, double *tri = nullptr);

// Eigenvalues of the tridiagonal T = Q^T A Q the tq kernels form (assembled mode, `tri`:
// per point d_0..d_{KP-1} then c(i, i+1), 2 KP words): ascending, by Sturm-count bisection
// in fp64 (cwbl_eig.hip), i.e. the eigenvalues of A that dsyevd returns (module_eigen.f90:49)
hipError_t launch_tridiag_eigvals(hipStream_t s, int kp, int k, int npts, const double *tri,
                                  double *evals);

// The analysis search from uniform bins: the same fixed-radius sets as launch_search (the
// same fp32 distances and <= r2 test) in bin order, which differs from kdtree2's visiting
// order; a point whose list would pass max_lz on any tree is appended to flag_idx
// (flag_cnt, zeroed by the caller) for launch_search_flagged, which reruns the tree search
// there so Q4 truncation keeps the reference's order.  rbox: the bounding-box half-width,
// sqrt(r2) with a margin.
hipError_t launch_search_binned(hipStream_t s, const TreeDesc *trees, int ntrees, int list_cap,
                                float r2, float rbox, SlabDev slab, long long g0, int npts,
                                int *nbr_cnt, int *nbr_idx, int *flag_cnt, int *flag_idx);
hipError_t launch_search_flagged(hipStream_t s, const TreeDesc *trees, int ntrees, int depth,
                                 int list_cap, float r2, SlabDev slab, long long g0, int npts,
                                 const int *flag_cnt, const int *flag_idx, int *nbr_cnt,
                                 int *nbr_idx, DevStats *stats);

hipError_t launch_search_single(hipStream_t s, const TreeDesc *tree, int depth, float r2,
                                int nq, const float *q_xyz, int max_lz, int *nfound, int *idx,
                                float *r2out);

hipError_t launch_reduce_info(hipStream_t s, const int2 *info, int n, DevStats *stats);

constexpr int kSearchStackDepth = 40;  // max k-d tree depth the search kernel supports

// Neighbour lists of the analysis path are interleaved by groups of kListLanes points and
// kListGroup slots: slot s of point g lives at list_index(g, cap, off) + list_slot(s).  A
// search wave then stores 16 B per lane side by side (whole cache lines) instead of 64
// scattered 4-B streams, and a solve reading 32 consecutive slots of one point touches 8
// lines instead of 32.  cap and off are multiples of kListGroup (list_span); buffers hold
// round_up(npts, kListLanes) * cap entries.
constexpr int kListLanes = 64;
constexpr int kListGroup = 4;
// points of padding after a tree's bins: search_binned_kernel reads ahead past a run's end
constexpr int kBinPad = 8;
__host__ __device__ inline int list_span(int max_lz) {
  return (max_lz + kListGroup - 1) / kListGroup * kListGroup;
}
__host__ __device__ inline long long list_index(long long g, int cap, int off) {
  return (g / kListLanes) * (long long)cap * kListLanes + (long long)off * kListLanes +
         (g % kListLanes) * kListGroup;
}
__host__ __device__ inline unsigned list_slot(int s) {  // s >= 0
  return (unsigned)s / kListGroup * (kListGroup * kListLanes) + (unsigned)s % kListGroup;
}

int supported_kp(int k);      // smallest compiled KP >= k, or -1
// sets the message cwbl_last_error() returns and returns `code` (cwbl_abi.hip)
int set_last_error(int code, const char *msg);
constexpr int kMaxWaveKP = 64;  // largest KP of the one-wavefront kernels

}  // namespace cwbl
