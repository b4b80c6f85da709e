/*
 * cwb_letkf_core.h — C ABI of the MI355X LETKF analysis core.
 *
 * This is the drop-in boundary for the per-variable hot loop of the reference
 * LETKF (lopunch/CWBNWP-LETKF).  A Fortran host binds it with iso_c_binding
 * (see cwbnwp-letkf_amd/fortran/letkf_core_gpu.f90 and INTEGRATION.md); Python
 * binds it with ctypes (cwbnwp-letkf_amd/cwbl/abi.py).
 *
 * Entry point                reference interface it replaces
 * -------------------------  ------------------------------------------------------------
 * cwbl_init                  set_optimal_workspace_for_eigen + set_ensemble_constants
 *                            (module_eigen.f90:16-35, module_param.f90:241-247,
 *                            called at cwb_letkf.f90:37-38)
 * cwbl_set_obs               the obs state after gts%distribute / rad%distribute
 *                            (module_gts_omboma.f90:508-611, module_radar.f90:120-186),
 *                            i.e. wrfda_gts%platform(:) and cwb_radar%radarobs(:)
 * cwbl_analyze_var           one pass of letkf_driver's update loop for one variable:
 *                            build_tree x2 (module_letkf_core.f90:63-64) + the grid-point
 *                            loop (module_letkf_core.f90:209-240) + destroy_tree (:295)
 * cwbl_solve_batch           letkf_solve (module_letkf_core.f90:598-700) for many points
 *                            with pre-assembled yo/yb (KAT / diagnostics entry)
 * cwbl_search                build_tree + get_lz for one obs type
 *                            (module_localization.f90:35-167, 188-331) (KAT entry)
 * cwbl_finalize              destroy_eigen_array (module_eigen.f90:110-113)
 * cwbl_last_error            replaces `stop "<msg>"`: the library never exits
 *
 * Conventions
 *  - float <-> real(c_float), double <-> real(c_double), int <-> integer(c_int),
 *    long long <-> integer(c_long_long).  Fortran logicals cross as int 0/1.
 *  - Arrays are passed in the reference's Fortran (column-major) layout, first index
 *    fastest; the comment next to each pointer gives the Fortran shape.
 *  - Observation / result indices are 0-based on this side of the ABI.
 *  - All calls are synchronous, from one host thread per process; `memory` says whether
 *    the array pointers of a struct are host pointers (copied in/out inside the call) or
 *    HIP device pointers already resident on the library's device.
 *  - Device inputs only need to be *queued* on the caller's stream (cwbl_set_stream; the
 *    legacy null stream by default): every call that takes device pointers first makes the
 *    library's streams wait for an event recorded there, so work queued on OTHER streams
 *    (torch's non-default streams, an RCCL collective's stream) must be complete or ordered
 *    before that stream by the caller.  All library work on those buffers has completed when
 *    the call returns.
 *  - Return value 0 = success; nonzero = error code, message in cwbl_last_error().
 *  - There is no CPU fallback: without a usable gfx950 device every compute entry point
 *    returns CWBL_ERR_NO_DEVICE.
 */
#ifndef CWB_LETKF_CORE_H
#define CWB_LETKF_CORE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CWBL_ABI_VERSION 2

#define CWBL_MAX_NVAR        5   /* obs variables per GTS report (u,v,t,p,q) */
#define CWBL_NUM_GTS_TYPES  29   /* module_param.f90:172 num_gts_indexes     */
#define CWBL_NUM_RADAR_TYPES 4   /* module_param.f90:212 num_radar_indexes   */
#define CWBL_MAX_MEMBERS    128  /* largest k the solve kernels support      */

/* GTS type ids (module_param.f90:143-171); only these five are assimilated
 * (module_localization.f90:59-72). */
enum {
  CWBL_GTS_SOUND = 1, CWBL_GTS_SYNOP = 2, CWBL_GTS_GPSPW = 8,
  CWBL_GTS_METAR = 10, CWBL_GTS_SHIPS = 11
};
/* radar type ids (module_param.f90:208-211) */
enum { CWBL_RADAR_DBZ = 1, CWBL_RADAR_VR = 2, CWBL_RADAR_ZDR = 3, CWBL_RADAR_KDP = 4 };

enum { CWBL_MEM_HOST = 0, CWBL_MEM_DEVICE = 1 };

enum {
  CWBL_OK = 0,
  CWBL_ERR_ARG = 1,          /* invalid argument / shape                        */
  CWBL_ERR_STATE = 2,        /* call order (e.g. analyze before init/set_obs)    */
  CWBL_ERR_NO_DEVICE = 3,    /* no HIP device / wrong architecture              */
  CWBL_ERR_HIP = 4,          /* HIP runtime error                               */
  CWBL_ERR_UNSUPPORTED = 5,  /* configuration outside this build (e.g. k > 128)  */
  CWBL_ERR_OOM = 6
};

/* Q1: build_tree picks the tree dimension from the last type appended
 * (module_localization.f90:151).  CWBL_Q1_REPLICATE follows it wherever the result is
 * defined (a 3-D type in a 2-D tree family is searched in 2-D); a 2-D type in a 3-D
 * family reads an undefined qv(3) in the reference, and is searched in 2-D with its own
 * tree (counted in cwbl_stats.q1_undefined).  CWBL_Q1_PER_TYPE uses every type's own
 * vclr for its tree. */
enum { CWBL_Q1_REPLICATE = 0, CWBL_Q1_PER_TYPE = 1 };

typedef struct cwbl_init_params {
  int    nmember;          /* k = config%nmember (module_config.f90:306), 2..128 */
  int    device;           /* HIP device ordinal, -1 = current device */
  int    weight_function;  /* 0 Gaussian, 1 Gaspari-Cohn (module_config.f90:307) */
  float  norain_value;     /* control_nml norain_value (module_config.f90:295) */
  int    q1_mode;          /* CWBL_Q1_* */
  int    reserved;
  size_t workspace_bytes;  /* device workspace budget for neighbour lists (0 = 2 GiB); the
                            * solve's per-batch records come on top: 6.9 KB per point of a
                            * search batch at k = 17..40 (two buffers); at k = 65..128 the
                            * hand-off records (135 KB per point) are bounded by this value
                            * when it is given, else by min(13 GB, 40% of the device memory
                            * free at cwbl_init), with sub-batches shrunk to fit */
} cwbl_init_params;

/* One GTS platform: type(gts_structure), module_gts_omboma.f90:13-22. */
typedef struct cwbl_gts_obs {
  int          type_id;   /* CWBL_GTS_* */
  int          nvar;      /* 5 synop/metar/ships, 4 sound, 1 gpspw */
  int          nobs;
  int          reserved;
  const float *xyz;       /* xyz(3,nobs), projected metres (module_param.f90:7) */
  const float *obs;       /* obs(nvar,nobs) */
  const float *error;     /* error(nvar,nobs) */
  const float *hdxb;      /* hdxb(nvar,nobs,0:k-1) = H(x_b) per member (:171) */
  const int   *qc;        /* qc(nvar,nobs,0:k-1) */
} cwbl_gts_obs;

/* One radar variable: type(radar_structure), module_radar.f90:13-16. */
typedef struct cwbl_radar_obs {
  int          type_id;   /* CWBL_RADAR_* */
  int          nobs;
  const float *xyz;       /* xyz(3,nobs), metres */
  const float *obs;       /* obs(nobs) */
  const float *hdxb;      /* hdxb(nobs,0:k-1) */
} cwbl_radar_obs;

typedef struct cwbl_obs_set {
  int                   n_gts;
  int                   n_radar;
  const cwbl_gts_obs   *gts;     /* at most one entry per type id */
  const cwbl_radar_obs *radar;
  int                   memory;  /* CWBL_MEM_HOST / CWBL_MEM_DEVICE for the arrays */
  int                   reserved;
} cwbl_obs_set;

/* Namelist values of one obs type for the current variable (index ivar of the
 * per-variable arrays): gts_config / radar_variable_config, module_config.f90:7-34. */
typedef struct cwbl_type_params {
  int   use_it;                    /* %use_it */
  int   max_lz_pts;                /* %max_lz_pts */
  float hclr;                      /* %hclr(ivar) in km; <= 0 disables the type */
  float vclr;                      /* %vclr(ivar) in km; <= 0 = no vertical localization */
  float err_muti[CWBL_MAX_NVAR];   /* GTS: per obs variable %u..%q%err_muti; radar: [0] = %error */
  float err_rej[CWBL_MAX_NVAR];    /* GTS: per obs variable; radar: [0] = %err_rej */
  int   is_assim[CWBL_MAX_NVAR];   /* GTS: %u..%q%is_assim(ivar); radar: unused (hclr>0) */
} cwbl_type_params;

typedef struct cwbl_var_params {
  float multi_infl;      /* inflation_nml multi_infl(ivar): inflat=(k-1)/multi_infl (:68) */
  int   use_rtpp;
  float rtpp_alpha;
  int   use_rtps;
  float rtps_alpha;
  int   tune_q;          /* 1: letkf_tune_q (module_letkf_core.f90:702-733) on the analysed
                          * region after the analysis, as letkf_driver does for the Q
                          * species (QVAPOR ... QNHAIL, :253-278); Q3 (0/0 = NaN) replicated */
  cwbl_type_params gts[CWBL_NUM_GTS_TYPES];     /* index = gts type id - 1 */
  cwbl_type_params radar[CWBL_NUM_RADAR_TYPES]; /* index = radar type id - 1 */
} cwbl_var_params;

/* One variable's local slab, exactly as letkf_driver holds it (module_letkf_core.f90:85,
 * 171-172, 192-193): var(nx,ny,nz,0:k-1), lat/lon -> x/y(nx,ny), alt(alt_nx,alt_ny,nz). */
typedef struct cwbl_slab {
  int          nx, ny, nz;      /* leading dims of var and x/y */
  int          alt_nx, alt_ny;  /* leading dims of alt (cpu%loc_nx, cpu%loc_ny) */
  int          ix_lim, iy_lim;  /* analysed columns: i < ix_lim, j < iy_lim (:209-210, Q2) */
  int          memory;          /* CWBL_MEM_HOST / CWBL_MEM_DEVICE */
  const float *x;               /* proj%lonlat_to_xy(lon,lat)(1) per column, (nx,ny) */
  const float *y;               /* ... (2) */
  const float *alt;             /* alt(alt_nx,alt_ny,nz) metres */
  float       *var;             /* in/out var(nx,ny,nz,0:k-1) */
} cwbl_slab;

typedef struct cwbl_stats {
  long long points;          /* grid points visited (ix_lim*iy_lim*nz) */
  long long solved;          /* points with >= 1 accepted obs (letkf_solve called) */
  long long nobs_sum;        /* sum of p over solved points */
  long long lz_truncated;    /* (point, type) searches that hit max_lz_pts (Q4) */
  long long nonconverged;    /* Jacobi: eigensolves that hit the sweep cap (LAPACK info is */
                             /* ignored, module_eigen.f90:49); quadrature: points whose */
                             /* spectrum bound exceeds the last rule (max/min > 1e12) */
  long long q1_undefined;    /* (point, type) searches in the Q1 undefined case */
  long long sweeps_sum;      /* solver effort summed over solved points: Jacobi sweeps, or */
                             /* the quadrature rule's decade (default solver) */
  int       max_p;           /* max p over points */
  int       max_sweeps;      /* max of the same */
  int       ntrees;          /* trees built for this variable */
  int       reserved;
  double    ms_total;        /* wall time of the call */
  double    ms_prep;         /* tree build + obs QC tables */
  double    ms_search;       /* neighbour search kernels */
  double    ms_solve;        /* solve kernels (+ the tune_q pass when requested) */
  double    ms_copy;         /* host<->device copies of the slab (host memory only; for a */
                             /* pageable slab: host time in its page-locked bounce copies) */
} cwbl_stats;

int         cwbl_init(const cwbl_init_params *params);
/* Device-memory calls (CWBL_MEM_DEVICE and the transpose helpers) are ordered after the work
 * queued so far on the caller's stream: an event recorded there, waited on by the library's
 * own streams.  `stream` is a hipStream_t (NULL = the legacy null stream, the default).  No
 * reference counterpart: the reference has no device (its arrays are complete on entry). */
int         cwbl_set_stream(void *stream);
int         cwbl_set_obs(const cwbl_obs_set *obs);
int         cwbl_analyze_var(const cwbl_var_params *vp, const cwbl_slab *slab,
                             cwbl_stats *stats /* nullable */);

/* letkf_solve for npts points (module_letkf_core.f90:598-700).  Point i uses columns
 * [col_off[i], col_off[i+1]) of yo(ncol) and yb(k,ncol) (member fastest), xb(k,npts) ->
 * xa(k,npts).  evals (nullable) receives the eigenvalues of inflat*I + yb yb^T per point in
 * ascending order (k,npts), as dsyevd returns them in inverse_matrix (module_eigen.f90:48-49;
 * the reference keeps 1/lambda in eigen::eval afterwards), at every k <= 128. */
int         cwbl_solve_batch(int npts, const long long *col_off, const float *yo,
                             const float *yb, const float *xb, float inflat,
                             int use_rtpp, float rtpp_alpha, int use_rtps, float rtps_alpha,
                             float *xa, double *evals, int memory);

/* build_tree + get_lz for one obs type: obs_xyz(3,nobs) metres, hclr/vclr km
 * (vclr <= 0: 2-D), queries q_xyz(3,nq).  nfound(nq); idx/r2 (max_lz_pts,nq) in the
 * reference's traversal order (0-based obs indices). */
int         cwbl_search(int nobs, const float *obs_xyz, float hclr, float vclr,
                        int max_lz_pts, int nq, const float *q_xyz,
                        int *nfound, int *idx, float *r2, int memory);

/* ---- member <-> column transposes -----------------------------
 * The reference moves each variable between member layout (rank m holds member m's field
 * global(nx,ny,nz)) and column layout (each rank holds var(loc_nx,loc_ny,nz,0:k-1) for its
 * columns) with mpi_alltoallv (module_mpi_util.f90:190-358).  Columns are split cyclically,
 * block 1, over a px x py rank grid (letkf_local_info, :71-188; px >= py from
 * mpi_dims_create): rank r = id_x + id_y*px owns x = id_x + i*px, y = id_y + j*py (0-based).
 * The exchange itself is RCCL point-to-point (cwbl/transpose.py); these entry points do the
 * packing in device memory (all pointers are device pointers; px, py <= 64; each call has
 * completed when it returns). */

/* letkf_scatter_grid's send side (:224-258): global(nx,ny,nz) -> send, the rank-major
 * concatenation of global(xloc_r, yloc_r, :) for r = 0..px*py-1, each chunk
 * (loc_nx_r, loc_ny_r, nz) in Fortran order. */
int         cwbl_pack_columns(const float *global, int nx, int ny, int nz, int px, int py,
                              float *send);
/* letkf_gather_grid's receive side (:326-350): the inverse of cwbl_pack_columns. */
int         cwbl_unpack_columns(const float *recv, int nx, int ny, int nz, int px, int py,
                                float *global);
/* The same for nm member fields in one launch (the members a rank owns, k/N of them on an
 * N-GPU node): member i is global + i*gstride -> send + i*sstride (strides in elements, >= the
 * field's nx*ny*nz when nm > 1), and back. */
int         cwbl_pack_members(const float *global, long long gstride, int nm, int nx, int ny,
                              int nz, int px, int py, float *send, long long sstride);
int         cwbl_unpack_members(const float *recv, long long rstride, int nm, int nx, int ny,
                                int nz, int px, int py, float *global, long long gstride);
/* letkf_scatter_vcoord's reduction (:491-505): ph(n2d, nz_ph, 0:k-1), member slowest ->
 * alt(n2d, nz_out).  tmp = sgemv('n', n2d*nz_ph, k, 1.0/(g*k), ph, ., ones, 0.0) evaluated
 * in the reference BLAS order (y = 0; y += (alpha*1)*ph(:,m), m = 0..k-1, fp32); then
 * stagger 1: alt = tmp (nz_out = nz_ph); stagger 0: alt = (tmp(:,2:) + tmp(:,:nz_ph-1))*0.5
 * (nz_out = nz_ph - 1). */
int         cwbl_vcoord_mean(const float *ph, long long n2d, int nz_ph, int k, int stagger,
                             float g, float *alt);

/* ---- ensemble mean of the analysis (write_mean, module_grid.f90:700-840; SURVEY.md §8(f)
 * rank 4) ------------------------------------------------------------------------------------
 * The reference sums every analysed field over the member ranks with one mpi_reduce each
 * (:744-822) and scales the root's sums by nmember_inv with sscal (:827-...).  Here a rank
 * sums the members it holds (cwbl/transpose.py deals k/N members per rank), all fields packed
 * in one buffer; ONE RCCL reduce of that buffer follows, then the scale on the root.  Device
 * pointers; each call has completed when it returns. */
/* out(i) = sum over m = 0..nm-1 of fields(i, m), fp32, sequential in member order;
 * fields(n, nm) member slowest. */
int         cwbl_member_sum(const float *fields, long long n, int nm, float *out);
/* x(i) = alpha * x(i) (sscal, :827-...). */
int         cwbl_scale(float *x, long long n, float alpha);

/* ---- kernel timing (measurement; no reference counterpart) -------------------------------
 * With timing on, cwbl_analyze_var brackets every search and solve launch with a HIP event
 * pair on the stream the launch runs on and, after the call's final synchronisation, adds
 * the pair's elapsed time to that kernel's sum.  cwbl_set_kernel_timing(1) switches timing
 * on and clears the sums (0 switches it off); cwbl_kernel_times copies up to `cap` entries,
 * one per kernel launched since, and stores the number of such kernels in *n. */
typedef struct cwbl_kernel_time {
  char      name[64];   /* the kernel as rocprofv3 names it, template arguments included */
  long long launches;
  long long points;     /* grid points the launches processed (0: flagged-point re-search) */
  double    ms;         /* summed HIP-event time */
} cwbl_kernel_time;
int         cwbl_set_kernel_timing(int enable);
int         cwbl_kernel_times(cwbl_kernel_time *out, int cap, int *n);

/* ---- path options (no reference counterpart) ---------------------------------------------
 * The library reads no environment variable but OMP_NUM_THREADS (which caps the host threads
 * of the pageable-slab bounce fallback).  The alternative kernel paths and batch sizes below
 * are kept for A/B measurement and for the parity tests that compare one path with another;
 * they are set after cwbl_init, which resets every option to its default.  A value outside
 * an option's range returns CWBL_ERR_ARG.  No option changes a result beyond the fp64
 * summation order of the solve (every path meets the same parity bar). */
enum {
  CWBL_OPT_SOLVER = 1,         /* 0 Householder + quadrature (default); 1 the Jacobi
                                * eigensolver (k <= 64, analysis and solve_batch) */
  CWBL_OPT_SPLIT40 = 2,        /* k = 17..40: 1 assembly record + four-point solve (default);
                                * 0 the one-wavefront kernel */
  CWBL_OPT_SPLIT40_BATCH = 3,  /* points per record sub-batch of that path (0 = search batch) */
                               /* (4: the r4 two-stream record path, removed in r6: a tie) */
  CWBL_OPT_SEARCH = 5,         /* 0 uniform bins + tree for truncated lists (default); 1 the
                                * k-d tree walk for every point */
  CWBL_OPT_BIG_PATH = 6,       /* k = 65..128: 1 256-thread hand-off + one-wave tail (default);
                                * 0 one 256-thread kernel */
  CWBL_OPT_BIG_BATCH = 7,      /* points per k > 64 sub-batch (>= 64; default 98 304) */
  CWBL_OPT_PAGEABLE = 8,       /* pageable host slab: 0 page-lock in place (default); 1 bounce
                                * through the library's page-locked slots */
  CWBL_OPT_BIN_DIV = 9,        /* search bin side = radius / value, 1..8 (0 = by obs density);
                                * applies to the next cwbl_analyze_var (cached bins of another
                                * divisor are rebuilt) */
  CWBL_OPT_LEAD_DIV = 10,      /* first search batch = points / value (0 = off, default) */
  CWBL_OPT_MAX_BATCH = 11,     /* points per search batch, >= 256 (0 = automatic, default) */
  CWBL_OPT_INFO_WINDOW = 12    /* points per reduction of the per-point solve info, >= 256
                                * (0 = 2^25, default; smaller values exercise the rollover) */
};
int         cwbl_set_option(int option, long long value);

int         cwbl_finalize(void);
const char *cwbl_last_error(void);
int         cwbl_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* CWB_LETKF_CORE_H */
