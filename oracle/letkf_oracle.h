/*
 * letkf_oracle.h — CPU restatement of the reference LETKF hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product library (cwbnwp-letkf_amd/) links,
 * loads or calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker / reported CPU baseline.
 *
 * Parity of this restatement is pinned against the reference itself: oracle/ref/
 * builds the reference's own kdtree2, eigen, param and config modules and the
 * reference's letkf_solve / Gaspari_Cohn_1999 source text with amdflang + MKL
 * (oracle/_ref/ref_harness), and tests/golden/ holds the vectors it produced.
 */
#ifndef LETKF_ORACLE_H
#define LETKF_ORACLE_H

#include "../include/cwb_letkf_core.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Which LAPACK/BLAS the solve uses: "mkl" (dsyevd etc. through libmkl_rt, same calls
 * as module_letkf_core.f90:649-675 / module_eigen.f90:48-93) or "builtin-jacobi". */
const char *orc_lapack_name(void);
int         orc_lapack_init(void);   /* 1 = LAPACK found, 0 = builtin fallback */

float orc_expf(float x);             /* glibc 2.35 __expf_fma, bit-exact replica */
float orc_gaspari_cohn(float x);     /* module_localization.f90:333-364 */
float orc_search_r2(void);           /* gc1999**2, module_localization.f90:202 */

typedef struct orc_kdtree orc_kdtree;
/* kdtree2_create(input_data(3,n), dim) with rearrange=.true., sort=.false.
 * (module_kdtree2.f90:598-680) */
orc_kdtree *orc_kdtree_create(const float *xyz3, int n, int dim);
/* kdtree2_r_nearest (module_kdtree2.f90:1118-1179): returns nfound (<= nalloc);
 * idx (0-based) and dis in traversal order; *overflow set when truncated. */
int  orc_kdtree_r_nearest(const orc_kdtree *t, const float *qv, float r2, int nalloc,
                          int *idx, float *dis, int *overflow);
void orc_kdtree_destroy(orc_kdtree *t);

/* letkf_solve (module_letkf_core.f90:598-700).  yb(k,p) member fastest.
 * evals (nullable): eigenvalues of inflat*I + yb yb^T ascending. */
void orc_letkf_solve(int k, int p, const float *xb, const float *yo, const float *yb,
                     float inflat, int use_rtpp, float rtpp_alpha, int use_rtps,
                     float rtps_alpha, float *xa, double *evals);

/* Same contract as cwbl_search / cwbl_analyze_var (host memory only). */
int orc_search(int nobs, const float *obs_xyz, float hclr, float vclr, int max_lz_pts,
               int nq, const float *q_xyz, int *nfound, int *idx, float *r2);

int orc_analyze_var(int k, int weight_function, float norain_value, int q1_mode,
                    const cwbl_obs_set *obs, const cwbl_var_params *vp,
                    const cwbl_slab *slab, int nthreads, cwbl_stats *stats);

/* letkf_tune_q (module_letkf_core.f90:702-733) over var(nx,ny,nz,0:k-1), loops
 * i<ix_lim, j<iy_lim.  Reproduces Q3 (0/0 = NaN) exactly. */
void orc_tune_q(int k, int nx, int ny, int nz, int ix_lim, int iy_lim, float *var);

#ifdef __cplusplus
}
#endif
#endif
