/*
 * letkf_oracle.c — CPU restatement of the reference LETKF hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see letkf_oracle.h).  Compiled with -ffp-contract=off for
 * the x86-64 baseline (no FMA), which is how amdflang -O2 evaluates the reference's
 * fp32 stages; every fp32 expression below keeps the reference's operation order.
 *
 * Reference map (file:line in lopunch/CWBNWP-LETKF):
 *   orc_expf            glibc 2.35 sysdeps/ieee754/flt-32/e_expf.c as built with FMA
 *                       (the IFUNC variant flang's `exp` on real(4) calls on this CPU)
 *   orc_gaspari_cohn    module_localization.f90:333-364
 *   kd-tree             module_kdtree2.f90:598-979 (create), 1118-1179, 1381-1477,
 *                       1619-1712 (fixed-ball search)
 *   get_lz / build_tree module_localization.f90:35-167, 188-331
 *   yoyb                module_letkf_core.f90:300-595
 *   letkf_solve         module_letkf_core.f90:598-700 + module_eigen.f90:37-108
 *   driver loop         module_letkf_core.f90:59-70, 209-240
 *   tune_q              module_letkf_core.f90:702-733
 */
#define _GNU_SOURCE
#include "letkf_oracle.h"

#include <dlfcn.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------ */
/* expf: glibc 2.35 e_expf.c, FMA build (decoded from libm.so.6 __expf_fma).             */
/* ------------------------------------------------------------------------------------ */
static const uint64_t EXPF_T[32] = {
  0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
  0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
  0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
  0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
  0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
  0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
  0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
  0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

static double as_double(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t as_u64(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

float orc_expf(float x)
{
  const double shift = as_double(0x4338000000000000ull);   /* 0x1.8p52 */
  const double invln2n = as_double(0x40471547652b82feull); /* 32/ln2 */
  const double c0 = as_double(0x3ebc6af84b912394ull);
  const double c1 = as_double(0x3f2ebfce50fac4f3ull);
  const double c2 = as_double(0x3f962e42ff0c52d6ull);
  uint32_t ux; memcpy(&ux, &x, 4);
  uint32_t abstop = (ux >> 20) & 0x7ff;
  if (abstop >= 0x42b) {                       /* |x| >= 88: special cases */
    if (ux == 0xff800000u) return 0.0f;
    if (abstop >= 0x7f8) return x + x;
    return expf(x);                            /* over/underflow: not reached on the path */
  }
  double xd = (double)x;
  double kd = fma(invln2n, xd, shift);
  uint64_t ki = as_u64(kd);
  kd -= shift;
  double r = fma(invln2n, xd, -kd);
  uint64_t t = EXPF_T[ki % 32];
  t += ki << 47;
  double s = as_double(t);
  double z = fma(r, c0, c1);
  double r2 = r * r;
  double y = fma(r, c2, 1.0);
  y = fma(z, r2, y);
  y = y * s;
  return (float)y;
}

/* ------------------------------------------------------------------------------------ */
/* Gaspari & Cohn 1999, module_localization.f90:333-364 (fp32, unfused)                  */
/* ------------------------------------------------------------------------------------ */
float orc_gaspari_cohn(float x)
{
  const float a = sqrtf(10.0f / 3.0f);
  const float a1 = -0.25f, a2 = 0.5f, a3 = 0.625f, a4 = -5.0f / 3.0f, a5 = 1.0f;
  const float b1 = 1.0f / 12.0f, b2 = -0.5f, b3 = 0.625f, b4 = 5.0f / 3.0f, b5 = -5.0f,
              b6 = 4.0f, b7 = -2.0f / 3.0f;
  float z = x / a;
  if (z <= 1.0f) return z * z * (z * (z * (a1 * z + a2) + a3) + a4) + a5;
  if (z <= 2.0f) return z * (z * (z * (z * (b1 * z + b2) + b3) + b4) + b5) + b6 + b7 / z;
  return 0.0f;
}

float orc_search_r2(void)
{
  const float gc1999 = 2.0f * sqrtf(10.0f / 3.0f); /* module_param.f90:116 */
  return gc1999 * gc1999;                          /* module_localization.f90:202 */
}

/* ------------------------------------------------------------------------------------ */
/* kd-tree: Kennel's kdtree2 as configured by the reference (bucket 12, exact median,   */
/* rearranged data, unsorted fixed-ball results).                                      */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  int   cut_dim;                 /* 0-based; -1 terminal */
  float cut_val, cut_val_left, cut_val_right;
  int   l, u;                    /* 0-based inclusive range into ind */
  int   left, right;             /* node indices, -1 = null */
  float lo[3], hi[3];
} orc_node;

struct orc_kdtree {
  int       dim, n;
  float    *data;   /* the_data(3,n) */
  int      *ind;    /* permutation, 0-based */
  float    *rdata;  /* rearranged_data(dim,n) */
  orc_node *nodes;
  int       nnodes, cap, root;
};

#define ORC_BUCKET 12

static void orc_spread(const orc_kdtree *t, int c, int l, int u, float *lo, float *hi)
{
  float smin = t->data[3 * t->ind[l] + c], smax = smin;
  for (int i = l + 1; i <= u; ++i) {
    float v = t->data[3 * t->ind[i] + c];
    if (smin > v) smin = v;
    if (smax < v) smax = v;
  }
  *lo = smin; *hi = smax;
}

/* select_on_coordinate, module_kdtree2.f90:897-929 (0-based) */
static void orc_select(orc_kdtree *t, int c, int k, int li, int ui)
{
  int l = li, u = ui;
  int *ind = t->ind;
  while (l < u) {
    int tt = ind[l], m = l;
    for (int i = l + 1; i <= u; ++i) {
      if (t->data[3 * ind[i] + c] < t->data[3 * tt + c]) {
        ++m;
        int s = ind[m]; ind[m] = ind[i]; ind[i] = s;
      }
    }
    int s = ind[l]; ind[l] = ind[m]; ind[m] = s;
    if (m <= k) l = m + 1;
    if (m >= k) u = m - 1;
  }
}

static int orc_new_node(orc_kdtree *t)
{
  if (t->nnodes == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 64;
    t->nodes = (orc_node *)realloc(t->nodes, sizeof(orc_node) * (size_t)t->cap);
  }
  return t->nnodes++;
}

/* build_tree_for_range, module_kdtree2.f90:696-834 */
static int orc_build(orc_kdtree *t, int l, int u, int parent)
{
  if (u < l) return -1;
  int me = orc_new_node(t);
  orc_node *res = &t->nodes[me];
  res->left = res->right = -1;
  res->l = l; res->u = u;
  if (u - l <= ORC_BUCKET) {
    for (int i = 0; i < t->dim; ++i) orc_spread(t, i, l, u, &res->lo[i], &res->hi[i]);
    res->cut_dim = -1; res->cut_val = 0.0f;
    return me;
  }
  for (int i = 0; i < t->dim; ++i) {
    int recompute = 1;
    if (parent >= 0 && i != t->nodes[parent].cut_dim) recompute = 0;
    if (recompute) orc_spread(t, i, l, u, &t->nodes[me].lo[i], &t->nodes[me].hi[i]);
    else { t->nodes[me].lo[i] = t->nodes[parent].lo[i]; t->nodes[me].hi[i] = t->nodes[parent].hi[i]; }
  }
  int c = 0;
  float best = t->nodes[me].hi[0] - t->nodes[me].lo[0];
  for (int i = 1; i < t->dim; ++i) {
    float s = t->nodes[me].hi[i] - t->nodes[me].lo[i];
    if (s > best) { best = s; c = i; }
  }
  int m = (l + u) / 2;
  orc_select(t, c, m, l, u);
  t->nodes[me].cut_dim = c;
  int left = orc_build(t, l, m, me);
  int right = orc_build(t, m + 1, u, me);
  res = &t->nodes[me];
  res->left = left; res->right = right;
  const orc_node *L = &t->nodes[left], *R = &t->nodes[right];
  res->cut_val_right = R->lo[c];
  res->cut_val_left = L->hi[c];
  res->cut_val = (res->cut_val_left + res->cut_val_right) / 2.0f;
  for (int i = 0; i < t->dim; ++i) {
    res->hi[i] = L->hi[i] > R->hi[i] ? L->hi[i] : R->hi[i];
    res->lo[i] = L->lo[i] < R->lo[i] ? L->lo[i] : R->lo[i];
  }
  return me;
}

orc_kdtree *orc_kdtree_create(const float *xyz3, int n, int dim)
{
  orc_kdtree *t = (orc_kdtree *)calloc(1, sizeof(orc_kdtree));
  t->dim = dim; t->n = n;
  t->data = (float *)malloc(sizeof(float) * 3 * (size_t)(n > 0 ? n : 1));
  memcpy(t->data, xyz3, sizeof(float) * 3 * (size_t)n);
  t->ind = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  for (int j = 0; j < n; ++j) t->ind[j] = j;
  t->root = orc_build(t, 0, n - 1, -1);
  t->rdata = (float *)malloc(sizeof(float) * (size_t)dim * (size_t)(n > 0 ? n : 1));
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < dim; ++d) t->rdata[(size_t)dim * i + d] = t->data[3 * t->ind[i] + d];
  return t;
}

void orc_kdtree_destroy(orc_kdtree *t)
{
  if (!t) return;
  free(t->data); free(t->ind); free(t->rdata); free(t->nodes); free(t);
}

typedef struct {
  const orc_kdtree *t;
  const float *qv;
  float ballsize;
  int nfound, nalloc, overflow;
  int *idx; float *dis;
} orc_sr;

/* process_terminal_node_fixedball, module_kdtree2.f90:1619-1712 */
static void orc_terminal(orc_sr *sr, const orc_node *node)
{
  const int dimen = sr->t->dim;
  for (int i = node->l; i <= node->u; ++i) {
    float sd = 0.0f;
    int out = 0;
    for (int k = 0; k < dimen; ++k) {
      float d = sr->t->rdata[(size_t)dimen * i + k] - sr->qv[k];
      sd = sd + d * d;
      if (sd > sr->ballsize) { out = 1; break; }
    }
    if (out) continue;
    sr->nfound++;
    if (sr->nfound > sr->nalloc) {
      sr->overflow = 1;
      sr->nfound = sr->nalloc;
      break;
    }
    sr->dis[sr->nfound - 1] = sd;
    sr->idx[sr->nfound - 1] = sr->t->ind[i];
  }
}

static float orc_dis2_from_bnd(float x, float amin, float amax)
{
  if (x > amax) return (x - amax) * (x - amax);
  if (x < amin) return (amin - x) * (amin - x);
  return 0.0f;
}

/* search, module_kdtree2.f90:1381-1457 */
static void orc_search_node(orc_sr *sr, int ni)
{
  const orc_node *node = &sr->t->nodes[ni];
  if (node->left < 0 || node->right < 0) { orc_terminal(sr, node); return; }
  int cd = node->cut_dim;
  float qval = sr->qv[cd], dis;
  int closer, farther;
  if (qval < node->cut_val) {
    closer = node->left; farther = node->right;
    dis = (node->cut_val_right - qval) * (node->cut_val_right - qval);
  } else {
    closer = node->right; farther = node->left;
    dis = (node->cut_val_left - qval) * (node->cut_val_left - qval);
  }
  if (closer >= 0) orc_search_node(sr, closer);
  if (farther >= 0) {
    float ballsize = sr->ballsize;
    if (dis <= ballsize) {
      for (int i = 0; i < sr->t->dim; ++i) {
        if (i != cd) {
          dis = dis + orc_dis2_from_bnd(sr->qv[i], node->lo[i], node->hi[i]);
          if (dis > ballsize) return;
        }
      }
      orc_search_node(sr, farther);
    }
  }
}

int orc_kdtree_r_nearest(const orc_kdtree *t, const float *qv, float r2, int nalloc,
                         int *idx, float *dis, int *overflow)
{
  orc_sr sr = {t, qv, r2, 0, nalloc, 0, idx, dis};
  if (t->root >= 0) orc_search_node(&sr, t->root);
  if (overflow) *overflow = sr.overflow;
  return sr.nfound;
}

/* ------------------------------------------------------------------------------------ */
/* LAPACK / BLAS through dlopen (the reference links Fujitsu SSL2; the oracle uses MKL) */
/* ------------------------------------------------------------------------------------ */
typedef void (*dsyrk_t)(const char *, const char *, const int *, const int *, const double *,
                        const double *, const int *, const double *, double *, const int *);
typedef void (*dsyevd_t)(const char *, const char *, const int *, double *, const int *,
                         double *, double *, const int *, int *, const int *, int *);
typedef void (*dgemm_t)(const char *, const char *, const int *, const int *, const int *,
                        const double *, const double *, const int *, const double *,
                        const int *, const double *, double *, const int *);
typedef void (*dgemv_t)(const char *, const int *, const int *, const double *, const double *,
                        const int *, const double *, const int *, const double *, double *,
                        const int *);
typedef void (*dsymv_t)(const char *, const int *, const double *, const double *, const int *,
                        const double *, const int *, const double *, double *, const int *);
typedef void (*daxpy_t)(const int *, const double *, const double *, const int *, double *,
                        const int *);

static struct {
  int tried, ok;
  char name[64];
  dsyrk_t dsyrk; dsyevd_t dsyevd; dgemm_t dgemm; dgemv_t dgemv; dsymv_t dsymv; daxpy_t daxpy;
} LA;

int orc_lapack_init(void)
{
  if (LA.tried) return LA.ok;
#ifdef _OPENMP
#pragma omp critical(orc_lapack_init)
#endif
  {
    if (!LA.tried) {
      const char *env = getenv("CWBL_ORACLE_LAPACK");
      const char *cands[] = {env, "/opt/conda/lib/libmkl_rt.so", "libmkl_rt.so",
                             "libmkl_rt.so.1", NULL};
      strcpy(LA.name, "builtin-jacobi");
      if (!(env && strcmp(env, "builtin") == 0)) {
        setenv("MKL_THREADING_LAYER", "SEQUENTIAL", 0);
        setenv("MKL_CBWR", "COMPATIBLE", 0);
        setenv("MKL_NUM_THREADS", "1", 0);
        for (int i = 0; i < 4; ++i) {
          if (!cands[i]) continue;
          void *h = dlopen(cands[i], RTLD_NOW | RTLD_LOCAL);
          if (!h) continue;
          LA.dsyrk = (dsyrk_t)dlsym(h, "dsyrk_");
          LA.dsyevd = (dsyevd_t)dlsym(h, "dsyevd_");
          LA.dgemm = (dgemm_t)dlsym(h, "dgemm_");
          LA.dgemv = (dgemv_t)dlsym(h, "dgemv_");
          LA.dsymv = (dsymv_t)dlsym(h, "dsymv_");
          LA.daxpy = (daxpy_t)dlsym(h, "daxpy_");
          if (LA.dsyrk && LA.dsyevd && LA.dgemm && LA.dgemv && LA.dsymv && LA.daxpy) {
            LA.ok = 1;
            snprintf(LA.name, sizeof LA.name, "mkl");
            break;
          }
          dlclose(h);
        }
      }
      LA.tried = 1;
    }
  }
  return LA.ok;
}

const char *orc_lapack_name(void) { orc_lapack_init(); return LA.name; }

/* Builtin fallback: cyclic Jacobi (fp64), eigenvalues ascending, vectors in columns. */
static void orc_jacobi_eig(int n, double *a /* n*n col-major, full */, double *w, double *v)
{
  for (int i = 0; i < n * n; ++i) v[i] = 0.0;
  for (int i = 0; i < n; ++i) v[i * n + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    int rot = 0;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        double apq = a[q * n + p], app = a[p * n + p], aqq = a[q * n + q];
        if (apq == 0.0 || fabs(apq) <= 1e-300 ||
            fabs(apq) <= 2.2e-16 * sqrt(fabs(app * aqq))) continue;
        ++rot;
        double theta = (aqq - app) / (2.0 * apq);
        double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int r = 0; r < n; ++r) {
          double arp = a[p * n + r], arq = a[q * n + r];
          a[p * n + r] = c * arp - s * arq;
          a[q * n + r] = s * arp + c * arq;
        }
        for (int r = 0; r < n; ++r) {
          double apr = a[r * n + p], aqr = a[r * n + q];
          a[r * n + p] = c * apr - s * aqr;
          a[r * n + q] = s * apr + c * aqr;
        }
        for (int r = 0; r < n; ++r) {
          double vrp = v[p * n + r], vrq = v[q * n + r];
          v[p * n + r] = c * vrp - s * vrq;
          v[q * n + r] = s * vrp + c * vrq;
        }
      }
    if (!rot) break;
  }
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
  for (int i = 1; i < n; ++i) /* insertion sort ascending with vectors */
    for (int j = i; j > 0 && w[j - 1] > w[j]; --j) {
      double tw = w[j]; w[j] = w[j - 1]; w[j - 1] = tw;
      for (int r = 0; r < n; ++r) {
        double tv = v[j * n + r]; v[j * n + r] = v[(j - 1) * n + r]; v[(j - 1) * n + r] = tv;
      }
    }
}

/* letkf_solve, module_letkf_core.f90:598-700 (REAL64 build, Makefile:9) */
void orc_letkf_solve(int k, int p, const float *xb, const float *yo, const float *yb,
                     float inflat, int use_rtpp, float rtpp_alpha, int use_rtps,
                     float rtps_alpha, float *xa, double *evals)
{
  const int kk = k * k;
  const float nmember_inv = 1.0f / (float)k;         /* module_param.f90:245 */
  double *A = (double *)calloc((size_t)kk * 5 + (size_t)k * 4, sizeof(double));
  double *evect = A + kk, *tmp = evect + kk, *w = tmp + kk, *wbar2d = w + kk;
  double *eval = wbar2d + kk, *wbar = eval + k, *xbp = wbar + k;
  double *yb8 = (double *)malloc(sizeof(double) * (size_t)k * (size_t)(p > 0 ? p : 1));
  double *yo8 = (double *)malloc(sizeof(double) * (size_t)(p > 0 ? p : 1));
  const double one = 1.0, zero = 0.0;
  const int ione = 1;
  double inflat_r8 = (double)inflat;
  for (int i = 0; i < k; ++i) A[i * k + i] = 1.0;                      /* identity */
  for (size_t i = 0; i < (size_t)k * p; ++i) yb8[i] = (double)yb[i];
  for (int i = 0; i < p; ++i) yo8[i] = (double)yo[i];

  if (orc_lapack_init()) {
    LA.dsyrk("L", "N", &k, &p, &one, yb8, &k, &inflat_r8, A, &k);       /* :649 */
    /* inverse_matrix, module_eigen.f90:37-56 */
    memcpy(evect, A, sizeof(double) * kk);
    /* set_optimal_workspace_for_eigen (module_eigen.f90:16-35), once per thread and k */
    static __thread int ws_k = -1, lwork = 0, liwork = 0;
    static __thread double *work = NULL;
    static __thread int *iwork = NULL;
    int info = 0;
    if (ws_k != k) {
      int lq = -1, liq = -1, iwq = 0;
      double wq = 0;
      LA.dsyevd("V", "L", &k, evect, &k, eval, &wq, &lq, &iwq, &liq, &info);
      lwork = (int)wq; liwork = iwq;
      free(work); free(iwork);
      work = (double *)malloc(sizeof(double) * (size_t)(lwork > 1 ? lwork : 1));
      iwork = (int *)malloc(sizeof(int) * (size_t)(liwork > 1 ? liwork : 1));
      ws_k = k;
    }
    LA.dsyevd("V", "L", &k, evect, &k, eval, work, &lwork, iwork, &liwork, &info);
    if (evals) memcpy(evals, eval, sizeof(double) * k);
    for (int i = 0; i < k; ++i) {
      eval[i] = 1.0 / eval[i];
      for (int r = 0; r < k; ++r) tmp[i * k + r] = evect[i * k + r] * eval[i];
    }
    LA.dgemm("N", "T", &k, &k, &k, &one, tmp, &k, evect, &k, &zero, A, &k);  /* Pa */
    LA.dgemv("N", &k, &p, &one, yb8, &k, yo8, &ione, &zero, wbar, &ione);     /* :651 */
    LA.dsymv("L", &k, &one, A, &k, wbar, &ione, &zero, xbp, &ione);           /* :652 */
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < k; ++i) wbar2d[j * k + i] = xbp[i];                 /* :662 */
    /* sqrt_matrix, module_eigen.f90:78-93 */
    for (int i = 0; i < k; ++i)
      for (int r = 0; r < k; ++r) tmp[i * k + r] = evect[i * k + r] * sqrt(eval[i]);
    LA.dgemm("N", "T", &k, &k, &k, &one, tmp, &k, evect, &k, &zero, w, &k);
    double sk = sqrt((double)(k - 1));
    LA.daxpy(&kk, &sk, w, &ione, wbar2d, &ione);                              /* :666 */
  } else {
    for (int j = 0; j < k; ++j)
      for (int i = j; i < k; ++i) {
        double s = 0.0;
        for (int c = 0; c < p; ++c) s += yb8[(size_t)c * k + i] * yb8[(size_t)c * k + j];
        A[j * k + i] = s + inflat_r8 * A[j * k + i];
        A[i * k + j] = A[j * k + i];
      }
    double *acopy = tmp;
    memcpy(acopy, A, sizeof(double) * kk);
    orc_jacobi_eig(k, acopy, eval, evect);
    if (evals) memcpy(evals, eval, sizeof(double) * k);
    for (int i = 0; i < k; ++i) eval[i] = 1.0 / eval[i];
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < k; ++i) {
        double s = 0.0, s2 = 0.0;
        for (int c = 0; c < k; ++c) {
          s += evect[c * k + i] * eval[c] * evect[c * k + j];
          s2 += evect[c * k + i] * sqrt(eval[c]) * evect[c * k + j];
        }
        A[j * k + i] = s; w[j * k + i] = s2;
      }
    for (int i = 0; i < k; ++i) {
      double s = 0.0;
      for (int c = 0; c < p; ++c) s += yb8[(size_t)c * k + i] * yo8[c];
      wbar[i] = s;
    }
    for (int i = 0; i < k; ++i) {
      double s = 0.0;
      for (int j = 0; j < k; ++j) s += A[j * k + i] * wbar[j];
      xbp[i] = s;
    }
    double sk = sqrt((double)(k - 1));
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < k; ++i) wbar2d[j * k + i] = xbp[i] + sk * w[j * k + i];
  }

  /* :671-679 */
  float sxb = 0.0f;
  for (int i = 0; i < k; ++i) sxb = sxb + xb[i];
  double xb_mean = (double)(sxb * nmember_inv);
  for (int i = 0; i < k; ++i) { xbp[i] = (double)xb[i] - xb_mean; wbar[i] = xb_mean; }
  if (LA.ok) {
    LA.dgemv("T", &k, &k, &one, wbar2d, &k, xbp, &ione, &one, wbar, &ione);
  } else {
    for (int j = 0; j < k; ++j) {
      double s = 0.0;
      for (int i = 0; i < k; ++i) s += wbar2d[j * k + i] * xbp[i];
      wbar[j] = s + wbar[j];
    }
  }
  for (int i = 0; i < k; ++i) xa[i] = (float)wbar[i];

  /* RTPP / RTPS, :684-698 */
  if (use_rtpp || use_rtps) {
    float sxa = 0.0f;
    for (int i = 0; i < k; ++i) sxa = sxa + xa[i];
    float xa_mean = sxa * nmember_inv;
    float *xap = (float *)tmp; /* reuse */
    for (int i = 0; i < k; ++i) xap[i] = xa[i] - xa_mean;
    if (use_rtpp)
      for (int i = 0; i < k; ++i)
        xap[i] = (float)((double)((1.0f - rtpp_alpha) * xap[i]) + (double)rtpp_alpha * xbp[i]);
    if (use_rtps) {
      double d8 = 0.0;
      for (int i = 0; i < k; ++i) d8 = d8 + xbp[i] * xbp[i];
      float xb_std = (float)d8;
      float xa_std = 0.0f;
      for (int i = 0; i < k; ++i) xa_std = xa_std + xap[i] * xap[i];
      float fac = rtps_alpha * sqrtf(xb_std / xa_std) - rtps_alpha + 1.0f;
      for (int i = 0; i < k; ++i) xap[i] = xap[i] * fac;
    }
    for (int i = 0; i < k; ++i) xa[i] = xa_mean + xap[i];
  }
  free(yb8); free(yo8); free(A);
}

/* ------------------------------------------------------------------------------------ */
/* Localization set-up per variable (build_tree) and per point (get_lz)                   */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  int family;          /* 0 gts, 1 radar */
  int type_id;
  int entry;           /* index into obs->gts / obs->radar */
  float hclr_inv, vclr_inv;
  int tree_dim;        /* dimension of the built tree */
  int own3d;           /* this type's own query is 3-D */
  int q1_undef;        /* Q1 undefined case handled per type */
  int max_lz;
  orc_kdtree *tree;
} orc_tree_t;

static int orc_is_gts_assimilated(int id)
{
  return id == CWBL_GTS_SYNOP || id == CWBL_GTS_METAR || id == CWBL_GTS_SHIPS ||
         id == CWBL_GTS_SOUND || id == CWBL_GTS_GPSPW;
}

/* build_tree, module_localization.f90:35-167, for one family */
static int orc_build_family(int family, const cwbl_obs_set *obs, const cwbl_var_params *vp,
                            int q1_mode, orc_tree_t *out)
{
  int ntype = 0;
  int ntypes_total = family == 0 ? CWBL_NUM_GTS_TYPES : CWBL_NUM_RADAR_TYPES;
  for (int id = 1; id <= ntypes_total; ++id) {
    int entry = -1, nobs = 0;
    if (family == 0) {
      for (int e = 0; e < obs->n_gts; ++e)
        if (obs->gts[e].type_id == id) { entry = e; nobs = obs->gts[e].nobs; }
      if (entry < 0 || nobs <= 0 || !orc_is_gts_assimilated(id)) continue;
    } else {
      for (int e = 0; e < obs->n_radar; ++e)
        if (obs->radar[e].type_id == id) { entry = e; nobs = obs->radar[e].nobs; }
      if (entry < 0 || nobs <= 0) continue;
    }
    const cwbl_type_params *tp = family == 0 ? &vp->gts[id - 1] : &vp->radar[id - 1];
    if (!(tp->use_it && tp->hclr > 0.0f)) continue;
    orc_tree_t *T = &out[ntype++];
    memset(T, 0, sizeof *T);
    T->family = family; T->type_id = id; T->entry = entry; T->max_lz = tp->max_lz_pts;
    T->hclr_inv = 1.0f / (tp->hclr * 1e3f);
    T->vclr_inv = tp->vclr > 0.0f ? 1.0f / (tp->vclr * 1e3f) : -1.0f;
    T->own3d = T->vclr_inv > 0.0f;
  }
  if (ntype == 0) return 0;
  /* Q1: the dimension test at :151 reads the loop variable left by the last append */
  int fam3d = out[ntype - 1].vclr_inv > 0.0f;
  for (int i = 0; i < ntype; ++i) {
    orc_tree_t *T = &out[i];
    int dim3 = q1_mode == CWBL_Q1_PER_TYPE ? T->own3d : fam3d;
    if (dim3 && !T->own3d) { dim3 = 0; T->q1_undef = 1; }
    T->tree_dim = dim3 ? 3 : 2;
    int n; const float *xyz;
    if (family == 0) { n = obs->gts[T->entry].nobs; xyz = obs->gts[T->entry].xyz; }
    else { n = obs->radar[T->entry].nobs; xyz = obs->radar[T->entry].xyz; }
    float *nx = (float *)malloc(sizeof(float) * 3 * (size_t)n);
    for (int j = 0; j < n; ++j) {
      nx[3 * j + 0] = xyz[3 * j + 0] * T->hclr_inv;
      nx[3 * j + 1] = xyz[3 * j + 1] * T->hclr_inv;
      nx[3 * j + 2] = dim3 ? xyz[3 * j + 2] * T->vclr_inv : -1.0f;
    }
    T->tree = orc_kdtree_create(nx, n, T->tree_dim);
    free(nx);
  }
  return ntype;
}

int orc_search(int nobs, const float *obs_xyz, float hclr, float vclr, int max_lz_pts,
               int nq, const float *q_xyz, int *nfound, int *idx, float *r2)
{
  float hinv = 1.0f / (hclr * 1e3f);
  float vinv = vclr > 0.0f ? 1.0f / (vclr * 1e3f) : -1.0f;
  int dim = vinv > 0.0f ? 3 : 2;
  float *nx = (float *)malloc(sizeof(float) * 3 * (size_t)(nobs > 0 ? nobs : 1));
  for (int j = 0; j < nobs; ++j) {
    nx[3 * j + 0] = obs_xyz[3 * j + 0] * hinv;
    nx[3 * j + 1] = obs_xyz[3 * j + 1] * hinv;
    nx[3 * j + 2] = dim == 3 ? obs_xyz[3 * j + 2] * vinv : -1.0f;
  }
  orc_kdtree *t = orc_kdtree_create(nx, nobs, dim);
  free(nx);
  const float rr = orc_search_r2();
  for (int q = 0; q < nq; ++q) {
    float qv[3] = {q_xyz[3 * q] * hinv, q_xyz[3 * q + 1] * hinv,
                   dim == 3 ? q_xyz[3 * q + 2] * vinv : 0.0f};
    nfound[q] = orc_kdtree_r_nearest(t, qv, rr, max_lz_pts, idx + (size_t)q * max_lz_pts,
                                     r2 + (size_t)q * max_lz_pts, NULL);
  }
  orc_kdtree_destroy(t);
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* letkf_yoyb for one point, module_letkf_core.f90:300-595                              */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  int cap, total;
  float *yo, *yb;      /* yb(k,cap) */
} orc_cols;

static void orc_cols_push(orc_cols *c, int k, float yo, const float *yb)
{
  if (c->total == c->cap) {
    c->cap = c->cap ? 2 * c->cap : 256;
    c->yo = (float *)realloc(c->yo, sizeof(float) * (size_t)c->cap);
    c->yb = (float *)realloc(c->yb, sizeof(float) * (size_t)c->cap * k);
  }
  c->yo[c->total] = yo;
  memcpy(c->yb + (size_t)c->total * k, yb, sizeof(float) * k);
  c->total++;
}

static float orc_error_inv(int wf, float err, float r2)
{
  if (wf != 1) return 1.0f / (err * orc_expf(0.25f * r2));     /* :444 */
  return sqrtf(orc_gaspari_cohn(sqrtf(r2))) / err;             /* :449 */
}

static void orc_yoyb_one(int k, int wf, float norain, const cwbl_obs_set *obs,
                         const cwbl_var_params *vp, const orc_tree_t *T, int nlz,
                         const int *idxs, const float *r2s, orc_cols *cols, float *bg)
{
  const float ninv = 1.0f / (float)k, n1inv = 1.0f / (float)(k - 1);
  if (T->family == 0) {
    const cwbl_gts_obs *g = &obs->gts[T->entry];
    const cwbl_type_params *tp = &vp->gts[T->type_id - 1];
    const int nvar = g->nvar;
    int is_assim[CWBL_MAX_NVAR];
    for (int v = 0; v < nvar; ++v) is_assim[v] = tp->hclr > 0.0f ? tp->is_assim[v] : 0;
    for (int j = 0; j < nlz; ++j) {
      const int idx = idxs[j];
      const float r2 = r2s[j];
      for (int v = 0; v < nvar; ++v) {
        if (!is_assim[v]) continue;
        int anyqc = 0;
        for (int m = 0; m < k; ++m)
          if (g->qc[((size_t)m * g->nobs + idx) * nvar + v] >= 0) { anyqc = 1; break; }
        if (!anyqc) continue;
        float s = 0.0f;
        for (int m = 0; m < k; ++m) {
          bg[m] = g->hdxb[((size_t)m * g->nobs + idx) * nvar + v];
          s = s + bg[m];
        }
        float mean = s * ninv;
        float d = 0.0f;
        for (int m = 0; m < k; ++m) bg[m] = bg[m] - mean;
        for (int m = 0; m < k; ++m) d = d + bg[m] * bg[m];
        float omm = g->obs[(size_t)idx * nvar + v] - mean;
        float std = sqrtf(d * n1inv);
        float err = g->error[(size_t)idx * nvar + v] * tp->err_muti[v];
        if (fabsf(omm) > sqrtf(std * std + err * err) * tp->err_rej[v]) continue;
        float einv = orc_error_inv(wf, err, r2);
        omm = omm * einv;
        for (int m = 0; m < k; ++m) bg[m] = bg[m] * einv;
        orc_cols_push(cols, k, omm, bg);
      }
    }
  } else {
    const cwbl_radar_obs *R = &obs->radar[T->entry];
    const cwbl_type_params *tp = &vp->radar[T->type_id - 1];
    if (!(tp->hclr > 0.0f)) return;                                 /* :487,491 */
    const float err_muti = tp->err_muti[0], err_rej = tp->err_rej[0];
    for (int j = 0; j < nlz; ++j) {
      const int idx = idxs[j];
      const float r2 = r2s[j];
      float s = 0.0f;
      for (int m = 0; m < k; ++m) {
        bg[m] = R->hdxb[(size_t)m * R->nobs + idx];
        s = s + bg[m];
      }
      float mean = s * ninv;
      float d = 0.0f;
      for (int m = 0; m < k; ++m) bg[m] = bg[m] - mean;
      for (int m = 0; m < k; ++m) d = d + bg[m] * bg[m];
      float o = R->obs[idx];
      float omm = o - mean;
      float std = sqrtf(d * n1inv);
      float err = err_muti;
      int gross = fabsf(omm) > sqrtf(std * std + err * err) * err_rej;
      if (T->type_id == CWBL_RADAR_DBZ) {
        if (gross && o != norain) continue;                         /* :505-506 */
        if (o == norain && mean == norain) continue;                /* :507 */
      } else if (gross) continue;                                   /* :509 */
      float einv = orc_error_inv(wf, err, r2);
      omm = omm * einv;
      for (int m = 0; m < k; ++m) bg[m] = bg[m] * einv;
      orc_cols_push(cols, k, omm, bg);
    }
  }
}

/* ------------------------------------------------------------------------------------ */
/* One variable: module_letkf_core.f90:59-70 + 209-240                                  */
/* ------------------------------------------------------------------------------------ */
int orc_analyze_var(int k, int wf, float norain, int q1_mode, const cwbl_obs_set *obs,
                    const cwbl_var_params *vp, const cwbl_slab *slab, int nthreads,
                    cwbl_stats *stats)
{
  orc_tree_t trees[CWBL_NUM_GTS_TYPES + CWBL_NUM_RADAR_TYPES];
  int ng = orc_build_family(0, obs, vp, q1_mode, trees);
  int nr = orc_build_family(1, obs, vp, q1_mode, trees + ng);
  int nt = ng + nr;
  cwbl_stats st;
  memset(&st, 0, sizeof st);
  st.ntrees = nt;
  if (nt == 0) { if (stats) *stats = st; return 0; }                /* :66 */
  const float inflat = (float)(k - 1) / vp->multi_infl;             /* :68 */
  const float rr = orc_search_r2();
  const int nx = slab->nx, ny = slab->ny, nz = slab->nz;
  const size_t L = (size_t)nx * ny * nz;
  const long long npts = (long long)slab->ix_lim * slab->iy_lim * nz;
  int maxlz = 0;
  for (int t = 0; t < nt; ++t) maxlz += trees[t].max_lz;
  long long solved = 0, nobs_sum = 0, trunc = 0, q1u = 0;
  int max_p = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : solved, nobs_sum, trunc, q1u) reduction(max : max_p)
#endif
  {
    int *idx = (int *)malloc(sizeof(int) * (size_t)(maxlz + 1));
    float *r2 = (float *)malloc(sizeof(float) * (size_t)(maxlz + 1));
    int nlz[CWBL_NUM_GTS_TYPES + CWBL_NUM_RADAR_TYPES];
    float *bg = (float *)malloc(sizeof(float) * (size_t)k);
    float xb[256], xa[256];
    orc_cols cols = {0, 0, NULL, NULL};
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
    for (long long pt = 0; pt < npts; ++pt) {
      /* Fortran loop order j, i, k (:209-213); points are independent */
      const int kz = (int)(pt % nz);
      const int i = (int)((pt / nz) % slab->ix_lim);
      const int j = (int)(pt / ((long long)nz * slab->ix_lim));
      const float px = slab->x[(size_t)i + (size_t)nx * j];
      const float py = slab->y[(size_t)i + (size_t)nx * j];
      const float pz = slab->alt[(size_t)i + (size_t)slab->alt_nx * ((size_t)j + (size_t)slab->alt_ny * kz)];
      int off = 0, any = 0;
      for (int t = 0; t < nt; ++t) {
        const orc_tree_t *T = &trees[t];
        float qv[3] = {px * T->hclr_inv, py * T->hclr_inv, T->own3d ? pz * T->vclr_inv : 0.0f};
        int ovf = 0;
        nlz[t] = orc_kdtree_r_nearest(T->tree, qv, rr, T->max_lz, idx + off, r2 + off, &ovf);
        trunc += ovf;
        if (T->q1_undef) q1u++;
        if (nlz[t] > 0) any = 1;
        off += nlz[t];
      }
      if (!any) continue;                                           /* :220 */
      cols.total = 0;
      off = 0;
      for (int t = 0; t < nt; ++t) {
        orc_yoyb_one(k, wf, norain, obs, vp, &trees[t], nlz[t], idx + off, r2 + off, &cols, bg);
        off += nlz[t];
      }
      if (cols.total == 0) continue;                                /* :226 */
      const size_t P = (size_t)i + (size_t)nx * ((size_t)j + (size_t)ny * kz);
      for (int m = 0; m < k; ++m) xb[m] = slab->var[P + L * m];
      orc_letkf_solve(k, cols.total, xb, cols.yo, cols.yb, inflat, vp->use_rtpp,
                      vp->rtpp_alpha, vp->use_rtps, vp->rtps_alpha, xa, NULL);
      for (int m = 0; m < k; ++m) slab->var[P + L * m] = xa[m];
      solved++;
      nobs_sum += cols.total;
      if (cols.total > max_p) max_p = cols.total;
    }
    free(idx); free(r2); free(bg); free(cols.yo); free(cols.yb);
  }
  for (int t = 0; t < nt; ++t) orc_kdtree_destroy(trees[t].tree);
  st.points = npts; st.solved = solved; st.nobs_sum = nobs_sum; st.lz_truncated = trunc;
  st.q1_undefined = q1u; st.max_p = max_p;
  if (stats) *stats = st;
  return 0;
}

/* letkf_tune_q, module_letkf_core.f90:702-733 */
void orc_tune_q(int k, int nx, int ny, int nz, int ix_lim, int iy_lim, float *var)
{
  const size_t L = (size_t)nx * ny * nz;
  for (int kz = 0; kz < nz; ++kz)
    for (int j = 0; j < iy_lim; ++j)
      for (int i = 0; i < ix_lim; ++i) {
        const size_t P = (size_t)i + (size_t)nx * ((size_t)j + (size_t)ny * kz);
        float s = 0.0f, sp = 0.0f;
        for (int m = 0; m < k; ++m) s = s + var[P + L * m];
        for (int m = 0; m < k; ++m) if (var[P + L * m] > 0.0f) sp = sp + var[P + L * m];
        float ratio = s / sp;
        for (int m = 0; m < k; ++m) {
          float v = var[P + L * m];
          var[P + L * m] = v < 0.0f ? 0.0f : ratio * v;
        }
      }
}
