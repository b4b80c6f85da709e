// quad_tables.cpp — node/weight tables of the inverse-square-root quadrature used by
// solve_tq_kernel (cwbl_tq.hip).
//
//   x^-1/2 = (2/pi) int_0^inf dt / (t^2 + x),   x in [1, kappa]
// With t = sc(u | k^2), k^2 = 1 - 1/kappa, u in (0, K), the integrand is analytic in a strip
// whose width grows like 1/log(kappa), and the N-point midpoint rule in u converges
// geometrically (Hale, Higham & Trefethen, SIAM J. Numer. Anal. 46 (2008), method for
// A^-1/2 on a real positive spectrum):
//   x^-1/2 ~= sum_j w_j / (t2_j + x),  t2_j = sc^2(u_j),  w_j = (2/pi)(K/N) dn(u_j)/cn^2(u_j)
// Level L covers kappa = 10^L, L = 1..kQuadLevels (24).  The one-wavefront kernels use N = 31
// nodes up to level kQuadLevels31 (12) and N = 63 (two passes) above; solve_tq40_kernel runs
// 8 R - 1 nodes in R rounds (quad_rounds: N = 15 up to level 2, 23 at level 3, 31 to level
// 12, 63 above), each as accurate as the longer rule there (tests/test_quadrature.py).  The
// 31-node rule loses accuracy as log(kappa) grows (~1e-9 at 10^12); 63 nodes keep it below
// ~1e-9 up to 10^24.  Elliptic functions are evaluated in long double by the AGM / descending
// Landen scheme (Abramowitz & Stegun 16.4) from the complementary modulus k' = kappa^-1/2
// itself (1 - m is not representable once kappa passes ~1e19); nodes past K/2 use the
// reflection u -> K - u (sc(K-v) = 1/(k' sc(v)), dn/cn^2 (K-v) = dn(v)/(k' sn^2(v))) so that
// no quantity is formed from a cancelling cn.
#include "cwbl_internal.h"

#include <cmath>

namespace cwbl {
namespace {

constexpr long double kPi = 3.141592653589793238462643383279502884L;

struct Jac {
  long double sn, cn, dn;
};

// Jacobi elliptic functions of parameter m = k^2 = 1 - kc^2 (0 <= m < 1), A&S 16.4.
Jac ellipj(long double u, long double kc) {
  long double a[64], c[64];
  long double b = kc;
  a[0] = 1.0L;
  c[0] = sqrtl((1.0L - kc) * (1.0L + kc));
  int n = 0;
  while (fabsl(c[n]) > 1e-21L && n < 62) {
    a[n + 1] = 0.5L * (a[n] + b);
    c[n + 1] = 0.5L * (a[n] - b);
    b = sqrtl(a[n] * b);
    ++n;
  }
  long double phi = ldexpl(a[n] * u, n), phi1 = phi;
  for (int i = n; i > 0; --i) {
    phi1 = phi;
    phi = 0.5L * (phi + asinl(c[i] * sinl(phi) / a[i]));
  }
  Jac j;
  j.sn = sinl(phi);
  j.cn = cosl(phi);
  j.dn = n > 0 ? j.cn / cosl(phi1 - phi) : 1.0L;
  return j;
}

long double ellipk(long double kc) {  // K(m), m = 1 - kc^2
  long double a = 1.0L, b = kc;
  for (int i = 0; i < 64 && fabsl(a - b) > 1e-21L * a; ++i) {
    const long double an = 0.5L * (a + b);
    b = sqrtl(a * b);
    a = an;
  }
  return kPi / (2.0L * a);
}

}  // namespace

void quad_table(int level, double2 *out, int N) {
  const long double kappa = powl(10.0L, (long double)level);
  const long double kc = sqrtl(1.0L / kappa);  // k' (m = 1 - 1/kappa)
  const long double K = ellipk(kc);
  for (int j = 0; j < kQuadStride; ++j) {
    if (j >= N) {
      out[j] = make_double2(0.0, 0.0);
      continue;
    }
    const long double u = ((long double)j + 0.5L) * K / N;
    long double t2, wt;
    if (2.0L * u <= K) {
      const Jac e = ellipj(u, kc);
      const long double sc = e.sn / e.cn;
      t2 = sc * sc;
      wt = e.dn / (e.cn * e.cn);
    } else {
      const Jac e = ellipj(K - u, kc);
      const long double sc = e.cn / (kc * e.sn);
      t2 = sc * sc;
      wt = e.dn / (kc * e.sn * e.sn);
    }
    out[j] = make_double2((double)t2, (double)(2.0L / kPi * (K / N) * wt));
  }
}

}  // namespace cwbl

// Test hooks (not part of the public header): the table of one level, kQuadStride (t2, w)
// pairs, for the kQuadNodes-node rule and for an n-node rule (n <= 63; the rules of
// solve_tq40_kernel's rounds and the two-pass rule above level kQuadLevels31).
extern "C" int cwbl_debug_quad_table_n(int level, int n, double *t2w) {
  if (level < 1 || level > cwbl::kQuadLevels || n < 1 || n > 2 * cwbl::kQuadNodes + 1 || !t2w)
    return 1;
  cwbl::quad_table(level, reinterpret_cast<double2 *>(t2w), n);
  return 0;
}
extern "C" int cwbl_debug_quad_table(int level, double *t2w) {
  return cwbl_debug_quad_table_n(level, cwbl::kQuadNodes, t2w);
}
