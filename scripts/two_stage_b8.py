"""Design prototype (numpy; not product code) of the k = 128 two-stage reduction exactly as
the band kernels compute it (cwbl_band.hip): stage 1 reduces A = inflat I + Yb Yb^T to a band
of half-bandwidth b = 8 with 15 panel block reflectors (dgeqr2 + dlarft per panel, the
two-sided trailing update as GEMMs), stage 2 chases the band to tridiagonal form with 8-row
Householder reflectors, two sweeps in flight (lag 3 tasks) as one wavefront runs them.

Checks against numpy's eigh: T's spectrum, Q T Q^T = A, and the LETKF quantities the kernels
form (u1^T T^-1 u2 = b1^T A^-1 x', Q T^-1/2 Q^T x' = A^-1/2 x'), with Q^T applied to b1, x'
and Q applied to y in the kernels' orders (panels; then sweep by sweep, the reflectors of one
sweep at once).

Usage: python scripts/two_stage_b8.py [k] [p]
"""
import sys

import numpy as np

N, B = 128, 8


def house(x):
    """dlarfg: v (v_0 = 1), tau, beta with (I - tau v v^T) x = beta e_0."""
    alpha = x[0]
    xn2 = float(x[1:] @ x[1:])
    v = np.zeros_like(x)
    v[0] = 1.0
    if xn2 == 0.0:
        return v, 0.0, alpha
    beta = -np.copysign(np.sqrt(alpha * alpha + xn2), alpha)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def stage1(A, u1, u2):
    """15 panels of 8 columns: panel p = columns [8p, 8p+8), rows [r0, N), r0 = 8p + 8."""
    A = A.copy()
    panels = []
    for p in range(N // B - 1):
        c0, r0 = B * p, B * p + B
        P = A[r0:, c0:c0 + B].copy()
        m = P.shape[0]
        V = np.zeros((m, B))
        tau = np.zeros(B)
        for i in range(min(B, m - 1) if m > 1 else 0):  # dgeqr2 (a 1-row tail needs none)
            v, t, beta = house(P[i:, i])
            V[i:, i] = v
            tau[i] = t
            P[i:, i:] -= t * np.outer(v, v @ P[i:, i:])
        T = np.zeros((B, B))  # dlarft, forward columnwise: Q = I - V T V^T
        for i in range(B):
            T[i, i] = tau[i]
            if i:
                T[:i, i] = -tau[i] * (T[:i, :i] @ (V[:, :i].T @ V[:, i]))
        P = np.triu(P)  # R; the kernel stores exact zeros below it
        A[r0:, c0:c0 + B] = P
        A[c0:c0 + B, r0:] = P.T
        A22 = A[r0:, r0:]
        W = A22 @ V @ T                       # the kernel: W = (A22 V) T
        Z = W - 0.5 * V @ (T.T @ (V.T @ W))
        A[r0:, r0:] = A22 - V @ Z.T - Z @ V.T
        for u in (u1, u2):                    # u <- Q_p^T u = u - V T^T V^T u
            u[r0:] -= V @ (T.T @ (V.T @ u[r0:]))
        panels.append((r0, V, T))
    return A, panels


def n_tasks(j):
    return (N - 3 - j) // B + 1 if j <= N - 3 else 0


def schedule():
    """Rounds of the chase: two slots (even sweeps, odd sweeps); sweep j + 1 runs its task t
    in the round of sweep j's task t + 3 or later, sweep j + 2 starts when sweep j is done."""
    start = {}
    for j in range(N - 2):
        s = 0
        if j >= 1:
            s = max(s, start[j - 1] + 3)
        if j >= 2:
            s = max(s, start[j - 2] + n_tasks(j - 2))
        start[j] = s
    nr = max(start[j] + n_tasks(j) for j in start)
    rounds = [[] for _ in range(nr)]
    for j, s in start.items():
        for t in range(n_tasks(j)):
            rounds[s + t].append((j, t))
    assert all(len(r) <= 2 for r in rounds)
    return rounds, start


def stage2(Bm, rounds):
    """The chase on the full symmetric matrix (the kernel keeps the lower band + bulge in LDS:
    row i holds A(i, i - d), d = 0..15).  Task (j, t): r = j + 1 + 8t, column c = j (t = 0) or
    r - 8; reflector on rows [r, min(r + 8, N)) from column c; blocks left (rows [r, r+8) x
    columns (c, r)), diag [r, r+8)^2 two-sided, below (rows [r+8, r+16) x columns [r, r+8))."""
    A = Bm.copy()
    refl = {}
    for rnd in rounds:
        for (j, t) in rnd:
            r = j + 1 + B * t
            c = j if t == 0 else r - B
            hi = min(r + B, N)
            v, tau, beta = house(A[r:hi, c].copy())
            A[r:hi, c] = 0.0
            A[r, c] = beta
            A[c, r:hi] = A[r:hi, c]
            # left block (columns c+1 .. r-1), diag, below: H A H on the window
            lo, top = c + 1, min(hi + B, N)
            A[r:hi, lo:top] -= tau * np.outer(v, v @ A[r:hi, lo:top])
            A[lo:top, r:hi] -= tau * np.outer(A[lo:top, r:hi] @ v, v)
            refl[(j, t)] = (r, v, tau)
            # the kernel's storage bound: nothing below d = 15
            assert np.all(A[np.tril_indices(N, -16)] == 0.0), (j, t)
    return A, refl


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 216
    rng = np.random.default_rng(1)
    Y = rng.standard_normal((k, p)) * np.exp(rng.uniform(-3, 3, p))
    A = np.eye(N)
    A[:k, :k] = (k - 1) / 1.1 * np.eye(k) + Y @ Y.T   # identity padding past k
    b1 = np.zeros(N)
    xp = np.zeros(N)
    b1[:k] = rng.standard_normal(k)
    xp[:k] = rng.standard_normal(k)
    u1, u2 = b1.copy(), xp.copy()
    Bm, panels = stage1(A, u1, u2)
    band_err = np.max(np.abs(np.tril(Bm, -B - 1))) / np.max(np.abs(A))
    rounds, start = schedule()
    Tm, refl = stage2(Bm, rounds)
    d, e = np.diag(Tm).copy(), np.diag(Tm, -1).copy()
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    tri_err = np.max(np.abs(Tm - T)) / np.max(np.abs(A))
    bulge = max(np.max(np.abs(np.tril(Bm, -16))), 0.0)
    # Q2^T u: sweep by sweep (a sweep's reflectors act on disjoint rows), forward
    sweeps = sorted({j for (j, _) in refl})
    for j in sweeps:
        for t in range(n_tasks(j)):
            r, v, tau = refl[(j, t)]
            for u in (u1, u2):
                u[r:r + len(v)] -= tau * v * (v @ u[r:r + len(v)])
    w, U = np.linalg.eigh(T)
    z = U @ ((U.T @ u2) / w)
    y = U @ ((U.T @ u2) / np.sqrt(w))
    dd = u1 @ z
    # y <- Q2 y (sweeps in reverse), then Q1 y (panels in reverse)
    for j in reversed(sweeps):
        for t in range(n_tasks(j)):
            r, v, tau = refl[(j, t)]
            y[r:r + len(v)] -= tau * v * (v @ y[r:r + len(v)])
    for r0, V, Tp in reversed(panels):
        y[r0:] -= V @ (Tp @ (V.T @ y[r0:]))
    wa, Ua = np.linalg.eigh(A)
    y_ref = Ua @ ((Ua.T @ xp) / np.sqrt(wa))
    d_ref = b1 @ (Ua @ ((Ua.T @ xp) / wa))
    lam = np.linalg.eigvalsh(T)
    print(f"k={k} p={p}: band {band_err:.1e}, tridiagonal {tri_err:.1e}, tasks {len(refl)}, "
          f"rounds {len(rounds)} (of {sum(n_tasks(j) for j in range(N - 2))} tasks)")
    print(f"  eigenvalues rel {np.max(np.abs(lam - wa) / wa):.1e}; "
          f"A^-1/2 x' rel {np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref):.1e}; "
          f"b1 A^-1 x' rel {abs(dd - d_ref) / abs(d_ref):.1e}")


if __name__ == "__main__":
    main()
