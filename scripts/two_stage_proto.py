"""Design prototype (numpy, not product code): a two-stage reduction of the k = 128 LETKF matrix
A = (k-1)/rho I + Yb Yb^T to tridiagonal form, the route DESIGN.md §8 item 1 names for C4.

Stage 1 (full -> band of half-bandwidth b, the GEMM-rich part): for each panel of b columns,
QR of the rows below the band (dgeqr2 + dlarft: Q_p = I - V T V^T), then the two-sided
trailing update A22 <- Q_p^T A22 Q_p = A22 - V Z^T - Z V^T with W = A22 V T and
Z = W - 1/2 V (T^T V^T W) -- on the GPU, A22 V and the rank-2b update are MFMA GEMMs.
Stage 2 (band -> tridiagonal, bulge chasing, the sequential part): for each column j, one
Householder of length <= b annihilates rows j+2 .. j+b of the band column, and the bulge it
creates b rows further down is chased off the end, one length-<= b reflector per block.

The script checks, against numpy's eigh on the same matrix, that T's spectrum equals A's,
that Q T Q^T = A, and that the LETKF quantities the kernels form from T and Q
(wbar = A^-1 b1, W x' = sqrt(k-1) A^-1/2 x') agree; and it counts the sequential steps
and flops of each stage (the latency chain the GPU kernels would carry).

Usage: python scripts/two_stage_proto.py [k] [p] [b]
"""
import sys

import numpy as np


def house(x):
    """v, tau, beta with (I - tau v v^T) x = beta e_0, v_0 = 1 (LAPACK dlarfg convention)."""
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


def stage1_band(A, b):
    """Full symmetric A -> band (half-bandwidth b); returns the band matrix and the panels'
    (row offset, V, T) so that A = Q1 B Q1^T with Q1 = prod_p (I - V_p T_p V_p^T)."""
    n = A.shape[0]
    A = A.copy()
    panels = []
    steps = 0
    for p0 in range(0, n - b - 1, b):
        r0 = p0 + b  # first row below the band
        nb = min(b, n - r0)
        P = A[r0:, p0:p0 + nb].copy()  # the panel below the band
        m = P.shape[0]
        V = np.zeros((m, nb))
        taus = np.zeros(nb)
        for i in range(min(nb, m)):  # dgeqr2
            v, tau, beta = house(P[i:, i])
            steps += 1
            V[i:, i] = v
            taus[i] = tau
            P[i:, i:] -= tau * np.outer(v, v @ P[i:, i:])
        T = np.zeros((nb, nb))  # dlarft (forward, columnwise)
        for i in range(nb):
            T[i, i] = taus[i]
            if i:
                T[:i, i] = -taus[i] * T[:i, :i] @ (V[:, :i].T @ V[:, i])
        # the panel becomes R (upper triangular) in the band; zeros below
        A[r0:, p0:p0 + nb] = P
        A[p0:p0 + nb, r0:] = P.T
        # two-sided trailing update (GEMMs)
        A22 = A[r0:, r0:]
        W = A22 @ V @ T
        Z = W - 0.5 * V @ (T.T @ (V.T @ W))
        A[r0:, r0:] = A22 - V @ Z.T - Z @ V.T
        panels.append((r0, V, T))
    return A, panels, steps


def stage2_chase(B, b):
    """Band (half-bandwidth b) -> tridiagonal by bulge chasing (dsbtrd-like, unblocked).
    Returns d, e, the reflectors (row offset, v, tau) in application order, the step count."""
    n = B.shape[0]
    B = B.copy()
    refl = []
    for j in range(n - 2):
        # annihilate column j below the subdiagonal, then chase the bulge down
        c, r = j, j + 1
        while r < n - 1:
            hi = min(r + b, n)
            x = B[r:hi, c]
            if hi - r < 2:
                break
            v, tau, beta = house(x)
            if tau != 0.0:
                # two-sided application on the window the reflector touches
                lo = max(0, r - b)
                top = min(n, hi + b)
                B[r:hi, lo:top] -= tau * np.outer(v, v @ B[r:hi, lo:top])
                B[lo:top, r:hi] -= tau * np.outer(B[lo:top, r:hi] @ v, v)
            refl.append((r, v, tau))
            B[r + 1:hi, c] = 0.0
            B[c, r + 1:hi] = 0.0
            # the bulge: column r's entries below row r + b - 1 ... created at rows hi .. hi+b-1
            c, r = r, hi
            if r >= n or not np.any(np.abs(B[r:min(r + b, n), c]) > 0):
                break
    d = np.diag(B).copy()
    e = np.diag(B, -1).copy()
    return d, e, refl, B


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 216
    b = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    rng = np.random.default_rng(1)
    Y = rng.standard_normal((k, p)) * np.exp(rng.uniform(-3, 3, p))  # spread column scales
    A = (k - 1) / 1.1 * np.eye(k) + Y @ Y.T
    b1 = rng.standard_normal(k)
    xp = rng.standard_normal(k)

    Bm, panels, s1 = stage1_band(A, b)
    band_ok = np.max(np.abs(np.tril(Bm, -b - 1))) / np.max(np.abs(A))
    d, e, refl, Tm = stage2_chase(Bm, b)
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    off = np.max(np.abs(Tm - T)) / np.max(np.abs(A))

    # Q = Q1 Q2: apply to the identity (the kernels apply it to two vectors only)
    def apply_q(Xm):
        Xm = Xm.copy()
        for r, v, tau in reversed(refl):
            Xm[r:r + len(v)] -= tau * np.outer(v, v @ Xm[r:r + len(v)])
        for r0, V, Tp in reversed(panels):
            Xm[r0:] -= V @ (Tp @ (V.T @ Xm[r0:]))
        return Xm

    Q = apply_q(np.eye(k))
    rec = np.max(np.abs(Q @ T @ Q.T - A)) / np.max(np.abs(A))
    lam_t = np.linalg.eigvalsh(T)
    lam_a = np.linalg.eigvalsh(A)
    lam_err = np.max(np.abs(lam_t - lam_a) / lam_a)
    # LETKF quantities from T and Q, against eigh of A
    w, U = np.linalg.eigh(A)
    wbar_ref = U @ ((U.T @ b1) / w)
    wx_ref = np.sqrt(k - 1) * U @ ((U.T @ xp) / np.sqrt(w))
    wt, Ut = np.linalg.eigh(T)
    QtB, QtX = Q.T @ b1, Q.T @ xp
    wbar = Q @ (Ut @ ((Ut.T @ QtB) / wt))
    wx = np.sqrt(k - 1) * Q @ (Ut @ ((Ut.T @ QtX) / np.sqrt(wt)))
    rel = lambda a, r: np.linalg.norm(a - r) / np.linalg.norm(r)

    n_panels = len(panels)
    f1 = sum(4 * (k - r0) ** 2 * b + 2 * (k - r0) * b * b for r0, _, _ in panels)  # W + update + panel QR
    f2 = sum(4 * len(v) * (2 * b + len(v)) for _, v, _ in refl)
    print(f"k={k} p={p} b={b}")
    print(f"  stage 1: {n_panels} panels, {s1} panel Householder steps (sequential), ~{f1 / 1e6:.2f} MFLOP (GEMM part on MFMA)")
    print(f"  stage 2: {len(refl)} chase reflectors of length <= {b} (sequential), ~{f2 / 1e6:.2f} MFLOP")
    print(f"  one-stage dsytd2 for comparison: {k - 2} steps, ~{4 * k ** 3 / 3 / 1e6:.2f} MFLOP (matvec + rank-2 on the VALU)")
    print(f"  band check {band_ok:.1e}, tridiagonal check {off:.1e}, Q T Q^T = A to {rec:.1e}")
    print(f"  eigenvalues of T vs A: max rel {lam_err:.1e}")
    print(f"  wbar = A^-1 b1: rel {rel(wbar, wbar_ref):.1e};  sqrt(k-1) A^-1/2 x': rel {rel(wx, wx_ref):.1e}")


if __name__ == "__main__":
    main()
