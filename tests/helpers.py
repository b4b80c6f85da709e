"""Test helpers: golden-fixture loading and the oracle's ctypes binding.

The oracle (oracle/lib/liboracle.so) is TEST INFRASTRUCTURE: it is only ever used here as
the checker, never as the thing measured.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from cwbl import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_LIB = os.path.join(REPO, "oracle", "lib", "liboracle.so")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_LIB):
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "all"], check=True,
                           capture_output=True)
        lib = C.CDLL(ORACLE_LIB)
        vp = C.c_void_p
        lib.orc_lapack_name.restype = C.c_char_p
        lib.orc_expf.argtypes = [C.c_float]
        lib.orc_expf.restype = C.c_float
        lib.orc_gaspari_cohn.argtypes = [C.c_float]
        lib.orc_gaspari_cohn.restype = C.c_float
        lib.orc_search_r2.restype = C.c_float
        lib.orc_letkf_solve.argtypes = [C.c_int, C.c_int, vp, vp, vp, C.c_float, C.c_int,
                                        C.c_float, C.c_int, C.c_float, vp, vp]
        lib.orc_search.argtypes = [C.c_int, vp, C.c_float, C.c_float, C.c_int, C.c_int, vp,
                                   vp, vp, vp]
        lib.orc_analyze_var.argtypes = [C.c_int, C.c_int, C.c_float, C.c_int,
                                        C.POINTER(abi.ObsSet), C.POINTER(abi.VarParams),
                                        C.POINTER(abi.Slab), C.c_int, C.POINTER(abi.Stats)]
        lib.orc_tune_q.argtypes = [C.c_int] * 6 + [vp]
        _oracle = lib
    return _oracle


def oracle_solve(k, p, xb, yo, yb, inflat, rp, ra, sp, sa, want_evals=True):
    lib = oracle()
    xb, yo, yb = (np.ascontiguousarray(a, np.float32) for a in (xb, yo, yb))
    xa = np.empty(k, np.float32)
    ev = np.empty(k, np.float64)
    lib.orc_letkf_solve(k, p, xb.ctypes.data, yo.ctypes.data, yb.ctypes.data, inflat, rp, ra,
                        sp, sa, xa.ctypes.data, ev.ctypes.data if want_evals else None)
    return xa, ev


def inflat_of(k, multi_infl):
    """inflat = (nmember-1) / multi_infl(ivar) in fp32 (module_letkf_core.f90:68)."""
    return np.float32(np.float32(k - 1) / np.float32(multi_infl))


class DriverCase:
    """One G4 fixture as ABI inputs (obs set, var params, slab) + expected output."""

    def __init__(self, name):
        d = golden(name)
        self.name = name
        self.k = int(d["k"])
        nx, ny, nz, self.ix_lim, self.iy_lim = (int(v) for v in d["dims"])
        self.wf, rp, sp = (int(v) for v in d["ctl"])
        norain, minfl, ra, sa = (np.float32(v) for v in d["ctl_f"])
        self.norain = float(norain)
        self.x, self.y, self.alt = d["x"], d["y"], d["alt"]
        self.var_in, self.var_out = d["var_in"], d["var_out"]
        gts, radar = {}, {}
        self.types = []
        for it in range(int(d["ntypes"])):
            hi, hf = d[f"t{it}_hdr_i"], d[f"t{it}_hdr_f"]
            fam, tid, nvar, nobs, use_it, max_lz = (int(v) for v in hi[:6])
            tp = abi.type_params(use_it=use_it, max_lz_pts=max_lz, hclr=float(hf[0]),
                                 vclr=float(hf[1]), err_muti=list(hf[2:7]),
                                 err_rej=list(hf[7:12]), is_assim=[int(v) for v in hi[6:11]])
            (gts if fam == 0 else radar)[tid] = tp
            t = dict(family=fam, type_id=tid, nvar=nvar, nobs=nobs,
                     xyz=d[f"t{it}_xyz"], obs=d[f"t{it}_obs"], error=d[f"t{it}_error"],
                     hdxb=d[f"t{it}_hdxb"], qc=d[f"t{it}_qc"])
            self.types.append(t)
        self.vp = abi.var_params(multi_infl=float(minfl), use_rtpp=rp, rtpp_alpha=float(ra),
                                 use_rtps=sp, rtps_alpha=float(sa), gts=gts, radar=radar)

    def obs_set(self, memory=abi.MEM_HOST, to_device=None):
        b = abi.ObsSetBuilder(memory)
        dev = to_device or (lambda a: a)
        for t in self.types:
            if t["family"] == 0:
                b.add_gts(t["type_id"], dev(t["xyz"]), dev(t["obs"]), dev(t["error"]),
                          dev(t["hdxb"]), dev(t["qc"]))
            else:
                b.add_radar(t["type_id"], dev(t["xyz"]), dev(t["obs"][:, 0].copy()),
                            dev(t["hdxb"][:, :, 0].copy()))
        return b.build()

    def slab(self):
        var = np.ascontiguousarray(self.var_in, np.float32).copy()
        s = abi.make_slab(np.ascontiguousarray(self.x, np.float32),
                          np.ascontiguousarray(self.y, np.float32),
                          np.ascontiguousarray(self.alt, np.float32), var,
                          self.ix_lim, self.iy_lim)
        return s, var


def increment_rel_rms(xa, xa_ref, xb):
    """SURVEY.md §8(d) parity metric: rms(xa - xa_ref) / rms(xa_ref - xb).

    NaN-aware: the reference itself produces NaN analyses (Q8: with weight_function=1 the
    fp32 Gaspari-Cohn polynomial returns tiny negatives near z=2 and sqrt() gives NaN,
    module_localization.f90:360 / module_letkf_core.f90:449).  NaNs must occur at exactly
    the same places; the metric is taken over the finite values."""
    xa, xa_ref, xb = (np.asarray(a, np.float64) for a in (xa, xa_ref, xb))
    nan_a, nan_r = np.isnan(xa), np.isnan(xa_ref)
    if not np.array_equal(nan_a, nan_r):
        return float("inf")
    fin = ~nan_r
    den = np.sqrt(np.mean((xa_ref[fin] - xb[fin]) ** 2)) if fin.any() else 0.0
    num = np.sqrt(np.mean((xa[fin] - xa_ref[fin]) ** 2)) if fin.any() else 0.0
    return num / den if den > 0 else num


# ---- an independent fp64 evaluation of letkf_solve for ill-conditioned spectra ---------------
def eigen_direct_solve(k, xb, yo, yb, inflat, rp, ra, sp, sa):
    """letkf_solve (module_letkf_core.f90:598-700) with the eigendecomposition applied to the
    two vectors directly: wbar . x' = sum_a (q_a . Yb d)(q_a . x') / lam_a and
    W x' = sqrt(k-1) sum_a q_a (q_a . x') / sqrt(lam_a), never forming Pa = V L^-1 V^T.
    The reference forms Pa (dgemm) and multiplies it by Yb d; when tiny obs errors make
    |Yb d| ~ 1e13 the rounding of Pa's entries alone (~1e-17) moves wbar by ~1e-4 (measured
    against 60-digit arithmetic: scratch work, HISTORY.md §4), whereas here both factors of
    the ill-conditioned directions are small.  fp32 inputs and the fp32 epilogue follow the
    reference's order (oracle/letkf_oracle.c:506-541).  yb: (p, k) member fastest."""
    yb8 = np.asarray(yb, np.float64).reshape(-1, k)
    A = yb8.T @ yb8 + float(np.float32(inflat)) * np.eye(k)
    lam, Q = np.linalg.eigh(A)
    # A = inflat I + Yb Yb^T >= inflat: where |A| ~ 1e14 the computed eigenvalues of the
    # unobserved directions scatter by eps |A| around inflat (x' and Yb d have no part there)
    lam = np.maximum(lam, float(np.float32(inflat)))
    yd = yb8.T @ np.asarray(yo, np.float64)
    xb = np.asarray(xb, np.float32)
    s = np.float32(0.0)
    for v in xb:
        s = np.float32(s + v)
    xb_mean = float(np.float32(s * np.float32(1.0 / k)))
    xp = xb.astype(np.float64) - xb_mean
    cx = Q.T @ xp
    dot = float(np.sum((Q.T @ yd) * cx / lam))
    wx = np.sqrt(k - 1.0) * (Q @ (cx / np.sqrt(lam)))
    xa = (xb_mean + (dot + wx)).astype(np.float32)
    if rp or sp:
        ninv = np.float32(1.0 / k)
        s = np.float32(0.0)
        for v in xa:
            s = np.float32(s + v)
        xa_mean = np.float32(s * ninv)
        xap = (xa - xa_mean).astype(np.float32)
        if rp:
            a1 = np.float32(np.float32(1.0) - np.float32(ra))
            xap = ((a1 * xap).astype(np.float64) + float(np.float32(ra)) * xp).astype(np.float32)
        if sp:
            d8 = 0.0
            for v in xp:
                d8 = d8 + v * v
            xa_std = np.float32(0.0)
            for v in xap:
                xa_std = np.float32(xa_std + v * v)
            a = np.float32(sa)
            fac = np.float32(a * np.sqrt(np.float32(np.float32(d8) / xa_std)) - a + np.float32(1.0))
            xap = (xap * fac).astype(np.float32)
        xa = (xa_mean + xap).astype(np.float32)
    return xa


def radar_point_columns(w, kz, j, i, err):
    """letkf_yoyb's columns (module_letkf_core.f90:478-523) of grid point (kz, j, i) for a
    one-radar-type workload with Gaussian weights and no max_lz_pts truncation: the obs within
    the fixed ball (fp32 distances as kdtree2 computes them), reference fp32 order, the
    oracle's expf (glibc's).  Returns (yo (p,), yb (p, k)); the column order is obs-index
    order, not kdtree2's, which changes only the order of fp64 sums."""
    lib = oracle()
    k = w.k
    cfg = w.extra["cfg"]
    f = np.float32
    hinv, vinv = f(1.0) / f(f(cfg["hclr"]) * f(1e3)), f(1.0) / f(f(cfg["vclr"]) * f(1e3))
    on = np.stack([w.obs_xyz[:, 0] * hinv, w.obs_xyz[:, 1] * hinv, w.obs_xyz[:, 2] * vinv], 1)
    q = np.array([w.x[j, i] * hinv, w.y[j, i] * hinv, w.alt[kz, j, i] * vinv], np.float32)
    d = (on - q).astype(np.float32)
    r2 = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]).astype(np.float32) + d[:, 2] * d[:, 2]).astype(np.float32)
    sel = np.where(r2 <= lib.orc_search_r2())[0]
    hd = w.hdxb[:, sel]
    s = np.zeros(len(sel), np.float32)
    for m in range(k):
        s = (s + hd[m]).astype(np.float32)
    mean = (s * f(1.0 / k)).astype(np.float32)
    bg = (hd - mean).astype(np.float32)
    dd = np.zeros(len(sel), np.float32)
    for m in range(k):
        dd = (dd + bg[m] * bg[m]).astype(np.float32)
    omm = (w.obs[sel] - mean).astype(np.float32)
    std = np.sqrt((dd * f(1.0 / (k - 1))).astype(np.float32))
    e = f(err)
    rej = f(w.vp.radar[w.radar_type - 1].err_rej[0])
    keep = ~(np.abs(omm) > (np.sqrt((std * std + e * e).astype(np.float32)) * rej).astype(np.float32))
    einv = np.array([f(1.0) / f(e * f(lib.orc_expf(f(0.25) * v))) for v in r2[sel]], np.float32)
    yo = (omm * einv).astype(np.float32)[keep]
    yb = (bg * einv).astype(np.float32).T[keep]
    return yo, yb


def pair_ensemble(w, err, seed=5):
    """Replace a synthetic workload's values by a member-pair ensemble on a dyadic grid
    (members 2i, 2i+1 = mean +/- delta_i, k a power of two): the fp32 means are exact, so the
    perturbations are exactly zero-sum (in the reference too, module_letkf_core.f90:430-434,
    671).  The (k/2)-dimensional pair-symmetric subspace then carries eigenvalue inflat exactly
    and no part of x' or Yb d, so the problem stays well posed when tiny obs errors push the
    spectrum bound M/m far past 1e12: the reference's dsyevd path and the quadrature agree
    there, instead of both resolving an ill-conditioned direction to O(kappa eps)."""
    rng = np.random.default_rng(seed)
    k, n = w.k, w.obs.shape[0]
    dy = lambda a: (np.round(np.asarray(a) * 256.0) / 256.0).astype(np.float32)  # noqa: E731
    sgn = np.where(np.arange(k) % 2 == 0, 1.0, -1.0)[:, None]
    mu = dy(rng.standard_normal(n))
    delta = dy(2.0 * rng.standard_normal((k // 2, n)))
    w.hdxb = dy(mu[None, :] + sgn * np.repeat(delta, 2, axis=0))
    w.obs = dy(mu + rng.standard_normal(n))
    shape = w.var.shape[1:]
    xm = dy(rng.standard_normal(shape))
    eps = dy(rng.standard_normal((k // 2,) + shape))
    w.var = np.ascontiguousarray(dy(xm[None] + sgn.reshape((k, 1, 1, 1)) * np.repeat(eps, 2, axis=0)))
    from cwbl import synth
    cfg = w.extra["cfg"]
    w.vp = synth.radar_var_params(cfg["hclr"], cfg["vclr"], cfg["max_lz"], err, cfg["err_rej"],
                                  w.radar_type)
    # RTPS off: with every direction observed this precisely the analysis spread is ~1e-7 of
    # the background's, so the reference's fp32 xa' = xa - mean(xa) (:684-697) is pure
    # rounding, and RTPS would rescale that rounding by ~1e7 (RTPP keeps alpha xb')
    w.vp.use_rtps = 0
    return w
