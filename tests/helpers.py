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
