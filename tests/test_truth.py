"""The fp64 'eigen-direct' evaluation of letkf_solve (helpers.eigen_direct_solve) that pins
the GPU where tiny obs errors make the reference's own Pa-times-Yb d path inaccurate
(tests/test_gpu_parity.py::test_tiny_obs_errors_beyond_the_31_node_rule): it must equal the
oracle in the ordinary regime and 50-digit arithmetic in the tiny-error one."""
import ctypes as C

import numpy as np
import pytest

from cwbl import abi, synth
from helpers import (eigen_direct_solve, increment_rel_rms, inflat_of, oracle, pair_ensemble,
                     radar_point_columns)

POINTS = [(0, 5, 5), (1, 8, 3), (3, 10, 10), (2, 2, 14), (0, 0, 0)]


def test_eigen_direct_equals_the_oracle_in_the_ordinary_regime():
    w = synth.make("c2", seed=13, scale=0.06, nz=4, k=32)
    ref = w.var.copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    assert oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                    C.byref(abi.make_slab(w.x, w.y, w.alt, ref)), 4,
                                    C.byref(abi.Stats())) == 0
    vp = w.vp
    for kz, j, i in POINTS:
        yo, yb = radar_point_columns(w, kz, j, i, vp.radar[w.radar_type - 1].err_muti[0])
        assert len(yo) > 0
        xa = eigen_direct_solve(w.k, w.var[:, kz, j, i], yo, yb, inflat_of(w.k, vp.multi_infl),
                                vp.use_rtpp, vp.rtpp_alpha, vp.use_rtps, vp.rtps_alpha)
        assert increment_rel_rms(xa, ref[:, kz, j, i], w.var[:, kz, j, i]) <= 1e-12


@pytest.mark.parametrize("k", [16, 32])
def test_eigen_direct_equals_50_digits_with_tiny_obs_errors(k):
    mp = pytest.importorskip("mpmath")
    err = 2.0 ** -20
    w = pair_ensemble(synth.make("c2", seed=13, scale=0.06, nz=4, k=k), err)
    infl = inflat_of(k, w.vp.multi_infl)
    mp.mp.dps = 50
    for kz, j, i in POINTS[:2]:
        yo, yb = radar_point_columns(w, kz, j, i, err)
        p = len(yo)
        # eigen-direct before the fp32 epilogue (RTPP/RTPS off, analysis in fp64 kept)
        xb = w.var[:, kz, j, i]
        yb8 = yb.astype(np.float64)
        lam, Q = np.linalg.eigh(yb8.T @ yb8 + float(infl) * np.eye(k))
        lam = np.maximum(lam, float(infl))
        s = np.float32(0.0)
        for v in xb:
            s = np.float32(s + v)
        xm = float(np.float32(s * np.float32(1.0 / k)))
        cx = Q.T @ (xb.astype(np.float64) - xm)
        dot = np.sum((Q.T @ (yb8.T @ yo.astype(np.float64))) * cx / lam)
        pre = xm + (dot + np.sqrt(k - 1.0) * (Q @ (cx / np.sqrt(lam))))
        Y = mp.matrix(k, p)
        for a in range(k):
            for t in range(p):
                Y[a, t] = mp.mpf(float(yb[t, a]))
        A = Y * Y.T
        for a in range(k):
            A[a, a] += mp.mpf(float(infl))
        E, V = mp.eigsy(A)
        cy = V.T * (Y * mp.matrix([mp.mpf(float(v)) for v in yo]))
        cxm = V.T * mp.matrix([mp.mpf(float(v)) - mp.mpf(xm) for v in xb])
        dm = mp.fsum(cy[a] * cxm[a] / E[a] for a in range(k))
        wx = V * mp.matrix([cxm[a] / mp.sqrt(E[a]) for a in range(k)])
        hp = np.array([float(mp.mpf(xm) + dm + mp.sqrt(k - 1) * wx[m]) for m in range(k)])
        assert np.max(np.abs(pre - hp)) <= 1e-13, np.max(np.abs(pre - hp))
        assert float(mp.fsum(A[a, a] for a in range(k))) / float(infl) - (k - 1) > 1e12
