"""Pin the C restatement (oracle/) against the reference's own outputs (tests/golden/).

CPU only.  With MKL available (this image: /opt/conda/lib/libmkl_rt.so) the oracle makes
the same LAPACK/BLAS calls as the reference and must agree BIT FOR BIT; with the builtin
Jacobi fallback it must agree to the parity tolerance.
"""
import ctypes as C

import numpy as np
import pytest

from cwbl import abi
from helpers import (DriverCase, golden, inflat_of, increment_rel_rms, oracle, oracle_solve)

BITEXACT = None


def bitexact():
    global BITEXACT
    if BITEXACT is None:
        BITEXACT = oracle().orc_lapack_name().decode() == "mkl"
    return BITEXACT


def test_constants():
    g = golden("consts.npz")
    assert np.float32(oracle().orc_search_r2()).view(np.uint32) == g["r2"].view(np.uint32)
    assert g["nmember_inv_k8"] == np.float32(1.0) / np.float32(8)


def test_gaspari_cohn_bitexact():
    g = golden("gc.npz")
    f = oracle().orc_gaspari_cohn
    y = np.array([f(float(x)) for x in g["x"]], np.float32)
    np.testing.assert_array_equal(y.view(np.uint32), g["y"].view(np.uint32))


def test_expf_matches_libm_sample():
    libm = C.CDLL("libm.so.6")
    libm.expf.argtypes = [C.c_float]
    libm.expf.restype = C.c_float
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(0, 3.5, 20000), rng.uniform(-20, 20, 2000)]).astype(np.float32)
    o = oracle().orc_expf
    a = np.array([o(float(x)) for x in xs], np.float32)
    b = np.array([libm.expf(float(x)) for x in xs], np.float32)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("k", [8, 40, 64, 128])
def test_solve_kat(k):
    g = golden(f"solve_k{k}.npz")
    col = g["col_off"]
    worst = 0.0
    for i in range(len(g["p"])):
        p = int(g["p"][i])
        yo = g["yo"][col[i]:col[i + 1]]
        yb = g["yb"][col[i] * k:col[i + 1] * k]
        infl = inflat_of(k, g["multi_infl"][i])
        xa, lam = oracle_solve(k, p, g["xb"][i], yo, yb, infl, int(g["use_rtpp"][i]),
                               float(g["rtpp_alpha"][i]), int(g["use_rtps"][i]),
                               float(g["rtps_alpha"][i]))
        if bitexact():
            np.testing.assert_array_equal(xa.view(np.uint32), g["xa"][i].view(np.uint32),
                                          err_msg=f"point {i} p={p}")
            np.testing.assert_array_equal(lam, g["lam"][i])
        else:
            worst = max(worst, increment_rel_rms(xa, g["xa"][i], g["xb"][i]))
            np.testing.assert_allclose(lam, g["lam"][i], rtol=1e-12)
    assert worst <= 1e-6


SEARCHES = ["search_3d.npz", "search_3d_overflow.npz", "search_2d.npz",
            "search_2d_overflow_dups.npz", "search_3d_small.npz", "search_3d_bucket.npz"]


@pytest.mark.parametrize("name", SEARCHES)
def test_search_kat_traversal_order(name):
    g = golden(name)
    mlz = int(g["max_lz"])
    q = np.ascontiguousarray(g["q_xyz"], np.float32)
    o = np.ascontiguousarray(g["obs_xyz"], np.float32)
    nq = q.shape[0]
    nf = np.empty(nq, np.int32)
    idx = np.full((nq, mlz), -1, np.int32)
    r2 = np.zeros((nq, mlz), np.float32)
    oracle().orc_search(o.shape[0], o.ctypes.data, float(g["hclr"]), float(g["vclr"]), mlz, nq,
                        q.ctypes.data, nf.ctypes.data, idx.ctypes.data, r2.ctypes.data)
    np.testing.assert_array_equal(nf, g["nfound"])
    for iq in range(nq):
        n = nf[iq]
        np.testing.assert_array_equal(idx[iq, :n], g["idx"][iq, :n])
        np.testing.assert_array_equal(r2[iq, :n].view(np.uint32), g["r2"][iq, :n].view(np.uint32))


DRIVERS = ["driver_c1.npz", "driver_mixed.npz", "driver_gc_k40.npz", "driver_2d.npz",
           "driver_q1.npz", "driver_offset.npz", "driver_zdr.npz"]


@pytest.mark.parametrize("name", DRIVERS)
def test_driver_one_variable(name):
    case = DriverCase(name)
    obs = case.obs_set()
    slab, var = case.slab()
    st = abi.Stats()
    rc = oracle().orc_analyze_var(case.k, case.wf, case.norain, abi.Q1_REPLICATE,
                                  C.byref(obs), C.byref(case.vp), C.byref(slab), 4,
                                  C.byref(st))
    assert rc == 0
    if bitexact():
        np.testing.assert_array_equal(var.view(np.uint32), case.var_out.view(np.uint32))
    else:
        assert increment_rel_rms(var, case.var_out, case.var_in) <= 1e-6
    assert st.solved > 0


def tune_q_cases():
    g = golden("tune_q.npz")
    return [(int(g[f"k{i}"]), g[f"q_in{i}"], g[f"q_out{i}"]) for i in range(int(g["ncases"]))]


def test_tune_q_bitexact():
    """orc_tune_q against letkf_tune_q (module_letkf_core.f90:702-733) compiled from the
    reference: bit for bit, including the Q3 NaN columns (0/0) and the all-negative ones."""
    for k, q_in, q_out in tune_q_cases():
        nx, ny, nz, _ = q_in.shape
        var = np.asfortranarray(q_in.copy())
        oracle().orc_tune_q(k, nx, ny, nz, nx, ny, var.ctypes.data)
        np.testing.assert_array_equal(var.view(np.uint32), q_out.view(np.uint32))
        assert np.isnan(q_out[0, 0, 0, :]).all()  # Q3 replicated by the reference itself
