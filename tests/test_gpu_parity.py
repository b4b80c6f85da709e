"""GPU parity tests: the HIP core through the C ABI against the reference's golden vectors
(tests/golden/, produced by the reference's own compiled code) and against the oracle.

Tolerances (north_star / SURVEY.md §8(d)):
  analysis increments  rms(xa_gpu - xa_ref) / rms(xa_ref - xb) <= 1e-6   (INCR_TOL)
  eigenvalues          max |lam_gpu - lam_ref| / lam_ref        <= 1e-12  (EIG_TOL), ascending
  neighbour search     bit-exact (same indices, same traversal order, same fp32 r2)
"""
import numpy as np
import pytest

from cwbl import abi
from helpers import (DriverCase, golden, inflat_of, increment_rel_rms, oracle)

pytestmark = pytest.mark.gpu

INCR_TOL = 1e-6
EIG_TOL = 1e-12

_cores = {}


def core(k, wf=0, norain=-5.0, q1=abi.Q1_REPLICATE):
    """One library state per process: re-init when the configuration changes."""
    key = (k, wf, norain, q1)
    if _cores.get("key") != key:
        if "core" in _cores:
            _cores["core"].finalize()
        _cores["core"] = abi.Core(k, device=0, weight_function=wf, norain_value=norain,
                                  q1_mode=q1)
        _cores["key"] = key
    return _cores["core"]


@pytest.mark.parametrize("k,solver", [(8, "tq"), (40, "tq"), (64, "tq"), (128, "tq"),
                                      (8, "jacobi"), (40, "jacobi"), (64, "jacobi")])
def test_solve_batch_matches_reference(k, solver):
    """G1 through cwbl_solve_batch with the eigenvalue output: increments within 1e-6 and
    dsyevd's ascending eigenvalues within 1e-12 at every k.  Default: the tq kernels' T and
    bisection (cwbl_eig.hip); option solver = 1 (k <= 64): the Jacobi eigensolver."""
    g = golden(f"solve_k{k}.npz")
    _cores.clear()
    c = abi.Core(k, device=0, options={"solver": int(solver == "jacobi")})
    col = g["col_off"]
    # group points that share the solve parameters
    keys = list(zip(g["multi_infl"], g["use_rtpp"], g["use_rtps"], g["rtpp_alpha"], g["rtps_alpha"]))
    worst, worst_eig = 0.0, 0.0
    for key in sorted(set(keys)):
        sel = [i for i, kk in enumerate(keys) if kk == key]
        off = np.concatenate([[0], np.cumsum([col[i + 1] - col[i] for i in sel])]).astype(np.int64)
        yo = np.concatenate([g["yo"][col[i]:col[i + 1]] for i in sel])
        yb = np.concatenate([g["yb"][col[i] * k:col[i + 1] * k] for i in sel])
        xb = np.stack([g["xb"][i] for i in sel])
        infl, rp, sp, ra, sa = key
        xa, ev = c.solve_batch(off, yo, yb, xb, inflat_of(k, infl), int(rp), float(ra), int(sp),
                               float(sa), want_evals=True)
        for n, i in enumerate(sel):
            worst = max(worst, increment_rel_rms(xa[n], g["xa"][i], g["xb"][i]))
            rel = np.max(np.abs(ev[n] - g["lam"][i]) / np.abs(g["lam"][i]))
            worst_eig = max(worst_eig, rel)
    c.finalize()
    assert worst <= INCR_TOL, worst
    assert worst_eig <= EIG_TOL, worst_eig


@pytest.mark.parametrize("k", [2, 3, 9, 25, 33, 65, 97, 128])
def test_eigenvalues_at_every_padding_class(k):
    """Random batches at k's of every kernel class (KP = 8..64 one wavefront, k = 25..32 at
    KP = 40, KP = 96 and 128 on 256 threads), including points with p < k (k - p equal
    eigenvalues inflat), p = 0 and tiny p: ascending eigenvalues within 1e-12 of the
    oracle's dsyevd."""
    from helpers import oracle_solve
    rng = np.random.default_rng(k)
    ps = [0, 1, 2, k - 1, k, k + 3, 200][: 7 if k > 2 else 6]
    ps = [p for p in ps if p >= 0]
    col = np.concatenate([[0], np.cumsum(ps)]).astype(np.int64)
    yo = rng.standard_normal(col[-1]).astype(np.float32)
    yb = (rng.standard_normal((col[-1], k)) * rng.uniform(0.1, 3.0, (col[-1], 1))).astype(np.float32)
    xb = (280.0 + rng.standard_normal((len(ps), k))).astype(np.float32)
    infl = inflat_of(k, 1.6)
    c = core(k)
    xa, ev = c.solve_batch(col, yo, yb.ravel(), xb, infl, 1, 0.95, 1, 0.95, want_evals=True)
    for i, p in enumerate(ps):
        assert np.all(np.diff(ev[i]) >= 0), (p, ev[i])
        if p == 0:
            np.testing.assert_allclose(ev[i], np.float64(infl), rtol=4e-16, atol=0)
            np.testing.assert_array_equal(xa[i], xb[i])
            continue
        xr, lr = oracle_solve(k, p, xb[i], yo[col[i]:col[i + 1]], yb[col[i]:col[i + 1]], infl,
                              1, 0.95, 1, 0.95)
        assert np.max(np.abs(ev[i] - lr) / np.abs(lr)) <= EIG_TOL, (p, ev[i] - lr)
        assert increment_rel_rms(xa[i], xr, xb[i]) <= INCR_TOL


@pytest.mark.parametrize("k", [8, 40, 64, 128])
def test_solve_batch_tq_matches_reference(k):
    """Without an eigenvalue output cwbl_solve_batch runs the tridiagonalisation + quadrature
    kernel (cwbl_tq.hip): same increments as the reference's dsyevd path."""
    g = golden(f"solve_k{k}.npz")
    c = core(k)
    col = g["col_off"]
    worst = 0.0
    for i in range(len(g["xb"])):
        off = np.array([0, col[i + 1] - col[i]], np.int64)
        xa, _ = c.solve_batch(off, g["yo"][col[i]:col[i + 1]], g["yb"][col[i] * k:col[i + 1] * k],
                              g["xb"][i][None], inflat_of(k, g["multi_infl"][i]),
                              int(g["use_rtpp"][i]), float(g["rtpp_alpha"][i]),
                              int(g["use_rtps"][i]), float(g["rtps_alpha"][i]))
        worst = max(worst, increment_rel_rms(xa[0], g["xa"][i], g["xb"][i]))
    assert worst <= INCR_TOL, worst


def test_k_limits():
    """k up to 128 is supported (k > 64 on the 256-thread kernels); beyond that the library
    reports UNSUPPORTED."""
    with pytest.raises(abi.CwblError, match="UNSUPPORTED"):
        abi.Core(129, device=0)
    _cores.clear()


SEARCHES = ["search_3d.npz", "search_3d_overflow.npz", "search_2d.npz",
            "search_2d_overflow_dups.npz", "search_3d_small.npz", "search_3d_bucket.npz"]


@pytest.mark.parametrize("name", SEARCHES)
def test_search_matches_reference_order(name):
    g = golden(name)
    c = core(8)
    nf, idx, r2 = c.search(g["obs_xyz"], float(g["hclr"]), float(g["vclr"]), int(g["max_lz"]),
                           g["q_xyz"])
    np.testing.assert_array_equal(nf, g["nfound"])
    for q in range(len(nf)):
        n = nf[q]
        np.testing.assert_array_equal(idx[q, :n], g["idx"][q, :n])
        np.testing.assert_array_equal(r2[q, :n].view(np.uint32), g["r2"][q, :n].view(np.uint32))


DRIVERS = ["driver_c1.npz", "driver_mixed.npz", "driver_gc_k40.npz", "driver_2d.npz",
           "driver_q1.npz", "driver_offset.npz", "driver_zdr.npz"]


@pytest.mark.parametrize("name", DRIVERS)
def test_driver_variable_matches_reference(name):
    case = DriverCase(name)
    c = core(case.k, case.wf, case.norain)
    c.set_obs(case.obs_set())
    slab, var = case.slab()
    st = c.analyze_var(case.vp, slab)
    rel = increment_rel_rms(var, case.var_out, case.var_in)
    assert rel <= INCR_TOL, rel
    # untouched points stay bit-identical (no accepted obs / outside ix_lim, iy_lim)
    untouched = np.all(case.var_out == case.var_in, axis=0)
    np.testing.assert_array_equal(var[:, untouched], case.var_in[:, untouched])
    assert st.solved == int(np.sum(~untouched))
    assert st.nonconverged == 0


def test_device_memory_path_equals_host_path():
    torch = pytest.importorskip("torch")
    case = DriverCase("driver_mixed.npz")
    c = core(case.k, case.wf, case.norain)
    dev = torch.device("cuda:0")
    to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    c.set_obs(case.obs_set(memory=abi.MEM_DEVICE, to_device=to_dev))
    x, y, alt = (to_dev(np.asarray(a, np.float32)) for a in (case.x, case.y, case.alt))
    var = to_dev(np.asarray(case.var_in, np.float32).copy())
    torch.cuda.synchronize()
    slab = abi.make_slab(x, y, alt, var, case.ix_lim, case.iy_lim, memory=abi.MEM_DEVICE)
    c.analyze_var(case.vp, slab)
    got = var.cpu().numpy()
    # host path on the same inputs
    c.set_obs(case.obs_set())
    hslab, hvar = case.slab()
    c.analyze_var(case.vp, hslab)
    np.testing.assert_array_equal(got.view(np.uint32), hvar.view(np.uint32))


@pytest.mark.parametrize("where", ["side_stream", "default_stream"])
def test_device_inputs_only_need_to_be_queued(where):
    """cwbl_set_obs / cwbl_analyze_var on device buffers whose producers are still queued
    (behind a GPU spin) on the caller's stream: a side stream declared with cwbl_set_stream,
    or torch's default (legacy null) stream, the library's default.  The library orders
    itself after that stream's queued work by an event (not a device-wide synchronise)."""
    torch = pytest.importorskip("torch")
    case = DriverCase("driver_mixed.npz")
    c = core(case.k, case.wf, case.norain)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream() if where == "side_stream" else torch.cuda.default_stream()
    c.set_stream(s)
    staged = []

    def late(a):  # a device copy of `a` written only after ~10 ms of GPU spin on stream s
        src = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        dst = torch.zeros_like(src)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            torch.cuda._sleep(20_000_000)
            dst.copy_(src)
        staged.append(src)
        return dst

    c.set_obs(case.obs_set(memory=abi.MEM_DEVICE, to_device=late))
    x, y, alt = (late(np.asarray(a, np.float32)) for a in (case.x, case.y, case.alt))
    var = late(np.asarray(case.var_in, np.float32).copy())
    slab = abi.make_slab(x, y, alt, var, case.ix_lim, case.iy_lim, memory=abi.MEM_DEVICE)
    c.analyze_var(case.vp, slab)
    c.set_stream(None)
    got = var.cpu().numpy()
    c.set_obs(case.obs_set())
    hslab, hvar = case.slab()
    c.analyze_var(case.vp, hslab)
    np.testing.assert_array_equal(got.view(np.uint32), hvar.view(np.uint32))


def test_analyze_before_set_obs_is_a_state_error():
    c = abi.Core(8, device=0)
    _cores.clear()
    case = DriverCase("driver_c1.npz")
    slab, _ = case.slab()
    with pytest.raises(abi.CwblError, match="STATE"):
        c.analyze_var(case.vp, slab)
    c.finalize()


def _radar_case_scaled(scale, seed=11, **over):
    from cwbl import synth
    return synth.make("c2", seed=seed, scale=scale, **over)


def test_synthetic_c2_subdomain_vs_oracle():
    """C2-shaped workload (k=40, p~200) on a 60x60x50 sub-grid: GPU vs the oracle."""
    import ctypes as C
    w = _radar_case_scaled(0.2)
    c = core(w.k)
    b = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb)
    c.set_obs(b.build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    ref = w.var.copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    ost = abi.Stats()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(w.x, w.y, w.alt, ref)), 16, C.byref(ost))
    assert rc == 0
    assert st.solved == ost.solved and st.nobs_sum == ost.nobs_sum
    rel = increment_rel_rms(var, ref, w.var)
    assert rel <= INCR_TOL, rel
    assert st.nonconverged == 0


@pytest.mark.parametrize("k", [17, 20, 24, 25, 32, 33, 36, 40])
def test_split_kp40_path_vs_one_kernel_and_oracle(k):
    """The KP = 40 slab path runs split by default (assemble_record_kernel writes A and Yb d,
    solve_tq40_kernel runs the whole tridiagonalisation four points per wavefront, split40 = 1).
    k < 40 exercises the identity padding (the no-op steps past
    k - 2); k = 17..32 run at KP = 40 too (their one-kernel paths, split40 = 0, are KP = 24, 32).
    Both against the one-kernel path (split40 = 0) and the oracle on a 30x30x50 C2-shaped
    grid."""
    import ctypes as C
    w = _radar_case_scaled(0.1, k=k)
    out = {}
    for mode in ("0", "1"):
        _cores.clear()
        c = abi.Core(w.k, device=0, options={"split40": int(mode)})
        c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
        var = w.var.copy()
        st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
        c.finalize()
        assert st.nonconverged == 0 and st.solved > 0
        out[mode] = (var, st.solved, st.nobs_sum)
    assert out["0"][1:] == out["1"][1:]
    ref = w.var.copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(w.x, w.y, w.alt, ref)), 16,
                                  C.byref(abi.Stats()))
    assert rc == 0
    for mode in ("0", "1"):
        rel = increment_rel_rms(out[mode][0], ref, w.var)
        assert rel <= INCR_TOL, (mode, rel)
    rel = increment_rel_rms(out["1"][0], out["0"][0], w.var)
    assert rel <= INCR_TOL, rel


@pytest.mark.parametrize("n_obs", [40, 120])
def test_two_chunk_staging_at_sparse_densities(n_obs):
    """The record kernel stages two 32-column chunks per round (stage_columns_pair: lane
    (half, s) owns column s of chunk c + half and hands its slot and weight to the other half
    wave).  Sparse obs sets put the points' candidate counts all over 0..~150, so rounds with
    only chunk c, a partial chunk c + 1, exactly 32/64 candidates and empty lists all occur.
    Every point against the oracle."""
    import ctypes as C
    from cwbl import synth
    w = synth.make("c2", seed=11, nx=30, ny=30, n_obs=n_obs)
    c = core(w.k)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    ref = w.var.copy()
    ost = abi.Stats()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(w.x, w.y, w.alt, ref)), 16, C.byref(ost))
    assert rc == 0
    assert st.solved == ost.solved and st.nobs_sum == ost.nobs_sum
    assert st.solved > 0
    assert 10 < st.nobs_sum / st.solved < 100, st.nobs_sum / st.solved  # mean p: ~20, ~60
    assert increment_rel_rms(var, ref, w.var) <= INCR_TOL
    d = (var - ref).reshape(w.k, -1)
    inc = (ref - w.var).reshape(w.k, -1)
    dn = np.sqrt((d ** 2).sum(axis=0))
    tol = 1e-5 * np.maximum(np.sqrt((inc ** 2).sum(axis=0)), 1e-6)
    assert (dn <= tol).all(), int(np.argmax(dn - tol))


def test_split_kp40_ragged_record_batches():
    """Record sub-batches whose point count is not a multiple of four: the last wave of
    solve_tq40_kernel has lanes past the batch, which must not disturb a live point's record
    (they work on a spare record).  31x29x7 = 6293 points in sub-batches of 512 (the last has
    149).  Every point against the oracle, and the same analysis as one record batch."""
    import ctypes as C
    from cwbl import synth
    w = synth.make("c2", seed=11, nx=31, ny=29, nz=7, n_obs=240)
    assert w.points % 4 == 1
    out = {}
    for sub in ("512", "0"):
        _cores.clear()
        c = abi.Core(w.k, device=0, options={"split40_batch": int(sub)})
        c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
        var = w.var.copy()
        st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
        c.finalize()
        assert st.solved > 0 and st.nonconverged == 0
        out[sub] = var
    np.testing.assert_array_equal(out["512"].view(np.uint32), out["0"].view(np.uint32))
    ref = w.var.copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(w.x, w.y, w.alt, ref)), 16,
                                  C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(out["512"], ref, w.var)
    assert rel <= INCR_TOL, rel
    # the first point of every sub-batch (whose record a lane past the batch would share)
    # and the last point, individually
    d = (out["512"] - ref).reshape(w.k, -1)
    inc = (ref - w.var).reshape(w.k, -1)
    for g in list(range(0, w.points, 512)) + [w.points - 1]:
        assert np.sqrt((d[:, g] ** 2).sum()) <= 1e-5 * max(np.sqrt((inc[:, g] ** 2).sum()), 1e-6), g


def test_c2_full_size_properties():
    """Full C2 size (300x300x50, k=40): properties that do not need the oracle everywhere,
    plus an oracle check on a column block."""
    import ctypes as C
    from cwbl import synth
    w = synth.make("c2")
    c = core(w.k)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    assert st.points == w.points
    assert np.isfinite(var).all()
    assert st.nonconverged == 0
    mean_p = st.nobs_sum / max(st.solved, 1)
    assert 60 <= mean_p <= 400, mean_p
    # idempotence of the API on unchanged inputs: a second call on the same xb is identical
    var2 = w.var.copy()
    c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var2))
    np.testing.assert_array_equal(var.view(np.uint32), var2.view(np.uint32))
    # oracle on a 12x12 column block (all 50 levels) cut out of the same grid
    j0, i0, nb = 140, 150, 12
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    ref = sub(w.var).copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), ref)),
                                  16, C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(sub(var), ref, sub(w.var))
    assert rel <= INCR_TOL, rel


@pytest.mark.timeout(900)
def test_c2_full_grid_vs_oracle():
    """The headline configuration end to end against the oracle on EVERY point: the HIP core
    on the whole 300x300x50 C2 grid (k = 40, 22 500 obs, mean p ~216) and the C oracle's
    letkf_driver loop (module_letkf_core.f90:209-240) on the same 4.5 M points with all the
    host cores the job may use; whole-grid increments within 1e-6 relative RMS, the solved
    and accepted-obs counts equal, and per column block of 30x30 columns within 1e-6 as well
    (so that an error confined to a region cannot hide in the whole-grid mean)."""
    import ctypes as C
    from bench import baseline_procs
    from cwbl import synth
    w = synth.make("c2")
    c = core(w.k)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    ref = w.var.copy()
    ost = abi.Stats()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    threads, _ = baseline_procs()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(w.x, w.y, w.alt, ref)), threads,
                                  C.byref(ost))
    assert rc == 0
    assert st.solved == ost.solved and st.nobs_sum == ost.nobs_sum
    assert st.points == w.points == 300 * 300 * 50
    rel = increment_rel_rms(var, ref, w.var)
    assert rel <= INCR_TOL, rel
    worst = 0.0
    for j0 in range(0, 300, 30):
        for i0 in range(0, 300, 30):
            b = (Ellipsis, slice(j0, j0 + 30), slice(i0, i0 + 30))
            if np.array_equal(ref[b], w.var[b]):
                continue  # no solved point in the block: must be untouched
            worst = max(worst, increment_rel_rms(var[b], ref[b], w.var[b]))
    assert worst <= INCR_TOL, worst
    untouched = ref == w.var
    np.testing.assert_array_equal(var[untouched].view(np.uint32), w.var[untouched].view(np.uint32))


def test_batch_plan_does_not_change_the_analysis():
    """Points are independent, so the search/solve batch plan (batch cap, short lead batch,
    two list buffers alternating between overlapped searches and solves) must not change
    a single bit of the analysis."""
    from cwbl import synth
    w = synth.make("c2", scale=0.2)
    out = []
    for opts in ({}, {"max_batch": 9000, "lead_div": 8}):
        _cores.clear()
        c = abi.Core(w.k, device=0, options=opts)
        c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
        var = w.var.copy()
        c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
        c.finalize()
        out.append(var)
    _cores.clear()
    assert np.isfinite(out[0]).all()
    np.testing.assert_array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


@pytest.mark.timeout(600)
def test_c4_full_size_properties():
    """Full C4 size (300x300x50, k=128, the 256-thread kernel): finite, bitwise reproducible
    run to run (a cross-wave LDS race once showed up only as a few NaN points that moved
    between runs), and the oracle on a column block."""
    import ctypes as C
    from bench import baseline_procs
    from cwbl import synth
    w = synth.make("c4")
    c = core(w.k)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    assert st.points == w.points
    assert np.isfinite(var).all()
    assert st.nonconverged == 0
    var2 = w.var.copy()
    c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var2))
    np.testing.assert_array_equal(var.view(np.uint32), var2.view(np.uint32))
    # the oracle on a 20x20-column block (20 000 points, all 50 levels)
    j0, i0, nb = 140, 140, 20
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    ref = sub(w.var).copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), ref)),
                                  baseline_procs()[0], C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(sub(var), ref, sub(w.var))
    assert rel <= INCR_TOL, rel


@pytest.mark.parametrize("name", ["driver_mixed.npz", "driver_gc_k40.npz"])
def test_tq_and_jacobi_solvers_agree(name):
    """The two solve kernels (eigendecomposition by Jacobi, option solver = 1; and the
    default tridiagonalisation + quadrature) give the same analysis to the tolerance."""
    case = DriverCase(name)
    out = {}
    for solver in ("jacobi", "tq"):
        _cores.clear()
        c = abi.Core(case.k, device=0, weight_function=case.wf, norain_value=case.norain,
                     options={"solver": int(solver == "jacobi")})
        c.set_obs(case.obs_set())
        slab, var = case.slab()
        c.analyze_var(case.vp, slab)
        c.finalize()
        out[solver] = var
    rel = increment_rel_rms(out["tq"], out["jacobi"], case.var_in)
    assert rel <= INCR_TOL, rel


def test_tree_cache_across_variables():
    """Trees are cached per obs set and normalisation; column tables are rebuilt per
    variable.  A call with other localisation/QC parameters in between must not change the
    result of a repeated call (and a fresh state gives the same bits)."""
    import copy
    case = DriverCase("driver_mixed.npz")
    c = core(case.k, case.wf, case.norain)
    c.set_obs(case.obs_set())
    slab, var1 = case.slab()
    c.analyze_var(case.vp, slab)
    other = copy.deepcopy(case.vp)
    for tp in list(other.gts) + list(other.radar):
        tp.hclr = tp.hclr * 1.5
        tp.err_muti[0] = tp.err_muti[0] * 2.0
    slab2, _ = case.slab()
    c.analyze_var(other, slab2)
    slab3, var3 = case.slab()
    c.analyze_var(case.vp, slab3)
    np.testing.assert_array_equal(var3.view(np.uint32), var1.view(np.uint32))
    rel = increment_rel_rms(var1, case.var_out, case.var_in)
    assert rel <= INCR_TOL, rel


def test_dense_radar_c5_block_vs_oracle():
    """C5-shaped dense radar (dbz-like type, ~2000 local obs per point, max_lz 4000) on a
    30x30x60 cut of the 600x600x60 grid: GPU vs the oracle on a 6x6-column block.  A fifth
    of the obs are `norain` (some with all-norain backgrounds) to exercise the dbz rules
    (module_letkf_core.f90:504-507)."""
    import ctypes as C
    from cwbl import synth
    w = synth.make("c5", scale=0.05)
    norain = -5.0
    rng = np.random.default_rng(5)
    sel = rng.random(w.obs.shape[0]) < 0.2
    w.obs[sel] = norain
    allrain = sel & (rng.random(w.obs.shape[0]) < 0.5)
    w.hdxb[:, allrain] = norain
    c = core(w.k, 0, norain)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    assert np.isfinite(var).all()
    assert st.nonconverged == 0
    mean_p = st.nobs_sum / max(st.solved, 1)
    assert 600 <= mean_p <= 4000, mean_p
    j0, i0, nb = 12, 12, 6
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    ref = sub(w.var).copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, norain, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), ref)),
                                  16, C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(sub(var), ref, sub(w.var))
    assert rel <= INCR_TOL, rel


def test_c5_full_size_properties():
    """C5 at its stated size on one GPU (600x600x60 = 21.6 M points, k=40, 1.66 M dense
    radar obs, max_lz 4000; the configuration names 8 GPUs, whose rank shares are column
    blocks of this grid): finite, no non-convergence, run-to-run bitwise reproducible, and
    the oracle on a column block in the dense centre."""
    import ctypes as C
    from cwbl import synth
    w = synth.make("c5")
    c = core(w.k)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    assert st.points == w.points
    assert np.isfinite(var).all()
    assert st.nonconverged == 0
    mean_p = st.nobs_sum / max(st.solved, 1)
    assert 600 <= mean_p <= 4000, mean_p
    var2 = w.var.copy()
    c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var2))
    np.testing.assert_array_equal(var.view(np.uint32), var2.view(np.uint32))
    del var2
    j0, i0, nb = 297, 297, 4
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    ref = sub(w.var).copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), ref)),
                                  16, C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(sub(var), ref, sub(w.var))
    assert rel <= INCR_TOL, rel


@pytest.mark.parametrize("k", [80, 100, 128])
def test_large_ensemble_block_vs_oracle(k):
    """configs[3]-shaped large ensembles (k = 128, and k = 80 on the KP = 96 kernel) on a
    30x30x50 cut of the C2 grid: GPU vs the oracle on a 6x6-column block."""
    import ctypes as C
    from cwbl import synth
    w = synth.make("c4", scale=0.1, k=k)
    c = core(w.k)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    assert np.isfinite(var).all()
    assert st.nonconverged == 0
    j0, i0, nb = 12, 12, 6
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    ref = sub(w.var).copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), ref)),
                                  16, C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(sub(var), ref, sub(w.var))
    assert rel <= INCR_TOL, rel


@pytest.mark.parametrize("k,sparse", [(65, False), (80, True), (96, False), (97, False),
                                      (101, True), (127, False), (128, False), (128, True)])
def test_split_big_path_vs_one_kernel_and_oracle(k, sparse):
    """The KP = 96 / 128 slab paths run split by default: a 256-thread kernel per point
    (solve_tq_big_kernel<96, false, 32>, 4x4 register blocks; solve_tq_rows_kernel<128, 64>,
    half rows) hands the trailing 64x64 matrix and its reflectors to solve_tqb_tail_kernel
    (one point per wavefront); the kernel timing names the launched pair.  k < KP exercises
    the identity padding; the sparse obs set gives points with p < k (rank-deficient
    Yb Yb^T, exactly-zero reflectors, tau = 0).  Against the one-kernel path (big_path = 0)
    on the whole 30x30x50 grid and the oracle on a 5x5-column block; hand-off batches of
    1024 points."""
    import ctypes as C
    from cwbl import synth
    w = synth.make("c4", scale=0.1, k=k)
    if sparse:
        keep = np.arange(w.obs.shape[0]) % 25 == 0
        w.obs_xyz = np.ascontiguousarray(w.obs_xyz[keep])
        w.obs = np.ascontiguousarray(w.obs[keep])
        w.hdxb = np.ascontiguousarray(w.hdxb[:, keep])
    out = {}
    for mode in ("0", "1"):
        _cores.clear()
        c = abi.Core(w.k, device=0, options={"big_batch": 1024, "big_path": int(mode)})
        c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
        var = w.var.copy()
        c.set_kernel_timing(True)
        st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
        kt = c.kernel_times()
        c.finalize()
        if mode == "1":
            pair = (["solve_tq_rows_kernel<128, 64>", "solve_tqb_tail_kernel<128, 64, 3>"]
                    if k > 96 else
                    ["solve_tq_big_kernel<96, false, 32>", "solve_tqb_tail_kernel<96, 32, 2>"])
            for name in pair:
                assert kt.get(name, {}).get("launches", 0) > 0, (name, sorted(kt))
        assert np.isfinite(var).all()
        assert st.nonconverged == 0 and st.solved > 0
        out[mode] = (var, st.solved, st.nobs_sum)
    _cores.clear()
    assert out["0"][1:] == out["1"][1:]
    if sparse:
        assert out["1"][2] / out["1"][1] < k, out["1"][2] / out["1"][1]
    rel = increment_rel_rms(out["1"][0], out["0"][0], w.var)
    assert rel <= INCR_TOL, rel
    j0, i0, nb = 12, 12, 5
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    ref = sub(w.var).copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), ref)),
                                  16, C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(sub(out["1"][0]), ref, sub(w.var))
    assert rel <= INCR_TOL, rel


def test_info_window_rollover_matches_single_window():
    """The per-point solve info (solved flag, p) is reduced once per window of
    CWBL_OPT_INFO_WINDOW points (2^25 by default, so one window below 33.5 M points).  Small
    windows over small search batches force many rollovers (the g0 - win0 offsets, a window
    closing mid-call): the statistics and the analysis must equal the one-window run's."""
    from cwbl import synth
    w = synth.make("c2", seed=23, scale=0.1, nz=10)  # 30 x 30 x 10 = 9 000 points, k = 40
    runs = []
    for opts in ({}, {"max_batch": 256, "info_window": 256},
                 {"max_batch": 1000, "info_window": 2500}, {"info_window": 4096}):
        _cores.clear()
        c = abi.Core(w.k, device=0, options=opts)
        c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
        var = w.var.copy()
        st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
        c.finalize()
        runs.append((var, (st.points, st.solved, st.nobs_sum, st.max_p, st.lz_truncated,
                           st.nonconverged)))
    _cores.clear()
    assert runs[0][1][1] > 0
    for var, stats in runs[1:]:
        assert stats == runs[0][1]
        np.testing.assert_array_equal(var.view(np.uint32), runs[0][0].view(np.uint32))


def test_bin_div_option_applies_to_cached_trees():
    """CWBL_OPT_BIN_DIV set between two analyses of one obs set: the cached tree's bins are
    rebuilt for the new divisor (the cache is keyed by it), so the second call searches bins
    of r/1 and finds the same neighbour sets: equal solved / accepted-obs counts, increments
    equal up to the fp64 summation order of the new column order."""
    from cwbl import synth
    w = synth.make("c2", seed=29, scale=0.1, nz=10)
    _cores.clear()
    c = abi.Core(w.k, device=0)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    outs = []
    for div in (0, 1, 4, 0):
        c.set_option("bin_div", div)
        var = w.var.copy()
        st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
        outs.append((var, st.solved, st.nobs_sum, st.lz_truncated))
    c.finalize()
    _cores.clear()
    assert outs[0][1] > 0
    for var, *cnt in outs[1:]:
        assert cnt == list(outs[0][1:])
        assert increment_rel_rms(var, outs[0][0], w.var) <= 1e-10
    np.testing.assert_array_equal(outs[3][0].view(np.uint32), outs[0][0].view(np.uint32))


def test_tune_q_matches_reference():
    """letkf_tune_q on the device (cwbl_var_params.tune_q) against the reference's compiled
    letkf_tune_q (G5): bit for bit, including the Q3 NaN columns.  The single obs lies far
    outside the domain, so the analysis leaves var untouched and only tune_q acts."""
    g = golden("tune_q.npz")
    for i in range(int(g["ncases"])):
        k, q_in, q_out = int(g[f"k{i}"]), g[f"q_in{i}"], g[f"q_out{i}"]
        nx, ny, nz, _ = q_in.shape
        c = core(k)
        b = abi.ObsSetBuilder()
        far = np.array([[1e9, 1e9, 100.0]], np.float32)
        b.add_radar(abi.RADAR_VR, far, np.zeros(1, np.float32), np.zeros((1, k), np.float32))
        c.set_obs(b.build())
        tp = abi.type_params(use_it=1, max_lz_pts=100, hclr=12.0, vclr=3.0, err_muti=1.0,
                             err_rej=8.0)
        vp = abi.var_params(radar={abi.RADAR_VR: tp}, tune_q=1)
        var = np.ascontiguousarray(q_in.transpose(3, 2, 1, 0)).astype(np.float32)
        x = np.tile(np.arange(nx, dtype=np.float32) * 2e3, (ny, 1))
        y = np.tile((np.arange(ny, dtype=np.float32) * 2e3)[:, None], (1, nx))
        alt = np.tile((np.arange(nz, dtype=np.float32) * 500.0)[:, None, None], (1, ny, nx))
        slab = abi.make_slab(x, y, np.ascontiguousarray(alt), var)
        st = c.analyze_var(vp, slab)
        assert st.solved == 0 and st.ntrees == 1
        got = var.transpose(3, 2, 1, 0)
        np.testing.assert_array_equal(got.view(np.uint32), q_out.view(np.uint32))


def test_driver_with_tune_q_vs_oracle():
    """A Q-species variable: the analysis followed by tune_q, against the reference's
    analysis (G4) with the oracle's tune_q applied (itself pinned bit-exact by G5)."""
    import ctypes as C
    case = DriverCase("driver_mixed.npz")
    c = core(case.k, case.wf, case.norain)
    c.set_obs(case.obs_set())
    slab, var = case.slab()
    vp = case.vp
    vp.tune_q = 1
    c.analyze_var(vp, slab)
    vp.tune_q = 0
    ref = np.ascontiguousarray(case.var_out, np.float32).copy()
    k, nz, ny, nx = ref.shape
    oracle().orc_tune_q(k, nx, ny, nz, case.ix_lim, case.iy_lim, ref.ctypes.data_as(C.c_void_p))
    xb = np.ascontiguousarray(case.var_in, np.float32).copy()
    oracle().orc_tune_q(k, nx, ny, nz, case.ix_lim, case.iy_lim, xb.ctypes.data_as(C.c_void_p))
    rel = increment_rel_rms(var, ref, xb)
    assert rel <= INCR_TOL, rel


@pytest.mark.parametrize("k", [65, 80, 96, 101, 127, 128])
def test_large_k_random_batch_vs_oracle(k):
    """The 256-thread kernel (KP = 96 / 128) on seeded random batches, every k class of
    padding (k = KP, KP - 1, odd, just above 64): solve_batch vs the oracle's letkf_solve,
    p from 1 (rank-one Yb Yb^T, zero reflectors) to 300."""
    from helpers import oracle_solve
    rng = np.random.default_rng(20261016 + k)
    ps = [1, 2, 7, 40, 130, 300]
    col = np.concatenate([[0], np.cumsum(ps)]).astype(np.int64)
    yo = rng.normal(0, 1, col[-1]).astype(np.float32)
    yb = rng.normal(0, 1, (col[-1], k)).astype(np.float32)
    xb = rng.normal(5, 1, (len(ps), k)).astype(np.float32)
    inflat = inflat_of(k, np.float32(1.1))
    c = core(k)
    xa, _ = c.solve_batch(col, yo, yb.reshape(-1), xb, inflat, 1, 0.7, 1, 0.3)
    assert np.isfinite(xa).all()
    for i, p in enumerate(ps):
        ref, _ = oracle_solve(k, p, xb[i], yo[col[i]:col[i + 1]], yb[col[i]:col[i + 1]],
                              inflat, 1, 0.7, 1, 0.3, want_evals=False)
        rel = increment_rel_rms(xa[i], ref, xb[i])
        assert rel <= INCR_TOL, (p, rel)


@pytest.mark.parametrize("name", ["c2", "c2_far", "c5", "driver_mixed.npz", "driver_c1.npz"])
def test_binned_search_equals_tree_search(name):
    """The analysis search runs on uniform bins (search_binned_kernel) with the k-d tree as
    the fallback where max_lz truncates (Q4).  The neighbour SETS are identical, so the solved
    points, the accepted-obs counts and the truncation counts must match the tree search's
    exactly; the column order differs, which moves only the fp64 sums (increments to ~1e-12).
    driver_mixed has truncated lists (tree fallback), C5-shaped dense radar has ~1300
    neighbours per point."""
    from cwbl import synth
    if name.endswith(".npz"):
        case = DriverCase(name)
        mk = lambda o: (abi.Core(case.k, device=0, weight_function=case.wf,  # noqa: E731
                                 norain_value=case.norain, options=o), case.obs_set(), case.vp)
        slabs = lambda: case.slab()  # noqa: E731
        var_in = case.var_in
    else:
        w = synth.make(name[:2], scale=0.04 if name == "c5" else 0.12)
        if name == "c2_far":  # a domain 5000 km off the projection origin, 1.5 km localisation
            w.x = w.x + np.float32(5e6)
            w.y = w.y - np.float32(4e6)
            w.obs_xyz = w.obs_xyz + np.array([5e6, -4e6, 0.0], np.float32)
            for tp in w.vp.radar:
                tp.hclr = tp.hclr / 8.0
        ob = lambda: abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs,  # noqa: E731
                                                    w.hdxb).build()
        mk = lambda o: (abi.Core(w.k, device=0, options=o), ob(), w.vp)  # noqa: E731

        def slabs():
            var = w.var.copy()
            return abi.make_slab(w.x, w.y, w.alt, var), var
        var_in = w.var
    out = {}
    for mode in ("tree", "bins"):
        _cores.clear()
        c, obs, vp = mk({"search": int(mode == "tree")})
        c.set_obs(obs)
        slab, var = slabs()
        st = c.analyze_var(vp, slab)
        c.finalize()
        out[mode] = (var, st.solved, st.nobs_sum, st.lz_truncated, st.max_p)
    _cores.clear()
    assert out["tree"][1:] == out["bins"][1:], (out["tree"][1:], out["bins"][1:])
    if name == "driver_mixed.npz":
        assert out["bins"][3] > 0  # the fallback ran
    rel = increment_rel_rms(out["bins"][0], out["tree"][0], var_in)
    assert rel <= 1e-9, rel


@pytest.mark.parametrize("k,err,n_obs,tol", [(32, 2.0 ** -18, None, INCR_TOL),
                                             (16, 2.0 ** -19, None, INCR_TOL),
                                             (64, 2.0 ** -18, 120000, 2 * INCR_TOL),
                                             (128, 2.0 ** -19, 120000, INCR_TOL)])
def test_tiny_obs_errors_beyond_the_31_node_rule(k, err, n_obs, tol):
    """Obs errors of 2^-18 / 2^-19 put trace(A)/m above 1e12 (decades 13..14): the kernels
    switch to the 63-node rule (solve_tq40_kernel: 8 rounds; the one-wavefront kernels and the
    256-thread/tail pair: a second pass), where before round 3 such points were only counted
    as non-converged.  k = 32 runs the KP = 40 record path, 16 and 64 solve_tq_kernel, 128 the
    split big path.

    The reference itself is not accurate here: it forms Pa = V L^-1 V^T and multiplies it by
    Yb d (~1e13), so the rounding of Pa alone moves wbar by up to 1e-4..1e-3 of the increment
    (checked against 50-digit arithmetic).  The check is therefore against an fp64
    evaluation that applies the eigendecomposition to the two vectors directly
    (helpers.eigen_direct_solve, equal to 50-digit arithmetic to ~1e-15 on these points and
    bit-identical to the oracle in the ordinary regime, tests/test_truth.py), with the
    reference's columns and fp32 epilogue; the oracle's own deviation is in the message.  The
    cases are well posed (every ensemble direction the obs see is seen strongly: dense obs at
    k = 64, 128): where A also has moderate eigenvalues next to |A| ~ 1e14, every method that
    forms A in fp64 — the reference's, this core's, eigh's — is off by ~eps |A| / lambda.  At
    k = 64 (2^-18) that floor is ~1e-6: the core is within 1.03e-6 of the truth there (3x the
    fp32 rounding floor of the increments), the reference 1.5e-4, so that case's bound is
    2e-6."""
    import ctypes as C
    from cwbl import synth
    from helpers import eigen_direct_solve, pair_ensemble, radar_point_columns
    over = {} if n_obs is None else {"n_obs": n_obs}
    w = pair_ensemble(synth.make("c2", seed=13, scale=0.06, nz=4, k=k, **over), err)
    c = core(k)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    var = w.var.copy()
    st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
    assert st.max_sweeps > 12, st.max_sweeps          # the decade of the spectrum bound
    assert st.nonconverged == 0
    truth = w.var.copy()
    vp = w.vp
    infl = inflat_of(k, vp.multi_infl)
    nz, ny, nx = w.var.shape[1:]
    for kz in range(nz):
        for j in range(ny):
            for i in range(nx):
                yo, yb = radar_point_columns(w, kz, j, i, err)
                if len(yo):
                    truth[:, kz, j, i] = eigen_direct_solve(
                        k, w.var[:, kz, j, i], yo, yb, infl, vp.use_rtpp, vp.rtpp_alpha,
                        vp.use_rtps, vp.rtps_alpha)
    ref = w.var.copy()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    ost = abi.Stats()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(w.x, w.y, w.alt, ref)), 16, C.byref(ost))
    assert rc == 0
    assert st.solved == ost.solved > 0 and st.nobs_sum == ost.nobs_sum
    rel = increment_rel_rms(var, truth, w.var)
    rel_ref = increment_rel_rms(ref, truth, w.var)
    # the analyses are fp32: one ulp of xa at every point is this much of the increment, and
    # the fp64 values a point's fp32 epilogue rounds may differ by ~1e-13 relative
    upd = truth != w.var
    ulp = np.sqrt(np.mean(np.spacing(np.abs(truth[upd])).astype(np.float64) ** 2)) / \
        np.sqrt(np.mean((truth[upd].astype(np.float64) - w.var[upd]) ** 2))
    assert rel <= max(tol, ulp), (rel, ulp, rel_ref)


@pytest.mark.parametrize("k,emax", [(16, 24), (40, 24), (64, 24), (128, 24)])
def test_quadrature_on_an_exact_wide_spectrum(k, emax):
    """cwbl_solve_batch on a point whose A is diagonal and exact in fp64: column i of yb is
    2^e_i at member i (e_i spread over 0..emax), so A = inflat I + diag(4^e_i), the
    Householder steps are exact no-ops, T = A, and the analysis is known in closed form
    (wbar_i = s_i yo_i / lam_i, W x' = sqrt(k-1) x'_i / sqrt(lam_i)).  M/m reaches ~1e13..1e15,
    past the 31-node rule: the second pass of solve_tq_kernel (k <= 64) and
    solve_tq_big_kernel (k = 128) must reproduce the closed form to the fp32 output."""
    rng = np.random.default_rng(k)
    infl = inflat_of(k, 1.6)
    e = np.round(np.linspace(0, emax, k)).astype(int)
    rng.shuffle(e)
    sgn = rng.choice([-1.0, 1.0], k)
    yb = np.zeros((k, k), np.float32)
    yb[np.arange(k), np.arange(k)] = sgn * 2.0 ** e          # column i = member i
    yo = (np.round(rng.standard_normal(k) * 64) / 64).astype(np.float32)
    xb = (np.round((3.0 + rng.standard_normal(k)) * 256) / 256).astype(np.float32)
    lam = float(infl) + 4.0 ** e
    assert np.all(lam - 4.0 ** e == float(infl))               # exact in fp64
    s = np.float32(0.0)
    for v in xb:
        s = np.float32(s + v)
    xm = float(np.float32(s * np.float32(1.0 / k)))
    xp = xb.astype(np.float64) - xm
    wbar = np.diag(yb).astype(np.float64) * yo.astype(np.float64) / lam
    exact = (xm + (float(wbar @ xp) + np.sqrt(k - 1.0) * xp / np.sqrt(lam))).astype(np.float32)
    c = core(k)
    xa, ev = c.solve_batch(np.array([0, k], np.int64), yo, yb.ravel(), xb[None], infl, 0, 0.95,
                           0, 0.95, want_evals=True)
    np.testing.assert_allclose(ev[0], np.sort(lam), rtol=1e-14)
    assert np.max(np.abs(xa[0].astype(np.float64) - exact)) <= 2 * np.spacing(np.float32(8.0)), \
        (xa[0] - exact)
    assert increment_rel_rms(xa[0], exact, xb) <= INCR_TOL


def test_ingested_obs_set_analysis_vs_oracle():
    """The host ingest chain end to end: the reference-format files of tests/golden/ingest
    (three members' GTS and radar files, obs_gts) read by cwbl_ingest_* (pinned bit for bit
    against the reference's readers, tests/test_ingest.py), grid columns projected with
    cwbl_lonlat_to_xy, analysed on the GPU; the same inputs through the oracle."""
    import ctypes as C
    import os
    from cwbl import ingest
    from helpers import GOLDEN
    d = os.path.join(GOLDEN, "ingest")
    k = 3
    h = ingest.Ingest(k)
    for m in range(k):
        h.read_gts(os.path.join(d, f"gts_letkf_{m + 1:03d}"), os.path.join(d, "obs_gts"))
        h.read_radar(os.path.join(d, f"VR_letkf_{m + 1:03d}"), "VR")
        h.read_radar(os.path.join(d, f"MR_letkf_{m + 1:03d}"), "MR")
    ob = h.obs_set()
    nx, ny, nz = 14, 16, 6
    lon, lat = np.meshgrid(np.linspace(119.0, 123.0, nx, dtype=np.float32),
                           np.linspace(21.0, 26.0, ny, dtype=np.float32))
    x, y = ingest.lonlat_to_xy(lon.ravel(), lat.ravel())
    x, y = x.reshape(ny, nx), y.reshape(ny, nx)
    alt = np.ascontiguousarray(np.broadcast_to(np.linspace(0.0, 9000.0, nz, dtype=np.float32)
                                               [:, None, None], (nz, ny, nx)))
    rng = np.random.default_rng(3)
    var0 = (280.0 + rng.standard_normal((k, nz, ny, nx))).astype(np.float32)
    T = lambda hc, vc, ml, **kw: abi.type_params(use_it=1, max_lz_pts=ml, hclr=hc, vclr=vc,  # noqa: E731
                                                   **kw)
    vp = abi.var_params(multi_infl=1.6, use_rtpp=1, rtpp_alpha=0.95, use_rtps=1, rtps_alpha=0.95,
                        gts={abi.GTS_SOUND: T(150.0, 8.0, 100, err_muti=1.0, err_rej=8.0,
                                              is_assim=[1, 1, 1, 1]),
                             abi.GTS_SYNOP: T(150.0, 8.0, 100, err_muti=1.0, err_rej=8.0,
                                              is_assim=[1, 1, 1, 1, 1]),
                             abi.GTS_METAR: T(150.0, 8.0, 100, err_muti=1.0, err_rej=8.0,
                                              is_assim=[1, 1, 1, 1, 1]),
                             abi.GTS_SHIPS: T(150.0, 8.0, 100, err_muti=1.0, err_rej=8.0,
                                              is_assim=[1, 1, 1, 1, 1])},
                        radar={abi.RADAR_VR: T(120.0, 6.0, 300, err_muti=2.0, err_rej=20.0),
                               abi.RADAR_DBZ: T(120.0, 6.0, 300, err_muti=5.0, err_rej=20.0)})
    c = core(k)
    c.set_obs(ob)
    var = var0.copy()
    st = c.analyze_var(vp, abi.make_slab(x, y, alt, var))
    ref = var0.copy()
    ost = abi.Stats()
    rc = oracle().orc_analyze_var(k, 0, -5.0, 0, C.byref(ob), C.byref(vp),
                                  C.byref(abi.make_slab(x, y, alt, ref)), 4, C.byref(ost))
    assert rc == 0
    assert st.solved == ost.solved > 0 and st.nobs_sum == ost.nobs_sum
    rel = increment_rel_rms(var, ref, var0)
    assert rel <= INCR_TOL, rel


@pytest.mark.parametrize("tune_q", [0, 1])
@pytest.mark.parametrize("host", ["pageable", "pageable_bounce", "pinned"])
@pytest.mark.parametrize("staggered", [False, True])
def test_pipelined_host_slab_equals_device_slab(tune_q, host, staggered):
    """A host-memory slab whose analysed region is the whole horizontal slab moves var batch
    by batch (H2D before each batch's solve on its own stream, D2H behind each batch's last
    solve; with tune_q the copy back waits for the whole slab).  Pageable numpy arrays are
    page-locked in place for the call (hipHostRegister) or, with option pageable = 1, go
    through the library's page-locked bounce slots (host threads fill and drain them);
    page-locked ones (torch pin_memory) are copied directly.  A staggered slab (ix_lim < nx,
    the U variable's Q2 bounds) moves whole.  Bit-identical to the device-memory call, over
    many batches."""
    torch = pytest.importorskip("torch")
    opts = {"max_batch": 3000, "pageable": int(host == "pageable_bounce")}
    pinned = host == "pinned"
    _cores.clear()
    w = _radar_case_scaled(0.1, nz=12)
    vp = w.vp
    vp.tune_q = tune_q
    ix_lim = w.x.shape[1] - 1 if staggered else None
    c = abi.Core(w.k, device=0, options=opts)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    if pinned:
        t = torch.empty(w.var.shape, dtype=torch.float32, pin_memory=True)
        t.copy_(torch.from_numpy(w.var))
        hv = t.numpy()
    else:
        hv = w.var.copy()
    st = c.analyze_var(vp, abi.make_slab(w.x, w.y, w.alt, hv, ix_lim=ix_lim))
    dev = torch.device("cuda:0")
    x, y, alt, dv = (torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                     for a in (w.x, w.y, w.alt, w.var.copy()))
    c.analyze_var(vp, abi.make_slab(x, y, alt, dv, ix_lim=ix_lim, memory=abi.MEM_DEVICE))
    c.finalize()
    assert st.solved > 0
    np.testing.assert_array_equal(hv.view(np.uint32), dv.cpu().numpy().view(np.uint32))


def test_bounce_slots_after_repeated_init():
    """The bounce-slot path (option pageable = 1) right after finalize / init, three times:
    each Core's host worker threads start at the pool's current generation, so no worker runs
    a stale pass; every result bit-identical to the device-memory call."""
    torch = pytest.importorskip("torch")
    _cores.clear()
    w = _radar_case_scaled(0.1, nz=6)
    dev = torch.device("cuda:0")
    x, y, alt, dv = (torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                     for a in (w.x, w.y, w.alt, w.var.copy()))
    c = abi.Core(w.k, device=0)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    c.analyze_var(w.vp, abi.make_slab(x, y, alt, dv, memory=abi.MEM_DEVICE))
    c.finalize()
    want = dv.cpu().numpy().view(np.uint32)
    for _ in range(3):
        c = abi.Core(w.k, device=0, options={"max_batch": 2000, "pageable": 1})
        c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
        hv = w.var.copy()
        st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, hv))
        c.finalize()
        assert st.solved > 0
        np.testing.assert_array_equal(hv.view(np.uint32), want)


def test_set_option_ranges_and_reset():
    """cwbl_set_option: unknown options and out-of-range values are CWBL_ERR_ARG, the Jacobi
    solver past k = 64 is CWBL_ERR_UNSUPPORTED, and cwbl_init resets every option (the
    library reads no environment knob)."""
    _cores.clear()
    c = abi.Core(40, device=0)
    for opt, val in ((99, 0), (abi.OPT_SPLIT40, 2), (abi.OPT_BIG_BATCH, 8),
                     (abi.OPT_MAX_BATCH, 100), (abi.OPT_BIN_DIV, 9)):
        with pytest.raises(abi.CwblError, match="CWBL_ERR_ARG"):
            c.set_option(opt, val)
    c.set_option("max_batch", 0)
    c.finalize()
    c = abi.Core(128, device=0)
    with pytest.raises(abi.CwblError, match="CWBL_ERR_UNSUPPORTED"):
        c.set_option("solver", 1)
    c.finalize()
