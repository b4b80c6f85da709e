"""The two-stage k = 128 design (band_head_kernel / band_tail_kernel, CWBL_OPT_BIG_PATH = 2) on
the CPU: scripts/two_stage_b8.py restates the kernels' panels, chase schedule, storage bounds
and application orders in numpy.  These tests pin that restatement against numpy's
eigendecomposition and check the schedule's invariants that the tail kernel relies on (two
tasks per round at most, one per slot parity; sweeps three tasks apart; the constexpr plan's
586 rounds)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "scripts"))
import two_stage_b8 as ts  # noqa: E402


def _case(k, p, seed):
    rng = np.random.default_rng(seed)
    y = rng.standard_normal((k, p)) * np.exp(rng.uniform(-3, 3, p))
    a = np.eye(ts.N)
    a[:k, :k] = (k - 1) / 1.1 * np.eye(k) + y @ y.T  # identity padding past k
    b1 = np.zeros(ts.N)
    xp = np.zeros(ts.N)
    b1[:k] = rng.standard_normal(k)
    xp[:k] = rng.standard_normal(k)
    return a, b1, xp


def test_schedule_invariants():
    rounds, start = ts.schedule()
    assert len(rounds) == 586  # cwbl_band.h: kChase.rounds
    assert sum(len(r) for r in rounds) == 1056  # BandRec::NTASK
    for r in rounds:
        assert len(r) <= 2
        assert len({j % 2 for j, _ in r}) == len(r)  # one task per slot (sweep parity)
        if len(r) == 2:  # tasks of a round touch disjoint rows (16-row windows, >= 3 tasks apart)
            (j0, t0), (j1, t1) = sorted(r)
            r0, r1 = j0 + 1 + 8 * t0, j1 + 1 + 8 * t1
            assert abs(r0 - r1) >= 16, r
    for j in range(1, 126):
        assert start[j] >= start[j - 1] + 3  # sweep j + 1 three tasks behind sweep j


@pytest.mark.parametrize("k,p", [(128, 216), (128, 40), (100, 300), (97, 60)])
def test_two_stage_matches_eigh(k, p):
    a, b1, xp = _case(k, p, seed=k + p)
    u1, u2 = b1.copy(), xp.copy()
    bm, panels = ts.stage1(a, u1, u2)
    assert np.max(np.abs(np.tril(bm, -ts.B - 1))) == 0.0  # band of half-bandwidth 8
    rounds, _ = ts.schedule()
    tm, refl = ts.stage2(bm, rounds)  # asserts nothing is stored below d = 15
    d, e = np.diag(tm), np.diag(tm, -1)
    t = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    assert np.max(np.abs(tm - t)) <= 1e-14 * np.max(np.abs(a))
    # Q2^T on u sweep by sweep, the quantities the kernels form, and back through Q2, Q1
    sweeps = sorted({j for (j, _) in refl})
    for j in sweeps:
        for tt in range(ts.n_tasks(j)):
            r, v, tau = refl[(j, tt)]
            for u in (u1, u2):
                u[r:r + len(v)] -= tau * v * (v @ u[r:r + len(v)])
    w, uu = np.linalg.eigh(t)
    y = uu @ ((uu.T @ u2) / np.sqrt(w))
    dd = u1 @ (uu @ ((uu.T @ u2) / w))
    for j in reversed(sweeps):
        for tt in range(ts.n_tasks(j)):
            r, v, tau = refl[(j, tt)]
            y[r:r + len(v)] -= tau * v * (v @ y[r:r + len(v)])
    for r0, v, tp in reversed(panels):
        y[r0:] -= v @ (tp @ (v.T @ y[r0:]))
    wa, ua = np.linalg.eigh(a)
    y_ref = ua @ ((ua.T @ xp) / np.sqrt(wa))
    d_ref = b1 @ (ua @ ((ua.T @ xp) / wa))
    assert np.max(np.abs(np.linalg.eigvalsh(t) - wa) / wa) < 1e-12
    assert np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref) < 1e-12
    assert abs(dd - d_ref) / abs(d_ref) < 1e-12
