"""CPU tests of the inverse-square-root quadrature tables of the tridiagonal solve kernel
(csrc/quad_tables.cpp, used by csrc/cwbl_tq.hip).  The tables are host code inside
libcwbl.so; no GPU is needed.

The rule: x^-1/2 ~= sum_j w_j / (t2_j + x) for x in [1, 10^L] (31 nodes, level L).  The
kernel uses it on A/m with m = (k-1)/infl, whose spectrum lies in [1, trace(A)/m - (k-1)].
"""
import ctypes as C

import numpy as np
import pytest

from cwbl import abi


@pytest.fixture(scope="module")
def lib():
    return abi.load_library()


def table(lib, level, n=31):
    buf = np.zeros(128)  # kQuadStride (t2, w) pairs
    p = buf.ctypes.data_as(C.POINTER(C.c_double))
    if n == 31:
        assert lib.cwbl_debug_quad_table(level, p) == 0
    else:
        assert lib.cwbl_debug_quad_table_n(level, n, p) == 0
    assert np.all(buf.reshape(64, 2)[n:] == 0.0)
    return buf.reshape(64, 2)[:n, 0], buf.reshape(64, 2)[:n, 1]


def rule_error(t2, w, level):
    lam = np.geomspace(1.0, 10.0 ** level, 20000)
    approx = (w[None, :] / (t2[None, :] + lam[:, None])).sum(1)
    return np.max(np.abs(approx * np.sqrt(lam) - 1.0))


# relative accuracy the kernel relies on, per decade of the spectrum (31 nodes: levels 1..12)
BOUND = {1: 2e-15, 2: 2e-15, 3: 2e-15, 4: 2e-15, 5: 4e-15, 6: 2e-14, 7: 1e-13, 8: 5e-12,
         9: 1e-10, 10: 1e-9, 11: 5e-9, 12: 2e-8}


@pytest.mark.parametrize("level", sorted(BOUND))
def test_rule_accuracy(lib, level):
    t2, w = table(lib, level)
    assert np.all(t2 > 0) and np.all(w > 0) and np.all(np.diff(t2) > 0)
    err = rule_error(t2, w, level)
    assert err <= BOUND[level], err


# solve_tq40_kernel runs 8 R - 1 nodes (R = quad_rounds(level), cwbl_internal.h: 2 rounds up to
# level 3, 3 to level 5, 4 to level 12, 8 above) with the exact T^-1 solve in the last slot; a
# wave runs the largest R its four points need, each point with its own level's table, so a
# point can run a longer rule than its level needs.  Every short rule a level can run stays
# within 1e-12 relative error (as the 31-node rule does to level 7).
SHORT = {(1, 15): 1e-15, (2, 15): 1e-15, (3, 15): 5e-13, (1, 23): 2e-15, (2, 23): 2e-15,
         (3, 23): 2e-15, (4, 23): 2e-15, (5, 23): 2e-13, (1, 63): 2e-15, (2, 63): 2e-15,
         (3, 63): 2e-15, (5, 63): 2e-15}


@pytest.mark.parametrize("level,n", sorted(SHORT))
def test_short_rules_accuracy(lib, level, n):
    t2, w = table(lib, level, n)
    assert np.all(t2 > 0) and np.all(w > 0) and np.all(np.diff(t2) > 0)
    err = rule_error(t2, w, level)
    assert err <= SHORT[(level, n)], err


def test_quad_rounds_stay_within_1e12():
    """The rounds solve_tq40_kernel runs at each level (quad_rounds): every rule a wave can hand
    a point of levels 1..7 (its own R or a larger one) is within 1e-12 (above, the 31-node
    rule's own BOUND governs)."""
    rounds = lambda L: 2 if L <= 3 else 3 if L <= 5 else 4 if L <= 12 else 8  # noqa: E731
    lib_ = abi.load_library()
    for L in range(1, 8):
        for R in sorted({2, 3, 4, 8} & set(range(rounds(L), 9))):
            err = rule_error(*table(lib_, L, 8 * R - 1), L)
            assert err <= 1e-12, (L, R, err)


# above level kQuadLevels31 (12) the one-wavefront kernels run a second pass (63 nodes) and
# solve_tq40_kernel 8 rounds: spectrum bounds up to 10^24 stay far inside the parity tolerance
# (before round 3 these points were only counted as non-converged)
@pytest.mark.parametrize("level", list(range(4, 25, 2)))
def test_63_node_rule_accuracy(lib, level):
    t2, w = table(lib, level, 63)
    assert np.all(t2 > 0) and np.all(w > 0) and np.all(np.diff(t2) > 0)
    err = rule_error(t2, w, level)
    assert err <= (3e-15 if level <= 12 else 5e-9), err


def test_bad_level_rejected(lib):
    buf = np.zeros(128)
    p = buf.ctypes.data_as(C.POINTER(C.c_double))
    assert lib.cwbl_debug_quad_table(0, p) != 0
    assert lib.cwbl_debug_quad_table(25, p) != 0
    assert lib.cwbl_debug_quad_table_n(2, 64, p) != 0


def test_matrix_function_on_spd_tridiagonal(lib):
    """sum_j w_j (T + s_j I)^-1 u on a random SPD tridiagonal equals T^-1/2 u (eigh)."""
    rng = np.random.default_rng(3)
    n = 40
    d = rng.uniform(30, 900, n)
    e = rng.uniform(-100, 100, n - 1)
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    lam, V = np.linalg.eigh(T)
    assert lam[0] > 0
    m = lam[0] * 0.9
    level = int(np.ceil(np.log10(lam[-1] / m)))
    t2, w = table(lib, level)
    u = rng.normal(size=n)
    y = sum(np.sqrt(m) * wj * np.linalg.solve(T + m * tj * np.eye(n), u) for tj, wj in zip(t2, w))
    ref = V @ ((V.T @ u) / np.sqrt(lam))
    assert np.max(np.abs(y - ref)) <= 1e-13 * np.max(np.abs(ref))
