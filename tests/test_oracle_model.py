"""Pin the oracle's HKD model restatement against the reference's own CasADi kernels.

Golden vectors: tests/golden/hkd_model_golden.npz (tests/golden/make_golden.py, generated from
oracle/_ref = the reference's CasadiGen sources compiled in place).  When oracle/_ref is present
(build container) the comparison also runs live on fresh random points.
Tolerance: 1e-12 relative to the largest entry (fp64 model arithmetic, different operation order).
"""
import numpy as np
import pytest

import oracle_lib as O

TOL = 1e-12


def _rel(a, b):
    return np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))


def test_step_matches_golden(golden):
    for q in range(golden["x"].shape[0]):
        xn = O.hkd_step(golden["x"][q], golden["u"][q], float(golden["dt"]), golden["c"][q])
        assert _rel(xn, golden["xn"][q]) < TOL


def test_partial_matches_golden(golden):
    for q in range(golden["x"].shape[0]):
        A, B = O.hkd_partial(golden["x"][q], golden["u"][q], float(golden["dt"]), golden["c"][q])
        assert _rel(A, golden["A"][q]) < TOL
        assert _rel(B, golden["B"][q]) < TOL
        # structural zeros (hkinodyn_par_casadi.cpp:177-178): B has <= 60 non-zeros
        assert np.count_nonzero(golden["B"][q]) <= 60
        assert np.array_equal(B == 0, golden["B"][q] == 0) or _rel(B, golden["B"][q]) < TOL


def test_foot_kinematics_match_golden(golden):
    import ctypes as C
    L = O.lib()
    for q in range(golden["fx"].shape[0]):
        x = golden["fx"][q]
        for leg in range(4):
            p = np.zeros(3)
            L.orc_foot_position(leg, O.dp(np.ascontiguousarray(x[3:6])), O.dp(np.ascontiguousarray(x[0:3])),
                                O.dp(np.ascontiguousarray(x[12 + 3 * leg:15 + 3 * leg])), O.dp(p))
            assert _rel(p, golden["fp"][q, leg]) < TOL
            J = np.zeros((3, 18))
            L.orc_foot_jacobian(leg, O.dp(np.ascontiguousarray(x[3:6])), O.dp(np.ascontiguousarray(x[0:3])),
                                O.dp(np.ascontiguousarray(x[12 + 3 * leg:15 + 3 * leg])), O.dp(J))
            assert _rel(J, golden["fJ"][q, leg]) < TOL
    del C


def test_resetmap_matches_golden(golden):
    for q in range(golden["rx"].shape[0]):
        xn = O.resetmap(golden["rx"][q], golden["rc"][q], golden["rcn"][q])
        Px = O.resetmap_partial(golden["rx"][q], golden["rc"][q], golden["rcn"][q])
        assert _rel(xn, golden["rxn"][q]) < TOL
        assert _rel(Px, golden["rPx"][q]) < TOL


def test_partial_is_derivative_of_step():
    """Finite-difference check of A and B (SURVEY §4 known-answer test 3.2)."""
    rng = np.random.default_rng(5)
    x = rng.uniform(-0.4, 0.4, 24); x[5] = 0.25
    u = rng.uniform(-20, 20, 24); c = np.array([1.0, 0.0, 1.0, 1.0])
    A, B = O.hkd_partial(x, u, 0.01, c)
    h = 1e-6
    for j in range(24):
        e = np.zeros(24); e[j] = h
        fa = (O.hkd_step(x + e, u, 0.01, c) - O.hkd_step(x - e, u, 0.01, c)) / (2 * h)
        fb = (O.hkd_step(x, u + e, 0.01, c) - O.hkd_step(x, u - e, 0.01, c)) / (2 * h)
        assert np.max(np.abs(fa - A[:, j])) < 1e-8
        assert np.max(np.abs(fb - B[:, j])) < 1e-8


def test_reset_partial_is_derivative_of_reset():
    """Px against finite differences of resetmap (z rows are zeroed by the reference's cmap)."""
    rng = np.random.default_rng(6)
    x = rng.uniform(-0.4, 0.4, 24); x[5] = 0.25
    c, cn = np.array([0, 1, 1, 0], np.int32), np.array([1, 1, 0, 0], np.int32)
    Px = O.resetmap_partial(x, c, cn)
    h = 1e-6
    for j in range(24):
        e = np.zeros(24); e[j] = h
        fd = (O.resetmap(x + e, c, cn) - O.resetmap(x - e, c, cn)) / (2 * h)
        assert np.max(np.abs(fd - Px[:, j])) < 1e-8


@pytest.mark.skipif(O.ref_lib() is None, reason="oracle/_ref needs /root/reference (build container only)")
def test_live_against_reference_kernels():
    R = O.ref_lib()
    rng = np.random.default_rng(77)
    for _ in range(50):
        x = rng.uniform(-0.7, 0.7, 24); x[5] = rng.uniform(0.1, 0.4)
        u = rng.uniform(-50, 50, 24); c = rng.integers(0, 2, 4).astype(float)
        a = np.zeros(24); R.ref_hkinodyn(O.dp(x), O.dp(u), 0.01, O.dp(c), O.dp(a))
        assert _rel(O.hkd_step(x, u, 0.01, c), a) < TOL
        A = np.zeros(576); B = np.zeros(576)
        R.ref_hkinodyn_par(O.dp(x), O.dp(u), 0.01, O.dp(c), O.dp(A), O.dp(B))
        Ao, Bo = O.hkd_partial(x, u, 0.01, c)
        assert _rel(Ao, A.reshape(24, 24).T) < TOL
        assert _rel(Bo, B.reshape(24, 24).T) < TOL
