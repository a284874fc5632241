"""Known-answer pins of the oracle's cost / constraint arithmetic (the reference
solver cannot execute here, so its restatement is pinned by what the reference's formulas imply):

* the running derivatives lx, lu, lxx, luu (and lux = 0) the oracle's LQ_approximation produces
  are the derivatives of its own compute_cost (SinglePhase.cpp:235-296) — central differences;
* the terminal Phix, Phixx are the derivatives of Phi where no augmented-Lagrangian term is
  active (no touchdown);
* the relaxed-barrier terms equal their closed forms on both branches g > delta and g <= delta
  (ConstraintsBase.h:204-263), the augmented-Lagrangian terms theirs, including quirk A4's
  Hessian (sigma (1 + h) + lambda) h_x h_x^T (ConstraintsBase.h:374-399);
* quirk A2: after a failed line search the working trajectory is the last trial
  (MultiPhaseDDP.cpp:345-353), so the next LQ_approximation runs there.

The evaluation unit is oracle/hsddp_oracle.c's orc_knot_eval: one knot and one phase end, run
through the same compute_cost / LQ_approximation code as the solve."""
import numpy as np
import pytest

import oracle_lib as O
from hsddp import synthetic as syn

DT = 0.01
MU = 0.7
GRF_ROWS = np.array([[0, 0, 1], [-1, 0, MU], [1, 0, MU], [0, -1, MU], [0, 1, MU]])  # HKDConstraints.cpp:7-66


def _state(contact, seed):
    rng = np.random.default_rng(seed)
    x = syn.initial_state(seed, contact)
    x[:12] += 0.05 * rng.standard_normal(12)
    x[12:] += 0.02 * rng.standard_normal(12)
    return x


def _control(contact, seed):
    """GRFs inside the friction pyramid with rows on both sides of delta = 0.1, joint velocities."""
    rng = np.random.default_rng(seed + 100)
    u = np.zeros(24)
    for lg in range(4):
        if contact[lg]:
            fz = rng.uniform(15, 30)
            u[3 * lg:3 * lg + 3] = [rng.uniform(-0.5, 0.5) * MU * fz, rng.uniform(-0.5, 0.5) * MU * fz, fz]
    u[12:] = 0.3 * rng.standard_normal(12)
    return u


def _refs(contact):
    rx, ru, rf = syn._reference_slots([contact, contact], [1])
    return rx[0], ru[0], rf[0]


CASES = [((1, 0, 0, 1), (0, 1, 1, 0), 1), ((1, 1, 1, 1), (1, 1, 1, 1), 2), ((0, 0, 0, 0), (0, 0, 0, 0), 3),
         ((1, 1, 0, 0), (0, 0, 1, 1), 4)]


def _fd(f, z, h):
    g = []
    for j in range(len(z)):
        zp, zm = z.copy(), z.copy()
        zp[j] += h; zm[j] -= h
        g.append((f(zp) - f(zm)) / (2 * h))
    return np.array(g)


@pytest.mark.parametrize("c,cn,seed", CASES)
def test_running_derivatives_are_derivatives_of_the_cost(c, cn, seed):
    x, u = _state(c, seed), _control(c, seed)
    xr, ur, pf = _refs(c)
    ev = lambda xx, uu: O.knot_eval(c, cn, xx, uu, xr, ur, pf)
    r = ev(x, u)
    lx_fd = _fd(lambda z: ev(z, u)["l"], x, 1e-6)
    lu_fd = _fd(lambda z: ev(x, z)["l"], u, 1e-6)
    assert np.allclose(r["lx"], lx_fd, rtol=1e-6, atol=1e-9)
    assert np.allclose(r["lu"], lu_fd, rtol=1e-6, atol=1e-9)
    lxx_fd = _fd(lambda z: ev(z, u)["lx"], x, 1e-5)
    luu_fd = _fd(lambda z: ev(x, z)["lu"], u, 1e-5)
    lux_fd = _fd(lambda z: ev(z, u)["lu"], x, 1e-5)
    assert np.allclose(r["lxx"], lxx_fd, rtol=1e-6, atol=1e-9)
    assert np.allclose(r["luu"], luu_fd, rtol=1e-6, atol=1e-9)
    assert np.all(r["lux"] == 0) and np.allclose(lux_fd, 0, atol=1e-12)
    # the LQ model's dynamics Jacobians are the derivatives of hkinodyn (HKDModel.h:33-61)
    cd = np.asarray(c, float)
    A_fd = _fd(lambda z: O.hkd_step(z, u, DT, cd), x, 1e-6).T
    B_fd = _fd(lambda z: O.hkd_step(x, z, DT, cd), u, 1e-6).T
    assert np.allclose(r["A"], A_fd, rtol=1e-6, atol=1e-9)
    assert np.allclose(r["B"], B_fd, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("c,seed", [((1, 0, 0, 1), 5), ((1, 1, 1, 1), 6), ((0, 0, 0, 0), 7)])
def test_terminal_derivatives_without_touchdown(c, seed):
    """No leg touches down at this phase end (cn = c): Phi is the tracking Qf term plus
    foot_term_cost times the foot regularisation (HKDCost.cpp:39-63), Phix / Phixx its derivatives."""
    x = _state(c, seed)
    xr, ur, pf = _refs(c)
    ev = lambda z: O.knot_eval(c, c, x, np.zeros(24), xr, ur, pf, x_end=z)
    r = ev(x)
    assert np.allclose(r["Phix"], _fd(lambda z: ev(z)["Phi"], x, 1e-6), rtol=1e-6, atol=1e-9)
    assert np.allclose(r["Phixx"], _fd(lambda z: ev(z)["Phix"], x, 1e-5), rtol=1e-6, atol=1e-9)


def _height_and_grad(x, leg):
    """Foot height h and its gradient h_x in state order (eul, pos, omega, v, qdummy): the
    reference's comp_foot_jacob z row, columns [pos | eul | qJ] (HKDConstraints.cpp:120-171)."""
    p = np.zeros(3)
    O.lib().orc_foot_position(leg, O.dp(np.ascontiguousarray(x[3:6])), O.dp(np.ascontiguousarray(x[0:3])),
                              O.dp(np.ascontiguousarray(x[12 + 3 * leg:15 + 3 * leg])), O.dp(p))
    J = np.zeros(54)
    O.lib().orc_foot_jacobian(leg, O.dp(np.ascontiguousarray(x[3:6])), O.dp(np.ascontiguousarray(x[0:3])),
                              O.dp(np.ascontiguousarray(x[12 + 3 * leg:15 + 3 * leg])), O.dp(J))
    J = J.reshape(3, 18)  # row-major 3 x 18: [pos | eul | qJ]
    hx = np.zeros(24)
    hx[0:3], hx[3:6], hx[12:] = J[2, 3:6], J[2, 0:3], J[2, 6:]
    return p[2], hx


@pytest.mark.parametrize("sigma,lam", [(50.0, 0.0), (120.0, 3.5), (1e4, -2.0)])
def test_al_terms_closed_form(sigma, lam):
    """Touchdown of legs 1 and 2 (c = 1001 -> cn = 1111): the augmented-Lagrangian terms of
    SinglePhase::update_terminal_cost(_par)_with_tconstr (SinglePhase.cpp:401-426) equal
    1/2 sigma h^2 + lambda h, (sigma h + lambda) h_x and — quirk A4 (ConstraintsBase.h:397) —
    (sigma (1 + h) + lambda) h_x h_x^T, per touchdown leg."""
    c, cn = (1, 0, 0, 1), (1, 1, 1, 1)
    x = _state((1, 0, 0, 1), 11)
    xr, ur, pf = _refs(c)
    sg, lm = np.full(4, sigma), np.full(4, lam)
    on = O.knot_eval(c, cn, x, np.zeros(24), xr, ur, pf, sigma=sg, lam=lm)
    off = O.knot_eval(c, cn, x, np.zeros(24), xr, ur, pf, sigma=sg, lam=lm, options=O.default_options(AL_active=0))
    phi = np.zeros(()); phix = np.zeros(24); phixx = np.zeros((24, 24))
    for leg in (1, 2):
        h, hx = _height_and_grad(x, leg)
        phi = phi + 0.5 * sigma * h * h + lam * h
        phix += (sigma * h + lam) * hx
        phixx += (sigma * (1 + h) + lam) * np.outer(hx, hx)
    assert abs((on["Phi"] - off["Phi"]) - phi) <= 1e-12 * max(1.0, abs(phi))
    assert np.allclose(on["Phix"] - off["Phix"], phix, rtol=1e-12, atol=1e-12)
    assert np.allclose(on["Phixx"] - off["Phixx"], phixx, rtol=1e-12, atol=1e-12)
    # ... which is not the exact Hessian sigma h_x h_x^T + (sigma h + lambda) h_xx (the quirk is kept)
    exact_fd = _fd(lambda z: O.knot_eval(c, cn, x, np.zeros(24), xr, ur, pf, x_end=z, sigma=sg, lam=lm)["Phix"]
                   - O.knot_eval(c, cn, x, np.zeros(24), xr, ur, pf, x_end=z, sigma=sg, lam=lm,
                                 options=O.default_options(AL_active=0))["Phix"], x, 1e-6)
    h1, hx1 = _height_and_grad(x, 1)
    assert not np.allclose(on["Phixx"] - off["Phixx"], exact_fd, rtol=1e-3, atol=1e-6) or abs(h1) < 1e-12


def _reb(g, delta):
    if g > delta:
        return -np.log(g), -1.0 / g, 1.0 / g ** 2
    t = (g - 2 * delta) / delta
    return 0.5 * (t * t - 1) - np.log(delta), (g - 2 * delta) / delta ** 2, 1.0 / delta ** 2


@pytest.mark.parametrize("delta,eps", [(0.1, 0.1), (2.0, 0.5), (8.0, 1.0)])
def test_reb_terms_closed_form(delta, eps):
    """GRF friction-pyramid rows g = A f (HKDConstraints.cpp:7-66) under the relaxed barrier
    (ConstraintsBase.h:204-263): dt * sum eps * B(g) into l, dt * eps * B'(g) A^T into lu and
    dt * eps * B''(g) A^T A into luu, for stance legs — with deltas that put rows on both branches."""
    c = (1, 1, 0, 1)
    x, u = _state(c, 21), _control(c, 21)
    u[3:6] = [1.0, -0.5, 3.0]  # leg 1: small normal force, rows below delta = 2, 8
    xr, ur, pf = _refs(c)
    d, e = np.full(20, delta), np.full(20, eps)
    on = O.knot_eval(c, c, x, u, xr, ur, pf, reb_delta=d, reb_eps=e)
    off = O.knot_eval(c, c, x, u, xr, ur, pf, reb_delta=d, reb_eps=e, options=O.default_options(ReB_active=0))
    l = 0.0; lu = np.zeros(24); luu = np.zeros((24, 24)); branches = set()
    for lg in range(4):
        if not c[lg]:
            continue
        f = u[3 * lg:3 * lg + 3]
        for row in GRF_ROWS:
            g = float(row @ f)
            b0, b1, b2 = _reb(g, delta)
            branches.add(g > delta)
            l += eps * b0
            lu[3 * lg:3 * lg + 3] += eps * b1 * row
            luu[3 * lg:3 * lg + 3, 3 * lg:3 * lg + 3] += eps * b2 * np.outer(row, row)
    assert branches == {True, False} or delta == 0.1
    assert abs((on["l"] - off["l"]) - DT * l) <= 1e-12 * max(1.0, abs(DT * l))
    assert np.allclose(on["lu"] - off["lu"], DT * lu, rtol=1e-12, atol=1e-14)
    assert np.allclose(on["luu"] - off["luu"], DT * luu, rtol=1e-12, atol=1e-14)


def test_failed_line_search_keeps_the_last_trial():
    """Quirk A2 (MultiPhaseDDP.cpp:345-353): gamma = 1e6 rejects every trial; after the iteration
    Xbar / Ubar are unchanged and the working X / U are the last trial (eps = 0.001,
    X = Xbar + eps dX at every shooting state, U = Ubar + eps dU + K (X - Xbar)) — the point the
    next LQ_approximation linearises about."""
    prob = syn.make_batch(2, 2, 8, "trot")
    o0 = O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=0)
    r0 = O.solve_batch(prob, o0)
    o1 = O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1, gamma=1e6)
    r1 = O.solve_batch(prob, o1)
    assert np.all(r1["n_ls_trials"] == 4) and np.all(r1["status"] == 0)
    assert np.array_equal(r1["Xbar"], r0["Xbar"]) and np.array_equal(r1["Ubar"], r0["Ubar"])
    eps = 0.1 ** 3
    assert np.array_equal(r1["X"], r1["Xbar"] + eps * r1["dX"])
    dx = r1["X"] - r1["Xbar"]
    S = prob["S"]
    kc = 0
    for i, N in enumerate(prob["horizons"]):
        s0 = sum(n + 1 for n in prob["horizons"][:i])
        for k in range(N):
            u = r1["Ubar"][:, kc] + eps * r1["dU"][:, kc] + np.einsum("bij,bj->bi", r1["K"][:, kc], dx[:, s0 + k])
            assert np.allclose(r1["U"][:, kc], u, rtol=1e-14, atol=1e-14)
            kc += 1
    assert S == dx.shape[1]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_riccati_recursion_converges_to_the_dare_solution(seed):
    """Outside pin of the Riccati recursion (SinglePhase.cpp:298-367): on
    time-invariant LQ data the oracle's backward sweep, run long enough, reaches the discrete
    algebraic Riccati solution scipy computes independently — H[0] -> P and K[0] -> -(R + B^T P B)^-1
    B^T P A, with dU[0], G[0] -> 0 for zero gradients.  The system has 24 states and 24 controls,
    open-loop unstable (spectral radius 1.05), dense."""
    la = pytest.importorskip("scipy.linalg")
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((24, 24))
    A *= 1.05 / np.max(np.abs(np.linalg.eigvals(A)))
    B = rng.standard_normal((24, 24)) / 5
    M = rng.standard_normal((24, 24))
    Q = M @ M.T / 24 + np.eye(24)
    N2 = rng.standard_normal((24, 24))
    R = N2 @ N2.T / 24 + 0.5 * np.eye(24)
    P = la.solve_discrete_are(A, B, Q, R)
    Kd = -np.linalg.solve(R + B.T @ P @ B, B.T @ P @ A)
    ok, K0, dU0, G0, H0 = O.riccati_lq(400, A, B, Q, R)
    assert ok
    assert np.max(np.abs(H0 - P)) / np.max(np.abs(P)) <= 1e-10
    assert np.max(np.abs(K0 - Kd)) / np.max(np.abs(Kd)) <= 1e-10
    assert np.all(dU0 == 0) and np.all(G0 == 0)
    # one knot from the DARE solution is its fixed point (P, Kd as terminal data)
    ok1, K1, _, _, H1 = O.riccati_lq(1, A, B, Q, R, Phixx=P)
    assert ok1 and np.max(np.abs(H1 - P)) / np.max(np.abs(P)) <= 1e-10
    assert np.max(np.abs(K1 - Kd)) / np.max(np.abs(Kd)) <= 1e-10
