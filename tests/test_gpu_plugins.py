"""The HKD cost / constraint plugins on the device (C-ABI hsddp_hkd_running_cost / _terminal_cost /
_grf_constraint / _touchdown_constraint — the bodies of the C++ facade's hkd:: CostBase,
PathConstraintBase and TerminalConstraintBase plugins) against the oracle's knot evaluation.

The reference splits a knot's cost over plugins (HKDTrackingCost + HKDFootPlaceReg running costs,
HKDCost.h:8-99; the GRF constraint's relaxed barrier added by SinglePhase, ConstraintsBase.h:
201-263 / SinglePhase.cpp:380-394); the oracle (orc_knot_eval) evaluates the sum, so the plugin
terms plus the barrier assembled here from the plugin's g, gu must equal it."""
import numpy as np
import pytest

import hsddp
import oracle_lib as O
from hsddp import model
from test_oracle_pinning import CASES, _control, _refs, _state, _height_and_grad

DT = 0.01


def _close(a, b, tol=1e-12):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) <= tol * max(1.0, np.max(np.abs(b)))


@pytest.mark.gpu
@pytest.mark.parametrize("c,cn,seed", CASES)
def test_running_plugins_sum_to_the_oracle_knot(c, cn, seed):
    x, u = _state(c, seed), _control(c, seed)
    xr, ur, pf = _refs(c)
    r = O.knot_eval(c, cn, x, u, xr, ur, pf)
    rc = {k: v[0] for k, v in model.running_cost(x, u, c, xr, ur, pf).items()}
    track = {k: v[0] for k, v in model.running_cost(x, u, c, xr, ur, pf, terms=model.TERM_TRACKING).items()}
    foot = {k: v[0] for k, v in model.running_cost(x, u, c, xr, ur, pf, terms=model.TERM_FOOT).items()}
    for k in ("lx", "lu", "lxx", "luu"):   # the terms are additive (RCostData::add)
        assert _close(track[k] + foot[k], rc[k], 1e-15), k
    g, gu = model.grf_constraint(u, c)
    n = 5 * int(sum(c))
    cp = hsddp.load_constraint_params()
    delta, eps = cp.grf_delta, cp.grf_eps
    barr = bd = 0.0
    lu, luu = rc["lu"].copy(), rc["luu"].copy()
    rb = 0.0
    for i in range(n):
        gi = g[0, i]
        if gi > delta:
            b, d1, d2 = -np.log(gi), -1.0 / gi, gi ** -2.0
        else:
            t = (gi - 2 * delta) / delta
            b, d1, d2 = .5 * (t * t - 1) - np.log(delta), (gi - 2 * delta) / delta / delta, delta ** -2.0
        rb += eps * b
        lu += DT * eps * d1 * gu[0, i]
        luu += DT * eps * d2 * np.outer(gu[0, i], gu[0, i])
    assert np.all(g[0, n:] == 0) and np.all(gu[0, n:] == 0)
    l = rc["l"] + (DT * rb if n else 0.0)
    assert _close(l, r["l"], 1e-13)
    assert _close(rc["lx"], r["lx"]) and _close(rc["lxx"], r["lxx"])
    assert _close(lu, r["lu"]) and _close(luu, r["luu"])


@pytest.mark.gpu
@pytest.mark.parametrize("c,seed", [((1, 0, 0, 1), 5), ((1, 1, 1, 1), 6), ((0, 0, 0, 0), 7)])
def test_terminal_plugins_match_the_oracle(c, seed):
    x = _state(c, seed)
    xr, ur, pf = _refs(c)
    r = O.knot_eval(c, c, x, np.zeros(24), xr, ur, pf, x_end=x)   # no touchdown: no AL terms
    t = {k: v[0] for k, v in model.terminal_cost(x, c, xr, pf).items()}
    assert _close(t["Phi"], r["Phi"], 1e-13)
    assert _close(t["Phix"], r["Phix"]) and _close(t["Phixx"], r["Phixx"])


@pytest.mark.gpu
def test_touchdown_plugin_matches_foot_kinematics():
    c, cn = (1, 0, 0, 1), (1, 1, 1, 1)    # legs 1 and 2 touch down
    x = _state(c, 11)
    h, hx = model.touchdown_constraint(x, c, cn, ground=0.0)
    for row, leg in enumerate((1, 2)):
        hr, hxr = _height_and_grad(x, leg)
        assert _close(h[0, row], hr, 1e-13) and _close(hx[0, row], hxr, 1e-13)
    assert np.all(h[0, 2:] == 0) and np.all(hx[0, 2:] == 0)
