"""Known-answer tests that pin the oracle's HS-DDP restatement (solver-level parity has no
executable reference: the reference solver needs Eigen/Boost/LCM, absent here — SURVEY §8c).

* the oracle's first backward sweep + linear rollout equals an independent dense numpy Riccati
  (tests/numpy_riccati.py, numpy.linalg.inv) on the same LQ data, multi-phase with resets,
  ReB path constraints and AL touchdown constraints — tolerance 1e-9 relative;
* line-search step sequence: `while (eps > 1e-3) eps *= 0.1` runs four trials in binary64;
* solver-level regressions: deterministic, cost decreases, converged elements satisfy the
  reference's own termination tests.
"""
import numpy as np
import pytest

import numpy_riccati as NR
import oracle_lib as O
from hsddp import synthetic as syn


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


@pytest.mark.parametrize("gait,P,N", [("trot", 2, 12), ("jump", 3, 8), ("pronk", 2, 10)])
def test_first_sweep_matches_numpy_riccati(gait, P, N):
    prob = syn.make_batch(2, P, N, gait)
    opt = O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1)
    r = O.solve_batch(prob, opt)
    for b in range(2):
        X, U, D = NR.initial_rollout(prob, b)
        ref = NR.sweep(prob, b, X, U, D)
        assert _rel(r["K"][b], ref["K"]) < 1e-9
        assert _rel(r["dU"][b], ref["dU"]) < 1e-9
        # dX of the oracle is the linear rollout (eps = 1)
        assert _rel(r["dX"][b], ref["dX"]) < 1e-9


def test_line_search_step_sequence():
    eps, seq = 1.0, []
    while eps > 1e-3:
        seq.append(eps)
        eps *= 0.1
    assert len(seq) == 4  # 0.1**3 rounds to 0.0010000000000000002 > 1e-3


def test_oracle_deterministic_and_descending():
    prob = syn.make_batch(3, 4, 20, "trot")
    o = O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1)
    c1 = O.solve_batch(prob, o)["cost"]
    o5 = O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=5)
    r1 = O.solve_batch(prob, o5); r2 = O.solve_batch(prob, o5, n_threads=3)
    assert np.array_equal(r1["Xbar"], r2["Xbar"]) and np.array_equal(r1["cost"], r2["cost"])
    assert np.all(r1["cost"] <= c1 + 1e-12)


def test_converged_elements_meet_reference_tests():
    prob = syn.make_batch(4, 4, 30, "trot")
    r = O.solve_batch(prob, O.default_options(), n_threads=4)
    o = O.default_options()
    for b in range(4):
        if r["outer_iters"][b] < o.max_AL_iter:  # stopped by a test, not by the budget
            assert r["feas"][b] <= o.dynamics_feas_thresh
    assert np.all(r["status"] == 0)


def test_new_problem_rollout_break_keeps_zero_constraint_values():
    """Oracle restatement of a new problem's first rollout breaking at knot k (SinglePhase.cpp:
    205-208): the GRF values of the knots from k on stay zero (create_data) while the trial's
    control rows there are the warm start's, so the stored values differ from A U exactly there."""
    import divergence_case as DC
    prob, breaks, T, es = DC.make_init("trot", 2, 12, 4)
    r = O.solve_batch(prob, O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=0), n_threads=4)
    for b, j in enumerate(breaks):
        assert r["diverged_init"][b] == (j >= 0)
        stale = DC.stale_knots(prob, r["U"], r["grf_g"], b)
        if j < 0:
            assert stale == []
            continue
        # the initial rollout only: the break knot (state slot j + 1's control) and every later
        # stance knot keep zero values
        assert len(stale) > 8 and stale[0] == j and all(not r["grf_g"][b, kc].any() for kc in stale)
