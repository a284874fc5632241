"""The rollout divergence guard on the GPU against the oracle.

SinglePhase::hybrid_rollout returns at the first knot whose simulated state's 2-norm exceeds 1e6
(SinglePhase.cpp:205-208) and MultiPhaseDDP::hybrid_rollout skips the later phases (:83-87): X past
the break state, U past the break knot and the Defect of the break phase on keep the previous
trial's rows, the break knot's GRF constraint values stay those of its earlier control row, the
trial's cost and feasibility are sums over those mixed rows (:116-117), max_tconstr / max_pconstr
cover the phases before the break, and the trial is rejected (:127).  After a search whose last
trial diverged, quirk A2 carries the mixed rows, that feasibility and those constraint values into
the next inner iteration's cost, LQ model and merit.

Batches (tests/divergence_case.py): elements translated along x (an exact symmetry of the HKD
model) until the bound lies between two step sizes' largest simulated-state norms — "one": the
eps = 1 trial breaks and a later one is accepted; "all": every trial breaks (the search fails);
"none": no trial breaks.  jump 4 x 8 breaks in phase 0 (every later phase keeps its rows; no phase
before the break: max constraint violations 0); trot breaks in the last phase.

Tolerance: translated elements carry state entries of ~6e5, whose rounding (1e-10) the two
implementations place differently: rows are compared with the translation removed, to
max(1e-9 of their scale, 10x the oracle's own deviation under a 1e-15 relative x0 perturbation);
every branch decision (trial counts, statuses) exactly.
"""
import numpy as np
import pytest

import divergence_case as DC
import hsddp
import oracle_lib as O

pytestmark = pytest.mark.gpu


def _gpu(prob, ms, **kw):
    s = hsddp.Solver(prob, hsddp.load_settings(MS=ms, **kw))
    s.solve()
    out = {**s.trajectory(), **s.working(), **s.element_info()}
    s.close()
    return out


def _close(g, r, r2, tol=1e-9):
    scale = max(1.0, float(np.max(np.abs(r))))
    env = float(np.max(np.abs(r2 - r)))
    return float(np.max(np.abs(g - r))), max(tol * scale, 10 * env)


CASES = [("trot", 2, 10, 8), ("trot", 4, 12, 8), ("jump", 4, 8, 24)]


@pytest.mark.parametrize("n_iter", [1, 2, 3])
@pytest.mark.parametrize("gait,P,N,B", CASES)
def test_divergence_matches_oracle(gait, P, N, B, n_iter):
    prob, kinds, T, es = DC.make(gait, P, N, B)
    assert kinds.count("one") >= 1 and kinds.count("all") >= 1, kinds
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=n_iter)
    g = _gpu(prob, 1, **kw)
    r = O.solve_batch(prob, O.default_options(**kw), n_threads=8)
    p2 = dict(prob); p2["x0"] = prob["x0"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(**kw), n_threads=8)
    if n_iter == 1:  # the scenario the batch was built for
        for b, k in enumerate(kinds):
            assert r["n_ls_trials"][b] == {"none": r["n_ls_trials"][b], "one": 2, "all": 4}[k], (b, k)
    for f in ("iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f], r[f]), f
    for f in ("Xbar", "X", "dX"):
        tr = (lambda a: a) if f == "dX" else (lambda a: DC.untranslate(a, T, es))  # noqa: E731
        err, tol = _close(tr(g[f]), tr(r[f]), tr(r2[f]))
        assert err <= tol, (f, err, tol)
    for f in ("Ubar", "U", "K", "dU"):
        err, tol = _close(g[f], r[f], r2[f])
        assert err <= tol, (f, err, tol)
    for f in ("cost", "feas", "merit", "max_tconstr", "max_pconstr"):
        err, tol = _close(g[f], r[f], r2[f])
        assert err <= tol, (f, err, tol)


@pytest.mark.parametrize("gait,P,N,B", CASES[:1] + CASES[2:])
def test_divergence_single_shooting_matches_oracle(gait, P, N, B):
    """The same batches with MS 0: single-shot chains break where their own states cross the bound
    (the rows past the break are then the previous trial's, whatever the chain computed there)."""
    prob, kinds, T, es = DC.make(gait, P, N, B)
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2)
    g = _gpu(prob, 0, **kw)
    kw["MS"] = 0
    r = O.solve_batch(prob, O.default_options(**kw), n_threads=8)
    p2 = dict(prob); p2["x0"] = prob["x0"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(**kw), n_threads=8)
    for f in ("iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f], r[f]), f
    for f in ("Xbar", "X"):
        err, tol = _close(DC.untranslate(g[f], T, es), DC.untranslate(r[f], T, es), DC.untranslate(r2[f], T, es))
        assert err <= tol, (f, err, tol)
    for f in ("Ubar", "U", "K", "dU", "cost", "feas", "max_tconstr", "max_pconstr"):
        err, tol = _close(g[f], r[f], r2[f])
        assert err <= tol, (f, err, tol)


def test_divergence_full_solve_matches_oracle():
    """The shipped settings (early exits, AL / ReB outer loop, graph-replayed iterations) on a batch
    with diverging trials: the constraint values kept past a break feed the outer updates."""
    prob, kinds, T, es = DC.make("trot", 2, 10, 8)
    g = _gpu(prob, 1)
    r = O.solve_batch(prob, O.default_options(), n_threads=8)
    p2 = dict(prob); p2["x0"] = prob["x0"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(), n_threads=8)
    ok = [b for b in range(len(kinds)) if r["n_ls_trials"][b] == r2["n_ls_trials"][b] and r["iters"][b] == r2["iters"][b]]
    assert len(ok) >= len(kinds) - 1
    for f in ("iters", "outer_iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f][ok], r[f][ok]), f
    err, tol = _close(DC.untranslate(g["Xbar"], T, es)[ok], DC.untranslate(r["Xbar"], T, es)[ok],
                      DC.untranslate(r2["Xbar"], T, es)[ok], 1e-7)
    assert err <= tol, (err, tol)


# ---- rollouts that break before any trial ----------------------------------------------------
def _values_close(g, r, r2, fields=("grf_g", "td_h")):
    for f in fields:
        err, tol = _close(g[f], r[f], r2[f])
        assert err <= tol, (f, err, tol)


@pytest.mark.parametrize("kw", [dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1),
                                dict(no_early_exit=1, max_AL_iter=2, max_DDP_iter=3), {}])
def test_new_problem_initial_rollout_diverges(kw):
    """A new problem's constraint values are zero (create_data, ConstraintsBase.h:26-34, 50-54):
    when its first rollout breaks at knot k (SinglePhase.cpp:205-208), every GRF value from k on
    and every touchdown residual from the break phase on stay zero — here ~24 knots of an element
    whose every later trial breaks too, far more knots with older values than round 5's 8-entry
    table held — and the cost, the LQ model and the ReB / AL updates read them; X past the break is
    the warm start's.  Fixed iterations and the shipped settings, against the oracle."""
    prob, breaks, T, es = DC.make_init("trot", 4, 12, 8)
    s = hsddp.Solver(prob, hsddp.load_settings(**kw))
    s.solve()
    g = {**s.trajectory(), **s.working(), **s.element_info(), **s.constraint_values(), **s.constraint_params()}
    s.close()
    r = O.solve_batch(prob, O.default_options(**kw), n_threads=8)
    p2 = dict(prob); p2["x0"] = prob["x0"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(**kw), n_threads=8)
    for b, j in enumerate(breaks):
        assert r["diverged_init"][b] == (j >= 0), b
    most = max(len(DC.stale_knots(prob, r["U"], r["grf_g"], b)) for b in range(8))
    assert most > 8, most
    for f in ("iters", "outer_iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f], r[f]), f
    for f in ("Xbar", "X"):
        err, tol = _close(DC.untranslate(g[f], T, es), DC.untranslate(r[f], T, es), DC.untranslate(r2[f], T, es))
        assert err <= tol, (f, err, tol)
    for f in ("Ubar", "U", "K", "dU", "cost", "feas", "merit", "max_tconstr", "max_pconstr",
              "reb_delta", "reb_eps", "al_sigma", "al_lambda"):
        err, tol = _close(g[f], r[f], r2[f])
        assert err <= tol, (f, err, tol)
    _values_close(g, r, r2)
    # the device's own account of the older values agrees knot for knot
    for b in range(8):
        assert DC.stale_knots(prob, g["U"], g["grf_g"], b) == DC.stale_knots(prob, r["U"], r["grf_g"], b), b


# pronk element 3 of the receding-horizon batch (B, P, N = 8, 4, 5), translated so that the bound
# falls between the initial rollout's largest simulated-state norms of ticks 1 and 2: the window
# (found by bisection over oracle loops) is [447213.5389, 447213.58); its middle
MPC_T3 = {1: (447213.56, 1), 0: (447213.58, 4)}  # ms -> (translation of element 3, first tick that breaks)


@pytest.mark.parametrize("ms", [1, 0])
def test_mpc_tick_initial_rollout_diverges(ms):
    """HKDMPCSolver::update's loop (shift, new inputs, re-solve with max_AL_iter = 2, max_DDP_iter = 1)
    on a batch whose element 3 is translated until, from a later tick on, the initial rollout of
    every solve breaks (SinglePhase.cpp:205-208): from the 2nd tick on with multiple shooting, from
    the 5th on in single shooting (MS false; T chosen where the oracle's decisions hold over
    T +- 1e-5 and under a 1e-15 perturbation, the earlier ticks' line searches diverging too).  The reference's objects live on from tick to tick:
    past the break the solve keeps the working trajectory of the previous tick (shifted, quirk A2
    included) and the constraint objects' stored values (shifted with their knots; zero for pushed
    knots and new touchdown constraints), and the tick's cost, LQ model and merit read them.  Every
    tick against the oracle doing the same (mpc_oracle.shift_working / shift_constraints)."""
    B, P, N, ticks = 8, 4, 5, 8
    T = np.zeros(B); T[3], first = MPC_T3[ms]
    prob, r0, out = DC.mpc_loop_oracle(B, P, N, T, ticks, ms=ms)
    _, r0p, outp = DC.mpc_loop_oracle(B, P, N, T, ticks, ms=ms, perturb=1e-15)
    div = [t["r"]["diverged_init"][3] for t in out]
    assert r0["diverged_init"][3] == 0 and not any(div[:first]) and all(div[first:]), div
    assert all(t["r"]["diverged_init"][b] == 0 for t in out for b in range(B) if b != 3)
    s = hsddp.Solver(prob, hsddp.load_settings(MS=ms))
    s.solve()
    g = {**s.trajectory(), **s.element_info()}
    for f in ("n_ls_trials", "status"):
        assert np.array_equal(g[f], r0[f]), f
    s.set_options(hsddp.load_settings(max_AL_iter=2, max_DDP_iter=1, MS=ms))
    for it, (t, tp) in enumerate(zip(out, outp)):
        s.shift(t["flags"])
        inp = t["inp"]
        s.update_problem(inp["contacts"], inp["x0"], inp["ref_x"], inp["ref_u"], inp["ref_foot"])
        s.solve()
        g = {**s.trajectory(), **s.working(), **s.element_info(), **s.constraint_values(), **s.constraint_params()}
        r, r2 = t["r"], tp["r"]
        hz = t["prob"]["horizons"]
        es = np.stack([DC.direction_of(inp["contacts"][b], hz) for b in range(B)])
        for f in ("iters", "status", "n_ls_trials"):
            assert np.array_equal(g[f], r[f]), (it, f)
        assert np.array_equal(g["td_mask"], r["td_mask"]), it
        for f in ("Xbar", "X"):
            err, tol = _close(DC.untranslate(g[f], T, es), DC.untranslate(r[f], T, es), DC.untranslate(r2[f], T, es))
            assert err <= tol, (it, f, err, tol)
        for f in ("Ubar", "U", "K", "cost", "feas", "merit", "max_tconstr", "max_pconstr",
                  "reb_delta", "reb_eps", "al_sigma", "al_lambda", "grf_g", "td_h"):
            err, tol = _close(g[f], r[f], r2[f])
            assert err <= tol, (it, f, err, tol)
        assert DC.stale_knots(t["prob"], g["U"], g["grf_g"], 3) == DC.stale_knots(t["prob"], r["U"], r["grf_g"], 3), it
    s.close()
