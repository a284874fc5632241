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
