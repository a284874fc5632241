"""The column-split sweep (k_riccati_cs, hsddp_sweep.hip) against the one-wave sweep and the oracle.

launch_riccati sweeps batches of at most 512 elements (256 pairs) with two waves per element pair,
each forming half the columns of M, Z, Qxx and H; HSDDP_SWEEP_SPLIT = 0 / 1 forces the one-wave
kernel (k_riccati) / the split.  Every entry is formed by the same multiply-adds in the
same order either way, so the two must agree bit for bit: trajectories, gains, dU, branch
decisions.  Batches: B in {1, 5, 1024} (SURVEY.md §8's C1 and C2 sizes — C2 forced: it runs the
one-wave kernel by default — and a ragged batch with an inactive half), jump phases with resets (the impact-aware value transfer at phase ends), per-element
layouts (Bufs::pairs), single shooting (the sweep's dV), failing sweeps with the parallel retries
and the in-kernel regularisation loop, and the oracle at the small sizes.
"""
import numpy as np
import pytest

import hsddp
import oracle_lib as O
from hsddp import synthetic as syn

pytestmark = pytest.mark.gpu

FIELDS = ("Xbar", "Ubar", "K", "X", "U", "dU", "dX", "cost", "feas", "merit", "iters", "outer_iters", "status",
          "n_ls_trials")


def _run(monkeypatch, split, prob, weights=None, **kw):
    monkeypatch.setenv("HSDDP_SWEEP_SPLIT", split)
    s = hsddp.Solver(prob, hsddp.load_settings(**kw), weights=weights) if weights else \
        hsddp.Solver(prob, hsddp.load_settings(**kw))
    s.solve()
    out = {**s.trajectory(), **s.working(), **s.element_info()}
    s.close()
    return out


def _same(a, b):
    for f in FIELDS:
        if f in a:
            assert np.array_equal(a[f], b[f]), f


@pytest.mark.parametrize("B,gait,P,N", [(1, "trot", 1, 50), (5, "trot", 4, 50), (5, "jump", 8, 25),
                                         (1024, "trot", 4, 50)])
def test_split_equals_one_wave_sweep(monkeypatch, B, gait, P, N):
    """Full solves (AL / ReB outer loop, early exits, graph replay) with each kernel: bit-identical."""
    prob = syn.make_batch(B, P, N, gait)
    _same(_run(monkeypatch, "1", prob), _run(monkeypatch, "0", prob))


@pytest.mark.parametrize("gait,P,N", [("trot", 4, 50), ("jump", 8, 25)])
def test_split_single_shooting(monkeypatch, gait, P, N):
    """MS 0 (the sweep's dV, k_riccati_cs<EL, true>): bit-identical to the one-wave DV sweep."""
    prob = syn.make_batch(5, P, N, gait)
    _same(_run(monkeypatch, "1", prob, MS=0), _run(monkeypatch, "0", prob, MS=0))


def test_split_per_element_layouts(monkeypatch):
    """Mixed gaits with per-element layouts: the split sweeps layout pairs (Bufs::pairs), one of
    them with an empty half."""
    prob = syn.make_batch(7, 4, 50, "trot", mixed=True)
    kw = dict(max_AL_iter=2, max_DDP_iter=3)
    _same(_run(monkeypatch, "1", prob, **kw), _run(monkeypatch, "0", prob, **kw))


@pytest.mark.parametrize("mode", ["parallel", "cap2", "sequential"])
def test_split_failing_sweeps(monkeypatch, mode):
    """Negative joint-velocity weights make every first sweep fail the PSD test: the split's
    deferrals to the parallel retries, past the retry cap into its in-kernel regularisation loop,
    and that loop alone (HSDDP_SEQUENTIAL_RETRY) leave what the one-wave kernel leaves."""
    if mode == "cap2":
        monkeypatch.setenv("HSDDP_RETRY_CAP", "2")
    elif mode == "sequential":
        monkeypatch.setenv("HSDDP_SEQUENTIAL_RETRY", "1")
    prob = syn.make_batch(6, 2, 10, "trot")
    w = hsddp.Weights()
    hsddp._lib.lib().hsddp_default_weights(__import__("ctypes").byref(w))
    w.r_qJd = -0.5
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=3)
    a = _run(monkeypatch, "1", prob, weights=w, **kw)
    b = _run(monkeypatch, "0", prob, weights=w, **kw)
    _same(a, b)
    assert np.all(a["status"] == 0) and np.all(a["iters"] > 0)


@pytest.mark.parametrize("B,gait,P,N", [(1, "trot", 1, 50), (5, "jump", 8, 25)])
def test_split_matches_oracle(monkeypatch, B, gait, P, N):
    prob = syn.make_batch(B, P, N, gait)
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=3)
    g = _run(monkeypatch, "1", prob, **kw)
    r = O.solve_batch(prob, O.default_options(**kw), n_threads=8)
    p2 = dict(prob); p2["x0"] = prob["x0"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(**kw), n_threads=8)
    for f in ("Xbar", "Ubar", "K", "X", "U", "dX", "dU"):
        err = np.max(np.abs(g[f] - r[f])) / max(1.0, np.max(np.abs(r[f])))
        env = np.max(np.abs(r2[f] - r[f])) / max(1.0, np.max(np.abs(r[f])))
        assert err < max(1e-9, 10 * env), f
    for f in ("iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f], r[f]), f


@pytest.mark.parametrize("B,gait,P,N,mixed,ms", [(5, "trot", 4, 50, False, 1), (1024, "trot", 4, 50, False, 1),
                                                  (7, "trot", 4, 50, True, 1), (5, "jump", 8, 25, False, 0)])
def test_two_waves_per_workgroup_equals_one(monkeypatch, B, gait, P, N, mixed, ms):
    """The one-wave sweep at two element pairs per workgroup (k_riccati<..., 2>, launched for 257 ..
    1024 pairs) against one pair per workgroup, split off: bit-identical, including a workgroup whose
    second wave has no pair (an odd pair count) and per-element layouts (Bufs::pairs)."""
    prob = syn.make_batch(B, P, N, gait, mixed=mixed) if mixed else syn.make_batch(B, P, N, gait)
    kw = dict(MS=ms) if ms == 0 else {}
    monkeypatch.setenv("HSDDP_SWEEP_WPB", "2")
    a = _run(monkeypatch, "0", prob, **kw)
    monkeypatch.setenv("HSDDP_SWEEP_WPB", "1")
    b = _run(monkeypatch, "0", prob, **kw)
    _same(a, b)
