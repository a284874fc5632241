"""hsddp_solve's graph-replayed inner iteration (early-exit mode) against launch-by-launch issue.

The graph freezes each launch's arguments at capture, so it must be re-captured whenever Params,
the device buffers or the step sizes change; the results of both modes must be bit-identical
(same kernels, same inputs, same order).  HSDDP_NO_GRAPH is read at every solve.
"""
import os

import numpy as np
import pytest

import hsddp
from hsddp import synthetic as syn

pytestmark = pytest.mark.gpu


def _solve(prob, opt, graph, changes=()):
    prev = os.environ.get("HSDDP_NO_GRAPH")
    os.environ["HSDDP_NO_GRAPH"] = "0" if graph else "1"
    try:
        s = hsddp.Solver(prob, opt)
        out = []
        st = s.solve()
        out.append(({**s.trajectory(), **s.element_info()}, st.inner_iterations))
        for change in changes:  # a second solve on the same handle after a change
            change(s)
            st = s.solve()
            out.append(({**s.trajectory(), **s.element_info()}, st.inner_iterations))
        s.close()
        return out
    finally:
        if prev is None:
            os.environ.pop("HSDDP_NO_GRAPH", None)
        else:
            os.environ["HSDDP_NO_GRAPH"] = prev


def _equal(a, b):
    for (ga, ia), (gb, ib) in zip(a, b):
        assert ia == ib
        for f in ("Xbar", "Ubar", "cost", "iters", "outer_iters", "status", "n_ls_trials"):
            assert np.array_equal(ga[f], gb[f]), f


@pytest.mark.parametrize("B,P,N,gait", [(1, 1, 50, "trot"), (16, 8, 25, "jump"), (16, 4, 50, "trot")])
def test_graph_solve_equals_launches(B, P, N, gait):
    prob = syn.make_batch(B, P, N, gait)
    opt = hsddp.load_settings()
    prob2 = syn.make_batch(B, P, N, gait, seed=7)

    def new_x0(s):  # same layout, new inputs: the graph is replayed as captured
        s.upload_problem(prob2["contacts"], prob2["x0"], prob2["ref_x"], prob2["ref_u"], prob2["ref_foot"])

    def new_alpha(s):  # other step sizes: the graph must be re-captured
        o = hsddp.load_settings()
        o.alpha = 0.5
        s.set_options(o)
        new_x0(s)

    changes = (new_x0, new_alpha)
    _equal(_solve(prob, opt, True, changes), _solve(prob, opt, False, changes))


def test_graph_cache_eviction_equals_launches():
    """More distinct (alpha, Params) keys than the handle's 8 cached graphs: every miss past the
    eighth evicts a graph that may be the iteration queued last; the results must still equal
    launch-by-launch issue (eviction drains the stream before destroying the exec)."""
    prob = syn.make_batch(4, 2, 10, "trot")
    opt = hsddp.load_settings()

    def with_alpha(a):
        def ch(s):
            o = hsddp.load_settings()
            o.alpha = a
            s.set_options(o)
            s.upload_problem(prob["contacts"], prob["x0"], prob["ref_x"], prob["ref_u"], prob["ref_foot"])
        return ch

    changes = tuple(with_alpha(a) for a in (0.5, 0.3, 0.2, 0.15, 0.25, 0.35, 0.45, 0.55, 0.6, 0.5, 0.1, 0.3))
    _equal(_solve(prob, opt, True, changes), _solve(prob, opt, False, changes))


@pytest.mark.parametrize("gait,P,N", [("trot", 4, 10), ("jump", 8, 5)])
def test_graph_nonuniform_reb_schedule_equals_launches(gait, P, N):
    """update_ReB = 7, update_relax = 0.1 with several outer iterations and early exits on: the
    second and later outer iterations run k_lq's slot-recompute variant (lq_slots = 1) inside the
    captured graph."""
    prob = syn.make_batch(8, P, N, gait)
    opt = hsddp.load_settings(max_AL_iter=3, update_ReB=7.0, update_relax=0.1)
    _equal(_solve(prob, opt, True), _solve(prob, opt, False))


def test_graph_mixed_layouts_equals_launches():
    """Per-element layouts (trot-like n x N beside jumps on 2n x N/2) with early exits."""
    names = ["trot", "jump", "pace", "jump", "bound", "pronk", "jump"]
    lays = [(g, 8, 5) if g == "jump" else (g, 4, 10) for g in (names[b % len(names)] for b in range(11))]
    prob = syn.make_layout_batch(lays)
    opt = hsddp.load_settings(max_AL_iter=3)
    _equal(_solve(prob, opt, True), _solve(prob, opt, False))


@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("B,P,N,gait", [(1, 1, 50, "trot"), (5, 8, 25, "jump"), (16, 4, 20, "trot")])
def test_fused_decide_equals_separate_launch(monkeypatch, B, P, N, gait, graph):
    """Batches of <= 16 elements decide each line-search trial in the rollout launch (the last block
    to finish, k_rollout FUSE, with a ticket counter it resets itself); HSDDP_NO_FUSED_DECIDE=1 keeps
    the k_decide launch.  Both give the same solve bit for bit, over full solves with early exits
    (graph-replayed and launch by launch) and across repeated solves on one handle (the ticket
    counter must be back at 0 after every trial)."""
    prob = syn.make_batch(B, P, N, gait)
    prob2 = syn.make_batch(B, P, N, gait, seed=7)
    opt = hsddp.load_settings()

    def new_x0(s):
        s.upload_problem(prob2["contacts"], prob2["x0"], prob2["ref_x"], prob2["ref_u"], prob2["ref_foot"])

    monkeypatch.setenv("HSDDP_NO_FUSED_DECIDE", "0")
    a = _solve(prob, opt, graph, changes=(new_x0, new_x0))
    monkeypatch.setenv("HSDDP_NO_FUSED_DECIDE", "1")
    b = _solve(prob, opt, graph, changes=(new_x0, new_x0))
    _equal(a, b)
    assert a[1][0]["n_ls_trials"].sum() > 0
