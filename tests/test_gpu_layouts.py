"""Per-element phase layouts (hsddp_set_element_layouts): one handle whose elements segment the same
Kc knots into their own phases, as HKDProblem::initialization does per problem (HKDProblem.cpp:
40-68) — here trot-like gaits on n x N beside jumps on 2n x N/2.

Each element of a mixed handle must be solved exactly as in a handle of its own layout: the mixed
solve is compared bit for bit with uniform-layout solves of the same elements (same kernels, same
arithmetic — the layout only changes which slots and phases a kernel visits and how the sweep
pairs elements), and a sample against the oracle."""
import numpy as np
import pytest

import hsddp
import oracle_lib as O
from hsddp import synthetic as syn

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def _mixed(B, P=4, N=10, seed=syn.SEED):
    names = ["trot", "jump", "pace", "jump", "bound", "pronk", "jump"]
    lays = [(g, 2 * P, N // 2) if g == "jump" else (g, P, N) for g in (names[b % len(names)] for b in range(B))]
    return syn.make_layout_batch(lays, seed=seed)


def _run(prob, opt, weights=None, **kw):
    s = hsddp.Solver(prob, opt, weights=weights, **kw)
    s.solve()
    out = {**s.trajectory(), **s.working(), **s.element_info()}
    out["lq"], out["term"] = s.lq(), s.terminal()
    s.close()
    return out


def _check_against_uniform(prob, opt, weights=None):
    g = _run(prob, opt, weights)
    for hz, idx in syn.layout_groups(prob).items():
        sub = syn.sub_batch(prob, idx, hz)
        u = _run(sub, opt, weights)
        S, P = sub["S"], len(hz)
        for f in ("Xbar", "X", "Defect", "dX"):
            assert np.array_equal(g[f][idx, :S], u[f]), (hz, f)
        for f in ("Ubar", "U", "dU", "K"):
            assert np.array_equal(g[f][idx], u[f]), (hz, f)
        for f in ("cost", "feas", "merit", "max_tconstr", "max_pconstr", "iters", "outer_iters", "status", "n_ls_trials"):
            assert np.array_equal(g[f][idx], u[f]), (hz, f)
        for f in ("A", "B", "lx", "lu", "lxx", "luu", "l"):
            assert np.array_equal(g["lq"][f][idx], u["lq"][f]), (hz, f)
        for f in ("Phi", "Phix", "Phixx", "Px"):
            assert np.array_equal(g["term"][f][idx, :P], u["term"][f]), (hz, f)
            assert np.all(g["term"][f][idx, P:] == 0), (hz, f)
    return g


@pytest.mark.parametrize("B", [7, 24])
def test_mixed_layouts_equal_uniform_handles_fixed_iterations(B):
    prob = _mixed(B)
    opt = hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=3)
    g = _check_against_uniform(prob, opt)
    # and against the oracle, per layout
    for hz, idx in syn.layout_groups(prob).items():
        sub = syn.sub_batch(prob, idx, hz)
        r = O.solve_batch(sub, O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=3), n_threads=8)
        S = sub["S"]
        assert np.array_equal(g["n_ls_trials"][idx], r["n_ls_trials"])
        for f in ("Xbar", "Ubar", "K"):
            a = g[f][idx, :S] if f == "Xbar" else g[f][idx]
            assert rel(a, r[f]) < 1e-9, (hz, f)


def test_mixed_layouts_full_solve_equal_uniform_handles():
    """The reference loop with its early exits (default settings): per-element exits differ
    between layouts inside one handle."""
    _check_against_uniform(_mixed(21), hsddp.load_settings())


def test_mixed_layouts_regularisation_retries(monkeypatch):
    """Every first sweep fails (r_qJd < 0, test_gpu_parity.py::test_retries_match_oracle): the
    parallel retries of a mixed handle pair attempts of one element per wave; the result equals
    the uniform handles' and the sequential loop's."""
    w = hsddp.Weights()
    hsddp.lib().hsddp_default_weights(__import__("ctypes").byref(w))
    w.r_qJd = -0.5
    prob = _mixed(9)
    opt = hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2)
    g = _check_against_uniform(prob, opt, w)
    monkeypatch.setenv("HSDDP_SEQUENTIAL_RETRY", "1")
    q = _run(prob, opt, w)
    for f in ("Xbar", "Ubar", "K", "dU", "cost", "status", "n_ls_trials"):
        assert np.array_equal(g[f], q[f]), f


def test_layouts_validation():
    prob = _mixed(4)
    bad = dict(prob, layouts=[[10, 10, 10, 10], [5] * 8, [10, 10, 10, 9], [10] * 4])
    with pytest.raises(hsddp.HSDDPError, match="Kc"):
        hsddp.Solver(bad, hsddp.load_settings())
    s = hsddp.Solver(prob, hsddp.load_settings())
    s.solve()
    cmd = s.extract_commands()  # each element's own knot walk (per-element layouts)
    assert np.all(cmd["N_mpcsteps"] == 8) and np.all(np.isfinite(cmd["hkd_controls"]))
    s.close()


def _inputs(gaits, horizons_list, offset, Pmax, Smax, B):
    """contacts / references of each element's (possibly new) layout: the gait's schedule from
    phase `offset`, the closed-form references on that layout."""
    contacts = np.zeros((B, Pmax + 1, 4), np.int32)
    rx = np.zeros((B, Smax, 24)); ru = np.zeros((B, Smax, 24)); rf = np.zeros((B, Smax, 12))
    for b, (g, hz) in enumerate(zip(gaits, horizons_list)):
        sched = syn.phase_schedule(g, len(hz), offset)
        contacts[b, :len(hz) + 1] = sched
        x, u, f = syn._reference_slots(sched, hz, t0=offset)
        S = x.shape[0]
        rx[b, :S], ru[b, :S], rf[b, :S] = x, u, f
    return contacts, rx, ru, rf


def test_shift_elements_equals_uniform_shifts():
    """hsddp_shift_elements: robots crossing contact boundaries at different knots.  Group A's flags
    add a phase (the first change marks the last phase's end, the second starts a new phase), group
    B's only grow the last phase; each group must end exactly as a uniform handle of its elements
    shifted by hsddp_shift with its flags — warm start after the shift, then a re-solve."""
    B, P, N = 7, 4, 10
    prob = syn.make_batch(B, P, N, "trot")
    for k in ("ref_x", "ref_u", "ref_foot"):  # per-element references (the layouts diverge)
        prob[k] = np.ascontiguousarray(np.repeat(prob[k], B, axis=0))
    opt = hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2)
    flagsA, flagsB = [1, 1, 0], [0, 0, 0]
    ga, gb = [0, 2, 3, 6], [1, 4, 5]
    cc = np.array([flagsA if b in ga else flagsB for b in range(B)], np.int32)

    m = hsddp.Solver(prob, opt)
    m.solve()
    lay = m.shift_elements(cc)
    hzs = lay["horizons"]
    assert hzs[ga[0]] != hzs[gb[0]] and all(hzs[b] == hzs[ga[0]] for b in ga) and all(hzs[b] == hzs[gb[0]] for b in gb)
    gaits = ["trot"] * B
    Pm, Sm = m.P, m.S
    c, rx, ru, rf = _inputs(gaits, hzs, 1, Pm, Sm, B)
    # the warm start right after the shift and the new inputs (update_problem keeps Xbar / Ubar / K
    # and the working rows, as the reference's objects live on into the next tick)
    m.update_problem(c, prob["x0"], rx, ru, rf)
    wm = m.trajectory()
    m.solve()
    gm = {**m.trajectory(), **m.element_info()}
    m.close()
    for idx, flags in ((ga, flagsA), (gb, flagsB)):
        sub = {k: (v[idx] if isinstance(v, np.ndarray) and v.shape[:1] == (B,) else v) for k, v in prob.items()}
        sub["batch"] = len(idx)
        u = hsddp.Solver(sub, opt)
        u.solve()
        ul = u.shift(flags)
        assert ul["horizons"] == hzs[idx[0]]
        S = u.S
        cu, rxu, ruu, rfu = _inputs(["trot"] * len(idx), [ul["horizons"]] * len(idx), 1, u.P, S, len(idx))
        u.update_problem(cu, prob["x0"][idx], rxu, ruu, rfu)
        wu = u.trajectory()
        for f in ("Xbar", "Ubar", "K"):
            a = wm[f][idx, :S] if f == "Xbar" else wm[f][idx]
            assert np.array_equal(a, wu[f]), ("warm start", f)
        u.solve()
        gu = {**u.trajectory(), **u.element_info()}
        u.close()
        assert np.array_equal(gm["Xbar"][idx, :S], gu["Xbar"]) and np.array_equal(gm["K"][idx], gu["K"])
        for f in ("Ubar", "cost", "n_ls_trials", "iters", "status"):
            assert np.array_equal(gm[f][idx], gu[f]), f


def test_diverging_shift_with_shared_references_fails_and_keeps_the_handle():
    """A handle with one reference for the batch cannot hold per-element layouts: a per-element shift
    whose elements diverge is refused before any device work, and the handle still solves as
    before (the shared layout untouched); hsddp_set_element_layouts refuses likewise."""
    prob = syn.make_batch(4, 2, 10, "trot")
    opt = hsddp.load_settings(max_AL_iter=1, max_DDP_iter=1, no_early_exit=1)
    s = hsddp.Solver(prob, opt)
    s.solve()
    before = s.trajectory()
    with pytest.raises(hsddp.HSDDPError, match="per-element references"):
        s.shift_elements(np.array([[1], [0], [0], [0]]))  # element 0 alone crosses a contact change
    lay = s.layout()
    assert list(lay["horizons"]) == list(prob["horizons"])
    with pytest.raises(hsddp.HSDDPError, match="per-element references"):
        hz = np.zeros((4, 16), np.int32); hz[:, 0] = 20
        hsddp.check(hsddp.lib().hsddp_set_element_layouts(s._h, hsddp.ip(np.ones(4, np.int32)), hsddp.ip(hz)))
    s.warm_start(before["Xbar"], before["Ubar"], before["K"])
    s.solve()
    assert np.all(np.isfinite(s.trajectory()["Xbar"]))
    # value export off: the download is refused instead of returning a stale buffer
    s.set_value_export(True)
    s.solve()
    assert np.all(np.isfinite(s.value()["H"]))
    s.set_value_export(False)
    with pytest.raises(hsddp.HSDDPError, match="value export is off"):
        s.value()
    s.close()


def test_mixed_gait_mpc_loop_equals_uniform_handles():
    """HKDMPCSolver's loop for robots on different gaits in one handle (SURVEY.md §8 config C4's
    MPC side): windows into the reference's trot and flytrot files (one table, per-element window
    starts) segment into different phase layouts at initialization (HKDProblem.cpp:40-68); then 16
    ticks of hsddp_advance — each element's own contact changes, per-element shifts — re-solve and
    command extraction (each element's own knot walk, HKDMPC.cpp:207-298).  Every element's layout,
    warm start, solution and command record equal, bit for bit, those of a uniform handle of the
    elements of its file alone."""
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    ta, dt = hsddp.load_quad_reference(os.path.join(gold, "ref_trot.csv"))
    tb, _ = hsddp.load_quad_reference(os.path.join(gold, "ref_flytrot.csv"))
    tab = np.concatenate([ta, tb])
    B = 6
    starts = [0 if b % 2 == 0 else len(ta) + 2 for b in range(B)]
    rng = np.random.default_rng(4)
    x0 = np.zeros((B, 24))
    x0[:, 5] = 0.25
    x0[:, 12:] = np.float32([.2, -.14, 0, .2, .14, 0, -.2, -.14, 0, -.2, .14, 0])
    x0[:, 6:12] += rng.uniform(-.2, .2, (B, 6))
    p = hsddp.reference_problem(tab, dt, starts, x0)
    assert p.get("layouts") is not None  # the two files segment the 60 knots differently
    opt, kw = hsddp.load_settings(), dict(max_AL_iter=2, max_DDP_iter=1)
    m = hsddp.Solver(p, opt)
    m.solve()
    groups = [list(range(0, B, 2)), list(range(1, B, 2))]
    uni = []
    for idx in groups:
        q = hsddp.reference_problem(tab, dt, [starts[i] for i in idx], x0[idx])
        assert q.get("layouts") is None
        u = hsddp.Solver(q, opt)
        u.solve()
        uni.append(u)
    m.set_options(hsddp.load_settings(**kw))
    for u in uni:
        u.set_options(hsddp.load_settings(**kw))
    feet = rng.standard_normal((B, 12)).astype(np.float32)
    diverged = 0
    for it in range(16):
        xt = x0 + rng.uniform(-.01, .01, x0.shape)
        m.advance(xt, 1)
        lay = m.element_layouts()
        diverged += any(h != lay["horizons"][0] for h in lay["horizons"])
        m.solve()
        g = {**m.trajectory(), **m.element_info()}
        info = m.phase_info()
        cm = m.extract_commands(1, 0.01 * (it + 1), 0.01, info["durations"], feet, 0.5)
        for idx, u in zip(groups, uni):
            u.advance(xt[idx], 1)
            ul = u.layout()
            u.solve()
            gu = {**u.trajectory(), **u.element_info()}
            cu = u.extract_commands(1, 0.01 * (it + 1), 0.01, u.phase_info()["durations"], feet[idx], 0.5)
            S = u.S
            for j, b in enumerate(idx):
                assert lay["horizons"][b] == ul["horizons"] and lay["shooting"][b] == ul["shooting"], (it, b)
                assert np.array_equal(g["Xbar"][b, :S], gu["Xbar"][j]), (it, b)
                for f in ("Ubar", "K"):
                    assert np.array_equal(g[f][b], gu[f][j]), (it, b, f)
                for f in ("cost", "iters", "status", "n_ls_trials"):
                    assert g[f][b] == gu[f][j], (it, b, f)
                for f in cm.dtype.names:
                    assert np.array_equal(cm[f][b], cu[f][j]), (it, b, f)
    assert diverged >= 4  # the loop ran on per-element layouts
    m.close()
    for u in uni:
        u.close()
