"""GPU checks of the batched reference construction through the C-ABI:
HKDSinglePhaseReference::get_reference_at_t at every slot of every element, built on the device
(k_build_refs) from a reference file's samples, against oracle/ref_oracle.py — bit-exact (data
movement and float time rounding) — and the solve that reads them against the same solve with the
oracle's references uploaded from the host (bit for bit) and against the oracle solver.

Data: the first samples of the reference's own trot / flytrot files (tests/golden/ref_*.csv)."""
import os
import sys

import numpy as np
import pytest

import hsddp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, HERE)
import oracle_lib as O  # noqa: E402
import ref_oracle as R  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = os.path.join(HERE, "golden")
N_WIN = 62


def _load(name, reorder=False):
    p = os.path.join(GOLD, f"ref_{name}.csv")
    tab, dt = hsddp.load_quad_reference(p, reorder)
    ref, _ = R.load_quad_reference(p, reorder)
    return tab, ref, dt


def _x0(B, seed=3):
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 24))
    x0[:, 5] = 0.25
    x0[:, 12:] = np.float32([.2, -.14, 0, .2, .14, 0, -.2, -.14, 0, -.2, .14, 0])
    x0[:, :3] += rng.uniform(-.05, .05, (B, 3))
    x0[:, 6:12] += rng.uniform(-.2, .2, (B, 6))
    return x0


def _oracle_refs(ref, starts, horizons, dt, pst=None):
    out = [R.reference_slots(ref, int(w), N_WIN, dt, horizons, 0.01, pst) for w in starts]
    return tuple(np.stack([o[q] for o in out]) for q in range(3))


@pytest.mark.parametrize("start", [0, 7, 30])
def test_build_references_match_oracle(start):
    tab, ref, dt = _load("trot")
    p = hsddp.reference_problem(tab, dt, [start], _x0(5))
    s = hsddp.Solver(p)
    got = s.references()
    rx, ru, rf = _oracle_refs(ref, [start], p["horizons"], dt)
    assert np.array_equal(got["ref_x"], rx) and np.array_equal(got["ref_u"], ru) and np.array_equal(got["ref_foot"], rf)
    # explicit phase start times (HKDProblem::update's t_offset) give the same samples
    s.build_references([start], N_WIN, p["phase_start_times"], 0.01)
    again = s.references()
    rx2, _, _ = _oracle_refs(ref, [start], p["horizons"], dt, p["phase_start_times"])
    assert np.array_equal(again["ref_x"], rx2) and np.array_equal(again["ref_x"], rx)
    # the default warm start is the reference (HKDProblem.cpp:84-90)
    tr = s.trajectory()
    assert np.array_equal(tr["Xbar"], np.repeat(rx, 5, axis=0))
    s.close()


def test_per_element_windows_match_oracle():
    """Per-element references: one table holding two files (trot and its leg-reordered copy, whose
    contact switches fall on the same knots), every element its own window start."""
    t1, r1, dt = _load("trot")
    t2, r2, _ = _load("trot", reorder=True)
    tab = np.concatenate([t1, t2])
    ref = r1 + r2
    p0 = hsddp.plan_phases(tab[3:3 + N_WIN], dt)
    n1 = len(t1)
    starts = [3, n1 + 3, 3, n1 + 3, 3, n1 + 3]
    p = hsddp.reference_problem(tab, dt, starts, _x0(6))
    assert p["horizons"] == p0["horizons"]
    s = hsddp.Solver(p)
    got = s.references()
    rx, ru, rf = _oracle_refs(ref, starts, p["horizons"], dt)
    assert got["ref_x"].shape[0] == 6
    assert np.array_equal(got["ref_x"], rx) and np.array_equal(got["ref_u"], ru) and np.array_equal(got["ref_foot"], rf)
    # samples past the table's end read its last sample
    late = len(tab) - 10
    s.build_references([late] * 6, N_WIN, None, 0.01)
    rx3, _, _ = _oracle_refs(ref, [late] * 6, p["horizons"], dt)
    assert np.array_equal(s.references()["ref_x"], rx3)
    with pytest.raises(hsddp.HSDDPError):
        s.build_references([len(tab) + 40] * 6, N_WIN, None, 0.01)  # window outside the table
    s.close()


def _host_prob(p, ref, dt):
    rx, ru, rf = _oracle_refs(ref, p["window_start"], p["horizons"], dt)
    q = {k: v for k, v in p.items() if k not in ("ref_table", "window_start")}
    q.update(ref_x=rx, ref_u=ru, ref_foot=rf, Xbar=np.repeat(rx, p["batch"], axis=0) if rx.shape[0] == 1 else rx,
             Ubar=np.zeros((p["batch"], p["Kc"], 24)))
    return q


@pytest.mark.parametrize("name,start", [("trot", 0), ("flytrot", 11)])
def test_solve_from_file_matches_host_refs_and_oracle(name, start):
    tab, ref, dt = _load(name)
    B = 6
    p = hsddp.reference_problem(tab, dt, [start], _x0(B))
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2)
    a = hsddp.Solver(p, hsddp.load_settings(**kw))
    a.solve()
    ga = {**a.trajectory(), **a.working(), **a.element_info()}
    q = _host_prob(p, ref, dt)
    b = hsddp.Solver(q, hsddp.load_settings(**kw))
    b.solve()
    gb = {**b.trajectory(), **b.working(), **b.element_info()}
    for f in ("Xbar", "Ubar", "K", "X", "U", "cost", "n_ls_trials"):
        assert np.array_equal(ga[f], gb[f]), f
    r = O.solve_batch(q, O.default_options(**kw), n_threads=8)
    for f in ("Xbar", "Ubar", "X", "U"):
        assert np.max(np.abs(ga[f] - r[f])) <= 1e-9 * np.max(np.abs(r[f])), f
    assert np.array_equal(ga["n_ls_trials"], r["n_ls_trials"])
    a.close()
    b.close()


def test_mpc_loop_from_file():
    """Initialise from the trot file, then 12 receding-horizon updates driven step by step: shift on
    the device, build the next window's references on the device, re-solve; a twin solver fed the
    oracle's references from the host stays bit-identical, and the built references equal the
    oracle's every step."""
    tab, ref, dt = _load("trot")
    B = 4
    p = hsddp.reference_problem(tab, dt, [0], _x0(B))
    kw = dict(max_AL_iter=2, max_DDP_iter=1)
    dev = hsddp.Solver(p, hsddp.load_settings(**kw))
    host = hsddp.Solver(_host_prob(p, ref, dt), hsddp.load_settings(**kw))
    dev.solve(); host.solve()
    tk = R.ProblemTracker(ref, 0, dt)
    assert tk.horizons == p["horizons"]
    x0 = _x0(B, 9)
    for it in range(12):
        flag = tk.step()
        la = dev.shift([flag]); lb = host.shift([flag])
        assert la == lb and la["horizons"] == tk.horizons and la["reach_end"] == tk.reach_end, it
        contacts = np.repeat(tk.contact_rows()[None], B, axis=0)
        dev.build_references([tk.start], N_WIN, None, 0.01)
        dev.update_problem(contacts, x0)
        rx, ru, rf = _oracle_refs(ref, [tk.start], tk.horizons, dt)
        assert np.array_equal(dev.references()["ref_x"], rx), it
        host.update_problem(contacts, x0, rx, ru, rf)
        dev.solve(); host.solve()
        ga, gb = dev.trajectory(), host.trajectory()
        for f in ("Xbar", "Ubar", "K"):
            assert np.array_equal(ga[f], gb[f]), (it, f)
        assert np.all(np.isfinite(dev.element_info()["cost"]))
    tk.step()
    dev.shift([0])
    with pytest.raises(hsddp.HSDDPError):
        dev.update_problem(np.repeat(tk.contact_rows()[None], B, axis=0), x0)  # old layout's references
    dev.close(); host.close()


@pytest.mark.parametrize("name,start,steps,n", [("trot", 0, 36, 1), ("flytrot", 6, 8, 2), ("flytrot", 3, 12, 3)])
def test_advance_matches_tracker(name, start, steps, n):
    """hsddp_advance (HKDProblem::update from the table, the whole MPC tick's input side in one
    call) against the oracle's ProblemTracker: step flags, layout, phase contacts (row P: the
    touchdown target), contact durations and references equal; the re-solves bit-identical to a
    twin driven through hsddp_shift / hsddp_update_problem with the oracle's inputs."""
    tab, ref, dt = _load(name)
    B = 3
    p = hsddp.reference_problem(tab, dt, [start], _x0(B))
    kw = dict(max_AL_iter=2, max_DDP_iter=1)
    dev = hsddp.Solver(p, hsddp.load_settings(**kw))
    host = hsddp.Solver(_host_prob(p, ref, dt), hsddp.load_settings(**kw))
    tk = R.ProblemTracker(ref, start, dt)
    info = dev.phase_info()
    assert np.array_equal(info["contacts"][0], tk.contact_rows())
    assert np.array_equal(info["durations"][0], np.array(tk.durations))
    dev.solve(); host.solve()
    rng = np.random.default_rng(5)
    n_new = 0
    for it in range(steps // n):
        x0 = _x0(B, 100 + it)
        flags = dev.advance(x0, n)
        want = [tk.step() for _ in range(n)]
        assert flags == want, it
        lay = dev.layout()
        assert lay["horizons"] == tk.horizons and lay["reach_end"] == tk.reach_end, it
        n_new += sum(flags)
        info = dev.phase_info()
        rows = tk.contact_rows()
        for b in range(B):
            assert np.array_equal(info["contacts"][b], rows), it
            assert np.array_equal(info["durations"][b], np.array(tk.durations)), it
        rx, ru, rf = _oracle_refs(ref, [tk.start], tk.horizons, dt)
        got = dev.references()
        assert np.array_equal(got["ref_x"], rx) and np.array_equal(got["ref_u"], ru), it
        host.shift(want)
        host.update_problem(np.repeat(rows[None], B, axis=0), x0, rx, ru, rf)
        dev.solve(); host.solve()
        ga, gb = dev.trajectory(), host.trajectory()
        for f in ("Xbar", "Ubar", "K"):
            assert np.array_equal(ga[f], gb[f]), (it, f)
        if it % 4 == 0:  # the commands of the tick, durations from the handle's bookkeeping
            cmd = dev.extract_commands(1, 0.01 * it, 0.01, info["durations"], rng.standard_normal(12).astype(np.float32))
            assert np.all(cmd["N_mpcsteps"] == 8)
    assert n_new >= 2  # the window crossed contact switches
    dev.close(); host.close()


def test_advance_loop_matches_oracle():
    """HKDMPCSolver's loop on the reference's trot file (HKDMPC.cpp:57-165): the initial solve with
    the shipped settings, then 25 ticks of hsddp_advance + re-solve (max_AL_iter = 2, max_DDP_iter =
    1), against the oracle doing the same with the restated bookkeeping — warm start
    (mpc_oracle.shift), references, and the constraint objects that live on in the phases: per-knot
    ReB and per-constraint AL parameters carried over (reset_params is a no-op) and one more
    touchdown constraint at every step a last phase has reached its end (mpc_oracle.
    shift_constraints; HKDProblem.cpp:199-202).  The run crosses phases carrying two touchdown
    constraints."""
    import mpc_oracle as M
    tab, ref, dt = _load("trot")
    B = 2
    p = hsddp.reference_problem(tab, dt, [0], _x0(B))
    dev = hsddp.Solver(p, hsddp.load_settings())
    dev.solve()
    q = _host_prob(p, ref, dt)
    r = O.solve_batch(q, O.default_options(), n_threads=2)
    g = dev.trajectory()
    for f in ("Xbar", "Ubar", "K"):
        assert np.max(np.abs(g[f] - r[f])) <= 1e-8 * np.max(np.abs(r[f])), f
    kw = dict(max_AL_iter=2, max_DDP_iter=1)
    dev.set_options(hsddp.load_settings(**kw))
    op, _ = O.default_problem(p["horizons"], p["dt"])
    tk = R.ProblemTracker(ref, 0, dt)
    n_td = 0
    for it in range(25):
        lay0 = dev.layout()
        x0 = _x0(B, 100 + it)
        flags = dev.advance(x0, 1)
        assert flags == tk.update(1), it
        lay = dev.layout()
        assert lay["horizons"] == tk.horizons and lay["shooting"] == tk.shooting, it
        rows = tk.contact_rows()
        sh = [M.shift(lay0["horizons"], lay0["shooting"], lay0["reach_end"], r["Xbar"][b], r["X"][b], r["Ubar"][b],
                      r["K"][b], flags) for b in range(B)]
        cons = [M.resolve_td(M.shift_constraints(lay0["horizons"], lay0["reach_end"],
                                                 {k: r[k][b] for k in O.CONSTRAINT_FIELDS}, flags, op.grf_delta,
                                                 op.grf_eps, op.td_sigma, op.td_lambda), rows) for b in range(B)]
        cons = {k: np.stack([c[k] for c in cons]) for k in O.CONSTRAINT_FIELDS}
        rx, ru, rf = _oracle_refs(ref, [tk.start], tk.horizons, dt)
        p2 = {"batch": B, "horizons": tk.horizons, "shooting": tk.shooting, "dt": p["dt"],
              "S": sum(n + 1 for n in tk.horizons), "Kc": sum(tk.horizons), "x0": x0,
              "contacts": np.repeat(rows[None], B, axis=0), "ref_x": rx, "ref_u": ru, "ref_foot": rf,
              "Xbar": np.stack([s[3] for s in sh]), "Ubar": np.stack([s[4] for s in sh]), "K": np.stack([s[5] for s in sh])}
        dc = dev.constraint_params()
        assert np.array_equal(dc["td_mask"], cons["td_mask"]), it
        assert [[m for m in dc["td_mask"][0, i] if m] for i in range(len(tk.horizons))] == tk.td, it
        n_td = max(n_td, max(len(t) for t in tk.td))
        dev.solve()
        r = O.solve_batch(p2, O.default_options(**kw), n_threads=2, constraints=cons)
        g, dc = {**dev.trajectory(), **dev.working(), **dev.element_info()}, dev.constraint_params()
        for f in ("al_sigma", "al_lambda", "reb_delta", "reb_eps"):
            assert np.max(np.abs(dc[f] - r[f])) <= 1e-9 * max(1.0, np.max(np.abs(r[f]))), (it, f)
        for f in ("Xbar", "Ubar", "X", "K"):
            assert np.max(np.abs(g[f] - r[f])) <= 1e-8 * np.max(np.abs(r[f])), (it, f)
        assert np.array_equal(g["n_ls_trials"], r["n_ls_trials"]), it
    assert n_td >= 2
    dev.close()


def test_references_uploaded_after_begin_reach_the_line_search():
    """The line search reads the references from an entry-major copy (Bufs::ref_t), refreshed
    from the uploaded rows before the next launches that read them — also when new references
    arrive between hsddp_solve_begin and hsddp_iterate.  A handle that began with other references
    and then took the new ones must iterate exactly as one that had the new ones from the start
    (the trials' running costs decide acceptance, so stale columns would part them)."""
    from hsddp import synthetic as syn
    prob = syn.make_batch(64, 4, 50, "trot")
    rx2 = prob["ref_x"].copy()
    rx2[..., 5] += 0.03   # a higher body (and the foot references with it: a different running cost)
    rx2[..., 3] += 0.02
    prob1 = dict(prob)
    prob2 = dict(prob, ref_x=rx2)
    opts = hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=3)
    out = []
    for p in (prob1, prob2):
        s = hsddp.Solver(p, opts)
        s.begin()
        s.update_problem(prob["contacts"], prob["x0"], rx2, prob["ref_u"], prob["ref_foot"])
        s.iterate(3)
        out.append({**s.trajectory(), **s.element_info()})
        s.close()
    a, b = out
    for f in ("Xbar", "Ubar", "K", "cost", "n_ls_trials", "status"):
        assert np.array_equal(a[f], b[f]), f
