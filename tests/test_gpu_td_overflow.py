"""The touchdown-constraint limit (HSDDP_MAX_TD) through hsddp_advance, on both shift paths.

The reference registers one more TouchDownConstraint on the last phase at every step once that
phase has reached its end (HKDProblem.cpp:199-202) and keeps them in an unbounded list.  With one
reference sample per simulation step the next step's horizon-end contact differs and a new phase
starts, so a phase carries at most two (include/hsddp.h, hsddp_advance).  The limit is reached only
by contacts that change faster than the simulation step: here the trot fixture's contacts alternate
0000 / 0110 sample by sample from sample 64, and the simulation step is two samples (dt_sim = 0.02),
so every step sees flight at the horizon end and a touchdown one sample later.

What a step past the limit must leave (the state the C-ABI documents): HSDDP_ERR_UNSUPPORTED, the
phase keeping its first HSDDP_MAX_TD constraints, and otherwise the complete step — layout,
contacts, durations, references, warm start — with a handle that solves, equal to the oracle's
restatement of the same tick with the constraint list capped (mpc_oracle.shift_constraints(cap=True)).
"""
import os
import sys

import numpy as np
import pytest

import hsddp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import mpc_oracle as M  # noqa: E402
import oracle_lib as O  # noqa: E402
import ref_oracle as R  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = os.path.join(HERE, "golden")
N_WIN = 62
DT_SIM = 0.02
A, BC = (0, 0, 0, 0), (0, 1, 1, 0)


def _tables():
    """(device table, oracle table, dt): the trot fixture with alternating contacts from sample 64"""
    p = os.path.join(GOLD, "ref_trot.csv")
    tab, dt = hsddp.load_quad_reference(p)
    ref, _ = R.load_quad_reference(p)
    for k in range(64, len(ref)):
        c = A if (k - 64) % 2 == 0 else BC
        tab["contact"][k] = c
        ref[k]["contact"] = np.array(c)
    return tab, ref, dt


def _x0(B, seed):
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 24))
    x0[:, 5] = 0.25
    x0[:, 12:] = np.float32([.2, -.14, 0, .2, .14, 0, -.2, -.14, 0, -.2, .14, 0])
    x0[:, :3] += rng.uniform(-.05, .05, (B, 3))
    x0[:, 6:12] += rng.uniform(-.2, .2, (B, 6))
    return x0


def _refs(ref, start, horizons, dt):
    return R.reference_slots(ref, int(start), N_WIN, dt, horizons, DT_SIM)


def _advance(dev, x0):
    """dev.advance, returning (flags, overflow)"""
    try:
        return dev.advance(x0, 1), False
    except hsddp.HSDDPError as e:
        assert "HSDDP_MAX_TD" in str(e), str(e)
        return None, True


def test_overflow_shared_layout_matches_capped_oracle():
    """One layout for the batch: the deferred shift, whose overflow flag is read at the end of the
    advance.  Every tick against the oracle with the capped constraint list."""
    tab, ref, dt = _tables()
    B = 2
    p = hsddp.reference_problem(tab, dt, [0], _x0(B, 3), dt_sim=DT_SIM)
    kw = dict(max_AL_iter=2, max_DDP_iter=1)
    dev = hsddp.Solver(p, hsddp.load_settings(**kw))
    dev.solve()
    rx, ru, rf = _refs(ref, 0, p["horizons"], dt)
    q = {k: v for k, v in p.items() if k not in ("ref_table", "window_start")}
    q.update(ref_x=rx[None], ref_u=ru[None], ref_foot=rf[None], Xbar=np.repeat(rx[None], B, axis=0),
             Ubar=np.zeros((B, p["Kc"], 24)))
    r = O.solve_batch(q, O.default_options(**kw), n_threads=2)
    op, _ = O.default_problem(p["horizons"], p["dt"])
    tk = R.ProblemTracker(ref, 0, dt, dt_sim=DT_SIM)
    n_over = 0
    for it in range(8):
        lay0 = dev.layout()
        x0 = _x0(B, 100 + it)
        flags, over = _advance(dev, x0)
        want = tk.update(1)
        # the complete step, overflow or not
        lay = dev.layout()
        assert lay["horizons"] == tk.horizons and lay["shooting"] == tk.shooting, it
        rows = tk.contact_rows()
        info = dev.phase_info()
        for b in range(B):
            assert np.array_equal(info["contacts"][b], rows), it
            assert np.array_equal(info["durations"][b], np.array(tk.durations)), it
        rx, ru, rf = _refs(ref, tk.start, tk.horizons, dt)
        got = dev.references()
        assert np.array_equal(got["ref_x"][0], rx) and np.array_equal(got["ref_u"][0], ru), it
        if flags is not None:
            assert flags == want, it
        sh = [M.shift(lay0["horizons"], lay0["shooting"], lay0["reach_end"], r["Xbar"][b], r["X"][b], r["Ubar"][b],
                      r["K"][b], want) for b in range(B)]
        cons = [M.shift_constraints(lay0["horizons"], lay0["reach_end"], {k: r[k][b] for k in O.CONSTRAINT_FIELDS},
                                    want, op.grf_delta, op.grf_eps, op.td_sigma, op.td_lambda, cap=True) for b in range(B)]
        assert over == cons[0]["overflow"], it
        n_over += over
        cons = [M.resolve_td(c, rows) for c in cons]
        cons = {k: np.stack([c[k] for c in cons]) for k in O.CONSTRAINT_FIELDS}
        dc = dev.constraint_params()
        assert np.array_equal(dc["td_mask"], cons["td_mask"]), it
        # the tracker's unbounded lists, of which the device keeps the first HSDDP_MAX_TD
        for i in range(len(tk.horizons)):
            assert [m for m in dc["td_mask"][0, i] if m] == tk.td[i][:M.MAX_TD], (it, i)
        dev.solve()
        p2 = {"batch": B, "horizons": tk.horizons, "shooting": tk.shooting, "dt": p["dt"],
              "S": sum(n + 1 for n in tk.horizons), "Kc": sum(tk.horizons), "x0": x0,
              "contacts": np.repeat(rows[None], B, axis=0), "ref_x": rx[None], "ref_u": ru[None], "ref_foot": rf[None],
              "Xbar": np.stack([s[3] for s in sh]), "Ubar": np.stack([s[4] for s in sh]), "K": np.stack([s[5] for s in sh])}
        r = O.solve_batch(p2, O.default_options(**kw), n_threads=2, constraints=cons)
        g, dc = {**dev.trajectory(), **dev.working(), **dev.element_info()}, dev.constraint_params()
        for f in ("al_sigma", "al_lambda", "reb_delta", "reb_eps"):
            assert np.max(np.abs(dc[f] - r[f])) <= 1e-9 * max(1.0, np.max(np.abs(r[f]))), (it, f)
        for f in ("Xbar", "Ubar", "X", "K"):
            assert np.max(np.abs(g[f] - r[f])) <= 1e-8 * np.max(np.abs(r[f])), (it, f)
        assert np.array_equal(g["n_ls_trials"], r["n_ls_trials"]), it
    assert n_over >= 2 and max(len(t) for t in tk.td) > M.MAX_TD
    dev.close()


def test_overflow_per_element_layouts_completes_the_step():
    """Elements that disagree on a contact change take the per-element shift (hsddp_shift_elements
    inside the advance, synchronous): its overflow no longer returns before the references, the
    contacts, the durations and the clock of the step (the advance finishes, then reports it), and
    the handle keeps solving tick after tick."""
    tab_alt, ref_alt, dt = _tables()
    p0 = os.path.join(GOLD, "ref_trot.csv")
    tab_trot, _ = hsddp.load_quad_reference(p0)
    ref_trot, _ = R.load_quad_reference(p0)
    tab = np.concatenate([tab_alt, tab_trot])
    ref = ref_alt + ref_trot
    n1 = len(tab_alt)
    B = 2
    p = hsddp.reference_problem(tab, dt, [0, n1], _x0(B, 4), dt_sim=DT_SIM)
    dev = hsddp.Solver(p, hsddp.load_settings(max_AL_iter=2, max_DDP_iter=1))
    dev.solve()
    tks = [R.ProblemTracker(ref, 0, dt, dt_sim=DT_SIM), R.ProblemTracker(ref, n1, dt, dt_sim=DT_SIM)]
    n_over = n_elem = 0
    for it in range(8):
        flags, over = _advance(dev, _x0(B, 200 + it))
        want = [tk.update(1) for tk in tks]
        n_over += over
        lays = dev.element_layouts()
        n_elem += lays["horizons"][0] != lays["horizons"][1]
        info = dev.phase_info()
        got = dev.references()
        dc = dev.constraint_params()
        for b, tk in enumerate(tks):
            assert lays["horizons"][b] == tk.horizons and lays["shooting"][b] == tk.shooting, (it, b)
            P = len(tk.horizons)
            assert np.array_equal(info["contacts"][b][:P + 1], tk.contact_rows()), (it, b)
            assert np.array_equal(info["durations"][b][:P], np.array(tk.durations)), (it, b)
            rx, _, _ = _refs(ref, tk.start, tk.horizons, dt)
            assert np.array_equal(got["ref_x"][b][:len(rx)], rx), (it, b)
            for i in range(P):
                assert [m for m in dc["td_mask"][b, i] if m] == tk.td[i][:M.MAX_TD], (it, b, i)
        if flags is not None:
            assert flags == [int(w0 or w1) for w0, w1 in zip(*want)], it
        dev.solve()
        info = dev.element_info()
        assert np.all(info["status"] == 0) and np.all(np.isfinite(dev.trajectory()["Xbar"])), it
    assert n_over >= 2 and n_elem >= 1
    assert max(len(t) for t in tks[0].td) > M.MAX_TD
    dev.close()
