"""HKDProblem's own registrations through the C++ facade (the drop-in boundary).

hkd-mpc_amd/facade/hkd_problem_example.cpp builds the phases call for call as
HKDProblem::create_problem_one_phase / add_tconstr_one_phase do (HKDProblem.cpp:225-310): std::bind
of HKD::Model<T>::dynamics(_partial) with the phase contact and dt, HKDTrackingCost<T>(contact) on
an HKDSinglePhaseReference, HKDFootPlaceReg<T>(contact) on the QuadReference,
GRFConstraint<T>(contact) + initialize_params(grf_reb_param), std::bind of
HKDReset<T>::resetmap(_partial), TouchDownConstraint<T>(touchdown legs) + initialize_params(td).

CPU: MultiPhaseDDP::describe (what solve() uploads, no device work) equals the problem the
reference's own planning gives — phase plan, contacts, weights, ReB / AL parameters, per-knot
references at t_offset + k dt and the reference-initialised warm start — restated independently by
oracle/ref_oracle.py and the C-ABI's INFO loader.  Integer / float-rounding work: bit-exact.
GPU: the facade's solve equals the ctypes path (hsddp.reference_problem + Solver, device-built
references) bit for bit, Trajectory exports included.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import hsddp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hkd-mpc_amd")
GOLD = os.path.join(ROOT, "tests", "golden")
SETTINGS = os.path.join(PKG, "settings", "ddp_setting.info")
CPARAMS = os.path.join(PKG, "settings", "constraint_params.info")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_oracle as R  # noqa: E402

F32 = np.float32


DRIVERS = os.path.join(ROOT, "tests", "drivers")


def _make():
    for d in (os.path.join(PKG, "facade"), DRIVERS):
        r = subprocess.run(["make", "-C", d], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr


def _run(out, csv, ticks=0, describe=False):
    _make()
    cmd = [os.path.join(DRIVERS, "hkd_problem_example"), csv, SETTINGS, CPARAMS, str(out), str(ticks)]
    if describe:
        cmd.append("describe")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r


def _desc(out, n):
    lines = open(os.path.join(out, f"desc_{n}.txt")).read().split("\n")
    head = lines[0].split()
    P, dt = int(head[0]), float(head[1])
    return {"P": P, "dt": dt, "horizons": [int(v) for v in head[2:2 + P]],
            "contacts": np.array([int(v) for v in lines[1].split()]).reshape(P + 1, 4),
            "weights": np.array([float(v) for v in lines[2].split()]),
            "cparams": np.array([float(v) for v in lines[3].split()])}


def _struct_doubles(s):
    return np.frombuffer(bytes(memoryview(s)), dtype=np.float64)


@pytest.mark.parametrize("name", ["trot", "flytrot"])
def test_describe_equals_reference_planning(tmp_path, name):
    """Tick 0 (HKDProblem::initialization): the facade's device problem from the reference's own
    registrations equals the independently restated plan, parameters and references."""
    csv = os.path.join(GOLD, f"ref_{name}.csv")
    _run(tmp_path, csv, describe=True)
    d = _desc(tmp_path, 0)
    table, dt_ref = R.load_quad_reference(csv)
    n_win = int(round(0.6 / float(dt_ref))) + 2
    plan = R.plan_phases(table[:n_win], dt_ref)
    assert d["horizons"] == plan["horizons"] and sum(d["horizons"]) == 60
    assert np.array_equal(d["contacts"], np.array(plan["contacts"]))
    assert d["dt"] == float(F32(0.01))
    w = hsddp.Weights()
    hsddp.lib().hsddp_default_weights(ctypes.byref(w))
    assert np.array_equal(d["weights"], _struct_doubles(w))      # HKDCost.h's Q, R, Qf, Qfoot
    assert np.array_equal(d["cparams"], _struct_doubles(hsddp.load_constraint_params(CPARAMS)))
    S = sum(n + 1 for n in d["horizons"])
    rx, ru, rf = R.reference_slots(table, 0, n_win, dt_ref, d["horizons"], 0.01, plan["start_times"])
    got = lambda f, w: np.fromfile(os.path.join(tmp_path, f"{f}_0.f64")).reshape(S, w)  # noqa: E731
    assert np.array_equal(got("ref_x", 24), rx)
    assert np.array_equal(got("ref_u", 24), ru)
    assert np.array_equal(got("ref_foot", 12), rf)
    # warm start: HKDProblem.cpp:84-90 reads the state reference at phase_start + k dt_sim (float)
    xb = np.zeros((S, 24))
    s = 0
    for i, n in enumerate(d["horizons"]):
        for k in range(n + 1):
            t = F32(F32(plan["start_times"][i]) + F32(F32(k) * F32(0.01)))
            xb[s] = R.reference_at(table[R.sample_at(t, dt_ref, n_win - 1)])[0]
            s += 1
    assert np.array_equal(got("Xbar", 24), xb)


def test_describe_refuses_what_the_device_cannot_hold():
    """plugin_check covers user plugins; here: a registration whose dynamics is not the HKD model is
    refused by describe() before any device work (facade_check runs it)."""
    _make()
    r = subprocess.run([os.path.join(ROOT, "tests", "drivers", "facade_check"), SETTINGS], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "facade_check ok" in r.stdout, r.stdout + r.stderr


def _hkd_state(x, contact):
    xs = np.repeat(x, 4, axis=0)
    pos = hsddp.model.foot_position(xs, np.tile(np.arange(4), x.shape[0])).reshape(x.shape[0], 4, 3)
    out = x.copy()
    for leg in range(4):
        if contact[0][leg]:
            out[0, 12 + 3 * leg:15 + 3 * leg] = pos[0, leg]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["trot", "flytrot"])
def test_reference_registrations_solve_equals_ctypes_path(tmp_path, name):
    """HKDMPCSolver::initialize's solve (HKDMPC.cpp:18-70) through the facade from the reference's
    own registrations equals the Python/ctypes path on the same window bit for bit."""
    csv = os.path.join(GOLD, f"ref_{name}.csv")
    _run(tmp_path, csv)
    table, dt_ref = hsddp.load_quad_reference(csv)
    x0 = np.zeros((1, 24)); x0[0, 5] = 0.2486
    x0[0, 12:] = np.tile([0.0, -0.8, 1.6], 4)
    p = hsddp.reference_problem(table, dt_ref, [0], x0)
    p["x0"] = _hkd_state(x0, p["contacts"][:, 0])
    assert np.array_equal(np.fromfile(os.path.join(tmp_path, "x0_0.f64")), p["x0"][0])
    s = hsddp.Solver(p, hsddp.load_settings(SETTINGS))
    s.set_value_export(True)
    s.solve()
    tr, info, lq, val = s.trajectory(), s.element_info(), s.lq(), s.value()
    s.close()
    S, Kc, P = p["S"], p["Kc"], len(p["horizons"])
    rd = lambda f, shape: np.fromfile(os.path.join(tmp_path, f"{f}_0.f64")).reshape(shape)  # noqa: E731
    assert np.array_equal(rd("Xbar", (S, 24)), tr["Xbar"][0])
    assert np.array_equal(rd("Ubar", (Kc, 24)), tr["Ubar"][0])
    assert np.array_equal(rd("K", (Kc, 24, 24)), tr["K"][0])
    assert np.array_equal(rd("A", (Kc, 24, 24)), lq["A"][0])
    assert np.array_equal(rd("lx", (Kc, 24)), lq["lx"][0])
    assert np.array_equal(rd("G0", (P, 24)), val["G"][0])
    assert np.array_equal(rd("H0", (P, 24, 24)), val["H"][0])
    cost, feas, iters, outer, status, nls = open(os.path.join(tmp_path, "info_0.txt")).read().split()
    assert float(cost) == info["cost"][0]
    assert (int(iters), int(outer), int(status), int(nls)) == (
        info["iters"][0], info["outer_iters"][0], info["status"][0], info["n_ls_trials"][0])


def _layout(out, n):
    v = [int(t) for t in open(os.path.join(out, f"layout_{n}.txt")).read().split()]
    P = v[0]
    return v[1:1 + P], v[1 + P:1 + 2 * P]


TICKS = 30


@pytest.mark.parametrize("name", ["trot", "flytrot"])
def test_describe_ticks_equal_reference_update(tmp_path, name):
    """Ticks 1..30 (HKDProblem::update, HKDProblem.cpp:117-222, on the facade's phases): every tick's
    device problem — layout, shooting states (SS_set: a new last phase of <= 2 knots keeps an empty
    one, SinglePhase.cpp:34 / HKDProblem.cpp:214-218), contacts, references at the phases' float
    time offsets and the shifted warm start — equals the restated bookkeeping (oracle
    ProblemTracker + mpc_oracle.shift).  Bit-exact."""
    import mpc_oracle as M
    csv = os.path.join(GOLD, f"ref_{name}.csv")
    _run(tmp_path, csv, ticks=TICKS, describe=True)
    table, dt_ref = R.load_quad_reference(csv)
    n_win = int(round(0.6 / float(dt_ref))) + 2
    tk = R.ProblemTracker(table, 0, dt_ref)
    xb = None
    tails = multi = 0
    for n in range(TICKS + 1):
        flags = tk.update(1) if n > 0 else []
        d = _desc(tmp_path, n)
        P = d["P"]
        shooting = [int(v) for v in open(os.path.join(tmp_path, f"desc_{n}.txt")).readline().split()[2 + P:2 + 2 * P]]
        assert d["horizons"] == tk.horizons and sum(d["horizons"]) == 60, n
        assert shooting == tk.shooting, n
        tails += shooting[-1] < d["horizons"][-1] + 1
        assert np.array_equal(d["contacts"], tk.contact_rows()), n
        td = [int(v) for v in open(os.path.join(tmp_path, f"desc_{n}.txt")).read().split("\n")[4].split()]
        assert [[m for m in td[4 * i:4 * i + 4] if m] for i in range(P)] == tk.td, n
        multi += max(len(t) for t in tk.td) > 1
        S = sum(h + 1 for h in d["horizons"])
        rx, ru, rf = R.reference_slots(table, tk.start, n_win, dt_ref, d["horizons"], 0.01, tk.start_times)
        got = lambda f, w: np.fromfile(os.path.join(tmp_path, f"{f}_{n}.f64")).reshape(S, w)  # noqa: E731
        assert np.array_equal(got("ref_x", 24), rx), n
        assert np.array_equal(got("ref_u", 24), ru), n
        assert np.array_equal(got("ref_foot", 12), rf), n
        if n == 0:
            xb = got("Xbar", 24)
            hz, ss, re = list(d["horizons"]), list(shooting), [0] * P
            ub, kk = np.zeros((60, 24)), np.zeros((60, 24, 24))
        else:  # no solve in between: the warm start is the initial one, shifted (X = Xbar)
            hz, ss, re, xb, ub, kk = M.shift(hz, ss, re, xb, xb, ub, kk, flags)
            assert hz == d["horizons"] and ss == shooting, n
            assert np.array_equal(got("Xbar", 24), xb), n
    assert tails >= 1  # the run crosses ticks whose new last phase has no shooting states
    if name == "trot":  # ... and ticks with a phase carrying more than one touchdown constraint
        assert multi >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["trot", "flytrot"])
def test_facade_ticks_equal_capi_mpc_path(tmp_path, name):
    """HKDMPCSolver's loop through the facade — HKDProblem::update on the host Trajectory deques,
    a new MultiPhaseDDP per tick (HKDMPC.cpp:96-143) — equals the C-ABI MPC path on one handle
    (hsddp_advance: the same bookkeeping and the warm-start shift on the device, then
    hsddp_update_problem + hsddp_solve) bit for bit at every tick: Xbar, Ubar, K, the LQ model,
    G[0] / H[0], cost and iteration counts.  The facade keeps one device handle over all ticks."""
    csv = os.path.join(GOLD, f"ref_{name}.csv")
    _run(tmp_path, csv, ticks=TICKS)
    assert open(os.path.join(tmp_path, "handles.txt")).read().split() == ["1"]
    table, dt_ref = hsddp.load_quad_reference(csv)
    rd = lambda f, n, shape: np.fromfile(os.path.join(tmp_path, f"{f}_{n}.f64")).reshape(shape)  # noqa: E731
    x0 = rd("x0", 0, (1, 24))
    p = hsddp.reference_problem(table, dt_ref, [0], x0)
    s = hsddp.Solver(p, hsddp.load_settings(SETTINGS))
    s.set_value_export(True)
    tails = 0
    for n in range(TICKS + 1):
        if n > 0:
            s.advance(None)
            s.update_problem(None, rd("x0", n, (1, 24)))
            s.set_options(hsddp.load_settings(SETTINGS, max_AL_iter=2, max_DDP_iter=1))
        s.solve()
        lay = s.layout()
        hz, ss = _layout(tmp_path, n)
        assert lay["horizons"] == hz and lay["shooting"] == ss, n
        tails += ss[-1] < hz[-1] + 1
        S, Kc, P = sum(h + 1 for h in hz), sum(hz), len(hz)
        tr, info, lq, val = s.trajectory(), s.element_info(), s.lq(), s.value()
        assert np.array_equal(rd("Xbar", n, (S, 24)), tr["Xbar"][0]), n
        assert np.array_equal(rd("Ubar", n, (Kc, 24)), tr["Ubar"][0]), n
        assert np.array_equal(rd("K", n, (Kc, 24, 24)), tr["K"][0]), n
        assert np.array_equal(rd("A", n, (Kc, 24, 24)), lq["A"][0]), n
        assert np.array_equal(rd("lx", n, (Kc, 24)), lq["lx"][0]), n
        assert np.array_equal(rd("G0", n, (P, 24)), val["G"][0]), n
        assert np.array_equal(rd("H0", n, (P, 24, 24)), val["H"][0]), n
        cost, feas, iters, outer, status, nls = open(os.path.join(tmp_path, f"info_{n}.txt")).read().split()
        assert float(cost) == info["cost"][0], n
        assert (int(iters), int(outer), int(status), int(nls)) == (
            info["iters"][0], info["outer_iters"][0], info["status"][0], info["n_ls_trials"][0]), n
    s.close()
    assert tails >= 1
