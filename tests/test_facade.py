"""C++ facade (hkd-mpc_amd/facade/hsddp_facade.hpp): the reference's MultiPhaseDDP / SinglePhase
call sequence over the C-ABI.

CPU: the facade builds with g++ against include/hsddp.h, its option defaults and INFO loader match
the C-ABI, and a non-HKD plugin is refused before any device work.  GPU: a solve through the
facade (hkd_solve_example, one trajectory) equals the Python/ctypes path on the same problem —
both drive the same device kernels, so the comparison is exact.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hkd-mpc_amd")


def _make():
    for d in (os.path.join(PKG, "facade"), os.path.join(ROOT, "tests", "drivers")):
        r = subprocess.run(["make", "-C", d], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr


def test_facade_builds_and_checks():
    _make()
    r = subprocess.run([os.path.join(ROOT, "tests", "drivers", "facade_check"), os.path.join(PKG, "settings", "ddp_setting.info")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade_check ok" in r.stdout


def test_reference_plugin_api_compiles_and_works_on_the_host():
    """plugin_check: a cost / constraints written with the reference's HKD plugin declarations
    (HKDCost.h:75-81, HKDConstraints.h:21-37) and a user SinglePhaseBase compile against the facade;
    the bases' ReB / AL helpers give their closed forms; a user cost is refused by solve()."""
    _make()
    r = subprocess.run([os.path.join(ROOT, "tests", "drivers", "plugin_check")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "plugin_check ok" in r.stdout


@pytest.mark.gpu
def test_hkd_plugins_evaluate_on_the_device():
    """The facade's hkd:: plugins' virtuals (running_cost(_par), terminal_cost(_par),
    compute_violation / compute_partial) through the device primitives."""
    _make()
    r = subprocess.run([os.path.join(ROOT, "tests", "drivers", "plugin_check"), "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "plugin_check ok" in r.stdout


def _write_problem(d, prob):
    P = len(prob["horizons"])
    with open(os.path.join(d, "problem.txt"), "w") as f:
        f.write(f"{P} {prob['dt']!r} " + " ".join(str(n) for n in prob["horizons"]) + "\n")
    prob["contacts"][0].astype(np.int32).tofile(os.path.join(d, "contacts.i32"))
    prob["x0"][0].astype(np.float64).tofile(os.path.join(d, "x0.f64"))
    prob["ref_x"][0].astype(np.float64).tofile(os.path.join(d, "ref_x.f64"))
    prob["ref_u"][0].astype(np.float64).tofile(os.path.join(d, "ref_u.f64"))
    prob["ref_foot"][0].astype(np.float64).tofile(os.path.join(d, "ref_foot.f64"))


@pytest.mark.gpu
@pytest.mark.parametrize("gait,P,N", [("trot", 4, 20), ("jump", 4, 15)])
def test_facade_solve_matches_ctypes_path(tmp_path, gait, P, N):
    import hsddp
    from hsddp import synthetic as syn
    _make()
    prob = syn.make_batch(1, P, N, gait)
    _write_problem(str(tmp_path), prob)
    r = subprocess.run([os.path.join(PKG, "hkd_solve_example"), str(tmp_path), "2", "4",
                        os.path.join(PKG, "settings", "ddp_setting.info")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    S, Kc = prob["S"], prob["Kc"]
    Xb = np.fromfile(os.path.join(tmp_path, "Xbar.f64")).reshape(S, 24)
    Ub = np.fromfile(os.path.join(tmp_path, "Ubar.f64")).reshape(Kc, 24)
    K = np.fromfile(os.path.join(tmp_path, "K.f64")).reshape(Kc, 24, 24)
    cost, feas, iters, outer, status, nls = open(os.path.join(tmp_path, "info.txt")).read().split()

    s = hsddp.Solver(prob, hsddp.load_settings(max_AL_iter=2, max_DDP_iter=4))
    s.set_value_export(True)   # as the facade (get_value_approx)
    s.solve()
    tr, info, wk, lq, term, val, hist = s.trajectory(), s.element_info(), s.working(), s.lq(), s.terminal(), s.value(), s.solver_info()
    s.close()
    # Trajectory exports (TrajectoryManagement.h:49-81) equal the C-ABI downloads
    rd = lambda n, shape, dt=np.float64: np.fromfile(os.path.join(tmp_path, n), dtype=dt).reshape(shape)
    assert np.array_equal(rd("Xsim.f64", (S, 24)), wk["X"][0] + wk["Defect"][0])
    assert np.array_equal(rd("A.f64", (Kc, 24, 24)), lq["A"][0])
    assert np.array_equal(rd("l.f64", (Kc,)), lq["l"][0])
    assert np.array_equal(rd("lx.f64", (Kc, 24)), lq["lx"][0])
    assert np.array_equal(rd("luu.f64", (Kc, 24, 24)), lq["luu"][0])
    assert np.array_equal(rd("Phix.f64", (P, 24)), term["Phix"][0])
    assert np.array_equal(rd("G0.f64", (P, 24)), val["G"][0])
    assert np.array_equal(rd("H0.f64", (P, 24, 24)), val["H"][0])
    hz = np.cumsum([0] + list(prob["horizons"]))
    pc = [lq["l"][0][hz[i]:hz[i + 1]].sum() + term["Phi"][0][i] for i in range(P)]
    assert np.allclose(rd("phase_cost.f64", (P,)), pc, rtol=1e-14, atol=0)
    got = rd("solver_info.f32", (-1, 4), np.float32)
    want = np.stack([hist[k][0] for k in ("cost", "dyn_feas", "eqn_feas", "ineq_feas")], 1)
    assert np.array_equal(got, want) and got.shape[0] >= 2
    assert np.array_equal(Xb, tr["Xbar"][0])
    assert np.array_equal(Ub, tr["Ubar"][0])
    assert np.array_equal(K, tr["K"][0])
    assert float(cost) == info["cost"][0]
    assert (int(iters), int(outer), int(status), int(nls)) == (
        info["iters"][0], info["outer_iters"][0], info["status"][0], info["n_ls_trials"][0])


def _message(t, b):
    """hkd_mpc_example's robot-state message of robot b at tick t (float32 arithmetic, same order)."""
    f = np.float32
    ft, fb = f(t), f(b)
    p = np.array([f(0.001) * ft + f(0.002) * fb, f(0.0005) * fb, f(0.25)], np.float32)
    v = np.array([0.1, 0, 0], np.float32)
    rpy = np.array([f(0.002) * fb, f(0.001) * ft, 0], np.float32)
    om = np.array([0, 0, f(0.01) * fb], np.float32)
    dq = f(0.001) * f(t % 5)
    qJ = np.array([[dq, f(-0.8) + dq, f(1.6) - dq]] * 4, np.float32).reshape(12)
    pf = np.zeros(12, np.float32)
    for leg in range(4):
        pf[3 * leg] = (f(0.2) if leg < 2 else f(-0.2)) + f(0.001) * ft
        pf[3 * leg + 1] = f(0.14) if leg % 2 else f(-0.14)
    return p, v, rpy, om, qJ, pf


def _hkd_state(hsddp, x, contact):
    """compute_hkd_state (HKDModel.h:65-96): stance legs' qdummy = foot position (device FK)."""
    B = x.shape[0]
    xs = np.repeat(x, 4, axis=0)
    pos = hsddp.model.foot_position(xs, np.tile(np.arange(4), B)).reshape(B, 4, 3)
    out = x.copy()
    for b in range(B):
        for leg in range(4):
            if contact[b][leg]:
                out[b, 12 + 3 * leg:15 + 3 * leg] = pos[b, leg]
    return out


@pytest.mark.gpu
def test_mpc_example_matches_python(tmp_path):
    """The C++ HKDMPCSolver (hkd_mpc.hpp: initialize, mpcdata_lcm_handler -> update on the worker
    thread, publish) against the same MPC loop written with the Python mirror (reference_problem,
    advance, update_problem, solve, extract_commands): every command field of every tick equal
    bit for bit (solve_time excepted: a wall-clock reading)."""
    import hsddp
    _make()
    B, ticks = 3, 14
    ref_csv = os.path.join(ROOT, "tests", "golden", "ref_trot.csv")
    info_file = os.path.join(PKG, "settings", "ddp_setting.info")
    r = subprocess.run([os.path.join(PKG, "hkd_mpc_example"), ref_csv, info_file, str(tmp_path), str(B), str(ticks)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(os.path.join(tmp_path, "commands.bin"), dtype=hsddp.MPC_COMMAND).reshape(ticks, B)

    tab, dt = hsddp.load_quad_reference(ref_csv)
    x0 = np.zeros((B, 24)); x0[:, 5] = 0.2486
    x0[:, 12:] = np.tile([0.0, -0.8, 1.6], 4)
    p = hsddp.reference_problem(tab, dt, [0], x0)
    p["x0"] = _hkd_state(hsddp, x0, p["contacts"][:, 0])
    s = hsddp.Solver(p, hsddp.load_settings(info_file))
    s.solve()
    dt_mpc = float(np.float32(0.01))
    for t in range(1, ticks + 1):
        s.set_options(hsddp.load_settings(info_file, max_AL_iter=2, max_DDP_iter=1))
        s.advance(None, 1, 0.6, dt_mpc)
        info = s.phase_info()
        xs = np.zeros((B, 24)); pfs = np.zeros((B, 12), np.float32)
        for b in range(B):
            pp, v, rpy, om, qJ, pf = _message(t, b)
            xs[b, 0:3] = rpy[::-1]; xs[b, 3:6] = pp; xs[b, 6:9] = om; xs[b, 9:12] = v; xs[b, 12:] = qJ
            pfs[b] = pf
        s.update_problem(None, _hkd_state(hsddp, xs, info["contacts"][:, 0]))
        s.solve()
        cmd = s.extract_commands(1, 0.01 * t, dt_mpc, info["durations"], pfs, 0.0)
        for b in range(B):
            for f in ("N_mpcsteps", "mpc_times", "hkd_controls", "des_body_state", "contacts", "statusTimes",
                      "foot_placement", "feedback"):
                assert np.array_equal(got[t - 1][b][f], cmd[b][f]), (t, b, f)
    s.close()
