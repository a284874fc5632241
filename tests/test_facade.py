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
    r = subprocess.run(["make", "-C", os.path.join(PKG, "facade")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_facade_builds_and_checks():
    _make()
    r = subprocess.run([os.path.join(PKG, "facade_check"), os.path.join(PKG, "settings", "ddp_setting.info")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade_check ok" in r.stdout


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
    s.solve()
    tr, info = s.trajectory(), s.element_info()
    s.close()
    assert np.array_equal(Xb, tr["Xbar"][0])
    assert np.array_equal(Ub, tr["Ubar"][0])
    assert np.array_equal(K, tr["K"][0])
    assert float(cost) == info["cost"][0]
    assert (int(iters), int(outer), int(status), int(nls)) == (
        info["iters"][0], info["outer_iters"][0], info["status"][0], info["n_ls_trials"][0])
