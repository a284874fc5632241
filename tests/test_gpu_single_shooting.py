"""Single shooting (HSDDP_OPTION::MS = false, `MS 0` in ddp_setting.info) on the GPU against the
oracle.

What the reference does without multiple shooting:
  * SinglePhase::hybrid_rollout (SinglePhase.cpp:181-233) takes X[k+1] = Xsim[k+1] at every knot
    whatever SS_set says (:214-220); a phase's first state stays Xbar[0] + eps dX[0] when SS_set
    holds 0 (:187-193), else x_init;
  * the linear rollout is skipped (MultiPhaseDDP.cpp:326-329), so dX keeps its last values (zero on
    a problem that never ran it);
  * the merit uses the sweep's own dV_1 / dV_2 (SinglePhase.cpp:359-362 summed by
    MultiPhaseDDP::backward_sweep, :224-226; merit at :331-335).
Tolerances as test_gpu_parity.py: 1e-9 relative (or 10x the oracle's own deviation under a 1e-15
relative x0 perturbation) with every branch decision equal; full solves 1e-7 on elements whose
oracle solution is insensitive to that perturbation.
"""
import os

import numpy as np
import pytest

import hsddp
import oracle_lib as O
from hsddp import synthetic as syn

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-300, np.max(np.abs(b))))


def _batch(B, P, N, gait, seed=5):
    """A synthetic batch whose warm starts differ per element.  Without multiple shooting the
    first state of phase 0 stays Xbar[0] + eps dX[0] = Xbar[0] (dX is never computed): x0 enters
    only through that state's Defect, so the elements of one synthetic gait would all follow one
    trajectory; noise on the warm start makes every element its own problem."""
    prob = syn.make_batch(B, P, N, gait)
    rng = np.random.default_rng(seed)
    prob["Xbar"] = prob["Xbar"] + 0.01 * rng.standard_normal(prob["Xbar"].shape)
    return prob


def _run(prob, weights=None, **kw):
    s = hsddp.Solver(prob, hsddp.load_settings(MS=0, **kw), weights=weights)
    s.solve()
    out = {**s.trajectory(), **s.working(), **s.element_info()}
    out["hist"] = s.solver_info()["cost"]
    s.close()
    return out


@pytest.mark.parametrize("n_iter", [1, 3])
@pytest.mark.parametrize("gait,P,N", [("trot", 4, 50), ("jump", 8, 25), ("pronk", 4, 20)])
def test_fixed_iterations_match_oracle(gait, P, N, n_iter):
    prob = _batch(8, P, N, gait)
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=n_iter)
    g = _run(prob, **kw)
    r = O.solve_batch(prob, O.default_options(MS=0, **kw), n_threads=8)
    p2 = dict(prob); p2["x0"] = prob["x0"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(MS=0, **kw), n_threads=8)
    for f in ("Xbar", "Ubar", "K", "X", "U", "dU"):
        assert rel(g[f], r[f]) < max(1e-9, 10 * rel(r2[f], r[f])), f
    for f in ("cost", "feas", "max_tconstr", "merit"):
        assert rel(g[f], r[f]) < max(1e-9, 10 * rel(r2[f], r[f])), f
    for f in ("iters", "outer_iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f], r[f]), f
    # no linear rollout: dX is never written (zero on a new problem), and within a phase X = Xsim
    # (Defect zero past each phase's first state)
    assert np.all(g["dX"] == 0)


def test_per_element_layouts_match_oracle():
    """MS 0 on a mixed-gait batch (config C4's per-element layouts, jumps on 8 x 25 beside 4 x 50):
    each element's own phase walk in the sweep (Bufs::pairs), in k_rollout_ss and in the decisions."""
    prob = syn.make_batch(6, 4, 50, "trot", mixed=True)
    rng = np.random.default_rng(11)
    prob["Xbar"] = prob["Xbar"] + 0.01 * rng.standard_normal(prob["Xbar"].shape)
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2)
    g = _run(prob, **kw)
    r = O.solve_batch(prob, O.default_options(MS=0, **kw), n_threads=6)
    p2 = dict(prob); p2["x0"] = prob["x0"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(MS=0, **kw), n_threads=6)
    for f in ("Xbar", "Ubar", "K", "X", "U", "dU", "cost", "feas"):
        assert rel(g[f], r[f]) < max(1e-9, 10 * rel(r2[f], r[f])), f
    for f in ("iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f], r[f]), f


@pytest.mark.parametrize("gait,P,N", [("trot", 4, 50), ("jump", 8, 25)])
def test_full_solve_matches_oracle(gait, P, N):
    """The shipped settings with MS 0: early exits, AL / ReB outer loop, graph-replayed iterations.
    The rounding envelope comes from a 1e-15 relative perturbation of the warm start (x0 enters a
    single-shooting solve only through the first Defect, and moving it by 1e-15 changes nothing):
    measured on the oracle, trot elements move by up to 4e-5 over 50 iterations under it (element
    15), jump elements by 1e-14.  Each element is held to max(1e-7, 10x its own envelope)."""
    B = 16
    prob = _batch(B, P, N, gait)
    g = _run(prob)
    r = O.solve_batch(prob, O.default_options(MS=0), n_threads=8)
    p2 = dict(prob); p2["Xbar"] = prob["Xbar"] * (1 + 1e-15)
    r2 = O.solve_batch(p2, O.default_options(MS=0), n_threads=8)
    chaotic = {b for b in range(B) if r["n_ls_trials"][b] != r2["n_ls_trials"][b]
               or r["iters"][b] != r2["iters"][b]}
    ok = [b for b in range(B) if b not in chaotic]
    assert len(ok) >= B - 2, sorted(chaotic)
    for f in ("iters", "outer_iters", "status", "n_ls_trials"):
        assert np.array_equal(g[f][ok], r[f][ok]), f
    for b in ok:
        for f in ("Xbar", "Ubar", "cost"):
            env = rel(r2[f][b], r[f][b])
            assert rel(g[f][b], r[f][b]) < max(1e-7, 10 * env), (b, f, env)
        ho, hp = r["solver_info"][b][:, 0].astype(float), r2["solver_info"][b][:, 0].astype(float)
        hist_env = max(1e-5, 10 * float(np.max(np.abs(hp - ho) / np.abs(ho))))  # entry by entry
        assert np.allclose(g["hist"][b], r["solver_info"][b][:, 0], rtol=hist_env), (b, hist_env)
    for b in sorted(chaotic):
        assert g["status"][b] == r["status"][b], b
        assert np.all(np.isfinite(g["Xbar"][b])), b


def test_single_and_multiple_shooting_differ():
    """The option reaches the device: the same problem under MS 1 and MS 0 takes different steps
    (the oracle agrees with each, test_fixed_iterations_match_oracle and test_gpu_parity)."""
    prob = syn.make_batch(4, 4, 20, "trot")
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2)
    g0 = _run(prob, **kw)
    s = hsddp.Solver(prob, hsddp.load_settings(MS=1, **kw))
    s.solve()
    g1 = {**s.trajectory(), **s.working()}
    s.close()
    assert not np.allclose(g0["Xbar"], g1["Xbar"])
    assert np.any(g1["dX"] != 0)


@pytest.mark.parametrize("B,cap", [(5, None), (200, None), (7, "2")])
def test_retries_match_oracle(monkeypatch, B, cap):
    """backward_sweep_regularized's retries (MultiPhaseDDP.cpp:141-181) with single shooting: the
    parallel retries carry each attempt's dV (Bufs::retry_dv) and k_riccati_select forms the merit
    from the winning one; in-kernel, overflow and sequential paths give one result, the oracle's."""
    if cap:
        monkeypatch.setenv("HSDDP_RETRY_CAP", cap)
    prob = syn.make_batch(B, 2, 10, "trot")
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=3)
    w = hsddp.Weights()
    hsddp._lib.lib().hsddp_default_weights(__import__("ctypes").byref(w))
    w.r_qJd = -0.5
    g = _run(prob, weights=w, **kw)
    monkeypatch.setenv("HSDDP_SEQUENTIAL_RETRY", "1")
    q = _run(prob, weights=w, **kw)
    for f in ("Xbar", "Ubar", "K", "dU", "cost", "merit", "status", "n_ls_trials"):
        assert np.array_equal(g[f], q[f]), f
    sample = list(range(0, B, max(1, B // 8)))
    r = O.solve_batch(prob, O.default_options(MS=0, **kw), n_threads=8, elements=sample, weights={"r_qJd": -0.5})
    assert np.array_equal(g["status"][sample], r["status"]) and np.all(r["status"] == 0)
    assert np.array_equal(g["n_ls_trials"][sample], r["n_ls_trials"])
    for f in ("Xbar", "Ubar", "K", "dU", "merit"):
        assert rel(g[f][sample], r[f]) < 1e-9, f


def test_info_file_ms0(tmp_path):
    """`MS 0` read from a ddp_setting.info file (loadHSDDPSetting, HSDDP_CompoundTypes.h:85) solves."""
    src = open(os.path.join(hsddp.SETTINGS_DIR, "ddp_setting.info")).read()
    lines = [("    MS                      false" if ln.strip().startswith("MS ") else ln) for ln in src.splitlines()]
    assert sum(ln.split()[:2] == ["MS", "false"] for ln in lines) == 1
    f = tmp_path / "ddp_setting_ss.info"
    f.write_text("\n".join(lines) + "\n")
    o = hsddp.load_settings(str(f), no_early_exit=1, max_AL_iter=1, max_DDP_iter=2)
    assert o.MS == 0
    prob = _batch(3, 2, 10, "jump")
    s = hsddp.Solver(prob, o)
    s.solve()
    g = {**s.trajectory(), **s.element_info()}
    s.close()
    r = O.solve_batch(prob, O.default_options(MS=0, no_early_exit=1, max_AL_iter=1, max_DDP_iter=2), n_threads=3)
    assert rel(g["Xbar"], r["Xbar"]) < 1e-9 and np.array_equal(g["n_ls_trials"], r["n_ls_trials"])


def test_fp32_single_shooting_close_to_fp64():
    """C5's fp32 Riccati mode with single shooting: the sweep's dV in fp32 (accumulated in fp64);
    one iteration on trot stays within 1e-4 of the fp64 path (measured 2.6e-5 on Xbar: the gains'
    fp32 rounding is carried through 50-knot single-shot rollouts, against 6.6e-6 per knot with
    multiple shooting)."""
    prob = _batch(8, 4, 50, "trot")
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1)
    g = _run(prob, **kw)
    s = hsddp.Solver(prob, hsddp.load_settings(MS=0, **kw), riccati_fp32=True)
    s.solve()
    f = {**s.trajectory(), **s.element_info()}
    s.close()
    assert np.array_equal(f["n_ls_trials"], g["n_ls_trials"])
    assert rel(f["Xbar"], g["Xbar"]) < 1e-4
    assert rel(f["cost"], g["cost"]) < 1e-4
