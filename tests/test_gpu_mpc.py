"""GPU checks of the MPC-side steps through the C-ABI against oracle/mpc_oracle.py.

Command extraction (update_foot_placement + publish_mpc_cmd, HKDMPC.cpp:207-298) is data movement
and double -> float conversion: bit-exact against the restatement applied to the downloaded
trajectory, for mixed per-element gaits (per-element contacts and foot-placement searches), short
phases (the knot walk crosses phase boundaries) and the fp32 Riccati mode (gains held in fp32).
"""
import os
import sys

import numpy as np
import pytest

import hsddp
from hsddp import synthetic as syn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import mpc_oracle as M  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P,N,mixed,fp32,nsteps", [(4, 3, True, False, 1), (8, 2, True, False, 3),
                                                     (4, 50, False, False, 1), (6, 4, True, True, 2)])
def test_commands_match_oracle(P, N, mixed, fp32, nsteps):
    B = 37
    prob = syn.make_batch(B, P, N, "jump" if P == 8 else "trot", mixed=mixed)
    s = hsddp.Solver(prob, hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2), riccati_fp32=fp32)
    s.solve()
    tr = s.trajectory()
    rng = np.random.default_rng(P * N)
    dur = rng.uniform(0.1, 0.4, (B, P, 4))
    feet = rng.standard_normal((B, 12)).astype(np.float32)
    cmd = s.extract_commands(nsteps, 3.25, 0.01, dur, feet, 0.75)
    # shared (non-per-element) durations / feet
    cmd1 = s.extract_commands(nsteps, 3.25, 0.01, dur[0], feet[0], 0.75)
    s.close()
    for b in range(B):
        for variant, d_, f_ in ((cmd, dur[b], feet[b]), (cmd1, dur[0], feet[0])):
            r = M.mpc_command(tr["Xbar"][b], tr["Ubar"][b], tr["K"][b], prob["contacts"][b], prob["horizons"],
                              nsteps, 3.25, 0.01, d_, f_, 0.75)
            g = variant[b]
            for f in ("N_mpcsteps", "mpc_times", "hkd_controls", "des_body_state", "contacts", "statusTimes",
                      "foot_placement", "feedback", "solve_time"):
                assert np.array_equal(g[f], r[f]), (b, f)


def test_async_commands_equal_sync_across_ticks():
    """hsddp_extract_commands_async: the records of tick t, copied on the handle's copy stream while
    tick t + 1 is shifted and re-solved, equal the synchronous extraction of tick t field for field;
    the two pinned buffers alternate and a buffer is reused only after its copy completed."""
    B, P, N = 19, 4, 5
    sc, prob = _scenario_batch(B, P, N)
    s = hsddp.Solver(prob, hsddp.load_settings(max_AL_iter=2, max_DDP_iter=1))
    s.solve()
    rng = np.random.default_rng(11)
    pending = None
    for it in range(7):
        dur = rng.uniform(0.1, 0.4, (B, len(s.layout()["horizons"]), 4))
        feet = rng.standard_normal((B, 12)).astype(np.float32)
        want = s.extract_commands(1, 0.01 * it, 0.01, dur, feet, 0.5)
        ticket = s.extract_commands_async(1, 0.01 * it, 0.01, dur, feet, 0.5)
        assert ticket == it % 2
        if pending is not None:  # the previous tick's records, copied during this tick's work
            _same_records(s.commands_wait(pending[0]), pending[1], it)
        pending = (ticket, want)
        flags = sc.step(1)
        s.shift(flags)
        inp = sc.inputs(prob["x0"])
        s.update_problem(inp["contacts"], inp["x0"], inp["ref_x"], inp["ref_u"], inp["ref_foot"])
        s.solve()
    _same_records(s.commands_wait(pending[0]), pending[1], "last")
    s.close()


def _same_records(a, b, where):
    for f in a.dtype.names:  # field by field (the record has padding bytes nothing writes)
        assert np.array_equal(a[f], b[f]), (where, f)


# ---- receding-horizon update (HKDProblem::update, HKDProblem.cpp:117-222) --------------------
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_lib as O  # noqa: E402
from mpc_scenario import Scenario  # noqa: E402


def _scenario_batch(B, P, N):
    names = ["trot", "pace", "bound", "pronk"]
    gaits = [names[b % 4] for b in range(B)]
    sc = Scenario(gaits, P, N)
    prob = syn.make_batch(B, P, N, "trot")
    inp = sc.inputs(prob["x0"])
    prob.update(inp)
    prob["Xbar"] = inp["ref_x"].copy()
    return sc, prob


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


@pytest.mark.parametrize("steps", [[1, 1, 1, 1, 1, 1, 1], [3, 4, 2], [9]])
def test_shift_matches_oracle(steps):
    """The device gather reproduces the restated phase bookkeeping bit for bit: dropped front knots
    and phases, X.back() copies, zero new phases, Ubar[0] zeroed; layout and shooting sets agree."""
    B, P, N = 6, 4, 5
    sc, prob = _scenario_batch(B, P, N)
    s = hsddp.Solver(prob, hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2))
    s.solve()
    for n in steps:
        before = {**s.trajectory(), **s.working()}
        lay0 = s.layout()
        flags = sc.step(n)
        lay = s.shift(flags)
        assert lay["horizons"] == sc.horizons and lay["reach_end"] == sc.reach_end
        ref = [M.shift(lay0["horizons"], lay0["shooting"], lay0["reach_end"], before["Xbar"][b], before["X"][b],
                       before["Ubar"][b], before["K"][b], flags) for b in range(B)]
        assert lay["shooting"] == ref[0][1]
        with pytest.raises(hsddp.HSDDPError):
            s.solve()  # inputs of the new layout are required first
        inp = sc.inputs(np.stack([r[3][0] for r in ref]))
        s.update_problem(inp["contacts"], inp["x0"], inp["ref_x"], inp["ref_u"], inp["ref_foot"])
        tr = s.trajectory()
        for b in range(B):
            assert np.array_equal(tr["Xbar"][b], ref[b][3])
            assert np.array_equal(tr["Ubar"][b], ref[b][4])
            assert np.array_equal(tr["K"][b], ref[b][5])
        s.solve()
    s.close()


@pytest.mark.parametrize("ms", [1, 0])
def test_mpc_loop_matches_oracle(ms):
    """HKDMPCSolver::update's loop (HKDMPC.cpp:96-165): shift one step, new inputs with the warm
    start kept, re-solve with max_AL_iter = 2, max_DDP_iter = 1 (quirk A17) — including the
    updates whose new last phase has no shooting states — against the oracle doing the same; with
    multiple (MS 1) and single (MS 0) shooting."""
    B, P, N = 8, 4, 5
    sc, prob = _scenario_batch(B, P, N)
    s = hsddp.Solver(prob, hsddp.load_settings(MS=ms))
    s.solve()
    r = O.solve_batch(prob, O.default_options(MS=ms), n_threads=8)
    g = {**s.trajectory(), **s.working(), **s.element_info()}
    assert _rel(g["Xbar"], r["Xbar"]) < 1e-9
    kw = dict(max_AL_iter=2, max_DDP_iter=1, MS=ms)
    s.set_options(hsddp.load_settings(**kw))
    tails = n_td = 0
    op, _ = O.default_problem(prob["horizons"], prob["dt"])  # the initial ReB / AL parameters
    for it in range(9):
        lay0 = s.layout()
        flags = sc.step(1)
        lay = s.shift(flags)
        tails += any(ss < n + 1 for ss, n in zip(lay["shooting"], lay["horizons"]))
        sh = [M.shift(lay0["horizons"], lay0["shooting"], lay0["reach_end"], r["Xbar"][b], r["X"][b],
                      r["Ubar"][b], r["K"][b], flags) for b in range(B)]
        inp = sc.inputs(np.stack([q[3][0] for q in sh]))
        # the constraint objects live on: ReB / AL parameters carried over, one more touchdown
        # constraint on a last phase that has reached its end (HKDProblem.cpp:199-202)
        cons = [M.resolve_td(M.shift_constraints(lay0["horizons"], lay0["reach_end"],
                                                 {k: r[k][b] for k in O.CONSTRAINT_FIELDS}, flags, op.grf_delta,
                                                 op.grf_eps, op.td_sigma, op.td_lambda), inp["contacts"][b])
                for b in range(B)]
        cons = {k: np.stack([c[k] for c in cons]) for k in O.CONSTRAINT_FIELDS}
        s.update_problem(inp["contacts"], inp["x0"], inp["ref_x"], inp["ref_u"], inp["ref_foot"])
        s.solve()
        g = {**s.trajectory(), **s.working(), **s.element_info()}
        p2 = {"batch": B, "horizons": lay["horizons"], "shooting": lay["shooting"], "dt": prob["dt"],
              "S": sum(n + 1 for n in lay["horizons"]), "Kc": sum(lay["horizons"]), **inp,
              "Xbar": np.stack([q[3] for q in sh]), "Ubar": np.stack([q[4] for q in sh]),
              "K": np.stack([q[5] for q in sh])}
        r = O.solve_batch(p2, O.default_options(**kw), n_threads=8, constraints=cons)
        dc = s.constraint_params()
        assert np.array_equal(dc["td_mask"], r["td_mask"]), it
        n_td = max(n_td, int((dc["td_mask"] != 0).sum(axis=2).max()))
        for f in ("al_sigma", "al_lambda", "reb_delta", "reb_eps"):
            assert _rel(dc[f], r[f]) < 1e-9, (it, f)
        for f in ("Xbar", "Ubar", "X", "K"):
            assert _rel(g[f], r[f]) < 1e-8, (it, f)
        assert np.array_equal(g["n_ls_trials"], r["n_ls_trials"]), it
        assert _rel(g["cost"], r["cost"]) < 1e-9, it
    assert tails >= 2  # the loop passed through last phases without shooting states
    assert n_td >= 1   # (phases carrying two touchdown constraints: test_gpu_reference.py's file-driven loop)
    s.close()


def test_command_records_are_the_same_bytes_wherever_extracted():
    """hsddp_mpc_command has padding (after N_mpcsteps and after solve_time).  The extraction
    kernel writes every byte of a record, so records extracted into buffers that held different
    bytes — device memory from any allocator, the handle's scratch for the host path — compare
    equal byte for byte (the multi-GPU gather sends the records as bytes).  Device buffers come
    from the HIP runtime the library uses (no torch: this module may load before it)."""
    import ctypes as C
    from hsddp import shard
    hip = C.CDLL("libamdhip64.so")
    prob = syn.make_batch(8, 4, 20, "trot", mixed=True)
    s = hsddp.Solver(prob, hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2))
    s.solve()
    n = prob["batch"] * hsddp.MPC_COMMAND.itemsize
    out = []
    for fill in (0xAB, 0x11):
        ptr = C.c_void_p()
        assert hip.hipMalloc(C.byref(ptr), C.c_size_t(n)) == 0
        assert hip.hipMemset(ptr, C.c_int(fill), C.c_size_t(n)) == 0
        s.extract_commands_device(ptr.value)
        host = np.empty(n, np.uint8)
        assert hip.hipMemcpy(C.c_void_p(host.ctypes.data), ptr, C.c_size_t(n), C.c_int(2)) == 0  # device to host
        assert hip.hipFree(ptr) == 0
        out.append(host)
    ref = shard.command_bytes(s.extract_commands())
    s.close()
    assert np.array_equal(out[0], out[1])
    assert np.array_equal(out[0], ref)
