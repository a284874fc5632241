"""Host-side checks of the MPC-side steps: the C and numpy layouts of
hsddp_mpc_command agree, and the oracle restatement of update_foot_placement / publish_mpc_cmd
(HKDMPC.cpp:207-298) follows the reference's rules on hand-built cases."""
import os
import subprocess
import sys

import numpy as np
import pytest

import hsddp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import mpc_oracle as M  # noqa: E402


def test_command_record_layout_matches_c(tmp_path):
    fields = [f for f in hsddp.MPC_COMMAND.names]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "hsddp.h"\nint main(void){\n'
                   'printf("%zu\\n", sizeof(hsddp_mpc_command));\n' +
                   "".join(f'printf("%zu\\n", offsetof(hsddp_mpc_command, {f}));\n' for f in fields) +
                   "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == hsddp.MPC_COMMAND.itemsize
    assert vals[1:] == [hsddp.MPC_COMMAND.fields[f][1] for f in fields]


def _traj(horizons, seed=0):
    rng = np.random.default_rng(seed)
    S, Kc = sum(n + 1 for n in horizons), sum(horizons)
    return rng.standard_normal((S, 24)), rng.standard_normal((Kc, 24)), rng.standard_normal((Kc, 24, 24))


def test_command_knot_walk_crosses_phases():
    horizons = [3, 2, 4, 5]
    Xbar, Ubar, K = _traj(horizons)
    contacts = np.array([[1, 0, 0, 1], [0, 1, 1, 0], [1, 0, 0, 1], [0, 1, 1, 0], [1, 0, 0, 1]], np.int32)
    dur = np.arange(16, dtype=float).reshape(4, 4)
    c = M.mpc_command(Xbar, Ubar, K, contacts, horizons, 1, 2.0, 0.01, dur, np.zeros(12), 1.5)
    assert c["N_mpcsteps"] == 8
    # rows 0-2 phase 0 (slots 0..2), 3-4 phase 1 (state slots 4, 5), 5-7 phase 2 (state slots 7..9)
    assert np.array_equal(c["des_body_state"][3], Xbar[4][:12].astype(np.float32))
    assert np.array_equal(c["hkd_controls"][5], Ubar[5].astype(np.float32))
    assert np.array_equal(c["des_body_state"][7], Xbar[9][:12].astype(np.float32))
    assert np.array_equal(c["contacts"][4], contacts[1]) and np.array_equal(c["statusTimes"][6], dur[2])
    assert np.allclose(c["mpc_times"][:8], 2.0 + 0.01 * np.arange(8)) and np.all(c["mpc_times"][8:] == 0)
    assert np.all(c["hkd_controls"][8:] == 0)


def test_foot_placement_search_rules():
    horizons = [2] * 7
    Xbar, _, _ = _traj(horizons, 1)
    s0, _ = M.phase_offsets(horizons)
    cur = np.arange(12, dtype=np.float32)
    # leg 0: swing->stance between phases 1 and 2 (first match wins over the later one at 3->4)
    # leg 1: never touches down -> current position; leg 2: transition only at phase 5->6, beyond
    # the search (i <= 4) -> current; leg 3: transition 4->5 (i = 4, still searched)
    c = np.array([[1, 1, 0, 1], [0, 1, 0, 0], [1, 1, 0, 0], [0, 1, 0, 0], [1, 0, 0, 0],
                  [1, 0, 0, 1], [1, 0, 1, 1], [1, 0, 1, 1]], np.int32)
    pf = M.foot_placement(Xbar, c, horizons, cur)
    assert np.array_equal(pf[0:3], Xbar[s0[2]][12:15].astype(np.float32))
    assert np.array_equal(pf[3:6], cur[3:6]) and np.array_equal(pf[6:9], cur[6:9])
    assert np.array_equal(pf[9:12], Xbar[s0[5]][21:24].astype(np.float32))


def test_shift_working_follows_the_trajectory_edits():
    """mpc_oracle.shift_working (Trajectory::pop_front / push_back_state, TrajectoryManagement.cpp:
    118-207): the working X moves like the nominal (X.back() pushed), U and Defect get zero rows,
    a new phase is zero; with X = Xbar it reproduces shift()'s Xbar."""
    horizons, reach = [3, 2, 4], [0, 0, 0]
    X, U, _ = _traj(horizons, 2)
    D = np.random.default_rng(3).standard_normal(X.shape)
    flags = [1, 1, 0]  # mark the end, then a new phase, then grow it
    hz, ss, re, Xb, Ub, _ = M.shift(horizons, [n + 1 for n in horizons], reach, X, X, U, np.zeros((9, 24, 24)), flags)
    Xw, Uw, Dw = M.shift_working(horizons, reach, X, U, D, flags)
    # [3, 2, 4] -> pop, push (end reached) [2, 2, 5] -> pop, new phase [1, 2, 5, 1] -> phase 0 gone, push [2, 5, 2]
    assert hz == [2, 5, 2] and np.array_equal(Xw, Xb)
    assert np.array_equal(Uw[0], U[3]) and not Ub[0].any()            # Ubar[0] zeroed, U[0] kept
    assert np.array_equal(Uw[:6], U[3:9]) and not Uw[6:].any()         # pushed knot and new phase: zero
    assert np.array_equal(Dw[:8], D[4:12]) and not Dw[8:].any()        # pushed state and new phase: zero


def test_shift_constraints_carries_stored_values():
    """The constraint objects' stored values follow their knots and constraints (PathConstraintBase::
    pop_front / push_back, ConstraintsBase.h:271-291): a pushed knot's GRF row and a new phase's are
    zero, a newly registered touchdown constraint's residual is zero, the others move unchanged."""
    horizons, reach = [3, 2, 4], [0, 0, 0]
    rng = np.random.default_rng(5)
    cons = {"reb_delta": rng.random((9, 20)), "reb_eps": rng.random((9, 20)),
            "td_mask": np.array([[3, 0, 0, 0], [0, 0, 0, 0], [12, 0, 0, 0]], np.int32),
            "al_sigma": rng.random((3, 4, 4)), "al_lambda": rng.random((3, 4, 4)),
            "grf_g": rng.random((9, 20)), "td_h": rng.random((3, 4, 4)) * (np.arange(4) == 0)[None, :, None]}
    out = M.shift_constraints(horizons, reach, cons, [1, 0], 0.1, 0.1, 50.0, 0.0)
    # step 1: pop knot 0, push a zero knot on the last phase, mark its end -> a pending constraint
    # step 2: pop knot 1 (phase 0 keeps knot 2), push another zero knot, one more pending constraint
    assert np.array_equal(out["grf_g"][:7], cons["grf_g"][2:9])
    assert not out["grf_g"][7:].any()
    assert np.array_equal(out["td_h"][:, 0], cons["td_h"][:, 0])
    assert list(out["td_mask"][2]) == [12, M.TD_PENDING, M.TD_PENDING, 0]
    assert not out["td_h"][2, 1:].any()
