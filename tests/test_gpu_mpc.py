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
