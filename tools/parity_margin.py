#!/usr/bin/env python3
"""Parity margins of the fixed-iteration GPU tests (tests/test_gpu_parity.py): the largest
relative deviation from the oracle per field, for the library HSDDP_LIB selects.  Test
infrastructure only (imports the oracle as the checker).

    HSDDP_LIB=... python tools/parity_margin.py
"""
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hsddp  # noqa: E402
import oracle_lib as O  # noqa: E402
from hsddp import synthetic as syn  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-300, np.max(np.abs(b))))


for gait, P, N in (("trot", 4, 50), ("jump", 8, 25), ("pronk", 4, 20)):
    for n_iter in (1, 3):
        prob = syn.make_batch(8, P, N, gait)
        kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=n_iter)
        s = hsddp.Solver(prob, hsddp.load_settings(**kw))
        s.solve()
        g = {**s.trajectory(), **s.working(), **s.element_info()}
        s.close()
        r = O.solve_batch(prob, O.default_options(**kw), n_threads=8)
        errs = {f: rel(g[f], r[f]) for f in ("Xbar", "Ubar", "K", "X", "U", "dX", "dU", "cost")}
        same = all(np.array_equal(g[f], r[f]) for f in ("iters", "status", "n_ls_trials"))
        print(f"{gait:5s} it={n_iter} decisions_equal={same} " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()))
