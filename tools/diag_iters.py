#!/usr/bin/env python3
"""GPU vs oracle, iteration by iteration, on a few synthetic elements: statuses, line-search trial
counts and the largest relative deviation of the nominal trajectory after each inner iteration.

    python tools/diag_iters.py [gait P N n_iter elem ...]
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


def stack(idx, P, N, gait):
    ps = [syn.make_batch(1, P, N, gait, first_element=i) for i in idx]
    q = dict(ps[0]); q["batch"] = len(idx)
    for k in ("contacts", "x0", "Xbar", "Ubar"):
        q[k] = np.concatenate([p[k] for p in ps])
    return q


def main():
    a = sys.argv[1:]
    gait, P, N, n_iter = (a[0], int(a[1]), int(a[2]), int(a[3])) if a else ("jump", 8, 25, 12)
    elems = [int(x) for x in a[4:]] or [377, 760, 656, 321, 0]
    prob = stack(elems, P, N, gait)
    for it in range(1, n_iter + 1):
        kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=it)
        s = hsddp.Solver(prob, hsddp.load_settings(**kw))
        s.solve()
        g = {**s.trajectory(), **s.element_info()}
        s.close()
        r = O.solve_batch(prob, O.default_options(**kw), n_threads=8)
        dev = [float(np.max(np.abs(g["Xbar"][j] - r["Xbar"][j])) / max(1e-300, np.max(np.abs(r["Xbar"][j]))))
               for j in range(len(elems))]
        dk = [float(np.max(np.abs(g["K"][j] - r["K"][j])) / max(1e-300, np.max(np.abs(r["K"][j]))))
              for j in range(len(elems))]
        print(f"it {it:2d} status gpu {list(g['status'])} orc {list(r['status'])} "
              f"ls gpu {list(g['n_ls_trials'])} orc {list(r['n_ls_trials'])}\n"
              f"      Xbar dev {['%.1e' % v for v in dev]}  K dev {['%.1e' % v for v in dk]}", flush=True)


if __name__ == "__main__":
    main()
