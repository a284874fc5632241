#!/usr/bin/env python3
"""MPC tick benchmark: the reference's HKDMPCSolver::update loop for a
batch of robots driven by the reference's trot data (tests/golden/ref_trot.csv, 0.6 s plan =
60 knots), per tick: hsddp_advance (HKDProblem::update: host bookkeeping, k_shift_gather,
k_build_refs, inputs), hsddp_solve with max_AL_iter = 2, max_DDP_iter = 1 (quirk A17), and
hsddp_extract_commands (k_extract_commands).  Every C-ABI call returns synchronised, so the
wall-clock split is per stage; kernel durations come from rocprofv3 over the same script.

    python tools/mpc_bench.py [--batch B] [--ticks T]     -> one JSON line
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (binds the library to torch's HIP runtime, as bench.py does)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
import hsddp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--sync", action="store_true",
                    help="synchronous extraction into pageable memory (round 3's path) instead of the "
                         "asynchronous copy into the handle's pinned buffers")
    args = ap.parse_args()
    B = args.batch
    tab, dt = hsddp.load_quad_reference(os.path.join(ROOT, "tests", "golden", "ref_trot.csv"))
    rng = np.random.default_rng(7)
    x0 = np.zeros((B, 24))
    x0[:, 5] = 0.25
    x0[:, 12:] = np.tile(np.float32([.2, -.14, 0, .2, .14, 0, -.2, -.14, 0, -.2, .14, 0]), 1)
    x0[:, 6:12] += rng.uniform(-.2, .2, (B, 6))
    p = hsddp.reference_problem(tab, dt, [0], x0)
    s = hsddp.Solver(p, hsddp.load_settings())
    s.solve()
    s.set_options(hsddp.load_settings(max_AL_iter=2, max_DDP_iter=1))
    feet = np.tile(np.float32([.2, -.14, 0, .2, .14, 0, -.2, -.14, 0, -.2, .14, 0]), (B, 1))
    t_adv, t_solve, t_cmd = [], [], []
    flags = 0
    ticket, cmd, t_last = None, None, 0.0
    for it in range(args.ticks):
        xt = x0 + rng.uniform(-.01, .01, x0.shape)
        t0 = time.perf_counter()
        flags += sum(s.advance(xt, 1))
        t1 = time.perf_counter()
        s.solve()
        t2 = time.perf_counter()
        info = s.phase_info()
        t3 = time.perf_counter()
        if args.sync:
            cmd = s.extract_commands(1, 0.01 * (it + 1), float(np.float32(0.01)), info["durations"], feet, 0.0)
        else:  # the records of tick t cross PCIe during tick t + 1's advance and solve
            if ticket is not None:
                cmd = s.commands_wait(ticket, copy=False)
            ticket = s.extract_commands_async(1, 0.01 * (it + 1), float(np.float32(0.01)), info["durations"], feet,
                                              0.0)
        t4 = time.perf_counter()
        t_adv.append(t1 - t0); t_solve.append(t2 - t1); t_cmd.append(t4 - t3)
    if not args.sync:
        t5 = time.perf_counter()
        cmd = s.commands_wait(ticket, copy=False)
        t_last = time.perf_counter() - t5
    lay = s.layout()
    finite = bool(np.isfinite(s.element_info()["cost"]).all()) and bool(np.isfinite(cmd["hkd_controls"]).all())
    S, Kc = sum(n + 1 for n in lay["horizons"]), sum(lay["horizons"])
    # k_shift_gather moves every element's warm start once: Xbar [S][24], Ubar [Kc][24] and the
    # compact gains [Kc][12][24] read (gathered) and written
    shift_bytes = 2 * B * (S * 24 + Kc * 24 + Kc * 12 * 24) * 8
    med = lambda v: float(np.median(v)) * 1e3  # noqa: E731
    out = {"metric": "MPC tick (advance + solve + extract), HKD trot reference file", "batch": B,
           "ticks": args.ticks, "plan_knots": Kc, "final_horizons": lay["horizons"], "contact_change_steps": flags,
           "ms_per_tick_median": {"advance": med(t_adv), "solve": med(t_solve), "extract_commands": med(t_cmd)},
           "extract_mode": "sync (pageable)" if args.sync else "async (pinned, overlapped with the next tick)",
           "last_copy_wait_ms": t_last * 1e3,
           "robot_ticks_per_s": B / (np.median(t_adv) + np.median(t_solve) + np.median(t_cmd)),
           "shift_gather_algorithmic_bytes": shift_bytes, "all_finite": finite}
    print(json.dumps(out), flush=True)
    s.close()


if __name__ == "__main__":
    main()
