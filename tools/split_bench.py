#!/usr/bin/env python3
"""Experiment: the metric batch (trot 4x50, B = 4096) split into G handles of B / G elements, each
on its own stream, iterated from G host threads at once, against one handle of B (the bench).  The
sweep is fp64-issue-bound and the other kernels memory / latency-bound: concurrent groups could
overlap one group's sweep with another's memory phases.  Measured: 2 groups +1-2 %,
4 groups -17 %; with the two groups' sweeps forced to alternate (events between the streams) +2 %:
a 2048-element sweep beside the other group's memory kernels takes 1.4-1.8 ms, about what the
whole batch's sweep takes alone (one wave per SIMD is latency-bound at 12.5 k cycles per knot).

    python tools/split_bench.py [--groups G] [--steps K]   -> one JSON line
"""
import argparse
import json
import os
import sys
import threading
import time

import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
import hsddp  # noqa: E402
from hsddp import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    G, B = args.groups, args.batch
    opt = hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=args.warmup + args.steps)
    sols = []
    for g in range(G):
        prob = synthetic.make_batch(B // G, 4, 50, "trot", first_element=g * (B // G))
        s = hsddp.Solver(prob, opt)
        s.begin()
        s.iterate(args.warmup)
        s.synchronize()
        sols.append(s)
    it0 = sum(int(s.element_info()["iters"].sum()) for s in sols)
    t0 = time.perf_counter()
    ths = [threading.Thread(target=s.iterate, args=(args.steps,)) for s in sols]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for s in sols:
        s.synchronize()
    t1 = time.perf_counter()
    it1 = sum(int(s.element_info()["iters"].sum()) for s in sols)
    print(json.dumps({"groups": G, "batch": B, "steps": args.steps, "ms_per_step": (t1 - t0) / args.steps * 1e3,
                      "traj_iter_per_s": (it1 - it0) / (t1 - t0)}), flush=True)
    for s in sols:
        s.close()


if __name__ == "__main__":
    main()
