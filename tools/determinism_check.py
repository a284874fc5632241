#!/usr/bin/env python3
"""Bitwise determinism of the GPU path: the same problem solved twice in one process, and (with
--save/--compare) across processes.  python tools/determinism_check.py [--fp32] [--save F | --compare F]"""
import argparse
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
import hsddp  # noqa: E402
from hsddp import synthetic as syn  # noqa: E402


def solve(prob, fp32, **kw):
    s = hsddp.Solver(prob, hsddp.load_settings(**kw), riccati_fp32=fp32)
    s.solve()
    out = {**s.trajectory(), **s.element_info()}
    s.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--save")
    ap.add_argument("--compare")
    ap.add_argument("--gait", default="jump")
    a = ap.parse_args()
    P, N = (8, 25) if a.gait == "jump" else (4, 50)
    prob = syn.make_batch(4096, P, N, a.gait)
    for kw in (dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=10), {}):
        r1, r2 = solve(prob, a.fp32, **kw), solve(prob, a.fp32, **kw)
        bad = {f: int(np.sum(np.any((r1[f] != r2[f]).reshape(4096, -1), axis=1))) for f in ("Xbar", "Ubar", "K", "cost", "n_ls_trials")}
        print("in-process", kw or "shipped settings", "elements differing:", bad, flush=True)
        tag = "fixed" if kw else "full"
        crc = np.array([zlib.crc32(r1["Xbar"][b].tobytes()) for b in range(4096)], dtype=np.uint64)
        if a.save:
            np.save(f"{a.save}_{tag}.npy", crc)
        if a.compare:
            z = np.load(f"{a.compare}_{tag}.npy")
            print("cross-process", tag, "elements differing:", int(np.sum(z != crc)), flush=True)


if __name__ == "__main__":
    main()
