#!/usr/bin/env python3
"""Config C5's tail: which full trot solves of the fp32 Riccati mode end
away from the fp64 solve, and is that fp32's doing or the problem's own sensitivity?

Full solves with the shipped settings (AL + ReB outer loop, early exits) of the C5 batch (trot
4 x 50, B = 4096, the bench's synthetic batch) in fp64 from x0 and from x0 (1 + delta) for several
relative perturbations delta, and in the fp32 Riccati mode from x0.  For each run against the
unperturbed fp64 solve: the number of elements whose final cost differs by more than 1e-6 / 1e-3
(relative) and the elements with equal decisions (inner / outer iterations and line-search trial
counts).  The fp32 tail elements are then looked up in the perturbed fp64 runs: an element that also
parts under a 1e-9 perturbation of x0 in fp64 is sensitive in itself; fp32's gains carry ~1e-7
relative rounding, so a delta of 1e-7 is the like-for-like comparison.

Writes gpurun_out/fp32_tail.json (commit a copy under profiles/).
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
import hsddp  # noqa: E402
from hsddp import synthetic as syn  # noqa: E402


def solve(prob, fp32, delta):
    p = dict(prob)
    p["x0"] = prob["x0"] * (1 + delta)
    s = hsddp.Solver(p, hsddp.load_settings(), riccati_fp32=fp32)
    s.solve()
    info = s.element_info()
    hist = s.solver_info()["cost"]
    trace = np.zeros((s.B, 16), np.uint64)  # HSDDP_TRACE's per-iteration decisions (k_decide)
    hsddp.lib().hsddp_debug_stamps(s._h, trace.ctypes.data_as(ctypes.c_void_p))
    s.close()
    return {"cost": info["cost"], "iters": info["iters"], "outer": info["outer_iters"], "n_ls": info["n_ls_trials"],
            "status": info["status"], "hist": hist, "trace": trace}


def decisions(trace_row, n):
    """(trials, accepted, round(log2 mu) or None) of inner iterations 0 .. n - 1"""
    out = []
    for it in range(min(n, 64)):
        v = int((int(trace_row[it // 4]) >> (16 * (it % 4))) & 0xffff)
        code = v >> 4
        out.append((v & 7, (v >> 3) & 1, None if code == 0 else code - 64))
    return out


def compare(a, b):
    dc = np.abs(b["cost"] - a["cost"]) / np.maximum(np.abs(a["cost"]), 1e-30)
    same = (a["iters"] == b["iters"]) & (a["outer"] == b["outer"]) & (a["n_ls"] == b["n_ls"])
    return dc, same


def main():
    os.environ["HSDDP_TRACE"] = "1"
    B = int(os.environ.get("TAIL_B", "4096"))
    prob = syn.make_batch(B, 4, 50, "trot")
    base = solve(prob, False, 0.0)
    runs = {"fp32": solve(prob, True, 0.0)}
    for d in (1e-15, 1e-12, 1e-9, 1e-7):
        runs[f"fp64_x0_delta_{d:g}"] = solve(prob, False, d)
    out = {"batch": B, "workload": "trot 4x50, shipped ddp_setting.info (max_AL_iter 5, max_DDP_iter 10, early exits)",
           "runs": {}}
    dcs = {}
    for k, r in runs.items():
        dc, same = compare(base, r)
        dcs[k] = dc
        out["runs"][k] = {"n_gt_1e-6": int(np.sum(dc > 1e-6)), "n_gt_1e-3": int(np.sum(dc > 1e-3)),
                          "max": float(dc.max()), "median": float(np.median(dc)),
                          "frac_same_decisions": float(np.mean(same)),
                          "status_agreement": float(np.mean(r["status"] == base["status"]))}
    tail = np.nonzero(dcs["fp32"] > 1e-3)[0]
    out["fp32_tail_elements"] = [int(b) for b in tail]
    # the fp32 tail in the perturbed fp64 runs: how far each of those elements moves there
    out["fp32_tail_in_fp64_perturbed"] = {k: [float(dcs[k][b]) for b in tail] for k in runs if k != "fp32"}
    for thr in (1e-3, 1e-6):
        t = np.nonzero(dcs["fp32"] > thr)[0]
        out[f"fp32_tail_{thr:g}_also_parting_fp64_delta_1e-7"] = float(np.mean(dcs["fp64_x0_delta_1e-07"][t] > thr)) if len(t) else None
        out[f"fp32_tail_{thr:g}_also_parting_fp64_delta_1e-9"] = float(np.mean(dcs["fp64_x0_delta_1e-09"][t] > thr)) if len(t) else None
    # where each fp32 tail element's decisions first part from fp64's: a different trial count /
    # acceptance (a merit comparison across the line search's test) or a different regularisation
    # (a Quu pivot across the PSD test, MultiPhaseDDP.cpp:141-181)
    part = []
    a, f = base, runs["fp32"]
    for b in tail:
        da = decisions(a["trace"][b], int(a["iters"][b]))
        df = decisions(f["trace"][b], int(f["iters"][b]))
        first = next((i for i, (x, y) in enumerate(zip(da, df)) if x != y), None)
        kind = None
        if first is not None:
            x, y = da[first], df[first]
            kind = "regularisation (PSD test)" if x[2] != y[2] else "line search (merit test)"
        part.append({"element": int(b), "cost_rel_diff": float(dcs["fp32"][b]), "first_parting_iteration": first,
                     "kind": kind, "fp64": da[first] if first is not None else None,
                     "fp32": df[first] if first is not None else None,
                     "iters": [int(a["iters"][b]), int(f["iters"][b])]})
    out["fp32_tail_decisions"] = part
    kinds = [q["kind"] for q in part]
    out["fp32_tail_parting_kinds"] = {k: kinds.count(k) for k in set(kinds)}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "fp32_tail.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("fp32_tail_in_fp64_perturbed", "runs")}))


if __name__ == "__main__":
    main()
