#!/usr/bin/env python3
"""Config C5: fp32 Riccati mode against the fp64 path — tolerance and throughput.

Writes gpurun_out/fp32_tolerance.json:
  * one fixed inner iteration, trot 4x50, B = 64: fp32 gains K / dU / dX against the oracle (fp64);
  * 10 fixed inner iterations, B = 4096 (C5 batch): cost / feasibility of fp32 vs fp64 GPU runs,
    line-search decisions that differ, time per inner iteration of each;
  * full solves with the shipped settings (AL + ReB outer loop, early exits), B = 4096, trot 4x50
    and jump 8x25: final cost relative difference (median / p99 / max), statuses, iterations;
  * impact-heavy jump 8x25 (7 reset boundaries), B = 4096, 1 and 3 fixed inner iterations: the
    "flip" rate — elements whose line-search trial count or status differs from the fp64 path (an
    fp32 rounding that moves a Quu pivot across the PSD threshold or a merit comparison across
    acceptance changes the element's branch) — and, on the elements that did not flip, the
    per-element relative difference of K, dU, dX, Xbar, Ubar and cost against the fp64 path.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hsddp  # noqa: E402
import oracle_lib as O  # noqa: E402
from hsddp import synthetic as syn  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def run(prob, fp32, **kw):
    s = hsddp.Solver(prob, hsddp.load_settings(**kw), riccati_fp32=fp32)
    t0 = time.perf_counter()
    st = s.solve()
    dt = time.perf_counter() - t0
    out = {**s.trajectory(), **s.working(), **s.element_info(), "wall_s": dt, "ms_total": st.ms_total,
           "elem_iters": st.element_iterations}
    s.close()
    return out


def per_element_rel(a, b):
    """max |a - b| / max |b| per element (leading axis)"""
    a = np.asarray(a).reshape(len(a), -1); b = np.asarray(b).reshape(len(b), -1)
    return np.max(np.abs(a - b), axis=1) / np.maximum(1e-300, np.max(np.abs(b), axis=1))


def flips(prob, iters):
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=iters)
    a, b = run(prob, False, **kw), run(prob, True, **kw)
    flip = (a["n_ls_trials"] != b["n_ls_trials"]) | (a["status"] != b["status"])
    keep = ~flip
    out = {"elements": int(len(flip)), "flip_rate": float(np.mean(flip)), "flipped": int(flip.sum()),
           "status_fp32_nonzero": int(np.sum(b["status"] != 0)), "status_fp64_nonzero": int(np.sum(a["status"] != 0))}
    for f in ("K", "dU", "dX", "Xbar", "Ubar", "cost"):
        e = per_element_rel(b[f], a[f])[keep]
        out[f"nonflip_{f}_rel_max"] = float(e.max()) if e.size else None
        out[f"nonflip_{f}_rel_p99"] = float(np.quantile(e, .99)) if e.size else None
    return out


def main():
    res = {}
    for iters in (1, 3):
        res[f"jump_flips_{iters}it"] = flips(syn.make_batch(4096, 8, 25, "jump"), iters)
        print("jump flips", iters, res[f"jump_flips_{iters}it"], flush=True)
    res["trot_flips_3it"] = flips(syn.make_batch(4096, 4, 50, "trot"), 3)
    print("trot flips", res["trot_flips_3it"], flush=True)
    prob = syn.make_batch(64, 4, 50, "trot")
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1)
    g = run(prob, True, **kw)
    r = O.solve_batch(prob, O.default_options(**kw), n_threads=16)
    res["one_iteration_vs_oracle"] = {f: rel(g[f], r[f]) for f in ("K", "dU", "dX", "Xbar", "Ubar", "cost")}
    res["one_iteration_vs_oracle"]["ls_trials_equal_frac"] = float(np.mean(g["n_ls_trials"] == r["n_ls_trials"]))
    print("one iteration", res["one_iteration_vs_oracle"], flush=True)

    for gait, P, N in (("trot", 4, 50), ("jump", 8, 25)):
        prob = syn.make_batch(4096, P, N, gait)
        kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=10)
        a, b = run(prob, False, **kw), run(prob, True, **kw)
        d = np.abs(b["cost"] - a["cost"]) / np.abs(a["cost"])
        res[f"fixed10_{gait}"] = {
            "cost_rel_median": float(np.median(d)), "cost_rel_p99": float(np.quantile(d, .99)),
            "cost_rel_max": float(d.max()), "ls_trials_equal_frac": float(np.mean(a["n_ls_trials"] == b["n_ls_trials"])),
            "ms_per_iteration_fp64": a["ms_total"] / 10, "ms_per_iteration_fp32": b["ms_total"] / 10,
            "all_finite_fp32": bool(np.isfinite(b["cost"]).all())}
        print(gait, "fixed10", res[f"fixed10_{gait}"], flush=True)
        a, b = run(prob, False), run(prob, True)
        d = np.abs(b["cost"] - a["cost"]) / np.abs(a["cost"])
        res[f"full_solve_{gait}"] = {
            "cost_rel_median": float(np.median(d)), "cost_rel_p99": float(np.quantile(d, .99)),
            "cost_rel_max": float(d.max()), "feas_max_fp64": float(a["feas"].max()), "feas_max_fp32": float(b["feas"].max()),
            "status_equal_frac": float(np.mean(a["status"] == b["status"])),
            "iters_equal_frac": float(np.mean(a["iters"] == b["iters"])),
            "mean_iters_fp64": float(a["iters"].mean()), "mean_iters_fp32": float(b["iters"].mean()),
            "wall_s_fp64": a["wall_s"], "wall_s_fp32": b["wall_s"]}
        print(gait, "full", res[f"full_solve_{gait}"], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "fp32_tolerance.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
