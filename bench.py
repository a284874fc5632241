#!/usr/bin/env python3
"""Throughput benchmark of the batched HS-DDP solver (BASELINE.json metric).

A step = one DDP inner iteration (LQ approximation, regularised backward Riccati sweep, MS
linear rollout, line search, nominal update; MultiPhaseDDP.cpp:304-381) over the whole batch
of B = 4096 independent 4-phase x 50-knot HKD trot problems per GPU, fp64, inputs resident in HBM.
value = trajectory-iterations/s over all ranks (sum of per-element inner iterations / max rank
time).  N GPUs: one process per GPU, disjoint shards (weak scaling), no collective on the data
path; a final gather of per-element summaries to rank 0 after the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # imported before the solver so libhsddp_amd.so binds to torch's HIP runtime
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))

import hsddp  # noqa: E402
from hsddp import synthetic  # noqa: E402

METRIC = "batched DDP iters/sec (fwd+bwd), 4-phase 200-knot HKD fp64, batch=4096"
UNIT = "trajectory-iterations/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


# algorithmic bytes per knot per DDP iteration of the BWD pass (r A, B, l*, Defect
# 2952 fp64; w K, dU 600 fp64) — the per-unit figure the roofline is quoted on.  One k_riccati
# launch processes every control knot of every element once.
BWD_BYTES_PER_KNOT = 8 * (2952 + 600)


def load_traffic(cfg_key: str):
    """Measured HBM bytes per k_riccati launch from the committed rocprofv3 PMC summary (or None)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            data = json.load(f)
        return data.get(cfg_key, {}).get("k_riccati", {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(args):
    """The oracle (CPU restatement of the reference solver, C, one trajectory per thread) timed on a
    bounded sample of the same workload on this host."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    prob = synthetic.make_batch(args.cpu_elements, args.phases, args.knots, args.gait)
    opt = O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=args.cpu_iters)
    t0 = time.perf_counter()
    r = O.solve_batch(prob, opt, n_threads=threads)
    dt = time.perf_counter() - t0
    n = float(np.sum(r["iters"]))
    return {"value": n / dt, "unit": UNIT, "cores": threads, "kind": "port",
            "sample": f"oracle/hsddp_oracle.c, {args.cpu_elements} elements x {args.cpu_iters} inner iterations "
                      f"(+ initial rollout), same {args.gait} {args.phases}x{args.knots} workload, {threads} threads, {dt:.1f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="trajectories per GPU")
    ap.add_argument("--phases", type=int, default=4)
    ap.add_argument("--knots", type=int, default=50)
    ap.add_argument("--gait", default="trot")
    ap.add_argument("--mixed", action="store_true",
                    help="config C4: per-element gait drawn from {trot, pace, bound, pronk} (per-element references)")
    ap.add_argument("--cpu-elements", type=int, default=2048)
    ap.add_argument("--cpu-iters", type=int, default=10)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--riccati-fp32", action="store_true",
                    help="config C5: fp32 LQ records / Riccati sweep / linear rollout (fp64 rollout, costs, outer loop)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    B = args.batch
    prob = synthetic.make_batch(B, args.phases, args.knots, args.gait, mixed=args.mixed, first_element=rank * B)
    opt = hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=args.warmup + args.steps)
    solver = hsddp.Solver(prob, opt, device=local, riccati_fp32=args.riccati_fp32)
    solver.begin()
    if args.warmup:
        solver.iterate(args.warmup)
    it0 = solver.element_info()["iters"].sum()
    solver.synchronize(); torch.cuda.synchronize(); barrier()
    t0 = time.perf_counter()
    st = solver.iterate(args.steps)
    solver.synchronize(); torch.cuda.synchronize(); barrier()
    t1 = time.perf_counter()
    info = solver.element_info()
    elem_iters = float(info["iters"].sum() - it0)

    red = torch.tensor([t1 - t0, elem_iters, float(st.ls_trials)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = red[0:1].clone(); dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = red[1:3].clone(); dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, total_iters, total_ls = float(tmax[0]), float(tsum[0]), float(tsum[1])
        # final gather of per-element summaries to rank 0 (outside the timed region)
        summ = torch.from_numpy(np.stack([info["cost"], info["feas"], info["max_tconstr"],
                                          info["max_pconstr"]], 1)).to(dev)
        gathered = [torch.empty_like(summ) for _ in range(world)] if rank == 0 else None
        dist.gather(summ, gathered, dst=0)
        finite = bool(torch.isfinite(torch.cat(gathered)).all()) if rank == 0 else True
    else:
        elapsed, total_iters, total_ls = t1 - t0, elem_iters, float(st.ls_trials)
        finite = bool(np.isfinite(info["cost"]).all())

    if rank == 0:
        S, Kc, P = prob["S"], prob["Kc"], len(prob["horizons"])
        # k_riccati time from HIP events recorded around its launches on the solver's stream
        avg_bwd_ms = st.ms_backward / max(1, st.n_backward_launches)
        # fp32 mode (C5) halves every term of the per-knot bytes
        bytes_launch = BWD_BYTES_PER_KNOT * Kc * B // (2 if args.riccati_fp32 else 1)
        achieved = bytes_launch / (avg_bwd_ms * 1e-3) / 1e9
        gait = "mixed" if args.mixed else args.gait
        metric_cfg = (gait, args.phases, args.knots, B) == ("trot", 4, 50, 4096)
        label = ("config C5: fp32 Riccati" if args.riccati_fp32 else "BASELINE metric config" if metric_cfg
                 else "config C3: jump with resets" if gait == "jump" else "config C4 shard: mixed gaits" if args.mixed
                 else "custom")
        cfg_key = f"{gait}_{args.phases}x{args.knots}_b{B}" + ("_fp32" if args.riccati_fp32 else "")
        traffic = load_traffic(cfg_key)
        out = {
            "metric": METRIC, "value": total_iters / elapsed, "unit": UNIT, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 Riccati / f64 rollout" if args.riccati_fp32 else "f64",
            "data": f"synthetic: seeded random initial states (splitmix64), closed-form {gait} reference "
                    "(SURVEY.md §8d); no dataset or checkpoint",
            "config": {"workload": f"HKD {gait}, {args.phases} phases x {args.knots} knots, "
                                   f"batch={B} per GPU ({label})",
                       "global_batch": B * world, "batch_per_gpu": B, "phases": args.phases,
                       "knots_per_phase": args.knots, "nx": 24, "nu": 24, "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_riccati", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "algorithmic_bytes_per_launch": bytes_launch,
                         "avg_launch_ms": avg_bwd_ms},
            "extra": {"batch_iterations_per_s": total_iters / elapsed / (B * world),
                      "mean_ls_trials": total_ls / max(1.0, total_iters),
                      "device_ms_per_step": {"total": st.ms_total / args.steps, "lq": st.ms_lq / args.steps,
                                             "backward": st.ms_backward / args.steps,
                                             "linear_rollout": st.ms_linear / args.steps,
                                             "forward_ls": st.ms_forward / args.steps},
                      "all_costs_finite": finite, "device_bytes": solver.device_bytes()},
        }
        if world == 1 and not args.no_cpu_baseline and not args.riccati_fp32 and not args.mixed:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
