#!/usr/bin/env python3
"""Throughput benchmark of the batched HS-DDP solver (BASELINE.json metric).

A step = one DDP inner iteration (LQ approximation, regularised backward Riccati sweep, MS
linear rollout, line search, nominal update; MultiPhaseDDP.cpp:304-381) over the whole batch
of B = 4096 independent 4-phase x 50-knot HKD trot problems per GPU, fp64, inputs resident in HBM.
value = trajectory-iterations/s over all ranks (sum of per-element inner iterations / max rank
time).  N GPUs: one process per GPU, disjoint shards (weak scaling), no collective on the data
path; a final RCCL gather of per-element summaries to rank 0 after the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]

`--gpus N` with N > 1 outside a torch.distributed launch starts the N ranks itself (a child
`torch.distributed.run`, before this process touches the GPU) and exits with its status.

Roofline: `achieved` = the dominant kernel's (k_riccati) algorithmic bytes per launch
in this design's compact layout (hsddp/traffic.py) / its average launch time from HIP events on
the solver's stream.  `traffic` = HBM bytes per launch measured by rocprofv3 PMC passes
(profiles/pmc_summary.json, tools/pmc.sh).  The sweep is fp64-issue-bound, so its fp64 FLOP rate
against the vector peak is reported next to it, and the whole step's algorithmic bytes / step time.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch  # imported before the solver so libhsddp_amd.so binds to torch's HIP runtime
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))

import hsddp  # noqa: E402
from hsddp import shard, synthetic, traffic  # noqa: E402

METRIC = "batched DDP iters/sec (fwd+bwd), 4-phase 200-knot HKD fp64, batch=4096"
UNIT = "trajectory-iterations/s"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 vector (= fp64 matrix) peak, spec; 60-75 measured (tools/micro/rates.hip)


def load_traffic(cfg_key: str, kernel: str = "k_riccati"):
    """Measured HBM bytes per launch from the committed rocprofv3 PMC summary (or None)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            data = json.load(f)
        return data.get(cfg_key, {}).get(kernel, {}).get("hbm_bytes_per_launch"), data.get("_source", "profiles/pmc_summary.json")
    except (OSError, ValueError):
        return None, None


def host_cpu():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return model, os.cpu_count() or 1, affinity


def cpu_baseline(args):
    """The oracle (CPU restatement of the reference solver, C, one trajectory per thread) timed on a
    bounded sample of the same workload on this host's cores: every core this process may run on,
    limited by the job's CPU share where the launcher sets one (OMP_NUM_THREADS; 16 on the GPU box)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    model, nproc, affinity = host_cpu()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = args.cpu_threads or (min(affinity, share) if share > 0 else affinity)
    prob = synthetic.make_batch(args.cpu_elements, args.phases, args.knots, args.gait)
    opt = O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=args.cpu_iters)
    t0 = time.perf_counter()
    r = O.solve_batch(prob, opt, n_threads=threads)
    dt = time.perf_counter() - t0
    n = float(np.sum(r["iters"]))
    return {"value": n / dt, "unit": UNIT, "cores": threads, "kind": "port",
            "host": {"cpu_model": model, "nproc": nproc, "affinity_cpus": affinity, "job_cpu_share": share or None},
            "sample": f"oracle/hsddp_oracle.c (-O2, fp64), {args.cpu_elements} elements x {args.cpu_iters} inner iterations "
                      f"(+ initial rollout), same {args.gait} {args.phases}x{args.knots} workload, one trajectory per thread, "
                      f"{threads} threads, {dt:.1f} s wall"}


def full_solve_c5(prob, device) -> dict:
    """Config C5's other half (BASELINE.json: "fp32 Riccati + ReB/AL outer loop, ... tolerance vs
    fp64 reference reported"): one full MultiPhaseDDP::solve of the same batch with the shipped
    settings (AL / ReB outer loop, early exits) in the fp32 Riccati mode and in fp64, each timed
    (synchronised wall clock, after an untimed solve of the same handle from the same start), and
    the fp32 result against
    the fp64 one: status agreement, relative final-cost difference, max |Xbar| difference.  After the
    timed region of the bench line; not part of its value."""
    res = {}
    for fp32 in (True, False):
        s = hsddp.Solver(prob, hsddp.load_settings(), device=device, riccati_fp32=fp32)
        s.solve()  # warm: graph capture, allocation
        # the same start again (the constructor's): inputs, then the batch's warm start
        s.upload_problem(prob["contacts"], prob["x0"], prob["ref_x"], prob["ref_u"], prob["ref_foot"])
        s.warm_start(prob.get("Xbar"), prob.get("Ubar"), prob.get("K"))
        s.synchronize(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.solve()
        s.synchronize(); torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        info = s.element_info()
        res[fp32] = {"ms": ms, "Xbar": s.trajectory()["Xbar"], "status": info["status"], "cost": info["cost"],
                     "iters": info["iters"], "outer": info["outer_iters"], "n_ls": info["n_ls_trials"],
                     "hist": s.solver_info()["cost"]}
        s.close()
    a, b = res[False], res[True]
    dc = np.abs(b["cost"] - a["cost"]) / np.maximum(np.abs(a["cost"]), 1e-30)
    same_path = (a["iters"] == b["iters"]) & (a["outer"] == b["outer"]) & (a["n_ls"] == b["n_ls"])
    w = int(np.argmax(dc))

    def parting(ha, hb, tol):
        """first solver-info entry (the initial one is 0) whose costs differ by more than tol, relative"""
        n = min(len(ha), len(hb))
        for j in range(n):
            if abs(float(hb[j]) - float(ha[j])) > tol * max(abs(float(ha[j])), 1e-30):
                return j
        return None if len(ha) == len(hb) else n
    return {"settings": "ddp_setting.info (max_AL_iter 5, max_DDP_iter 10, early exits)",
            "ms_fp32": b["ms"], "ms_fp64": a["ms"],
            "mean_inner_iters_fp32": float(b["iters"].mean()), "mean_inner_iters_fp64": float(a["iters"].mean()),
            "mean_outer_iters_fp32": float(b["outer"].mean()), "mean_outer_iters_fp64": float(a["outer"].mean()),
            "status_agreement": float(np.mean(a["status"] == b["status"])),
            "cost_rel_diff_median": float(np.median(dc)), "cost_rel_diff_max": float(np.max(dc)),
            # the tail: how many elements part from the fp64 solve, and where the worst one does
            "n_cost_rel_diff_gt_1e-6": int(np.sum(dc > 1e-6)), "n_cost_rel_diff_gt_1e-3": int(np.sum(dc > 1e-3)),
            "frac_same_decisions": float(np.mean(same_path)),  # equal inner / outer iterations and trial counts
            "cost_rel_diff_max_same_decisions": float(np.max(dc[same_path])) if same_path.any() else None,
            "worst": {"element": w, "cost_fp64": float(a["cost"][w]), "cost_fp32": float(b["cost"][w]),
                      "iters": [int(a["iters"][w]), int(b["iters"][w])], "outer": [int(a["outer"][w]), int(b["outer"][w])],
                      "ls_trials": [int(a["n_ls"][w]), int(b["n_ls"][w])],
                      "first_info_entry_parting_1e-6": parting(a["hist"][w], b["hist"][w], 1e-6),
                      "first_info_entry_parting_1e-3": parting(a["hist"][w], b["hist"][w], 1e-3),
                      "cost_history_fp64": [float(v) for v in a["hist"][w]],
                      "cost_history_fp32": [float(v) for v in b["hist"][w]]},
            "xbar_abs_diff_max": float(np.max(np.abs(b["Xbar"] - a["Xbar"]))),
            "all_finite": bool(np.isfinite(b["Xbar"]).all())}


def latency_c1(args) -> None:
    """BASELINE config 1 (Mini Cheetah trot, 1 phase x 50 knots, batch = 1): the reference's own use
    of the solver — one robot, one full MultiPhaseDDP::solve with the shipped ddp_setting.info
    (early exits on) through the C-ABI — as solve latency, with the oracle's single-problem CPU solve
    of the same problem beside it (one thread).  Not the driver's metric line (that is the default
    run); written for the record by `bench.py --config c1`."""
    prob = synthetic.make_batch(1, 1, 50, "trot")
    opt = hsddp.load_settings()
    solver = hsddp.Solver(prob, opt, device=0)
    times, iters = [], []
    for rep in range(args.warmup + args.steps):
        # a fresh problem each time: Xbar = reference, Ubar = K = 0 (HKDProblem.cpp:84-90)
        solver.upload_problem(prob["contacts"], prob["x0"], prob["ref_x"], prob["ref_u"], prob["ref_foot"])
        solver.synchronize()
        t0 = time.perf_counter()
        solver.solve()
        t1 = time.perf_counter()
        if rep >= args.warmup:
            times.append((t1 - t0) * 1e3)
            iters.append(int(solver.element_info()["iters"][0]))
    info = solver.element_info()
    solver.close()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    reps = max(5, args.steps)
    t0 = time.perf_counter()
    for _ in range(reps):
        r = O.solve_batch(prob, O.default_options(), n_threads=1)
    cpu_ms = (time.perf_counter() - t0) / reps * 1e3
    model, nproc, affinity = host_cpu()
    ms = float(np.median(times))
    out = {"metric": "full solve latency, 1-phase 50-knot HKD trot, batch=1 (BASELINE config 1)", "value": ms,
           "unit": "ms/solve", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
           "higher_is_better": False, "scaling": "none", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic: seeded random initial state (splitmix64), closed-form trot reference (SURVEY.md §8d)",
           "config": {"workload": "HKD trot, 1 phase x 50 knots, batch=1 (BASELINE config 1), ddp_setting.info "
                                  "(max_AL_iter 5, max_DDP_iter 10, early exits)", "global_batch": 1},
           "extra": {"ms_min": float(np.min(times)), "ms_max": float(np.max(times)), "inner_iterations": iters[0],
                     "iterations_equal_oracle": bool(iters[0] == int(r["iters"][0])),
                     "cost_rel_diff_vs_oracle": float(abs(info["cost"][0] - r["cost"][0]) / abs(r["cost"][0])),
                     "us_per_inner_iteration": ms * 1e3 / max(1, iters[0])},
           "cpu_baseline": {"value": cpu_ms, "unit": "ms/solve", "cores": 1, "kind": "port",
                            "host": {"cpu_model": model, "nproc": nproc, "affinity_cpus": affinity},
                            "sample": f"oracle/hsddp_oracle.c (-O2, fp64), the same problem and options, "
                                      f"{reps} solves on one thread"}}
    print(json.dumps(out), flush=True)


# BASELINE.json's configs: C1 = 1x50 trot at batch 1 (latency), C2 = 4x50 trot at
# batch 1024, C3 = 8x25 jump at 4096, C4 = the mixed-gait shard of the 8-GPU run (4096 per GPU),
# C5 = fp32 Riccati at 4096; the metric line is 4x50 trot at 4096.
CONFIGS = {"metric": {}, "c2": {"batch": 1024}, "c3": {"gait": "jump", "phases": 8, "knots": 25},
           "c4": {"mixed": True}, "c5": {"riccati_fp32": True}}


def spawn_ranks(args) -> int:
    """Run this script as N torch.distributed ranks (one per GPU) in a child launcher."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


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
                    help="config C4: per-element gait drawn from {trot, pace, bound, pronk, jump} (per-element references)")
    ap.add_argument("--cpu-elements", type=int, default=2048)
    ap.add_argument("--cpu-iters", type=int, default=10)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core of this process's share")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--riccati-fp32", action="store_true",
                    help="config C5: fp32 LQ records / Riccati sweep / linear rollout (fp64 rollout, costs, outer loop)")
    ap.add_argument("--config", default="metric", choices=["metric", "c1", "c2", "c3", "c4", "c5"],
                    help="BASELINE.json config (c1: batch-1 solve latency; default: the metric config)")
    args = ap.parse_args()
    for k, v in CONFIGS.get(args.config, {}).items():
        setattr(args, k, v)
    if args.config == "c1":
        torch.cuda.set_device(0)
        latency_c1(args)
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))  # nothing above touched the GPU

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # the RCCL leg runs whenever this is a torch.distributed.run rank — world size 1 included, so a
    # one-GPU box executes the same init / all_gather / gather path the N-GPU run takes
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if distributed:
            dist.barrier()

    B = args.batch
    # --mixed (config C4): per-element gaits, jumps on twice the phases of half the knots (8 x 25 beside
    # 4 x 50: per-element layouts in one handle)
    prob = synthetic.make_batch(B, args.phases, args.knots, args.gait, mixed=args.mixed, first_element=rank * B,
                                jump_layout=args.mixed)
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
    rank_ms = [(t1 - t0) / args.steps * 1e3]
    # after the timed region: every element's command block (hkd_command_lcmt, HKDMPC.cpp:232-298)
    # extracted on the device into the tensor the final gather sends (per-element layouts: each
    # element's own knot walk)
    cmd = torch.empty(B * hsddp.MPC_COMMAND.itemsize, dtype=torch.uint8, device=dev)
    solver.extract_commands_device(cmd.data_ptr())
    gather = {"summary_bytes_per_element": 48, "command_bytes_per_element": hsddp.MPC_COMMAND.itemsize if cmd is not None else 0}
    if distributed:
        allr = [torch.zeros_like(red) for _ in range(world)]
        dist.all_gather(allr, red)
        rank_ms = [float(r[0]) / args.steps * 1e3 for r in allr]
        elapsed = max(float(r[0]) for r in allr)
        total_iters = sum(float(r[1]) for r in allr)
        total_ls = sum(float(r[2]) for r in allr)
        # the one collective of the path (RCCL): per-element summaries and command blocks to rank 0
        summ = torch.from_numpy(shard.summary_rows(info)).to(dev)
        torch.cuda.synchronize(); barrier()
        g0 = time.perf_counter()
        rows, cmds = shard.final_gather(dist, summ, cmd)
        torch.cuda.synchronize()
        gather["ms"] = (time.perf_counter() - g0) * 1e3
        finite = bool(np.isfinite(rows).all()) if rank == 0 else True
        gathered_rows = int(rows.shape[0]) if rank == 0 else 0
        if rank == 0 and cmds is not None:
            gather["commands_ok"] = bool(np.all(cmds["N_mpcsteps"] == 8) and np.isfinite(cmds["hkd_controls"]).all())
    else:
        elapsed, total_iters, total_ls = t1 - t0, elem_iters, float(st.ls_trials)
        finite = bool(np.isfinite(info["cost"]).all())
        gathered_rows = B
        if cmd is not None:
            cmds = np.frombuffer(cmd.cpu().numpy().tobytes(), dtype=hsddp.MPC_COMMAND)
            gather["commands_ok"] = bool(np.all(cmds["N_mpcsteps"] == 8) and np.isfinite(cmds["hkd_controls"]).all())

    if rank == 0:
        S, Kc, P = prob["S"], prob["Kc"], len(prob["horizons"])
        if prob.get("layouts"):  # per-element layouts: the byte model at the batch's mean layout
            P = float(np.mean([len(h) for h in prob["layouts"]]))
            S = Kc + P
        ms_step = elapsed / args.steps * 1e3
        mean_ls = total_ls / max(1.0, total_iters)
        # per-knot ReB parameters are read unless the schedule keeps them uniform (default
        # constraint parameters: delta = delta_min = 0.1, hsddp_default_constraint_params)
        reb_rows = traffic.reb_rows_per_knot(prob, opt, 0.1, 0.1)
        kb = traffic.kernel_bytes(B, S, Kc, P, fp32=args.riccati_fp32, ref_per_element=args.mixed, reb_rows=reb_rows)
        # k_riccati time from HIP events recorded around its launches on the solver's stream
        avg_bwd_ms = st.ms_backward / max(1, st.n_backward_launches)
        bytes_launch = kb["k_riccati"]
        achieved = bytes_launch / (avg_bwd_ms * 1e-3) / 1e9
        flop_launch = traffic.RICCATI_FLOP_PER_KNOT * Kc * B
        tflops = flop_launch / (avg_bwd_ms * 1e-3) / 1e12
        step_b = traffic.step_bytes(B, S, Kc, P, mean_ls, fp32=args.riccati_fp32, ref_per_element=args.mixed,
                                    reb_rows=reb_rows)
        gait = "mixed" if args.mixed else args.gait
        metric_cfg = (gait, args.phases, args.knots, B) == ("trot", 4, 50, 4096)
        c2_cfg = (gait, args.phases, args.knots, B) == ("trot", 4, 50, 1024)
        label = ("config C5: fp32 Riccati (a trot-gait mode: DESIGN.md §5)" if args.riccati_fp32 else "BASELINE metric config" if metric_cfg
                 else "config C2: batch 1024" if c2_cfg
                 else "config C3: jump with resets" if gait == "jump" else "config C4 shard: mixed gaits, 4x50 / 8x25 layouts" if args.mixed
                 else "custom")
        cfg_key = f"{gait}_{args.phases}x{args.knots}_b{B}" + ("_fp32" if args.riccati_fp32 else "")
        meas, meas_src = load_traffic(cfg_key)
        n = max(1, args.steps)
        dms = {"total": st.ms_total / n, "lq+terminal": st.ms_lq / n, "backward": st.ms_backward / n,
               "linear_rollout": st.ms_linear / n, "forward_ls+update": st.ms_forward / n}  # (no update kernel left)
        gbs = {"k_lq+k_terminal": (kb["k_lq"] + kb["k_terminal"]) / (dms["lq+terminal"] * 1e6),
               "k_riccati": achieved,
               "k_lin_rollout": kb["k_lin_rollout"] / (dms["linear_rollout"] * 1e6),
               "k_rollout x trials + k_decide": mean_ls * kb["k_rollout"] / (dms["forward_ls+update"] * 1e6)}
        out = {
            "metric": METRIC, "value": total_iters / elapsed, "unit": UNIT, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 Riccati / f64 rollout" if args.riccati_fp32 else "f64",
            "data": f"synthetic: seeded random initial states (splitmix64), closed-form {gait} reference "
                    "(SURVEY.md §8d); no dataset or checkpoint",
            "config": {"workload": f"HKD {gait}, {args.phases} phases x {args.knots} knots, "
                                   f"batch={B} per GPU ({label})",
                       "global_batch": B * world, "batch_per_gpu": B, "phases": args.phases,
                       "knots_per_phase": args.knots, "nx": 24, "nu": 24, "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_riccati", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": meas,
                         "traffic_source": meas_src if meas is not None else None,
                         "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_ms": avg_bwd_ms,
                         "bytes_model": "compact layout, hsddp/traffic.py (DESIGN.md §3)",
                         "limiter": "fp64 issue (the sweep's dependent per-knot chain), see fp64",
                         "fp64": {"flop_per_launch": flop_launch, "achieved_tflops": tflops,
                                  "peak_tflops": FP64_PEAK_TFLOPS, "frac": tflops / FP64_PEAK_TFLOPS},
                         "step": {"algorithmic_bytes": step_b, "achieved": step_b / (ms_step * 1e6),
                                  "frac": step_b / (ms_step * 1e6) / HBM_PEAK_GBS,
                                  "kernel_GBps": gbs}},
            "extra": {"batch_iterations_per_s": total_iters / elapsed / (B * world),
                      "mean_ls_trials": mean_ls, "device_ms_per_step": dms,
                      "rank_ms_per_step": rank_ms, "rccl_world_size": world if distributed else 0, "gathered_elements": gathered_rows,
                      "final_gather": gather,
                      "all_costs_finite": finite, "device_bytes": solver.device_bytes()},
        }
        if world == 1 and not args.no_cpu_baseline and not args.riccati_fp32 and not args.mixed:
            out["cpu_baseline"] = cpu_baseline(args)
        if world == 1 and args.riccati_fp32:
            out["extra"]["full_solve"] = full_solve_c5(prob, local)
        print(json.dumps(out), flush=True)
    solver.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
