#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/pmc.sh) into profiles/pmc_summary.json.

Per kernel: mean counter values over its dispatches, and HBM bytes per launch
    = 2 * FETCH_SIZE + WRITE_SIZE   (FETCH_SIZE / WRITE_SIZE in KiB)
with the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a
streaming read, so it is doubled; WRITE_SIZE is taken as is.  Wait / busy fractions come from
the SQ pass (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).

    python tools/pmc_summary.py gpurun_out [cfg_key]
"""
import collections
import csv
import json
import os
import sys


def read_pass(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            # "void hsddp::k_riccati<double>(hsddp::Params, ...)" -> "k_riccati" (the precision is
            # part of the configuration key)
            k = r["Kernel_Name"].split("(")[0].replace("hsddp::", "").replace("void ", "").split("<")[0]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    cfg_key = sys.argv[2] if len(sys.argv) > 2 else "trot_4x50_b4096"
    pfx = sys.argv[3] if len(sys.argv) > 3 else "pmc"
    kernels = collections.defaultdict(dict)
    for name in ("sq", "fetch", "write"):
        path = os.path.join(out_dir, f"{pfx}_{name}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for k, cs in read_pass(path).items():
            kernels[k].update(cs)
    summary = {}
    for k, cs in sorted(kernels.items()):
        e = {c: round(v, 1) for c, v in cs.items()}
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["hbm_bytes_per_launch"] = int((2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024)
        if "SQ_WAVE_CYCLES" in cs and cs["SQ_WAVE_CYCLES"] > 0:
            w = cs["SQ_WAVE_CYCLES"]
            e["wait_frac"] = round(cs.get("SQ_WAIT_ANY", 0) / w, 3)
            e["issue_stall_frac"] = round(cs.get("SQ_WAIT_INST_ANY", 0) / w, 3)
            e["active_frac"] = round(cs.get("SQ_ACTIVE_INST_ANY", 0) / w, 3)
        summary[k] = e
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_summary.json")
    try:
        with open(dst) as f:
            allcfg = json.load(f)
    except (OSError, ValueError):
        allcfg = {}
    allcfg[cfg_key] = summary
    allcfg["_note"] = ("rocprofv3 --pmc passes over `bench.py --steps 2 --warmup 1` (tools/pmc.sh); "
                       "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH correction")
    with open(dst, "w") as f:
        json.dump(allcfg, f, indent=1, sort_keys=True)
    for k, e in summary.items():
        print(k, {c: e[c] for c in ("hbm_bytes_per_launch", "wait_frac", "active_frac") if c in e})


if __name__ == "__main__":
    main()
