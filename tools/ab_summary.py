#!/usr/bin/env python3
"""Summarise tools/ab_bench.sh runs (gpurun_out/ab_<name>_<rep>.log): per library and repetition,
traj-iter/s, ms per step and the device time per kernel group."""
import glob
import json
import os
import re

O = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
for p in sorted(glob.glob(os.path.join(O, "ab_*_*.log")), key=lambda q: (re.sub(r"_\d+\.log$", "", q), q)):
    lines = [x for x in open(p) if x.startswith("{")]
    name = os.path.basename(p)[3:-4]
    if not lines:
        print(f"{name:14s} no result")
        continue
    d = json.loads(lines[-1])
    ms = {k: round(v, 3) for k, v in d["extra"]["device_ms_per_step"].items()}
    print(f"{name:14s} {d['value']:9.0f} traj-iter/s  {d['ms_per_step']:.3f} ms/step  {ms}")
