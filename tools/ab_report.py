#!/usr/bin/env python3
"""Print the A/B results gathered by tools/ab.sh (gpurun_out/)."""
import json
import os

O = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
with open(os.path.join(O, "pytest_gpu.log")) as f:
    print("pytest:", f.read().strip().splitlines()[-1])
for name in ("new", "base"):
    p = os.path.join(O, name + ".log")
    if not os.path.exists(p):
        continue
    lines = [x for x in open(p) if x.startswith("{")]
    if not lines:
        print(name, "no result")
        continue
    d = json.loads(lines[-1])
    ms = {k: round(v, 3) for k, v in d["extra"]["device_ms_per_step"].items()}
    print(f"{name:5s} {d['value']:9.0f} traj-iter/s  {d['ms_per_step']:.3f} ms/step  {ms}")
for b in (1024, 4096):
    p = os.path.join(O, f"stamps_{b}.log")
    if os.path.exists(p):
        print(f"-- stamps B={b}")
        print("".join(x for x in open(p) if "cycles" in x), end="")
