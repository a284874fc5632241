#!/usr/bin/env python3
"""Per-kernel mean / max duration from tools/kprof.sh traces: python tools/kprof_report.py x0 x1 ..."""
import collections
import csv
import glob
import os
import sys

O = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
for lib in sys.argv[1:]:
    d = collections.defaultdict(list)
    for f in glob.glob(os.path.join(O, f"kp_{lib}", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d[r["Kernel_Name"].split("(")[0].replace("hsddp::", "")].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"== {lib}")
    for k in sorted(d, key=lambda k: -sum(d[k])):
        v = d[k]
        if sum(v) < 50:
            continue
        print(f"  {k:24s} n={len(v):3d} mean={sum(v) / len(v):8.1f} max={max(v):8.1f} us")
