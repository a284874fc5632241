"""Average kernel durations (µs) per variant from tools/kprof.sh's kernel traces.

usage: python tools/kp_summary.py main te1 ... [--kernels k_terminal,k_lq]
"""
import collections
import csv
import re
import sys


def main(argv):
    kern = None
    names = []
    it = iter(argv)
    for a in it:
        if a == "--kernels":
            kern = set(next(it).split(","))
        else:
            names.append(a)
    for n in names:
        path = f"gpurun_out/kp_{n}/run_kernel_trace.csv"
        try:
            rows = list(csv.DictReader(open(path)))
        except OSError:
            print(n, "missing", path)
            continue
        d = collections.defaultdict(list)
        for r in rows:
            m = re.search(r"hsddp\d*(k_[a-z_0-9]+)", r["Kernel_Name"].replace("::", ""))
            if not m:
                continue
            d[m.group(1)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        out = {k: (len(v), round(sum(v) / len(v) / 1000, 1)) for k, v in sorted(d.items())
               if kern is None or k in kern}
        print(n, out)


if __name__ == "__main__":
    main(sys.argv[1:])
