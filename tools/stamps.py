#!/usr/bin/env python3
"""Where a k_riccati knot spends its cycles: run the diagnostic build (-DHSDDP_STAMPS=1,
hkd-mpc_amd/libhsddp_amd_stamps.so, selected through HSDDP_LIB) and print each stage's share of
the stamped cycles.  Read the shares, not the totals: the stamps' fences forbid overlaps.

    HSDDP_LIB=$PWD/hkd-mpc_amd/libhsddp_amd_stamps.so python tools/stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch  # noqa: F401  (bind to torch's HIP runtime first, as bench.py does)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
import hsddp  # noqa: E402
from hsddp import synthetic  # noqa: E402

STAGES = ["wait DMA, coefficients", "Gn, T, M rows", "M columns, Z, Qux_c, Qu_c", "Qxx (symmetrise)",
          "Quu_cc columns, DMA", "elimination (12 steps)", "dU, K broadcast, G", "value update (DPP)",
          "K / dU stores"]
LIN_STAGES = ["DMA issue, stores, image wait", "K dX, du", "A - I, B rows (DPP)", "row tail, dV"]
RO_STAGES = ["element state, layout, u_prev row", "state rows staged (loads, LDS, barrier)",
             "contacts, trial control row", "running cost (references, ReB)", "dynamics, Defect, feasibility",
             "U rows (earlier), Defect rows stored (drained)"]


def main():
    B = int(os.environ.get("STAMP_B", "4096"))
    prob = synthetic.make_batch(B, 4, 50, "trot")
    s = hsddp.Solver(prob, hsddp.load_settings(no_early_exit=1, max_AL_iter=1, max_DDP_iter=4))
    s.begin()
    s.iterate(3)
    out = np.zeros((B, 16), np.uint64)
    L = hsddp._lib.lib()
    L.hsddp_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
    rc = L.hsddp_debug_stamps(s._h, out.ctypes.data)
    s.close()
    assert rc == 0, rc
    cyc = out[0::2, 1:10].astype(np.float64).mean(0)  # one stamp record per wave (its first element)
    tot = cyc.sum()
    for name, c in zip(STAGES, cyc):
        print(f"{name:28s} {c / (3 * 200):10.0f} cycles/knot  {100 * c / tot:5.1f} %")
    print(f"{'total':28s} {tot / (3 * 200):10.0f} cycles/knot")
    # k_lin_rollout (hsddp_linear.hip LSTAMP): written to the wave's second element, slots 8 + stage
    lc = out[1::2, 9:13].astype(np.float64).mean(0)
    lt = lc.sum()
    print("k_lin_rollout")
    for name, c in zip(LIN_STAGES, lc):
        print(f"{name:28s} {c / (3 * 200):10.0f} cycles/knot  {100 * c / max(lt, 1):5.1f} %")
    print(f"{'total':28s} {lt / (3 * 200):10.0f} cycles/knot")
    # k_rollout slot waves (hsddp_kernels.hip RSTAMP): element 0's slots 12..15, element 1's 0..3
    flat = out.reshape(-1)
    rc = flat[12:19].astype(np.float64)
    nw = max(float(flat[19]), 1.0)
    rt = rc.sum()
    print(f"k_rollout slot waves ({nw:.0f} stamped)")
    for name, c in zip(RO_STAGES, rc):
        print(f"{name:44s} {c / nw:10.0f} cycles/wave  {100 * c / max(rt, 1):5.1f} %")
    print(f"{'total':44s} {rt / nw:10.0f} cycles/wave")


if __name__ == "__main__":
    main()
