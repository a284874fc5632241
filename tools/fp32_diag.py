"""fp32 Riccati mode diagnostic: per-knot error of K / dU against the fp64 GPU path (one iteration)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hkd-mpc_amd"), os.path.join(ROOT, "tests")]
import hsddp
from hsddp import synthetic as syn

gait, P, N = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("trot", 4, 50)
prob = syn.make_batch(16, P, N, gait)
kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1)
out = {}
for fp32 in (False, True):
    s = hsddp.Solver(prob, hsddp.load_settings(**kw), riccati_fp32=fp32)
    s.solve()
    out[fp32] = {**s.trajectory(), **s.working()}
    s.close()
a, b = out[False], out[True]
K64, K32 = a["K"], b["K"]
scale = np.abs(K64).max()
err = np.abs(K32 - K64).max(axis=(2, 3)) / scale  # [B][Kc]
print("max rel K", err.max(), "at", np.unravel_index(err.argmax(), err.shape))
for e in range(3):
    print("elem", e, "K err by kc (every 10th, from the end):", " ".join(f"{err[e, k]:.1e}" for k in range(err.shape[1] - 1, -1, -10)))
e, k = np.unravel_index(err.argmax(), err.shape)
d = np.abs(K32[e, k] - K64[e, k])
r, c = np.unravel_index(d.argmax(), d.shape)
print("worst entry row", r, "col", c, K64[e, k, r, c], K32[e, k, r, c])
print("rows with err > 1e-4 * scale:", sorted(set(np.nonzero(d > 1e-4 * scale)[0].tolist())))
print("cols:", sorted(set(np.nonzero(d > 1e-4 * scale)[1].tolist())))
du = np.abs(b["dU"] - a["dU"]).max() / np.abs(a["dU"]).max()
print("dU rel", du)
