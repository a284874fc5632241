"""Generate tests/golden/hkd_model_golden.npz from the reference's own CasADi kernels.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden.py

oracle/_ref/libhkd_casadi_ref.so is compiled in place from
HKDMPC/HKD-TrajOpt/CasadiGen/source/*.cpp by oracle/Makefile; this script only evaluates it at
seeded points and stores inputs and outputs (data, no reference source):
  * hkinodyn      32 points  (x, u, c, dt=0.01) -> x+          hkinodyn_casadi.cpp:177-658
  * hkinodyn_par  same points -> A, B (row-major 24x24)          hkinodyn_par_casadi.cpp:181-2800
  * compute_foot_position  16 points x 4 legs -> p               comp_foot_pos_casadi.cpp:46-160
  * comp_foot_jacob_{1..4} same -> J (3x18 row-major)            comp_foot_jacob_1_casadi.cpp:46-520
  * resetmap / resetmap_partial for every per-leg switch type (stance->stance, stance->swing,
    swing->stance, swing->swing), composed per HKDReset.h:41-136 from the reference FK / Jacobian.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

SEED = 20240807


def dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def main():
    R = O.ref_lib()
    if R is None:
        raise SystemExit("oracle/_ref not built (needs /root/reference): make -C oracle ref")
    rng = np.random.default_rng(SEED)
    n = 32
    x = rng.uniform(-0.6, 0.6, (n, 24))
    x[:, 5] = rng.uniform(0.12, 0.38, n)
    u = rng.uniform(-40, 40, (n, 24))
    c = rng.integers(0, 2, (n, 4)).astype(float)
    c[0] = 1; c[1] = 0  # all-stance and flight cases always present
    dt = 0.01
    xn = np.zeros((n, 24)); A = np.zeros((n, 24, 24)); B = np.zeros((n, 24, 24))
    for q in range(n):
        xq, uq, cq = (np.ascontiguousarray(v[q]) for v in (x, u, c))
        o = np.zeros(24); R.ref_hkinodyn(dp(xq), dp(uq), dt, dp(cq), dp(o)); xn[q] = o
        a = np.zeros(576); b = np.zeros(576)
        R.ref_hkinodyn_par(dp(xq), dp(uq), dt, dp(cq), dp(a), dp(b))
        A[q] = a.reshape(24, 24).T; B[q] = b.reshape(24, 24).T  # CasADi column-major -> row-major
    m = 16
    fx = rng.uniform(-0.6, 0.6, (m, 24)); fx[:, 5] = rng.uniform(0.12, 0.38, m)
    fp = np.zeros((m, 4, 3)); fJ = np.zeros((m, 4, 3, 18))
    for q in range(m):
        for leg in range(4):
            pos = np.ascontiguousarray(fx[q, 3:6]); eul = np.ascontiguousarray(fx[q, 0:3])
            ql = np.ascontiguousarray(fx[q, 12 + 3 * leg:15 + 3 * leg])
            p = np.zeros(3); R.ref_foot_position(dp(pos), dp(eul), dp(ql), float(leg + 1), dp(p)); fp[q, leg] = p
            J = np.zeros(54); R.ref_foot_jacobian(leg, dp(pos), dp(eul), dp(ql), dp(J)); fJ[q, leg] = J.reshape(18, 3).T
    # reset maps: per-leg (c, cn) patterns covering all four switch types on every leg
    pats = [((1, 1, 1, 1), (0, 0, 1, 1)), ((0, 0, 1, 1), (0, 0, 0, 0)), ((0, 0, 0, 0), (1, 1, 0, 0)),
            ((1, 0, 0, 1), (0, 1, 1, 0)), ((0, 1, 1, 0), (1, 0, 0, 1)), ((1, 1, 0, 0), (1, 1, 1, 1)),
            ((0, 0, 0, 0), (1, 1, 1, 1)), ((1, 0, 1, 0), (1, 0, 1, 0))]
    k = len(pats)
    rx = rng.uniform(-0.5, 0.5, (k, 24)); rx[:, 5] = rng.uniform(0.15, 0.35, k)
    rc = np.array([p[0] for p in pats], np.int32); rcn = np.array([p[1] for p in pats], np.int32)
    rxn = np.zeros((k, 24)); rPx = np.zeros((k, 24, 24))
    for q in range(k):
        xq = rx[q]; xo = xq.copy(); Px = np.eye(24)
        for leg in range(4):
            if rc[q, leg] and not rcn[q, leg]:  # stance -> swing (HKDReset.h:51-56, :85-88)
                xo[12 + 3 * leg:15 + 3 * leg] = (0.0, -0.8, 1.7)
                Px[12 + 3 * leg:15 + 3 * leg, :] = 0
            if not rc[q, leg] and rcn[q, leg]:  # swing -> stance (:58-72, :89-134)
                pos = np.ascontiguousarray(xq[3:6]); eul = np.ascontiguousarray(xq[0:3])
                ql = np.ascontiguousarray(xq[12 + 3 * leg:15 + 3 * leg])
                p = np.zeros(3); R.ref_foot_position(dp(pos), dp(eul), dp(ql), float(leg + 1), dp(p))
                xo[12 + 3 * leg:15 + 3 * leg] = (p[0], p[1], 0.0)
                J = np.zeros(54); R.ref_foot_jacobian(leg, dp(pos), dp(eul), dp(ql), dp(J))
                J = J.reshape(18, 3).T * np.array([[1.0], [1.0], [0.0]])
                rows = slice(12 + 3 * leg, 15 + 3 * leg)
                Px[rows, 0:3] = J[:, 3:6]; Px[rows, 3:6] = J[:, 0:3]; Px[rows, 12:24] = J[:, 6:18]
        rxn[q] = xo; rPx[q] = Px
    out = os.path.join(HERE, "hkd_model_golden.npz")
    np.savez_compressed(out, x=x, u=u, c=c, dt=dt, xn=xn, A=A, B=B, fx=fx, fp=fp, fJ=fJ,
                        rx=rx, rc=rc, rcn=rcn, rxn=rxn, rPx=rPx)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
