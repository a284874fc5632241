"""Batched HKD model primitives on the GPU (C-ABI hsddp_hkd_*).

Host-array convenience wrappers: copy in, run the kernel, copy out.  These replace the
reference's per-call CasADi wrappers (HKDModel.h:33-61, HKDReset.h:41-136, casadi_interface.cpp).
Matrix outputs use the reference's Eigen column-major layout; the wrappers return them as
row-major numpy [n, 24, 24] (A[i, r, c] = dx+_r / dx_c).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import ctypes as _C

from ._lib import HSDDPError, Weights, check, lib


class _Dev:
    def __init__(self, nbytes: int, device: int = 0):
        self.ptr = lib().hsddp_device_alloc(max(int(nbytes), 16), device)
        if not self.ptr:
            raise HSDDPError(lib().hsddp_last_error().decode())
        self.nbytes = nbytes

    def put(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        check(lib().hsddp_memcpy_h2d(self.ptr, a.ctypes.data, a.nbytes))
        return self

    def get(self, shape, dtype=np.float64):
        out = np.empty(shape, dtype=dtype)
        check(lib().hsddp_memcpy_d2h(out.ctypes.data, self.ptr, out.nbytes))
        return out

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().hsddp_device_free(self.ptr)
            self.ptr = None


def _dev(a, dtype=np.float64):
    a = np.ascontiguousarray(a, dtype=dtype)
    return _Dev(a.nbytes).put(a)


def dynamics(x, u, c, dt=0.01):
    x = np.atleast_2d(x); n = x.shape[0]
    dx, du, dc = _dev(x), _dev(np.atleast_2d(u)), _dev(np.atleast_2d(c))
    out = _Dev(n * 24 * 8)
    check(lib().hsddp_hkd_dynamics(dx.ptr, du.ptr, dc.ptr, dt, out.ptr, n, None))
    return out.get((n, 24))


def dynamics_partial(x, u, c, dt=0.01):
    x = np.atleast_2d(x); n = x.shape[0]
    dx, du, dc = _dev(x), _dev(np.atleast_2d(u)), _dev(np.atleast_2d(c))
    A, B = _Dev(n * 576 * 8), _Dev(n * 576 * 8)
    check(lib().hsddp_hkd_dynamics_partial(dx.ptr, du.ptr, dc.ptr, dt, A.ptr, B.ptr, n, None))
    return A.get((n, 24, 24)).transpose(0, 2, 1), B.get((n, 24, 24)).transpose(0, 2, 1)


def foot_position(x, leg):
    x = np.atleast_2d(x); n = x.shape[0]
    dx, dl = _dev(x), _dev(np.broadcast_to(np.asarray(leg), (n,)), np.int32)
    out = _Dev(n * 3 * 8)
    check(lib().hsddp_hkd_foot_position(dx.ptr, dl.ptr, out.ptr, n, None))
    return out.get((n, 3))


def foot_jacobian(x, leg):
    x = np.atleast_2d(x); n = x.shape[0]
    dx, dl = _dev(x), _dev(np.broadcast_to(np.asarray(leg), (n,)), np.int32)
    out = _Dev(n * 54 * 8)
    check(lib().hsddp_hkd_foot_jacobian(dx.ptr, dl.ptr, out.ptr, n, None))
    return out.get((n, 18, 3)).transpose(0, 2, 1)


def resetmap(x, c, cn):
    x = np.atleast_2d(x); n = x.shape[0]
    dx = _dev(x)
    dc = _dev(np.broadcast_to(np.asarray(c), (n, 4)), np.int32)
    dn = _dev(np.broadcast_to(np.asarray(cn), (n, 4)), np.int32)
    out = _Dev(n * 24 * 8)
    check(lib().hsddp_hkd_resetmap(dx.ptr, dc.ptr, dn.ptr, out.ptr, n, None))
    return out.get((n, 24))


def resetmap_partial(x, c, cn):
    x = np.atleast_2d(x); n = x.shape[0]
    dx = _dev(x)
    dc = _dev(np.broadcast_to(np.asarray(c), (n, 4)), np.int32)
    dn = _dev(np.broadcast_to(np.asarray(cn), (n, 4)), np.int32)
    out = _Dev(n * 576 * 8)
    check(lib().hsddp_hkd_resetmap_partial(dx.ptr, dc.ptr, dn.ptr, out.ptr, n, None))
    return out.get((n, 24, 24)).transpose(0, 2, 1)


# ---- cost / constraint plugins (HKDCost.h, HKDConstraints.cpp; the C++ facade's hkd:: plugins) ----
TERM_TRACKING, TERM_FOOT = 1, 2


def _weights(w):
    if w is None:
        w = Weights()
        lib().hsddp_default_weights(_C.byref(w))
    return w


def _pts(a, n, width, dtype=np.float64):
    return _dev(np.broadcast_to(np.asarray(a, dtype=dtype), (n, width)), dtype)


def running_cost(x, u, c, xr, ur, pf, terms=TERM_TRACKING | TERM_FOOT, dt=0.01, weights=None):
    """RCostData of HKDTrackingCost (terms 1) / HKDFootPlaceReg (terms 2) at n points:
    dict l [n], lx, lu [n, 24], lxx, luu [n, 24, 24]."""
    x = np.atleast_2d(x); n = x.shape[0]
    w = _weights(weights)
    ins = [_dev(x), _pts(u, n, 24), _pts(c, n, 4, np.int32), _pts(xr, n, 24), _pts(ur, n, 24), _pts(pf, n, 12)]
    outs = [_Dev(n * 8), _Dev(n * 192), _Dev(n * 192), _Dev(n * 4608), _Dev(n * 4608)]
    check(lib().hsddp_hkd_running_cost(*[a.ptr for a in ins], _C.byref(w), dt, terms, *[o.ptr for o in outs], n, None))
    return {"l": outs[0].get((n,)), "lx": outs[1].get((n, 24)), "lu": outs[2].get((n, 24)),
            "lxx": outs[3].get((n, 24, 24)), "luu": outs[4].get((n, 24, 24))}


def terminal_cost(x, c, xr, pf, terms=TERM_TRACKING | TERM_FOOT, weights=None):
    """TCostData (Phi [n], Phix [n, 24], Phixx [n, 24, 24]) of the HKD terminal cost terms."""
    x = np.atleast_2d(x); n = x.shape[0]
    w = _weights(weights)
    ins = [_dev(x), _pts(c, n, 4, np.int32), _pts(xr, n, 24), _pts(pf, n, 12)]
    outs = [_Dev(n * 8), _Dev(n * 192), _Dev(n * 4608)]
    check(lib().hsddp_hkd_terminal_cost(*[a.ptr for a in ins], _C.byref(w), terms, *[o.ptr for o in outs], n, None))
    return {"Phi": outs[0].get((n,)), "Phix": outs[1].get((n, 24)), "Phixx": outs[2].get((n, 24, 24))}


def grf_constraint(u, c, mu=0.7):
    """GRFConstraint rows (5 per stance leg, leg order): g [n, 20], gu [n, 20, 24]."""
    u = np.atleast_2d(u); n = u.shape[0]
    du, dc = _dev(u), _pts(c, n, 4, np.int32)
    g, gu = _Dev(n * 160), _Dev(n * 3840)
    check(lib().hsddp_hkd_grf_constraint(du.ptr, dc.ptr, mu, g.ptr, gu.ptr, n, None))
    return g.get((n, 20)), gu.get((n, 20, 24))


def touchdown_constraint(x, c, cn, ground=0.0):
    """TouchDownConstraint rows (legs with c = 0, cn = 1, leg order): h [n, 4], hx [n, 4, 24]."""
    x = np.atleast_2d(x); n = x.shape[0]
    dx, dc, dn = _dev(x), _pts(c, n, 4, np.int32), _pts(cn, n, 4, np.int32)
    h, hx = _Dev(n * 32), _Dev(n * 768)
    check(lib().hsddp_hkd_touchdown_constraint(dx.ptr, dc.ptr, dn.ptr, ground, h.ptr, hx.ptr, n, None))
    return h.get((n, 4)), hx.get((n, 4, 24))
