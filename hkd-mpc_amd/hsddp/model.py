"""Batched HKD model primitives on the GPU (C-ABI hsddp_hkd_*).

Host-array convenience wrappers: copy in, run the kernel, copy out.  These replace the
reference's per-call CasADi wrappers (HKDModel.h:33-61, HKDReset.h:41-136, casadi_interface.cpp).
Matrix outputs use the reference's Eigen column-major layout; the wrappers return them as
row-major numpy [n, 24, 24] (A[i, r, c] = dx+_r / dx_c).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import HSDDPError, check, lib


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
