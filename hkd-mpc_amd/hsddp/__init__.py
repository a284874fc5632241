"""hsddp — MI355X-native batched Hybrid-Systems DDP for the HKD quadruped model.

Python mirror of the reference's solver surface (HSDDPSolver/header/MultiPhaseDDP.h:19-122):
``Solver`` wraps one C-ABI handle (include/hsddp.h) holding B independent multi-phase problems on
one GPU; ``solve()`` runs MultiPhaseDDP::solve for all of them.  ``load_settings`` reads the
reference's ``ddp_setting.info`` surface (loadHSDDPSetting, HSDDP_CompoundTypes.h:62-87).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import model, synthetic  # noqa: F401
from ._lib import (MPC_COMMAND, ConstraintParams, ElementInfo, HSDDPError, Options, ProblemDesc, Stats, Weights,
                   check, dp, ip, lib)

SETTINGS_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "settings")

__all__ = ["Solver", "Options", "default_options", "load_settings", "load_constraint_params",
           "HSDDPError", "model"]


def default_options(**overrides) -> Options:
    """HSDDP_OPTION in-class defaults (HSDDP_CompoundTypes.h:20-45)."""
    o = Options()
    lib().hsddp_default_options(C.byref(o))
    for k, v in overrides.items():
        setattr(o, k, v)
    return o


def load_settings(path: str | None = None, base: Options | None = None, **overrides) -> Options:
    """loadHSDDPSetting: start from HSDDP_OPTION defaults, overlay the INFO file's keys."""
    o = base if base is not None else default_options()
    path = path or os.path.join(SETTINGS_DIR, "ddp_setting.info")
    check(lib().hsddp_load_settings(path.encode(), C.byref(o)))
    for k, v in overrides.items():
        setattr(o, k, v)
    return o


def load_constraint_params(path: str | None = None) -> ConstraintParams:
    cp = ConstraintParams()
    lib().hsddp_default_constraint_params(C.byref(cp))
    path = path or os.path.join(SETTINGS_DIR, "constraint_params.info")
    check(lib().hsddp_load_constraint_params(path.encode(), C.byref(cp)))
    return cp


class Solver:
    """B independent HKD trajectory optimisations on one GPU (one C-ABI handle)."""

    def __init__(self, prob: dict, options: Options | None = None, device: int = 0,
                 cparams: ConstraintParams | None = None, weights: Weights | None = None,
                 riccati_fp32: bool = False):
        """riccati_fp32: SURVEY.md §8 config C5 — LQ records, backward Riccati sweep, gains and the
        linear rollout in fp32; dynamics, costs, line search and the AL/ReB outer loop in fp64."""
        L = lib()
        self.prob = prob
        self.B = int(prob["batch"])
        self.S, self.Kc = int(prob["S"]), int(prob["Kc"])
        self.P = len(prob["horizons"])
        desc = ProblemDesc()
        desc.device = device
        desc.batch = self.B
        desc.n_phases = self.P
        for i, n in enumerate(prob["horizons"]):
            desc.horizons[i] = int(n)
        desc.dt = float(prob["dt"])
        desc.ref_per_element = 0 if prob["ref_x"].shape[0] == 1 else 1
        desc.riccati_fp32 = 1 if riccati_fp32 else 0
        if weights is None:
            L.hsddp_default_weights(C.byref(desc.weights))
        else:
            desc.weights = weights
        if cparams is None:
            L.hsddp_default_constraint_params(C.byref(desc.cparams))
        else:
            desc.cparams = cparams
        h = C.c_void_p()
        check(L.hsddp_create(C.byref(desc), C.byref(h)))
        self._h = h
        self.options = options if options is not None else load_settings()
        check(L.hsddp_set_options(h, C.byref(self.options)))
        self._contacts = np.ascontiguousarray(prob["contacts"], dtype=np.int32)
        check(L.hsddp_upload_problem(h, ip(self._contacts), dp(np.ascontiguousarray(prob["x0"])),
                                     dp(np.ascontiguousarray(prob["ref_x"])),
                                     dp(np.ascontiguousarray(prob["ref_u"])),
                                     dp(np.ascontiguousarray(prob["ref_foot"]))))
        self.warm_start(prob.get("Xbar"), prob.get("Ubar"), prob.get("K"))

    # -- MultiPhaseDDP surface ---------------------------------------------------------------
    def set_options(self, options: Options) -> None:
        self.options = options
        check(lib().hsddp_set_options(self._h, C.byref(options)))

    def warm_start(self, Xbar=None, Ubar=None, K=None) -> None:
        keep = [np.ascontiguousarray(a, dtype=np.float64) if a is not None else None for a in (Xbar, Ubar, K)]
        check(lib().hsddp_upload_warm_start(self._h, *(None if a is None else dp(a) for a in keep)))

    def solve(self) -> Stats:
        """MultiPhaseDDP::solve for every element (MultiPhaseDDP.cpp:232-428)."""
        st = Stats()
        check(lib().hsddp_solve(self._h, C.byref(st)))
        return st

    def begin(self) -> None:
        check(lib().hsddp_solve_begin(self._h))

    def iterate(self, n: int) -> Stats:
        """n inner DDP iterations of every active element (throughput mode)."""
        st = Stats()
        check(lib().hsddp_iterate(self._h, int(n), C.byref(st)))
        return st

    def end(self) -> None:
        check(lib().hsddp_solve_end(self._h))

    def trajectory(self) -> dict:
        Xbar = np.empty((self.B, self.S, 24)); Ubar = np.empty((self.B, self.Kc, 24))
        K = np.empty((self.B, self.Kc, 24, 24))
        check(lib().hsddp_download_trajectory(self._h, dp(Xbar), dp(Ubar), dp(K)))
        return {"Xbar": Xbar, "Ubar": Ubar, "K": K}

    def working(self) -> dict:
        X = np.empty((self.B, self.S, 24)); U = np.empty((self.B, self.Kc, 24))
        D = np.empty((self.B, self.S, 24)); dX = np.empty((self.B, self.S, 24)); dU = np.empty((self.B, self.Kc, 24))
        check(lib().hsddp_download_working(self._h, dp(X), dp(U), dp(D), dp(dX), dp(dU)))
        return {"X": X, "U": U, "Defect": D, "dX": dX, "dU": dU}

    def element_info(self) -> dict:
        info = (ElementInfo * self.B)()
        check(lib().hsddp_download_element_info(self._h, info))
        out = {}
        for f, _ in ElementInfo._fields_:
            out[f] = np.array([getattr(info[b], f) for b in range(self.B)])
        return out

    def extract_commands(self, nsteps_between_mpc: int = 1, mpc_time: float = 0.0, dt_mpc: float = 0.01,
                         status_durations=None, foot_placements=None, solve_time: float = 0.0) -> np.ndarray:
        """HKDMPCSolver::update_foot_placement + publish_mpc_cmd (HKDMPC.cpp:207-298) for every
        element: a [B] record array of hsddp_mpc_command (= hkd_command_lcmt).
        status_durations: [P, 4] or [B, P, 4]; foot_placements: [12] or [B, 12]."""
        out = np.zeros(self.B, dtype=MPC_COMMAND)
        dur = None if status_durations is None else np.ascontiguousarray(status_durations, dtype=np.float64)
        feet = None if foot_placements is None else np.ascontiguousarray(foot_placements, dtype=np.float32)
        check(lib().hsddp_extract_commands(
            self._h, int(nsteps_between_mpc), float(mpc_time), float(dt_mpc),
            None if dur is None else dur.ctypes.data, int(dur is not None and dur.ndim == 3),
            None if feet is None else feet.ctypes.data, int(feet is not None and feet.ndim == 2),
            float(solve_time), out.ctypes.data))
        return out

    # -- receding horizon (HKDProblem::update, HKDProblem.cpp:117-222) ------------------------
    def layout(self) -> dict:
        n = C.c_int()
        hz, ss, re = (C.c_int * 16)(), (C.c_int * 16)(), (C.c_int * 16)()
        check(lib().hsddp_get_layout(self._h, C.byref(n), hz, ss, re))
        P = n.value
        return {"horizons": list(hz[:P]), "shooting": list(ss[:P]), "reach_end": list(re[:P])}

    def shift(self, contact_change) -> dict:
        """len(contact_change) simulation steps of HKDProblem::update on the device-held warm start;
        returns the new layout.  Call update_problem with inputs of that layout before solving."""
        cc = np.ascontiguousarray(np.asarray(contact_change, dtype=np.int32).reshape(-1))
        check(lib().hsddp_shift(self._h, int(cc.size), ip(cc)))
        lay = self.layout()
        self.P = len(lay["horizons"])
        self.S = sum(n + 1 for n in lay["horizons"])
        self.Kc = sum(lay["horizons"])
        return lay

    def update_problem(self, contacts, x0, ref_x, ref_u, ref_foot) -> None:
        """Inputs of the current layout, keeping the warm start (hsddp_update_problem)."""
        self._contacts = np.ascontiguousarray(contacts, dtype=np.int32)
        check(lib().hsddp_update_problem(self._h, ip(self._contacts), dp(np.ascontiguousarray(x0, dtype=np.float64)),
                                         dp(np.ascontiguousarray(ref_x, dtype=np.float64)),
                                         dp(np.ascontiguousarray(ref_u, dtype=np.float64)),
                                         dp(np.ascontiguousarray(ref_foot, dtype=np.float64))))

    def synchronize(self) -> None:
        check(lib().hsddp_synchronize(self._h))

    def device_bytes(self) -> int:
        return int(lib().hsddp_device_bytes(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().hsddp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
