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
from ._lib import (MPC_COMMAND, PHASE_PLAN, QUAD_STATE, ConstraintParams, ElementInfo, HSDDPError, Options, ProblemDesc, Stats, Weights,
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


# -- reference construction (QuadReference / HKDProblem::initialization) ------------------------
def load_quad_reference(path: str, reorder: bool = False):
    """QuadReference::load_top_level_data (QuadReference.cpp:129-290): (samples [n] QUAD_STATE, dt)."""
    L = lib()
    dt = C.c_float()
    n = L.hsddp_load_quad_reference(path.encode(), int(reorder), C.byref(dt), None, 0)
    check(min(n, 0))
    out = np.zeros(n, dtype=QUAD_STATE)
    check(min(L.hsddp_load_quad_reference(path.encode(), int(reorder), C.byref(dt), out.ctypes.data, n), 0))
    return out, float(dt.value)


def plan_phases(window: np.ndarray, dt_ref: float, plan_duration: float = 0.6, dt_sim: float = 0.01,
                dt_mpc: float = 0.01) -> dict:
    """HKDProblem::initialization's phase segmentation (HKDProblem.cpp:15-68) of a reference window."""
    w = np.ascontiguousarray(window, dtype=QUAD_STATE)
    plan = np.zeros(1, dtype=PHASE_PLAN)
    check(lib().hsddp_plan_phases(w.ctypes.data, int(w.size), dt_ref, plan_duration, dt_sim, dt_mpc, plan.ctypes.data))
    P = int(plan["n_phases"][0])
    return {"horizons": [int(v) for v in plan["horizons"][0][:P]], "contacts": plan["contacts"][0][:P + 1].copy(),
            "durations": plan["durations"][0][:P].copy(), "start_times": plan["start_times"][0][:P].copy(),
            "end_times": plan["end_times"][0][:P].copy()}


def reference_problem(table: np.ndarray, dt_ref: float, window_start, x0: np.ndarray, plan_duration: float = 0.6,
                      dt_sim: float = 0.01, dt_mpc: float = 0.01) -> dict:
    """HKDProblem::initialization (HKDProblem.cpp:15-111) for a batch: the phase plan of the window
    at table[window_start[0]] (the batch shares its layout; with per-element window starts every
    element reads its own samples, e.g. windows into different gait files concatenated into one
    table), contacts per element from its own window, and the inputs Solver needs to build the
    references on the device.  Pass the result to Solver(prob)."""
    ws = np.asarray(window_start, dtype=np.int32).reshape(-1)
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, 24)
    B = x0.shape[0]
    n_win = int(round(plan_duration / dt_ref)) + 2  # QuadReference::initialize: sz + 1 samples, sz = round(T/dt) + 1
    plans = [plan_phases(table[w:w + n_win], dt_ref, plan_duration, dt_sim, dt_mpc) for w in ws]
    hz = plans[0]["horizons"]
    shared = all(q["horizons"] == hz for q in plans[1:])
    Kc = sum(hz)
    if any(sum(q["horizons"]) != Kc for q in plans):
        raise HSDDPError("every window's plan must have the same number of knots")
    Pmax = max(len(q["horizons"]) for q in plans)
    contacts = np.zeros((len(plans), Pmax + 1, 4), np.int32)
    for b, q in enumerate(plans):  # [B][Pmax + 1][4]: element b's rows 0 .. P_b
        contacts[b, :len(q["horizons"]) + 1] = q["contacts"]
    if contacts.shape[0] == 1 and B > 1:
        contacts = np.repeat(contacts, B, axis=0)
    S = Kc + Pmax
    # dt: HKDProblem's float dt_sim widened to double by Trajectory(dt_sim, N) (HKDProblem.cpp:81)
    out = {"batch": B, "horizons": hz, "S": S, "Kc": Kc, "dt": float(np.float32(dt_sim)), "x0": x0, "contacts": contacts,
           "shooting": [n + 1 for n in hz], "ref_table": table, "dt_ref": dt_ref, "window_start": ws,
           "window_len": n_win, "phase_start_times": plans[0]["start_times"], "plan": plans[0]}
    if not shared:  # windows of different gaits: every element segmented by its own (HKDProblem.cpp:40-68)
        out.update(layouts=[q["horizons"] for q in plans], phase_start_times=None, plans=plans)
    return out


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
        from_table = "ref_x" not in prob  # references built on the device from prob["ref_table"]
        self.ref_per_element = (np.size(prob["window_start"]) != 1) if from_table else (prob["ref_x"].shape[0] != 1)
        desc.ref_per_element = int(self.ref_per_element)
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
        if prob.get("layouts") is not None:  # per-element phase layouts (largest layout = strides)
            lays = prob["layouts"]
            npz = np.array([len(x) for x in lays], np.int32)
            hz = np.zeros((self.B, 16), np.int32)
            for b, x in enumerate(lays):
                hz[b, :len(x)] = x
            check(L.hsddp_set_element_layouts(h, ip(npz), ip(hz)))
            self.P = int(npz.max())
            self.S = int(prob["S"])
        self.options = options if options is not None else load_settings()
        check(L.hsddp_set_options(h, C.byref(self.options)))
        if from_table:
            self.set_reference_table(prob["ref_table"], prob["dt_ref"])
            self.build_references(prob["window_start"], prob["window_len"], prob.get("phase_start_times"),
                                  prob["dt"])
            self.upload_problem(prob["contacts"], prob["x0"])
        else:
            self.upload_problem(prob["contacts"], prob["x0"], prob["ref_x"], prob["ref_u"], prob["ref_foot"])
        self.warm_start(prob.get("Xbar"), prob.get("Ubar"), prob.get("K"))

    def upload_problem(self, contacts, x0, ref_x=None, ref_u=None, ref_foot=None) -> None:
        """Inputs with the default warm start Xbar = reference, Ubar = K = 0 (HKDProblem.cpp:84-90;
        TrajectoryManagement.cpp:5-35).  References None: the ones hsddp_build_references made."""
        self._contacts = np.ascontiguousarray(contacts, dtype=np.int32)
        refs = [None if r is None else np.ascontiguousarray(r, dtype=np.float64) for r in (ref_x, ref_u, ref_foot)]
        check(lib().hsddp_upload_problem(self._h, ip(self._contacts), dp(np.ascontiguousarray(x0, dtype=np.float64)),
                                         *(None if r is None else dp(r) for r in refs)))

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

    def solver_info(self, capacity: int | None = None) -> dict:
        """MultiPhaseDDP::get_solver_info (MultiPhaseDDP.cpp:532-541) for every element: the
        per-iteration buffers of the last solve as lists of float32 arrays (cost, dyn_feas,
        eqn_feas, ineq_feas), the initial entry first."""
        cap = capacity or (1 + self.options.max_AL_iter * self.options.max_DDP_iter)
        arrs = [np.zeros((self.B, cap), np.float32) for _ in range(4)]
        cnt = np.zeros(self.B, np.int32)
        check(lib().hsddp_download_solver_info(self._h, cap, *(a.ctypes.data for a in arrs), cnt.ctypes.data))
        names = ("cost", "dyn_feas", "eqn_feas", "ineq_feas")
        return {n: [a[b, :cnt[b]].copy() for b in range(self.B)] for n, a in zip(names, arrs)}

    def lq(self) -> dict:
        """The LQ model of the last LQ_approximation (SinglePhase.cpp:264-296) as the reference
        Trajectory's dense blocks (TrajectoryManagement.h:65-81): A, B, lxx, luu [B][Kc][24][24],
        lx, lu [B][Kc][24], l [B][Kc] (lux = 0)."""
        B, Kc = self.B, self.Kc
        out = {k: np.empty((B, Kc, 24, 24)) for k in ("A", "B", "lxx", "luu")}
        out.update(lx=np.empty((B, Kc, 24)), lu=np.empty((B, Kc, 24)), l=np.empty((B, Kc)))
        check(lib().hsddp_download_lq(self._h, *(out[k].ctypes.data for k in ("A", "B", "l", "lx", "lu", "lxx", "luu"))))
        return out

    def terminal(self) -> dict:
        """Terminal data of every phase (TCostData + AL terms, reset-map Jacobian Px; zero after the
        last phase): Phi [B][P], Phix [B][P][24], Phixx, Px [B][P][24][24]."""
        P = self.P
        out = {"Phi": np.empty((self.B, P)), "Phix": np.empty((self.B, P, 24)),
               "Phixx": np.empty((self.B, P, 24, 24)), "Px": np.empty((self.B, P, 24, 24))}
        check(lib().hsddp_download_terminal(self._h, *(out[k].ctypes.data for k in ("Phi", "Phix", "Phixx", "Px"))))
        return out

    MAX_TD = 4  # HSDDP_MAX_TD

    def constraint_params(self) -> dict:
        """The ReB / AL parameters the solve reads and updates: reb_delta, reb_eps [B][Kc][20];
        td_mask [B][P][MAX_TD] (each phase's touchdown constraints, bit l = leg l); al_sigma,
        al_lambda [B][P][MAX_TD][4]."""
        B, P, Kc, T = self.B, self.P, self.Kc, self.MAX_TD
        out = {"reb_delta": np.empty((B, Kc, 20)), "reb_eps": np.empty((B, Kc, 20)),
               "td_mask": np.empty((B, P, T), np.int32), "al_sigma": np.empty((B, P, T, 4)),
               "al_lambda": np.empty((B, P, T, 4))}
        check(lib().hsddp_download_constraint_params(self._h, *(out[k].ctypes.data for k in
                                                               ("reb_delta", "reb_eps", "td_mask", "al_sigma", "al_lambda"))))
        return out

    def constraint_values(self) -> dict:
        """The constraint objects' stored values after the last solve (hsddp_download_constraint_values):
        grf_g [B][Kc][20] (GRF rows of the stance legs), td_h [B][P][MAX_TD][4] (touchdown residuals)."""
        B, P, Kc, T = self.B, self.P, self.Kc, self.MAX_TD
        out = {"grf_g": np.empty((B, Kc, 20)), "td_h": np.empty((B, P, T, 4))}
        check(lib().hsddp_download_constraint_values(self._h, out["grf_g"].ctypes.data, out["td_h"].ctypes.data))
        return out

    def upload_constraint_params(self, reb_delta=None, reb_eps=None, td_mask=None, al_sigma=None, al_lambda=None):
        """hsddp_upload_constraint_params (None keeps a field); shapes as constraint_params()'s.  The C
        side reads B x Kc x 20 / B x P x MAX_TD (x 4) values from each pointer, so the shapes are
        checked here (a [Kc][20] array for B > 1 would be read past its end)."""
        B, P, Kc, T = self.B, self.P, self.Kc, self.MAX_TD
        arrs = []
        for name, a, t, shape in (("reb_delta", reb_delta, np.float64, (B, Kc, 20)),
                                  ("reb_eps", reb_eps, np.float64, (B, Kc, 20)),
                                  ("td_mask", td_mask, np.int32, (B, P, T)),
                                  ("al_sigma", al_sigma, np.float64, (B, P, T, 4)),
                                  ("al_lambda", al_lambda, np.float64, (B, P, T, 4))):
            if a is not None:
                a = np.ascontiguousarray(a, dtype=t)
                if a.shape != shape:
                    raise HSDDPError(f"{name}: shape {a.shape}, expected {shape}")
            arrs.append(a)
        check(lib().hsddp_upload_constraint_params(self._h, *(None if a is None else a.ctypes.data for a in arrs)))

    def set_value_export(self, on: bool = True) -> None:
        """Store G[0], H[0] of every phase in each sweep (SinglePhase::get_value_approx)."""
        check(lib().hsddp_set_value_export(self._h, int(bool(on))))

    def value(self) -> dict:
        P = self.P
        G = np.empty((self.B, P, 24)); H = np.empty((self.B, P, 24, 24))
        check(lib().hsddp_download_value(self._h, G.ctypes.data, H.ctypes.data))
        return {"G": G, "H": H}

    def extract_commands(self, nsteps_between_mpc: int = 1, mpc_time: float = 0.0, dt_mpc: float = 0.01,
                         status_durations=None, foot_placements=None, solve_time: float = 0.0) -> np.ndarray:
        """HKDMPCSolver::update_foot_placement + publish_mpc_cmd (HKDMPC.cpp:207-298) for every
        element: a [B] record array of hsddp_mpc_command (= hkd_command_lcmt).
        status_durations: [P, 4] or [B, P, 4]; foot_placements: [12] or [B, 12]."""
        out = np.zeros(self.B, dtype=MPC_COMMAND)
        dur = None if status_durations is None else np.ascontiguousarray(status_durations, dtype=np.float64)
        feet = None if foot_placements is None else np.ascontiguousarray(foot_placements, dtype=np.float32)
        self._check_cmd_inputs(dur, feet)
        check(lib().hsddp_extract_commands(
            self._h, int(nsteps_between_mpc), float(mpc_time), float(dt_mpc),
            None if dur is None else dur.ctypes.data, int(dur is not None and dur.ndim == 3),
            None if feet is None else feet.ctypes.data, int(feet is not None and feet.ndim == 2),
            float(solve_time), out.ctypes.data))
        return out

    def _check_cmd_inputs(self, dur, feet):
        """the C side reads [P][4] or [B][P][4] durations and [12] or [B][12] feet by the arrays' rank"""
        if dur is not None and dur.shape not in ((self.P, 4), (self.B, self.P, 4)):
            raise HSDDPError(f"status_durations: shape {dur.shape}, expected ({self.P}, 4) or ({self.B}, {self.P}, 4)")
        if feet is not None and feet.shape not in ((12,), (self.B, 12)):
            raise HSDDPError(f"foot_placements: shape {feet.shape}, expected (12,) or ({self.B}, 12)")

    def extract_commands_async(self, nsteps_between_mpc: int = 1, mpc_time: float = 0.0, dt_mpc: float = 0.01,
                               status_durations=None, foot_placements=None, solve_time: float = 0.0) -> int:
        """hsddp_extract_commands_async: the records cross PCIe on the handle's copy stream while the
        caller goes on (the next tick's advance / solve); returns the ticket for commands_wait."""
        dur = None if status_durations is None else np.ascontiguousarray(status_durations, dtype=np.float64)
        feet = None if foot_placements is None else np.ascontiguousarray(foot_placements, dtype=np.float32)
        self._check_cmd_inputs(dur, feet)
        t = C.c_int()
        check(lib().hsddp_extract_commands_async(
            self._h, int(nsteps_between_mpc), float(mpc_time), float(dt_mpc),
            None if dur is None else dur.ctypes.data, int(dur is not None and dur.ndim == 3),
            None if feet is None else feet.ctypes.data, int(feet is not None and feet.ndim == 2),
            float(solve_time), C.byref(t)))
        return t.value

    def commands_wait(self, ticket: int, copy: bool = True) -> np.ndarray:
        """the [B] records of an asynchronous extraction (a copy, or a view of the pinned buffer that
        the extraction after next overwrites)"""
        ptr = C.c_void_p()
        check(lib().hsddp_commands_wait(self._h, int(ticket), C.byref(ptr)))
        buf = (C.c_char * (self.B * MPC_COMMAND.itemsize)).from_address(ptr.value)
        v = np.frombuffer(buf, dtype=MPC_COMMAND, count=self.B)
        return v.copy() if copy else v

    def extract_commands_device(self, out_ptr: int, nsteps_between_mpc: int = 1, mpc_time: float = 0.0,
                                dt_mpc: float = 0.01, solve_time: float = 0.0) -> None:
        """extract_commands into device memory at out_ptr ([B] hsddp_mpc_command on the handle's
        device, e.g. a torch uint8 tensor's data_ptr()): the command block of the final gather."""
        check(lib().hsddp_extract_commands_device(self._h, int(nsteps_between_mpc), float(mpc_time), float(dt_mpc),
                                                  None, 0, None, 0, float(solve_time), C.c_void_p(out_ptr)))

    def set_reference_table(self, table: np.ndarray, dt_ref: float) -> None:
        t = np.ascontiguousarray(table, dtype=QUAD_STATE)
        check(lib().hsddp_set_reference_table(self._h, t.ctypes.data, int(t.size), float(dt_ref)))

    def build_references(self, window_start, window_len: int, phase_start_times=None, dt_sim: float = 0.01) -> None:
        """get_reference_at_t at every slot of every element on the device (HKDReference.cpp:8-57);
        then upload_problem / update_problem with ref_x = ref_u = ref_foot = None keep them."""
        ws = np.ascontiguousarray(np.asarray(window_start, dtype=np.int32).reshape(-1))
        ps = None if phase_start_times is None else np.ascontiguousarray(phase_start_times, dtype=np.float32)
        check(lib().hsddp_build_references(self._h, ip(ws), int(window_len), None if ps is None else ps.ctypes.data,
                                           float(dt_sim)))

    def references(self) -> dict:
        """The references the solve reads: ref_x, ref_u [Bref][S][24], ref_foot [Bref][S][12]."""
        Br = self.B if self.ref_per_element else 1
        rx = np.empty((Br, self.S, 24)); ru = np.empty((Br, self.S, 24)); rf = np.empty((Br, self.S, 12))
        check(lib().hsddp_download_references(self._h, dp(rx), dp(ru), dp(rf)))
        return {"ref_x": rx, "ref_u": ru, "ref_foot": rf}

    # -- receding horizon (HKDProblem::update, HKDProblem.cpp:117-222) ------------------------
    def shift_elements(self, contact_change) -> dict:
        """hsddp_shift_elements: contact_change [B][n_steps], each element's own flags; returns the
        per-element layouts afterwards (element_layouts)."""
        cc = np.ascontiguousarray(contact_change, dtype=np.int32).reshape(self.B, -1)
        rc = lib().hsddp_shift_elements(self._h, int(cc.shape[1]), ip(cc))
        lay = self.element_layouts()
        self.P = int(lay["n_phases"].max())
        self.S = self.Kc + self.P
        check(rc)  # (a touchdown overflow is reported after the complete shift)
        return lay

    def _layout_arrays(self):
        """Every element's layout as arrays: n_phases [B], horizons / shooting / reach_end [B][16]
        (zeros past an element's phases)."""
        n = np.zeros(self.B, np.int32)
        hz, ss, re = (np.zeros((self.B, 16), np.int32) for _ in range(3))
        check(lib().hsddp_get_element_layouts(self._h, ip(n), ip(hz), ip(ss), ip(re)))
        return n, hz, ss, re

    def _follow_layout(self) -> bool:
        """The solver's P and S after a layout change (vectorised: the per-element Python lists of
        element_layouts cost milliseconds at B = 4096); True when the elements' layouts differ."""
        n, hz, _, _ = self._layout_arrays()
        if np.any(n != n[0]) or np.any(hz != hz[0]):
            self.P = int(n.max())
            self.S = self.Kc + self.P
            return True
        self.P = int(n[0])
        self.S = int((hz[0, :self.P] + 1).sum())
        return False

    def element_layouts(self) -> dict:
        n, hz, ss, re = self._layout_arrays()
        return {"n_phases": n, "horizons": [list(hz[b, :n[b]]) for b in range(self.B)],
                "shooting": [list(ss[b, :n[b]]) for b in range(self.B)],
                "reach_end": [list(re[b, :n[b]]) for b in range(self.B)]}

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
        rc = lib().hsddp_shift(self._h, int(cc.size), ip(cc))
        if self._follow_layout():  # per-element layouts
            check(rc)
            return self.element_layouts()
        lay = self.layout()
        self.P = len(lay["horizons"])
        self.S = sum(n + 1 for n in lay["horizons"])
        self.Kc = sum(lay["horizons"])
        check(rc)  # (a touchdown overflow is reported after the complete shift)
        return lay

    def update_problem(self, contacts, x0, ref_x=None, ref_u=None, ref_foot=None) -> None:
        """Inputs of the current layout, keeping the warm start (hsddp_update_problem).  References
        None: keep the ones hsddp_build_references made on the device for this layout."""
        self._contacts = None if contacts is None else np.ascontiguousarray(contacts, dtype=np.int32)
        refs = [None if r is None else np.ascontiguousarray(r, dtype=np.float64) for r in (ref_x, ref_u, ref_foot)]
        check(lib().hsddp_update_problem(self._h, None if contacts is None else ip(self._contacts),
                                         dp(np.ascontiguousarray(x0, dtype=np.float64)),
                                         *(None if r is None else dp(r) for r in refs)))

    def advance(self, x0=None, n_steps: int = 1, plan_duration: float = 0.6, dt_mpc: float = 0.01) -> list:
        """HKDProblem::update from the reference table (hsddp_advance): the window moves n_steps
        simulation steps, the layout, warm start, references and contacts follow, x0 [B][24] is the
        new initial state (None: call update_problem(None, x0) next, e.g. with x0 formed from the
        new first phase's contact).  Returns the contact-change flag of every step."""
        flags = np.zeros(max(1, n_steps), np.int32)
        rc = lib().hsddp_advance(self._h, int(n_steps), float(plan_duration), float(dt_mpc),
                                 None if x0 is None else dp(np.ascontiguousarray(x0, dtype=np.float64)), ip(flags))
        # a touchdown overflow (HSDDP_ERR_UNSUPPORTED) is reported after a complete step: the layout
        # is followed first
        self._follow_layout()
        check(rc)
        return [int(f) for f in flags[:n_steps]]

    def phase_info(self) -> dict:
        """contacts [B][P+1][4] (row P: the last phase's next contact); durations [B][P][4] when the
        references come from a table (else None)."""
        c = np.zeros((self.B, self.P + 1, 4), np.int32)
        d = np.zeros((self.B, self.P, 4))
        try:
            check(lib().hsddp_get_phase_info(self._h, ip(c), dp(d)))
        except HSDDPError:
            check(lib().hsddp_get_phase_info(self._h, ip(c), None))
            d = None
        return {"contacts": c, "durations": d}

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
