"""CPU tests of the host-side logic: INFO loaders (the ddp_setting.info surface), the C-ABI library
(loads, exports every declared symbol, refuses to run without a GPU), synthetic problem assembly."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import hsddp
from hsddp import _lib, synthetic as syn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "hsddp.h")).read()
    declared = set(re.findall(r"\b(hsddp_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS)
    L = C.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(L, name), name


def test_no_device_fails_loudly():
    import ctypes
    ndev = ctypes.c_int(0)
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipGetDeviceCount(ctypes.byref(ndev))
    except OSError:
        pass
    if ndev.value > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(hsddp.HSDDPError, match="no HIP device"):
        hsddp.Solver(syn.make_batch(2, 2, 5))


def test_settings_loader_matches_reference_semantics(tmp_path):
    o = hsddp.load_settings()
    assert o.alpha == 0.1 and o.gamma == 0.01 and o.update_penalty == 5
    assert o.max_DDP_iter == 10 and o.max_AL_iter == 5 and o.merit_offset == 100
    assert o.AL_active == 1 and o.ReB_active == 1 and o.MS == 1
    # quirk A1: update_regularization / smooth_active are never read by loadHSDDPSetting
    assert o.update_regularization == 2 and o.smooth_active == 0
    # a missing key raises like boost::property_tree::ptree_bad_path (stale HKDMPC/ddp_setting.info)
    bad = tmp_path / "stale.info"
    bad.write_text("ddp\n{\n alpha 0.1\n gamma 0.01\n}\n")
    with pytest.raises(hsddp.HSDDPError, match="No such node"):
        hsddp.load_settings(str(bad))
    # comments, quoting, ';' after a value (ddp_setting.info:15 "1e-3;")
    good = tmp_path / "ok.info"
    txt = open(os.path.join(ROOT, "hkd-mpc_amd", "settings", "ddp_setting.info")).read()
    good.write_text(txt.replace("dynamics_feas_thresh    1e-3", 'dynamics_feas_thresh    "2e-3";'))
    assert hsddp.load_settings(str(good)).dynamics_feas_thresh == 2e-3
    with pytest.raises(hsddp.HSDDPError):
        hsddp.load_settings(str(tmp_path / "missing.info"))


def test_constraint_params_loader():
    cp = hsddp.load_constraint_params()
    assert (cp.grf_delta, cp.grf_delta_min, cp.grf_eps) == (0.1, 0.1, 0.1)
    assert (cp.td_sigma, cp.td_sigma_max, cp.td_lambda) == (50, 1e4, 0)
    assert cp.mu_fric == 0.7


def test_default_options_are_hsddp_option_defaults():
    o = hsddp.default_options()
    assert (o.alpha, o.gamma, o.update_penalty, o.update_relax, o.update_ReB) == (0.1, 0.1, 8, 0.1, 7)
    assert (o.max_DDP_iter, o.max_AL_iter, o.merit_offset) == (3, 2, 10)


@pytest.mark.parametrize("gait,P,N", [("trot", 4, 50), ("jump", 8, 25)])
def test_synthetic_batch_layout(gait, P, N):
    prob = syn.make_batch(5, P, N, gait)
    S, Kc = prob["S"], prob["Kc"]
    assert S == P * (N + 1) and Kc == P * N
    assert prob["contacts"].shape == (5, P + 1, 4) and prob["contacts"].dtype == np.int32
    assert prob["ref_x"].shape == (1, S, 24) and prob["Xbar"].shape == (5, S, 24)
    cyc = syn.GAITS[gait]
    for i in range(P + 1):
        assert tuple(prob["contacts"][0, i]) == cyc[i % len(cyc)]
    # x0: stance feet from forward kinematics, swing legs at the nominal joint angles
    c0 = prob["contacts"][0, 0]
    for leg in range(4):
        if not c0[leg]:
            assert np.allclose(prob["x0"][0, 12 + 3 * leg:15 + 3 * leg], syn.QJ_NOMINAL)
    # seeded splitmix64: the same element always gets the same x0
    again = syn.make_batch(2, P, N, gait)
    assert np.array_equal(again["x0"], prob["x0"][:2])


def test_mixed_batch_has_per_element_reference():
    prob = syn.make_batch(16, 4, 10, mixed=True)
    assert prob["ref_x"].shape[0] == 16
    assert len(set(prob["gaits"])) > 1


def test_splitmix64_known_values():
    # first outputs of splitmix64 seeded with 0 (published test vector)
    s, v = syn.splitmix64(0)
    assert v == 0xE220A8397B1DCDAF
    s, v = syn.splitmix64(s)
    assert v == 0x6E789E6AA1B965F4


def test_validate_options_refuses_unending_regularisation_schedule():
    """backward_sweep_regularized (MultiPhaseDDP.cpp:150-167) never reaches mu > 1e2 with a factor
    <= 1; the C-ABI refuses such options (hsddp_set_options applies the same check) instead of
    leaving a GPU wave spinning."""
    L = _lib.lib()
    ok = hsddp.default_options()
    assert L.hsddp_validate_options(C.byref(ok)) == 0
    for f in (1.0, 0.5, -2.0, float("nan"), 1.01):  # 1.01: > HSDDP_MAX_REG_ATTEMPTS retries
        o = hsddp.default_options(update_regularization=f)
        assert L.hsddp_validate_options(C.byref(o)) == -1, f  # HSDDP_ERR_ARG
        assert b"update_regularization" in L.hsddp_last_error()
    o = hsddp.default_options(update_regularization=1.5)   # 30 retries: accepted
    assert L.hsddp_validate_options(C.byref(o)) == 0
    o = hsddp.default_options(alpha=1.0)
    assert L.hsddp_validate_options(C.byref(o)) == -1


def test_every_handle_entry_point_refuses_a_null_handle():
    """Every C-ABI function that takes a handle returns HSDDP_ERR_ARG for a NULL handle (NULL
    pointers and zeros elsewhere) without touching a device; hsddp_destroy(NULL) is a no-op and
    hsddp_device_bytes(NULL) is 0 (include/hsddp.h)."""
    hdr = open(os.path.join(ROOT, "include", "hsddp.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    hdr = re.sub(r"//[^\n]*", "", hdr)
    L = C.CDLL(_lib.LIB_PATH)
    err_arg = int(re.search(r"HSDDP_ERR_ARG\s*=\s*(-?\d+)", open(os.path.join(ROOT, "include", "hsddp.h")).read()).group(1))
    seen = 0
    for ret, name, args in re.findall(r"\b([a-z_0-9 ]+?\**)\s*\b(hsddp_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", hdr):
        params = [a.strip() for a in args.split(",") if a.strip()]
        if not params or not params[0].startswith("hsddp_handle"):
            continue
        vals = []
        for a in params:
            if "*" in a or a.startswith("hsddp_handle"):
                vals.append(None)
            elif a.startswith("double"):
                vals.append(C.c_double(0))
            elif a.startswith("float"):
                vals.append(C.c_float(0))
            else:
                vals.append(C.c_int(0))
        f = getattr(L, name)
        f.restype = C.c_size_t if "size_t" in ret else C.c_int
        rc = f(*vals)
        want = 0 if name in ("hsddp_destroy", "hsddp_device_bytes") else err_arg
        assert rc == want, (name, rc)
        seen += 1
    assert seen >= 30
