"""Build-time checks of the device code (no GPU): the inline-asm DPP instructions of the sweep
(hsddp_wave.h) are invisible to LLVM's hazard recognizer, so the emitted gfx950 assembly of every
kernel file is scanned for a DPP read of a VGPR written by a VALU instruction fewer than two wait
states earlier (tools/dpp_hazards.py; such a read returns the register's previous value)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_dpp_hazards_in_device_code():
    r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "hkd-mpc_amd", "csrc"), "hazards"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "0 DPP read(s)" in r.stdout
