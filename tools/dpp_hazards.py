"""Scan gfx950 assembly for VALU-write -> DPP-read hazards the compiler cannot see.

DPP instructions issued from inline asm (hsddp_wave.h) bypass LLVM's hazard recognizer: a DPP
source VGPR written by a VALU instruction fewer than two wait states earlier reads a stale value
(LLVM GCNHazardRecognizer::checkDPPHazards, DppVgprWaitStates = 2).  This walks each kernel's
instruction stream linearly (fall-through order; s_nop N = N + 1 wait states, every other
instruction 1) and reports DPP reads of a VGPR written by a VALU instruction within the last two
wait states.

usage: python tools/dpp_hazards.py file.s [more.s ...]   (exit status 1 when a hazard is found)
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok):
    out = []
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.append(int(m.group(3)))
        else:
            out.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan(path):
    bad = []
    kernel = "?"
    last_write = {}  # vgpr -> wait-state clock of its last VALU write
    clock = 0
    for ln, line in enumerate(open(path), 1):
        s = line.split(";")[0].strip()
        if not s or s.startswith("."):
            continue  # directives and basic-block labels: fall-through order is kept
        if s.endswith(":"):
            kernel = s[:-1]
            last_write.clear()
            continue
        mn, _, rest = s.partition(" ")
        ops = [o.strip() for o in rest.split(",")] if rest else []
        if mn == "s_nop":
            clock += (int(ops[0], 0) if ops else 0) + 1
            continue
        clock += 1
        if not mn.startswith("v_"):
            continue
        if "_dpp" in mn or "row_" in rest or "quad_perm" in rest:
            src0 = ops[1].split(" ")[0] if len(ops) > 1 else ""
            for r in regs(src0):
                if r in last_write and clock - last_write[r] <= 2:
                    bad.append((path, ln, kernel, s))
                    break
        # destinations: the first operand (vcc / sgpr destinations have no VGPR); the swaps write both
        dsts = []
        if ops and not mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
            dsts += regs(ops[0].split(" ")[0])
        if mn.startswith("v_permlane") and "swap" in mn and len(ops) > 1:
            dsts += regs(ops[1])
        for r in dsts:
            last_write[r] = clock
    return bad


def main():
    bad = []
    for p in sys.argv[1:]:
        bad += scan(p)
    for path, ln, k, s in bad:
        print(f"{path}:{ln}: [{k[:60]}] {s}")
    print(f"{len(bad)} DPP read(s) within two wait states of a VALU write")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
