#!/usr/bin/env python3
"""Fixtures for the reference-construction tests: the first samples of
three of the reference's own trajectory data files, unchanged (data, not source):

    Reference/Data/trot/quad_reference.csv            -> ref_trot.csv      (130 samples)
    Reference/Data/flytrot/quad_reference.csv         -> ref_flytrot.csv   (110 samples)
    Reference/Data/gaitLib/run_jump/quad_reference.csv -> ref_run_jump.csv (40 samples; its dt is NaN, quirk A16)

Run in the build container (where /root/reference exists):  python tests/golden/make_ref_fixtures.py
"""
import os

SRC = "/root/reference/Reference/Data"
HERE = os.path.dirname(os.path.abspath(__file__))
FILES = [("trot/quad_reference.csv", "ref_trot.csv", 130), ("flytrot/quad_reference.csv", "ref_flytrot.csv", 110),
         ("gaitLib/run_jump/quad_reference.csv", "ref_run_jump.csv", 40)]

for src, dst, n in FILES:
    out, count = [], 0
    with open(os.path.join(SRC, src)) as f:
        lines = f.read().split("\n")
    i = 0
    while i < len(lines) and count < n:
        out.append(lines[i])
        if "status_dur" in lines[i]:
            out.append(lines[i + 1])
            i += 1
            count += 1
        i += 1
    with open(os.path.join(HERE, dst), "w") as f:
        f.write("\n".join(out) + "\n")
    print(dst, count, "samples")
