#!/usr/bin/env python3
"""Static VALU issue cycles of kernels in the built library (lab A/B before a
GPU run): instruction count and sum of per-mnemonic issue cycles
(profiles/r6_valu_rates.json) over one pass of the code, loops counted once.

usage: static_cycles.py SUBSTRING [SUBSTRING ...] [--lib PATH]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import isa_mix  # noqa: E402
import valu_roofline as vr  # noqa: E402

args = sys.argv[1:]
lib = isa_mix.LIB
if "--lib" in args:
    i = args.index("--lib")
    lib = args[i + 1]
    del args[i:i + 2]
rates = vr.load_rates()
names = sorted(isa_mix._disassembly(os.path.abspath(lib)))
for sub in args:
    for name in names:
        if sub in name:
            m = isa_mix.valu_mix(name, lib)
            cyc = sum(c * vr.issue_cycles(k, rates)[0] for k, c in m.items())
            print(f"{name[:90]:90s} insts {sum(m.values()):7d} cycles {cyc:9.0f}")
