#!/usr/bin/env python3
"""Static instruction mix of one kernel in a built object (lab tool).
usage: isa_stats.py <obj.o> <kernel-substring> [--dump]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj, sub = sys.argv[1], sys.argv[2]
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True, text=True).stdout
funcs = re.split(r"\n(?=[0-9a-f]+ <)", txt)
for f in funcs:
    head = f.split("\n", 1)[0]
    name = subprocess.run(["c++filt"], input=head.split("<", 1)[-1].rstrip(">:"), capture_output=True, text=True).stdout.strip()
    if sub not in name:
        continue
    ins = [l.strip().split()[0] for l in f.split("\n")[1:] if l.strip() and not l.strip().startswith(";") and ":" not in l.split()[0]]
    c = collections.Counter()
    for i in ins:
        if i.startswith("v_mul") or i.startswith("v_mad"):
            c["v_mul/mad"] += 1
        elif i.startswith("v_"):
            c["v_other"] += 1
        elif i.startswith("ds_"):
            c[i] += 1
        elif i.startswith("buffer_") or i.startswith("global_") or i.startswith("scratch_"):
            c[i.split("_")[0] + "_" + i.split("_")[1]] += 1
        elif i in ("s_waitcnt", "s_barrier", "s_nop"):
            c[i] += 1
        elif i.startswith("s_load") or i.startswith("s_buffer"):
            c["s_load"] += 1
        elif i.startswith("s_"):
            c["s_other"] += 1
    print(name[:120])
    print("  total", len(ins), dict(sorted(c.items())))
    if "--dump" in sys.argv:
        print(f)
