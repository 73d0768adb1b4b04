#!/usr/bin/env python3
"""Static VALU instruction mix of a kernel in the shipped library.

Reads node-fhe-accelerate_amd/build/libfhe_gpu.so itself (its .hip_fatbin
section holds one offload bundle per translation unit), disassembles the
gfx950 code objects and counts, for the kernel whose demangled name equals
the one a profile summary records, its vector-ALU instructions by mnemonic.
bench.py weights the dynamic SQ_INSTS_VALU count of a profile by this mix
and the measured per-instruction issue costs (profiles/r6_valu_rates.json)
to get the kernel's VALU issue floor (its second roofline).

usage: python3 tools/isa_mix.py "<demangled kernel name>" [lib.so]
"""
import collections
import functools
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "node-fhe-accelerate_amd", "build", "libfhe_gpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


@functools.lru_cache(maxsize=2)
def _disassembly(lib):
    """{demangled kernel name: [mnemonic, ...]} for every gfx950 kernel in lib."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "x.so")],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
        for i, s in enumerate(starts):
            e = starts[i + 1] if i + 1 < len(starts) else len(blob)
            part, co = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"b{i}.co")
            open(part, "wb").write(blob[s:e])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                f"--targets={TARGET}", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                                 text=True).stdout
            funcs = re.split(r"\n(?=[0-9a-f]+ <)", txt)
            heads, bodies = [], []
            for f in funcs:
                head = f.split("\n", 1)[0]
                if "<" not in head:
                    continue
                heads.append(head.split("<", 1)[-1].rstrip(">:"))
                bodies.append(f)
            if not heads:
                continue
            names = subprocess.run(["c++filt"], input="\n".join(heads), capture_output=True, text=True).stdout.split("\n")
            for name, f in zip(names, bodies):
                ins = []
                for line in f.split("\n")[1:]:
                    t = line.strip()
                    if not t or t.startswith(";") or t.endswith(":"):
                        continue
                    ins.append(t.split()[0])
                out[name.strip()] = ins
    return out


def base_mnemonic(m):
    """v_add_u32_e32 -> v_add_u32 (encoding suffix dropped)."""
    return re.sub(r"_(e32|e64|sdwa|dpp)$", "", m)


def valu_mix(kernel_name, lib=LIB):
    """Counter {base mnemonic: static count} of the kernel's v_* instructions
    (MFMA excluded: none in this library), or None if the kernel is absent."""
    ins = _disassembly(os.path.abspath(lib)).get(kernel_name)
    if ins is None:
        return None
    return collections.Counter(base_mnemonic(i) for i in ins if i.startswith("v_") and not i.startswith("v_mfma"))


if __name__ == "__main__":
    mix = valu_mix(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else LIB)
    print(json.dumps(dict(mix.most_common()) if mix is not None else None, indent=1))
