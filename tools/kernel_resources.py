#!/usr/bin/env python3
"""Per-kernel resource usage of the built gfx950 code objects.

Reads the AMDGPU metadata notes of every kernel in
node-fhe-accelerate_amd/build/obj/*.o (the .hip_fatbin offload bundle of
each object) and reports VGPRs, AGPRs, spills, scratch (private segment) and
LDS per kernel.  Used by tests/test_abi.py to assert that no shipped kernel
uses scratch, and by hand:

  python tools/kernel_resources.py [--spills-only] [obj ...]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ_DIR = os.path.join(ROOT, "node-fhe-accelerate_amd", "build", "obj")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _notes(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                              text=True).stdout


def _field(entry, key):
    m = re.search(r"\." + key + r":\s+(\S+)", entry)
    return m.group(1) if m else None


def kernels(objs=None):
    """[{obj, name, vgpr, agpr, vgpr_spill, sgpr_spill, scratch, lds}] for every kernel."""
    out = []
    for obj in objs or sorted(glob.glob(os.path.join(OBJ_DIR, "*.o"))):
        if os.path.basename(obj) == "fhe_gpu.o":
            continue
        text = _notes(obj)
        for ent in text.split("  - .agpr_count")[1:]:
            ent = ".agpr_count" + ent
            out.append({
                "obj": os.path.basename(obj), "name": _field(ent, "name"),
                "vgpr": int(_field(ent, "vgpr_count")), "agpr": int(_field(ent, "agpr_count")),
                "vgpr_spill": int(_field(ent, "vgpr_spill_count")), "sgpr_spill": int(_field(ent, "sgpr_spill_count")),
                "scratch": int(_field(ent, "private_segment_fixed_size")),
                "lds": int(_field(ent, "group_segment_fixed_size")),
            })
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.split("\n")


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ks = kernels(args or None)
    if "--spills-only" in sys.argv:
        ks = [k for k in ks if k["scratch"] or k["vgpr_spill"]]
    dem = demangle([k["name"] for k in ks])
    for k, d in zip(ks, dem):
        print(f"{k['obj']:16s} vgpr {k['vgpr']:3d} agpr {k['agpr']:3d} spill {k['vgpr_spill']:3d} "
              f"scratch {k['scratch']:4d} lds {k['lds']:6d}  {d[:110]}")
    print(f"{len(ks)} kernels")


if __name__ == "__main__":
    main()
