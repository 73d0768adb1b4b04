#!/usr/bin/env python3
"""Lab diagnostic: run bench.py's main() in this process and, at Python exit,
save /proc/self/maps (and the loaded libfhe_gpu contexts still alive) to a
file, so the addresses of a crash in C-level exit handlers (after Python's
own finalisation) can be mapped to the libraries they belong to.

usage: python3 tools/lab/exit_maps.py <maps-out> [--close] -- <bench.py args>
  --close: also destroy every live context (fhe_ctx_destroy) in the atexit
           hook, before interpreter teardown
Run under rocprofv3 with `-- python3 tools/lab/exit_maps.py ...` (never a
shell or env hop)."""
import atexit
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = sys.argv[1]
args = sys.argv[sys.argv.index("--") + 1:]
CLOSE = "--close" in sys.argv[: sys.argv.index("--")]


def _dump():
    live = 0
    try:
        import fhe_gpu

        objs = [o for o in gc.get_objects() if isinstance(o, (fhe_gpu.NTTProcessor, fhe_gpu.RNSPolynomialRing))]
        live = sum(1 for o in objs if getattr(o, "_h", None) is not None)
        if CLOSE:
            for o in objs:
                o.close()
    except Exception:
        pass
    with open(out, "w") as f:
        f.write(f"# live contexts at Python atexit: {live}\n")
        f.write(open("/proc/self/maps").read())


atexit.register(_dump)
sys.argv = [os.path.join(ROOT, "bench.py")] + args
sys.path.insert(0, ROOT)
import bench  # noqa: E402

bench.main()
