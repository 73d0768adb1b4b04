#!/usr/bin/env python3
"""Phase shares of the two-CU blind rotation (lab; needs the stamp build).

  tools/lab/quick_variant2.sh stamp "ntt_br" -DFHE_BR_STAMPS=1
  FHE_GPU_LIB=node-fhe-accelerate_amd/build/libfhe_gpu_stamp.so FHE_BR_STAMPS=1 \
      python tools/lab/br_stamps.py [--batch 64] [--dim 256]

The library prints one "[br stamps]" line per launch to stderr; also times
the production kernel of FHE_GPU_LIB without stamps when FHE_BR_STAMPS=0.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "node-fhe-accelerate_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import fhe_gpu  # noqa: E402
from bench import BR_PRESETS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--dim", type=int, default=0, help="LWE dimension (0 = the preset's)")
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(5)
for name, n, dim, bl, lv, q in BR_PRESETS + [("tfhe-128-fast/q62", 1024, 742, 23, 1, 4611686018326724609)]:
    dim = args.dim or dim
    ring = fhe_gpu.PolynomialRing(n, q)
    be = fhe_gpu.BootstrapEngine(ring, bl, lv, 1)
    bsk = be.prepare_ggsw(torch.randint(0, q, (dim, 2 * lv, 2, n), device="cuda", dtype=torch.int64, generator=g))
    b = args.batch
    la = torch.randint(0, q, (b, dim), device="cuda", dtype=torch.int64, generator=g)
    lb = torch.randint(0, q, (b,), device="cuda", dtype=torch.int64, generator=g)
    acc = torch.randint(0, q, (b, 2, n), device="cuda", dtype=torch.int64, generator=g)
    be.blind_rotate(acc, la, lb, bsk)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        be.blind_rotate(acc, la, lb, bsk)
    e1.record()
    torch.cuda.synchronize()
    print(f"{name} N={n} dim={dim} batch={b}: {e0.elapsed_time(e1) / args.reps:.3f} ms per launch", flush=True)
