#!/usr/bin/env python3
"""Timing of the composed blind rotation (GLWE dimension k > 1, N > 16384;
fhe_gpu.cpp blind_rotate_composed) on device-resident buffers (lab tool).

usage: br_composed.py [--dim 742] [--batches 1,64]
Prints one JSON line per shape: ms per batch and bootstraps/s."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "node-fhe-accelerate_amd"))
import torch  # noqa: E402
import fhe_gpu  # noqa: E402

P62 = 4611686018326724609
ap = argparse.ArgumentParser()
ap.add_argument("--dim", type=int, default=742)
ap.add_argument("--batches", default="1,64")
args = ap.parse_args()
for n, k, bl, lv in ((1024, 2, 15, 2), (2048, 2, 15, 2), (32768, 1, 23, 1)):
    r = fhe_gpu.PolynomialRing(n, P62)
    be = fhe_gpu.BootstrapEngine(r, bl, lv, k)
    g = torch.Generator(device="cuda").manual_seed(3)
    bsk = torch.randint(0, P62, (args.dim, (k + 1) * lv, k + 1, n), device="cuda", dtype=torch.int64, generator=g)
    bsk_ntt = be.prepare_ggsw(bsk)
    for b in [int(x) for x in args.batches.split(",")]:
        lwe_a = torch.randint(0, P62, (b, args.dim), device="cuda", dtype=torch.int64, generator=g)
        lwe_b = torch.randint(0, P62, (b,), device="cuda", dtype=torch.int64, generator=g)
        acc = torch.randint(0, P62, (b, k + 1, n), device="cuda", dtype=torch.int64, generator=g)
        be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"n": n, "k": k, "base_log": bl, "level": lv, "lwe_dim": args.dim, "batch": b,
                          "ms_per_batch": round(ms, 2), "per_s": round(b / ms * 1e3, 1)}), flush=True)
