#!/usr/bin/env python3
"""Kernel timing of ONE libfhe_gpu variant (lab tool; tools/gpu_ab.sh
interleaves variants across processes and rounds).

usage: FHE_GPU_LIB=build/libfhe_gpu_x.so ab_bench.py TAG [--ops fwd_mul,polymul] [--qs ...]
Prints one line per (op, q): TAG op q kernel_ms checksum.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "node-fhe-accelerate_amd"))
import torch  # noqa: E402
import fhe_gpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("--ops", default="fwd_mul,polymul")
ap.add_argument("--qs", default="132120577,4611686018326724609")
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--mode", default="compat")
args = ap.parse_args()
n, B = args.n, args.batch
for q in [int(x) for x in args.qs.split(",")]:
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.randint(0, q, (B, n), device="cuda", dtype=torch.int64, generator=g)
    b = torch.randint(0, q, (B, n), device="cuda", dtype=torch.int64, generator=g)
    out = torch.randint(0, q, (B, n), device="cuda", dtype=torch.int64, generator=g)
    ring = fhe_gpu.PolynomialRing(n, q, mode=args.mode)
    eps = {}
    for bl, lv in ((23, 1), (15, 2)):
        ggsw = torch.randint(0, q, (2 * lv, 2, n), device="cuda", dtype=torch.int64, generator=g)
        eps[lv] = fhe_gpu.ExternalProduct(ring, ggsw, bl, lv)
    eng = fhe_gpu.EncryptionEngine(ring)
    nct = B // 4  # ciphertexts for ct_mul / relin
    cx, cy = a[: 2 * nct].view(nct, 2, n), b[: 2 * nct].view(nct, 2, n)
    c3 = out[: 3 * nct].view(nct, 3, n)
    c2 = a[2 * nct: 4 * nct].view(nct, 2, n)
    ek = fhe_gpu.EvaluationKey(ring, torch.randint(0, q, (7, 2, n), device="cuda", dtype=torch.int64, generator=g), 4)
    glwe = a[: B // 2].view(B // 4, 2, n)  # B/4 ciphertexts (k = 1)
    gout = out[: B // 2].view(B // 4, 2, n)
    # br256: tfhe-256-secure blind rotation (N = 4096, n = 1024, (10, 3),
    # Q_60_1), batch 64 -- only with --n 4096 --qs 1152921504606584833
    br = None
    if "br256" in args.ops and n == 4096:
        be = fhe_gpu.BootstrapEngine(ring, 10, 3, 1)
        bsk = be.prepare_ggsw(torch.randint(0, q, (1024, 6, 2, n), device="cuda", dtype=torch.int64, generator=g))
        la = torch.randint(0, q, (64, 1024), device="cuda", dtype=torch.int64, generator=g)
        lb = torch.randint(0, q, (64,), device="cuda", dtype=torch.int64, generator=g)
        acc = torch.randint(0, q, (64, 2, n), device="cuda", dtype=torch.int64, generator=g)
        acc0 = acc.clone()
        br = (be, bsk, la, lb, acc, acc0)

    # br8192: N = 8192 (per-step k_dmac MODE 2 launches), q62, (23, 1), 64
    # steps, batch 64 -- only with --n 8192
    if "br8192" in args.ops and n == 8192:
        be = fhe_gpu.BootstrapEngine(ring, 23, 1, 1)
        bsk = be.prepare_ggsw(torch.randint(0, q, (64, 2, 2, n), device="cuda", dtype=torch.int64, generator=g))
        la = torch.randint(0, q, (64, 64), device="cuda", dtype=torch.int64, generator=g)
        lb = torch.randint(0, q, (64,), device="cuda", dtype=torch.int64, generator=g)
        acc = torch.randint(0, q, (64, 2, n), device="cuda", dtype=torch.int64, generator=g)
        br = (be, bsk, la, lb, acc, acc.clone())

    def br_run():
        be_, bsk_, la_, lb_, acc_, acc0_ = br
        acc_.copy_(acc0_)
        be_.blind_rotate(acc_, la_, lb_, bsk_)
    for op in args.ops.split(","):
        fn = {"fwd_mul": lambda: ring.forward_ntt_mul(a, b, out=out),
              "polymul": lambda: ring.multiply(a, b, out=out),
              "fwd": lambda: ring.forward_ntt(a, out=out),
              "inv": lambda: ring.inverse_ntt(a, out=out),
              "ext1": lambda: eps[1](glwe, out=gout),
              "ext2": lambda: eps[2](glwe, out=gout),
              "ct_mul": lambda: eng.multiply(cx, cy, out=c3),
              "relin": lambda: eng.relinearize(c3, ek, out=c2),
              "br256": br_run, "br8192": br_run}[op]
        fn()
        torch.cuda.synchronize()
        res = {"ext1": gout, "ext2": gout, "relin": c2, "ct_mul": c3}.get(op, out) if not op.startswith("br") else br[4]
        chk = int(res.sum().item()) ^ int(res[-1].sum().item())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        qtag = q if args.mode == "compat" else f"{q}/{args.mode}"
        print(f"AB {args.tag} {op} {qtag} {ms:.4f} {chk}", flush=True)
    del a, b, out
    torch.cuda.empty_cache()
