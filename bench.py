#!/usr/bin/env python3
"""Benchmark of the NTT hot path on MI355X (BASELINE.json metric:
"NTTs/s + polymuls/s at degree 16384 (batched), 1/2/4/8 MI355X; % HBM roofline").

Workload (one "step" = one pass of the hot path over one batch):
  C3  forward NTT fused with pointwise modmul, N=16384, batch 65536 per GPU,
      q = 132120577 (SURVEY.md 8 primary prime); value = NTTs/s (all GPUs)
  C4  polynomial multiply inv(fwd(a).fwd(b)), same batch -> polymuls/s
Inputs are synthetic uniform residues generated on device and resident in
HBM before the timed region.  Multi-GPU: one process per GPU, the batch is
sharded (each rank owns its own 65536 polynomials: weak scaling), no
collective in the data path; barrier + max-over-ranks timing.

  python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "node-fhe-accelerate_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

P27 = 132120577
P62 = 4611686018326724609
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--batch", type=int, default=65536, help="polynomials per GPU")
    ap.add_argument("--q", type=int, default=P27)
    ap.add_argument("--q62", action="store_true", help="also measure the 62-bit prime")
    ap.add_argument("--no-q62", dest="q62", action="store_false")
    ap.set_defaults(q62=True)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--mode", default="compat", choices=["compat", "negacyclic"],
                    help="transform of the --only profiling runs (the default run reports both)")
    ap.add_argument("--only", default="", help="run only this kernel (fwd_mul|polymul|fwd|inv) for profiling")
    ap.add_argument("--no-check", action="store_true", help="skip the oracle spot check (profiling runs)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-resident (FHE_HOST, PCIe) measurement")
    ap.add_argument("--only-host", action="store_true", help="only the host-resident measurement (lab)")
    ap.add_argument("--no-cipher", dest="cipher", action="store_false",
                    help="skip the ciphertext-level side metrics (ct multiply, relinearize, blind rotate)")
    return ap.parse_args()


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) started without a launcher: run N fresh
    rank processes under torch.distributed.run (one per GPU) as CHILDREN of
    this process and return their exit code.  Called before anything touches
    the GPU; the parent never re-execs itself.  Rank 0 prints the JSON line."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # one process per GPU.  More ranks than devices (rehearsing N ranks on a
    # one-GPU box) share devices round-robin and need FHE_DIST_BACKEND=gloo:
    # RCCL refuses two ranks on one GPU.
    ndev = max(1, torch.cuda.device_count())
    dev = local % ndev
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("FHE_DIST_BACKEND", "nccl" if world <= ndev else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        return dist, rank, world, dev
    return None, rank, world, dev


def barrier(dist):
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(dist, v):
    if dist is None:
        return v
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(dist, fn, steps, warmup):
    """Returns (wall seconds for `steps` calls max over ranks, avg kernel ms by
    HIP events on the launch stream)."""
    for _ in range(warmup):
        fn()
    barrier(dist)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(steps):
        fn()
    e1.record(s)
    barrier(dist)
    wall = time.perf_counter() - t0
    kernel_ms = e0.elapsed_time(e1) / steps
    return max_over_ranks(dist, wall), max_over_ranks(dist, kernel_ms)


def gpu_workload(fhe_gpu, n, q, batch, steps, warmup, dist, only="", check=True, mode="compat"):
    ring = fhe_gpu.PolynomialRing(n, q, mode=mode, device=torch.cuda.current_device())
    g = torch.Generator(device="cuda").manual_seed(1234 + int(os.environ.get("RANK", "0")))
    a = torch.randint(0, q, (batch, n), device="cuda", dtype=torch.int64, generator=g)
    b = torch.randint(0, q, (batch, n), device="cuda", dtype=torch.int64, generator=g)
    out = torch.empty_like(a)
    res = {}
    checks = []
    # after each timed region: rows 0, mid and last of the output buffer the
    # timed launches wrote, bit-exact vs the oracle (outside timing)
    if only in ("", "fwd_mul"):
        res["fwd_mul"] = timed(dist, lambda: ring.forward_ntt_mul(a, b, out=out), steps, warmup)
        if check and mode == "compat":
            checks.append(_check_rows("fwd_mul", a, b, out, n, q))
    if dist is not None and only in ("", "fwd_mul"):
        res["gather"] = time_gather(dist, out, n)
    if only in ("", "polymul"):
        res["polymul"] = timed(dist, lambda: ring.multiply(a, b, out=out), steps, warmup)
        if check and mode == "compat":
            checks.append(_check_rows("polymul", a, b, out, n, q))
    if only == "fwd":
        res["fwd"] = timed(dist, lambda: ring.forward_ntt(a, out=out), steps, warmup)
    if only == "inv":
        res["inv"] = timed(dist, lambda: ring.inverse_ntt(a, out=out), steps, warmup)
    if not check:
        res["parity_ok"] = "skipped"
    elif mode == "negacyclic":
        res["parity_ok"] = _spot_check_negacyclic(ring, a, b, out, n, q)
    else:
        res["parity_ok"] = all(c is True for c in checks) if checks else "unchecked"
        res["parity_rows"] = f"rows 0, {batch // 2}, {batch - 1} of each timed output buffer"
        if any(c is not True for c in checks):
            res["parity_detail"] = [c for c in checks if c is not True]
    del a, b, out
    torch.cuda.empty_cache()
    return res


def time_gather(dist, out, n, polys=4096):
    """the optional result gather to rank 0 (RCCL over xGMI
    with the nccl backend), timed on its own and never part of `value`:
    `polys` result polynomials per rank (512 MiB at N=16384) gathered into
    rank 0."""
    from fhe_gpu.shard import gather_to_root

    world, rank = dist.get_world_size(), dist.get_rank()
    g = min(polys, out.shape[0])
    local = out[:g]
    if dist.get_backend() != "nccl":
        local = local.cpu()  # gloo gathers host tensors
    gather_to_root(local, g * world, rank, world)  # warm-up (communicator setup)
    barrier(dist)
    t0 = time.perf_counter()
    full = gather_to_root(local, g * world, rank, world)
    barrier(dist)
    ms = max_over_ranks(dist, (time.perf_counter() - t0) * 1e3)
    del full
    nbytes = g * n * 8 * world
    return {"backend": dist.get_backend(), "polys_per_rank": g, "bytes_into_root": nbytes, "ms": ms,
            "GBps_into_root": nbytes / (ms * 1e-3) / 1e9}


def host_resident(fhe_gpu, n, q, polys=8192, reps=3):
    """SURVEY.md 8(d) / BASELINE.md section 2: the FHE_HOST path (what the
    N-API addon hands over: pageable host arrays in, host array out), timed
    end to end -- H2D + kernel + D2H, pipelined over pinned staging slots
    (fhe_gpu.cpp staged()).  Never `value`.  Also the raw pageable H2D / D2H
    copy rates on this box (torch), for the PCIe bound."""
    ring = fhe_gpu.PolynomialRing(n, q, device=torch.cuda.current_device())
    rng = np.random.default_rng(5)
    a = rng.integers(0, q, size=(polys, n), dtype=np.uint64)
    w = rng.integers(0, q, size=(polys, n), dtype=np.uint64)
    o = np.empty_like(a)
    ring.forward_ntt_mul(a[:64], w[:64], out=o[:64])  # warm-up (staging buffers)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        ring.forward_ntt_mul(a, w, out=o)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    moved = 24 * n * polys  # a, w in; out back
    res = {"polys": polys, "n": n, "q": q, "ntt_per_s": polys / best, "ms": best * 1e3,
           "pcie_GBs_moved": moved / best / 1e9, "bytes_per_ntt": 24 * n}
    # raw copy rates, pageable host memory (as the FHE_HOST caller has it)
    x = torch.from_numpy(a.view(np.int64))
    d = torch.empty(x.shape, dtype=torch.int64, device="cuda")
    d.copy_(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(x)
    torch.cuda.synchronize()
    h2d = x.numel() * 8 / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    x.copy_(d)
    torch.cuda.synchronize()
    d2h = x.numel() * 8 / (time.perf_counter() - t0) / 1e9
    res["h2d_pageable_GBs"], res["d2h_pageable_GBs"] = h2d, d2h
    # bound: 16N bytes in and 8N out per NTT, the two directions overlapped
    res["pcie_bound_ntt_per_s"] = min(h2d * 1e9 / (16 * n), d2h * 1e9 / (8 * n))
    res["frac_of_pcie_bound"] = res["ntt_per_s"] / res["pcie_bound_ntt_per_s"]
    ok = bool((o[[0, polys - 1]] == __import__("oracle").NTT(n, q).fwd_mul(a[[0, polys - 1]], w[[0, polys - 1]])).all())
    res["parity_ok"] = ok
    del d
    torch.cuda.empty_cache()
    return res


def _check_rows(kind, a, b, out, n, q):
    """Rows 0, mid and last of the buffer the timed launches wrote, bit-exact
    against the CPU oracle (fwd_mul or polymul), outside the timed region."""
    try:
        import oracle

        torch.cuda.synchronize()
        t = oracle.NTT(n, q)
        rows = [0, a.shape[0] // 2, a.shape[0] - 1]
        xa = a[rows].cpu().numpy().view(np.uint64)
        xb = b[rows].cpu().numpy().view(np.uint64)
        got = out[rows].cpu().numpy().view(np.uint64)
        exp = t.fwd_mul(xa, xb) if kind == "fwd_mul" else t.polymul(xa, xb)
        return True if bool((got == exp).all()) else f"{kind}: mismatch"
    except Exception as e:  # pragma: no cover
        return f"{kind} unchecked: {e}"


def _spot_check_negacyclic(ring, a, b, out, n, q):
    """Negacyclic mode: the polymul rows are the ring product a*b mod (X^N+1)
    (checked by the identity (a*b)(x) = a(x) b(x) at a random point x of the
    field, for X^N = -1: x^N = -1 mod q picks x = psi^(2j+1)), and the
    fwd_mul rows satisfy inv(fwd_mul(a, fwd(b))) == a*b."""
    try:
        rows = [0, a.shape[0] - 1]
        xa, xb = a[rows].contiguous(), b[rows].contiguous()
        c = ring.multiply(xa, xb).cpu().numpy().view(np.uint64)
        psi = ring.primitive_root
        x = pow(psi, 2 * 12345 + 1, q)  # a root of X^N + 1
        ok = True
        def ev(p):  # Horner evaluation of p at x mod q
            acc = 0
            for coef in reversed(p.tolist()):
                acc = (acc * x + coef) % q
            return acc

        for r in range(len(rows)):
            pa, pb = xa[r].cpu().numpy().view(np.uint64), xb[r].cpu().numpy().view(np.uint64)
            ok &= (ev(pa) * ev(pb)) % q == ev(c[r])
        fb = ring.forward_ntt(xb)
        fm = ring.forward_ntt_mul(xa, fb)
        ok &= bool((ring.inverse_ntt(fm).cpu().numpy().view(np.uint64) == c).all())
        torch.cuda.synchronize()
        return bool(ok)
    except Exception as e:  # pragma: no cover
        return f"unchecked: {e}"


def negacyclic_workload(fhe_gpu, n, q, batch, steps, warmup, dist):
    """north_star's forward negacyclic NTT (psi-twisted cyclic transform,
    FHE_MODE_NEGACYCLIC) timed like the headline: C3 fwd NTT + modmul and C4
    polymul, same batch, HIP-event kernel time, HBM fraction."""
    r = gpu_workload(fhe_gpu, n, q, batch, steps, warmup, None if dist is None else dist, mode="negacyclic")
    out = {"mode": "negacyclic", "n": n, "q": q, "batch": batch, "parity_ok": r["parity_ok"]}
    for key in ("fwd_mul", "polymul"):
        wall, kms = r[key]
        ach = 24 * n * batch / (kms * 1e-3) / 1e9
        out[key] = {"per_s": batch * steps / wall, "kernel_ms": kms, "achieved_GBs": ach,
                    "frac": ach / HBM_PEAK_GBS, "bytes_per_unit": 24 * n}
        _attach(out[key], pmc_traffic(key, n, batch, q, mode="negacyclic"), 24 * n * batch, kms)
    return out


def engine_chain(fhe_gpu, n=16384, q=1152921504606584833, t=65537, batch=256, reps=3):
    """The FHEEngine chain encrypt -> multiply -> relinearize -> decrypt per
    second at N=16384 (q = Q_60_1, t = 65537, base 2^20, 3 levels), on the
    host-resident (FHE_HOST: every call stages host arrays through HBM, what
    the N-API array calls do) and the device-resident (DeviceBuffer handles:
    what lib/engine.js keeps) paths.  Never `value`."""
    dev = torch.cuda.current_device()
    ring = fhe_gpu.PolynomialRing(n, q, device=dev)
    kg = fhe_gpu.KeyGenerator(ring, 2024, noise_std=3.2)
    eng = fhe_gpu.EncryptionEngine(ring, t)
    sk = kg.secret_key(1)
    pk = fhe_gpu.PublicKey(ring, kg.public_key(sk, 2))
    skp = fhe_gpu.SecretKey(ring, sk)
    ek = fhe_gpu.EvaluationKey(ring, kg.eval_key(sk, 20, 3, 10), 20)
    vals = np.random.default_rng(3).integers(0, t, size=(batch, n), dtype=np.uint64)

    def chain(v, pkx, skx, ekx):
        c1 = eng.encrypt_sampled(v, pkx, 7, 100, 3.2)
        c2 = eng.encrypt_sampled(v, pkx, 7, 200, 3.2)
        return eng.decrypt(eng.relinearize(eng.multiply(c1, c2), ekx), skx)

    res = {"n": n, "q": q, "t": t, "batch": batch, "chain": "encrypt x2 -> multiply -> relinearize -> decrypt"}
    chain(vals[:2], pk, skp, ek)  # warm-up
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        chain(vals, pk, skp, ek)
        best = min(best or 1e9, time.perf_counter() - t0)
    res["host_resident"] = {"per_s": batch / best, "ms": best * 1e3}
    # device-resident: the keys and plaintext slots in HBM, outputs stay there
    dv = torch.from_numpy(vals.view(np.int64)).to(f"cuda:{dev}")
    pkd = fhe_gpu.PublicKey(ring, torch.from_numpy(pk.poly.view(np.int64)).to(f"cuda:{dev}"))
    skd = fhe_gpu.SecretKey(ring, torch.from_numpy(sk.view(np.int64)).to(f"cuda:{dev}"))
    ekd = fhe_gpu.EvaluationKey(ring, torch.from_numpy(kg.eval_key(sk, 20, 3, 10).view(np.int64)).to(f"cuda:{dev}"),
                                20)
    chain(dv[:2], pkd, skd, ekd)
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        chain(dv, pkd, skd, ekd)
        torch.cuda.synchronize()
        best = min(best or 1e9, time.perf_counter() - t0)
    res["device_resident"] = {"per_s": batch / best, "ms": best * 1e3}
    del dv
    torch.cuda.empty_cache()
    return res


def cpu_baseline_c2(n, q, seconds, threads):
    """SURVEY.md 8(d) / BASELINE config 2 (N=4096, batch 1024, fwd + inv +
    polymul, "1xMI355X vs CPU"): the oracle's restated NTTProcessor /
    PolynomialRing on the host cores, each op in turn over contiguous chunks."""
    import oracle

    t = oracle.NTT(n, q)
    B = max(threads * 4, 64)
    a = oracle.splitmix_fill(11, q, B * n).reshape(B, n)
    b = oracle.splitmix_fill(12, q, B * n).reshape(B, n)
    c = np.empty_like(a)
    out = {"n": n, "q": q, "cores": threads, "kind": "port"}
    for name, op in (("fwd", 0), ("inv", 1), ("polymul", 2)):
        done, t0 = 0, time.perf_counter()
        while True:
            x = a.copy()
            t.batch_threaded(op, x, b if op == 2 else None, c if op == 2 else None, threads=threads)
            done += B
            el = time.perf_counter() - t0
            if el >= seconds / 3:
                break
        out[name] = {"per_s": done / el, "sample": f"{done} x {name}, {threads} threads, {el:.1f}s"}
    return out


def cipher_workload(fhe_gpu, steps, warmup, dist, only=""):
    """Ciphertext-level ops: BFV-style multiply and
    relinearisation at N=16384, TFHE blind rotation at N=1024.  Reported
    beside the headline metric, never as `value`."""
    res = {}
    dev = torch.cuda.current_device()
    g = torch.Generator(device="cuda").manual_seed(77)
    if only in ("", "ct_mul", "relin"):
        n, q, B, bl, lv = 16384, P27, 8192, 4, 7
        ring = fhe_gpu.PolynomialRing(n, q, device=dev)
        eng = fhe_gpu.EncryptionEngine(ring)
        x = torch.randint(0, q, (B, 2, n), device="cuda", dtype=torch.int64, generator=g)
        y = torch.randint(0, q, (B, 2, n), device="cuda", dtype=torch.int64, generator=g)
        ct3 = torch.empty((B, 3, n), device="cuda", dtype=torch.int64)
        if only in ("", "ct_mul"):
            wall, kms = timed(dist, lambda: eng.multiply(x, y, out=ct3), steps, warmup)
            res["ct_multiply"] = {"n": n, "q": q, "batch": B, "per_s": B * steps / wall, "kernel_ms": kms,
                                  "transforms_per_unit": 7, "bytes_per_unit": 56 * n,
                                  "achieved_GBs": 56 * n * B / (kms * 1e-3) / 1e9}
            _attach(res["ct_multiply"], profile_traffic("ct_multiply", {"kernel": "ct_mul", "n": n, "batch": B, "q": q}),
                    56 * n * B, kms)
        if only in ("", "relin"):
            ek = fhe_gpu.EvaluationKey(ring, torch.randint(0, q, (lv, 2, n), device="cuda", dtype=torch.int64,
                                                           generator=g), bl)
            out = torch.empty((B, 2, n), device="cuda", dtype=torch.int64)
            eng.multiply(x, y, out=ct3)
            wall, kms = timed(dist, lambda: eng.relinearize(ct3, ek, out=out), steps, warmup)
            res["relinearize"] = {"n": n, "q": q, "batch": B, "base_log": bl, "level": lv, "per_s": B * steps / wall,
                                  "kernel_ms": kms, "transforms_per_unit": lv + 2, "bytes_per_unit": 40 * n,
                                  "achieved_GBs": 40 * n * B / (kms * 1e-3) / 1e9}
            _attach(res["relinearize"], profile_traffic("relinearize", {"kernel": "relin", "n": n, "batch": B, "q": q}),
                    40 * n * B, kms)
            del out, ek
        del x, y, ct3
    if only in ("", "c5"):
        # C5 (BASELINE.json configs[4]): TFHE external product at N=16384,
        # q = 62-bit prime, k=1, (B, L) in {(23, 1), (15, 2)}, a batch of GLWE
        # ciphertexts against one GGSW; plus the 2-limb Montgomery batch.
        n, q, B = 16384, P62, 4096
        ring = fhe_gpu.PolynomialRing(n, q, device=dev)
        glwe = torch.randint(0, q, (B, 2, n), device="cuda", dtype=torch.int64, generator=g)
        out = torch.empty_like(glwe)
        c5 = {"n": n, "q": q, "k": 1, "batch": B}
        for bl, lv in ((23, 1), (15, 2)):
            ggsw = torch.randint(0, q, (2 * lv, 2, n), device="cuda", dtype=torch.int64, generator=g)
            ep = fhe_gpu.ExternalProduct(ring, ggsw, bl, lv)
            wall, kms = timed(dist, lambda: ep(glwe, out=out), steps, warmup)
            alg = 32 * n * B  # the GLWE in and out; the GGSW rows are shared by the batch (L2)
            c5[f"extprod_B{bl}_L{lv}"] = {"per_s": B * steps / wall, "kernel_ms": kms,
                                          "transforms_per_unit": 2 * lv + 2,
                                          "algorithmic_bytes_per_launch": alg,
                                          "achieved_GBs": alg / (kms * 1e-3) / 1e9}
            _attach(c5[f"extprod_B{bl}_L{lv}"], profile_traffic(f"extprod_B{bl}_L{lv}"), alg, kms)
        del glwe, out
        cnt = 16384 * 1024
        ml = fhe_gpu.MultiLimbModularArithmetic([0xFFFFFFFF00000001, 0x3FFFFFFFFFFFFFFF])
        ma = torch.randint(0, 1 << 62, (cnt, 2), device="cuda", dtype=torch.int64, generator=g)
        mb = torch.randint(0, 1 << 62, (cnt, 2), device="cuda", dtype=torch.int64, generator=g)
        mo = torch.empty_like(ma)
        wall, kms = timed(dist, lambda: ml.montgomery_mul_batch(ma, mb, out=mo), steps, warmup)
        c5["ml_montmul_2limb"] = {"count": cnt, "per_s": cnt * steps / wall, "kernel_ms": kms,
                                  "achieved_GBs": 48 * cnt / (kms * 1e-3) / 1e9}
        res["c5"] = c5
        del ma, mb, mo
    if only in ("", "c2"):
        # C2 (configs[1]): N=4096 fwd + inv NTT and polymul, batch 1024
        n, q, B = 4096, P27, 1024
        ring = fhe_gpu.PolynomialRing(n, q, device=dev)
        a = torch.randint(0, q, (B, n), device="cuda", dtype=torch.int64, generator=g)
        b = torch.randint(0, q, (B, n), device="cuda", dtype=torch.int64, generator=g)
        o = torch.empty_like(a)
        c2 = {"n": n, "q": q, "batch": B}
        for name, fn in (("fwd", lambda: ring.forward_ntt(a, out=o)), ("inv", lambda: ring.inverse_ntt(a, out=o)),
                         ("polymul", lambda: ring.multiply(a, b, out=o))):
            wall, kms = timed(dist, fn, steps * 4, warmup)
            c2[name] = {"per_s": B * steps * 4 / wall, "kernel_ms": kms}
        res["c2"] = c2
        del a, b, o
    if only in ("", "blind_rotate"):
        # tfhe-128-fast shape (parameter_set.cpp): N=1024, k=1, B=23, L=1, n=742;
        # q = the 62-bit prime (Q_40_1 = 2^40+1 is not prime)
        n, q, bl, lv, dim, B = 1024, P62, 23, 1, 742, 8192
        ring = fhe_gpu.PolynomialRing(n, q, device=dev)
        be = fhe_gpu.BootstrapEngine(ring, bl, lv, 1)
        bsk = be.prepare_ggsw(torch.randint(0, q, (dim, 2 * lv, 2, n), device="cuda", dtype=torch.int64, generator=g))
        lwe_a = torch.randint(0, q, (B, dim), device="cuda", dtype=torch.int64, generator=g)
        lwe_b = torch.randint(0, q, (B,), device="cuda", dtype=torch.int64, generator=g)
        acc = torch.zeros((B, 2, n), device="cuda", dtype=torch.int64)
        st = max(1, steps // 4)
        wall, kms = timed(dist, lambda: be.blind_rotate(acc, lwe_a, lwe_b, bsk), st, 1)
        res["blind_rotate"] = {"n": n, "q": q, "k": 1, "base_log": bl, "level": lv, "lwe_dim": dim, "batch": B,
                               "per_s": B * st / wall, "ms_per_batch": kms,
                               "cmux_per_s": B * dim * st / wall}
        # latency of a small batch (64 ciphertexts): launch-bound, replayed as a hipGraph
        Bs = 64
        acc_s, la_s, lb_s = acc[:Bs].contiguous(), lwe_a[:Bs].contiguous(), lwe_b[:Bs].contiguous()
        wall, kms = timed(dist, lambda: be.blind_rotate(acc_s, la_s, lb_s, bsk), st * 4, 1)
        res["blind_rotate"]["batch64_ms"] = kms
        res["blind_rotate"]["batch64_per_s"] = Bs * st * 4 / wall
        del bsk, lwe_a, lwe_b, acc, acc_s, la_s, lb_s
    if only in ("", "br_presets"):
        res["blind_rotate_presets"] = br_presets(fhe_gpu, dist, g)
    torch.cuda.empty_cache()
    return res


# The reference's larger TFHE presets (parameter_set.cpp:144-184): blind
# rotation at their (N, n, B, L, q), k = 1, LWE modulus = q.
BR_PRESETS = [
    ("tfhe-128-balanced", 2048, 830, 15, 2, 1125899906826241),   # Q_50_1
    ("tfhe-256-secure", 4096, 1024, 10, 3, 1152921504606584833),  # Q_60_1
]


def br_presets(fhe_gpu, dist, g, batches=(1, 64, 8192)):
    """Latency (batch 1 and 64) and throughput (batch 8192) at the reference
    presets: the blind rotation alone (`batch*`), and the whole
    bootstrap_with_test_poly (`bootstrap`: blind rotation + sample extract +
    LWE key switch back to dimension n, fhe_bootstrap_batch,
    bootstrap_engine.cpp:684-711) with its key switch also timed alone
    (`key_switch`: key of the bootstrap's (B, L), in_dim = k N, out_dim = n,
    as generate_key_switch_key builds it, :367-420).  The reference's target is
    < 20 ms per bootstrap (.kiro/specs/fhe-accelerate/requirements.md:146)."""
    out = {}
    dev = torch.cuda.current_device()
    for name, n, dim, bl, lv, q in BR_PRESETS:
        ring = fhe_gpu.PolynomialRing(n, q, device=dev)
        be = fhe_gpu.BootstrapEngine(ring, bl, lv, 1)
        bsk = be.prepare_ggsw(torch.randint(0, q, (dim, 2 * lv, 2, n), device="cuda", dtype=torch.int64, generator=g))
        ksk_a = torch.randint(0, q, (n * lv, dim), device="cuda", dtype=torch.int64, generator=g)
        ksk_b = torch.randint(0, q, (n * lv,), device="cuda", dtype=torch.int64, generator=g)
        tp = torch.randint(0, q, (n,), device="cuda", dtype=torch.int64, generator=g)
        rec = {"n": n, "lwe_dim": dim, "base_log": bl, "level": lv, "q": q, "k": 1,
               "ks_base_log": bl, "ks_level": lv, "ks_in_dim": n, "ks_out_dim": dim}
        boot, ks = {}, {}
        for b in batches:
            la = torch.randint(0, q, (b, dim), device="cuda", dtype=torch.int64, generator=g)
            lb = torch.randint(0, q, (b,), device="cuda", dtype=torch.int64, generator=g)
            acc = torch.randint(0, q, (b, 2, n), device="cuda", dtype=torch.int64, generator=g)
            reps = 3 if b <= 64 else 1
            wall, kms = timed(dist, lambda: be.blind_rotate(acc, la, lb, bsk), reps, 1)
            rec[f"batch{b}"] = {"ms": kms, "per_s": b * reps / wall, "ms_per_bootstrap_at_batch": kms / b}
            if b == 64 and name == "tfhe-256-secure":
                # unique bytes of one launch: the bootstrapping key once, the
                # accumulators in and out, the LWE masks
                alg = dim * 2 * lv * 2 * n * 8 + 2 * b * 2 * n * 8 + b * (dim + 1) * 8
                rec[f"batch{b}"]["algorithmic_bytes_per_launch"] = alg
                _attach(rec[f"batch{b}"], profile_traffic("br_pair/tfhe-256-secure",
                                                          {"kernel": "br_pair", "n": n, "batch": b, "q": q}), alg, kms)
            wall, kms = timed(dist, lambda: be.bootstrap(la, lb, bsk, tp, ksk_a, ksk_b, bl, lv), reps, 1)
            boot[f"batch{b}"] = {"ms": kms, "per_s": b * reps / wall}
            ea = torch.randint(0, q, (b, n), device="cuda", dtype=torch.int64, generator=g)
            wall, kms = timed(dist, lambda: fhe_gpu.BootstrapEngine.key_switch(q, bl, lv, ksk_a, ksk_b, ea, lb,
                                                                              device=dev), reps, 1)
            ks[f"batch{b}"] = {"ms": kms, "per_s": b * reps / wall}
            del la, lb, acc, ea
        rec["bootstrap"], rec["key_switch"] = boot, ks
        rec["repairs"] = be.repair_count()  # two-CU pairs recomputed on one CU (0 when co-resident)
        out[name] = rec
        del bsk, ksk_a, ksk_b
        torch.cuda.empty_cache()
    return out


# The exact kernels this bench launches (the library's dispatch for these
# shapes).  A PMC traffic figure is attached only from a profile summary of
# that exact demangled symbol, measured on the library now loaded (same
# fhe_build_id(): same sources, flags and code objects); anything else gives
# traffic null.  tests/test_abi.py checks each symbol exists in the build.
def _nargs(w):
    return f"(unsigned long const*, unsigned long const*, unsigned long*, unsigned long, fhe::NttArgs<unsigned {w}>)"


BENCH_KERNELS = {
    "fwd_mul/q27": "void fhe::k_ntt_fwd_mul<14, unsigned int, true>" + _nargs("int"),
    "polymul/q27": "void fhe::k_polymul2<1294, unsigned int, true>" + _nargs("int"),
    "fwd_mul/q62": "void fhe::k_ntt_fwd_mul<1294, unsigned long, false>" + _nargs("long"),
    # the 62-bit prime takes the prime-specialised kernels (key bit 12: gk_sparse(14, 1) = 4110),
    # the compat-mode polymul also the unit-twiddle form (bit 14: gk_compat(4110) = 20494)
    "polymul/q62": "void fhe::k_polymul2<20494, unsigned long, false>" + _nargs("long"),
    "extprod_B23_L1": "void fhe::k_extprod2<4110, unsigned long>(fhe::DmArgs, fhe::NttArgs<unsigned long>)",
    "extprod_B15_L2": "void fhe::k_extprod_acc<1294>(fhe::ExtAccArgs, fhe::NttArgs<unsigned long>)",
    "ct_multiply": "void fhe::k_ct_mul2<1294, unsigned int, true>" + _nargs("int"),
    "relinearize": "void fhe::k_dmac<14, unsigned int, 2, false, 1>(fhe::DmArgs, fhe::NttArgs<unsigned int>)",
    # tfhe-256-secure blind rotation at batch 64: two CUs per ciphertext, unit
    # twiddles (gk_compat(12) = 16396), its three digit levels in lockstep
    "br_pair/tfhe-256-secure": "void fhe::k_br_pair<16396, unsigned long, 3>(fhe::BrArgs, fhe::NttArgs<unsigned long>, "
                               "fhe::BrPairX, unsigned int)",
}


def _build_id():
    try:
        import fhe_gpu

        return fhe_gpu.build_id()
    except Exception:  # pragma: no cover
        return None


def matched_summary(key, workload=None):
    """(summary dict, path) of the newest profiles/*/summary.json of kernel
    BENCH_KERNELS[key] stamped with the loaded library's build id (and, when
    given, the same workload), or None.  Written by tools/gpu_evidence.sh +
    tools/summarize_profile.py."""
    import glob

    sym, bid = BENCH_KERNELS[key], _build_id()
    if bid is None:
        return None
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "*", "summary.json")):
        try:
            s = json.load(open(f))
        except Exception:
            continue
        if s.get("build_id") != bid or s.get("kernel_name") != sym or "hbm_traffic_bytes_per_launch" not in s:
            continue
        if workload is not None:
            w = dict(s.get("workload", {}))
            w.setdefault("mode", "compat")
            if any(w.get(k) != v for k, v in workload.items()):
                continue
        key_ = (s.get("generated", ""), f)
        if best is None or key_ > best[0]:
            best = (key_, s, os.path.relpath(f, ROOT))
    return best[1:] if best else None


def profile_traffic(key, workload=None):
    """(HBM bytes per launch, summary path, profiled kernel ms, summary) of
    matched_summary(), or None."""
    m = matched_summary(key, workload)
    if m is None:
        return None
    s, path = m
    kt = s.get("kernel_trace_full_batch", {})
    return s["hbm_traffic_bytes_per_launch"], path, kt.get("avg_ns", 0) / 1e6 or None, s


def pmc_traffic(kernel, n, batch, q, mode="compat"):
    """profile_traffic() of the headline kernels (fwd_mul / polymul)."""
    if n != 16384 or kernel not in ("fwd_mul", "polymul") or q not in (P27, P62):
        return None
    key = f"{kernel}/{'q27' if q == P27 else 'q62'}"
    return profile_traffic(key, {"kernel": kernel, "n": n, "batch": batch, "q": q, "mode": mode})


def _attach(d, tr, alg, kernel_ms=None):
    """Traffic and second-roofline fields of a roofline / side-metric record
    (traffic null when unmatched).  From the matched profile summary: the
    HBM fraction priced on the profile's own kernel time beside the
    event-timed one (`frac_profile`), and the VALU-issue roofline
    (tools/valu_roofline.py) priced on both times."""
    if tr:
        d["traffic"], d["traffic_source"], d["profile_kernel_ms"] = tr[:3]
        d["traffic_over_algorithmic"] = tr[0] / alg
        s = tr[3] if len(tr) > 3 else None
        if s is not None:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import valu_roofline as vr

            fp = vr.hbm_frac_profile(s, alg, HBM_PEAK_GBS)
            if fp is not None:
                d["frac_profile"] = fp
            v = vr.valu_roofline(s, vr.load_rates(), kernel_ms=kernel_ms)
            d["valu_roofline"] = v if v is not None else "no VALU counters / static mix in the matched profile"
    else:
        d["traffic"] = None
        d["traffic_source"] = "no profile of this exact kernel on this build (fhe_build_id)"


def host_info():
    """Host CPU facts for the cpu_baseline record."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff}


def cpu_calibration(n, q):
    """BASELINE.md section 2's calibration of the port against the compiled
    reference: tools/calibrate_cpu.py times oracle/ref_cpu.c in the survey
    container class at SURVEY.md section 6's configs (one thread) and divides
    by the reference timings recorded there (profiles/r6_cpu_calibration.json).
    ratio > 1: the port is slower than the reference by that factor, so the
    reference's own throughput would be cpu_baseline.value x ratio."""
    path = os.path.join(ROOT, "profiles", "r6_cpu_calibration.json")
    try:
        cal = json.load(open(path))
    except (OSError, ValueError):
        return {"status": "uncalibrated: profiles/r6_cpu_calibration.json missing"}
    rows = {(r["op"], r["q"], r["n"]): r for r in cal["rows"]}
    out = {"source": os.path.relpath(path, ROOT), "host": cal.get("host"), "generated": cal.get("generated"),
           "meaning": "port time / compiled-reference time per call, one thread, same container class "
                      "(reference: SURVEY.md section 6 [verified] timings; not buildable on the GPU box)",
           "ratio_median_all_configs": cal["ratio_median"], "ratio_range": [cal["ratio_min"], cal["ratio_max"]]}
    for op in ("forward_ntt", "multiply"):
        r = rows.get((op, q, n))
        if r:
            out[f"{op}_N{n}"] = {"port_us": r["port_us"], "reference_us": r["reference_us"], "ratio": r["ratio"]}
    fw = rows.get(("forward_ntt", q, n))
    if fw:
        out["within_10pct_at_this_config"] = 0.9 <= fw["ratio"] <= 1.1
    # a later rerun of the same script in the same container (idle) ran 1.5x
    # slower across every config: the container's host speed varies, so the
    # ratio is quoted with both runs
    try:
        re_ = json.load(open(os.path.join(ROOT, "profiles", "r6_cpu_calibration_rerun.json")))
        out["rerun"] = {"generated": re_.get("generated"), "ratio_median_all_configs": re_["ratio_median"],
                        "ratio_range": [re_["ratio_min"], re_["ratio_max"]]}
    except (OSError, ValueError, KeyError):
        pass
    return out


def cpu_baseline(n, q, seconds, threads=None):
    """The oracle (C restatement of the reference NTTProcessor + pointwise,
    same % -based op sequence) on the host cores, bounded sample.  Threads:
    every core this process may run on, capped by OMP_NUM_THREADS when the
    host sets one (the GPU box sets it to the job's CPU share: its affinity
    mask lists the whole machine, shared with other jobs)."""
    import oracle

    info = host_info()
    if threads is None:
        threads = info["affinity_cpus"]
        omp = os.environ.get("OMP_NUM_THREADS", "")
        if omp.isdigit() and int(omp) > 0:
            threads = min(threads, int(omp))
    t = oracle.NTT(n, q)
    chunk = threads * 2
    a = oracle.splitmix_fill(1, q, chunk * n).reshape(chunk, n)
    w = oracle.splitmix_fill(2, q, chunk * n).reshape(chunk, n)
    out = np.empty_like(a)
    done, t0 = 0, time.perf_counter()
    while True:
        t.batch_threaded(3, a.copy(), w, out, threads=threads)
        done += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    if threads == 1:
        basis = "one thread (the reference's sequential forward_ntt_batch, ntt_processor.cpp:394-408)"
    elif threads < info["affinity_cpus"]:
        basis = ("the job's CPU share on this host (OMP_NUM_THREADS; the GPU box's affinity mask lists the whole "
                 "shared machine, nproc above)")
    else:
        basis = "every CPU this process may run on"
    return {"value": done / el, "unit": "NTTs/s", "cores": threads, "cores_basis": basis, "kind": "port",
            "calibration": cpu_calibration(n, q),
            **info,
            "sample": f"{done} x (forward NTT + pointwise modmul), N={n}, q={q}, {threads} threads, {el:.1f}s; "
                      f"oracle/ref_cpu.c restatement of NTTProcessor::forward_ntt + pointwise_multiply"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    dist, rank, world, local = dist_setup(args)
    import fhe_gpu

    n, B, K, W = args.n, args.batch, args.steps, args.warmup
    extra = {}
    if args.only_host:
        if rank == 0:
            print(json.dumps({"host_resident": host_resident(fhe_gpu, n, args.q)}), flush=True)
        return
    if args.only in ("ct_mul", "relin", "blind_rotate", "c5", "c2", "br_presets"):  # profiling runs of the side metrics
        c = cipher_workload(fhe_gpu, K, W, dist, args.only)
        if rank == 0:
            print(json.dumps({"cipher": c}), flush=True)
        return
    if args.only == "engine":
        if rank == 0:
            print(json.dumps({"engine_chain": engine_chain(fhe_gpu)}), flush=True)
        return
    r = gpu_workload(fhe_gpu, n, args.q, B, K, W, dist, args.only, check=not args.no_check, mode=args.mode)
    if args.q62 and not args.only:
        r62 = gpu_workload(fhe_gpu, n, P62, B, max(3, K // 4), 1, dist)
        ach62 = 24 * n * B / (r62["fwd_mul"][1] * 1e-3) / 1e9
        achp62 = 24 * n * B / (r62["polymul"][1] * 1e-3) / 1e9
        extra["q62"] = {
            "q": P62,
            "ntt_fwd_mul_per_s": world * B * max(3, K // 4) / r62["fwd_mul"][0],
            "polymuls_per_s": world * B * max(3, K // 4) / r62["polymul"][0],
            "fwd_mul_kernel_ms": r62["fwd_mul"][1], "polymul_kernel_ms": r62["polymul"][1],
            "parity_ok": r62["parity_ok"],
            "roofline": {"bound": "hbm", "achieved": ach62, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach62 / HBM_PEAK_GBS, "kernel": "fwd_mul"},
            "polymul_roofline": {"achieved": achp62, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": achp62 / HBM_PEAK_GBS},
        }
        for key, rl in (("fwd_mul", extra["q62"]["roofline"]), ("polymul", extra["q62"]["polymul_roofline"])):
            _attach(rl, pmc_traffic(key, n, B, P62), 24 * n * B, r62[key][1])
    if not args.only:
        nk = max(3, K // 4)
        extra["negacyclic"] = negacyclic_workload(fhe_gpu, n, args.q, B, nk, 1, dist)
    if args.cipher and not args.only:
        extra["cipher"] = cipher_workload(fhe_gpu, max(3, K // 4), 1, dist)
    if rank == 0 and not args.only and not args.no_host:
        extra["host_resident"] = host_resident(fhe_gpu, n, args.q)
        extra["engine_chain"] = engine_chain(fhe_gpu)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    key = args.only or "fwd_mul"
    wall, kms = r[key]
    units = world * B * K
    value = units / wall
    bytes_per_unit = {"fwd_mul": 24, "polymul": 24, "fwd": 16, "inv": 16}[key] * n
    achieved = bytes_per_unit * B / (kms * 1e-3) / 1e9
    line = {
        "metric": "NTTs/s at degree 16384 (batched, forward NTT + pointwise modmul)",
        "value": value,
        "unit": "NTTs/s",
        "n_gpus": world,
        "ranks_seen": dist.get_world_size() if dist is not None else 1,
        "devices_used": len({(r % max(1, torch.cuda.device_count())) for r in range(world)}),
        "steps": K,
        "warmup": W,
        "ms_per_step": wall / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64 (32-bit Shoup/Montgomery lanes for q<2^30)" if args.q < (1 << 30) else "u64",
        "data": "synthetic uniform residues mod q, generated on device",
        "config": {"workload": f"C3: N={n} forward NTT + modmul, batch {B} per GPU, q={args.q}",
                   "n": n, "batch_per_gpu": B, "global_batch": world * B, "q": args.q,
                   "parallelism": f"batch-sharded x{world}, no data-path collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "traffic_unit": "bytes per launch (rocprofv3 PMC, gfx950-corrected)",
                     "kernel": key, "kernel_ms": kms, "algorithmic_bytes_per_launch": bytes_per_unit * B},
        "parity_ok": r["parity_ok"],
        "parity_rows": r.get("parity_rows"),
    }
    _attach(line["roofline"], pmc_traffic(key, n, B, args.q), bytes_per_unit * B, kms)
    line["build_id"] = _build_id()
    if "gather" in r:
        line["gather"] = r["gather"]
    if "polymul" in r:
        pw, pk = r["polymul"]
        line["polymuls_per_s"] = world * B * K / pw
        line["polymul_roofline"] = {"achieved": 24 * n * B / (pk * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "kernel_ms": pk, "frac": 24 * n * B / (pk * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                    "bound": "valu",
                                    "bound_note": "3 transforms per 24N bytes: the VALU-issue roofline is "
                                                  "valu_roofline (DESIGN.md section 6)"}
        _attach(line["polymul_roofline"], pmc_traffic("polymul", n, B, args.q), 24 * n * B, pk)
    line.update(extra)
    if not args.no_cpu and world == 1 and not args.only:
        line["cpu_baseline"] = cpu_baseline(n, args.q, args.cpu_seconds)
        # also one thread (the reference's sequential forward_ntt_batch)
        line["cpu_baseline_1thread"] = cpu_baseline(n, args.q, min(4.0, args.cpu_seconds), threads=1)
        line["speedup_vs_cpu"] = value / line["cpu_baseline"]["value"]
        # BASELINE config 2 beside its GPU figures (cipher.c2)
        c2cpu = cpu_baseline_c2(4096, args.q, min(9.0, args.cpu_seconds), line["cpu_baseline"]["cores"])
        line["cpu_baseline_c2"] = c2cpu
        g2 = line.get("cipher", {}).get("c2")
        if g2:
            line["c2_speedup_vs_cpu"] = {k: g2[k]["per_s"] / c2cpu[k]["per_s"] for k in ("fwd", "inv", "polymul")}
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
