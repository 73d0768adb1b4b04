#!/usr/bin/env python3
"""Lab diagnostic: repeat one blind-rotation configuration through its three
dispatch paths (two-CU k_br_pair, one-CU k_br_persist, per-step launches) and
compare every row with the oracle, reporting which path and row differ and
the repair count (k_br_pair's timeout path) of each call.

usage: br_diag.py N Q BASE_LOG LEVEL K [trials] [mode]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "node-fhe-accelerate_amd"))
import numpy as np  # noqa: E402

import fhe_gpu as fg  # noqa: E402
import oracle  # noqa: E402

n, q, bl, lv, k = (int(x) for x in sys.argv[1:6])
trials = int(sys.argv[6]) if len(sys.argv) > 6 else 8
mode = sys.argv[7] if len(sys.argv) > 7 else "compat"


def rnd(seed, *shape):
    return oracle.splitmix_fill(seed, q, int(np.prod(shape))).reshape(shape)


b, dim = 5, 24
r = fg.PolynomialRing(n, q, mode=mode)
be = fg.BootstrapEngine(r, bl, lv, k)
bsk = rnd(71 + n, dim, (k + 1) * lv, k + 1, n)
bsk_ntt = be.prepare_ggsw(bsk)
lwe_a = rnd(72, b, dim)
lwe_a[0, :3] = [0, q - 1, 1]
lwe_a[1, :] = 0
lwe_b = rnd(73, b)
acc0 = rnd(74, b, k + 1, n)
acc0[2, 0, :3] = [2**64 - 1, q, q + 1]
os.environ["FHE_BR_PAIR"], os.environ["FHE_BR_PERSIST_MAX"] = "1", "0"  # per-step launches
exp = acc0.copy()
be.blind_rotate(exp, lwe_a, lwe_b, bsk_ntt)
if mode == "compat":
    t = oracle.NTT(n, q)
    assert all((exp[i] == t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])).all() for i in range(b))
bad = 0
for trial in range(trials):
    for pmax, pair, multi in (("4096", "1", "1"), ("4096", "1", "0"), ("4096", "0", "1")):
        os.environ["FHE_BR_PERSIST_MAX"], os.environ["FHE_BR_PAIR"], os.environ["FHE_BR_MULTI"] = pmax, pair, multi
        before = be.repair_count()
        acc = acc0.copy()
        be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
        rows = [i for i in range(b) if not (acc[i] == exp[i]).all()]
        rep = be.repair_count() - before
        if rows or rep:
            bad += bool(rows)
            diff = {i: [int((acc[i][c] != exp[i][c]).sum()) for c in range(k + 1)] for i in rows}
            print(f"trial {trial} pmax={pmax} pair={pair} multi={multi}: rows differing {diff} repairs {rep}", flush=True)
print(f"N={n} q={q} ({bl},{lv}) k={k}: {bad} bad calls of {3 * trials}", flush=True)
