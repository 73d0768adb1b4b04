#!/usr/bin/env python3
"""Lab diagnostic for the multi-CU blind rotation: one CMux step (lwe_dim 1,
no initial rotation), the result decomposed over the GGSW rows' individual
contributions (oracle external products with one row kept): prints which
weights w_j in {0, 1, 2} give got = acc + sum_j w_j C_j.

usage: br_multi_diag.py N Q BASE_LOG LEVEL [mode]"""
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "node-fhe-accelerate_amd"))
import numpy as np  # noqa: E402

import fhe_gpu as fg  # noqa: E402
import oracle  # noqa: E402

n, q, bl, lv = (int(x) for x in sys.argv[1:5])
k, b, dim = 1, 1, 1
r = fg.PolynomialRing(n, q)
be = fg.BootstrapEngine(r, bl, lv, k)
bsk = oracle.splitmix_fill(71, q, dim * 2 * lv * 2 * n).reshape(dim, 2 * lv, 2, n)
bsk_ntt = be.prepare_ggsw(bsk)
lwe_a = np.array([[3 * (q // (4 * n)) if q > 2**40 else q // 3]], dtype=np.uint64)
lwe_b = np.zeros(1, dtype=np.uint64)
acc0 = oracle.splitmix_fill(74, q, b * 2 * n).reshape(b, 2, n)
t = oracle.NTT(n, q)
res = {}
for tag, pair, multi, pmax in (("multi", "1", "1", "4096"), ("pair", "1", "0", "4096"), ("step", "1", "1", "0")):
    os.environ["FHE_BR_PAIR"], os.environ["FHE_BR_MULTI"], os.environ["FHE_BR_PERSIST_MAX"] = pair, multi, pmax
    acc = acc0.copy()
    be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
    res[tag] = acc[0]
exp = t.blind_rotate(k, bl, lv, lwe_a[0], int(lwe_b[0]), q, bsk, acc0[0])
print({tg: bool((v == exp).all()) for tg, v in res.items()}, flush=True)
rot = int((int(lwe_a[0, 0]) * 2 * n + q // 2) // q)
D = np.stack([oracle.poly_sub(q, oracle.rotate(q, acc0[0][c], rot), acc0[0][c]) for c in range(2)])
C = []
for j in range(2 * lv):
    g = np.zeros_like(bsk[0])
    g[j] = bsk[0][j]
    C.append(t.external_product(k, bl, lv, D, g))
for tag, got in res.items():
    hits = []
    for w in itertools.product(range(3), repeat=2 * lv):
        s = acc0[0].copy()
        for j, wj in enumerate(w):
            for _ in range(wj):
                s = np.stack([oracle.poly_add(q, s[c], C[j][c]) for c in range(2)])
        for c in range(2):
            if (s[c] == got[c]).all():
                hits.append((c, w))
    print(tag, "component/weights matching:", hits, flush=True)
