"""CPU checks of the oracle's ciphertext-level restatements (oracle/ref_cpu.c:
oracle_ct_multiply, oracle_relinearize, oracle_cmux, oracle_blind_rotate,
oracle_key_switch) against a second, independently written pure-Python
restatement of the reference code (encryption.cpp:737-980,
bootstrap_engine.cpp:122-145, 520-674) built on ``oracle.pyref``'s big-integer
transform, plus the committed golden vectors.  No GPU needed.
"""
import json
import os

import numpy as np
import pytest

import oracle
from oracle import pyref

P27 = 132120577
P62 = 4611686018326724609
M64 = (1 << 64) - 1


def rnd(seed, q, *shape):
    return oracle.splitmix_fill(seed, q, int(np.prod(shape))).reshape(shape)


def I(a):
    return [int(v) for v in np.asarray(a).ravel()]


# ---- pure-Python restatement (test-local; exact ints, u64 wrap where the reference wraps)
def mod_add(q, a, b):  # modular_arithmetic.cpp:122-138
    a %= q
    b %= q
    s = (a + b) & M64
    return s - q if (s < a or s >= q) else s


def mod_sub(q, a, b):  # :140-153
    a %= q
    b %= q
    return a - b if a >= b else q - (b - a)


def pw(q, a, b):
    return [(x * y) % q for x, y in zip(a, b)]


def py_ct_multiply(ct1, ct2, q, is_ntt=False):
    x0, x1, y0, y1 = (I(v) for v in (ct1[0], ct1[1], ct2[0], ct2[1]))
    if not is_ntt:
        x0, x1, y0, y1 = (pyref.forward(v, q) for v in (x0, x1, y0, y1))
    c0 = pw(q, x0, y0)
    c1 = [mod_add(q, a, b) for a, b in zip(pw(q, x0, y1), pw(q, x1, y0))]
    c2 = pw(q, x1, y1)
    if not is_ntt:
        c0, c1, c2 = (pyref.inverse(v, q) for v in (c0, c1, c2))
    return [c0, c1, c2]


def py_relinearize(ct3, rlk, q, bl, lv):  # encryption.cpp:904-980
    r0, r1 = I(ct3[0]), I(ct3[1])
    for l in range(lv):
        d = [(c >> (l * bl)) & ((1 << bl) - 1) for c in I(ct3[2])]
        dn = pyref.forward(d, q)
        pa = pyref.inverse(pw(q, dn, pyref.forward(I(rlk[l][0]), q)), q)
        pb = pyref.inverse(pw(q, dn, pyref.forward(I(rlk[l][1]), q)), q)
        r0 = [mod_add(q, a, b) for a, b in zip(r0, pb)]
        r1 = [mod_add(q, a, b) for a, b in zip(r1, pa)]
    return [r0, r1]


def py_decompose(poly, q, bl, lv):  # bootstrap_engine.cpp:152-185
    base = 1 << bl
    out = []
    for l in range(lv):
        sh = (lv - 1 - l) * bl
        row = []
        for c in poly:
            d = (c >> sh) & (base - 1)
            row.append((q - (base - d)) % q if d > base // 2 else d)
        out.append(row)
    return out


def py_extprod(glwe, ggsw, q, bl, lv, k=1):  # :431-518
    n = len(glwe[0])
    res = [[0] * n for _ in range(k + 1)]
    row = 0
    for i in range(k + 1):
        for d in py_decompose(glwe[i], q, bl, lv):
            dn = pyref.forward(d, q)
            for j in range(k + 1):
                p = pyref.inverse(pw(q, dn, pyref.forward(I(ggsw[row][j]), q)), q)
                res[j] = [mod_add(q, a, b) for a, b in zip(res[j], p)]
            row += 1
    return res


def py_rotate(poly, rot, q):  # :122-145
    n = len(poly)
    two_n = 2 * n
    r = int(np.int32(rot)) % two_n  # same residue as C's ((rot % 2N) + 2N) % 2N
    out = [0] * n
    for i, c in enumerate(poly):
        ni = (i + r) % two_n
        if ni < n:
            out[ni] = c
        else:
            out[ni - n] = ((q - c) & M64) % q
    return out


def py_cmux(ggsw, ct0, ct1, q, bl, lv, k=1):  # :520-540
    diff = [[mod_sub(q, a, b) for a, b in zip(I(ct1[i]), I(ct0[i]))] for i in range(k + 1)]
    p = py_extprod(diff, ggsw, q, bl, lv, k)
    return [[mod_add(q, a, b) for a, b in zip(p[i], I(ct0[i]))] for i in range(k + 1)]


def c_int32_trunc(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def py_blind_rotate(acc, lwe_a, lwe_b, bsk, q, bl, lv, k=1):  # :547-577
    n = len(acc[0])
    acc = [I(p) for p in acc]
    b_rot = -c_int32_trunc((((lwe_b * 2 * n) & M64) + q // 2) // q)
    acc = [py_rotate(p, b_rot, q) for p in acc]
    for i, a in enumerate(I(lwe_a)):
        a_rot = c_int32_trunc((((a * 2 * n) & M64) + q // 2) // q)
        if a_rot == 0:
            continue
        rot = [py_rotate(p, a_rot, q) for p in acc]
        acc = py_cmux(bsk[i], acc, rot, q, bl, lv, k)
    return acc


def py_key_switch(q, bl, lv, ksk_a, ksk_b, lwe_a, lwe_b):  # :626-674
    out_dim = ksk_a.shape[1]
    ra = [0] * out_dim
    rb = lwe_b
    idx = 0
    for c in I(lwe_a):
        for l in range(lv):
            d = (c >> ((lv - 1 - l) * bl)) & ((1 << bl) - 1)
            if d == 0:
                idx += 1
                continue
            ka = I(ksk_a[idx])
            ra = [(x + q - ((d * y) & M64) % q) % q for x, y in zip(ra, ka)]
            rb = (((rb + q - ((d * int(ksk_b[idx])) & M64) % q) & M64)) % q
            idx += 1
    return ra, rb


# ---- tests
@pytest.mark.parametrize("n,q", [(8, 17), (16, 97), (64, 257), (128, P62)])
def test_ct_multiply_oracle_vs_python(n, q):
    t = oracle.NTT(n, q)
    x, y = rnd(1, q, 2, n), rnd(2, q, 2, n)
    assert [I(r) for r in t.ct_multiply(x, y)] == py_ct_multiply(x, y, q)
    assert [I(r) for r in t.ct_multiply(x, y, True)] == py_ct_multiply(x, y, q, True)


@pytest.mark.parametrize("n,q,bl,lv", [(16, 97, 2, 4), (64, 257, 3, 3), (32, P62, 16, 4), (64, 7681, 63, 1)])
def test_relinearize_oracle_vs_python(n, q, bl, lv):
    t = oracle.NTT(n, q)
    ct3 = rnd(3, q, 3, n)
    ct3[2, 0] = M64
    rlk = rnd(4, q, lv, 2, n)
    assert [I(r) for r in t.relinearize(bl, lv, ct3, rlk)] == py_relinearize(ct3, rlk, q, bl, lv)


@pytest.mark.parametrize("n,q,bl,lv", [(16, 97, 2, 3), (32, P62, 23, 1)])
def test_cmux_oracle_vs_python(n, q, bl, lv):
    t = oracle.NTT(n, q)
    ggsw = rnd(5, q, 2 * lv, 2, n)
    ct0, ct1 = rnd(6, q, 2, n), rnd(7, q, 2, n)
    assert [I(r) for r in t.cmux(1, bl, lv, ggsw, ct0, ct1)] == py_cmux(ggsw, ct0, ct1, q, bl, lv)


def test_rotate_oracle_vs_python():
    q, n = 97, 16
    p = rnd(8, q, n)
    p[0] = M64
    for rot in (0, 1, -1, 15, 16, 17, 31, 32, -33, 1000, -(2**31)):
        assert I(oracle.rotate(q, p, rot)) == py_rotate(I(p), rot, q), rot


@pytest.mark.parametrize("n,q,bl,lv,dim", [(16, 97, 2, 3, 6), (32, 193, 3, 2, 5)])
def test_blind_rotate_oracle_vs_python(n, q, bl, lv, dim):
    t = oracle.NTT(n, q)
    bsk = rnd(9, q, dim, 2 * lv, 2, n)
    lwe_a = rnd(10, q, dim)
    lwe_a[0] = 0
    lwe_a[1] = q - 1
    acc = np.zeros((2, n), np.uint64)
    acc[1] = rnd(11, q, n)
    got = t.blind_rotate(1, bl, lv, lwe_a, 37, q, bsk, acc)
    assert [I(r) for r in got] == py_blind_rotate(acc, lwe_a, 37, bsk, q, bl, lv)


@pytest.mark.parametrize("q,bl,lv,b", [(P27, 4, 3, 5), (P62, 7, 4, M64 - 2), (97, 2, 4, 0)])
def test_key_switch_oracle_vs_python(q, bl, lv, b):
    in_dim, out_dim = 12, 9
    ka, kb = rnd(12, q, in_dim * lv, out_dim), rnd(13, q, in_dim * lv)
    la = rnd(14, q, in_dim)
    oa, ob = oracle.key_switch(q, bl, lv, ka, kb, la, b)
    ea, eb = py_key_switch(q, bl, lv, ka, kb, la, b)
    assert I(oa) == ea and ob == eb
    # no non-zero digit: the body is returned unreduced
    oa, ob = oracle.key_switch(q, bl, lv, ka, kb, np.zeros(in_dim, np.uint64), M64)
    assert I(oa) == [0] * out_dim and ob == M64


def test_cipher_golden(golden_dir):
    path = os.path.join(golden_dir, "cipher.json")
    with open(path) as f:
        cases = json.load(f)
    for c in cases:
        n, q = c["n"], c["q"]
        t = oracle.NTT(n, q)
        if c["op"] == "ct_multiply":
            x = np.array(c["ct1"], np.uint64).reshape(2, n)
            y = np.array(c["ct2"], np.uint64).reshape(2, n)
            assert I(t.ct_multiply(x, y)) == c["out"]
        elif c["op"] == "relinearize":
            ct3 = np.array(c["ct3"], np.uint64).reshape(3, n)
            rlk = np.array(c["rlk"], np.uint64).reshape(c["level"], 2, n)
            assert I(t.relinearize(c["base_log"], c["level"], ct3, rlk)) == c["out"]
        elif c["op"] == "blind_rotate":
            lv, dim = c["level"], c["dim"]
            bsk = np.array(c["bsk"], np.uint64).reshape(dim, 2 * lv, 2, n)
            acc = np.array(c["acc"], np.uint64).reshape(2, n)
            got = t.blind_rotate(1, c["base_log"], lv, np.array(c["lwe_a"], np.uint64), c["lwe_b"], q, bsk, acc)
            assert I(got) == c["out"]


# ---- EncryptionEngine encrypt / decrypt / add_plain, BootstrapEngine::bootstrap
def py_encode(q, t, values):  # encryption.cpp:107-131 (u64 product wraps)
    delta = q // (t or 4)
    return [((v * delta) & M64) % q for v in I(values)]


def py_encrypt(q, t, pk, values, u, e1, e2):  # :171-205
    un = pyref.forward(I(u), q)
    c0 = pyref.inverse(pw(q, pyref.forward(I(pk[1]), q), un), q)  # pk = (a, b)
    c0 = [mod_add(q, a, b) for a, b in zip(c0, I(e1))]
    c0 = [mod_add(q, a, b) for a, b in zip(c0, py_encode(q, t, values))]
    c1 = pyref.inverse(pw(q, pyref.forward(I(pk[0]), q), un), q)
    c1 = [mod_add(q, a, b) for a, b in zip(c1, I(e2))]
    return [c0, c1]


def py_decrypt(q, t, sk, ct, is_ntt=False):  # :234-300, :150-163, :364-400
    c1 = I(ct[1]) if is_ntt else pyref.forward(I(ct[1]), q)
    s = pyref.forward(I(sk), q)
    c0 = pyref.inverse(I(ct[0]), q) if is_ntt else I(ct[0])
    res = [mod_sub(q, a, b) for a, b in zip(c0, pyref.inverse(pw(q, c1, s), q))]
    if len(ct) == 3:
        c2 = I(ct[2]) if is_ntt else pyref.forward(I(ct[2]), q)
        res = [mod_sub(q, a, b) for a, b in zip(res, pyref.inverse(pw(q, c2, pw(q, s, s)), q))]
    tt = t or 4
    delta = q // tt
    vals, mx = [], 0
    for c in res:
        rounded = (c * tt + q // 2) // q
        vals.append(rounded % tt)
        noise = abs(c - (rounded * delta) % q)
        if noise > q // 2:
            noise = q - noise
        mx = max(mx, noise)
    return vals, res, mx


def py_add_plain(q, t, ct, values, is_ntt=False):  # :638-665
    m = py_encode(q, t, values)
    if is_ntt:
        m = pyref.forward(m, q)
    return [[mod_add(q, a, b) for a, b in zip(I(ct[0]), m)], I(ct[1])]


@pytest.mark.parametrize("n,q,t", [(16, 97, 4), (64, 7681, 16), (32, P62, 0), (128, P27, 1 << 40)])
def test_encrypt_decrypt_oracle_vs_python(n, q, t):
    o = oracle.NTT(n, q)
    pk, u, e1, e2, sk = rnd(21, q, 2, n), rnd(22, 3, n), rnd(23, q, n), rnd(24, q, n), rnd(25, 3, n)
    vals = rnd(26, t or 4, n)
    vals[0] = M64  # the u64 product wraps before % q
    ct = o.encrypt(t, pk, vals, u, e1, e2)
    assert [I(r) for r in ct] == py_encrypt(q, t, pk, vals, u, e1, e2)
    ct3 = rnd(27, q, 3, n)
    for c, is_ntt in ((ct, False), (ct, True), (ct3, False), (ct3, True)):
        v, ph, mx = o.decrypt(t, sk, c, is_ntt)
        ev, eph, emx = py_decrypt(q, t, sk, c, is_ntt)
        assert I(v) == ev and I(ph) == eph and mx == emx
    for is_ntt in (False, True):
        assert [I(r) for r in o.add_plain(t, ct, vals, is_ntt)] == py_add_plain(q, t, ct, vals, is_ntt)


@pytest.mark.parametrize("n,q,t", [(64, 7681, 16), (1024, P27, 4), (256, P62, 1 << 20)])
def test_noise_free_encryption_decrypts(n, q, t):
    """Algebraic pin of the restated encrypt/decrypt: the reference's product
    inv(fwd(a) . fwd(b)) is the pointwise algebra carried back through one
    linear bijection, hence commutative and associative.  With pk = (a, a*s)
    and e1 = e2 = 0, decrypt(encrypt(m)) = c0 - c1 s = (a s) u + m delta -
    (a u) s = m delta exactly: the values come back and the max noise is 0."""
    o = oracle.NTT(n, q)
    a, s, u = rnd(31, q, n), rnd(32, 3, n), rnd(33, 3, n)
    m = rnd(34, t, n)
    pk = np.stack([a, o.polymul(a, s)])
    z = np.zeros(n, np.uint64)
    ct = o.encrypt(t, pk, m, u, z, z)
    v, ph, mx = o.decrypt(t, s, ct)
    assert (v == m).all() and mx == 0
    assert (ph == oracle.encode(q, t, m)).all()


@pytest.mark.parametrize("n,q,bl,lv,dim", [(16, 97, 2, 3, 5), (32, 193, 3, 2, 4)])
def test_bootstrap_oracle_vs_python(n, q, bl, lv, dim):
    o = oracle.NTT(n, q)
    bsk = rnd(41, q, dim, 2 * lv, 2, n)
    lwe_a, test_poly = rnd(42, q, dim), rnd(43, q, n)
    ks_bl, ks_lv, out_dim = 3, 2, 7
    ksk_a, ksk_b = rnd(44, q, n * ks_lv, out_dim), rnd(45, q, n * ks_lv)
    oa, ob = o.bootstrap(1, bl, lv, lwe_a, 29, q, bsk, test_poly, ks_bl, ks_lv, ksk_a, ksk_b)
    acc = np.zeros((2, n), np.uint64)
    acc[1] = test_poly
    acc = np.array(py_blind_rotate(acc, lwe_a, 29, bsk, q, bl, lv), dtype=np.uint64)
    ea = [int(acc[0][0])] + [(q - int(acc[0][n - j])) % q for j in range(1, n)]
    ra, rb = py_key_switch(q, ks_bl, ks_lv, ksk_a, ksk_b, np.array(ea, np.uint64), int(acc[1][0]))
    assert I(oa) == ra and ob == rb
