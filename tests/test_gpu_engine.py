"""GPU parity of the EncryptionEngine / BootstrapEngine entry points around
the transform: encrypt, decrypt (+ decode + noise),
add_plain and the composed bootstrap -- HIP kernels through the C-ABI vs the
CPU oracle's restatement (oracle/ref_cpu.c: oracle_encrypt, oracle_decrypt,
oracle_add_plain, oracle_bootstrap), bit-exact; plus the algebraic identity
decrypt(encrypt(m)) = m at full degree.

Run on an MI355X with ``pytest -m gpu``.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

P27 = 132120577
P62 = 4611686018326724609
M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def fg():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import fhe_gpu

    return fhe_gpu


def rnd(seed, q, *shape):
    return oracle.splitmix_fill(seed, q, int(np.prod(shape))).reshape(shape)


Q62 = 4611686018429485057     # 2^62 + 2^21 + 1
Q63 = 9223370937344327681     # just below 2^63
QG = 18446744069414584321     # 2^64 - 2^32 + 1
SIZES = [(16, 97), (256, 7681), (1024, P27), (1024, P62), (4096, P27), (8192, P62), (16384, P27), (16384, P62),
         # composed paths (engine_composed.hip): q >= 2^62 and N > 16384
         (1024, Q62), (1024, Q63), (4096, QG), (32768, P27), (32768, P62), (65536, P27)]


@pytest.mark.parametrize("n,q", SIZES)
@pytest.mark.parametrize("t", [0, 16, 1 << 40])
def test_encrypt_vs_oracle(fg, n, q, t):
    b = 3 if n >= 8192 else 5
    r = fg.PolynomialRing(n, q)
    o = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r, t)
    pk = rnd(n + 1, q, 2, n)
    u, e1, e2 = rnd(n + 2, 3, b, n), rnd(n + 3, q, b, n), rnd(n + 4, q, b, n)
    vals = rnd(n + 5, t or 4, b, n)
    vals[0, 0] = M64          # the u64 product v * delta wraps before % q
    e1[1, :3] = [M64, q, q + 1]  # raw words behave as x mod q
    ct = eng.encrypt(vals, fg.PublicKey(r, pk), u, e1, e2)
    assert ct.shape == (b, 2, n)
    for i in range(b):
        assert (ct[i] == o.encrypt(t, pk, vals[i], u[i], e1[i], e2[i])).all(), i


@pytest.mark.parametrize("n,q", SIZES)
@pytest.mark.parametrize("comps", [2, 3])
def test_decrypt_vs_oracle(fg, n, q, comps):
    b = 3 if n >= 8192 else 4
    t = 16
    r = fg.PolynomialRing(n, q)
    o = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r, t)
    sk = rnd(n + 7, 3, n)
    key = fg.SecretKey(r, sk)
    ct = rnd(n + 8, q, b, comps, n)
    ct[0, 0, :2] = [M64, q]
    for is_ntt in (False, True):
        res = eng.decrypt(ct, key, is_ntt=is_ntt, with_phase=True)
        for i in range(b):
            ev, eph, emx = o.decrypt(t, sk, ct[i], is_ntt)
            assert (res.phase[i] == eph).all(), (is_ntt, i)
            assert (res.values[i] == ev).all(), (is_ntt, i)
            assert int(res.max_noise[i]) == emx, (is_ntt, i)
        # without a phase buffer (degree 2 in coefficient form uses a device workspace)
        res2 = eng.decrypt(ct, key, is_ntt=is_ntt)
        assert (res2.values == res.values).all() and (res2.max_noise == res.max_noise).all()


@pytest.mark.parametrize("n,q", [(16, 97), (1024, P27), (4096, P62), (16384, P27), (1024, QG), (32768, P62)])
def test_add_plain_vs_oracle(fg, n, q):
    b, t = 3, 4
    r = fg.PolynomialRing(n, q)
    o = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r, t)
    ct = rnd(n + 9, q, b, 2, n)
    ct[0, 1, 0] = M64  # c1 is copied raw (clone)
    vals = rnd(n + 10, t, b, n)
    for is_ntt in (False, True):
        got = eng.add_plain(ct, vals, is_ntt=is_ntt)
        for i in range(b):
            assert (got[i] == o.add_plain(t, ct[i], vals[i], is_ntt)).all(), (is_ntt, i)
    # one scalar plaintext for every ciphertext (encode_plaintext)
    got = eng.add_plain(ct, 3)
    one = np.zeros(n, np.uint64)
    one[0] = 3
    assert (got[1] == o.add_plain(t, ct[1], one, False)).all()


@pytest.mark.parametrize("n,q,t,mode", [(n, q, t, m) for n, q, t in [(16384, P27, 4), (16384, P62, 1 << 20),
                                                                     (4096, P27, 256), (65536, P62, 256)]
                                         for m in ("compat", "negacyclic")]
                         + [(4096, QG, 1 << 20, "negacyclic"), (32768, Q63, 16, "negacyclic")])
def test_encrypt_decrypt_identity_full_degree(fg, n, q, t, mode):
    """Size-independent property: the transform product is commutative and
    associative in both modes, so with pk = (a, a s) and e1 = e2 = 0 the phase
    of encrypt(m) is exactly encode(m) and decrypt returns m with max noise
    0; with small errors (|e| <= 3) decryption still succeeds and returns m
    in the negacyclic ring."""
    import torch

    b = 16
    r = fg.PolynomialRing(n, q, mode=mode)
    eng = fg.EncryptionEngine(r, t)
    dev = "cuda:0"

    def D(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)

    a = rnd(901, q, n)
    s = rnd(902, 3, n)
    s = np.where(s == 2, np.uint64(q - 1), s).astype(np.uint64)  # ternary {-1, 0, 1}
    pk = fg.PublicKey(r, D(np.stack([a, r.multiply(a, s)])))
    key = fg.SecretKey(r, D(s))
    m = rnd(903, t, b, n)
    u = rnd(904, 3, b, n)
    u = np.where(u == 2, np.uint64(q - 1), u).astype(np.uint64)
    z = np.zeros((b, n), np.uint64)
    ct = eng.encrypt(D(m), pk, D(u), D(z), D(z))
    res = eng.decrypt(ct, key, with_phase=True)
    torch.cuda.synchronize()
    assert (res.values.cpu().numpy().view(np.uint64) == m).all()
    assert (res.max_noise == 0).all() and res.success.all()
    assert (res.phase.cpu().numpy().view(np.uint64) == oracle.encode(q, t, m)).all()
    if mode == "negacyclic":
        e = rnd(905, 7, 2, b, n).astype(np.int64) - 3
        e = np.where(e < 0, np.uint64(q) - (-e).astype(np.uint64), e.astype(np.uint64)).astype(np.uint64)
        ct = eng.encrypt(D(m), pk, D(u), D(e[0]), D(e[1]))
        res = eng.decrypt(ct, key)
        assert (res.values.cpu().numpy().view(np.uint64) == m).all() and res.success.all()


@pytest.mark.parametrize("n,q,bl,lv,dim", [(256, 7681, 4, 3, 8), (1024, P62, 23, 1, 12), (2048, P62, 15, 2, 6)])
def test_bootstrap_vs_oracle(fg, n, q, bl, lv, dim):
    k, b = 1, 3
    ks_bl, ks_lv, out_dim = 4, 3, 37
    r = fg.PolynomialRing(n, q)
    o = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(61, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a, lwe_b = rnd(62, q, b, dim), rnd(63, q, b)
    lwe_a[0, 0] = 0  # a skipped CMux step
    tp = be.create_lookup_table(lambda x: (3 * x + 1) % 8, 8, 8)
    ksk_a, ksk_b = rnd(64, q, k * n * ks_lv, out_dim), rnd(65, q, k * n * ks_lv)
    oa, ob = be.bootstrap(lwe_a, lwe_b, bsk_ntt, tp, ksk_a, ksk_b, ks_bl, ks_lv)
    assert oa.shape == (b, out_dim) and ob.shape == (b,)
    for i in range(b):
        ea, eb = o.bootstrap(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, tp, ks_bl, ks_lv, ksk_a, ksk_b)
        assert (oa[i] == ea).all() and int(ob[i]) == eb, i


def test_engine_ops_on_multi_device_context(fg):
    import torch

    devs = [0, 0] if torch.cuda.device_count() < 2 else list(range(min(4, torch.cuda.device_count())))
    n, q, t, b = 2048, P62, 8, 5
    r = fg.PolynomialRing(n, q, devices=devs)
    o = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r, t)
    pk, sk = rnd(71, q, 2, n), rnd(72, 3, n)
    u, e1, e2, vals = rnd(73, 3, b, n), rnd(74, q, b, n), rnd(75, q, b, n), rnd(76, t, b, n)
    ct = eng.encrypt(vals, fg.PublicKey(r, pk), u, e1, e2)
    res = eng.decrypt(ct, fg.SecretKey(r, sk), with_phase=True)
    for i in range(b):
        assert (ct[i] == o.encrypt(t, pk, vals[i], u[i], e1[i], e2[i])).all(), i
        ev, eph, emx = o.decrypt(t, sk, ct[i])
        assert (res.values[i] == ev).all() and (res.phase[i] == eph).all() and int(res.max_noise[i]) == emx


def test_engine_errors(fg):
    # N > 16384 is composed (engine_composed.hip), no longer refused
    r = fg.PolynomialRing(32768, P27)
    assert not fg.SecretKey(r, np.zeros(32768, np.uint64)).prep.any()
    r = fg.PolynomialRing(16, 97)
    eng = fg.EncryptionEngine(r)
    with pytest.raises(fg.FHEError):
        eng.decrypt(np.zeros((2, 4, 16), np.uint64), fg.SecretKey(r, np.zeros(16, np.uint64)))
