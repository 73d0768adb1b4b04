"""Device randomness and key material (keygen.hip) vs the CPU oracle.

The sampler is the seeded ChaCha20 stream of include/fhe_gpu.h (restated in
oracle/ref_cpu.c, oracle_sample); the keys follow key_manager.cpp:218-333
and bootstrap_engine.cpp:268-420 over the context's transform product.  Every
GPU result must equal the oracle's on the same (seed, stream).
"""
import numpy as np
import pytest

import oracle

P27 = 132120577
P62 = 4611686018326724609
Q50 = 1125899906826241  # Q_50_1 (tfhe-128-balanced)
Q63 = 9223370937344327681  # just below 2^63
QG = 18446744069414584321  # 2^64 - 2^32 + 1: (int64_t)q < 0 in the reference's Gaussian loop
SEED = [0x0123456789ABCDEF, 0x0F1E2D3C4B5A6978, 42, 7]


@pytest.fixture(scope="module")
def fg():
    import fhe_gpu

    return fhe_gpu


gpu = pytest.mark.gpu


@gpu
@pytest.mark.parametrize("q", [97, P27, Q50, P62, Q63, QG])
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_sample_vs_oracle(fg, q, kind):
    """Every sampler vs the oracle; at QG the Gaussian's negative samples
    take the closed form of the reference loop's int64 wrap (keygen.hip)."""
    ring = fg.PolynomialRing(16 if q == 97 else 1024, q)  # 97 = 3 * 2^5 + 1: degrees up to 16
    for count in (1, 1000, 65536 + 3):
        got = fg.sample(ring, kind, SEED, 11, count, std_dev=3.2)
        ref = oracle.sample(kind, SEED, 11, q, count, 3.2)
        assert (got == ref).all(), (q, kind, count)


@gpu
def test_sample_device_output_and_statistics(fg):
    import torch

    ring = fg.PolynomialRing(1024, P62)
    n = 1 << 20
    d = fg.sample(ring, fg.SAMPLE_GAUSSIAN, SEED, 5, n, std_dev=3.2, device_out=True)
    torch.cuda.synchronize()
    v = d.cpu().numpy().view(np.uint64)
    assert (v == oracle.sample(2, SEED, 5, P62, n, 3.2)).all()
    s = np.where(v > P62 // 2, v.astype(object) - P62, v.astype(object)).astype(np.int64)
    assert abs(s.mean()) < 0.02 and abs(s.std() - 3.2) < 0.02
    t = fg.sample(ring, fg.SAMPLE_TERNARY, SEED, 6, n)
    counts = [(t == P62 - 1).sum(), (t == 0).sum(), (t == 1).sum()]
    assert sum(counts) == n and min(counts) > 0.33 * n


@gpu
@pytest.mark.parametrize("n,q,mode", [(1024, P27, "compat"), (4096, P62, "compat"), (2048, Q50, "negacyclic"),
                                      (8192, 1152921504606584833, "compat"), (1024, Q63, "compat"),
                                      (1024, QG, "compat")])
def test_public_and_eval_key_vs_oracle(fg, n, q, mode):
    ring = fg.PolynomialRing(n, q, mode=mode)
    ref = oracle.NTT(n, q) if mode == "compat" else None
    kg = fg.KeyGenerator(ring, SEED, noise_std=3.2)
    sk = kg.secret_key(1)
    assert (sk == oracle.sample(1, SEED, 1, q, n)).all()
    pk = kg.public_key(sk, 2)
    base_log = 60 if q.bit_length() > 59 else 8
    rlk = kg.eval_key(sk, base_log, 3, 10)
    if ref is not None:
        assert (pk == ref.public_key_generate(sk, SEED, 2, 3.2)).all()
        assert (rlk == ref.eval_key_generate(sk, base_log, 3, SEED, 10, 3.2)).all()
    else:  # negacyclic: b - a s = e exactly (the ring product is the true one)
        e = oracle.sample(2, SEED, 3, q, n, 3.2)
        as_ = ring.multiply(pk[0], sk)
        assert (ring.subtract(pk[1], as_) == e).all()


@gpu
@pytest.mark.parametrize("n,q,k,bl,lv", [(512, P62, 1, 23, 1), (1024, Q50, 1, 15, 2), (256, P27, 2, 8, 2)])
def test_ggsw_and_ksk_vs_oracle(fg, n, q, k, bl, lv):
    ring = fg.PolynomialRing(n, q)
    ref = oracle.NTT(n, q)
    kg = fg.KeyGenerator(ring, SEED, noise_std=3.2)
    sk = kg.secret_key(1)
    vals = np.array([0, 1, -1, 3, 1, 0, -2], dtype=np.int64)
    g = kg.ggsw(vals, sk, k, bl, lv, 20)
    assert g.shape == (len(vals), (k + 1) * lv, k + 1, n)
    assert (g == ref.ggsw_encrypt(k, bl, lv, vals, sk, SEED, 20, 3.2)).all()
    lwe_sk = oracle.sample(3, SEED, 30, q, 37).astype(np.int64)
    ka, kb = kg.key_switch_key(sk, lwe_sk, bl, lv, 40)
    ra, rb = oracle.ksk_generate(q, bl, lv, sk, lwe_sk, SEED, 40)
    assert (ka == ra).all() and (kb == rb).all()


@gpu
def test_ggsw_device_resident_matches_host(fg):
    import torch

    ring = fg.PolynomialRing(1024, P62)
    kg = fg.KeyGenerator(ring, SEED)
    sk = kg.secret_key(1)
    vals = np.arange(-3, 5, dtype=np.int64)
    host = kg.ggsw(vals, sk, 1, 23, 1, 3)
    dev = kg.ggsw(torch.as_tensor(vals, device="cuda"), torch.as_tensor(sk.view(np.int64), device="cuda"),
                  1, 23, 1, 3)
    torch.cuda.synchronize()
    assert (dev.cpu().numpy().view(np.uint64) == host).all()


@gpu
@pytest.mark.parametrize("q,t", [(P62, 4), (Q50, 16), (P27, 65537)])
def test_lwe_decrypt_vs_oracle(fg, q, t):
    dim, batch = 742, 257
    sk = oracle.sample(3, SEED, 1, q, dim).astype(np.int64) - (oracle.sample(3, SEED, 2, q, dim).astype(np.int64))
    a = oracle.sample(0, SEED, 3, q, batch * dim).reshape(batch, dim)
    b = oracle.sample(4, SEED, 4, 0, batch)  # raw u64 bodies: any word is x mod q
    vals, ph = fg.lwe_decrypt(q, t, sk, a, b)
    for i in range(batch):
        rv, rp = oracle.lwe_decrypt(q, t, sk, a[i], b[i])
        assert (int(vals[i]), int(ph[i])) == (rv, rp)


@gpu
@pytest.mark.parametrize("n,q", [(1024, P27), (4096, P62), (8192, 1152921504606584833)])
def test_encrypt_sampled_vs_oracle(fg, n, q):
    ring = fg.PolynomialRing(n, q)
    ref = oracle.NTT(n, q)
    kg = fg.KeyGenerator(ring, SEED)
    sk = kg.secret_key(1)
    pk = kg.public_key(sk, 2)
    eng = fg.EncryptionEngine(ring, 65537)
    batch = 3
    vals = oracle.sample(0, SEED, 50, 65537, batch * n).reshape(batch, n)
    ct = eng.encrypt_sampled(vals, fg.PublicKey(ring, pk), SEED, 100, 3.2)
    u = oracle.sample(1, SEED, 100, q, batch * n).reshape(batch, n)
    e1 = oracle.sample(2, SEED, 101, q, batch * n, 3.2).reshape(batch, n)
    e2 = oracle.sample(2, SEED, 102, q, batch * n, 3.2).reshape(batch, n)
    for i in range(batch):
        assert (ct[i] == ref.encrypt(65537, pk, vals[i], u[i], e1[i], e2[i])).all()
    res = eng.decrypt(ct, fg.SecretKey(ring, sk))
    for i in range(batch):
        rv, _, rmx = ref.decrypt(65537, sk, ct[i])
        assert (res.values[i] == rv).all() and int(res.max_noise[i]) == rmx


@gpu
def test_negacyclic_keys_decrypt_to_the_plaintext(fg):
    # semantic check in the true ring: encrypt(pk(sk)) decrypts to the slots
    n, q, t = 4096, P62, 65537
    ring = fg.PolynomialRing(n, q, mode="negacyclic")
    kg = fg.KeyGenerator(ring, SEED)
    sk = kg.secret_key(1)
    pk = fg.PublicKey(ring, kg.public_key(sk, 2))
    eng = fg.EncryptionEngine(ring, t)
    vals = oracle.sample(0, SEED, 50, t, 2 * n).reshape(2, n)
    ct = eng.encrypt_sampled(vals, pk, SEED, 100, 3.2)
    res = eng.decrypt(ct, fg.SecretKey(ring, sk))
    assert (res.values == vals).all() and res.success.all()
