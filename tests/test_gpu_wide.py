"""Moduli 2^62 <= q < 2^64 (ntt_wide.hip): the reference takes any odd u64 q
whose root search succeeds (ntt_processor.cpp:140-153; every product is a
128-bit %), so the GPU path must too.  HIP vs the CPU oracle, bit-exact:
ring ops and the composed ciphertext paths (encrypt / decrypt / add_plain
in tests/test_gpu_engine.py).

At q >= 2^63 the reference's NTTProcessor::mod_inverse (ntt_processor.cpp:
63-89) runs its signed Euclid on a negative int64 modulus and returns 0 for
N^-1 (1 for psi^-1), so its inverse transform -- and everything built on it
-- yields zeros; the compat mode reproduces that (the oracle restates the
same loop), while negacyclic mode, which the reference lacks, uses the true
inverses and is checked as a ring product."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

Q62 = 4611686018429485057     # 2^62 + 2^21 + 1 (smallest prime above 2^62 that is 1 mod 2^17)
Q63 = 9223370937344327681     # just below 2^63
QG = 18446744069414584321     # 2^64 - 2^32 + 1 (above 2^63: sums carry out of 64 bits)
WIDE = [Q62, Q63, QG]


@pytest.fixture(scope="module")
def fg():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import fhe_gpu

    return fhe_gpu


@pytest.mark.parametrize("n", [4, 8, 64, 1024, 4096, 16384, 32768, 65536])
@pytest.mark.parametrize("q", WIDE)
def test_wide_transforms_vs_oracle(fg, n, q):
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    assert r.primitive_root == t.psi
    b = 2 if n > 16384 else 3 if n >= 4096 else 9
    x = oracle.splitmix_fill(n * 7 + 1, q, b * n).reshape(b, n)
    y = oracle.splitmix_fill(n * 7 + 2, q, b * n).reshape(b, n)
    assert (r.forward_ntt(x) == t.forward(x)).all()
    assert (r.inverse_ntt(x) == t.inverse(x)).all()
    assert (r.multiply(x, y) == t.polymul(x, y)).all()
    assert (r.forward_ntt_mul(x, y) == t.fwd_mul(x, y)).all()
    assert (r.pointwise_multiply(x, y) == oracle.pointwise(q, x.ravel(), y.ravel()).reshape(b, n)).all()
    assert (r.add(x, y) == oracle.poly_add(q, x.ravel(), y.ravel()).reshape(b, n)).all()
    assert (r.subtract(x, y) == oracle.poly_sub(q, x.ravel(), y.ravel()).reshape(b, n)).all()


@pytest.mark.parametrize("n,q", [(1024, QG), (16384, Q63), (32768, QG)])
def test_wide_raw_u64_inputs(fg, n, q):
    """Any u64 word behaves as x mod q (values >= q, the top of the range)."""
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    rng = np.random.default_rng(n)
    x = rng.integers(0, 2 ** 64 - 1, (2, n), dtype=np.uint64, endpoint=True)
    x[0, :3] = [0, q, 2 ** 64 - 1]
    y = rng.integers(0, 2 ** 64 - 1, (2, n), dtype=np.uint64, endpoint=True)
    assert (r.forward_ntt(x) == t.forward(x)).all()
    assert (r.inverse_ntt(x) == t.inverse(x)).all()
    assert (r.multiply(x, y) == t.polymul(x, y)).all()
    assert (r.forward_ntt_mul(x, y) == t.fwd_mul(x, y)).all()


@pytest.mark.parametrize("q", WIDE)
def test_wide_in_place_and_aliasing(fg, q):
    import torch

    n = 2048
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    x = oracle.splitmix_fill(11, q, 4 * n).reshape(4, n)
    y = oracle.splitmix_fill(12, q, 4 * n).reshape(4, n)
    dx = torch.from_numpy(x.view(np.int64)).cuda()
    dy = torch.from_numpy(y.view(np.int64)).cuda()
    r.multiply(dx, dy, out=dy)  # out aliases b
    torch.cuda.synchronize()
    assert (dy.cpu().numpy().view(np.uint64) == t.polymul(x, y)).all()
    r.forward_ntt(dx, out=dx)  # in place
    torch.cuda.synchronize()
    assert (dx.cpu().numpy().view(np.uint64) == t.forward(x)).all()


@pytest.mark.parametrize("q", [Q62, QG])
def test_wide_negacyclic_ring_product(fg, q):
    n = 4096
    r = fg.PolynomialRing(n, q, mode="negacyclic")
    x = oracle.splitmix_fill(5, q, n).reshape(1, n)
    X = np.zeros((1, n), np.uint64)
    X[0, 1] = 1
    expect = np.roll(x, 1, axis=1)
    expect[0, 0] = (q - int(x[0, -1])) % q
    assert (r.multiply(x, X) == expect).all()
    assert (r.inverse_ntt(r.forward_ntt(x)) == x).all()


@pytest.mark.parametrize("n,q", [(1024, QG), (4096, Q62)])
def test_wide_ciphertext_multiply_and_relinearize(fg, n, q):
    """Composed paths (transforms + the exact pointwise tensor + the canonical
    Montgomery key MAC) at q >= 2^62, vs the oracle's reference loops."""
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r)
    x = oracle.splitmix_fill(21, q, 2 * 2 * n).reshape(2, 2, n)
    y = oracle.splitmix_fill(22, q, 2 * 2 * n).reshape(2, 2, n)
    ct3 = eng.multiply(x, y)
    for i in range(2):
        assert (ct3[i] == t.ct_multiply(x[i], y[i])).all(), i
    bl, lv = 16, 4
    rlk = oracle.splitmix_fill(23, q, lv * 2 * n).reshape(lv, 2, n)
    out = eng.relinearize(ct3, fg.EvaluationKey(r, rlk, bl))
    for i in range(2):
        assert (out[i] == t.relinearize(bl, lv, ct3[i], rlk)).all(), i


@pytest.mark.parametrize("q", [Q62, QG])
def test_wide_external_product(fg, q):
    n, k, bl, lv = 1024, 1, 20, 2
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    ggsw = oracle.splitmix_fill(31, q, (k + 1) * lv * (k + 1) * n).reshape((k + 1) * lv, k + 1, n)
    glwe = oracle.splitmix_fill(32, q, 3 * (k + 1) * n).reshape(3, k + 1, n)
    got = fg.ExternalProduct(r, ggsw, bl, lv, k)(glwe)
    for i in range(3):
        assert (got[i] == t.external_product(k, bl, lv, glwe[i], ggsw)).all(), i


def test_wide_keys_prepare(fg):
    """encrypt / decrypt / add_plain at q >= 2^62 are composed from the wide
    transforms (engine_composed.hip; checked against the oracle in
    tests/test_gpu_engine.py): the key preparation no longer refuses them."""
    r = fg.PolynomialRing(1024, QG)
    pk = fg.PublicKey(r, np.zeros((2, 1024), np.uint64))
    assert pk.prep.shape == (2, 1024) and not pk.prep.any()
    sk = fg.SecretKey(r, np.zeros(1024, np.uint64))
    assert not sk.prep.any()


# ------------------------------------------------------------ q >= 2^63, negacyclic
# Compat mode at q >= 2^63 reproduces the reference's zero inverse, so its
# inverse-side paths compare zeros with zeros.  Negacyclic mode uses the true
# inverses: these checks exercise the wide inverse (the HBM stage kernel at
# N > 16384) and the 65-bit key MAC with non-zero data, through the identity
# p(x) for a root x of X^N + 1 (x = psi^(2j+1)): ring products evaluate to
# products, so every output is checked exactly at several such points.
def _roots(q, psi, count=3):
    return [pow(psi, 2 * j + 1, q) for j in (1, 1234, 98765)[:count]]


def _ev(p, x, q):
    acc = 0
    for c in reversed([int(v) for v in np.asarray(p).ravel()]):
        acc = (acc * x + c) % q
    return acc


@pytest.mark.parametrize("n", [32768, 65536])
def test_wide_negacyclic_big_degree_qg(fg, n):
    q = QG
    r = fg.PolynomialRing(n, q, mode="negacyclic")
    x = oracle.splitmix_fill(n + 3, q, 2 * n).reshape(2, n)
    y = oracle.splitmix_fill(n + 4, q, 2 * n).reshape(2, n)
    f = r.forward_ntt(x)
    assert (r.inverse_ntt(f) == x).all()
    m = r.multiply(x, y)
    for pt in _roots(q, r.primitive_root):
        for i in range(2):
            assert _ev(m[i], pt, q) == _ev(x[i], pt, q) * _ev(y[i], pt, q) % q
    # the forward transform is evaluation: X_k = a(psi^(2 brv-free k + 1)) for some ordering;
    # inverse(pointwise(fwd x, fwd y)) is the same product
    assert (r.inverse_ntt(r.pointwise_multiply(f, r.forward_ntt(y))) == m).all()


@pytest.mark.parametrize("n", [1024, 32768])
def test_wide_negacyclic_relinearize_and_extprod_qg(fg, n):
    """relinearize (encryption.cpp:904-980): c_j' = c_j + sum_l d_l(c2) rlk_l
    with unsigned digits d_l = (c2 >> l B) & (2^B - 1); external product
    (bootstrap_engine.cpp:431-518): res_j = sum_r D_r g_rj with the signed
    TFHE digits -- both checked by evaluation at roots of X^N + 1."""
    q = QG
    r = fg.PolynomialRing(n, q, mode="negacyclic")
    eng = fg.EncryptionEngine(r)
    bl, lv = 16, 4
    ct3 = oracle.splitmix_fill(41, q, 3 * n).reshape(1, 3, n)
    rlk = oracle.splitmix_fill(42, q, lv * 2 * n).reshape(lv, 2, n)
    out = eng.relinearize(ct3, fg.EvaluationKey(r, rlk, bl))[0]
    c2 = ct3[0, 2]
    digits = [(c2 >> np.uint64(l * bl)) & np.uint64((1 << bl) - 1) for l in range(lv)]
    for pt in _roots(q, r.primitive_root, 2):
        d = [_ev(dl, pt, q) for dl in digits]
        e0 = (_ev(ct3[0, 0], pt, q) + sum(d[l] * _ev(rlk[l, 1], pt, q) for l in range(lv))) % q
        e1 = (_ev(ct3[0, 1], pt, q) + sum(d[l] * _ev(rlk[l, 0], pt, q) for l in range(lv))) % q
        assert (_ev(out[0], pt, q), _ev(out[1], pt, q)) == (e0, e1)
    k, bl, lv = 1, 20, 2
    ggsw = oracle.splitmix_fill(43, q, (k + 1) * lv * (k + 1) * n).reshape((k + 1) * lv, k + 1, n)
    glwe = oracle.splitmix_fill(44, q, (k + 1) * n).reshape(1, k + 1, n)
    got = fg.ExternalProduct(r, ggsw, bl, lv, k)(glwe)[0]
    rows = np.concatenate([oracle.decompose(q, glwe[0, i], bl, lv) for i in range(k + 1)])
    for pt in _roots(q, r.primitive_root, 2):
        dv = [_ev(rw, pt, q) for rw in rows]
        for j in range(k + 1):
            assert _ev(got[j], pt, q) == sum(dv[t] * _ev(ggsw[t, j], pt, q) for t in range(len(rows))) % q
