"""Pin the CPU oracle (oracle/ref_cpu.c) before trusting it.

1. The reference's own known-answer tests and properties
   (cpp/tests/test_ntt_processor.cpp, test_polynomial_ring.cpp,
   test_multi_limb.cpp) pass on the restatement.
2. The psi table measured on the compiled reference.
3. An independent big-integer restatement (oracle/pyref.py, following the
   reference's TypeScript restatement) agrees bit for bit.
4. The committed golden fixtures regenerate identically.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import pyref

P27 = 132120577
P62 = 4611686018326724609


@pytest.fixture(scope="module")
def kat(golden_dir):
    with open(os.path.join(golden_dir, "reference_kat.json")) as f:
        return json.load(f)


def load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


def U(x):
    return np.array(x, dtype=np.uint64)


# --------------------------------------------------- reference known answers
def test_static_helpers(kat):
    for n in kat["is_power_of_two_true"]:
        assert oracle.is_power_of_two(n)
    for n in kat["is_power_of_two_false"]:
        assert not oracle.is_power_of_two(n)
    for n, l in kat["log2_pow2"]:
        assert oracle.log2_pow2(n) == l
    for i, r in kat["bit_reverse_3"]:
        assert oracle.bit_reverse(i, 3) == r
    for b, e, m, r in kat["mod_pow"]:
        assert oracle.mod_pow(b, e, m) == r
    for a, m in kat["mod_inverse_products"]:
        assert (a * oracle.mod_inverse(a, m)) % m == 1


def test_psi_table_matches_compiled_reference(kat):
    for n, q, psi in kat["psi_table"]:
        t = oracle.NTT(n, q)
        assert t.psi == psi
        assert oracle.mod_pow(psi, 2 * n, q) == 1 and oracle.mod_pow(psi, n, q) == q - 1


def test_constructor_errors():
    with pytest.raises(oracle.OracleError, match="power of 2"):
        oracle.NTT(12, 97)
    with pytest.raises(oracle.OracleError, match="between 4 and 65536"):
        oracle.NTT(2, 97)
    with pytest.raises(oracle.OracleError, match="odd"):
        oracle.NTT(8, 96)
    with pytest.raises(oracle.OracleError, match="NTT-friendly"):
        oracle.NTT(16, 17)


def test_ntt_simple_q17():  # test_ntt_processor.cpp:152-179
    t = oracle.NTT(8, 17)
    x = U([1, 2, 3, 4, 5, 6, 7, 8])
    assert (t.inverse(t.forward(x)) == x).all()


def test_round_trip_property(kat):  # test_ntt_processor.cpp:193-268, seed 42 draw order
    for n, q, iters, seed in kat["round_trip_configs"]:
        t = oracle.NTT(n, q)
        draws = oracle.testrandom_coeffs(seed, q, n * iters).reshape(iters, n)
        assert (t.inverse(t.forward(draws)) == draws).all()


def test_transforms_data():  # test_ntt_processor.cpp:327-356
    t = oracle.NTT(1024, P27)
    x = oracle.testrandom_coeffs(42, P27, 1024)
    assert int((t.forward(x) != x).sum()) > 100


def test_ring_q17(kat):  # test_polynomial_ring.cpp:69-185
    for a, b, c in kat["ring_q17"]["add"]:
        assert list(oracle.poly_add(17, U(a), U(b))) == c
    for a, b, c in kat["ring_q17"]["sub"]:
        assert list(oracle.poly_sub(17, U(a), U(b))) == c
    a = U([0, 1, 5, 16])
    assert list(oracle.poly_neg(17, a)) == [0, 16, 12, 1]


def test_polymul_identity_zero():  # test_polynomial_ring.cpp:191-219
    t = oracle.NTT(64, 257)
    x = oracle.testrandom_coeffs(3, 257, 64)
    one = np.zeros(64, np.uint64)
    one[0] = 1
    # the compat transform is not the ring product, but fwd(1) is all ones
    assert (t.forward(one) == 1).all()
    assert (t.polymul(x, one) == x).all()
    assert (t.polymul(x, np.zeros(64, np.uint64)) == 0).all()


def test_multi_limb_round_trip():  # test_multi_limb.cpp:16-208 (Montgomery round trip)
    for qm in ([P62, 1], [0x1234567890ABCDEF, 0x0FEDCBA987654321]):
        k = oracle.ml_constants(qm)
        qv = qm[0] | (qm[1] << 64)
        R = 1 << 128
        assert (k[2] | (k[3] << 64)) == R % qv
        assert (k[4] | (k[5] << 64)) == (R * R) % qv
        assert (k[6] * qm[0]) % (1 << 64) == (1 << 64) - 1  # -q^-1 mod 2^64
        rng = np.random.default_rng(1)
        for _ in range(50):
            v = int(rng.integers(0, 2 ** 63)) * int(rng.integers(1, 2 ** 62)) % qv
            a = U([[v & (2 ** 64 - 1), v >> 64]])
            r2 = U([[k[4], k[5]]])
            am = oracle.ml_montmul_batch(qm, a, r2)  # to_montgomery
            one = U([[1, 0]])
            back = oracle.ml_montmul_batch(qm, am, one)  # from_montgomery
            assert int(back[0, 0]) | (int(back[0, 1]) << 64) == v


def test_barrett_is_exact():  # barrett_mul correct
    rng = np.random.default_rng(3)
    for q in (P27, P62, 17, 2 ** 63 + 29):
        a = rng.integers(0, 2 ** 64 - 1, 2000, dtype=np.uint64, endpoint=True)
        b = rng.integers(0, 2 ** 64 - 1, 2000, dtype=np.uint64, endpoint=True)
        c = oracle.modmul_batch(q, a, b)
        assert [int(x) for x in c] == [int(x) * int(y) % q for x, y in zip(a, b)]


def test_compat_montgomery_is_reference_quirk():  # 0/10000 correct
    k = oracle.mont_constants(P27)
    rng = np.random.default_rng(5)
    ok = 0
    for _ in range(2000):
        a, b = int(rng.integers(0, P27)), int(rng.integers(0, P27))
        r = oracle.from_mont(k, oracle.mont_mul(k, oracle.to_mont(k, a), oracle.to_mont(k, b)))
        ok += r == a * b % P27
    assert ok == 0
    assert k[1] == (1 << 64) % P27 and k[2] == ((1 << 64) % P27) ** 2 % P27


def test_mt19937_64_known_value():
    # std::mt19937_64 default seed 5489: 10000th output (C++11 [rand.predef])
    assert int(oracle.mt19937_64_raw(5489, 10000)[-1]) == 9981545732273789042


# --------------------------------------------------- independent restatement
@pytest.mark.parametrize("n,q", [(8, 17), (16, 97), (32, 193), (256, 7681), (512, 12289), (1024, P27), (1024, P62)])
def test_oracle_matches_pyref(n, q):
    t = oracle.NTT(n, q)
    x = oracle.testrandom_coeffs(9, q, n)
    y = oracle.testrandom_coeffs(10, q, n)
    xs, ys = [int(v) for v in x], [int(v) for v in y]
    assert [int(v) for v in t.forward(x)] == pyref.forward(xs, q)
    assert [int(v) for v in t.inverse(x)] == pyref.inverse(xs, q)
    assert [int(v) for v in t.polymul(x, y)] == pyref.polymul(xs, ys, q)


@pytest.mark.parametrize("n,q", [(32768, P62), (65536, P27)])
def test_oracle_matches_pyref_large_degree(n, q):
    """The degrees the two-pass GPU path serves: N = 32768 with the 62-bit
    prime is the TS round-trip suite's largest case
    (ntt-round-trip.prop.test.ts:43); 65536 is NTTProcessor's maximum
    (ntt_processor.cpp:146)."""
    t = oracle.NTT(n, q)
    x = oracle.splitmix_fill(n + 5, q, n)
    xs = [int(v) for v in x]
    f = t.forward(x)
    assert [int(v) for v in f] == pyref.forward(xs, q)
    assert (t.inverse(f) == x).all()


def test_non_canonical_inputs_behave_mod_q():
    t = oracle.NTT(64, 257)
    x = np.random.default_rng(2).integers(0, 2 ** 64 - 1, 64, dtype=np.uint64, endpoint=True)
    assert (t.forward(x) == t.forward(x % np.uint64(257))).all()
    assert (t.inverse(x) == t.inverse(x % np.uint64(257))).all()


def test_negacyclic_pyref_is_ring_product(golden_dir):
    for case in load(golden_dir, "negacyclic.json"):
        q = case["q"]
        fx = pyref.negacyclic_forward(case["x"], q)
        fy = pyref.negacyclic_forward(case["y"], q)
        assert pyref.negacyclic_inverse([(a * b) % q for a, b in zip(fx, fy)], q) == case["product"]
        assert case["product"] == pyref.negacyclic_schoolbook(case["x"], case["y"], q)


# --------------------------------------------------- fixtures regenerate
def test_golden_ntt_small(golden_dir):
    for c in load(golden_dir, "ntt_small.json"):
        t = oracle.NTT(c["n"], c["q"])
        assert t.psi == c["psi"]
        x, y, w = U(c["x"]), U(c["y"]), U(c["w"])
        assert [int(v) for v in t.forward(x)] == c["forward"]
        assert [int(v) for v in t.inverse(x)] == c["inverse"]
        assert [int(v) for v in t.polymul(x, y)] == c["polymul"]
        assert [int(v) for v in t.fwd_mul(x, w)] == c["fwd_mul"]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


def test_golden_ntt_large(golden_dir):
    for c in load(golden_dir, "ntt_large.json"):
        n, q, b = c["n"], c["q"], c["batch"]
        t = oracle.NTT(n, q)
        x = oracle.splitmix_fill(c["seed_x"], q, b * n).reshape(b, n)
        y = oracle.splitmix_fill(c["seed_y"], q, b * n).reshape(b, n)
        assert _sha(t.forward(x)) == c["sha_forward"]
        assert _sha(t.polymul(x, y)) == c["sha_polymul"]


def test_golden_extprod_and_ml(golden_dir):
    for c in load(golden_dir, "extprod.json"):
        t = oracle.NTT(c["n"], c["q"])
        k, lv, n = c["k"], c["level"], c["n"]
        glwe = U(c["glwe"]).reshape(k + 1, n)
        ggsw = U(c["ggsw"]).reshape((k + 1) * lv, k + 1, n)
        assert [int(v) for v in t.external_product(k, c["base_log"], lv, glwe, ggsw).ravel()] == c["out"]
    for c in load(golden_dir, "multi_limb.json"):
        assert oracle.ml_constants(c["q"]) == c["constants"]
        a, b = U(c["a"]).reshape(-1, 2), U(c["b"]).reshape(-1, 2)
        assert [int(v) for v in oracle.ml_montmul_batch(c["q"], a, b).ravel()] == c["c"]
    for c in load(golden_dir, "modmul.json"):
        assert [int(v) for v in oracle.modmul_batch(c["q"], U(c["a"]), U(c["b"]))] == c["c"]


def test_external_product_equals_ntt_domain_accumulation(golden_dir):
    """The linearity the GPU kernel relies on: sum_r inv(X_r) == inv(sum_r X_r)."""
    c = load(golden_dir, "extprod.json")[2]
    q, n, k, lv, bl = c["q"], c["n"], c["k"], c["level"], c["base_log"]
    t = oracle.NTT(n, q)
    glwe = U(c["glwe"]).reshape(k + 1, n)
    ggsw = U(c["ggsw"]).reshape((k + 1) * lv, k + 1, n)
    acc = [0] * (k + 1)
    rows = []
    for i in range(k + 1):
        for d in oracle.decompose(q, glwe[i], bl, lv):
            rows.append(t.forward(d))
    for j in range(k + 1):
        s = np.zeros(n, dtype=object)
        for r, fd in enumerate(rows):
            s = (s + oracle.pointwise(q, fd, t.forward(ggsw[r, j])).astype(object)) % q
        acc[j] = t.inverse(U(list(s)))
    assert [int(v) for v in np.concatenate(acc)] == c["out"]


# ---------------------------------------------------------------- keygen randomness (oracle_sample)
def test_chacha20_block_rfc8439_vector():
    """RFC 8439 section 2.3.2 test vector through the oracle's block function
    (key 00..1f; counter word 1 and nonce 00000009 0000004a 00000000 map to
    the 64-bit counter / 64-bit nonce layout of include/fhe_gpu.h)."""
    import ctypes as C

    L = oracle.lib()
    u64p = C.POINTER(C.c_uint64)
    L.oracle_chacha_block.argtypes = [u64p, C.c_uint64, C.c_uint64, u64p]
    seed = np.frombuffer(bytes(range(32)), dtype=np.uint64).copy()
    out = np.zeros(8, dtype=np.uint64)
    L.oracle_chacha_block(seed.ctypes.data_as(u64p), 1 | (0x09000000 << 32), 0x4A000000, out.ctypes.data_as(u64p))
    assert out.tobytes().hex() == (
        "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
        "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def test_sample_kinds_follow_secure_random():
    """random_u64_range / sample_ternary / sample_binary (key_manager.cpp:60-114)
    over the raw stream: every kind is a function of the same raw draws."""
    seed, q = [5, 6, 7, 8], 97
    raw = oracle.sample(4, seed, 3, 0, 1000)
    binary = oracle.sample(3, seed, 3, q, 1000)
    assert (binary == (raw & 1)).all()
    thr = ((1 << 64) - q) % q
    uni = oracle.sample(0, seed, 3, q, 1000)
    ok = raw >= thr  # first draw accepted: value = raw % q
    assert (uni[ok] == raw[ok] % q).all()
    tern = oracle.sample(1, seed, 3, q, 1000)
    t3 = raw % 3  # (2^64 - 3) % 3 == 1: raw 0 is rejected, never drawn here
    assert (tern == np.where(t3 == 0, q - 1, np.where(t3 == 1, 0, 1))).all()
    g = oracle.sample(2, seed, 3, 1 << 61, 200000, 3.2).astype(object)
    s = np.array([int(v) - (1 << 61) if v > (1 << 60) else int(v) for v in g], dtype=np.int64)
    assert abs(s.mean()) < 0.05 and abs(s.std() - 3.2) < 0.05
    # element i of a stream does not depend on the other elements' rejections
    assert (oracle.sample(0, seed, 3, q, 1000)[:10] == oracle.sample(0, seed, 3, q, 1000)[:10]).all()


def test_keygen_restatements_are_consistent():
    """pk / eval key / GGSW / KSK restatements satisfy their defining
    equations under the restated transform product."""
    n, q = 64, 7681
    t = oracle.NTT(n, q)
    seed = [1, 2, 3, 4]
    sk = oracle.sample(1, seed, 1, q, n)
    pk = t.public_key_generate(sk, seed, 2, 3.2)
    e = oracle.sample(2, seed, 3, q, n, 3.2)
    assert (oracle.poly_sub(q, pk[1], t.polymul(pk[0], sk)) == e).all()
    rlk = t.eval_key_generate(sk, 4, 3, seed, 10, 3.2)
    s2 = t.polymul(sk, sk)
    for lv in range(3):
        el = oracle.sample(2, seed, 10 + 2 * lv + 1, q, n, 3.2)
        diff = oracle.poly_sub(q, oracle.poly_sub(q, rlk[lv, 1], t.polymul(rlk[lv, 0], sk)), el)
        assert (diff == oracle.poly_mul_scalar(q, s2, (1 << (4 * lv)) % q)).all()
    vals = np.array([1, -1, 0], dtype=np.int64)
    g = t.ggsw_encrypt(1, 4, 2, vals, sk, seed, 20, 3.2)
    masks = oracle.sample(0, seed, 20, q, 3 * 4 * n).reshape(3, 4, n)
    for c in range(3):
        for r in range(4):
            m = masks[c, r].copy()
            grp, lv = divmod(r, 2)
            gad = (abs(int(vals[c])) * q) >> ((lv + 1) * 4)
            if vals[c] < 0:
                gad = (q - gad) % q
            if grp == 0:
                m[0] = (int(m[0]) + gad) % q
            assert (g[c, r, 0] == m).all()
    lwe = np.array([1, 0, 1, 1, 0], dtype=np.int64)
    ka, kb = oracle.ksk_generate(q, 4, 2, sk[:8], lwe, seed, 40)
    assert ka.shape == (16, 5) and kb.shape == (16,)
    v, ph = oracle.lwe_decrypt(q, 4, lwe, ka[0], kb[0])
    assert 0 <= ph < q and 0 <= v < 4


def test_gaussian_wrap_closed_form_matches_loop():
    """The reference's Gaussian at q >= 2^63 (key_manager.cpp:102-109):
    (int64_t)q is negative, so the `while (v < 0) v += q` loop ends only when
    the sum wraps past INT64_MIN.  ref_cpu.c / keygen.hip compute that wrapped
    value in closed form (k = floor((v + 2^63) / m) + 1, m = 2^64 - q); here
    the same derivation at 16-bit width is checked against the literal loop."""
    import random

    B = 16

    def wrap(x):
        x &= (1 << B) - 1
        return x - (1 << B) if x >> (B - 1) else x

    rnd = random.Random(5)
    for _ in range(5000):
        q = rnd.randrange((1 << (B - 1)) | 1, 1 << B, 2)
        v = -rnd.randrange(1, 40)
        s = wrap(wrap(q) + v)
        while s < 0:
            s = wrap(s + wrap(q))
        m = (1 << B) - q
        k = (v + (1 << (B - 1))) // m + 1
        assert (s & ((1 << B) - 1)) % q == ((v - k * m) & ((1 << B) - 1)) % q


def test_gaussian_wide_modulus_terminates():
    """q = 2^64 - 2^32 + 1: the oracle returns at once, every value < q, and
    the non-negative samples are the plain rounded draws."""
    QG = 18446744069414584321
    seed = [1, 2, 3, 4]
    v = oracle.sample(2, seed, 9, QG, 4096, 3.2)
    assert (v < np.uint64(QG)).all()
    same = oracle.sample(2, seed, 9, 4611686018326724609, 4096, 3.2)
    small = same < np.uint64(64)  # non-negative draws are the same at both moduli
    assert small.sum() > 1000 and (v[small] == same[small]).all()
