"""Generate the golden fixtures in tests/golden/ (committed; rerun to refresh).

Provenance (see DESIGN.md "Oracle and pinning"):
  * ``reference_kat.json`` -- known answers copied as DATA from the
    reference's own tests (cpp/tests/test_ntt_processor.cpp:34-150,
    cpp/tests/test_polynomial_ring.cpp:69-185) and the psi table of
    SURVEY.md section 8 (values measured on the compiled reference when the
    survey was written).
  * every other file -- outputs of the C restatement ``oracle/ref_cpu.c``;
    for sizes where it is feasible each vector is ALSO recomputed by the
    independent big-integer restatement ``oracle/pyref.py`` (which follows
    the reference's TypeScript restatement) and generation aborts on any
    mismatch.  The reference C++ itself cannot be built in this image
    (modular_arithmetic.h:5 includes <arm_neon.h>), so these are restatement
    vectors, cross-checked, not reference-binary outputs.

Inputs: TestRandom(seed) = std::mt19937_64 raw draws % q, exactly as the
reference tests draw coefficients (cpp/tests/test_harness.h:29-73), and
splitmix64(seed ^ index) % q for the larger sizes.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from oracle import pyref  # noqa: E402

P27 = 132120577
P62 = 4611686018326724609
P40 = 1099511627777  # 2^40 + 1: not prime, the root search never ends (as in the reference)
Q2048 = 40961  # 10*4096 + 1, prime

SMALL = [(8, 17), (16, 97), (32, 193), (64, 257), (128, 769), (256, 7681), (512, 12289),
         (1024, P27), (1024, P62), (2048, Q2048), (4096, P27)]
LARGE = [(4096, P62), (16384, P27), (16384, P62), (32768, P27), (32768, P62), (65536, P27), (65536, P62)]


def L(a):
    return [int(x) for x in np.asarray(a).ravel()]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, separators=(",", ":"))
    print("wrote", name)


def reference_kat():
    return {
        "source": "cpp/tests/test_ntt_processor.cpp:34-150, cpp/tests/test_polynomial_ring.cpp:69-185, SURVEY.md 8",
        "is_power_of_two_true": [1, 2, 4, 1024, 32768],
        "is_power_of_two_false": [0, 3, 5, 1000],
        "log2_pow2": [[1, 0], [2, 1], [4, 2], [1024, 10], [32768, 15]],
        "bit_reverse_3": [[0, 0], [1, 4], [2, 2], [3, 6], [4, 1], [5, 5], [6, 3], [7, 7]],
        "mod_pow": [[2, 10, 1000, 24], [3, 5, 7, 5], [123, 0, 1000, 1], [3, 16, 17, 1]],
        "mod_inverse_products": [[3, 7], [12345, P27]],
        "psi_table": [[1024, P27, 113022246], [4096, P27, 67542050], [16384, P27, 39393627],
                      [16384, P62, 4096621604056103545]],
        "ring_q17": {
            "add": [[[1, 2, 3, 4, 5, 6, 7, 8], [8, 7, 6, 5, 4, 3, 2, 1], [9] * 8],
                    [[10] * 8, [10] * 8, [3] * 8]],
            "sub": [[[10] * 8, [3] * 8, [7] * 8]],
        },
        "round_trip_configs": [[8, 17, 100, 42], [16, 97, 100, 42], [1024, P27, 20, 42]],
    }


def ntt_small():
    out = []
    for n, q in SMALL:
        t = oracle.NTT(n, q)
        x = oracle.testrandom_coeffs(42, q, n)
        y = oracle.testrandom_coeffs(43, q, n)
        w = oracle.testrandom_coeffs(44, q, n)
        f = t.forward(x)
        i = t.inverse(x)
        m = t.polymul(x, y)
        fm = t.fwd_mul(x, w)
        if n <= 1024:
            xs, ys = L(x), L(y)
            assert L(f) == pyref.forward(xs, q), (n, q)
            assert L(i) == pyref.inverse(xs, q), (n, q)
            assert L(m) == pyref.polymul(xs, ys, q), (n, q)
        assert (t.inverse(f) == x).all()
        out.append({"n": n, "q": q, "psi": t.psi, "x": L(x), "y": L(y), "w": L(w),
                    "forward": L(f), "inverse": L(i), "polymul": L(m), "fwd_mul": L(fm)})
    return out


def ntt_large():
    out = []
    for n, q in LARGE:
        t = oracle.NTT(n, q)
        b = 4
        x = oracle.splitmix_fill(0x5EED, q, b * n).reshape(b, n)
        y = oracle.splitmix_fill(0xB0B, q, b * n).reshape(b, n)
        f = t.forward(x)
        i = t.inverse(x)
        m = t.polymul(x, y)
        fm = t.fwd_mul(x, y)
        e = {"n": n, "q": q, "batch": b, "seed_x": 0x5EED, "seed_y": 0xB0B,
             "sha_forward": sha(f), "sha_inverse": sha(i), "sha_polymul": sha(m), "sha_fwd_mul": sha(fm),
             "head_forward": L(f[0, :8]), "head_polymul": L(m[0, :8])}
        if n >= 32768:
            # two ciphertexts: rows (0, 1), (2, 3) of x times those of y
            # (EncryptionEngine::multiply at the two-pass degrees)
            ct = np.stack([t.ct_multiply(x[2 * j:2 * j + 2], y[2 * j:2 * j + 2]) for j in range(2)])
            e["sha_ct_multiply"] = sha(ct)
        out.append(e)
    return out


def modmul():
    rng = np.random.default_rng(7)
    qs = [17, 97, P27, P40, P62, 3, 2 ** 61 - 1, 2 ** 63 + 29, 2 ** 64 - 59, 1000, 2 ** 62, 1]
    out = []
    for q in qs:
        a = rng.integers(0, 2 ** 64 - 1, 64, dtype=np.uint64, endpoint=True)
        b = rng.integers(0, 2 ** 64 - 1, 64, dtype=np.uint64, endpoint=True)
        c = oracle.modmul_batch(q, a, b)
        assert L(c) == [(int(u) * int(v)) % q for u, v in zip(a, b)]
        out.append({"q": q, "a": L(a), "b": L(b), "c": L(c)})
    return out


def multi_limb():
    rng = np.random.default_rng(11)
    mods = [[P62, 1], [0xFFFFFFFFFFFFFFC5, 0xFFFFFFFFFFFFFFFF], [1, 1 << 63], [0x1234567890ABCDEF, 0x0FEDCBA987654321]]
    out = []
    for qm in mods:
        k = oracle.ml_constants(qm)
        qv = qm[0] | (qm[1] << 64)
        a = rng.integers(0, 2 ** 64 - 1, (32, 2), dtype=np.uint64, endpoint=True)
        b = rng.integers(0, 2 ** 64 - 1, (32, 2), dtype=np.uint64, endpoint=True)
        # canonical operands (< q), as Montgomery arithmetic expects
        for arr in (a, b):
            for r in range(arr.shape[0]):
                v = (int(arr[r, 0]) | (int(arr[r, 1]) << 64)) % qv
                arr[r, 0], arr[r, 1] = v & (2 ** 64 - 1), v >> 64
        c = oracle.ml_montmul_batch(qm, a, b)
        out.append({"q": qm, "constants": k, "a": L(a), "b": L(b), "c": L(c)})
    return out


def extprod():
    out = []
    for n, q, bl, lv in [(64, 257, 3, 2), (256, 7681, 4, 3), (1024, P27, 9, 3), (1024, P62, 23, 1), (1024, P62, 15, 2)]:
        t = oracle.NTT(n, q)
        k = 1
        glwe = oracle.testrandom_coeffs(5, q, (k + 1) * n).reshape(k + 1, n)
        ggsw = oracle.testrandom_coeffs(6, q, (k + 1) * lv * (k + 1) * n).reshape((k + 1) * lv, k + 1, n)
        res = t.external_product(k, bl, lv, glwe, ggsw)
        out.append({"n": n, "q": q, "base_log": bl, "level": lv, "k": k, "glwe": L(glwe), "ggsw": L(ggsw),
                    "out": L(res)})
    return out


def negacyclic():
    out = []
    for n, q in [(8, 17), (16, 97), (64, 257), (256, 7681)]:
        x = L(oracle.testrandom_coeffs(1, q, n))
        y = L(oracle.testrandom_coeffs(2, q, n))
        prod = pyref.negacyclic_schoolbook(x, y, q)
        fx = pyref.negacyclic_forward(x, q)
        assert pyref.negacyclic_inverse(fx, q) == x
        assert pyref.negacyclic_inverse([(a * b) % q for a, b in zip(fx, pyref.negacyclic_forward(y, q))], q) == prod
        out.append({"n": n, "q": q, "x": x, "y": y, "forward": fx, "product": prod})
    return out


def cipher():
    """Ciphertext-level vectors (EncryptionEngine::multiply / relinearize,
    BootstrapEngine::blind_rotate) from the C restatement; the multiply
    vectors are cross-checked against pyref's independent transform."""
    out = []
    for n, q in [(16, 97), (256, 7681), (1024, P27), (1024, P62)]:
        t = oracle.NTT(n, q)
        x = oracle.testrandom_coeffs(21, q, 2 * n).reshape(2, n)
        y = oracle.testrandom_coeffs(22, q, 2 * n).reshape(2, n)
        res = t.ct_multiply(x, y)
        if n <= 256:
            xs, ys = [L(v) for v in x], [L(v) for v in y]
            c1 = [(a + b) % q for a, b in zip(pyref.polymul(xs[0], ys[1], q), pyref.polymul(xs[1], ys[0], q))]
            assert [L(r) for r in res] == [pyref.polymul(xs[0], ys[0], q), c1, pyref.polymul(xs[1], ys[1], q)]
        out.append({"op": "ct_multiply", "n": n, "q": q, "ct1": L(x), "ct2": L(y), "out": L(res)})
    for n, q, bl, lv in [(16, 97, 2, 4), (256, 7681, 4, 4), (1024, P27, 4, 7), (1024, P62, 16, 4)]:
        t = oracle.NTT(n, q)
        ct3 = oracle.testrandom_coeffs(23, q, 3 * n).reshape(3, n)
        rlk = oracle.testrandom_coeffs(24, q, lv * 2 * n).reshape(lv, 2, n)
        out.append({"op": "relinearize", "n": n, "q": q, "base_log": bl, "level": lv, "ct3": L(ct3), "rlk": L(rlk),
                    "out": L(t.relinearize(bl, lv, ct3, rlk))})
    for n, q, bl, lv, dim in [(32, 193, 3, 2, 6), (256, 7681, 4, 3, 8)]:
        t = oracle.NTT(n, q)
        bsk = oracle.testrandom_coeffs(25, q, dim * 2 * lv * 2 * n).reshape(dim, 2 * lv, 2, n)
        lwe_a = oracle.testrandom_coeffs(26, q, dim)
        lwe_a[0] = 0
        acc = np.zeros((2, n), np.uint64)
        acc[1] = oracle.testrandom_coeffs(27, q, n)
        lwe_b = int(oracle.testrandom_coeffs(28, q, 1)[0])
        got = t.blind_rotate(1, bl, lv, lwe_a, lwe_b, q, bsk, acc)
        out.append({"op": "blind_rotate", "n": n, "q": q, "base_log": bl, "level": lv, "dim": dim, "bsk": L(bsk),
                    "lwe_a": L(lwe_a), "lwe_b": lwe_b, "acc": L(acc), "out": L(got)})
    return out


def _ternary(seed, q, n):
    r = oracle.splitmix_fill(seed, 3, n)
    return np.where(r == 2, np.uint64(q - 1), r).astype(np.uint64)


def _small(seed, q, n):  # errors in [-3, 3] as residues
    r = oracle.splitmix_fill(seed, 7, n).astype(np.int64) - 3
    return np.where(r < 0, r + q, r).astype(np.uint64)


def engine():
    """EncryptionEngine encrypt / decrypt / add_plain vectors from the C
    restatement (full arrays at small n), and the bfv-128-simd flow
    (N=8192, q = Q_60_1, t = 65537): keys, encrypt x2 -> multiply ->
    relinearize (base_log 60, 2 levels) -> decrypt, inputs from splitmix
    seeds (tests/js/napi_test.js regenerates them), outputs as SHA-256."""
    out = []
    for n, q, t in [(16, 97, 4), (256, 7681, 16)]:
        o = oracle.NTT(n, q)
        pk = oracle.splitmix_fill(31, q, 2 * n).reshape(2, n)
        sk = _ternary(32, q, n)
        vals, u = oracle.splitmix_fill(33, t, n), _ternary(34, q, n)
        e1, e2 = _small(35, q, n), _small(36, q, n)
        ct = o.encrypt(t, pk, vals, u, e1, e2)
        dv, ph, mx = o.decrypt(t, sk, ct)
        ap = o.add_plain(t, ct, vals)
        out.append({"op": "engine", "n": n, "q": q, "t": t, "pk": L(pk), "sk": L(sk), "values": L(vals), "u": L(u),
                    "e1": L(e1), "e2": L(e2), "ct": L(ct), "dec": L(dv), "phase": L(ph), "max_noise": mx,
                    "add_plain": L(ap)})
    # the bfv-128-simd flow
    n, q, t, bl, lv = 8192, 1152921504606584833, 65537, 60, 2
    o = oracle.NTT(n, q)
    sk = _ternary(41, q, n)
    a = oracle.splitmix_fill(42, q, n)
    pk = np.stack([a, oracle.poly_add(q, o.polymul(a, sk), _small(43, q, n))])
    cts = []
    for j in range(2):
        vals = oracle.splitmix_fill(44 + j, t, n)
        cts.append(o.encrypt(t, pk, vals, _ternary(46 + j, q, n), _small(48 + j, q, n), _small(50 + j, q, n)))
    ct3 = o.ct_multiply(cts[0], cts[1])
    s2 = o.polymul(sk, sk)
    rlk = np.zeros((lv, 2, n), np.uint64)
    power = 1
    for l in range(lv):
        al = oracle.splitmix_fill(52 + l, q, n)
        b = oracle.poly_add(q, oracle.poly_add(q, o.polymul(al, sk), _small(54 + l, q, n)),
                            oracle.poly_mul_scalar(q, s2, power))
        rlk[l, 0], rlk[l, 1] = al, b
        power = power * (1 << bl) % q
    rel = o.relinearize(bl, lv, ct3, rlk)
    dv, ph, mx = o.decrypt(t, sk, rel)
    dv0, _, mx0 = o.decrypt(t, sk, cts[0])
    out.append({"op": "bfv_flow", "preset": "bfv-128-simd", "n": n, "q": q, "t": t, "base_log": bl, "level": lv,
                "seeds": {"sk": 41, "a": 42, "e_pk": 43, "values": [44, 45], "u": [46, 47], "e1": [48, 49],
                          "e2": [50, 51], "rlk_a": [52, 53], "rlk_e": [54, 55]},
                "sha_pk": sha(pk), "sha_ct0": sha(cts[0]), "sha_ct1": sha(cts[1]), "sha_ct3": sha(ct3),
                "sha_rlk": sha(rlk), "sha_relin": sha(rel), "sha_dec": sha(dv), "max_noise": mx,
                "sha_dec_ct0": sha(dv0), "max_noise_ct0": mx0})
    return out


ENGINE_SEED = bytes(range(32))  # createEngine(params, { seed }) of tests/js/engine_test.js


def _seed_words(b):
    return [int(x) for x in np.frombuffer(b, dtype=np.uint64)]


def _identity_test_poly(n, q, t):
    """init_default_test_poly (bootstrap_engine.cpp:57-77)"""
    delta = q // t
    return np.array([((((i * t) // (2 * n)) * delta) & ((1 << 64) - 1)) % q for i in range(n)], dtype=np.uint64)


def fhe_engine():
    """The FHEEngine surface flows of tests/js/engine_test.js, regenerated with
    the oracle's restatement of the seeded ChaCha20 sampler (oracle_sample)
    and the key / encryption / ciphertext restatements.  Stream ids follow
    lib/engine.js: a counter from 1, secret key 1 stream, public key 2,
    encrypt 3, eval key 2 per level, bootstrap key 1 + 2 + 2."""
    seed = _seed_words(ENGINE_SEED)
    out = []
    # bfv-128-simd: keys -> encryptPacked x2 -> multiply -> generateEvalKey -> relinearize -> decrypt
    n, q, t, bl, lv, std = 8192, 1152921504606584833, 65537, 60, 2, 3.2
    o = oracle.NTT(n, q)
    sk = oracle.sample(1, seed, 1, q, n)
    pk = o.public_key_generate(sk, seed, 2, std)
    vals = [oracle.splitmix_fill(44 + j, t, n) for j in range(2)]
    cts = []
    for j in range(2):
        s0 = 4 + 3 * j
        cts.append(o.encrypt(t, pk, vals[j], oracle.sample(1, seed, s0, q, n),
                             oracle.sample(2, seed, s0 + 1, q, n, std), oracle.sample(2, seed, s0 + 2, q, n, std)))
    ct3 = o.ct_multiply(cts[0], cts[1])
    rlk = o.eval_key_generate(sk, bl, lv, seed, 10, std)
    rel = o.relinearize(bl, lv, ct3, rlk)
    dv, _, mx = o.decrypt(t, sk, rel)
    dv0, _, mx0 = o.decrypt(t, sk, cts[0])
    added = oracle.poly_add(q, cts[0].ravel(), cts[1].ravel()).reshape(2, n)
    dva, _, mxa = o.decrypt(t, sk, added)
    out.append({"op": "engine_flow", "preset": "bfv-128-simd", "n": n, "q": q, "t": t, "base_log": bl, "level": lv,
                "values_seeds": [44, 45], "sha_ct0": sha(cts[0]), "sha_ct1": sha(cts[1]), "sha_ct3": sha(ct3),
                "sha_relin": sha(rel), "sha_dec": sha(dv), "max_noise": mx, "sha_dec_ct0": sha(dv0),
                "max_noise_ct0": mx0, "sha_add": sha(added), "sha_dec_add": sha(dva), "max_noise_add": mxa})
    # tfhe-128-balanced: keys -> generateBootstrapKey -> encryptValue -> bootstrap -> decrypt (LWE)
    n, q, t, bl, lv, dim, std = 2048, 1125899906826241, 8, 15, 2, 830, 2.9e-11
    o = oracle.NTT(n, q)
    sk = oracle.sample(1, seed, 1, q, n)
    pk = o.public_key_generate(sk, seed, 2, std)
    lwe_sk = oracle.sample(3, seed, 4, q, dim).astype(np.int64)
    bsk = o.ggsw_encrypt(1, bl, lv, lwe_sk, sk, seed, 5, std)
    ksk_a, ksk_b = oracle.ksk_generate(q, bl, lv, sk, lwe_sk, seed, 7, std)
    value = 3
    slots = np.zeros(n, dtype=np.uint64)
    slots[0] = value
    ct = o.encrypt(t, pk, slots, oracle.sample(1, seed, 9, q, n), oracle.sample(2, seed, 10, q, n, std),
                   oracle.sample(2, seed, 11, q, n, std))
    glwe = np.stack([ct[1], ct[0]])
    ea, eb = oracle.sample_extract(q, glwe)
    la, lb = oracle.key_switch(q, bl, lv, ksk_a, ksk_b, ea, eb)
    oa, ob = o.bootstrap(1, bl, lv, la, lb, q, bsk, _identity_test_poly(n, q, t), bl, lv, ksk_a, ksk_b)
    lwe_out = np.concatenate([oa, np.array([ob], dtype=np.uint64)])
    v, ph = oracle.lwe_decrypt(q, t, lwe_sk, oa, ob)
    out.append({"op": "tfhe_flow", "preset": "tfhe-128-balanced", "n": n, "q": q, "t": t, "dim": dim, "value": value,
                "sha_bsk": sha(bsk), "sha_ksk_a": sha(ksk_a), "sha_ksk_b": sha(ksk_b), "sha_ct": sha(ct),
                "sha_keyswitched": sha(np.concatenate([la, np.array([lb], dtype=np.uint64)])),
                "sha_bootstrapped": sha(lwe_out), "decrypted": v, "phase": ph})
    return out


GENERATORS = {
    "reference_kat.json": reference_kat, "ntt_small.json": ntt_small, "ntt_large.json": ntt_large,
    "modmul.json": modmul, "multi_limb.json": multi_limb, "extprod.json": extprod, "negacyclic.json": negacyclic,
    "cipher.json": cipher, "engine.json": engine, "fhe_engine.json": fhe_engine,
}

if __name__ == "__main__":
    # python make_golden.py [file.json ...]   (default: all)
    for name in sys.argv[1:] or list(GENERATORS):
        dump(name, GENERATORS[name]())
