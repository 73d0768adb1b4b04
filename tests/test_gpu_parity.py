"""GPU parity: the HIP kernels (through the C-ABI) vs the CPU oracle and the
committed golden fixtures.  Bit-exact throughout (integer arithmetic).

Run on an MI355X with ``pytest -m gpu``.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import pyref

pytestmark = pytest.mark.gpu

P27 = 132120577
P62 = 4611686018326724609


@pytest.fixture(scope="module")
def fg():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import fhe_gpu

    return fhe_gpu


def load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


def U(x):
    return np.array(x, dtype=np.uint64)


def L(a):
    return [int(v) for v in np.asarray(a).ravel()]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


def _ctx_ok(n):
    return 4 <= n <= 16384


# ------------------------------------------------------------ golden vectors
def test_golden_small(fg, golden_dir):
    for c in load(golden_dir, "ntt_small.json"):
        n, q = c["n"], c["q"]
        r = fg.PolynomialRing(n, q)
        assert r.primitive_root == c["psi"]
        x, y, w = U(c["x"]), U(c["y"]), U(c["w"])
        assert L(r.forward_ntt(x)) == c["forward"], (n, q)
        assert L(r.inverse_ntt(x)) == c["inverse"], (n, q)
        assert L(r.multiply(x, y)) == c["polymul"], (n, q)
        assert L(r.forward_ntt_mul(x, w)) == c["fwd_mul"], (n, q)


def test_golden_large(fg, golden_dir):
    for c in load(golden_dir, "ntt_large.json"):
        n, q, b = c["n"], c["q"], c["batch"]
        r = fg.PolynomialRing(n, q)
        x = oracle.splitmix_fill(c["seed_x"], q, b * n).reshape(b, n)
        y = oracle.splitmix_fill(c["seed_y"], q, b * n).reshape(b, n)
        assert _sha(r.forward_ntt(x)) == c["sha_forward"], (n, q)
        assert _sha(r.inverse_ntt(x)) == c["sha_inverse"], (n, q)
        assert _sha(r.multiply(x, y)) == c["sha_polymul"], (n, q)
        assert _sha(r.forward_ntt_mul(x, y)) == c["sha_fwd_mul"], (n, q)


# ------------------------------------------------------------ oracle sweeps
CONFIGS = [(4, 17), (8, 17), (16, 97), (32, 193), (64, 257), (128, 769), (256, 7681), (512, 12289),
           (1024, P27), (1024, P62), (2048, 40961), (4096, P27), (4096, P62), (8192, P27), (8192, P62),
           (16384, P27), (16384, P62), (1024, 1152921504606584833), (2048, 1073479681),
           (32768, P27), (32768, P62), (65536, P27), (65536, P62),
           # q in (2^27, 2^30): 32-bit lanes without the lazy forward (the
           # 32-coefficient polymul's non-lazy instantiation at N=8192/16384)
           (8192, 1073643521), (16384, 1073643521),
           # the paired-transform polymul at N = 4096 / 8192 (round 5): 32-bit
           # non-lazy, Q_60_1 (prime-specialised), a dense 62-bit prime (generic)
           (4096, 1073643521), (4096, 1152921504606584833), (8192, 1152921504606584833),
           (4096, 3458764513825652737), (8192, 3458764513825652737)]


@pytest.mark.parametrize("n,q", CONFIGS)
def test_transforms_vs_oracle(fg, n, q):
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    b = 3 if n > 16384 else 5 if n >= 4096 else 37  # ragged: not a multiple of polys-per-block
    x = oracle.splitmix_fill(n * 31 + 1, q, b * n).reshape(b, n)
    y = oracle.splitmix_fill(n * 31 + 2, q, b * n).reshape(b, n)
    assert (r.forward_ntt(x) == t.forward(x)).all()
    assert (r.inverse_ntt(x) == t.inverse(x)).all()
    assert (r.multiply(x, y) == t.polymul(x, y)).all()
    assert (r.forward_ntt_mul(x, y) == t.fwd_mul(x, y)).all()
    assert (r.pointwise_multiply(x, y) == oracle.pointwise(q, x.ravel(), y.ravel()).reshape(b, n)).all()


@pytest.mark.parametrize("n,q", [(64, 257), (1024, P27), (1024, P62), (16384, P27), (16384, P62), (32768, P27),
                                 (65536, P62)])
def test_non_canonical_inputs(fg, n, q):
    """Inputs are any u64 and behave as x mod q (the reference reduces in
    mod_add/mod_sub and the 128-bit %)."""
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    rng = np.random.default_rng(n)
    x = rng.integers(0, 2 ** 64 - 1, (3, n), dtype=np.uint64, endpoint=True)
    x[0, :4] = [0, q, 2 * q, 2 ** 64 - 1]
    y = rng.integers(0, 2 ** 64 - 1, (3, n), dtype=np.uint64, endpoint=True)
    assert (r.forward_ntt(x) == t.forward(x)).all()
    assert (r.inverse_ntt(x) == t.inverse(x)).all()
    assert (r.multiply(x, y) == t.polymul(x, y)).all()
    assert (r.forward_ntt_mul(x, y) == t.fwd_mul(x, y)).all()


@pytest.mark.parametrize("n,q", [(1024, P27), (16384, P62)])
def test_edge_values(fg, n, q):
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    z = np.zeros((2, n), np.uint64)
    m = np.full((2, n), q - 1, np.uint64)
    for v in (z, m):
        assert (r.forward_ntt(v) == t.forward(v)).all()
        assert (r.inverse_ntt(v) == t.inverse(v)).all()
        assert (r.multiply(v, m) == t.polymul(v, m)).all()
    # empty batch
    e = np.zeros((0, n), np.uint64)
    assert r.forward_ntt(e).shape == (0, n)


def test_in_place_and_device_tensors(fg):
    import torch

    n, q = 4096, P62
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    x = oracle.splitmix_fill(77, q, 8 * n).reshape(8, n)
    y = oracle.splitmix_fill(78, q, 8 * n).reshape(8, n)
    # host in place
    h = x.copy()
    r.forward_ntt(h, out=h)
    assert (h == t.forward(x)).all()
    # device: int64 tensors carry the u64 bits
    dx = torch.from_numpy(x.view(np.int64)).cuda()
    dy = torch.from_numpy(y.view(np.int64)).cuda()
    out = r.multiply(dx, dy)
    r.forward_ntt(dx, out=dx)  # in place on device
    torch.cuda.synchronize()
    assert (out.cpu().numpy().view(np.uint64) == t.polymul(x, y)).all()
    assert (dx.cpu().numpy().view(np.uint64) == t.forward(x)).all()


def test_round_trip_full_config_sizes(fg):
    """Size-independent properties at the BASELINE batch scale for N=4096
    (config C2: batch 1024) and a large N=16384 batch."""
    import torch

    for n, q, b in ((4096, P27, 1024), (4096, P62, 1024), (16384, P27, 2048), (16384, P62, 1024)):
        r = fg.PolynomialRing(n, q)
        g = torch.Generator(device="cuda").manual_seed(n + b)
        x = torch.randint(0, q, (b, n), device="cuda", dtype=torch.int64, generator=g)
        f = r.forward_ntt(x)
        back = r.inverse_ntt(f)
        assert torch.equal(back, x)
        # fwd(1) == all ones; multiply by the identity polynomial is identity
        one = torch.zeros_like(x)
        one[:, 0] = 1
        assert torch.equal(r.multiply(x, one), x)
        # linearity: fwd(x + y) == fwd(x) + fwd(y)
        y = torch.roll(x, 1, 0)
        assert torch.equal(r.forward_ntt(r.add(x, y)), r.add(f, r.forward_ntt(y)))
        # checksum of a few rows against the oracle
        rows = [0, b // 2, b - 1]
        t = oracle.NTT(n, q)
        xs = x[rows].cpu().numpy().view(np.uint64)
        assert (f[rows].cpu().numpy().view(np.uint64) == t.forward(xs)).all()


def test_full_c3_batch_rows_vs_oracle(fg):
    """The bench workload itself (BASELINE configs[2], C3): N=16384, batch
    65536, q=132120577 -- 8 GiB per operand, every launch over the whole
    batch.  First, middle and last rows of forward NTT + modmul and of the
    polymul (C4) bit-exact against the oracle; the rest by a property
    (fwd_mul against an independent forward NTT then pointwise product)."""
    import torch

    n, q, b = 16384, P27, 65536
    r = fg.PolynomialRing(n, q)
    g = torch.Generator(device="cuda").manual_seed(3)
    a = torch.randint(0, q, (b, n), device="cuda", dtype=torch.int64, generator=g)
    w = torch.randint(0, q, (b, n), device="cuda", dtype=torch.int64, generator=g)
    out = torch.empty_like(a)
    rows = [0, 1, b // 2, b - 2, b - 1]
    t = oracle.NTT(n, q)
    xa, xw = a[rows].cpu().numpy().view(np.uint64), w[rows].cpu().numpy().view(np.uint64)
    r.forward_ntt_mul(a, w, out=out)
    assert (out[rows].cpu().numpy().view(np.uint64) == t.fwd_mul(xa, xw)).all()
    # whole batch: fwd_mul == pointwise(fwd(a), w) (an independent kernel pair)
    f = r.forward_ntt(a[: b // 8])
    assert torch.equal(out[: b // 8], r.pointwise_multiply(f, w[: b // 8]))
    del f
    r.multiply(a, w, out=out)
    assert (out[rows].cpu().numpy().view(np.uint64) == t.polymul(xa, xw)).all()
    del a, w, out
    torch.cuda.empty_cache()


def test_large_degree_chunk_boundaries(fg):
    """N > 16384 runs as two passes over ctx-owned scratch in chunks of
    2^25 / N polynomials (ntt_big.hip): batches that straddle a chunk and
    the XCD grouping (multiples of 8) must not matter.  Rows around the
    boundary are checked against the oracle, the rest by properties."""
    import torch

    for n, q, b in ((65536, P27, 514), (32768, P62, 1027)):
        chunk = (1 << 25) // n
        r = fg.PolynomialRing(n, q)
        g = torch.Generator(device="cuda").manual_seed(n + b)
        x = torch.randint(0, q, (b, n), device="cuda", dtype=torch.int64, generator=g)
        y = torch.roll(x, 1, 0)
        f = r.forward_ntt(x)
        assert torch.equal(r.inverse_ntt(f), x)
        m = r.multiply(x, y)
        fm = r.forward_ntt_mul(x, y)
        rows = [0, 7, chunk - 1, chunk, chunk + 1, b - 1]
        t = oracle.NTT(n, q)
        xs = x[rows].cpu().numpy().view(np.uint64)
        ys = y[rows].cpu().numpy().view(np.uint64)
        assert (f[rows].cpu().numpy().view(np.uint64) == t.forward(xs)).all()
        assert (m[rows].cpu().numpy().view(np.uint64) == t.polymul(xs, ys)).all()
        assert (fm[rows].cpu().numpy().view(np.uint64) == t.fwd_mul(xs, ys)).all()
        # in place (out aliases an input) goes through the scratch as well
        r.multiply(x, y, out=x)
        assert torch.equal(x, m)


@pytest.mark.parametrize("n,q", [(32768, P27), (65536, P62)])
def test_large_degree_host_staging_chunks(fg, n, q, monkeypatch):
    """Host arrays at N > 16384 with an 8 MiB staging buffer (FHE_STAGE_MB,
    read per call): one call spans at least three staging chunks, each on
    its own stream, all sharing the context's big-N scratch (ordered by
    BigSync, fhe_internal.hpp).  Every row vs the oracle; a ciphertext
    multiply (2 polys in, 3 out per unit) across the chunks as well."""
    monkeypatch.setenv("FHE_STAGE_MB", "8")
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    per_chunk = (8 << 20) // (n * 8)
    b = 3 * per_chunk + 3  # ragged last chunk
    x = oracle.splitmix_fill(n + 41, q, b * n).reshape(b, n)
    y = oracle.splitmix_fill(n + 42, q, b * n).reshape(b, n)
    assert (r.forward_ntt(x) == t.forward(x)).all()
    assert (r.multiply(x, y) == t.polymul(x, y)).all()
    assert (r.forward_ntt_mul(x, y) == t.fwd_mul(x, y)).all()
    eng = fg.EncryptionEngine(r)
    nct = (8 << 20) // (3 * n * 8) * 3 + 1  # three chunks of whole ciphertexts and one more
    cx = x[: 2 * nct].reshape(nct, 2, n)
    cy = y[: 2 * nct].reshape(nct, 2, n)
    got = eng.multiply(cx, cy)
    for i in (0, nct // 2, nct - 1):
        assert (got[i] == t.ct_multiply(cx[i], cy[i])).all(), i


def test_large_degree_golden_ct_multiply(fg, golden_dir):
    """EncryptionEngine::multiply at the two-pass degrees vs the committed
    golden hash (two ciphertexts from the ntt_large seeds)."""
    for c in load(golden_dir, "ntt_large.json"):
        if "sha_ct_multiply" not in c:
            continue
        n, q = c["n"], c["q"]
        r = fg.PolynomialRing(n, q)
        x = oracle.splitmix_fill(c["seed_x"], q, 4 * n).reshape(2, 2, n)
        y = oracle.splitmix_fill(c["seed_y"], q, 4 * n).reshape(2, 2, n)
        assert _sha(fg.EncryptionEngine(r).multiply(x, y)) == c["sha_ct_multiply"], (n, q)


@pytest.mark.parametrize("n,q,bl,lv,k", [(32768, P62, 23, 1, 1), (65536, P27, 9, 3, 1), (1024, P62, 15, 2, 2),
                                         (256, 7681, 4, 3, 3), (32768, P27, 10, 2, 2)])
def test_external_product_composed_vs_oracle(fg, n, q, bl, lv, k):
    """Shapes the fused kernels do not take -- GLWE dimension k > 1 and
    N > 16384 -- run composed (decompose, batched forward, key MAC,
    inverse); bit-exact vs the oracle's reference loop."""
    b = 2
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    ggsw = oracle.splitmix_fill(n + k, q, (k + 1) * lv * (k + 1) * n).reshape((k + 1) * lv, k + 1, n)
    glwe = oracle.splitmix_fill(n + k + 1, q, b * (k + 1) * n).reshape(b, k + 1, n)
    glwe[0, 0, :3] = [2**64 - 1, q, q + 5]
    got = fg.ExternalProduct(r, ggsw, bl, lv, k)(glwe)
    for i in range(b):
        assert (got[i] == t.external_product(k, bl, lv, glwe[i], ggsw)).all(), i


def test_glwe_dimension_limits(fg):
    r = fg.PolynomialRing(1024, P62)
    with pytest.raises(fg.FHEError) as ei:
        fg.ExternalProduct(r, np.zeros((18, 18, 1024), np.uint64), 23, 1, k=17)  # k <= 16
    assert ei.value.code == -10


# ------------------------------------------------------------ ring elementwise
@pytest.mark.parametrize("n,q", [(8, 17), (1024, P27), (4096, P62)])
def test_ring_elementwise(fg, n, q):
    r = fg.PolynomialRing(n, q)
    rng = np.random.default_rng(q % 1000)
    a = rng.integers(0, 2 ** 64 - 1, (3, n), dtype=np.uint64, endpoint=True)
    b = rng.integers(0, 2 ** 64 - 1, (3, n), dtype=np.uint64, endpoint=True)
    a[0, : min(n, 4)] = [0, q - 1, q, 0][: min(n, 4)]
    assert (r.add(a, b) == oracle.poly_add(q, a.ravel(), b.ravel()).reshape(a.shape)).all()
    assert (r.subtract(a, b) == oracle.poly_sub(q, a.ravel(), b.ravel()).reshape(a.shape)).all()
    assert (r.negate(a) == oracle.poly_neg(q, a.ravel()).reshape(a.shape)).all()
    for s in (0, 1, 12345, 2 ** 64 - 1):
        assert (r.multiply_scalar(a, s) == oracle.poly_mul_scalar(q, a.ravel(), s).reshape(a.shape)).all()


def test_ring_q17_kat(fg, golden_dir):
    kat = load(golden_dir, "reference_kat.json")
    r = fg.PolynomialRing(8, 17)
    for a, b, c in kat["ring_q17"]["add"]:
        assert L(r.add(U(a), U(b))) == c
    for a, b, c in kat["ring_q17"]["sub"]:
        assert L(r.subtract(U(a), U(b))) == c


def test_round_trip_property_reference_configs(fg, golden_dir):  # test_ntt_processor.cpp:193-268
    kat = load(golden_dir, "reference_kat.json")
    for n, q, iters, seed in kat["round_trip_configs"]:
        r = fg.NTTProcessor(n, q)
        draws = oracle.testrandom_coeffs(seed, q, n * iters).reshape(iters, n)
        assert (r.inverse_ntt(r.forward_ntt(draws)) == draws).all()


# ------------------------------------------------------------ modmul kernels
def test_modmul_golden(fg, golden_dir):
    for c in load(golden_dir, "modmul.json"):
        assert L(fg.modmul_batch(c["q"], U(c["a"]), U(c["b"]))) == c["c"], c["q"]


def test_modmul_large_and_odd_sizes(fg):
    rng = np.random.default_rng(9)
    for q in (P27, P62, 2 ** 63 + 29, 1000):
        for count in (1, 3, 1 << 20, (1 << 20) + 7):
            a = rng.integers(0, 2 ** 64 - 1, count, dtype=np.uint64, endpoint=True)
            b = rng.integers(0, 2 ** 64 - 1, count, dtype=np.uint64, endpoint=True)
            assert (fg.modmul_batch(q, a, b) == oracle.modmul_batch(q, a, b)).all()


def test_multi_limb_golden(fg, golden_dir):
    for c in load(golden_dir, "multi_limb.json"):
        m = fg.MultiLimbModularArithmetic(c["q"])
        a, b = U(c["a"]).reshape(-1, 2), U(c["b"]).reshape(-1, 2)
        assert L(m.montgomery_mul_batch(a, b)) == c["c"]


def test_multi_limb_batch_vs_oracle(fg):
    rng = np.random.default_rng(4)
    for qm in ([P62, 1], [0xFFFFFFFFFFFFFFC5, 0xFFFFFFFFFFFFFFFF]):
        m = fg.MultiLimbModularArithmetic(qm)
        a = rng.integers(0, 2 ** 64 - 1, (16384 * 64, 2), dtype=np.uint64, endpoint=True)
        b = rng.integers(0, 2 ** 64 - 1, (16384 * 64, 2), dtype=np.uint64, endpoint=True)
        a[:, 1] %= np.uint64(max(qm[1], 1))
        b[:, 1] %= np.uint64(max(qm[1], 1))
        assert (m.montgomery_mul_batch(a, b) == oracle.ml_montmul_batch(qm, a, b)).all()


# ------------------------------------------------------------ external product
def test_external_product_golden(fg, golden_dir):
    for c in load(golden_dir, "extprod.json"):
        n, q, k, lv, bl = c["n"], c["q"], c["k"], c["level"], c["base_log"]
        r = fg.PolynomialRing(n, q)
        ggsw = U(c["ggsw"]).reshape((k + 1) * lv, k + 1, n)
        ep = fg.ExternalProduct(r, ggsw, bl, lv, k)
        glwe = U(c["glwe"]).reshape(1, k + 1, n)
        assert L(ep(glwe)) == c["out"], (n, q, bl, lv)


@pytest.mark.parametrize("q,bl,lv", [(P62, 23, 1), (P62, 15, 2), (P27, 9, 3)])
def test_external_product_16384(fg, q, bl, lv):
    n, k, b = 16384, 1, 3
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    ggsw = oracle.splitmix_fill(bl * 7 + lv, q, (k + 1) * lv * (k + 1) * n).reshape((k + 1) * lv, k + 1, n)
    glwe = oracle.splitmix_fill(bl * 11 + lv, q, b * (k + 1) * n).reshape(b, k + 1, n)
    ep = fg.ExternalProduct(r, ggsw, bl, lv, k)
    got = ep(glwe)
    for i in range(b):
        assert (got[i] == t.external_product(k, bl, lv, glwe[i], ggsw)).all(), i


@pytest.mark.parametrize("n,q,bl", [(4096, P62, 20), (8192, P62, 23), (8192, 1152921504606584833, 30),
                                     (16384, P62, 1)])
def test_external_product_single_level_vs_oracle(fg, n, q, bl):
    """Level 1 with 64-bit words runs the paired-transform kernel
    (k_extprod2): digit(c0) and digit(c1) transformed in lockstep, key MAC in
    place, both inverses in lockstep.  Raw (non-canonical) GLWE words and
    the largest / smallest digit bases included."""
    k, b, lv = 1, 4, 1
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    ggsw = oracle.splitmix_fill(n + bl, q, (k + 1) * lv * (k + 1) * n).reshape((k + 1) * lv, k + 1, n)
    glwe = oracle.splitmix_fill(n * 3 + bl, q, b * (k + 1) * n).reshape(b, k + 1, n)
    glwe[1, 0, :4] = [2**64 - 1, q, q - 1, 0]
    got = fg.ExternalProduct(r, ggsw, bl, lv, k)(glwe)
    for i in range(b):
        assert (got[i] == t.external_product(k, bl, lv, glwe[i], ggsw)).all(), i


def test_external_product_single_level_negacyclic_is_linear(fg):
    """Negacyclic mode (no oracle restatement): ExtProd(G, c) computed by the
    fused kernel equals the composition of the library's own independent
    kernels -- decompose, forward, pointwise by the prepared key rows, sum,
    inverse."""
    import torch

    n, q, bl, lv, k = 8192, P62, 23, 1, 1
    r = fg.PolynomialRing(n, q, mode="negacyclic")
    ggsw = oracle.splitmix_fill(5, q, 2 * 2 * n).reshape(2, 2, n)
    glwe = oracle.splitmix_fill(6, q, 2 * 2 * n).reshape(2, 2, n)
    got = fg.ExternalProduct(r, ggsw, bl, lv, k)(glwe)
    for i in range(2):
        digits = [fg.decompose_polynomial(r, glwe[i, j:j + 1], bl, lv)[0] for j in range(2)]
        for j in range(2):
            acc = np.zeros((1, n), np.uint64)
            for row in range(2):
                f = r.forward_ntt(np.ascontiguousarray(digits[row].reshape(1, n)))
                g = r.forward_ntt(np.ascontiguousarray(ggsw[row, j].reshape(1, n)))
                acc = r.add(acc, r.pointwise_multiply(f, g))
            assert (got[i, j] == r.inverse_ntt(acc)[0]).all(), (i, j)


def test_decompose(fg):
    n, q = 1024, P62
    r = fg.PolynomialRing(n, q)
    x = oracle.splitmix_fill(5, q, 3 * n).reshape(3, n)
    from fhe_gpu import decompose_polynomial

    got = decompose_polynomial(r, x, 15, 2)
    for i in range(3):
        assert (got[i] == oracle.decompose(q, x[i], 15, 2)).all()


# ------------------------------------------------------------ negacyclic mode
def test_negacyclic_mode_is_ring_product(fg, golden_dir):
    for c in load(golden_dir, "negacyclic.json"):
        n, q = c["n"], c["q"]
        r = fg.PolynomialRing(n, q, mode="negacyclic")
        assert L(r.forward_ntt(U(c["x"]))) == c["forward"]
        assert L(r.multiply(U(c["x"]), U(c["y"]))) == c["product"]
    # larger: schoolbook via the oracle's exact integer arithmetic is too slow,
    # check the convolution identity x * X == shift with sign
    for n, q in ((4096, P62), (8192, P27), (16384, P27), (16384, 1073643521), (32768, P62), (65536, P27)):
        r = fg.PolynomialRing(n, q, mode="negacyclic")
        x = oracle.splitmix_fill(3, q, n).reshape(1, n)
        X = np.zeros((1, n), np.uint64)
        X[0, 1] = 1
        expect = np.roll(x, 1, axis=1)
        expect[0, 0] = (q - int(x[0, -1])) % q
        assert (r.multiply(x, X) == expect).all()
        assert (r.inverse_ntt(r.forward_ntt(x)) == x).all()


# ------------------------------------------------------------ sparse primes
def rnd(seed, q, *shape):
    return oracle.splitmix_fill(seed, q, int(np.prod(shape))).reshape(shape)


Q60 = 1152921504606584833        # Q_60_1 = 2^60 - 2^18 + 1
Q_DENSE62 = 3458764513825652737  # 3 2^60 + 0x4e0001: 62 bits, not 2^k - d with d < 2^32


@pytest.mark.parametrize("q", [P62, Q60])
def test_sparse_prime_kernels_match_generic(fg, monkeypatch, q):
    """The reference's 64-bit primes take prime-specialised kernels at
    N = 16384 (fhe_arith.hpp kSparsePrimes: h q mod 2^64 as (h << k) - h d);
    FHE_SPARSE=0 at context creation keeps the generic ones.  Both must agree
    word for word on fwd, fwd*w, inverse, polymul and the external product
    (levels 1 and 2), and rows match the oracle."""
    n, b = 16384, 6
    x, y = rnd(501, q, b, n), rnd(502, q, b, n)
    x[0, :3] = [2**64 - 1, q, q + 1]  # raw words
    glwe = rnd(503, q, b, 2, n)
    out = {}
    for sp in ("0", "1"):
        monkeypatch.setenv("FHE_SPARSE", sp)
        r = fg.PolynomialRing(n, q)
        res = [r.forward_ntt(x), r.forward_ntt_mul(x, y), r.inverse_ntt(x), r.multiply(x, y)]
        for bl, lv in ((23, 1), (15, 2)):
            ggsw = rnd(504 + lv, q, 2 * lv, 2, n)
            res.append(fg.ExternalProduct(r, ggsw, bl, lv)(glwe))
        out[sp] = res
    for a, c in zip(out["0"], out["1"]):
        assert (a == c).all()
    t = oracle.NTT(n, q)
    assert (out["1"][3][[0, b - 1]] == t.polymul(x[[0, b - 1]], y[[0, b - 1]])).all()
    assert (out["1"][1][[0, b - 1]] == t.fwd_mul(x[[0, b - 1]], y[[0, b - 1]])).all()


def test_dense_62bit_prime_vs_oracle(fg):
    """A 62-bit NTT prime far from any power of two: the generic 64-bit
    kernels at N = 16384 (never the sparse ones) vs the oracle."""
    n, q, b = 16384, Q_DENSE62, 3
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    x, y = rnd(511, q, b, n), rnd(512, q, b, n)
    assert (r.forward_ntt(x) == t.forward(x)).all()
    assert (r.forward_ntt_mul(x, y) == t.fwd_mul(x, y)).all()
    assert (r.multiply(x, y) == t.polymul(x, y)).all()
    assert (r.inverse_ntt(x) == t.inverse(x)).all()


@pytest.mark.parametrize("q", [P62, Q_DENSE62])
def test_unit_twiddle_kernels_match_generic(fg, monkeypatch, q):
    """Compat-mode contexts take unit-twiddle kernels for the 64-bit polymul
    (ntt_core.hpp gk_compat: pass-0 butterflies of group 0 skip the Shoup
    product); FHE_UNIT_TW=0 at context creation keeps the generic ones.  Both
    agree word for word (raw input words included), negacyclic contexts never
    take them, and rows match the oracle."""
    n, b = 16384, 4
    x, y = rnd(521, q, b, n), rnd(522, q, b, n)
    x[0, :3] = [2**64 - 1, q, q + 1]
    out = {}
    for u in ("0", "1"):
        monkeypatch.setenv("FHE_UNIT_TW", u)
        out[u] = fg.PolynomialRing(n, q).multiply(x, y)
    assert (out["0"] == out["1"]).all()
    t = oracle.NTT(n, q)
    assert (out["1"][[0, b - 1]] == t.polymul(x[[0, b - 1]], y[[0, b - 1]])).all()
    # negacyclic context (no unit twiddle): x * X is the signed shift
    monkeypatch.setenv("FHE_UNIT_TW", "1")
    X = np.zeros((1, n), np.uint64)
    X[0, 1] = 1
    expect = np.roll(x[1:2], 1, axis=1)
    expect[0, 0] = (q - int(x[1, -1])) % q
    assert (fg.PolynomialRing(n, q, mode="negacyclic").multiply(x[1:2], X) == expect).all()
