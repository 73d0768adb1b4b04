"""GPU parity of the ciphertext-level ops:
EncryptionEngine::multiply / relinearize / multiply_relin and the
BootstrapEngine pieces (cmux, monomial rotation, blind_rotate,
sample_extract, key_switch) -- HIP kernels through the C-ABI vs the CPU
oracle's restatement (oracle/ref_cpu.c), bit-exact.

Run on an MI355X with ``pytest -m gpu``.
"""
import numpy as np
import pytest

import oracle

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


def rnd(seed, q, *shape):
    return oracle.splitmix_fill(seed, q, int(np.prod(shape))).reshape(shape)


# ------------------------------------------------------------ ciphertext multiply
# (4096, P27) takes the VGPR-slot layout (FHE_CTMUL_PREFER_REGS); 64-bit words
# at N = 4096 / 8192 / 16384 the paired kernel (round 5: also Q_60_1 at 8192)
# (8192 / 16384, 1073643521): the non-lazy 32-bit paired kernel (q in (2^27, 2^30))
@pytest.mark.parametrize("n,q", [(4, 17), (16, 97), (256, 7681), (1024, P27), (2048, P62), (4096, P27),
                                 (4096, P62), (8192, P27), (8192, P62), (16384, P27), (16384, P62),
                                 (8192, 1073643521), (16384, 1073643521), (8192, 1152921504606584833)])
def test_ct_multiply_vs_oracle(fg, n, q):
    b = 3 if n >= 8192 else 5
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r)
    x = rnd(n + 1, q, b, 2, n)
    y = rnd(n + 2, q, b, 2, n)
    got = eng.multiply(x, y)
    assert got.shape == (b, 3, n)
    for i in range(b):
        assert (got[i] == t.ct_multiply(x[i], y[i])).all(), i
    got_ntt = eng.multiply(x, y, is_ntt=True)
    for i in range(b):
        assert (got_ntt[i] == t.ct_multiply(x[i], y[i], is_ntt=True)).all(), i


def test_ct_multiply_large_degree_and_raw_inputs(fg):
    # n > 16384 takes the composed path; inputs are arbitrary u64 (x mod q)
    for n, q in ((32768, P27), (1024, P62)):
        r = fg.PolynomialRing(n, q)
        t = oracle.NTT(n, q)
        x = oracle.splitmix_fill(7, 0, 2 * 2 * n).reshape(2, 2, n)  # q = 0: raw 64-bit words
        y = rnd(8, q, 2, 2, n)
        got = fg.EncryptionEngine(r).multiply(x, y)
        for i in range(2):
            assert (got[i] == t.ct_multiply(x[i], y[i])).all(), (n, q, i)


def test_ct_multiply_negacyclic_is_ring_tensor(fg):
    n, q = 4096, P27
    r = fg.PolynomialRing(n, q, mode="negacyclic")
    x = rnd(11, q, 2, 2, n)
    y = rnd(12, q, 2, 2, n)
    got = fg.EncryptionEngine(r).multiply(x, y)
    for i in range(2):
        c0 = r.multiply(x[i, 0], y[i, 0])
        c1 = r.add(r.multiply(x[i, 0], y[i, 1]), r.multiply(x[i, 1], y[i, 0]))
        c2 = r.multiply(x[i, 1], y[i, 1])
        assert (got[i, 0] == c0).all() and (got[i, 1] == c1).all() and (got[i, 2] == c2).all()


@pytest.mark.parametrize("n,q,bl,lv", [(64, 257, 2, 4), (1024, P27, 4, 7), (1024, P27, 9, 3), (4096, P62, 16, 4),
                                       (8192, P62, 12, 5), (16384, P27, 4, 7), (16384, P62, 20, 3),
                                       (256, 7681, 63, 1),
                                       # L B <= 32 with a lazy and a non-lazy context, L B > 32, N = 16384
                                       (16384, P27, 8, 4), (16384, 1073643521, 4, 7), (16384, P27, 11, 3)])
def test_relinearize_vs_oracle(fg, n, q, bl, lv):
    b = 2 if n >= 16384 else 4
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    ct3 = rnd(n * 3 + bl, q, b, 3, n)
    ct3[0, 2, :5] = [0, q - 1, 2**63 + 5, 2**64 - 1, 1 << bl]  # raw c2 words decompose as given
    rlk = rnd(lv * 13 + n, q, lv, 2, n)
    ek = fg.EvaluationKey(r, rlk, bl)
    eng = fg.EncryptionEngine(r)
    got = eng.relinearize(ct3, ek)
    assert got.shape == (b, 2, n)
    for i in range(b):
        assert (got[i] == t.relinearize(bl, lv, ct3[i], rlk)).all(), i


def test_relinearize_without_keys_copies(fg):
    n, q = 256, 7681
    r = fg.PolynomialRing(n, q)
    ct3 = oracle.splitmix_fill(3, 0, 2 * 3 * n).reshape(2, 3, n)
    ek = fg.EvaluationKey(r, np.zeros((0, 2, n), np.uint64), 4)
    got = fg.EncryptionEngine(r).relinearize(ct3, ek)
    assert (got == ct3[:, :2]).all()


@pytest.mark.parametrize("n,q", [(1024, P27), (16384, P27)])
def test_multiply_relin_is_composition(fg, n, q):
    r = fg.PolynomialRing(n, q)
    eng = fg.EncryptionEngine(r)
    x, y = rnd(21, q, 2, 2, n), rnd(22, q, 2, 2, n)
    ek = fg.EvaluationKey(r, rnd(23, q, 7, 2, n), 4)
    assert (eng.multiply_relin(x, y, ek) == eng.relinearize(eng.multiply(x, y), ek)).all()


def test_ct_ops_device_tensors(fg):
    import torch

    n, q = 4096, P27
    r = fg.PolynomialRing(n, q)
    eng = fg.EncryptionEngine(r)
    x, y = rnd(31, q, 4, 2, n), rnd(32, q, 4, 2, n)
    rlk = rnd(33, q, 7, 2, n)
    host = eng.multiply_relin(x, y, fg.EvaluationKey(r, rlk, 4))
    dev = eng.multiply_relin(torch.from_numpy(x.view(np.int64)).cuda(), torch.from_numpy(y.view(np.int64)).cuda(),
                             fg.EvaluationKey(r, torch.from_numpy(rlk.view(np.int64)).cuda(), 4))
    torch.cuda.synchronize()
    assert (dev.cpu().numpy().view(np.uint64) == host).all()


# ------------------------------------------------------------ TFHE pieces
@pytest.mark.parametrize("n,q,bl,lv", [(256, 7681, 4, 3), (1024, P62, 23, 1), (1024, P62, 15, 2),
                                       (16384, P62, 15, 2)])
def test_cmux_vs_oracle(fg, n, q, bl, lv):
    k, b = 1, 2
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    ggsw = rnd(bl + n, q, (k + 1) * lv, k + 1, n)
    ct0, ct1 = rnd(41, q, b, k + 1, n), rnd(42, q, b, k + 1, n)
    got = be.cmux(be.prepare_ggsw(ggsw), ct0, ct1)
    for i in range(b):
        assert (got[i] == t.cmux(k, bl, lv, ggsw, ct0[i], ct1[i])).all(), i


def test_glwe_rotate_vs_oracle(fg):
    n, q, k = 1024, P27, 1
    r = fg.PolynomialRing(n, q)
    be = fg.BootstrapEngine(r, 4, 3, k)
    rots = [0, 1, -1, n, -n, 2 * n - 1, 5 * n + 3, -(2**31)]
    g = rnd(51, q, len(rots), k + 1, n)
    g[0, 0, :3] = [2**64 - 1, q, q + 1]  # raw words: copied, or (q - x) % q when negated
    got = be.multiply_glwe_by_monomial(g, rots)
    for i, rot in enumerate(rots):
        for j in range(k + 1):
            assert (got[i, j] == oracle.rotate(q, g[i, j], rot)).all(), (rot, j)


@pytest.mark.parametrize("n,q,bl,lv,dim", [(256, 7681, 4, 3, 12), (1024, P27, 9, 3, 10), (1024, P62, 23, 1, 16)])
def test_blind_rotate_vs_oracle(fg, n, q, bl, lv, dim):
    k, b = 1, 3
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(61, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a = rnd(62, q, b, dim)
    lwe_a[0, 0] = 0          # rotation 0: the step is skipped
    lwe_a[0, 1] = q - 1      # rotation 2N: computed (not skipped)
    lwe_a[1, :] = 0          # whole ciphertext skipped
    lwe_b = rnd(63, q, b)
    acc0 = np.zeros((b, k + 1, n), np.uint64)
    acc0[:, k] = rnd(64, q, b, n)   # (0, test polynomial)
    acc0[2, k, :4] = [2**64 - 1, q, 0, 1]  # raw body words
    acc = acc0.copy()
    be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
    for i in range(b):
        exp = t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])
        assert (acc[i] == exp).all(), i


@pytest.mark.parametrize("n,q,bl,lv,mode,k", [(512, 12289, 4, 3, "compat", 1), (1024, P62, 23, 1, "compat", 1),
                                              (1024, P27, 9, 3, "negacyclic", 1), (1024, P62, 15, 2, "negacyclic", 1),
                                              (2048, P62, 23, 1, "compat", 1), (2048, 40961, 5, 2, "compat", 1),
                                              (512, 12289, 4, 3, "compat", 2), (1024, P62, 15, 2, "compat", 2),
                                              (1024, P27, 9, 3, "negacyclic", 2), (2048, 40961, 5, 2, "compat", 2),
                                              # the reference's larger TFHE presets (parameter_set.cpp:144-184):
                                              # tfhe-128-balanced (Q_50_1) and tfhe-256-secure (Q_60_1)
                                              (2048, 1125899906826241, 15, 2, "compat", 1),
                                              (4096, 1152921504606584833, 10, 3, "compat", 1),
                                              (4096, 40961, 5, 2, "compat", 1), (4096, P27, 9, 3, "negacyclic", 1),
                                              # GLWE dimension 3 / 4 (K1 = 4 / 5 accumulators in LDS)
                                              (512, 12289, 4, 3, "compat", 3), (1024, P62, 15, 2, "compat", 3),
                                              (2048, 40961, 5, 2, "compat", 3), (512, 12289, 4, 3, "compat", 4),
                                              (1024, P62, 23, 1, "compat", 4)])
def test_blind_rotate_single_launch_matches_step_launches(fg, monkeypatch, n, q, bl, lv, mode, k):
    """Small batches take the single-launch blind rotation (ntt_br.hip,
    accumulators in LDS for the whole loop; k = 1 on two CUs per ciphertext
    (k_br_pair) or, with FHE_BR_PAIR=0, on one (k_br_persist); k = 2 with K1 = 3
    accumulators); FHE_BR_PERSIST_MAX=0 forces the per-step launches (k = 1)
    or the composed steps (k = 2).  All bit-exact with each other, and rows vs
    the oracle (compat mode)."""
    b, dim = 5, 24
    r = fg.PolynomialRing(n, q, mode=mode)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(71 + n, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a = rnd(72, q, b, dim)
    lwe_a[0, :3] = [0, q - 1, 1]   # skipped step, rotation 2N, tiny rotation
    lwe_a[1, :] = 0                 # all steps skipped
    lwe_b = rnd(73, q, b)
    acc0 = rnd(74, q, b, k + 1, n)  # both components non-zero
    acc0[2, 0, :3] = [2**64 - 1, q, q + 1]  # raw words
    got, reps = {}, {}
    # "40961": 2 lv CUs per ciphertext (k_br_multi) at lv = 2 / 3, the pair
    # at lv = 1; "40961p": the pair (FHE_BR_MULTI=0)
    for pmax, pair, multi in (("4096", "1", "1"), ("4096", "1", "0"), ("4096", "0", "1"), ("0", "1", "1")):
        monkeypatch.setenv("FHE_BR_PERSIST_MAX", pmax)
        monkeypatch.setenv("FHE_BR_PAIR", pair)
        monkeypatch.setenv("FHE_BR_MULTI", multi)
        key = pmax + pair + ("" if multi == "1" else "p")
        before = be.repair_count() if k == 1 else 0
        acc = acc0.copy()
        be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
        got[key] = acc
        reps[key] = (be.repair_count() if k == 1 else 0) - before
    monkeypatch.delenv("FHE_BR_MULTI")
    if mode == "compat" and not all((got[x] == got["01"]).all() for x in ("40961", "40961p", "40960")):
        # name the path that disagrees with the oracle (and any repairs it took)
        t = oracle.NTT(n, q)
        exp = [t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i]) for i in range(b)]
        bad = {p: [i for i in range(b) if not (v[i] == exp[i]).all()] for p, v in got.items()}
        raise AssertionError(f"paths disagree: rows differing from the oracle per path {bad}, repairs {reps}")
    assert (got["40961"] == got["01"]).all(), reps
    assert (got["40961p"] == got["01"]).all(), reps
    assert (got["40960"] == got["01"]).all(), reps
    got["4096"] = got["40961"]
    if mode == "compat":
        t = oracle.NTT(n, q)
        for i in (0, 1, 2):
            exp = t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])
            assert (got["4096"][i] == exp).all(), i


Q50 = 1125899906826241      # Q_50_1 (parameter_set.cpp), tfhe-128-balanced
Q60 = 1152921504606584833    # Q_60_1, tfhe-256-secure


@pytest.mark.parametrize("coop,multi", [("1", "0"), ("0", "0"), ("0", "1")])
@pytest.mark.parametrize("n,q,bl,lv", [(1024, P62, 23, 1), (2048, Q50, 15, 2), (4096, Q60, 10, 3),
                                       (2048, 40961, 5, 2)])  # 32-bit words: the u32 repair kernel
def test_br_pair_timeout_takes_repair_pass(fg, monkeypatch, n, q, bl, lv, coop, multi):
    """k_br_pair (and, with multi at lv = 2 / 3, k_br_multi) with a zero poll
    budget: every workgroup that reaches a hand-off before its partners gives
    its ciphertext up (ABORT flag, fail word, nothing stored), and the repair
    pass recomputes those from the saved input -- the result still equals the
    one-CU kernel and the oracle, and the repairs are counted."""
    k, b, dim = 1, 6, 20
    r = fg.PolynomialRing(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(171 + n, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a, lwe_b = rnd(172, q, b, dim), rnd(173, q, b)
    lwe_a[1, :] = 0                 # every step skipped: no hand-off at all
    acc0 = rnd(174, q, b, k + 1, n)
    acc0[2, 0, :3] = [2**64 - 1, q, q + 1]  # raw words
    monkeypatch.setenv("FHE_BR_PAIR", "0")
    ref = acc0.copy()
    be.blind_rotate(ref, lwe_a, lwe_b, bsk_ntt)
    monkeypatch.setenv("FHE_BR_PAIR", "1")
    monkeypatch.setenv("FHE_BR_PAIR_COOP", coop)
    monkeypatch.setenv("FHE_BR_MULTI", multi)
    monkeypatch.setenv("FHE_BR_PAIR_TIMEOUT_US", "0")
    before = be.repair_count()
    acc = acc0.copy()
    be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
    assert (acc == ref).all()
    # the timeout path ran for exactly the ciphertexts that reach a hand-off:
    # all but row 1, whose steps are all skipped
    assert be.repair_count() - before == b - 1
    t = oracle.NTT(n, q)
    for i in (0, 2):
        assert (acc[i] == t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])).all(), i
    # with the default budget the same call needs no repair
    monkeypatch.delenv("FHE_BR_PAIR_TIMEOUT_US")
    before = be.repair_count()
    acc = acc0.copy()
    be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
    assert (acc == ref).all() and be.repair_count() == before


@pytest.mark.parametrize("b", [37, 64, 65, 100])
def test_br_pair_ragged_batches(fg, monkeypatch, b):
    """Batches that fill the multi-CU grid (b <= 64 at lv = 2: 32 workgroups
    per 8 ciphertexts, ct = (block / 32) * 8 + (block & 7)) or the two-CU grid
    (16 per 8, b > 64) only partly: the workgroups past the batch leave at
    once and every ciphertext equals the one-CU kernel's, rows 0 and b - 1 the
    oracle's (tfhe-128-balanced shape, compat mode: the unit-twiddle
    kernels)."""
    n, q, bl, lv, k, dim = 2048, Q50, 15, 2, 1, 6
    r = fg.PolynomialRing(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(191, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a, lwe_b = rnd(192, q, b, dim), rnd(193, q, b)
    acc0 = rnd(194, q, b, k + 1, n)
    got = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("FHE_BR_PAIR", pair)
        acc = acc0.copy()
        be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
        got[pair] = acc
    assert (got["1"] == got["0"]).all()
    t = oracle.NTT(n, q)
    for i in (0, b - 1):
        assert (got["1"][i] == t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])).all(), i


@pytest.mark.parametrize("serial,b", [("1", 128), ("0", 128), ("1", 40), ("0", 40), ("1", 64), ("0", 64)])
def test_br_pair_concurrent_contexts(fg, monkeypatch, serial, b):
    """Two contexts run two-CU blind rotations on two streams at once, with
    grids that together need twice the CUs (2 x 256 workgroups at batch
    128).  Serialised (the default) the launches queue behind each other;
    with FHE_BR_PAIR_SERIAL=0 they may interleave, and a pair that is not
    co-resident in time goes to the repair pass.  Either way both results
    are exact (vs the one-CU kernel, and rows vs the oracle).  At batch 40
    the same on six CUs per ciphertext (k_br_multi: 2 x 240 workgroups), at
    batch 64 in its dense form (two workgroups per CU: 2 x 384)."""
    import torch

    n, q, bl, lv, dim, k = 4096, Q60, 10, 3, 12, 1
    monkeypatch.setenv("FHE_BR_PAIR_SERIAL", serial)
    monkeypatch.setenv("FHE_BR_PAIR_TIMEOUT_US", "3000")
    rings = [fg.PolynomialRing(n, q) for _ in range(2)]
    bes = [fg.BootstrapEngine(r, bl, lv, k) for r in rings]
    bsk = rnd(181, q, dim, (k + 1) * lv, k + 1, n)

    def T(x):
        return torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()

    bsk_ntt = [T(be.prepare_ggsw(bsk)) for be in bes]
    lwe_a = [rnd(182 + i, q, b, dim) for i in range(2)]
    lwe_b = [rnd(184 + i, q, b) for i in range(2)]
    acc0 = [rnd(186 + i, q, b, k + 1, n) for i in range(2)]
    ins = [(T(lwe_a[i]), T(lwe_b[i])) for i in range(2)]
    accs = [T(acc0[i]) for i in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    for i in range(2):
        with torch.cuda.stream(streams[i]):
            bes[i].blind_rotate(accs[i], ins[i][0], ins[i][1], bsk_ntt[i])
    torch.cuda.synchronize()
    monkeypatch.setenv("FHE_BR_PAIR", "0")
    t = oracle.NTT(n, q)
    for i in range(2):
        ref = T(acc0[i])
        bes[i].blind_rotate(ref, ins[i][0], ins[i][1], bsk_ntt[i])
        torch.cuda.synchronize()
        got = accs[i].cpu().numpy().view(np.uint64)
        assert (got == ref.cpu().numpy().view(np.uint64)).all(), i
        exp = t.blind_rotate(k, bl, lv, lwe_a[i][b - 1], int(lwe_b[i][b - 1]), q, bsk, acc0[i][b - 1])
        assert (got[b - 1] == exp).all(), i


@pytest.mark.parametrize("n,q,bl,lv,k", [(1024, P62, 15, 2, 2), (32768, P62, 23, 1, 1)])
def test_cmux_composed_vs_oracle(fg, n, q, bl, lv, k):
    """CMux for k > 1 / N > 16384: ct0 + ExtProd(ct1 - ct0) composed."""
    b = 2
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    ggsw = rnd(n + 7, q, (k + 1) * lv, k + 1, n)
    g_ntt = be.prepare_ggsw(ggsw[None])[0]
    ct0, ct1 = rnd(n + 8, q, b, k + 1, n), rnd(n + 9, q, b, k + 1, n)
    got = be.cmux(g_ntt, ct0, ct1)
    for i in range(b):
        assert (got[i] == t.cmux(k, bl, lv, ggsw, ct0[i], ct1[i])).all(), i


@pytest.mark.parametrize("n,q,bl,lv,k,dim", [(512, 12289, 4, 3, 2, 6), (1024, P62, 15, 2, 3, 4),
                                              (32768, P62, 23, 1, 1, 2)])
def test_blind_rotate_composed_vs_oracle(fg, n, q, bl, lv, k, dim):
    """Blind rotation where no fused CMux exists (GLWE dimension k > 1,
    N > 16384): composed steps (X^r acc - acc, composed external product,
    + acc), bit-exact vs the oracle; skipped steps and a rotation of 2N."""
    b = 3
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(n + 31, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a = rnd(n + 32, q, b, dim)
    lwe_a[0, 0] = 0          # rotation 0: the step is skipped
    lwe_a[0, 1] = q - 1      # rotation 2N: computed
    lwe_a[1, :] = 0          # every step skipped
    lwe_b = rnd(n + 33, q, b)
    acc0 = rnd(n + 34, q, b, k + 1, n)
    acc = acc0.copy()
    be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
    for i in range(b):
        exp = t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])
        assert (acc[i] == exp).all(), i


def test_bootstrap_glwe_dim2_vs_oracle(fg):
    """bootstrap_with_test_poly at GLWE dimension k = 2 (composed blind
    rotation, then sample extract and key switch over k*N mask words)."""
    n, q, bl, lv, dim, k, b = 512, 12289, 4, 3, 5, 2, 2
    ks_bl, ks_lv, out_dim = 4, 3, 21
    r = fg.PolynomialRing(n, q)
    o = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(161, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a, lwe_b = rnd(162, q, b, dim), rnd(163, q, b)
    lwe_a[0, 0] = 0
    tp = be.create_lookup_table(lambda x: (3 * x + 1) % 8, 8, 8)
    ksk_a, ksk_b = rnd(164, q, k * n * ks_lv, out_dim), rnd(165, q, k * n * ks_lv)
    oa, ob = be.bootstrap(lwe_a, lwe_b, bsk_ntt, tp, ksk_a, ksk_b, ks_bl, ks_lv)
    for i in range(b):
        ea, eb = o.bootstrap(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, tp, ks_bl, ks_lv, ksk_a, ksk_b)
        assert (oa[i] == ea).all() and int(ob[i]) == eb, i


@pytest.mark.parametrize("n,q,bl,lv", [(32768, P27, 4, 7), (65536, P62, 20, 3)])
def test_relinearize_large_degree_vs_oracle(fg, n, q, bl, lv):
    """Relinearisation above 16384 runs composed (relinearize digits,
    batched transforms, key MAC, inverse, + c_j)."""
    b = 2
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    ct3 = rnd(n + bl, q, b, 3, n)
    ct3[0, 2, :3] = [2**64 - 1, q, 1 << bl]
    rlk = rnd(n + lv, q, lv, 2, n)
    eng = fg.EncryptionEngine(r)
    got = eng.relinearize(ct3, fg.EvaluationKey(r, rlk, bl))
    for i in range(b):
        assert (got[i] == t.relinearize(bl, lv, ct3[i], rlk)).all(), i
    # multiply_relin composes the large-degree ct multiply with it
    x, y = rnd(n + 1, q, b, 2, n), rnd(n + 2, q, b, 2, n)
    ek = fg.EvaluationKey(r, rlk, bl)
    assert (eng.multiply_relin(x, y, ek) == eng.relinearize(eng.multiply(x, y), ek)).all()


def test_sample_extract_vs_oracle(fg):
    n, q, k = 1024, P27, 1
    r = fg.PolynomialRing(n, q)
    be = fg.BootstrapEngine(r, 4, 3, k)
    g = rnd(71, q, 3, k + 1, n)
    g[1, 0, 5] = 2**64 - 1
    a, b = be.sample_extract(g)
    for i in range(3):
        ea, eb = oracle.sample_extract(q, g[i])
        assert (a[i] == ea).all() and int(b[i]) == eb


@pytest.mark.parametrize("q,bl,lv", [(P27, 4, 3), (P27, 2, 8), (P62, 7, 4), ((1 << 61) + 1, 10, 6)])
def test_key_switch_vs_oracle(fg, q, bl, lv):
    in_dim, out_dim, b = 96, 70, 37
    ksk_a = rnd(81, q, in_dim * lv, out_dim)
    ksk_b = rnd(82, q, in_dim * lv)
    lwe_a = rnd(83, q, b, in_dim)
    lwe_b = rnd(84, q, b)
    lwe_a[0, :] = 0                  # no digit: body returned raw
    lwe_b[0] = 2**64 - 3
    lwe_b[1] = 2**64 - 2             # b + q wraps in the first update
    lwe_a[2, :] = 1 << (bl * lv - 1) if bl * lv < 64 else 1
    oa, ob = fg.BootstrapEngine.key_switch(q, bl, lv, ksk_a, ksk_b, lwe_a, lwe_b)
    for i in range(b):
        ea, eb = oracle.key_switch(q, bl, lv, ksk_a, ksk_b, lwe_a[i], int(lwe_b[i]))
        assert (oa[i] == ea).all(), i
        assert int(ob[i]) == eb, i


@pytest.mark.parametrize("b", [1, 3, 17])
@pytest.mark.parametrize("q,bl,lv,in_dim,out_dim", [(Q60, 10, 3, 4096, 300), (Q50, 15, 2, 2048, 130),
                                                    (P27, 4, 7, 1024, 257)])
def test_key_switch_split_vs_oracle(fg, q, bl, lv, in_dim, out_dim, b):
    """The deferred-reduction key switch at the TFHE presets' shapes (k N
    input coefficients, (B, L) of the bootstrap key) for 1, 3 and 17
    ciphertexts: one, four or sixteen ciphertexts per workgroup, the (i, l)
    entries split over many workgroups with partial sums, the 96-bit
    accumulator reduced once -- bit-exact vs the reference's per-term
    remainder loop (oracle)."""
    ksk_a = rnd(301 + bl, q, in_dim * lv, out_dim)
    ksk_b = rnd(302 + bl, q, in_dim * lv)
    lwe_a = rnd(303 + b, q, b, in_dim)
    lwe_b = rnd(304 + b, q, b)
    lwe_a[0, : in_dim // 2] = 0          # half the digits zero (the reference's skip)
    if b > 1:
        lwe_a[1, :] = q - 1              # every digit at its maximum
    oa, ob = fg.BootstrapEngine.key_switch(q, bl, lv, ksk_a, ksk_b, lwe_a, lwe_b)
    for i in range(b):
        ea, eb = oracle.key_switch(q, bl, lv, ksk_a, ksk_b, lwe_a[i], int(lwe_b[i]))
        assert (oa[i] == ea).all(), i
        assert int(ob[i]) == eb, i


@pytest.mark.parametrize("name,n,q,bl,lv", [("tfhe-128-balanced", 2048, Q50, 15, 2),
                                             ("tfhe-256-secure", 4096, Q60, 10, 3)])
@pytest.mark.parametrize("b", [1, 5, 64])  # 64: tfhe-256 on the dense multi-CU form
def test_bootstrap_presets_vs_oracle(fg, name, n, q, bl, lv, b):
    """fhe_bootstrap_batch (bootstrap_with_test_poly, bootstrap_engine.cpp:
    684-711: blind rotation on two CUs per ciphertext, sample extract, key
    switch back to the LWE dimension with the bootstrap's (B, L) as
    generate_key_switch_key builds it, :367-420) at the reference presets'
    (N, q, B, L), LWE dimension reduced to 12, vs the oracle."""
    k, dim = 1, 12
    r = fg.PolynomialRing(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    o = oracle.NTT(n, q)
    bsk = rnd(601 + n, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a, lwe_b = rnd(602, q, b, dim), rnd(603, q, b)
    lwe_a[0, 0] = 0  # a skipped step
    tp = be.create_lookup_table(lambda x: (5 * x + 3) % 16, 16, 16)
    ksk_a, ksk_b = rnd(604, q, k * n * lv, dim), rnd(605, q, k * n * lv)
    oa, ob = be.bootstrap(lwe_a, lwe_b, bsk_ntt, tp, ksk_a, ksk_b, bl, lv)
    for i in range(b):
        ea, eb = o.bootstrap(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, tp, bl, lv, ksk_a, ksk_b)
        assert (oa[i] == ea).all() and int(ob[i]) == eb, (name, i)


def test_bootstrap_pipeline_device(fg):
    """blind_rotate -> sample_extract -> key_switch on device tensors equals
    the oracle's bootstrap_with_test_poly sequence (:676-708)."""
    import torch

    n, q, bl, lv, dim, k, b = 512, 12289, 4, 3, 8, 1, 4
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(91, q, dim, (k + 1) * lv, k + 1, n)
    lwe_a, lwe_b = rnd(92, q, b, dim), rnd(93, q, b)
    test_poly = rnd(94, q, n)
    ksk_a, ksk_b = rnd(95, q, k * n * 2, dim), rnd(96, q, k * n * 2)

    def T(x):
        return torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()

    acc = torch.zeros((b, k + 1, n), dtype=torch.int64, device="cuda")
    acc[:, k] = T(test_poly)
    be.blind_rotate(acc, T(lwe_a), T(lwe_b), be.prepare_ggsw(T(bsk)))
    ea, eb = be.sample_extract(acc)
    oa, ob = fg.BootstrapEngine.key_switch(q, 7, 2, T(ksk_a), T(ksk_b), ea, eb)
    torch.cuda.synchronize()
    oa, ob = oa.cpu().numpy().view(np.uint64), ob.cpu().numpy().view(np.uint64)
    for i in range(b):
        a0 = np.zeros((k + 1, n), np.uint64)
        a0[k] = test_poly
        accx = t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, a0)
        xa, xb = oracle.sample_extract(q, accx)
        ka, kb = oracle.key_switch(q, 7, 2, ksk_a, ksk_b, xa, xb)
        assert (oa[i] == ka).all() and int(ob[i]) == kb, i


def test_cipher_golden_gpu(fg, golden_dir):
    import json
    import os

    with open(os.path.join(golden_dir, "cipher.json")) as f:
        cases = json.load(f)
    for c in cases:
        n, q = c["n"], c["q"]
        r = fg.PolynomialRing(n, q)
        U = lambda x, *s: np.array(x, np.uint64).reshape(s)  # noqa: E731
        if c["op"] == "ct_multiply":
            got = fg.EncryptionEngine(r).multiply(U(c["ct1"], 1, 2, n), U(c["ct2"], 1, 2, n))
        elif c["op"] == "relinearize":
            ek = fg.EvaluationKey(r, U(c["rlk"], c["level"], 2, n), c["base_log"])
            got = fg.EncryptionEngine(r).relinearize(U(c["ct3"], 1, 3, n), ek)
        else:
            be = fg.BootstrapEngine(r, c["base_log"], c["level"], 1)
            got = U(c["acc"], 1, 2, n).copy()
            be.blind_rotate(got, U(c["lwe_a"], 1, c["dim"]), U([c["lwe_b"]], 1),
                            be.prepare_ggsw(U(c["bsk"], c["dim"], 2 * c["level"], 2, n)))
        assert [int(v) for v in got.ravel()] == c["out"], (c["op"], n, q)


# ------------------------------------------------------------ RNS ring
@pytest.mark.parametrize("n,moduli", [(4096, [P27, P62, 40961, 114689]), (16384, [P27, P62]), (32768, [P27])])
def test_rns_ring_vs_oracle(fg, n, moduli):
    b = 2
    r = fg.RNSPolynomialRing(n, moduli)
    x = np.stack([rnd(100 + i, q, b, n) for i, q in enumerate(moduli)])
    y = np.stack([rnd(200 + i, q, b, n) for i, q in enumerate(moduli)])
    fx, ix, pm = r.forward_ntt(x), r.inverse_ntt(x), r.multiply(x, y)
    pw, ad, sb = r.pointwise_multiply(x, y), r.add(x, y), r.subtract(x, y)
    for i, q in enumerate(moduli):
        t = oracle.NTT(n, q)
        assert (fx[i] == t.forward(x[i])).all(), q
        assert (ix[i] == t.inverse(x[i])).all(), q
        assert (pm[i] == t.polymul(x[i], y[i])).all(), q
        assert (pw[i] == oracle.pointwise(q, x[i].ravel(), y[i].ravel()).reshape(b, n)).all(), q
        assert (ad[i] == oracle.poly_add(q, x[i].ravel(), y[i].ravel()).reshape(b, n)).all(), q
        assert (sb[i] == oracle.poly_sub(q, x[i].ravel(), y[i].ravel()).reshape(b, n)).all(), q


def test_rns_ring_device_and_errors(fg):
    import torch

    n, moduli = 1024, [P27, P62]
    r = fg.RNSPolynomialRing(n, moduli)
    x = np.stack([rnd(300 + i, q, 3, n) for i, q in enumerate(moduli)])
    dev = r.forward_ntt(torch.from_numpy(x.view(np.int64)).cuda())
    torch.cuda.synchronize()
    assert (dev.cpu().numpy().view(np.uint64) == r.forward_ntt(x)).all()
    with pytest.raises(fg.FHEError, match="NTT-friendly"):
        fg.RNSPolynomialRing(n, [P27, 97])


@pytest.mark.parametrize("ring", ["u32", "bfv-128-simd", "u64"])
def test_rns_ring_single_launch(fg, monkeypatch, ring):
    """Device-resident calls on a ring whose limbs share one kernel shape run
    every op as ONE launch (grid.y = limb, per-limb constants); bit-exact
    with the per-limb launches (FHE_RNS_ONE_LAUNCH=0) and with the oracle."""
    import torch
    from fhe_gpu import params as P

    if ring == "u32":
        n, moduli = 4096, [P27, 40961, 114689]
    elif ring == "u64":  # 16384: the paired u64 polymul and the 32-per-thread forward
        n, moduli = 16384, [P62, 1152921504606584833]
    else:
        ps = P.create_parameter_set(ring)
        n, moduli = ps.poly_degree, list(ps.moduli)
    b = 2
    r = fg.RNSPolynomialRing(n, moduli)
    x = np.stack([rnd(700 + i, q, b, n) for i, q in enumerate(moduli)])
    y = np.stack([rnd(800 + i, q, b, n) for i, q in enumerate(moduli)])
    x[0, 0, :2] = [2**64 - 1, moduli[0]]  # raw words (x mod q)
    dx = torch.from_numpy(x.view(np.int64)).cuda()
    dy = torch.from_numpy(y.view(np.int64)).cuda()
    ops = {"fwd": lambda: r.forward_ntt(dx), "inv": lambda: r.inverse_ntt(dx), "mul": lambda: r.multiply(dx, dy),
           "pw": lambda: r.pointwise_multiply(dx, dy), "add": lambda: r.add(dx, dy), "sub": lambda: r.subtract(dx, dy)}
    got = {}
    for one in ("1", "0"):
        monkeypatch.setenv("FHE_RNS_ONE_LAUNCH", one)
        for k, f in ops.items():
            out = f()
            torch.cuda.synchronize()
            got[k + one] = out.cpu().numpy().view(np.uint64)
    for k in ops:
        assert (got[k + "1"] == got[k + "0"]).all(), k
    for i, q in enumerate(moduli[:2]):
        t = oracle.NTT(n, q)
        assert (got["fwd1"][i] == t.forward(x[i])).all(), q
        assert (got["mul1"][i] == t.polymul(x[i], y[i])).all(), q
        assert (got["pw1"][i] == oracle.pointwise(q, x[i].ravel(), y[i].ravel()).reshape(b, n)).all(), q
        assert (got["sub1"][i] == oracle.poly_sub(q, x[i].ravel(), y[i].ravel()).reshape(b, n)).all(), q


# ------------------------------------------------------------ reference parameter presets
def test_presets_bfv_rns_and_tfhe_balanced(fg):
    """bfv-128-simd's modulus chain as an RNS ring, and tfhe-128-balanced's
    (N, q, B, L) through CMux + blind rotation (parameter_set.cpp:139-224)."""
    from fhe_gpu import params as P

    bfv = P.create_parameter_set("bfv-128-simd")
    n = bfv.poly_degree
    r = fg.RNSPolynomialRing(n, bfv.moduli)
    x = np.stack([rnd(400 + i, q, 1, n) for i, q in enumerate(bfv.moduli)])
    y = np.stack([rnd(500 + i, q, 1, n) for i, q in enumerate(bfv.moduli)])
    pm = r.multiply(x, y)
    for i, q in enumerate(bfv.moduli):
        assert (pm[i] == oracle.NTT(n, q).polymul(x[i], y[i])).all(), q

    tb = P.create_parameter_set("tfhe-128-balanced")
    n, q, bl, lv, dim = tb.poly_degree, tb.moduli[0], tb.decomp_base_log, tb.decomp_level, 6
    ring = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(ring, bl, lv, 1)
    bsk = rnd(601, q, dim, 2 * lv, 2, n)
    lwe_a, lwe_b = rnd(602, q, 2, dim), rnd(603, q, 2)
    acc0 = np.zeros((2, 2, n), np.uint64)
    acc0[:, 1] = rnd(604, q, 2, n)
    acc = acc0.copy()
    be.blind_rotate(acc, lwe_a, lwe_b, be.prepare_ggsw(bsk))
    for i in range(2):
        assert (acc[i] == t.blind_rotate(1, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])).all(), i


def test_ciphertext_linear_ops_and_plain(fg):
    """EncryptionEngine::add / subtract / negate / multiply_scalar /
    multiply_plain (encryption.cpp:594-902) and relinearize of a degree-1
    ciphertext (a copy, :906-909)."""
    n, q, b = 1024, P27, 3
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r)
    x, y = rnd(701, q, b, 2, n), rnd(702, q, b, 2, n)
    x[0, 0, :3] = [2**64 - 1, q, 0]
    pt = rnd(703, q, n)
    add, sub, neg = eng.add(x, y), eng.subtract(x, y), eng.negate(x)
    sc, pm = eng.multiply_scalar(x, 2**63 + 12345), eng.multiply_plain(x, pt)
    for i in range(b):
        for j in range(2):
            assert (add[i, j] == oracle.poly_add(q, x[i, j], y[i, j])).all()
            assert (sub[i, j] == oracle.poly_sub(q, x[i, j], y[i, j])).all()
            assert (neg[i, j] == oracle.poly_neg(q, x[i, j])).all()
            assert (sc[i, j] == oracle.poly_mul_scalar(q, x[i, j], 2**63 + 12345)).all()
            assert (pm[i, j] == t.polymul(x[i, j], pt)).all()
    ek = fg.EvaluationKey(r, rnd(704, q, 3, 2, n), 4)
    assert (eng.relinearize(x, ek) == x).all()


@pytest.mark.parametrize("n,q,bl,lv", [(16384, P27, 4, 7), (8192, P27, 4, 7), (8192, P62, 13, 5), (4096, P62, 16, 4)])
def test_decryption_identity_negacyclic(fg, n, q, bl, lv):
    """Size-independent property at full degree: in the negacyclic ring,
    noise-free ciphertexts ct_i = (m_i - a_i s, a_i) satisfy
      c0 + c1 s + c2 s^2 = m1 m2              after multiply, and
      c0' + c1' s       = m1 m2              after relinearize,
    with rlk_l = (a_l, s^2 B^l - a_l s) (key_manager.cpp:296-324 without noise)."""
    b = 8
    r = fg.PolynomialRing(n, q, mode="negacyclic")
    eng = fg.EncryptionEngine(r)
    s = rnd(801, q, n)
    S = np.broadcast_to(s, (b, n)).copy()
    m1, m2, a1, a2 = rnd(802, q, b, n), rnd(803, q, b, n), rnd(804, q, b, n), rnd(805, q, b, n)
    ct1 = np.stack([r.subtract(m1, r.multiply(a1, S)), a1], axis=1)
    ct2 = np.stack([r.subtract(m2, r.multiply(a2, S)), a2], axis=1)
    ct3 = eng.multiply(ct1, ct2)
    s2 = r.multiply(S, S)
    dec3 = r.add(r.add(ct3[:, 0], r.multiply(ct3[:, 1], S)), r.multiply(ct3[:, 2], s2))
    want = r.multiply(m1, m2)
    assert (dec3 == want).all()
    al = rnd(806, q, lv, n)
    s2_1 = s2[:lv]
    scaled = np.stack([r.multiply_scalar(s2_1[l:l + 1], pow(1 << bl, l, q))[0] for l in range(lv)])
    bl_keys = r.subtract(scaled, r.multiply(al, np.broadcast_to(s, (lv, n)).copy()))
    rlk = np.stack([al, bl_keys], axis=1)
    out = eng.relinearize(ct3, fg.EvaluationKey(r, rlk, bl))
    dec2 = r.add(out[:, 0], r.multiply(out[:, 1], S))
    assert (dec2 == want).all()
