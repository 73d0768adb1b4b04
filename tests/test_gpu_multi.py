"""GPU tests of the multi-device context (fhe_ctx_create_multi, SURVEY.md
8(b)/(e)) and of the stream/graph plumbing: every result bit-exact vs the CPU
oracle.  A one-GPU box lists device 0 twice, which exercises the split,
the per-device host threads and the per-device routing of device buffers.

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


def _devices():
    import torch

    nd = torch.cuda.device_count()
    return [0, 0] if nd < 2 else list(range(min(nd, 4)))


@pytest.mark.parametrize("n,q,b", [(1024, P27, 7), (16384, P27, 5), (4096, P62, 9), (32768, P27, 3)])
def test_multi_device_host_batches(fg, n, q, b):
    devs = _devices()
    r = fg.PolynomialRing(n, q, devices=devs)
    t = oracle.NTT(n, q)
    x, y = rnd(11, q, b, n), rnd(12, q, b, n)
    assert (r.forward_ntt(x) == t.forward(x)).all()
    assert (r.inverse_ntt(x) == t.inverse(x)).all()
    assert (r.multiply(x, y) == t.polymul(x, y)).all()
    assert (r.forward_ntt_mul(x, y) == t.fwd_mul(x, y)).all()
    assert (r.add(x, y) == oracle.poly_add(q, x, y)).all()
    # fewer polynomials than devices: some ranges are empty
    assert (r.multiply(x[:1], y[:1]) == t.polymul(x[:1], y[:1])).all()


def test_multi_device_ciphertext_ops(fg):
    n, q, b = 2048, P62, 5
    r = fg.PolynomialRing(n, q, devices=_devices())
    t = oracle.NTT(n, q)
    eng = fg.EncryptionEngine(r)
    x, y = rnd(21, q, b, 2, n), rnd(22, q, b, 2, n)
    ct3 = eng.multiply(x, y)
    rlk = rnd(23, q, 3, 2, n)
    out = eng.relinearize(ct3, fg.EvaluationKey(r, rlk, 9))
    for i in range(b):
        assert (ct3[i] == t.ct_multiply(x[i], y[i])).all(), i
        assert (out[i] == t.relinearize(9, 3, ct3[i], rlk)).all(), i


def test_multi_device_blind_rotate(fg):
    n, q, bl, lv, dim, k, b = 256, 7681, 4, 3, 6, 1, 5
    r = fg.PolynomialRing(n, q, devices=_devices())
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(31, q, dim, (k + 1) * lv, k + 1, n)
    bsk_ntt = be.prepare_ggsw(bsk)
    lwe_a, lwe_b = rnd(32, q, b, dim), rnd(33, q, b)
    acc0 = np.zeros((b, k + 1, n), np.uint64)
    acc0[:, k] = rnd(34, q, b, n)
    acc = acc0.copy()
    be.blind_rotate(acc, lwe_a, lwe_b, bsk_ntt)
    for i in range(b):
        assert (acc[i] == t.blind_rotate(k, bl, lv, lwe_a[i], int(lwe_b[i]), q, bsk, acc0[i])).all(), i


def test_multi_device_device_buffers_run_where_they_live(fg):
    import torch

    n, q, b = 4096, P27, 6
    r = fg.PolynomialRing(n, q, devices=_devices())
    t = oracle.NTT(n, q)
    x, y = rnd(41, q, b, n), rnd(42, q, b, n)
    dx = torch.from_numpy(x.view(np.int64)).to("cuda:0")
    dy = torch.from_numpy(y.view(np.int64)).to("cuda:0")
    got = r.multiply(dx, dy)
    torch.cuda.synchronize()
    assert (got.cpu().numpy().view(np.uint64) == t.polymul(x, y)).all()


def test_multi_device_context_info_and_errors(fg):
    import ctypes as C

    devs = _devices()
    r = fg.PolynomialRing(1024, P27, devices=devs)
    nd = C.c_int()
    fg._check(fg.lib().fhe_ctx_device_count(r._h, C.byref(nd)))
    assert nd.value == len(devs)
    assert r.primitive_root == oracle.NTT(1024, P27).psi
    with pytest.raises(fg.FHEError) as e:
        fg.PolynomialRing(1024, P27, devices=[0, 999])
    assert e.value.code == -9
    with pytest.raises(fg.FHEError):
        fg.PolynomialRing(1024, P27, devices=[])


def test_blind_rotate_graph_replay_on_side_stream(fg):
    """device-resident blind rotation on a non-default stream is
    captured once as a hipGraph and replayed while buffers and shape stay the
    same.  Replays with identical buffers, then with changed lwe_a contents
    (same pointers: the graph must read them at replay time), then a
    different batch (re-capture) -- each bit-exact vs the oracle."""
    import torch

    n, q, bl, lv, dim, k = 256, 7681, 4, 3, 8, 1
    r = fg.PolynomialRing(n, q)
    t = oracle.NTT(n, q)
    be = fg.BootstrapEngine(r, bl, lv, k)
    bsk = rnd(51, q, dim, (k + 1) * lv, k + 1, n)
    side = torch.cuda.Stream()

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda:0")

    la = torch.empty((4, dim), dtype=torch.int64, device="cuda:0")
    lb = torch.empty((4,), dtype=torch.int64, device="cuda:0")
    acc = torch.empty((4, k + 1, n), dtype=torch.int64, device="cuda:0")
    with torch.cuda.stream(side):
        bsk_ntt = be.prepare_ggsw(dev(bsk))
        for b, seed in ((4, 52), (4, 52), (4, 57), (3, 58)):
            lwe_a_h, lwe_b_h = rnd(seed, q, b, dim), rnd(seed + 100, q, b)
            acc0 = np.zeros((b, k + 1, n), np.uint64)
            acc0[:, k] = rnd(seed + 200, q, b, n)
            if b == 4:  # the same device buffers for the first three calls
                la.copy_(dev(lwe_a_h))
                lb.copy_(dev(lwe_b_h))
                acc.copy_(dev(acc0))
                la_, lb_, acc_ = la, lb, acc
            else:
                la_, lb_, acc_ = dev(lwe_a_h), dev(lwe_b_h), dev(acc0)
            be.blind_rotate(acc_, la_, lb_, bsk_ntt)
            side.synchronize()
            got = acc_.cpu().numpy().view(np.uint64)
            for i in range(b):
                exp = t.blind_rotate(k, bl, lv, lwe_a_h[i], int(lwe_b_h[i]), q, bsk, acc0[i])
                assert (got[i] == exp).all(), (b, seed, i)
