"""CPU oracle for parity tests (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package -- as the checker, never as the thing measured or
shipped.  The product library (``node-fhe-accelerate_amd``) never imports it.

Wraps ``liboracle.so`` (``ref_cpu.c``: a C restatement of the reference
NTTProcessor / PolynomialRing / ModularArithmetic / BootstrapEngine code, see
that file for citations) with numpy-friendly helpers.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: an alternative build of ref_cpu.c (the ASan/UBSan build of
# `make -C oracle sanitize`, loaded by tests/test_sanitize.py)
_LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
_lib = None

u64p = C.POINTER(C.c_uint64)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if "ORACLE_LIB" not in os.environ and (not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "ref_cpu.c")
        )):
            build()
        L = C.CDLL(_LIB_PATH)
        L.oracle_strerror.restype = C.c_char_p
        L.oracle_bit_reverse.restype = C.c_uint32
        L.oracle_log2_pow2.restype = C.c_uint32
        L.oracle_mod_pow.restype = C.c_uint64
        L.oracle_mod_pow.argtypes = [C.c_uint64] * 3
        L.oracle_ntt_mod_inverse.argtypes = [C.c_uint64, C.c_uint64, u64p]
        L.oracle_find_primitive_root.argtypes = [C.c_uint32, C.c_uint64, u64p]
        L.oracle_mont_constants.argtypes = [C.c_uint64, u64p]
        for nm in ("oracle_mont_mul",):
            getattr(L, nm).restype = C.c_uint64
            getattr(L, nm).argtypes = [u64p, C.c_uint64, C.c_uint64]
        L.oracle_mont_reduce.restype = C.c_uint64
        L.oracle_mont_reduce.argtypes = [u64p, C.c_uint64, C.c_uint64]
        for nm in ("oracle_to_mont", "oracle_from_mont"):
            getattr(L, nm).restype = C.c_uint64
            getattr(L, nm).argtypes = [u64p, C.c_uint64]
        for nm in ("oracle_mod_add", "oracle_mod_sub"):
            getattr(L, nm).restype = C.c_uint64
            getattr(L, nm).argtypes = [C.c_uint64] * 3
        L.oracle_barrett_mu.argtypes = [C.c_uint64, u64p]
        L.oracle_barrett_mul.restype = C.c_uint64
        L.oracle_barrett_mul.argtypes = [C.c_uint64] * 4
        L.oracle_modmul_batch.argtypes = [C.c_uint64, u64p, u64p, u64p, C.c_size_t]
        L.oracle_ml_constants.argtypes = [u64p, u64p]
        L.oracle_ml_montmul_batch.argtypes = [u64p, u64p, u64p, u64p, C.c_size_t]
        L.oracle_ntt_create.argtypes = [C.c_uint32, C.c_uint64, C.POINTER(C.c_void_p)]
        L.oracle_ntt_destroy.argtypes = [C.c_void_p]
        L.oracle_ntt_psi.restype = C.c_uint64
        L.oracle_ntt_psi.argtypes = [C.c_void_p]
        L.oracle_ntt_inv_n.restype = C.c_uint64
        L.oracle_ntt_inv_n.argtypes = [C.c_void_p]
        L.oracle_ntt_tables.argtypes = [C.c_void_p, u64p, u64p]
        for nm in ("oracle_ntt_forward_batch", "oracle_ntt_inverse_batch"):
            getattr(L, nm).argtypes = [C.c_void_p, u64p, C.c_size_t]
        L.oracle_polymul_batch.argtypes = [C.c_void_p, u64p, u64p, u64p, C.c_size_t]
        L.oracle_ntt_fwd_mul_batch.argtypes = [C.c_void_p, u64p, u64p, u64p, C.c_size_t]
        L.oracle_pointwise.argtypes = [C.c_uint64, u64p, u64p, u64p, C.c_size_t]
        L.oracle_poly_add.argtypes = [C.c_uint64, u64p, u64p, u64p, C.c_size_t]
        L.oracle_poly_sub.argtypes = [C.c_uint64, u64p, u64p, u64p, C.c_size_t]
        L.oracle_poly_neg.argtypes = [C.c_uint64, u64p, u64p, C.c_size_t]
        L.oracle_poly_mul_scalar.argtypes = [C.c_uint64, u64p, C.c_uint64, u64p, C.c_size_t]
        L.oracle_decompose.argtypes = [C.c_uint64, u64p, C.c_uint32, C.c_uint32, C.c_uint32, u64p]
        L.oracle_external_product.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, u64p, u64p, u64p]
        L.oracle_rotate.argtypes = [C.c_uint64, u64p, C.c_uint32, C.c_int32, u64p]
        L.oracle_sample_extract.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, u64p, u64p, u64p]
        L.oracle_cmux.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, u64p, u64p, u64p, u64p]
        L.oracle_blind_rotate.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u64p,
                                          C.c_uint64, C.c_uint64, u64p, u64p]
        L.oracle_key_switch.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u64p, u64p,
                                        u64p, C.c_uint64, u64p, u64p]
        L.oracle_ct_multiply.argtypes = [C.c_void_p, u64p, u64p, C.c_int, u64p]
        L.oracle_relinearize.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, u64p, u64p, u64p]
        L.oracle_encode.argtypes = [C.c_uint64, C.c_uint64, u64p, C.c_uint32, u64p]
        L.oracle_encrypt.argtypes = [C.c_void_p, C.c_uint64, u64p, u64p, u64p, u64p, u64p, u64p]
        L.oracle_decrypt.argtypes = [C.c_void_p, C.c_uint64, u64p, u64p, C.c_uint32, C.c_int, u64p, u64p, u64p]
        L.oracle_add_plain.argtypes = [C.c_void_p, C.c_uint64, u64p, u64p, C.c_int, u64p]
        L.oracle_bootstrap.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u64p, C.c_uint64,
                                       C.c_uint64, u64p, u64p, C.c_uint32, C.c_uint32, C.c_uint32, u64p, u64p, u64p,
                                       u64p]
        L.oracle_testrandom_coeffs.argtypes = [C.c_uint64, C.c_uint64, u64p, C.c_size_t]
        L.oracle_mt19937_64_raw.argtypes = [C.c_uint64, u64p, C.c_size_t]
        L.oracle_splitmix_fill.argtypes = [C.c_uint64, C.c_uint64, u64p, C.c_size_t, C.c_size_t]
        L.oracle_batch_threaded.argtypes = [C.c_void_p, C.c_int, u64p, u64p, u64p, C.c_size_t, C.c_int]
        i64p = C.POINTER(C.c_int64)
        L.oracle_sample.argtypes = [C.c_int, u64p, C.c_uint64, C.c_uint64, C.c_double, u64p, C.c_size_t]
        L.oracle_public_key_generate.argtypes = [C.c_void_p, u64p, u64p, C.c_uint64, C.c_double, u64p]
        L.oracle_eval_key_generate.argtypes = [C.c_void_p, u64p, C.c_uint32, C.c_uint32, u64p, C.c_uint64, C.c_double,
                                               u64p]
        L.oracle_ggsw_encrypt.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, i64p, C.c_size_t, u64p,
                                          u64p, C.c_uint64, C.c_double, u64p]
        L.oracle_ksk_generate.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, u64p, C.c_uint32, i64p, C.c_uint32,
                                          u64p, C.c_uint64, C.c_double, u64p, u64p]
        L.oracle_lwe_decrypt.argtypes = [C.c_uint64, C.c_uint64, i64p, C.c_uint32, u64p, C.c_uint64, u64p, u64p]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u64p)


class OracleError(ValueError):
    pass


def _check(rc):
    if rc != 0:
        raise OracleError(lib().oracle_strerror(rc).decode())


# ---------------------------------------------------------------- scalars
def bit_reverse(i, bits):
    return lib().oracle_bit_reverse(i, bits)


def log2_pow2(n):
    return lib().oracle_log2_pow2(n)


def is_power_of_two(n):
    return bool(lib().oracle_is_power_of_two(n))


def mod_pow(b, e, m):
    return lib().oracle_mod_pow(b, e, m)


def mod_inverse(a, m):
    out = C.c_uint64()
    _check(lib().oracle_ntt_mod_inverse(a, m, C.byref(out)))
    return out.value


def find_primitive_root(n, q):
    out = C.c_uint64()
    _check(lib().oracle_find_primitive_root(n, q, C.byref(out)))
    return out.value


def mont_constants(q):
    out = (C.c_uint64 * 4)()
    _check(lib().oracle_mont_constants(q, out))
    return list(out)


def _carr(c):
    return (C.c_uint64 * len(c))(*c)


def mont_mul(consts, a, b):
    return lib().oracle_mont_mul(_carr(consts), a, b)


def to_mont(consts, a):
    return lib().oracle_to_mont(_carr(consts), a)


def from_mont(consts, a):
    return lib().oracle_from_mont(_carr(consts), a)


def mod_add(q, a, b):
    return lib().oracle_mod_add(q, a, b)


def mod_sub(q, a, b):
    return lib().oracle_mod_sub(q, a, b)


def barrett_mu(q):
    out = C.c_uint64()
    _check(lib().oracle_barrett_mu(q, C.byref(out)))
    return out.value


def barrett_mul(q, a, b):
    return lib().oracle_barrett_mul(q, barrett_mu(q), a, b)


def ml_constants(q_limbs):
    out = (C.c_uint64 * 7)()
    _check(lib().oracle_ml_constants(_carr(q_limbs), out))
    return list(out)


# ---------------------------------------------------------------- vectors
def modmul_batch(q, a, b):
    c = np.empty_like(a)
    lib().oracle_modmul_batch(q, _p(a), _p(b), _p(c), a.size)
    return c


def ml_montmul_batch(q_limbs, a, b):
    consts = _carr(ml_constants(q_limbs))
    c = np.empty_like(a)
    lib().oracle_ml_montmul_batch(consts, _p(a), _p(b), _p(c), a.size // 2)
    return c


def pointwise(q, a, b):
    c = np.empty_like(a)
    lib().oracle_pointwise(q, _p(a), _p(b), _p(c), a.size)
    return c


def poly_add(q, a, b):
    c = np.empty_like(a)
    lib().oracle_poly_add(q, _p(a), _p(b), _p(c), a.size)
    return c


def poly_sub(q, a, b):
    c = np.empty_like(a)
    lib().oracle_poly_sub(q, _p(a), _p(b), _p(c), a.size)
    return c


def poly_neg(q, a):
    c = np.empty_like(a)
    lib().oracle_poly_neg(q, _p(a), _p(c), a.size)
    return c


def poly_mul_scalar(q, a, s):
    c = np.empty_like(a)
    lib().oracle_poly_mul_scalar(q, _p(a), s, _p(c), a.size)
    return c


def decompose(q, poly, base_log, level):
    poly = np.ascontiguousarray(poly, dtype=np.uint64)
    out = np.empty((level, poly.size), dtype=np.uint64)
    lib().oracle_decompose(q, _p(poly), poly.size, base_log, level, _p(out))
    return out


def rotate(q, poly, rotation):
    poly = np.ascontiguousarray(poly, dtype=np.uint64)
    out = np.empty_like(poly)
    lib().oracle_rotate(q, _p(poly), poly.size, rotation, _p(out))
    return out


def sample_extract(q, glwe):
    glwe = np.ascontiguousarray(glwe, dtype=np.uint64)
    kp1, n = glwe.shape
    a = np.empty((kp1 - 1) * n, dtype=np.uint64)
    b = C.c_uint64()
    lib().oracle_sample_extract(q, kp1 - 1, n, _p(glwe), _p(a), C.byref(b))
    return a, b.value


def key_switch(q, base_log, level, ksk_a, ksk_b, lwe_a, lwe_b):
    """BootstrapEngine::key_switch for one LWE ciphertext -> (out_a, out_b)."""
    ksk_a = np.ascontiguousarray(ksk_a, dtype=np.uint64)
    ksk_b = np.ascontiguousarray(ksk_b, dtype=np.uint64)
    lwe_a = np.ascontiguousarray(lwe_a, dtype=np.uint64)
    out_dim = ksk_a.shape[1]
    out_a = np.empty(out_dim, dtype=np.uint64)
    b = C.c_uint64()
    lib().oracle_key_switch(q, base_log, level, lwe_a.size, out_dim, _p(ksk_a), _p(ksk_b), _p(lwe_a), lwe_b,
                            _p(out_a), C.byref(b))
    return out_a, b.value


def encode(q, t, values):
    """encode_packed (encryption.cpp:117-131)."""
    values = np.ascontiguousarray(values, dtype=np.uint64)
    out = np.empty_like(values)
    lib().oracle_encode(q, t, _p(values), values.size, _p(out))
    return out


def testrandom_coeffs(seed, q, count):
    out = np.empty(count, dtype=np.uint64)
    lib().oracle_testrandom_coeffs(seed, q, _p(out), count)
    return out


def mt19937_64_raw(seed, count):
    out = np.empty(count, dtype=np.uint64)
    lib().oracle_mt19937_64_raw(seed, _p(out), count)
    return out


def splitmix_fill(seed, q, count, offset=0):
    out = np.empty(count, dtype=np.uint64)
    lib().oracle_splitmix_fill(seed, q, _p(out), count, offset)
    return out


# ---------------------------------------------------------------- key material / randomness
SAMPLE_UNIFORM, SAMPLE_TERNARY, SAMPLE_GAUSSIAN, SAMPLE_BINARY, SAMPLE_RAW = range(5)


def _seed(seed):
    s = np.ascontiguousarray(seed, dtype=np.uint64)
    assert s.size == 4
    return s


def _i64p(a):
    assert a.dtype == np.int64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def sample(kind, seed, stream, q, count, std_dev=0.0):
    """SecureRandom draws (key_manager.cpp:53-115) over the seeded ChaCha20 stream."""
    s = _seed(seed)
    out = np.empty(count, dtype=np.uint64)
    lib().oracle_sample(kind, _p(s), stream, q, std_dev, _p(out), count)
    return out


def ksk_generate(q, base_log, level, glwe_sk, lwe_sk, seed, stream, std_dev=0.0):
    """generate_key_switch_key (bootstrap_engine.cpp:367-420) -> (ksk_a [n_in*L][dim], ksk_b [n_in*L])."""
    g = np.ascontiguousarray(glwe_sk, dtype=np.uint64)
    ls = np.ascontiguousarray(lwe_sk, dtype=np.int64)
    s = _seed(seed)
    ka = np.empty((g.size * level, ls.size), dtype=np.uint64)
    kb = np.empty(g.size * level, dtype=np.uint64)
    lib().oracle_ksk_generate(q, base_log, level, _p(g), g.size, _i64p(ls), ls.size, _p(s), stream, std_dev,
                              _p(ka), _p(kb))
    return ka, kb


def lwe_decrypt(q, t, sk, a, b):
    """phase = b - <a, s> mod q; value = round(phase t / q) % t -> (value, phase)."""
    sk = np.ascontiguousarray(sk, dtype=np.int64)
    a = np.ascontiguousarray(a, dtype=np.uint64)
    v = np.zeros(1, dtype=np.uint64)
    ph = np.zeros(1, dtype=np.uint64)
    lib().oracle_lwe_decrypt(q, t, _i64p(sk), sk.size, _p(a), int(b), _p(v), _p(ph))
    return int(v[0]), int(ph[0])


class NTT:
    """Restated NTTProcessor(degree, modulus) (ntt_processor.cpp:134-160)."""

    def __init__(self, n, q):
        self.n, self.q = n, q
        h = C.c_void_p()
        _check(lib().oracle_ntt_create(n, q, C.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.oracle_ntt_destroy(h)
            self._h = None

    @property
    def psi(self):
        return lib().oracle_ntt_psi(self._h)

    @property
    def inv_n(self):
        return lib().oracle_ntt_inv_n(self._h)

    def tables(self):
        f = np.empty(self.n, dtype=np.uint64)
        i = np.empty(self.n, dtype=np.uint64)
        lib().oracle_ntt_tables(self._h, _p(f), _p(i))
        return f, i

    def _shape(self, a):
        a = np.array(a, dtype=np.uint64, copy=True, order="C")
        if a.shape[-1] != self.n:
            raise OracleError("Coefficient count must equal polynomial degree")
        return a

    def forward(self, a):
        a = self._shape(a)
        lib().oracle_ntt_forward_batch(self._h, _p(a), a.size // self.n)
        return a

    def inverse(self, a):
        a = self._shape(a)
        lib().oracle_ntt_inverse_batch(self._h, _p(a), a.size // self.n)
        return a

    def polymul(self, a, b):
        a = self._shape(a)
        b = self._shape(b)
        c = np.empty_like(a)
        lib().oracle_polymul_batch(self._h, _p(a), _p(b), _p(c), a.size // self.n)
        return c

    def fwd_mul(self, a, w):
        a = self._shape(a)
        w = self._shape(w)
        c = np.empty_like(a)
        lib().oracle_ntt_fwd_mul_batch(self._h, _p(a), _p(w), _p(c), a.size // self.n)
        return c

    def external_product(self, k, base_log, level, glwe, ggsw):
        glwe = np.ascontiguousarray(glwe, dtype=np.uint64)
        ggsw = np.ascontiguousarray(ggsw, dtype=np.uint64)
        out = np.empty(((k + 1), self.n), dtype=np.uint64)
        lib().oracle_external_product(self._h, k, base_log, level, _p(glwe), _p(ggsw), _p(out))
        return out

    def cmux(self, k, base_log, level, ggsw, ct0, ct1):
        ggsw, ct0, ct1 = (np.ascontiguousarray(x, dtype=np.uint64) for x in (ggsw, ct0, ct1))
        out = np.empty(((k + 1), self.n), dtype=np.uint64)
        lib().oracle_cmux(self._h, k, base_log, level, _p(ggsw), _p(ct0), _p(ct1), _p(out))
        return out

    def blind_rotate(self, k, base_log, level, lwe_a, lwe_b, lwe_q, bsk, acc):
        lwe_a, bsk = (np.ascontiguousarray(x, dtype=np.uint64) for x in (lwe_a, bsk))
        acc = np.array(acc, dtype=np.uint64, copy=True, order="C")
        lib().oracle_blind_rotate(self._h, k, base_log, level, lwe_a.size, _p(lwe_a), lwe_b, lwe_q, _p(bsk), _p(acc))
        return acc

    def ct_multiply(self, ct1, ct2, is_ntt=False):
        ct1, ct2 = (np.ascontiguousarray(x, dtype=np.uint64) for x in (ct1, ct2))
        out = np.empty((3, self.n), dtype=np.uint64)
        lib().oracle_ct_multiply(self._h, _p(ct1), _p(ct2), int(is_ntt), _p(out))
        return out

    def relinearize(self, base_log, level, ct3, rlk):
        ct3 = np.ascontiguousarray(ct3, dtype=np.uint64)
        rlk = np.ascontiguousarray(rlk, dtype=np.uint64) if level else np.zeros(1, dtype=np.uint64)
        out = np.empty((2, self.n), dtype=np.uint64)
        lib().oracle_relinearize(self._h, base_log, level, _p(ct3), _p(rlk), _p(out))
        return out

    # ---- EncryptionEngine encrypt / decrypt / add_plain, BootstrapEngine::bootstrap
    def encrypt(self, t, pk, values, u, e1, e2):
        """encrypt_internal (encryption.cpp:171-205); pk [2, n] = (a, b)."""
        pk, values, u, e1, e2 = (np.ascontiguousarray(x, dtype=np.uint64) for x in (pk, values, u, e1, e2))
        out = np.empty((2, self.n), dtype=np.uint64)
        lib().oracle_encrypt(self._h, t, _p(pk), _p(values), _p(u), _p(e1), _p(e2), _p(out))
        return out

    def decrypt(self, t, sk, ct, is_ntt=False):
        """decrypt (:234-300) -> (values [n], phase [n], max_noise)."""
        sk, ct = (np.ascontiguousarray(x, dtype=np.uint64) for x in (sk, ct))
        comps = ct.shape[0]
        vals = np.empty(self.n, dtype=np.uint64)
        ph = np.empty(self.n, dtype=np.uint64)
        mx = np.zeros(1, dtype=np.uint64)
        lib().oracle_decrypt(self._h, t, _p(sk), _p(ct), comps, int(is_ntt), _p(vals), _p(ph), _p(mx))
        return vals, ph, int(mx[0])

    def add_plain(self, t, ct, values, is_ntt=False):
        ct, values = (np.ascontiguousarray(x, dtype=np.uint64) for x in (ct, values))
        out = np.empty((2, self.n), dtype=np.uint64)
        lib().oracle_add_plain(self._h, t, _p(ct), _p(values), int(is_ntt), _p(out))
        return out

    def bootstrap(self, k, base_log, level, lwe_a, lwe_b, lwe_q, bsk, test_poly, ks_base_log, ks_level, ksk_a, ksk_b):
        """bootstrap_with_test_poly (bootstrap_engine.cpp:684-708) -> (a [out_dim], b)."""
        lwe_a, bsk, test_poly, ksk_a, ksk_b = (np.ascontiguousarray(x, dtype=np.uint64)
                                               for x in (lwe_a, bsk, test_poly, ksk_a, ksk_b))
        out_dim = ksk_a.shape[-1]
        oa = np.empty(out_dim, dtype=np.uint64)
        ob = np.zeros(1, dtype=np.uint64)
        lib().oracle_bootstrap(self._h, k, base_log, level, lwe_a.size, _p(lwe_a), int(lwe_b), lwe_q, _p(bsk),
                               _p(test_poly), ks_base_log, ks_level, out_dim, _p(ksk_a), _p(ksk_b), _p(oa), _p(ob))
        return oa, int(ob[0])

    # ---- key generation over the seeded stream (key_manager.cpp, bootstrap_engine.cpp)
    def public_key_generate(self, sk, seed, stream, std_dev):
        sk = np.ascontiguousarray(sk, dtype=np.uint64)
        pk = np.empty((2, self.n), dtype=np.uint64)
        lib().oracle_public_key_generate(self._h, _p(sk), _p(_seed(seed)), stream, std_dev, _p(pk))
        return pk

    def eval_key_generate(self, sk, base_log, level, seed, stream, std_dev):
        sk = np.ascontiguousarray(sk, dtype=np.uint64)
        rlk = np.empty((level, 2, self.n), dtype=np.uint64)
        lib().oracle_eval_key_generate(self._h, _p(sk), base_log, level, _p(_seed(seed)), stream, std_dev, _p(rlk))
        return rlk

    def ggsw_encrypt(self, k, base_log, level, values, sk, seed, stream, std_dev):
        v = np.ascontiguousarray(values, dtype=np.int64)
        sk = np.ascontiguousarray(sk, dtype=np.uint64)
        out = np.empty((v.size, (k + 1) * level, k + 1, self.n), dtype=np.uint64)
        lib().oracle_ggsw_encrypt(self._h, k, base_log, level, _i64p(v), v.size, _p(sk), _p(_seed(seed)), stream,
                                  std_dev, _p(out))
        return out

    def batch_threaded(self, op, a, b=None, c=None, threads=1):
        """op: 0 fwd (in place), 1 inv (in place), 2 polymul, 3 fwd+mul."""
        nb = a.size // self.n
        lib().oracle_batch_threaded(
            self._h, op, _p(a),
            _p(b) if b is not None else None,
            _p(c) if c is not None else None, nb, threads,
        )
