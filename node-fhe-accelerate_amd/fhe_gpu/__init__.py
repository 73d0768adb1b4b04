"""fhe_gpu -- Python host mirror of the reference operator interface over the
MI355X C-ABI (``include/fhe_gpu.h``, ``build/libfhe_gpu.so``).

Class and method names follow the reference C++ classes so parity tests read
like the reference's own tests:

=============================  ==============================================
reference (cpp/include/...)    here
=============================  ==============================================
NTTProcessor                   :class:`NTTProcessor`   (ntt_processor.h:49-306)
PolynomialRing                 :class:`PolynomialRing` (polynomial_ring.h:101-516)
PolynomialRing(degree, moduli) :class:`RNSPolynomialRing` (polynomial_ring.cpp:224-237)
ModularArithmetic              :class:`ModularArithmetic` (modular_arithmetic.h:20-80;
                               the N-API class of index.d.ts:32-44)
BarrettReducer                 :class:`BarrettReducer` (modular_arithmetic.h:82-)
MultiLimbModularArithmetic     :class:`MultiLimbModularArithmetic`
BootstrapEngine::external_product  :class:`ExternalProduct`
BootstrapEngine (cmux, blind_rotate, :class:`BootstrapEngine`
  sample_extract, key_switch, ...)
EncryptionEngine::multiply /   :class:`EncryptionEngine`, :class:`EvaluationKey`
  relinearize / multiply_relin
HardwareDetector::detect       :func:`detect_hardware`
=============================  ==============================================

Buffers: numpy ``uint64`` arrays (host; the call stages through HBM) or torch
CUDA tensors of dtype int64/uint64 (device-resident; enqueued on the current
torch stream, no host sync).  Shapes are ``[..., n]``: leading dims are the
batch.  Errors raise :class:`FHEError` carrying the reference's exception text.

There is no CPU fallback: if the HIP library is missing or no GPU is present
every compute call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import numpy as np

try:  # share torch's HIP runtime when torch is present (one runtime per process)
    import torch  # noqa: F401

    _HAVE_TORCH = True
except Exception:  # pragma: no cover
    torch = None
    _HAVE_TORCH = False

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)
LIB_PATH = os.environ.get("FHE_GPU_LIB", os.path.join(_ROOT, "build", "libfhe_gpu.so"))

FHE_OK = 0
FHE_HOST, FHE_DEVICE = 0, 1
MODE_COMPAT, MODE_NEGACYCLIC = 0, 1

ERROR_NAMES = {
    -1: "DEGREE_POW2", -2: "DEGREE_RANGE", -3: "MODULUS_EVEN", -4: "NOT_NTT_FRIENDLY",
    -5: "COUNT", -6: "NO_ROOT", -7: "MONT_MODULUS", -8: "ZERO_MODULUS", -9: "INVALID_ARG",
    -10: "UNSUPPORTED", -11: "DEVICE", -12: "OOM",
}


class FHEError(ValueError):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code
        self.name = ERROR_NAMES.get(code, "UNKNOWN")


class HwCaps(C.Structure):
    _fields_ = [
        ("device_count", C.c_int32), ("compute_units", C.c_int32), ("wavefront_size", C.c_int32),
        ("xcds", C.c_int32), ("hbm_bytes", C.c_uint64), ("lds_bytes_per_cu", C.c_uint64),
        ("arch", C.c_char * 32), ("name", C.c_char * 96),
    ]


class CtxInfo(C.Structure):
    _fields_ = [
        ("n", C.c_uint32), ("log_n", C.c_uint32), ("q", C.c_uint64), ("psi", C.c_uint64),
        ("psi_inv", C.c_uint64), ("inv_n", C.c_uint64), ("mode", C.c_int32), ("word_bits", C.c_int32),
        ("device", C.c_int32), ("polys_per_block", C.c_int32), ("threads_per_block", C.c_int32),
    ]


u64p = C.POINTER(C.c_uint64)
vp = C.c_void_p

# (name, restype, argtypes) of every entry point declared in include/fhe_gpu.h
SIGNATURES = [
    ("fhe_last_error", C.c_char_p, []),
    ("fhe_version", C.c_char_p, []),
    ("fhe_build_id", C.c_char_p, []),
    ("fhe_detect", C.c_int, [C.POINTER(HwCaps)]),
    ("fhe_ctx_create", C.c_int, [C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.POINTER(vp)]),
    ("fhe_ctx_destroy", None, [vp]),
    ("fhe_ctx_create_multi", C.c_int, [C.c_uint32, C.c_uint64, C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(vp)]),
    ("fhe_ctx_device_count", C.c_int, [vp, C.POINTER(C.c_int)]),
    ("fhe_ctx_sub", C.c_int, [vp, C.c_int, C.POINTER(vp)]),
    ("fhe_ctx_set_stream", C.c_int, [vp, vp]),
    ("fhe_ctx_stream", vp, [vp]),
    ("fhe_ctx_synchronize", C.c_int, [vp]),
    ("fhe_ctx_get_info", C.c_int, [vp, C.POINTER(CtxInfo)]),
    ("fhe_ctx_get_twiddles", C.c_int, [vp, vp, vp]),
    ("fhe_ntt_fwd_batch", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_ntt_inv_batch", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_ntt_fwd_mul_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_polymul_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_pointwise_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_poly_add_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_poly_sub_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_poly_neg_batch", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_poly_mul_scalar_batch", C.c_int, [vp, vp, C.c_uint64, vp, C.c_size_t, C.c_int]),
    ("fhe_ggsw_prepare", C.c_int, [vp, C.c_uint32, C.c_uint32, vp, vp, C.c_int]),
    ("fhe_external_product_batch", C.c_int,
     [vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_decompose_batch", C.c_int, [vp, C.c_uint32, C.c_uint32, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_rns_ctx_create", C.c_int, [C.c_uint32, u64p, C.c_uint32, C.c_int, C.c_int, C.POINTER(vp)]),
    ("fhe_rns_ctx_destroy", None, [vp]),
    ("fhe_rns_ctx_limb", C.c_int, [vp, C.c_uint32, C.POINTER(vp)]),
    ("fhe_rns_ntt_fwd_batch", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_rns_ntt_inv_batch", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_rns_polymul_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_rns_pointwise_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_rns_add_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_rns_sub_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_ct_multiply_batch", C.c_int, [vp, vp, vp, vp, C.c_size_t, C.c_int, C.c_int]),
    ("fhe_relin_key_prepare", C.c_int, [vp, C.c_uint32, vp, vp, C.c_int]),
    ("fhe_relinearize_batch", C.c_int, [vp, C.c_uint32, C.c_uint32, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_ct_multiply_relin_batch", C.c_int,
     [vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_glwe_rotate_batch", C.c_int, [vp, C.c_uint32, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_cmux_batch", C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_blind_rotate_batch", C.c_int,
     [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, C.c_uint64, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_sample_extract_batch", C.c_int, [vp, C.c_uint32, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_br_repair_count", C.c_int, [vp, C.POINTER(C.c_uint64)]),
    ("fhe_key_switch_batch", C.c_int,
     [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp, vp, C.c_size_t, C.c_int,
      C.c_int, vp]),
    ("fhe_secret_key_prepare", C.c_int, [vp, vp, vp, C.c_int]),
    ("fhe_public_key_prepare", C.c_int, [vp, vp, vp, C.c_int]),
    ("fhe_encrypt_batch", C.c_int, [vp, C.c_uint64, vp, vp, vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_decrypt_batch", C.c_int,
     [vp, C.c_uint64, vp, vp, C.c_uint32, C.c_int, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_add_plain_batch", C.c_int, [vp, C.c_uint64, vp, vp, C.c_int, vp, C.c_size_t, C.c_int]),
    ("fhe_bootstrap_batch", C.c_int,
     [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, C.c_uint64, vp, vp, C.c_uint32, C.c_uint32,
      C.c_uint32, vp, vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_sample_batch", C.c_int, [vp, C.c_int, u64p, C.c_uint64, C.c_double, vp, C.c_size_t, C.c_int]),
    ("fhe_encrypt_sampled_batch", C.c_int,
     [vp, C.c_uint64, vp, vp, u64p, C.c_uint64, C.c_double, vp, C.c_size_t, C.c_int]),
    ("fhe_public_key_generate", C.c_int, [vp, vp, u64p, C.c_uint64, C.c_double, vp, C.c_int]),
    ("fhe_eval_key_generate", C.c_int, [vp, vp, C.c_uint32, C.c_uint32, u64p, C.c_uint64, C.c_double, vp, C.c_int]),
    ("fhe_ggsw_encrypt_batch", C.c_int,
     [vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, C.c_size_t, vp, u64p, C.c_uint64, C.c_double, vp, C.c_int]),
    ("fhe_ksk_generate", C.c_int,
     [vp, C.c_uint32, C.c_uint32, vp, C.c_uint32, vp, C.c_uint32, u64p, C.c_uint64, C.c_double, vp, vp, C.c_int]),
    ("fhe_lwe_decrypt_batch", C.c_int,
     [C.c_uint64, C.c_uint64, vp, C.c_uint32, vp, vp, vp, vp, C.c_size_t, C.c_int, C.c_int, vp]),
    ("fhe_modmul_batch", C.c_int, [C.c_uint64, vp, vp, vp, C.c_size_t, C.c_int, C.c_int, vp]),
    ("fhe_ml_constants", C.c_int, [u64p, u64p]),
    ("fhe_ml_montmul_batch", C.c_int, [u64p, vp, vp, vp, C.c_size_t, C.c_int, C.c_int, vp]),
    ("fhe_mont_constants_compat", C.c_int, [C.c_uint64, u64p]),
    ("fhe_compat_montgomery_mul", C.c_uint64, [u64p, C.c_uint64, C.c_uint64]),
    ("fhe_compat_to_montgomery", C.c_uint64, [u64p, C.c_uint64]),
    ("fhe_compat_from_montgomery", C.c_uint64, [u64p, C.c_uint64]),
    ("fhe_compat_mod_add", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
    ("fhe_compat_mod_sub", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
    ("fhe_ctx_alloc", C.c_int, [vp, C.c_size_t, C.POINTER(vp)]),
    ("fhe_ctx_free", C.c_int, [vp, vp]),
    ("fhe_ctx_memcpy", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int]),
    ("fhe_dev_alloc", C.c_int, [C.c_int, C.c_size_t, C.POINTER(vp)]),
    ("fhe_dev_free", C.c_int, [vp]),
    ("fhe_memcpy_h2d", C.c_int, [vp, vp, C.c_size_t]),
    ("fhe_memcpy_d2h", C.c_int, [vp, vp, C.c_size_t]),
    ("fhe_device_synchronize", C.c_int, [C.c_int]),
    ("fhe_event_create", C.c_int, [C.POINTER(vp)]),
    ("fhe_event_destroy", C.c_int, [vp]),
    ("fhe_event_record", C.c_int, [vp, vp]),
    ("fhe_event_elapsed_ms", C.c_int, [vp, vp, C.POINTER(C.c_float)]),
]

_lib = None


def lib():
    """Load libfhe_gpu.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FHEError(-11, f"libfhe_gpu.so not found at {LIB_PATH}; run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        lab = "FHE_GPU_LIB" in os.environ  # lab A/B against an older build: skip its missing entries
        for name, res, args in SIGNATURES:
            if lab and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc: int):
    if rc != FHE_OK:
        raise FHEError(rc, lib().fhe_last_error().decode(errors="replace"))


def version() -> str:
    return lib().fhe_version().decode()


def build_id() -> str:
    """Hash of the sources and flags of the loaded library (Makefile)."""
    return lib().fhe_build_id().decode()


def detect_hardware() -> dict:
    """HardwareDetector::detect() / N-API detectHardware() for the MI355X."""
    caps = HwCaps()
    _check(lib().fhe_detect(C.byref(caps)))
    return {
        "deviceCount": caps.device_count, "computeUnits": caps.compute_units,
        "wavefrontSize": caps.wavefront_size, "xcds": caps.xcds, "hbmBytes": caps.hbm_bytes,
        "ldsBytesPerCu": caps.lds_bytes_per_cu, "arch": caps.arch.decode(), "name": caps.name.decode(),
    }


# ----------------------------------------------------------------- buffers
def _is_tensor(x) -> bool:
    return _HAVE_TORCH and isinstance(x, torch.Tensor)


def _stream_ptr(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class _Buf:
    """Pointer + placement for one argument."""

    __slots__ = ("ptr", "where", "count", "keep", "device")

    def __init__(self, x, writable=False):
        if _is_tensor(x):
            if not x.is_cuda:
                raise FHEError(-9, "torch tensors must be on a GPU (use numpy arrays for host data)")
            if x.dtype not in (torch.int64, torch.uint64):
                raise FHEError(-9, "device buffers must be int64/uint64 tensors")
            if not x.is_contiguous():
                raise FHEError(-9, "device buffers must be contiguous")
            self.ptr, self.where, self.count, self.keep = x.data_ptr(), FHE_DEVICE, x.numel(), x
            self.device = x.device
        else:
            a = x
            if not (isinstance(a, np.ndarray) and a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]):
                if writable:
                    raise FHEError(-9, "output must be a C-contiguous numpy uint64 array")
                a = np.ascontiguousarray(np.asarray(x, dtype=np.uint64))
            self.ptr, self.where, self.count, self.keep = a.ctypes.data, FHE_HOST, a.size, a
            self.device = None


_TLS = threading.local()  # device of the last _where() call's tensors (for _bind_stream)


def _where(*bufs: _Buf) -> int:
    w = {b.where for b in bufs if b is not None}
    if len(w) != 1:
        raise FHEError(-9, "all buffers of one call must be host arrays or all device tensors")
    devs = {b.device for b in bufs if b is not None and b.device is not None}
    if len(devs) > 1:
        raise FHEError(-9, "all device tensors of one call must be on the same GPU")
    _TLS.device = devs.pop() if devs else None
    return w.pop()


def _like(x):
    if _is_tensor(x):
        return torch.empty_like(x)
    return np.empty(np.shape(x), dtype=np.uint64)


def _as_u64(x):
    if _is_tensor(x):
        return x
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint64))


# ----------------------------------------------------------------- static helpers
def is_power_of_two(n: int) -> bool:  # ntt_processor.cpp:25-27
    return n > 0 and (n & (n - 1)) == 0


def log2_pow2(n: int) -> int:  # :29-36
    r = 0
    while n > 1:
        n >>= 1
        r += 1
    return r


def bit_reverse(index: int, bits: int) -> int:  # :38-45
    r = 0
    for _ in range(bits):
        r = (r << 1) | (index & 1)
        index >>= 1
    return r


def mod_pow(base: int, exp: int, mod: int) -> int:  # :47-62
    return pow(base % mod, exp, mod) if mod != 1 else 0


def mod_inverse(a: int, m: int) -> int:  # :64-90 (signed extended Euclid)
    if m == 0:
        raise FHEError(-8, "Modulus cannot be zero")
    if m == 1:
        return 0
    return pow(a % m, -1, m)


def find_primitive_root(degree: int, modulus: int) -> int:  # :92-128
    two_n = 2 * degree
    if (modulus - 1) % two_n:
        raise FHEError(-4, "Modulus is not NTT-friendly: q ≢ 1 (mod 2N)")
    e = (modulus - 1) // two_n
    for g in range(2, min(modulus, 1 << 22)):
        w = pow(g, e, modulus)
        if pow(w, two_n, modulus) == 1 and pow(w, degree, modulus) == modulus - 1:
            return w
    raise FHEError(-6, "Could not find primitive root for given parameters")


# ----------------------------------------------------------------- NTT / ring
def env_defaults(mode=None, device=None, devices=None):
    """Context defaults from the environment (SURVEY.md section 5 config flags):
    FHE_NTT_MODE = compat | negacyclic (mode when not given);
    FHE_GPU_DEVICES = comma-separated GPU ordinals (device list when neither
    device nor devices is given: one entry -> that device, several -> a
    multi-device context).  Returns (mode, device, devices)."""
    if mode is None:
        mode = os.environ.get("FHE_NTT_MODE", "compat").strip() or "compat"
    if device is None and devices is None:
        env = os.environ.get("FHE_GPU_DEVICES", "").strip()
        if env:
            try:
                devs = [int(x) for x in env.split(",") if x.strip()]
            except ValueError:
                raise FHEError(-9, f"FHE_GPU_DEVICES must be a comma-separated list of ordinals, got {env!r}")
            if len(devs) == 1:
                device = devs[0]
            elif devs:
                devices = devs
    if device is None:
        device = int(devices[0]) if devices else 0
    return mode, device, devices


class NTTProcessor:
    """NTTProcessor(degree, modulus) on the MI355X (ntt_processor.h:49-306).

    ``mode='compat'`` reproduces the reference transform bit for bit;
    ``mode='negacyclic'`` is the psi-twisted transform whose pointwise product
    is multiplication mod X^N + 1.
    """

    is_power_of_two = staticmethod(is_power_of_two)
    log2_pow2 = staticmethod(log2_pow2)
    bit_reverse = staticmethod(bit_reverse)
    mod_pow = staticmethod(mod_pow)
    mod_inverse = staticmethod(mod_inverse)
    find_primitive_root = staticmethod(find_primitive_root)

    def __init__(self, degree: int, modulus: int, mode: str = None, device: int = None, devices=None):
        """devices: a list of GPU ordinals for a multi-device context
        (fhe_ctx_create_multi): host-array batches are split across them, a
        device tensor runs on the GPU that holds it.  Unset arguments come
        from the environment (env_defaults): mode from FHE_NTT_MODE, the
        device list from FHE_GPU_DEVICES; otherwise compat on device 0."""
        mode, device, devices = env_defaults(mode, device, devices)
        m = {"compat": MODE_COMPAT, "negacyclic": MODE_NEGACYCLIC}.get(mode)
        if m is None:
            raise FHEError(-9, f"unknown mode {mode!r}")
        h = C.c_void_p()
        if devices is not None:
            devs = [int(d) for d in devices]
            arr = (C.c_int * max(1, len(devs)))(*devs)
            _check(lib().fhe_ctx_create_multi(degree, modulus, m, arr, len(devs), C.byref(h)))
            device = devs[0]
        else:
            _check(lib().fhe_ctx_create(degree, modulus, m, device, C.byref(h)))
        self._h = h
        self.devices = list(devices) if devices is not None else [device]
        self.degree, self.modulus, self.mode, self.device = degree, modulus, mode, device
        info = CtxInfo()
        _check(lib().fhe_ctx_get_info(h, C.byref(info)))
        self.info = info

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.fhe_ctx_destroy(h)
        self._h = None

    __del__ = close

    # -- introspection (get_degree/get_modulus/get_twiddles, ntt_processor.h)
    def get_degree(self):
        return self.degree

    def get_modulus(self):
        return self.modulus

    @property
    def primitive_root(self):
        return self.info.psi

    @property
    def inv_n(self):
        return self.info.inv_n

    def get_twiddles(self):
        f = np.empty(self.degree, dtype=np.uint64)
        i = np.empty(self.degree, dtype=np.uint64)
        _check(lib().fhe_ctx_get_twiddles(self._h, f.ctypes.data, i.ctypes.data))
        return {"forward": f, "inverse": i, "primitive_root": self.info.psi, "inv_n": self.info.inv_n}

    # -- plumbing
    def _batch(self, x) -> int:
        shape = tuple(x.shape)
        if not shape or shape[-1] != self.degree:
            raise FHEError(-5, "Coefficient count must equal polynomial degree")
        b = 1
        for s in shape[:-1]:
            b *= s
        return b

    def _bind_stream(self, where):
        if where == FHE_DEVICE:
            _check(lib().fhe_ctx_set_stream(self._h, _stream_ptr(getattr(_TLS, "device", None))))

    def _unary(self, fn, x, out):
        x = _as_u64(x)
        nb = self._batch(x)
        out = _like(x) if out is None else out
        bi, bo = _Buf(x), _Buf(out, True)
        w = _where(bi, bo)
        self._bind_stream(w)
        _check(fn(self._h, bi.ptr, bo.ptr, nb, w))
        return out

    def _binary(self, fn, a, b, out):
        a, b = _as_u64(a), _as_u64(b)
        nb = self._batch(a)
        if tuple(b.shape) != tuple(a.shape):
            raise FHEError(-9, "operand shapes differ")
        out = _like(a) if out is None else out
        ba, bb, bo = _Buf(a), _Buf(b), _Buf(out, True)
        w = _where(ba, bb, bo)
        self._bind_stream(w)
        _check(fn(self._h, ba.ptr, bb.ptr, bo.ptr, nb, w))
        return out

    # -- transforms
    def forward_ntt(self, coeffs, out=None):
        """forward_ntt (ntt_processor.cpp:262-319); pass out=coeffs for in place."""
        return self._unary(lib().fhe_ntt_fwd_batch, coeffs, out)

    def inverse_ntt(self, coeffs, out=None):
        """inverse_ntt (ntt_processor.cpp:325-388)."""
        return self._unary(lib().fhe_ntt_inv_batch, coeffs, out)

    forward_ntt_batch = forward_ntt
    inverse_ntt_batch = inverse_ntt

    def forward_ntt_mul(self, coeffs, w, out=None):
        """to_ntt(coeffs) then pointwise by w (config C3, fused)."""
        return self._binary(lib().fhe_ntt_fwd_mul_batch, coeffs, w, out)


class PolynomialRing(NTTProcessor):
    """PolynomialRing(degree, modulus) (polynomial_ring.h:101-516) over batches."""

    def multiply(self, a, b, out=None):
        """multiply (polynomial_ring.cpp:421-447): inv(fwd(a) (.) fwd(b)), fused."""
        return self._binary(lib().fhe_polymul_batch, a, b, out)

    def pointwise_multiply(self, a, b, out=None):
        return self._binary(lib().fhe_pointwise_batch, a, b, out)

    def add(self, a, b, out=None):
        return self._binary(lib().fhe_poly_add_batch, a, b, out)

    def subtract(self, a, b, out=None):
        return self._binary(lib().fhe_poly_sub_batch, a, b, out)

    def negate(self, a, out=None):
        return self._unary(lib().fhe_poly_neg_batch, a, out)

    def multiply_scalar(self, a, scalar: int, out=None):
        a = _as_u64(a)
        nb = self._batch(a)
        out = _like(a) if out is None else out
        ba, bo = _Buf(a), _Buf(out, True)
        w = _where(ba, bo)
        self._bind_stream(w)
        _check(lib().fhe_poly_mul_scalar_batch(self._h, ba.ptr, scalar, bo.ptr, nb, w))
        return out

    def to_ntt(self, p, out=None):
        return self.forward_ntt(p, out)

    def from_ntt(self, p, out=None):
        return self.inverse_ntt(p, out)


class RNSPolynomialRing:
    """PolynomialRing(degree, moduli) (polynomial_ring.cpp:224-237): one
    transform context per modulus on one stream.  Arrays are modulus-major
    [len(moduli), ..., n]; every operation applies to every limb (the
    reference's ring operations use moduli_[0] only)."""

    def __init__(self, degree: int, moduli, mode: str = None, device: int = None):
        mode, device, devs = env_defaults(mode, device, None)  # one device: the first of FHE_GPU_DEVICES
        m = {"compat": MODE_COMPAT, "negacyclic": MODE_NEGACYCLIC}.get(mode)
        if m is None:
            raise FHEError(-9, f"unknown mode {mode!r}")
        mods = [int(x) for x in moduli]
        arr = (C.c_uint64 * max(1, len(mods)))(*mods)
        h = C.c_void_p()
        _check(lib().fhe_rns_ctx_create(degree, arr, len(mods), m, device, C.byref(h)))
        self._h = h
        self.degree, self.moduli, self.mode, self.device = degree, mods, mode, device

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.fhe_rns_ctx_destroy(h)
        self._h = None

    __del__ = close

    def _batch(self, x) -> int:
        shape = tuple(x.shape)
        if len(shape) < 2 or shape[0] != len(self.moduli) or shape[-1] != self.degree:
            raise FHEError(-5, f"RNS arrays must be [{len(self.moduli)}, ..., {self.degree}]")
        return int(np.prod(shape[1:-1])) if len(shape) > 2 else 1

    def _bind(self, where):
        if where == FHE_DEVICE:
            first = C.c_void_p()
            _check(lib().fhe_rns_ctx_limb(self._h, 0, C.byref(first)))
            _check(lib().fhe_ctx_set_stream(first, _stream_ptr()))
            for i in range(1, len(self.moduli)):
                c = C.c_void_p()
                _check(lib().fhe_rns_ctx_limb(self._h, i, C.byref(c)))
                _check(lib().fhe_ctx_set_stream(c, _stream_ptr()))

    def _unary(self, fn, x, out):
        x = _as_u64(x)
        nb = self._batch(x)
        out = _like(x) if out is None else out
        bi, bo = _Buf(x), _Buf(out, True)
        w = _where(bi, bo)
        self._bind(w)
        _check(fn(self._h, bi.ptr, bo.ptr, nb, w))
        return out

    def _binary(self, fn, a, b, out):
        a, b = _as_u64(a), _as_u64(b)
        nb = self._batch(a)
        if tuple(b.shape) != tuple(a.shape):
            raise FHEError(-9, "operand shapes differ")
        out = _like(a) if out is None else out
        ba, bb, bo = _Buf(a), _Buf(b), _Buf(out, True)
        w = _where(ba, bb, bo)
        self._bind(w)
        _check(fn(self._h, ba.ptr, bb.ptr, bo.ptr, nb, w))
        return out

    def forward_ntt(self, x, out=None):
        return self._unary(lib().fhe_rns_ntt_fwd_batch, x, out)

    def inverse_ntt(self, x, out=None):
        return self._unary(lib().fhe_rns_ntt_inv_batch, x, out)

    def multiply(self, a, b, out=None):
        return self._binary(lib().fhe_rns_polymul_batch, a, b, out)

    def pointwise_multiply(self, a, b, out=None):
        return self._binary(lib().fhe_rns_pointwise_batch, a, b, out)

    def add(self, a, b, out=None):
        return self._binary(lib().fhe_rns_add_batch, a, b, out)

    def subtract(self, a, b, out=None):
        return self._binary(lib().fhe_rns_sub_batch, a, b, out)


class ExternalProduct:
    """BootstrapEngine::external_product (bootstrap_engine.cpp:431-518) for a
    batch of GLWE ciphertexts ([..., k+1, n]) against one GGSW
    ([(k+1)*level, k+1, n], coefficient form, reference row order)."""

    def __init__(self, ring: NTTProcessor, ggsw, base_log: int, level: int, k: int = 1):
        self.ring, self.base_log, self.level, self.k = ring, base_log, level, k
        g = _as_u64(ggsw)
        exp = ((k + 1) * level, k + 1, ring.degree)
        if tuple(g.shape) != exp:
            raise FHEError(-9, f"ggsw shape must be {exp}")
        self.ggsw_ntt = _like(g)
        bi, bo = _Buf(g), _Buf(self.ggsw_ntt, True)
        w = _where(bi, bo)
        ring._bind_stream(w)
        _check(lib().fhe_ggsw_prepare(ring._h, k, level, bi.ptr, bo.ptr, w))

    def __call__(self, glwe, out=None):
        glwe = _as_u64(glwe)
        shape = tuple(glwe.shape)
        if len(shape) < 2 or shape[-2:] != (self.k + 1, self.ring.degree):
            raise FHEError(-9, "glwe must have shape [..., k+1, n]")
        nb = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
        out = _like(glwe) if out is None else out
        bi, bk, bo = _Buf(glwe), _Buf(self.ggsw_ntt), _Buf(out, True)
        w = _where(bi, bk, bo)
        self.ring._bind_stream(w)
        _check(lib().fhe_external_product_batch(self.ring._h, self.k, self.base_log, self.level, bi.ptr, bk.ptr,
                                                bo.ptr, nb, w))
        return out


def _empty(like, shape):
    if _is_tensor(like):
        return torch.empty(shape, dtype=like.dtype, device=like.device)
    return np.empty(shape, dtype=np.uint64)


def _lead(x, tail) -> int:
    """Batch size of x with trailing shape `tail`."""
    shape = tuple(x.shape)
    if len(shape) < len(tail) or shape[len(shape) - len(tail):] != tuple(tail):
        raise FHEError(-9, f"expected shape [..., {', '.join(map(str, tail))}], got {list(shape)}")
    return int(np.prod(shape[: len(shape) - len(tail)])) if len(shape) > len(tail) else 1


class EvaluationKey:
    """Relinearisation key (KeySwitchKey of key_manager.h:85-111): the
    (a_l, b_l) pairs ``rlk`` [level, 2, n] in coefficient form, prepared once
    into the NTT domain on the GPU."""

    def __init__(self, ring: "PolynomialRing", rlk, decomp_base_log: int = 0):
        rlk = _as_u64(rlk)
        self.level = int(rlk.shape[0]) if rlk.ndim == 3 else 0
        if self.level and tuple(rlk.shape[1:]) != (2, ring.degree):
            raise FHEError(-9, "rlk must have shape [level, 2, n]")
        # encryption.cpp:935: base_log 0 -> 4
        self.decomp_base_log = decomp_base_log if decomp_base_log > 0 else 4
        self.ring = ring
        self.rlk_ntt = _like(rlk)
        if self.level:
            bi, bo = _Buf(rlk), _Buf(self.rlk_ntt, True)
            w = _where(bi, bo)
            ring._bind_stream(w)
            _check(lib().fhe_relin_key_prepare(ring._h, self.level, bi.ptr, bo.ptr, w))


class SecretKey:
    """SecretKey (key_manager.h): the polynomial s [n] and its NTT-domain
    form prepared once on the GPU (fhe_secret_key_prepare: s and s^2)."""

    def __init__(self, ring: "PolynomialRing", poly):
        s = _as_u64(poly)
        if tuple(s.shape) != (ring.degree,):
            raise FHEError(-9, "secret key must have shape [n]")
        self.poly, self.ring = s, ring
        self.prep = _empty(s, (2, ring.degree))
        bi, bo = _Buf(s), _Buf(self.prep, True)
        w = _where(bi, bo)
        ring._bind_stream(w)
        _check(lib().fhe_secret_key_prepare(ring._h, bi.ptr, bo.ptr, w))


class PublicKey:
    """PublicKey (key_manager.h:70-76): (a, b = a s + e) as [2, n], prepared
    once into the NTT domain (fhe_public_key_prepare)."""

    def __init__(self, ring: "PolynomialRing", a, b=None):
        pk = _as_u64(a) if b is None else (torch.stack([_as_u64(a), _as_u64(b)]) if _is_tensor(a)
                                            else np.stack([_as_u64(a), _as_u64(b)]))
        if tuple(pk.shape) != (2, ring.degree):
            raise FHEError(-9, "public key must have shape [2, n] = (a, b)")
        self.poly, self.ring = pk, ring
        self.prep = _like(pk)
        bi, bo = _Buf(pk), _Buf(self.prep, True)
        w = _where(bi, bo)
        ring._bind_stream(w)
        _check(lib().fhe_public_key_prepare(ring._h, bi.ptr, bo.ptr, w))


SAMPLE_UNIFORM, SAMPLE_TERNARY, SAMPLE_GAUSSIAN, SAMPLE_BINARY, SAMPLE_RAW = range(5)


def _seed_arr(seed):
    """A 256-bit ChaCha20 seed as 4 u64 words (an int, 4 ints, or bytes)."""
    if isinstance(seed, (bytes, bytearray)):
        seed = np.frombuffer(bytes(seed).ljust(32, b"\0")[:32], dtype=np.uint64)
    elif isinstance(seed, int):
        seed = [(seed >> (64 * i)) & ((1 << 64) - 1) for i in range(4)]
    a = (C.c_uint64 * 4)(*[int(x) for x in np.asarray(seed, dtype=np.uint64).reshape(4)])
    return a


def new_seed() -> bytes:
    """256 bits from the OS CSPRNG (the engine's default seed)."""
    return os.urandom(32)


def sample(ring: "NTTProcessor", kind: int, seed, stream: int, count: int, std_dev: float = 3.2, out=None,
           device_out: bool = False):
    """SecureRandom draws (key_manager.cpp:53-115) over the seeded ChaCha20
    stream of include/fhe_gpu.h (fhe_sample_batch), modulo the ring modulus."""
    if out is None:
        out = (torch.empty(count, dtype=torch.int64, device=f"cuda:{ring.device}") if device_out
               else np.empty(count, dtype=np.uint64))
    bo = _Buf(out, True)
    w = _where(bo)
    ring._bind_stream(w)
    _check(lib().fhe_sample_batch(ring._h, int(kind), _seed_arr(seed), int(stream), float(std_dev), bo.ptr, count, w))
    return out


class KeyGenerator:
    """KeyManager (key_manager.cpp:150-333) and the bootstrapping-key half of
    BootstrapEngine (bootstrap_engine.cpp:268-420) on the GPU, drawing from
    a seeded ChaCha20 stream: the same (seed, stream) gives the same keys on
    every device and in the CPU oracle.  Arrays follow the placement of the
    inputs (numpy: host, torch: device)."""

    def __init__(self, ring: "PolynomialRing", seed=None, noise_std: float = 3.2):
        self.ring = ring
        self.seed = seed if seed is not None else new_seed()
        self.noise_std = float(noise_std)

    def secret_key(self, stream: int, kind: int = SAMPLE_TERNARY, device_out: bool = False):
        """generate_secret_key (:150-196): TERNARY (default), GAUSSIAN, BINARY or UNIFORM coefficients."""
        return sample(self.ring, kind, self.seed, stream, self.ring.degree, self.noise_std, device_out=device_out)

    def public_key(self, sk, stream: int, out=None):
        """generate_public_key (:218-246) -> [2, n] = (a, a (*) s + e)."""
        r = self.ring
        sk = _as_u64(sk)
        out = _empty(sk, (2, r.degree)) if out is None else out
        bs, bo = _Buf(sk), _Buf(out, True)
        w = _where(bs, bo)
        r._bind_stream(w)
        _check(lib().fhe_public_key_generate(r._h, bs.ptr, _seed_arr(self.seed), stream, self.noise_std, bo.ptr, w))
        return out

    def eval_key(self, sk, base_log: int, level: int, stream: int, out=None):
        """generate_eval_key (:252-333) -> rlk [level, 2, n] (KeySwitchKey pairs (a_l, b_l))."""
        r = self.ring
        sk = _as_u64(sk)
        out = _empty(sk, (level, 2, r.degree)) if out is None else out
        bs, bo = _Buf(sk), _Buf(out, True)
        w = _where(bs, bo)
        r._bind_stream(w)
        _check(lib().fhe_eval_key_generate(r._h, bs.ptr, base_log, level, _seed_arr(self.seed), stream,
                                           self.noise_std, bo.ptr, w))
        return out

    def ggsw(self, values, sk, k: int, base_log: int, level: int, stream: int, out=None):
        """encrypt_ggsw (bootstrap_engine.cpp:268-306) of int64 values ->
        [count, (k+1) level, k+1, n] coefficient form."""
        r = self.ring
        if _is_tensor(values):
            vals = values.to(torch.int64).contiguous()
        else:
            vals = np.ascontiguousarray(np.asarray(values, dtype=np.int64)).view(np.uint64)
        sk = _as_u64(sk)
        cnt = int(vals.numel() if _is_tensor(vals) else vals.size)
        out = _empty(sk, (cnt, (k + 1) * level, k + 1, r.degree)) if out is None else out
        bv, bs, bo = _Buf(vals), _Buf(sk), _Buf(out, True)
        w = _where(bv, bs, bo)
        r._bind_stream(w)
        _check(lib().fhe_ggsw_encrypt_batch(r._h, k, base_log, level, bv.ptr, cnt, bs.ptr, _seed_arr(self.seed),
                                            stream, self.noise_std, bo.ptr, w))
        return out

    def key_switch_key(self, glwe_sk, lwe_sk, base_log: int, level: int, stream: int, std_dev: float = 0.0):
        """generate_key_switch_key (:367-420) -> (ksk_a [n_in level, dim], ksk_b [n_in level])."""
        r = self.ring
        g = _as_u64(glwe_sk)
        if _is_tensor(lwe_sk):
            ls = lwe_sk.to(torch.int64).contiguous()
        else:
            ls = np.ascontiguousarray(np.asarray(lwe_sk, dtype=np.int64)).view(np.uint64)
        n_in = int(g.numel() if _is_tensor(g) else g.size)
        dim = int(ls.numel() if _is_tensor(ls) else ls.size)
        ka, kb = _empty(g, (n_in * level, dim)), _empty(g, (n_in * level,))
        bg, bl, ba, bb = _Buf(g), _Buf(ls), _Buf(ka, True), _Buf(kb, True)
        w = _where(bg, bl, ba, bb)
        r._bind_stream(w)
        _check(lib().fhe_ksk_generate(r._h, base_log, level, bg.ptr, n_in, bl.ptr, dim, _seed_arr(self.seed), stream,
                                      float(std_dev), ba.ptr, bb.ptr, w))
        return ka, kb


def lwe_decrypt(q: int, t: int, sk, lwe_a, lwe_b, device: int = 0):
    """LWE decryption (fhe_lwe_decrypt_batch): (values [batch], phase [batch])."""
    if _is_tensor(lwe_a):
        skv = sk.to(torch.int64).contiguous() if _is_tensor(sk) else torch.as_tensor(np.asarray(sk, dtype=np.int64),
                                                                                      device=lwe_a.device)
    else:
        skv = np.ascontiguousarray(np.asarray(sk, dtype=np.int64)).view(np.uint64)
    a, b = _as_u64(lwe_a), _as_u64(lwe_b)
    batch = int(b.numel() if _is_tensor(b) else b.size)
    dim = int(skv.numel() if _is_tensor(skv) else skv.size)
    vals, ph = _empty(b, (batch,)), _empty(b, (batch,))
    bs, ba, bb, bv, bp = _Buf(skv), _Buf(a), _Buf(b), _Buf(vals, True), _Buf(ph, True)
    w = _where(bs, ba, bb, bv, bp)
    stream = _stream_ptr(bv.device) if w == FHE_DEVICE else None
    _check(lib().fhe_lwe_decrypt_batch(q, t, bs.ptr, dim, ba.ptr, bb.ptr, bv.ptr, bp.ptr, batch, w, device, stream))
    return vals, ph


class DecryptionResult:
    """Batched DecryptionResult (encryption.h): decoded slot values
    [..., n] (slot 0 is decrypt_value's result), the reference's noise budget
    log2(q / (2 max_noise)) per ciphertext, and success = budget >= 0
    (encryption.cpp:289-295)."""

    def __init__(self, values, max_noise, modulus, phase=None):
        import math

        self.values, self.phase = values, phase
        mx = np.asarray(max_noise.cpu() if _is_tensor(max_noise) else max_noise, dtype=np.uint64)
        self.max_noise = mx
        flat = mx.reshape(-1)
        self.noise_budget = np.array([math.log2(float(modulus) / (2.0 * max(float(int(v)), 1.0))) for v in flat])
        self.noise_budget = self.noise_budget.reshape(mx.shape)
        self.success = self.noise_budget >= 0
        self.error = ["" if ok else "Noise budget exhausted - decryption may be incorrect" for ok in
                      self.success.reshape(-1)]


class EncryptionEngine:
    """Ciphertext arithmetic of EncryptionEngine (encryption.cpp:594-980) over
    batches of ciphertexts [..., 2, n] (c0, c1) / [..., 3, n] (degree 2), and
    encrypt / decrypt / add_plain (:171-348, :638-665) with plaintext modulus
    t (0 selects the reference's default 4, :40-46)."""

    def __init__(self, ring: "PolynomialRing", plaintext_modulus: int = 0):
        self.ring = ring
        self.t = int(plaintext_modulus)
        self.delta = ring.modulus // (self.t or 4)

    def _slots(self, values, nb):
        """Plaintext slot values -> [nb, n] (a scalar or a short vector is
        zero-padded: encode_plaintext / encode_packed, :107-131)."""
        n = self.ring.degree
        if _is_tensor(values):
            v = values.reshape(-1, values.shape[-1]) if values.dim() else values.reshape(1, 1)
            if v.shape[-1] != n:
                pad = torch.zeros((v.shape[0], n), dtype=v.dtype, device=v.device)
                pad[:, : min(n, v.shape[-1])] = v[:, :n]
                v = pad
            if v.shape[0] == 1 and nb > 1:
                v = v.expand(nb, n)
            return v.contiguous()
        v = np.asarray(values, dtype=np.uint64)
        v = v.reshape(1, 1) if v.ndim == 0 else v.reshape(-1, v.shape[-1])
        if v.shape[-1] != n:
            pad = np.zeros((v.shape[0], n), dtype=np.uint64)
            pad[:, : min(n, v.shape[-1])] = v[:, :n]
            v = pad
        if v.shape[0] == 1 and nb > 1:
            v = np.broadcast_to(v, (nb, n))
        return np.ascontiguousarray(v)

    def encrypt(self, values, pk: PublicKey, u, e1, e2, out=None):
        """encrypt_internal (:171-205) with the sampled polynomials supplied:
        u (ternary), e1, e2 (error) [..., n]; values: plaintext slots
        [..., n] (or fewer, zero-padded).  -> ct [..., 2, n]."""
        r = self.ring
        u, e1, e2 = _as_u64(u), _as_u64(e1), _as_u64(e2)
        nb = r._batch(u)
        vals = self._slots(values, nb)
        if out is None:
            out = _empty(u, tuple(u.shape[:-1]) + (2, r.degree))
        bk, bv, bu, b1, b2, bo = _Buf(pk.prep), _Buf(vals), _Buf(u), _Buf(e1), _Buf(e2), _Buf(out, True)
        if not (bv.count == bu.count == b1.count == b2.count == nb * r.degree):
            raise FHEError(-9, "values, u, e1, e2 must all be [batch, n]")
        w = _where(bk, bv, bu, b1, b2, bo)
        r._bind_stream(w)
        _check(lib().fhe_encrypt_batch(r._h, self.t, bk.ptr, bv.ptr, bu.ptr, b1.ptr, b2.ptr, bo.ptr, nb, w))
        return out

    def encrypt_sampled(self, values, pk: PublicKey, seed, stream: int, noise_std: float = 3.2, batch=None,
                        out=None):
        """encrypt_internal (:171-205) with u (ternary), e1, e2 (error) drawn
        on the device from the seeded stream (streams stream .. stream + 2)."""
        r = self.ring
        v = _as_u64(values)
        nb = batch if batch is not None else (r._batch(v) if (v.shape[-1] if len(v.shape) else 0) == r.degree else 1)
        vals = self._slots(values, nb)
        if out is None:
            out = _empty(pk.prep, (nb, 2, r.degree))
        bk, bv, bo = _Buf(pk.prep), _Buf(vals), _Buf(out, True)
        w = _where(bk, bv, bo)
        r._bind_stream(w)
        _check(lib().fhe_encrypt_sampled_batch(r._h, self.t, bk.ptr, bv.ptr, _seed_arr(seed), stream,
                                               float(noise_std), bo.ptr, nb, w))
        return out

    def decrypt(self, ct, sk: SecretKey, is_ntt: bool = False, with_phase: bool = False):
        """decrypt / decrypt_packed (:234-348) for [..., 2, n] or degree-2
        [..., 3, n] ciphertexts -> DecryptionResult."""
        r = self.ring
        ct = _as_u64(ct)
        comps = int(ct.shape[-2]) if len(ct.shape) >= 2 else 0
        if comps not in (2, 3):
            raise FHEError(-9, "ciphertexts must be [..., 2, n] or [..., 3, n]")
        nb = _lead(ct, (comps, r.degree))
        lead = tuple(ct.shape[:-2])
        vals = _empty(ct, lead + (r.degree,))
        mx = _empty(ct, lead if lead else (1,))
        ph = _empty(ct, lead + (r.degree,)) if with_phase else None
        bs, bc, bv, bm = _Buf(sk.prep), _Buf(ct), _Buf(vals, True), _Buf(mx, True)
        bp = _Buf(ph, True) if ph is not None else None
        w = _where(bs, bc, bv, bm, bp)
        r._bind_stream(w)
        _check(lib().fhe_decrypt_batch(r._h, self.t, bs.ptr, bc.ptr, comps, int(bool(is_ntt)), bv.ptr,
                                       bp.ptr if bp else None, bm.ptr, nb, w))
        if _is_tensor(mx):
            torch.cuda.current_stream(mx.device).synchronize()
        return DecryptionResult(vals, mx, r.modulus, ph)

    def decrypt_value(self, ct, sk: SecretKey, is_ntt: bool = False):
        """decrypt_value (:303-310): slot 0, or None where decryption failed."""
        res = self.decrypt(ct, sk, is_ntt)
        v = res.values.cpu().numpy().view(np.uint64) if _is_tensor(res.values) else res.values
        return [int(x) if ok else None for x, ok in zip(v.reshape(-1, self.ring.degree)[:, 0], res.success.reshape(-1))]

    def add_plain(self, ct, values, is_ntt: bool = False, out=None):
        """add_plain (:638-665): (c0 + encode(values), c1)."""
        r = self.ring
        ct = _as_u64(ct)
        nb = _lead(ct, (2, r.degree))
        vals = self._slots(values, nb)
        out = _like(ct) if out is None else out
        bc, bv, bo = _Buf(ct), _Buf(vals), _Buf(out, True)
        w = _where(bc, bv, bo)
        r._bind_stream(w)
        _check(lib().fhe_add_plain_batch(r._h, self.t, bc.ptr, bv.ptr, int(bool(is_ntt)), bo.ptr, nb, w))
        return out

    def _pair(self, ct1, ct2):
        ct1, ct2 = _as_u64(ct1), _as_u64(ct2)
        _lead(ct1, (2, self.ring.degree))
        if tuple(ct2.shape) != tuple(ct1.shape):
            raise FHEError(-9, "ciphertext shapes differ")
        return ct1, ct2

    def add(self, ct1, ct2, out=None):
        """add (:594-617): componentwise mod_add of (c0, c1)."""
        ct1, ct2 = self._pair(ct1, ct2)
        return self.ring.add(ct1, ct2, out)

    def subtract(self, ct1, ct2, out=None):
        """subtract (:692-714)."""
        ct1, ct2 = self._pair(ct1, ct2)
        return self.ring.subtract(ct1, ct2, out)

    def negate(self, ct, out=None):
        """negate (:716-727)."""
        ct = _as_u64(ct)
        _lead(ct, (2, self.ring.degree))
        return self.ring.negate(ct, out)

    def multiply_scalar(self, ct, scalar: int, out=None):
        """multiply_scalar (:890-902)."""
        ct = _as_u64(ct)
        _lead(ct, (2, self.ring.degree))
        return self.ring.multiply_scalar(ct, scalar, out)

    def multiply_plain(self, ct, pt, out=None):
        """multiply_plain (:809-850) for an already-encoded plaintext
        polynomial pt [..., n] (one per ciphertext, or one for all): each
        component times pt through the fused polymul (coefficient form)."""
        r = self.ring
        ct = _as_u64(ct)
        nb = _lead(ct, (2, r.degree))
        pt = _as_u64(pt)
        if _is_tensor(ct):
            ptb = pt.reshape(-1, 1, r.degree).expand(nb, 2, r.degree).reshape(ct.shape).contiguous()
        else:
            ptb = np.ascontiguousarray(np.broadcast_to(np.asarray(pt).reshape(-1, 1, r.degree),
                                                       (nb, 2, r.degree)).reshape(ct.shape))
        return r.multiply(ct, ptb, out)

    def multiply(self, ct1, ct2, is_ntt: bool = False, out=None):
        """multiply (:737-798): tensor product -> [..., 3, n]."""
        r = self.ring
        ct1, ct2 = _as_u64(ct1), _as_u64(ct2)
        nb = _lead(ct1, (2, r.degree))
        if tuple(ct2.shape) != tuple(ct1.shape):
            raise FHEError(-9, "ciphertext shapes differ")
        if out is None:
            out = _empty(ct1, tuple(ct1.shape[:-2]) + (3, r.degree))
        b1, b2, bo = _Buf(ct1), _Buf(ct2), _Buf(out, True)
        w = _where(b1, b2, bo)
        r._bind_stream(w)
        _check(lib().fhe_ct_multiply_batch(r._h, b1.ptr, b2.ptr, bo.ptr, nb, int(bool(is_ntt)), w))
        return out

    def relinearize(self, ct3, ek: EvaluationKey, out=None):
        """relinearize (:904-980): [..., 3, n] -> [..., 2, n]; a degree-1
        input [..., 2, n] is returned as a copy (:906-909)."""
        r = self.ring
        ct3 = _as_u64(ct3)
        if len(ct3.shape) >= 2 and tuple(ct3.shape[-2:]) == (2, r.degree):
            if out is None:
                return ct3.clone() if _is_tensor(ct3) else ct3.copy()
            out[...] = ct3
            return out
        nb = _lead(ct3, (3, r.degree))
        if out is None:
            out = _empty(ct3, tuple(ct3.shape[:-2]) + (2, r.degree))
        bi, bk, bo = _Buf(ct3), _Buf(ek.rlk_ntt), _Buf(out, True)
        w = _where(bi, bo) if not ek.level else _where(bi, bk, bo)
        r._bind_stream(w)
        _check(lib().fhe_relinearize_batch(r._h, ek.decomp_base_log, ek.level, bi.ptr, bk.ptr if ek.level else None,
                                           bo.ptr, nb, w))
        return out

    def multiply_relin(self, ct1, ct2, ek: EvaluationKey, out=None):
        """multiply_relin (:800-807)."""
        r = self.ring
        ct1, ct2 = _as_u64(ct1), _as_u64(ct2)
        nb = _lead(ct1, (2, r.degree))
        if tuple(ct2.shape) != tuple(ct1.shape):
            raise FHEError(-9, "ciphertext shapes differ")
        out = _like(ct1) if out is None else out
        b1, b2, bk, bo = _Buf(ct1), _Buf(ct2), _Buf(ek.rlk_ntt), _Buf(out, True)
        w = _where(b1, b2, bo) if not ek.level else _where(b1, b2, bk, bo)
        r._bind_stream(w)
        _check(lib().fhe_ct_multiply_relin_batch(r._h, ek.decomp_base_log, ek.level, b1.ptr, b2.ptr,
                                                 bk.ptr if ek.level else None, bo.ptr, nb, w))
        return out


class BootstrapEngine:
    """The TFHE pieces of BootstrapEngine (bootstrap_engine.cpp) batched over
    ciphertexts: GLWE [..., k+1, n], GGSW [(k+1)*level, k+1, n], LWE masks
    [..., dim] with bodies [...]."""

    def __init__(self, ring: NTTProcessor, base_log: int, level: int, k: int = 1):
        self.ring, self.base_log, self.level, self.k = ring, base_log, level, k

    def prepare_ggsw(self, ggsw):
        """GGSW(s) [..., (k+1)*level, k+1, n] -> NTT-domain form (same shape)."""
        r, k, L = self.ring, self.k, self.level
        g = _as_u64(ggsw)
        nb = _lead(g, ((k + 1) * L, k + 1, r.degree))
        out = _like(g)
        bi, bo = _Buf(g), _Buf(out, True)
        w = _where(bi, bo)
        r._bind_stream(w)
        _check(lib().fhe_ggsw_prepare(r._h, k, L * nb, bi.ptr, bo.ptr, w))
        return out

    def external_product(self, glwe, ggsw_ntt, out=None):
        r = self.ring
        glwe = _as_u64(glwe)
        nb = _lead(glwe, (self.k + 1, r.degree))
        out = _like(glwe) if out is None else out
        bi, bk, bo = _Buf(glwe), _Buf(ggsw_ntt), _Buf(out, True)
        w = _where(bi, bk, bo)
        r._bind_stream(w)
        _check(lib().fhe_external_product_batch(r._h, self.k, self.base_log, self.level, bi.ptr, bk.ptr, bo.ptr,
                                                nb, w))
        return out

    def cmux(self, ggsw_ntt, ct0, ct1, out=None):
        """cmux (:520-540): ct0 + ggsw (x) (ct1 - ct0)."""
        r = self.ring
        ct0, ct1 = _as_u64(ct0), _as_u64(ct1)
        nb = _lead(ct0, (self.k + 1, r.degree))
        if tuple(ct1.shape) != tuple(ct0.shape):
            raise FHEError(-9, "ciphertext shapes differ")
        out = _like(ct0) if out is None else out
        bg, b0, b1, bo = _Buf(ggsw_ntt), _Buf(ct0), _Buf(ct1), _Buf(out, True)
        w = _where(bg, b0, b1, bo)
        r._bind_stream(w)
        _check(lib().fhe_cmux_batch(r._h, self.k, self.base_log, self.level, bg.ptr, b0.ptr, b1.ptr, bo.ptr, nb, w))
        return out

    def multiply_glwe_by_monomial(self, glwe, rotation, out=None):
        """multiply_glwe_by_monomial (:249-261); rotation: one int per ciphertext."""
        r = self.ring
        glwe = _as_u64(glwe)
        nb = _lead(glwe, (self.k + 1, r.degree))
        if _is_tensor(glwe):
            rot = torch.as_tensor(rotation, dtype=torch.int32, device=glwe.device).reshape(-1).contiguous()
            rp = rot.data_ptr()
        else:
            rot = np.ascontiguousarray(np.asarray(rotation, dtype=np.int32).reshape(-1))
            rp = rot.ctypes.data
        cnt = rot.numel() if _is_tensor(rot) else rot.size
        if cnt != nb:
            raise FHEError(-9, "one rotation per ciphertext")
        out = _like(glwe) if out is None else out
        bi, bo = _Buf(glwe), _Buf(out, True)
        w = _where(bi, bo)
        r._bind_stream(w)
        _check(lib().fhe_glwe_rotate_batch(r._h, self.k, rp, bi.ptr, bo.ptr, nb, w))
        return out

    def blind_rotate(self, acc, lwe_a, lwe_b, bsk_ntt, lwe_q: Optional[int] = None):
        """blind_rotate (:547-577), in place on acc [..., k+1, n]; lwe_a
        [..., dim], lwe_b [...]; bsk_ntt [dim, (k+1)*level, k+1, n] from
        prepare_ggsw.  lwe_q defaults to the ring modulus (:39-40)."""
        r = self.ring
        acc, lwe_a, lwe_b = _as_u64(acc), _as_u64(lwe_a), _as_u64(lwe_b)
        nb = _lead(acc, (self.k + 1, r.degree))
        dim = int(lwe_a.shape[-1])
        ba, bla, blb, bk = _Buf(acc, True), _Buf(lwe_a), _Buf(lwe_b), _Buf(bsk_ntt)
        if bla.count != nb * dim or blb.count != nb:
            raise FHEError(-9, "LWE masks must be [batch, dim] and bodies [batch]")
        w = _where(ba, bla, blb, bk)
        r._bind_stream(w)
        _check(lib().fhe_blind_rotate_batch(r._h, self.k, self.base_log, self.level, dim, bla.ptr, blb.ptr,
                                            lwe_q if lwe_q is not None else r.modulus, bk.ptr, ba.ptr, nb, w))
        return acc

    def repair_count(self) -> int:
        """Ciphertexts of this ring's two-CU blind rotations recomputed on one
        CU because a partner workgroup was not co-resident in time
        (fhe_br_repair_count; waits for the ring's stream)."""
        v = C.c_uint64(0)
        _check(lib().fhe_br_repair_count(self.ring._h, C.byref(v)))
        return int(v.value)

    def bootstrap(self, lwe_a, lwe_b, bsk_ntt, test_poly, ksk_a, ksk_b, ks_base_log: int, ks_level: int,
                  lwe_q: Optional[int] = None):
        """bootstrap_with_test_poly (bootstrap_engine.cpp:684-708) for a batch
        of LWE ciphertexts (lwe_a [..., dim], lwe_b [...]): blind rotation of
        (0, test_poly), sample extract, key switch (ksk_a [k*n*ks_level,
        out_dim], ksk_b [k*n*ks_level]).  -> (a [..., out_dim], b [...])."""
        r = self.ring
        lwe_a, lwe_b, test_poly, ksk_a, ksk_b = (_as_u64(x) for x in (lwe_a, lwe_b, test_poly, ksk_a, ksk_b))
        dim = int(lwe_a.shape[-1])
        nb = _lead(lwe_a, (dim,))
        out_dim = int(ksk_a.shape[-1])
        out_a = _empty(lwe_a, tuple(lwe_a.shape[:-1]) + (out_dim,))
        out_b = _like(lwe_b)
        bla, blb, bk, bt, bka, bkb, boa, bob = (_Buf(lwe_a), _Buf(lwe_b), _Buf(bsk_ntt), _Buf(test_poly), _Buf(ksk_a),
                                                _Buf(ksk_b), _Buf(out_a, True), _Buf(out_b, True))
        if blb.count != nb or bt.count != r.degree or bkb.count != self.k * r.degree * ks_level or \
                bka.count != bkb.count * out_dim:
            raise FHEError(-9, "LWE / test polynomial / key-switching key shapes disagree")
        w = _where(bla, blb, bk, bt, bka, bkb, boa, bob)
        r._bind_stream(w)
        _check(lib().fhe_bootstrap_batch(r._h, self.k, self.base_log, self.level, dim, bla.ptr, blb.ptr,
                                         lwe_q if lwe_q is not None else r.modulus, bk.ptr, bt.ptr, ks_base_log,
                                         ks_level, out_dim, bka.ptr, bkb.ptr, boa.ptr, bob.ptr, nb, w))
        return out_a, out_b

    programmable_bootstrap = bootstrap  # :716-722: the lookup table's polynomial as test_poly

    def create_lookup_table(self, func, input_modulus: int, output_modulus: int):
        """create_lookup_table (bootstrap_engine.cpp:725-758): the test
        polynomial encoding func (host-side, O(n))."""
        n, q = self.ring.degree, self.ring.modulus
        delta_out = q // output_modulus
        coeffs = np.zeros(n, dtype=np.uint64)
        for i in range(n):
            v = ((i * input_modulus + n) // (2 * n)) % input_modulus
            coeffs[i] = ((int(func(v)) % output_modulus) * delta_out) % q
        return coeffs

    def sample_extract(self, glwe):
        """sample_extract (:594-624) -> (a [..., k*n], b [...])."""
        r = self.ring
        glwe = _as_u64(glwe)
        nb = _lead(glwe, (self.k + 1, r.degree))
        lead = tuple(glwe.shape[:-2])
        a = _empty(glwe, lead + (self.k * r.degree,))
        b = _empty(glwe, lead if lead else (1,))
        bi, ba, bb = _Buf(glwe), _Buf(a, True), _Buf(b, True)
        w = _where(bi, ba, bb)
        r._bind_stream(w)
        _check(lib().fhe_sample_extract_batch(r._h, self.k, bi.ptr, ba.ptr, bb.ptr, nb, w))
        return a, b

    @staticmethod
    def key_switch(q: int, base_log: int, level: int, ksk_a, ksk_b, lwe_a, lwe_b, device: int = 0):
        """key_switch (:626-674): ksk_a [in_dim*level, out_dim], ksk_b
        [in_dim*level]; lwe_a [..., in_dim], lwe_b [...] -> (a, b)."""
        ksk_a, ksk_b, lwe_a, lwe_b = (_as_u64(x) for x in (ksk_a, ksk_b, lwe_a, lwe_b))
        in_dim = int(lwe_a.shape[-1])
        out_dim = int(ksk_a.shape[-1])
        nb = _lead(lwe_a, (in_dim,))
        out_a = _empty(lwe_a, tuple(lwe_a.shape[:-1]) + (out_dim,))
        out_b = _like(lwe_b)
        bka, bkb, bla, blb, boa, bob = (_Buf(ksk_a), _Buf(ksk_b), _Buf(lwe_a), _Buf(lwe_b), _Buf(out_a, True),
                                        _Buf(out_b, True))
        if bka.count != in_dim * level * out_dim or bkb.count != in_dim * level or blb.count != nb:
            raise FHEError(-9, "key switching key / LWE shapes disagree")
        w = _where(bka, bkb, bla, blb, boa, bob)
        s = _stream_ptr() if w == FHE_DEVICE else None
        _check(lib().fhe_key_switch_batch(q, base_log, level, in_dim, out_dim, bka.ptr, bkb.ptr, bla.ptr, blb.ptr,
                                          boa.ptr, bob.ptr, nb, w, device, s))
        return out_a, out_b


def decompose_polynomial(ring: NTTProcessor, poly, base_log: int, level: int, out=None):
    """BootstrapEngine::decompose_polynomial (bootstrap_engine.cpp:152-185);
    poly [..., n] -> [..., level, n]."""
    poly = _as_u64(poly)
    nb = ring._batch(poly)
    if out is None:
        shape = tuple(poly.shape[:-1]) + (level, ring.degree)
        out = torch.empty(shape, dtype=poly.dtype, device=poly.device) if _is_tensor(poly) else np.empty(
            shape, dtype=np.uint64)
    bi, bo = _Buf(poly), _Buf(out, True)
    w = _where(bi, bo)
    ring._bind_stream(w)
    _check(lib().fhe_decompose_batch(ring._h, base_log, level, bi.ptr, bo.ptr, nb, w))
    return out


# ----------------------------------------------------------------- modular arithmetic
def modmul_batch(q: int, a, b, out=None, device: int = 0):
    """BarrettReducer::barrett_mul contract, batched on the GPU: a*b mod q."""
    a, b = _as_u64(a), _as_u64(b)
    out = _like(a) if out is None else out
    ba, bb, bo = _Buf(a), _Buf(b), _Buf(out, True)
    if not (ba.count == bb.count == bo.count):
        raise FHEError(-9, "operand sizes differ")
    w = _where(ba, bb, bo)
    s = _stream_ptr() if w == FHE_DEVICE else None
    _check(lib().fhe_modmul_batch(q, ba.ptr, bb.ptr, bo.ptr, ba.count, w, device, s))
    return out


class BarrettReducer:
    """BarrettReducer(modulus) (modular_arithmetic.cpp:238-280)."""

    def __init__(self, modulus: int):
        if modulus == 0:
            raise FHEError(-8, "Modulus must be non-zero for Barrett reduction")
        self.modulus = modulus

    def barrett_mul_batch(self, a, b, out=None, device: int = 0):
        return modmul_batch(self.modulus, a, b, out, device)

    def barrett_mul(self, a: int, b: int) -> int:
        return int(self.barrett_mul_batch(np.array([a], np.uint64), np.array([b], np.uint64))[0])


class MultiLimbModularArithmetic:
    """2-limb MultiLimbModularArithmetic (modular_arithmetic.cpp:471-693)."""

    def __init__(self, modulus_limbs):
        self.q = (C.c_uint64 * 2)(*[int(x) for x in modulus_limbs])
        k = (C.c_uint64 * 7)()
        _check(lib().fhe_ml_constants(self.q, k))
        self.constants = list(k)

    def montgomery_mul_batch(self, a, b, out=None, device: int = 0):
        """a, b: [..., 2] little-endian limbs."""
        a, b = _as_u64(a), _as_u64(b)
        out = _like(a) if out is None else out
        ba, bb, bo = _Buf(a), _Buf(b), _Buf(out, True)
        if ba.count % 2 or not (ba.count == bb.count == bo.count):
            raise FHEError(-9, "operands must be [..., 2] limb arrays of equal size")
        w = _where(ba, bb, bo)
        s = _stream_ptr() if w == FHE_DEVICE else None
        _check(lib().fhe_ml_montmul_batch(self.q, ba.ptr, bb.ptr, bo.ptr, ba.count // 2, w, device, s))
        return out


class ModularArithmetic:
    """The N-API ``ModularArithmetic`` class (index.d.ts:32-44,
    src/native/lib.rs:42-121) with the reference's exact constants."""

    def __init__(self, modulus: int):
        if modulus <= 0:
            raise FHEError(-9, "Modulus must be positive")
        self._k = (C.c_uint64 * 4)()
        _check(lib().fhe_mont_constants_compat(modulus, self._k))
        self.modulus = modulus

    @staticmethod
    def _nn(*xs):
        for x in xs:
            if x < 0:
                raise FHEError(-9, "Inputs must be non-negative")

    def montgomery_mul(self, a, b):
        self._nn(a, b)
        return lib().fhe_compat_montgomery_mul(self._k, a, b)

    def mod_add(self, a, b):
        self._nn(a, b)
        return lib().fhe_compat_mod_add(self.modulus, a, b)

    def mod_sub(self, a, b):
        self._nn(a, b)
        return lib().fhe_compat_mod_sub(self.modulus, a, b)

    def to_montgomery(self, a):
        self._nn(a)
        return lib().fhe_compat_to_montgomery(self._k, a)

    def from_montgomery(self, a):
        self._nn(a)
        return lib().fhe_compat_from_montgomery(self._k, a)

    def get_modulus(self):
        return self.modulus

    @property
    def constants(self):
        return list(self._k)


# ----------------------------------------------------------------- timing helper
class HipEvent:
    """hipEvent on an explicit stream (for kernel timing in bench.py)."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().fhe_event_create(C.byref(h)))
        self._h = h

    def record(self, stream_ptr):
        _check(lib().fhe_event_record(self._h, C.c_void_p(stream_ptr)))

    def elapsed_ms(self, end: "HipEvent") -> float:
        ms = C.c_float()
        _check(lib().fhe_event_elapsed_ms(self._h, end._h, C.byref(ms)))
        return ms.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.fhe_event_destroy(h)
