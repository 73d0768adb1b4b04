"""Parameter presets of the reference (cpp/src/parameter_set.cpp:22-42 prime
table, :108-287 presets, :291-306 create_parameter_set) as plain data, plus
what the MI355X kernels can run for each.

The reference's prime table is not all prime:
Q_40_1 = 2^40 + 1 = 257 * 4278255361, Q_40_2 and Q_50_2 are composite, and
Q_50_1 only admits N <= 8192.  ``gpu_moduli(preset)`` reports, per modulus,
whether an NTT context of the preset's degree can be created (q odd, q = 1 mod
2N, a primitive 2N-th root exists, q < 2^62) -- the same checks
NTTProcessor's constructor makes (ntt_processor.cpp:134-160).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

# parameter_set.cpp:22-42
Q_60_1 = 1152921504606584833
Q_60_2 = 1152921504598720513
Q_60_3 = 1152921504597016577
Q_50_1 = 1125899906826241
Q_50_2 = 1125899906793473
Q_40_1 = 1099511627777
Q_40_2 = 1099511562241
Q_30_1 = 1073479681
Q_30_2 = 1073217537
Q_TFHE_BOOT = 4294967296


@dataclass(frozen=True)
class ParameterSet:
    name: str
    scheme: str
    security_bits: int
    poly_degree: int
    moduli: List[int] = field(default_factory=list)
    lwe_dimension: int = 0
    lwe_noise_std: float = 0.0
    glwe_dimension: int = 1
    decomp_base_log: int = 0
    decomp_level: int = 0
    plaintext_modulus: int = 0


PRESETS = {
    # :108-137
    "tfhe-128-fast": ParameterSet("tfhe-128-fast", "TFHE", 128, 1024, [Q_40_1], 742, 3.2e-11, 1, 23, 1, 4),
    # :139-164
    "tfhe-128-balanced": ParameterSet("tfhe-128-balanced", "TFHE", 128, 2048, [Q_50_1], 830, 2.9e-11, 1, 15, 2, 8),
    # :166-191
    "tfhe-256-secure": ParameterSet("tfhe-256-secure", "TFHE", 256, 4096, [Q_60_1], 1024, 2.0e-12, 1, 10, 3, 16),
    # :193-224
    "bfv-128-simd": ParameterSet("bfv-128-simd", "BFV", 128, 8192, [Q_60_1, Q_60_2, Q_60_3], 0, 3.2, 1, 60, 3, 65537),
    # :226-259
    "ckks-128-ml": ParameterSet("ckks-128-ml", "CKKS", 128, 16384, [Q_60_1, Q_50_1, Q_50_2, Q_40_1, Q_40_2], 0, 3.2,
                                1, 40, 5, 1 << 40),
    # :261-289
    "tfhe-128-voting": ParameterSet("tfhe-128-voting", "TFHE", 128, 1024, [Q_40_1], 742, 3.2e-11, 1, 23, 1, 4),
}


def create_parameter_set(preset_name: str) -> ParameterSet:
    """create_parameter_set (parameter_set.cpp:291-306)."""
    try:
        return PRESETS[preset_name]
    except KeyError:
        raise ValueError("Unknown parameter preset: " + preset_name) from None


def _is_prime(n: int) -> bool:  # deterministic Miller-Rabin for n < 3.3e24
    if n < 2:
        return False
    small = (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41)
    for p in small:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in small:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def gpu_moduli(preset: ParameterSet) -> List[dict]:
    """Per modulus of `preset`: can an MI355X NTT context of its degree be built?"""
    out = []
    n = preset.poly_degree
    for q in preset.moduli:
        reason = None
        if q % 2 == 0:
            reason = "Modulus must be odd"
        elif (q - 1) % (2 * n):
            reason = "Modulus is not NTT-friendly: q != 1 (mod 2N)"
        elif not _is_prime(q):
            reason = "composite modulus: no primitive 2N-th root search terminates (reference loops to q)"
        elif q >> 62:
            reason = "q >= 2^62 (GPU kernels implement q < 2^62)"
        out.append({"q": q, "prime": _is_prime(q), "usable": reason is None, "reason": reason})
    return out
