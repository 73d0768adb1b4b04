"""Independent big-integer restatement (TEST INFRASTRUCTURE ONLY).

A second, independently written oracle used to cross-check ``ref_cpu.c``.  It
follows the reference's own TypeScript restatement of the C++ transform,
``src/test-utils/ntt-round-trip.prop.test.ts:156-244`` (forward Cooley-Tukey
with twiddle ``psi^(j*n/groupSize)`` after a bit-reversal, inverse
Gentleman-Sande + bit-reversal + N^-1), its primitive-root search
(``findPrimitiveRoot``) and the negacyclic reference of
``src/test-utils/homomorphic-multiplication.prop.test.ts:126-189`` / schoolbook
convolution.  Pure Python ints: only for small cases.
"""
from __future__ import annotations


def mod_pow(b, e, m):
    return pow(b, e, m)


def find_psi(n, q):
    two_n = 2 * n
    if (q - 1) % two_n:
        raise ValueError("not NTT-friendly")
    e = (q - 1) // two_n
    g = 2
    while g < q:
        w = pow(g, e, q)
        if pow(w, two_n, q) == 1 and pow(w, n, q) == q - 1:
            return w
        g += 1
    raise ValueError("no root")


def bitrev(i, bits):
    r = 0
    for _ in range(bits):
        r = (r << 1) | (i & 1)
        i >>= 1
    return r


def _bitrev_perm(a):
    n = len(a)
    bits = n.bit_length() - 1
    return [a[bitrev(i, bits)] for i in range(n)]


def forward(coeffs, q):
    n = len(coeffs)
    logn = n.bit_length() - 1
    psi = find_psi(n, q)
    tw = [pow(psi, i, q) for i in range(n)]
    r = _bitrev_perm([c % q for c in coeffs])
    for s in range(logn):
        m = 1 << s
        gs = 2 * m
        for k in range(0, n, gs):
            for j in range(m):
                w = tw[j * (n // gs)]
                a, b = r[k + j], r[k + j + m]
                wb = (w * b) % q
                r[k + j] = (a + wb) % q
                r[k + j + m] = (a - wb) % q
    return r


def inverse(coeffs, q):
    n = len(coeffs)
    logn = n.bit_length() - 1
    psi = find_psi(n, q)
    pinv = pow(psi, -1, q)
    tw = [pow(pinv, i, q) for i in range(n)]
    r = [c % q for c in coeffs]
    for s in range(logn - 1, -1, -1):
        m = 1 << s
        gs = 2 * m
        for k in range(0, n, gs):
            for j in range(m):
                w = tw[j * (n // gs)]
                a, b = r[k + j], r[k + j + m]
                r[k + j] = (a + b) % q
                r[k + j + m] = ((a - b) * w) % q
    r = _bitrev_perm(r)
    ninv = pow(n, -1, q)
    return [(c * ninv) % q for c in r]


def polymul(a, b, q):
    fa, fb = forward(a, q), forward(b, q)
    return inverse([(x * y) % q for x, y in zip(fa, fb)], q)


def negacyclic_schoolbook(a, b, q):
    n = len(a)
    c = [0] * n
    for i in range(n):
        for j in range(n):
            k = i + j
            if k < n:
                c[k] = (c[k] + a[i] * b[j]) % q
            else:
                c[k - n] = (c[k - n] - a[i] * b[j]) % q
    return c


def negacyclic_forward(coeffs, q):
    """homomorphic-multiplication.prop.test.ts:126-189: twist by psi^i, then a
    cyclic DIT with omega = psi^2 (bit-reversed input, natural output)."""
    n = len(coeffs)
    logn = n.bit_length() - 1
    psi = find_psi(n, q)
    omega = psi * psi % q
    r = [(c % q) * pow(psi, i, q) % q for i, c in enumerate(coeffs)]
    r = _bitrev_perm(r)
    for s in range(logn):
        m = 1 << s
        gs = 2 * m
        wm = pow(omega, n // gs, q)
        for k in range(0, n, gs):
            w = 1
            for j in range(m):
                a, b = r[k + j], r[k + j + m] * w % q
                r[k + j] = (a + b) % q
                r[k + j + m] = (a - b) % q
                w = w * wm % q
    return r


def negacyclic_inverse(vals, q):
    n = len(vals)
    logn = n.bit_length() - 1
    psi = find_psi(n, q)
    omega_inv = pow(psi * psi % q, -1, q)
    r = _bitrev_perm([v % q for v in vals])
    for s in range(logn):
        m = 1 << s
        gs = 2 * m
        wm = pow(omega_inv, n // gs, q)
        for k in range(0, n, gs):
            w = 1
            for j in range(m):
                a, b = r[k + j], r[k + j + m] * w % q
                r[k + j] = (a + b) % q
                r[k + j + m] = (a - b) % q
                w = w * wm % q
    ninv = pow(n, -1, q)
    pinv = pow(psi, -1, q)
    return [r[i] * ninv % q * pow(pinv, i, q) % q for i in range(n)]
