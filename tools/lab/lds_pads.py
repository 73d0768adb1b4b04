#!/usr/bin/env python3
"""Bank-conflict simulator for the padded LDS exchange layouts of
ntt_core.hpp (lab tool: picks kPadA/kPadB per (logN, logE)).

Model (MI355X_MICROARCH.md, LDS): ds_read_b32 / ds_write_b32 serve a wave64
in two 32-lane groups; bank = word mod 32; each extra distinct address on a
busy bank adds one cycle.  Element i lives at word pad(i) = i + (i>>A) + (i>>B)
[+ (i>>C)].  Pass p of a transform owns, per lane tau and slot group u, the
elements lay(g) | (t << S), t < 2^R, g = brv(tau) (pass 0) or tau + u*T.

usage: lds_pads.py LOGN LOGE [--u64] [--eval A B [C]]
"""
import itertools
import sys


def brv(x, bits):
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def geo(L, LE):
    LE = min(LE, L)
    T = 1 << (L - LE)
    NP = (L + LE - 1) // LE
    return T, NP, [min(LE, L - p * LE) for p in range(NP)], LE


def patterns(L, LE):
    """Per pass: list of instructions, each a list of element indices by lane tau."""
    T, NP, Rs, LE = geo(L, LE)
    E = 1 << LE
    out = []
    for p in range(NP):
        S, R = p * LE, Rs[p]
        NU = E >> R
        insts = []
        for u in range(NU):
            for t in range(1 << R):
                els = []
                for tau in range(T):
                    g = brv(tau, L - LE) if p == 0 else tau + u * T
                    lay = (g & ((1 << S) - 1)) | ((g >> S) << (S + R))
                    els.append(lay | (t << S))
                insts.append(els)
        out.append(insts)
    return out


def cost(pats, pads, T, wide=False):
    """wide: 8-byte words (ds_read_b64: 32-lane groups, 64 banks; ds_write_b64:
    16-lane groups, 32 banks; each access covers two consecutive dwords)."""
    def pad(i):
        return i + sum(i >> a for a in pads if a)

    extra = 0
    groups = ((32, 64), (16, 32)) if wide else ((32, 32),)
    for insts in pats:
        for els in insts:
            for gsz, nb in groups:
                for g0 in range(0, T, gsz):
                    lanes = els[g0:g0 + gsz]
                    if not lanes:
                        continue
                    banks = {}
                    for e in lanes:
                        dw = 2 * pad(e) if wide else pad(e)
                        for d in ((dw, dw + 1) if wide else (dw,)):
                            banks.setdefault(d % nb, set()).add(d)
                    extra += max(len(s) for s in banks.values()) - 1
    return extra


def main():
    L, LE = int(sys.argv[1]), int(sys.argv[2])
    wide = "--u64" in sys.argv
    T, NP, Rs, LE = geo(L, LE)
    pats = patterns(L, LE)
    if "--eval" in sys.argv:
        pads = [int(x) for x in sys.argv[sys.argv.index("--eval") + 1:] if not x.startswith("--")]
        print("pads", pads, "extra cycles per (all passes store+load once):", cost(pats, pads, T, wide))
        return
    res = []
    for A, B in itertools.combinations_with_replacement(range(0, L + 1), 2):
        if A and B and A == B:
            continue
        res.append((cost(pats, [A, B], T, wide), A, B))
    res.sort()
    for r in res[:12]:
        words = (1 << L) - 1 + sum(((1 << L) - 1) >> a for a in r[1:] if a) + 1
        print(f"extra={r[0]:6d} A={r[1]:2d} B={r[2]:2d} words={words}")


if __name__ == "__main__":
    main()
