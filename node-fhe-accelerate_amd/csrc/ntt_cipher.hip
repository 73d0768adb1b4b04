// ntt_cipher.hip -- ciphertext x ciphertext multiplication
// (EncryptionEngine::multiply, encryption.cpp:737-798) for coefficient-form
// ciphertexts, one kernel per batch:
//
//   X0 = fwd(ct1.c0)  X1 = fwd(ct1.c1)  Y0 = fwd(ct2.c0)  Y1 = fwd(ct2.c1)
//   c0 = inv(X0 Y0)   c1 = inv(X0 Y1 + X1 Y0)   c2 = inv(X1 Y1)
//
// The reference runs 4 forward + 3 inverse transforms on cloned
// polynomials, 4 pointwise products and an add, each a separate pass over
// memory.  Here one workgroup owns one ciphertext pair and runs the 7
// transforms back to back through registers and LDS; the inputs are read
// once and the three outputs written once (56 B per coefficient).  Because
// all products are exact over Z_q, inv(X0 Y1) + inv(X1 Y0) == inv(X0 Y1 +
// X1 Y0) bit for bit.
//
// Between transforms a thread only touches its own positions (the last
// forward pass layout), so three spectra are parked in "slots" without
// synchronisation: LDS when it fits next to the exchange buffer, otherwise
// rows 1 and 2 of this ciphertext's own output (overwritten last) and LDS or
// registers for the third.  Schedule:
//   1. fwd(x0)            -> A = X0
//   2. fwd(y0)  = Y0      -> B = Y0,  c0 = inv(A Y0)               (row 0)
//   3. fwd(x1)  = X1      -> C = X1 B (part of c1),  B = X1
//   4. fwd(y1)  = Y1      -> c1 = C + A Y1,  C = B Y1 (= c2 spectrum)
//                            inv(c1) -> row 1, inv(C) -> row 2
// Products are Montgomery (x R^-1); the R is folded into the inverse's N^-1
// (ninv_r), as in k_polymul.
// streamed twiddles in the paired transforms (ntt_core.hpp FHE_STREAM_TW2):
// 4.61 vs 4.67 ms per 16,384 ciphertext pairs (profiles/r3e/ab.txt)
#ifndef FHE_STREAM_TW2
#define FHE_STREAM_TW2 1
#endif
// Each transform of the 32-bit kernels re-loads its wave-uniform twiddles
// (ntt_core.hpp opaque_tw): k_ct_mul2<1294, u32> 142 -> 10 spilled SGPRs,
// 13 -> 5 spilled VGPRs (round 6).
#ifndef FHE_OPAQUE_TW
#define FHE_OPAQUE_TW 2
#endif
// Flag-free 64-bit arithmetic with the carry-free mulhi in this unit (as in
// ntt_inv.hip; fhe_arith.hpp FHE_U64_NOVCC, FHE_MULHI64=4): fewer static VALU
// issue cycles in its 64-bit kernels and fewer of them with scratch (round 6,
// DESIGN.md section 5).
#ifndef FHE_U64_NOVCC
#define FHE_U64_NOVCC 1
#endif
#ifndef FHE_MULHI64
#define FHE_MULHI64 4
#endif
#include "fhe_internal.hpp"

namespace FHE_NS {

// Slots held in LDS: 3 (all), 1 (C only; A, B in HBM rows) or 0 (C in VGPRs).
#ifndef FHE_CTMUL_PREFER_REGS
#define FHE_CTMUL_PREFER_REGS 1
#endif
template <int LOGN, typename W>
constexpr int ctmul_lds_slots() {
    using G = Geo<LOGN>;
    // slots A/B in VGPRs and C in LDS keeps more workgroups resident than all
    // three in LDS (e.g. N=8192/u32: 2 workgroups per CU instead of 1)
    if (FHE_CTMUL_PREFER_REGS && G::P == 1 && (G::LW + G::N) * (int)sizeof(W) <= 160 * 1024) return 1;
    if (G::P * (G::LW + 3 * G::N) * (int)sizeof(W) <= 160 * 1024) return 3;
    if (G::P * (G::LW + G::N) * (int)sizeof(W) <= 160 * 1024) return 1;
    return 0;
}
template <int LOGN, typename W>
constexpr int ctmul_occ() {
    constexpr int NL = ctmul_lds_slots<LOGN, W>();
    return Geo<LOGN>::template occ_waves<W, NL * Geo<LOGN>::P * Geo<LOGN>::N>();
}

template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (ctmul_occ<LOGN, W>()))
k_ct_mul(const uint64_t *__restrict__ x, const uint64_t *__restrict__ y, uint64_t *out, size_t batch,
         NttArgs<W> A) {
    using G = Geo<LOGN>;
    constexpr int NL = ctmul_lds_slots<LOGN, W>();
    __shared__ W lds_all[G::P * G::LW + NL * G::P * G::N];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < batch;
    if (G::P == 1 && !valid) return;  // whole workgroup: no barrier is skipped
    W *lds = lds_all + pl * G::LW;
    const uint64_t *xr = x + poly * 2 * G::N, *yr = y + poly * 2 * G::N;
    uint64_t *orow = out + poly * 3 * G::N;
    W creg[NL == 0 ? G::E : 1];
    // NL == 1 (u32, N = 16384: one workgroup per CU, 128 VGPRs): slots A
    // and B stay in VGPRs instead of HBM rows (measured: A alone +6 %)
#ifndef FHE_CTMUL_AREG
#define FHE_CTMUL_AREG 1
#endif
    // u64 as well (re-enabled r3; DESIGN.md section 9 "k_ct_mul fault"):
    // the round-2 build of this layout at N = 8192 negacyclic (255 VGPRs, a
    // 68 B private segment) was withdrawn after a fault report; its code
    // object shows only constant-offset spill slots inside the segment and
    // compile-time slot indices, and today's build of the same layout needs
    // 205-221 VGPRs and no scratch (tests/test_abi.py keeps it that way).
    constexpr bool AREG = NL == 1 && FHE_CTMUL_AREG;
    W areg[AREG ? G::E : 1];
    W breg[AREG ? G::E : 1];
    // HBM slots (NL < 3) hold W words in the first half of their u64 row
    auto hrow = [&](int s) -> W * { return reinterpret_cast<W *>(orow + (size_t)(s + 1) * G::N); };
    // FHE_DEBUG_SLOTS (debug build, tests/test_gpu_cipher.py run once with
    // it): every slot access checks its slot number, register index and
    // position -- the round-2 fault in this kernel had no identified cause,
    // this is the guard that would name a bad index instead of faulting
#ifndef FHE_DEBUG_SLOTS
#define FHE_DEBUG_SLOTS 0
#endif
    auto check = [&](int s, uint32_t gi, int e) {
        if constexpr (FHE_DEBUG_SLOTS) {
            if (s < 0 || s > 2 || e < 0 || e >= G::E || gi >= (uint32_t)G::N) {
                printf("k_ct_mul slot index out of range: s=%d e=%d gi=%u (E=%d N=%d)\n", s, e, gi, G::E, G::N);
                __builtin_trap();
            }
        }
    };
    // slot s at global index gi (own positions only)
    auto ld = [&](int s, uint32_t gi, int e) -> W {
        check(s, gi, e);
        if (AREG && s == 0) return areg[AREG ? e : 0];
        if (AREG && s == 1) return breg[AREG ? e : 0];
        if (NL == 3 || (NL == 1 && s == 2)) return lds_all[G::P * G::LW + ((NL == 3 ? s : 0) * G::P + pl) * G::N + gi];
        if (s == 2) return creg[NL == 0 ? e : 0];
        return valid ? hrow(s)[gi] : W(0);
    };
    auto st = [&](int s, uint32_t gi, int e, W val) {
        check(s, gi, e);
        if (AREG && s == 0) areg[AREG ? e : 0] = val;
        else if (AREG && s == 1) breg[AREG ? e : 0] = val;
        else if (NL == 3 || (NL == 1 && s == 2)) lds_all[G::P * G::LW + ((NL == 3 ? s : 0) * G::P + pl) * G::N + gi] = val;
        else if (s == 2) creg[NL == 0 ? e : 0] = val;
        else if (valid) hrow(s)[gi] = val;
    };
    constexpr int SA = 0, SB = 1, SC = 2;
    // HBM slots A/B are prefetched into registers during the last pass of
    // the transform that consumes them (their latency overlaps it; with one
    // workgroup per CU nothing else would hide it).
    // (only the lab build FHE_CTMUL_AREG=0 keeps A/B in HBM at NL == 1;
    // NL == 0 (C in VGPRs) has no registers to spare for the prefetch)
    constexpr bool HB = NL == 1 && !AREG;
    W pre[2][HB ? G::E : 1];
    W v[G::E];
    // a fresh opaque copy of the lane index per phase: stops the compiler
    // from keeping one phase's address arithmetic live across the next
    // transform (scratch spills at N = 16384 otherwise)
    auto lane = [&]() {
        uint32_t t = tau;
        asm volatile("" : "+v"(t));
        return t;
    };
    uint32_t tp = 0;
    auto fetch = [&](int s, int k) {
        if (AREG && s <= 1) return;
        if constexpr (HB) {
#pragma unroll
            for (int e = 0; e < G::E; ++e) pre[k][e] = ld(s, gidx<LOGN, G::NP - 1>(tp, e), e);
        }
    };
    auto slot = [&](int s, int k, uint32_t gi, int e) -> W {
        check(s, gi, e);
        if (AREG && s == 0) return areg[AREG ? e : 0];
        if (AREG && s == 1) return breg[AREG ? e : 0];
        if constexpr (HB) return pre[k][e];
        else return ld(s, gi, e);
    };

    // 1. A = X0
    tp = lane();
    fwd_poly<LOGN, LAZY, kPfPolymul>(lds, v, tp, xr, valid, A);
#pragma unroll
    for (int e = 0; e < G::E; ++e) st(SA, gidx<LOGN, G::NP - 1>(tp, e), e, fwd_to_canon<LAZY>(v[e], A));
    if constexpr (G::NP > 1) __syncthreads();

    // 2. Y0: B = Y0, c0 = inv(X0 Y0)
    tp = lane();
    fwd_poly<LOGN, LAZY, kPfPolymul>(lds, v, tp, yr, valid, A, 0, [&] { fetch(SA, 0); });
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tp, e);
        const W y0 = v[e];
        st(SB, gi, e, fwd_to_canon<LAZY>(y0, A));
        v[e] = A.ar.mont(slot(SA, 0, gi, e), y0);
    }
    __syncthreads();
    tp = lane();
    inv_poly_from_regs<LOGN, kPfPolymul>(lds, v, tp, orow, valid, A, A.ninv_r);
    __syncthreads();

    // 3. X1: C = X1 Y0, B = X1
    tp = lane();
    fwd_poly<LOGN, LAZY, kPfPolymul>(lds, v, tp, xr + G::N, valid, A, 0, [&] { fetch(SB, 1); });
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tp, e);
        const W x1 = v[e];
        st(SC, gi, e, A.ar.mont(slot(SB, 1, gi, e), x1));
        st(SB, gi, e, fwd_to_canon<LAZY>(x1, A));
    }
    if constexpr (G::NP > 1) __syncthreads();

    // 4. Y1: c1 = C + X0 Y1, C = X1 Y1
    tp = lane();
    fwd_poly<LOGN, LAZY, kPfPolymul>(lds, v, tp, yr + G::N, valid, A, 0, [&] {
        fetch(SA, 0);
        fetch(SB, 1);
    });
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tp, e);
        const W y1 = v[e];
        const W c1 = A.ar.red2q(ld(SC, gi, e) + A.ar.mont(slot(SA, 0, gi, e), y1));
        st(SC, gi, e, A.ar.mont(slot(SB, 1, gi, e), y1));
        v[e] = c1;
    }
    __syncthreads();  // every slot read of rows 1/2 precedes their final stores
    tp = lane();
    inv_poly_from_regs<LOGN, kPfPolymul>(lds, v, tp, orow + G::N, valid, A, A.ninv_r);
    __syncthreads();
    tp = lane();
#pragma unroll
    for (int e = 0; e < G::E; ++e) v[e] = ld(SC, gidx<LOGN, G::NP - 1>(tp, e), e);
    inv_poly_from_regs<LOGN, kPfPolymul>(lds, v, tp, orow + 2 * G::N, valid, A, A.ninv_r);
}

// 32 coefficients per thread (q < 2^30, N = 8192 / 16384): two workgroups
// per CU, every transform pair in lockstep (fwd_poly2 / inv_poly2):
//   1. X0, Y0 = fwd(x0), fwd(y0)          stash canon(X0), canon(Y0) as W words
//                                          in rows 1 / 2 of the output (own
//                                          positions, overwritten last)
//   2. c0 = inv(X0 Y0)                     -> row 0
//   3. X1, Y1 = fwd(x1), fwd(y1)
//   4. c1 = X0 Y1 + X1 Y0, c2 = X1 Y1      (X0, Y0 back from the stash)
//   5. inv(c1), inv(c2)                    -> rows 1, 2
// 72 B per coefficient of HBM traffic (56 + the 16 B stash round trip) for
// two-workgroup occupancy and shared twiddles; FHE_CTMUL_E16=1 keeps the
// 16-per-thread kernel (lab A/B).
#ifndef FHE_CTMUL_E16
#define FHE_CTMUL_E16 0
#endif
// The paired kernel also for 64-bit words at N = 4096 / 8192 (instead of the
// slot kernel): per 16,384 ciphertext pairs at N = 8192 1.80 -> 1.55 ms
// (Q_60_1) and 1.73 -> 1.50 ms (62-bit prime), at N = 4096 0.80 -> 0.75 ms
// (round 5).
#ifndef FHE_CTMUL2_U64_SMALL
#define FHE_CTMUL2_U64_SMALL 1
#endif
// lab: X0 / Y0 kept in VGPRs instead of the HBM stash (one workgroup per CU):
// 1 = 32 per thread at a 256-VGPR budget (8 waves; 203 VGPRs), 2 = 16 per
// thread (16 waves; 99 VGPRs).  Both spill-free and 56 B per coefficient, and
// both slower than the stash at two workgroups per CU: 4.71 / 4.77 vs 4.59 ms
// per 16,384 ciphertext pairs (round 5, profiles/r5_ab).  The traffic of the
// stash (16 B per coefficient) costs less than the lost second workgroup.
#ifndef FHE_CTMUL_NOSTASH
#define FHE_CTMUL_NOSTASH 0
#endif
#ifndef FHE_CTMUL2_PF32
#define FHE_CTMUL2_PF32 1
#endif
template <int LOGN, typename W>
constexpr bool ctmul_regstash() { return FHE_CTMUL_NOSTASH != 0 && sizeof(W) == 4; }
template <int LOGN, typename W>
constexpr int ctmul2_occ() {
    return ctmul_regstash<LOGN, W>() ? (Geo<LOGN>::THREADS / 64 + 3) / 4 : Geo<LOGN>::template occ_waves<W>();
}
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (ctmul2_occ<LOGN, W>()))
k_ct_mul2(const uint64_t *__restrict__ x, const uint64_t *__restrict__ y, uint64_t *out, size_t batch,
          NttArgs<W> A) {
    using G = Geo<LOGN>;
    constexpr bool RS = ctmul_regstash<LOGN, W>();
    static_assert(G::P == 1 && (G::LOGE == 5 || sizeof(W) == 8 || RS), "one ciphertext pair per workgroup");
    constexpr int PF = sizeof(W) == 8 ? 0 : FHE_CTMUL2_PF32;  // u64: two 16-word spectra leave no VGPRs for lookahead
    __shared__ W lds[G::LW];
    const uint32_t tau = threadIdx.x;
    const size_t poly = blockIdx.x;
    if (poly >= batch) return;
    const uint64_t *xr = x + poly * 2 * G::N, *yr = y + poly * 2 * G::N;
    uint64_t *orow = out + poly * 3 * G::N;
    W *s1 = reinterpret_cast<W *>(orow + G::N), *s2 = reinterpret_cast<W *>(orow + 2 * G::N);
    W r1[RS ? G::E : 1], r2[RS ? G::E : 1];
    W a[G::E], b[G::E];
    // 1-2
    fwd_poly2<LOGN, LAZY, PF>(lds, a, b, tau, xr, yr, A);
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tau, e);
        const W x0 = fwd_to_canon<LAZY>(a[e], A);
        if constexpr (RS) {
            r1[e] = x0;
            r2[e] = fwd_to_canon<LAZY>(b[e], A);
        } else {
            s1[gi] = x0;
            s2[gi] = fwd_to_canon<LAZY>(b[e], A);
        }
        a[e] = A.ar.mont(x0, b[e]);
    }
    __syncthreads();
    uint32_t t1 = tau;
    asm volatile("" : "+v"(t1));
    inv_poly_from_regs<LOGN, PF>(lds, a, t1, orow, true, A, A.ninv_r);
    __syncthreads();
    // 3-4
    uint32_t t2 = tau;
    asm volatile("" : "+v"(t2));
    fwd_poly2<LOGN, LAZY, PF>(lds, a, b, t2, xr + G::N, yr + G::N, A);
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(t2, e);
        const W x1 = fwd_to_canon<LAZY>(a[e], A);
        const W X0 = RS ? r1[RS ? e : 0] : s1[gi], Y0 = RS ? r2[RS ? e : 0] : s2[gi];
        const W c1 = A.ar.red2q(A.ar.mont(X0, b[e]) + A.ar.mont(x1, Y0));
        b[e] = A.ar.mont(x1, b[e]);
        a[e] = c1;
        // u64: 4 stash pairs in flight at a time (all 16 hoisted spill)
        if (sizeof(W) == 8 && (e & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // every stash read precedes the final stores of rows 1 / 2
    uint32_t t3 = tau;
    asm volatile("" : "+v"(t3));
    inv_poly2<LOGN, PF>(lds, a, b, t3, orow + G::N, orow + 2 * G::N, A, A.ninv_r);
}

template <int LOGN, typename W>
static hipError_t ctmul_one(const Plan &p, const NttArgs<W> &A, const uint64_t *x, const uint64_t *y, uint64_t *out,
                            size_t batch) {
    using G = Geo<LOGN>;
    const size_t blocks = (batch + G::P - 1) / G::P;
    bool lazy = false;
    if constexpr (sizeof(W) == 4) lazy = p.lazy;
    if constexpr ((sizeof(W) == 4 && (LOGN == 13 || LOGN == 14) && !FHE_CTMUL_E16) ||
                  (sizeof(W) == 8 && (LOGN == 14 || (FHE_CTMUL2_U64_SMALL && (LOGN == 12 || LOGN == 13))))) {
        // u64 at N = 16384: 16 coefficients per thread, the pairs in lockstep
        // (no third slot in VGPRs: the single-transform kernel spilled there)
        constexpr int K = sizeof(W) == 4 ? gk(LOGN, FHE_CTMUL_NOSTASH == 2 ? 4 : 5) : LOGN;
        if constexpr (sizeof(W) == 4) {
            if (lazy) {
                hipLaunchKernelGGL((k_ct_mul2<K, W, true>), dim3(batch), dim3(Geo<K>::THREADS), 0, p.stream, x, y,
                                   out, batch, A);
                return hipGetLastError();
            }
        }
        hipLaunchKernelGGL((k_ct_mul2<K, W, false>), dim3(batch), dim3(Geo<K>::THREADS), 0, p.stream, x, y, out,
                           batch, A);
    } else {
        if (lazy) {
            if constexpr (sizeof(W) == 4)
                hipLaunchKernelGGL((k_ct_mul<LOGN, W, true>), dim3(blocks), dim3(G::THREADS), 0, p.stream, x, y,
                                   out, batch, A);
        } else
            hipLaunchKernelGGL((k_ct_mul<LOGN, W, false>), dim3(blocks), dim3(G::THREADS), 0, p.stream, x, y, out,
                               batch, A);
    }
    return hipGetLastError();
}

template <typename W>
static hipError_t ctmul_dispatch(const Plan &p, const NttArgs<W> &A, const uint64_t *x, const uint64_t *y,
                                 uint64_t *out, size_t batch) {
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return ctmul_one<L, W>(p, A, x, y, out, batch);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_ct_mul(const Plan &p, const uint64_t *x, const uint64_t *y, uint64_t *out, size_t batch) {
    if (batch == 0) return hipSuccess;
    if (p.word == 32)
        return ctmul_dispatch<uint32_t>(p, p.a32, x, y, out, batch);
    return ctmul_dispatch<uint64_t>(p, p.a64, x, y, out, batch);
}

}  // namespace FHE_NS
