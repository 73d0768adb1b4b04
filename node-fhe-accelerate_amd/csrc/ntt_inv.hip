// ntt_inv.hip -- inverse NTT (NTTProcessor::inverse_ntt,
// ntt_processor.cpp:325-380) and the fused polynomial multiply
// (PolynomialRing::multiply, polynomial_ring.cpp:421-447:
// inv(fwd(a) (.) fwd(b)) in ONE kernel: both spectra stay in VGPRs, the
// pointwise product is a Montgomery multiply whose R^-1 is folded into the
// inverse's N^-1 scaling).
#ifndef FHE_SPLIT_X64
#define FHE_SPLIT_X64 1
#endif
// Flag-free 64-bit arithmetic (fhe_arith.hpp FHE_U64_NOVCC; its bit selects
// as full-rate v_bitop3_b32) with the carry-free mulhi (FHE_MULHI64=4: the
// carry form cannot be combined with NOVCC in this unit -- an SGPR carry
// the backend cannot place).  Static VALU issue cycles per wave (measured
// rates, tools/valu_roofline.py): q62 polymul 36480 -> 34993, q62 inverse
// 13946 -> 12544, N = 8192 64-bit polymul 38951 -> 35061, and the two
// prime-specialised polymuls without their 6 spilled VGPRs (round 6).
#ifndef FHE_U64_NOVCC
#define FHE_U64_NOVCC 1
#endif
#ifndef FHE_MULHI64
#define FHE_MULHI64 4
#endif
#include "fhe_internal.hpp"

namespace FHE_NS {

template <int LOGN, typename W>
__device__ __forceinline__ void ntt_inv_body(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch,
                                             const NttArgs<W> &A) {
    using G = Geo<LOGN>;
    __shared__ W lds_all[G::P * lds_elems<LOGN, W>()];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < batch;
    W *lds = lds_all + pl * lds_elems<LOGN, W>();
    if (G::P == 1 && !valid) return;
    W v[G::E];
    const uint64_t *src = in + poly * G::N;
    const uint64_t lim = (uint64_t)A.ar.q2;  // GS inputs must be < 2q
    if constexpr (G::P == 1) {
        const auto r = brsrc(src);
        const uint32_t vo = LastIO<LOGN>::vo(tau);
        load_coeffs_r<G::E>(v, lim, SlowRed<W>{A}, [&](int e) -> uint64_t { return bload(r, vo, LastIO<LOGN>::so(e)); });
    } else {
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            uint64_t x = valid ? __builtin_nontemporal_load(src + gidx<LOGN, G::NP - 1>(tau, e)) : 0;
            v[e] = load_lazy<W>(x, lim, A.q64, A.mu64);
        }
    }
    inv_poly_from_regs<LOGN>(lds, v, tau, out + poly * G::N, valid, A, A.ninv);
}
template <int LOGN, typename W>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, Geo<LOGN>::template occ_waves<W>())
k_ntt_inv(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch, NttArgs<W> A) {
    ntt_inv_body<LOGN, W>(in, out, batch, A);
}
// RNS ring in one launch (k_ntt_fwd_limbs): limb blockIdx.y
template <int LOGN, typename W>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS)  // no occupancy floor: RNS calls are small
k_ntt_inv_limbs(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch,
                const NttArgs<W> *__restrict__ tab) {
    const size_t o = (size_t)blockIdx.y * batch * Geo<LOGN>::N;
    const NttArgs<W> A = tab[blockIdx.y];  // uniform: loaded into SGPRs like the kernel-argument form
    ntt_inv_body<LOGN, W>(in + o, out + o, batch, A);
}

// Where fwd(a) waits while fwd(b) runs: 0 = VGPRs (small N), 1 = a second
// LDS region, 2 = the output row in HBM (u64 at N = 16384, where LDS is
// full and the kernel is ALU-bound, so 16N extra bytes are cheap).  Keeping
// both spectra in VGPRs cost 150-255 VGPRs (N <= 8192) or scratch spills
// (N = 16384).
#ifndef FHE_POLY_PREFETCH
#define FHE_POLY_PREFETCH 1
#endif
#ifndef FHE_POLY_HBM_STASH
#define FHE_POLY_HBM_STASH 0
#endif
#ifndef FHE_POLY_REG_STASH_14
#define FHE_POLY_REG_STASH_14 0
#endif
template <int LOGN, typename W>
constexpr int polymul_stash() {
    using G = Geo<LOGN>;
    if (G::LOGE == 5 && sizeof(W) == 8) return 2;  // 64-bit words: two 64-word spectra do not fit
    if (G::L < 5 || G::LOGE == 5) return 0;  // 32 coefficients per thread: fwd(a) stays in VGPRs
    if (FHE_POLY_REG_STASH_14 && G::L == 14 && sizeof(W) == 4) return 0;
    if (FHE_POLY_HBM_STASH && G::L == 14) return 2;
    return G::P * (G::LW + G::N) * (int)sizeof(W) <= 160 * 1024 ? 1 : 2;
}
template <int LOGN, typename W>
constexpr int polymul_occ() {
    // with the stash in HBM the LDS footprint admits a second workgroup
    if (polymul_stash<LOGN, W>() == 0 && Geo<LOGN>::L >= 12) return Geo<LOGN>::template occ_waves<W>();
    return polymul_stash<LOGN, W>() == 2 && (FHE_POLY_HBM_STASH || Geo<LOGN>::LOGE == 5)
               ? Geo<LOGN>::template occ_waves<W>() : 1;
}
// Polymul geometry: at q < 2^30 and N >= 4096, 32 coefficients per thread
// (radix-32 passes: 2 LDS exchanges per transform instead of 3, N/32 threads,
// fwd(a) parked in VGPRs, conflict-free pads, two workgroups per CU so one's
// HBM traffic overlaps the other's transforms).  FHE_POLY_E16=1: the 16-per-
// thread kernel with the LDS stash (lab A/B).
#ifndef FHE_POLY_E16
#define FHE_POLY_E16 0
#endif
#ifndef FHE_PF_POLY32
#define FHE_PF_POLY32 1
#endif
// 64-bit words at N = 16384 (FHE_POLY64): 1 = the dual kernel at 16
// coefficients per thread (one workgroup per CU, 128 VGPRs, no stash);
// 2 = 32 per thread with streamed twiddles, the split exchange and fwd(a)
// stashed in c's row (two workgroups per CU, 1.67x the algorithmic bytes).
#ifndef FHE_POLY64
#define FHE_POLY64 1
#endif
// Inverse transform key: FHE_INV64_E32=1 runs 64-bit words at N = 16384 at
// 32 coefficients per thread with streamed twiddles and the split exchange
// (as the forward).  Measured slower than 16 per thread (7.91 vs 7.62 ms per
// 65,536 inverses, profiles/r3e/ab.txt), so off.
#ifndef FHE_INV64_E32
#define FHE_INV64_E32 0
#endif
template <int LOGN, typename W>
constexpr int inv_key() { return (FHE_INV64_E32 && sizeof(W) == 8 && LOGN == 14) ? gk(LOGN, 5) : LOGN; }
template <int LOGN, typename W>
constexpr int polymul_key() {
    if (sizeof(W) == 8) return (FHE_POLY64 == 2 && LOGN == 14) ? gk(LOGN, 5) : LOGN;
    return (!FHE_POLY_E16 && sizeof(W) == 4 && LOGN >= 13 && LOGN <= 14) ? gk(LOGN, 5) : LOGN;
}
template <int LOGN>
constexpr int polymul_pf() { return Geo<LOGN>::LOGE == 5 ? FHE_PF_POLY32 : kPfPolymul; }
// 64-bit words at N = 16384: the dual kernel at 16 coefficients per thread
// (two 16-word u64 spectra = 64 VGPRs; no stash of fwd(a) in LDS or HBM).
#ifndef FHE_POLY_DUAL
#define FHE_POLY_DUAL 1
#endif
#ifndef FHE_POLY_DUAL64
#define FHE_POLY_DUAL64 1
#endif
#ifndef FHE_PF_DUAL64
#define FHE_PF_DUAL64 0
#endif
// The 64-bit dual kernel also at N = 4096 / 8192 (16 per thread, one
// workgroup per pair, occupancy floor 4 waves per SIMD; 123-126 VGPRs, no
// spill): per 16,384 pairs at N = 8192 2.83 -> 2.23 ms (Q_60_1) and 2.75 ->
// 2.10 ms (the 62-bit prime), at N = 4096 1.23 -> 1.06 ms (Q_60_1) (round 5).
#ifndef FHE_POLY_DUAL64_SMALL
#define FHE_POLY_DUAL64_SMALL 1
#endif
// The dual kernel also at N = 4096 with 16 per thread (one 256-thread
// workgroup per pair, <= 128 VGPRs): 30.3 -> 28.1 us for C2's 1024 pairs,
// 1.67 -> 1.49 ms (q < 2^27, lazy) and 1.74 -> 1.62 ms (q < 2^30) per 65,536
// (round 5).  FHE_POLY_DUAL_E16=0 keeps the single-transform kernel.
#ifndef FHE_POLY_DUAL_E16
#define FHE_POLY_DUAL_E16 1
#endif
template <int LOGN, typename W>
constexpr bool polymul_dual() {
    using G = Geo<LOGN>;
    if constexpr (sizeof(W) == 4)
        return (G::LOGE == 5 && FHE_POLY_DUAL) || (FHE_POLY_DUAL_E16 && G::P == 1 && G::LOGE == 4 && G::L == 12);
    else return FHE_POLY_DUAL64 && G::P == 1 && G::LOGE == 4 &&
                ((G::L == 14 && FHE_POLY64 == 1) || (FHE_POLY_DUAL64_SMALL && (G::L == 12 || G::L == 13)));
}
template <int LOGN, typename W>
constexpr int polymul2_pf() { return sizeof(W) == 8 ? FHE_PF_DUAL64 : polymul_pf<LOGN>(); }

template <int LOGN, typename W, bool LAZY>
__device__ __forceinline__ void polymul_body(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *c,
                                             size_t batch, const NttArgs<W> &A) {
    using G = Geo<LOGN>;
    constexpr int STASH = polymul_stash<LOGN, W>();
    __shared__ W lds_all[G::P * lds_elems<LOGN, W>() + (STASH == 1 ? G::P * G::N : 0)];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < batch;
    W *lds = lds_all + pl * lds_elems<LOGN, W>();
    W *st = lds_all + G::P * lds_elems<LOGN, W>() + pl * G::N;
    uint64_t *crow = c + poly * G::N;
    if (G::P == 1 && !valid) return;
    W v[G::E];
    W va[STASH == 0 ? G::E : 1];
    // P == 1: b's coefficients are loaded during fwd(a)'s last pass, so
    // their HBM latency overlaps it (one workgroup per CU has no other
    // workgroup to hide it behind).
    constexpr bool PRE = G::P == 1 && FHE_POLY_PREFETCH && STASH == 1;  // no registers to spare at STASH 2
    uint64_t rb[PRE ? G::E : 1];
    auto hook = [&] {
        if constexpr (PRE) load_raw<LOGN>(*reinterpret_cast<uint64_t(*)[G::E]>(rb), tau, b + poly * G::N);
    };
    fwd_poly<LOGN, LAZY, polymul_pf<LOGN>()>(lds, v, tau, a + poly * G::N, valid, A, 0, hook);
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const W x = fwd_to_canon<LAZY>(v[e], A);  // canonical: times a raw output below
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tau, e);  // own positions: no sync needed
        if constexpr (STASH == 0) va[e] = x;
        else if constexpr (STASH == 1) st[gi] = x;
        else if (valid) reinterpret_cast<W *>(crow)[gi] = x;  // W-typed: first half of c's row
    }
    // keep b's raw loads (2 VGPRs per coefficient) out of the stash
    // conversion (a 64-bit mad result per coefficient): interleaved, the two
    // peak together and spill at 32 coefficients per thread
    if constexpr (G::LOGE == 5) __builtin_amdgcn_sched_barrier(0);
    if constexpr (G::NP > 1) __syncthreads();  // LDS exchange buffer is reused by the second transform
    // opaque copy of the lane index (u64 path): stops the compiler from
    // keeping the first transform's address arithmetic live for reuse.  At
    // u32 the reuse is cheaper than recomputing (measured, r05 A/B).
    uint32_t tb = tau;
    if constexpr (sizeof(W) == 8 || STASH == 2) asm volatile("" : "+v"(tb));
    if constexpr (PRE)
        fwd_poly<LOGN, LAZY, polymul_pf<LOGN>()>(lds, v, tb, b + poly * G::N, valid, A, 0, NoHook{},
                                               reinterpret_cast<uint64_t(*)[G::E]>(rb));
    else
        fwd_poly<LOGN, LAZY, polymul_pf<LOGN>()>(lds, v, tb, b + poly * G::N, valid, A);
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tb, e);
        W x;
        if constexpr (STASH == 0) x = va[e];
        else if constexpr (STASH == 1) x = st[gi];
        else x = valid ? reinterpret_cast<const W *>(crow)[gi] : W(0);
        v[e] = A.ar.mont(x, v[e]);  // a*b*R^-1 in [0, 2q): canonical x raw v[e] (< R)
    }
    if constexpr (G::NP > 1) __syncthreads();
    uint32_t ti = tau;
    if constexpr (sizeof(W) == 8 || STASH == 2) asm volatile("" : "+v"(ti));
    inv_poly_from_regs<LOGN, polymul_pf<LOGN>()>(lds, v, ti, crow, valid, A, A.ninv_r);
}
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (polymul_occ<LOGN, W>()))
k_polymul(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *c, size_t batch,
          NttArgs<W> A) {
    polymul_body<LOGN, W, LAZY>(a, b, c, batch, A);
}
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS)  // no occupancy floor: RNS calls are small
k_polymul_limbs(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *c, size_t batch,
                const NttArgs<W> *__restrict__ tab) {
    const size_t o = (size_t)blockIdx.y * batch * Geo<LOGN>::N;
    const NttArgs<W> A = tab[blockIdx.y];
    polymul_body<LOGN, W, LAZY>(a + o, b + o, c + o, batch, A);
}

// Polymul with 32 coefficients per thread: fwd(a) and fwd(b) run in
// lockstep (fwd_poly2: shared twiddles, two independent butterfly streams),
// then the pointwise Montgomery product and the inverse.  Two workgroups per
// CU (one 64 KiB exchange buffer each), so one's HBM traffic overlaps the
// other's transforms.
// A persistent grid (workgroups looping over pairs, with or without a phase
// stagger or an L2 touch of the next pair) measured no faster (round 4).
// lab only: 1 = HBM traffic without transforms, 2 = transforms without HBM
#ifndef FHE_POLY_LAB
#define FHE_POLY_LAB 0
#endif
template <int LOGN, typename W, bool LAZY>
__device__ __forceinline__ void polymul2_one(W *lds, uint32_t tau, const uint64_t *__restrict__ a,
                                             const uint64_t *__restrict__ b, uint64_t *c, size_t poly,
                                             const NttArgs<W> &A) {
    using G = Geo<LOGN>;
    W v[G::E], vb[G::E];
    fwd_poly2<LOGN, LAZY, polymul2_pf<LOGN, W>()>(lds, v, vb, tau, a + poly * G::N, b + poly * G::N, A);
#pragma unroll
    for (int e = 0; e < G::E; ++e) v[e] = A.ar.mont(fwd_to_canon<LAZY>(v[e], A), vb[e]);  // canonical x raw (< R)
    __syncthreads();  // the exchange buffer still holds b's last layout reads
    inv_poly_from_regs<LOGN, polymul2_pf<LOGN, W>()>(lds, v, tau, c + poly * G::N, true, A, A.ninv_r);
}

template <int LOGN, typename W>
constexpr int polymul2_occ() {
    constexpr int o = Geo<LOGN>::template occ_waves<W>();
    return (FHE_POLY_DUAL_E16 && Geo<LOGN>::LOGE == 4 && (sizeof(W) == 4 || gk_logn(LOGN) < 14) && o > 4) ? 4 : o;
}
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (polymul2_occ<LOGN, W>()))
k_polymul2(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *c, size_t batch,
           NttArgs<W> A) {
    using G = Geo<LOGN>;
    static_assert(G::P == 1, "one polynomial pair per workgroup");
    __shared__ W lds[lds_elems<LOGN, W>()];
    const uint32_t tau = threadIdx.x;
    const size_t poly = blockIdx.x;
    if (poly >= batch) return;
#if FHE_POLY_LAB == 1
    // lab: HBM traffic only (loads of a, b and the store of c, no transforms)
    {
        const auto ra = brsrc(a + poly * G::N), rb = brsrc(b + poly * G::N), rc = brsrc(c + poly * G::N);
#pragma unroll
        for (int ch = 0; ch < G::E; ch += 8) {
            uint64_t x[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = bload(ra, tau * 8u, (ch + e) * G::T * 8u) ^ bload(rb, tau * 8u, (ch + e) * G::T * 8u);
#pragma unroll
            for (int e = 0; e < 8; ++e) bstore(rc, tau * 8u, (ch + e) * G::T * 8u, x[e]);
        }
        return;
    }
#elif FHE_POLY_LAB == 2
    // lab: transforms only (inputs from the lane index, no HBM traffic)
    {
        W v[G::E], vb[G::E];
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            v[e] = (W)((tau * 131u + e * 7919u + (uint32_t)poly) & 0x3FFFFFFu);
            vb[e] = (W)((tau * 577u + e * 104729u) & 0x3FFFFFFu);
        }
        {
            Tw<W> t0[PassTw<LOGN, 0>::COUNT];
            load_tw<LOGN, 0>(tau, A.twf, t0);
            fwd_pass<LOGN, 0, LAZY, W>(v, t0, A.ar);
            fwd_pass<LOGN, 0, LAZY, W>(vb, t0, A.ar);
        }
        fwd_rest2<LOGN, 1, LAZY, polymul2_pf<LOGN, W>()>(lds, v, vb, tau, A.twf, A.ar);
#pragma unroll
        for (int e = 0; e < G::E; ++e) v[e] = A.ar.mont(fwd_to_canon<LAZY>(v[e], A), vb[e]);
        __syncthreads();
        inv_poly_from_regs<LOGN, polymul2_pf<LOGN, W>(), false>(lds, v, tau, c, true, A, A.ninv_r,
            0, [&](uint32_t gi, uint64_t x) -> uint64_t { if (x == ~0ull) c[gi] = x; return x; });
        return;
    }
#endif
    polymul2_one<LOGN, W, LAZY>(lds, tau, a, b, c, poly, A);
}
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS)  // no occupancy floor: RNS calls are small
k_polymul2_limbs(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *c, size_t batch,
                 const NttArgs<W> *__restrict__ tab) {
    __shared__ W lds[lds_elems<LOGN, W>()];
    const size_t poly = blockIdx.x;
    if (poly >= batch) return;
    const size_t o = (size_t)blockIdx.y * batch * Geo<LOGN>::N;
    const NttArgs<W> A = tab[blockIdx.y];
    polymul2_one<LOGN, W, LAZY>(lds, threadIdx.x, a + o, b + o, c + o, poly, A);
}

// tab != nullptr: the RNS form, `limbs` limbs of [batch][N] each in one launch
// (grid.y = limb), constants from tab[limb].
template <int LOGN, typename W>
static hipError_t inv_one(const Plan &p, const NttArgs<W> &A, hipStream_t s, const uint64_t *a, const uint64_t *b,
                          uint64_t *c, size_t batch, const NttArgs<W> *tab = nullptr, int limbs = 1) {
    // one launch of kernel K (or of its limb form KL when tab is given)
    auto go = [&](auto K, auto KL, size_t blocks, int threads, auto... args) -> hipError_t {
        if (tab)
            hipLaunchKernelGGL(KL, dim3((unsigned)blocks, (unsigned)limbs), dim3(threads), 0, s, args..., tab);
        else
            hipLaunchKernelGGL(K, dim3((unsigned)blocks), dim3(threads), 0, s, args..., A);
        return hipGetLastError();
    };
    bool lazy = false;
    if constexpr (sizeof(W) == 4) lazy = p.lazy;
    constexpr int PK = polymul_key<LOGN, W>();
    using GP = Geo<PK>;
    size_t pblocks = (batch + GP::P - 1) / GP::P;
    if constexpr (polymul_dual<PK, W>()) {
        if (b) {
            // (unit twiddles, gk_compat, at 32-bit words: 141 fewer multiplies
            // per wave, 6.32 vs 6.34 ms -- within noise; not instantiated)
            if constexpr (sizeof(W) == 4) {
                if (lazy)
                    return go(k_polymul2<PK, W, true>, k_polymul2_limbs<PK, W, true>, pblocks, GP::THREADS, a, b, c,
                              batch);
            }
            // a sparse prime (ntt_core.hpp gk_sparse): q62 polymul 19.2 -> 18.1 ms
            // per 65,536 (round 5; the forward, the inverse, the multi-level
            // external product and the blind rotation measured 0 to +2 % and
            // keep the generic arithmetic); compat mode (gk_compat, unit
            // twiddles in pass 0): 18.39 -> 17.70 ms, 333 fewer multiplies per
            // wave, and no spill
            if constexpr (sizeof(W) == 8) {
                if (!tab && A.ar.sp == 1 && p.compat)
                    return go(k_polymul2<gk_compat(gk_sparse(PK, 1)), W, false>, k_polymul2_limbs<PK, W, false>,
                              pblocks, GP::THREADS, a, b, c, batch);
                if (!tab && A.ar.sp == 1)
                    return go(k_polymul2<gk_sparse(PK, 1), W, false>, k_polymul2_limbs<PK, W, false>, pblocks,
                              GP::THREADS, a, b, c, batch);
                if (!tab && A.ar.sp == 2)
                    return go(k_polymul2<gk_sparse(PK, 2), W, false>, k_polymul2_limbs<PK, W, false>, pblocks,
                              GP::THREADS, a, b, c, batch);
                if (!tab && p.compat)
                    return go(k_polymul2<gk_compat(PK), W, false>, k_polymul2_limbs<PK, W, false>, pblocks,
                              GP::THREADS, a, b, c, batch);
            }
            return go(k_polymul2<PK, W, false>, k_polymul2_limbs<PK, W, false>, pblocks, GP::THREADS, a, b, c, batch);
        }
    } else {
        if (b && lazy) {
            if constexpr (sizeof(W) == 4)
                return go(k_polymul<PK, W, true>, k_polymul_limbs<PK, W, true>, pblocks, GP::THREADS, a, b, c, batch);
            return hipErrorInvalidValue;
        } else if (b) {
            return go(k_polymul<PK, W, false>, k_polymul_limbs<PK, W, false>, pblocks, GP::THREADS, a, b, c, batch);
        }
    }
    constexpr int IK = inv_key<LOGN, W>();
    using GI = Geo<IK>;
    const size_t iblocks = (batch + GI::P - 1) / GI::P;
    return go(k_ntt_inv<IK, W>, k_ntt_inv_limbs<IK, W>, iblocks, GI::THREADS, a, c, batch);
}

template <typename W>
static hipError_t inv_dispatch(const Plan &p, const NttArgs<W> &A, const uint64_t *a, const uint64_t *b,
                               uint64_t *c, size_t batch) {
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return inv_one<L, W>(p, A, p.stream, a, b, c, batch);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}

static hipError_t inv_any(const Plan &p, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch) {
    if (batch == 0) return hipSuccess;
    if (p.word == 32)
        return inv_dispatch<uint32_t>(p, p.a32, a, b, c, batch);
    return inv_dispatch<uint64_t>(p, p.a64, a, b, c, batch);
}

template <typename W>
static hipError_t inv_limbs_dispatch(const Plan &p, const void *tab, int limbs, const uint64_t *a, const uint64_t *b,
                                     uint64_t *c, size_t batch) {
    const NttArgs<W> *t = static_cast<const NttArgs<W> *>(tab);
    const NttArgs<W> *A0;  // unused by the limb kernels (their constants come from tab)
    if constexpr (sizeof(W) == 4) A0 = &p.a32;
    else A0 = &p.a64;
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return inv_one<L, W>(p, *A0, p.stream, a, b, c, batch, t, limbs);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}
// RNS ring: inverse (b == nullptr) or polymul of `limbs` limbs in one launch
hipError_t launch_inv_limbs(const Plan &p, const void *tab, int limbs, const uint64_t *a, const uint64_t *b,
                            uint64_t *c, size_t batch) {
    if (p.wide || p.logn > kMaxFusedLogN || limbs < 1 || limbs > 65535) return hipErrorInvalidValue;
    if (batch == 0) return hipSuccess;
    if (b && c == b) { const uint64_t *t = a; a = b; b = t; }
    return p.word == 32 ? inv_limbs_dispatch<uint32_t>(p, tab, limbs, a, b, c, batch)
                        : inv_limbs_dispatch<uint64_t>(p, tab, limbs, a, b, c, batch);
}

hipError_t launch_inv(const Plan &p, const uint64_t *in, uint64_t *out, size_t batch) {
    if (p.wide) return launch_wide(p, 3, in, nullptr, out, batch);
    if (p.logn > kMaxFusedLogN) return launch_big(p, 3, in, nullptr, out, batch);
    return inv_any(p, in, nullptr, out, batch);
}
hipError_t launch_polymul(const Plan &p, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch) {
    // The HBM stash writes fwd(a) into c before b is read: if c aliases b,
    // transform b first (the pointwise product commutes).
    if (p.logn > kMaxFusedLogN && !p.wide) return launch_big(p, 4, a, b, c, batch);
    if (c == b) { const uint64_t *t = a; a = b; b = t; }
    if (p.wide) return launch_wide(p, 4, a, b, c, batch);
    return inv_any(p, a, b, c, batch);
}

}  // namespace FHE_NS
