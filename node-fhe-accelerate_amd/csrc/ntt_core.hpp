// ntt_core.hpp -- one-workgroup-per-polynomial fused NTT building blocks.
//
// Transform reproduced (ntt_processor.cpp:262-380):
//   forward:  bit-reverse, then for stage s = 0..L-1 (m = 2^s), pairs
//             (k+j, k+j+m) with twiddle psi^(j*N/2m)  (compat mode), or
//             psi^((2j+1)*N/2m)  (negacyclic mode: the psi^i pre-twist of a
//             cyclic transform merged into the stage twiddles -- the same
//             butterflies, only the stage table differs, fhe_gpu.cpp);
//   inverse:  Gentleman-Sande stages L-1..0 with psi^-(...), bit-reverse,
//             scale by N^-1.
//
// Work decomposition (MI355X-first, not the reference's loop nest):
//   * one workgroup per polynomial (several for N < 1024), T = N/16 threads,
//     each thread owns E = 16 coefficients in VGPRs;
//   * the L stages are cut into passes of 4 (radix-16) -- a pass runs
//     entirely in registers, passes exchange through LDS (one barrier each);
//   * the bit-reversal is folded into the HBM load of pass 0 (forward) and
//     the store of the last inverse pass: every HBM access is coalesced;
//   * twiddles come from a stage-major table tw[2^s + j] (L2 resident);
//     pass-0 twiddles are wave-uniform (scalar loads);
//   * LDS uses a padded layout (pad_idx) so every access of a pass is one
//     base + an immediate offset, with few bank conflicts.
#pragma once
#include "fhe_arith.hpp"

namespace FHE_NS {

// Padded LDS layout: element i lives at word i + (i >> A) + (i >> B)
// (A, B per degree; 0 = unused).  For every pass layout the padded address
// of (g, t) splits as pad(lay(g)) + pad(t << S), so each thread computes one
// base per slot group and every ds_read/ds_write of the pass uses an
// immediate offset.  Pads chosen by simulating the lane groups of every pass
// layout: conflict-free up to N = 256, one 2-way
// conflicted exchange above.  An XOR swizzle (conflict-free everywhere) was
// replaced because its 16 per-layout addresses stayed live across whole
// kernels (64 VGPRs in polymul, forcing scratch spills).
constexpr int kPadA[17] = {0, 0, 0, 0, 0, 3, 3, 3, 4, 5, 5, 6, 7, 8, 5, 5, 0};
constexpr int kPadB[17] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 10, 10, 0};

// Geometry key: log2(N) in bits 0-7, log2(coefficients per thread) in bits
// 8-11 (0 = the default min(log2 N, 4)).  Every template below that takes
// `int LOGN` accepts a key, so a kernel opts into 32 coefficients per thread
// (radix-32 passes, N/32 threads) with gk(logn, 5).
constexpr int gk(int logn, int loge) { return logn | (loge << 8); }
constexpr int gk_logn(int k) { return k & 0xff; }
constexpr int gk_loge(int k) { return ((k >> 8) & 0xf) ? ((k >> 8) & 0xf) : ((k & 0xff) < 4 ? (k & 0xff) : 4); }
// Bits 12-13: one of the reference's sparse 64-bit primes q = 2^k - d
// (fhe_arith.hpp kSparsePrimes; Arith::sp at run time), compiled in as
// constants: the Shoup remainder's h q takes two multiplies instead of
// three.  Only the kernels that gain are instantiated with it; every other
// key leaves the bits clear.
constexpr int gk_sparse(int k, int sel) { return k | (sel << 12); }
constexpr int gk_sp(int k) { return (k >> 12) & 3; }
// Bit 14: the context is in compat mode (the reference's cyclic transform,
// whose stage-s twiddle of butterfly 0 is psi^0 = 1).  In pass 0 the twiddle
// slot of butterfly group 0 is that 1 for every lane, so those butterflies
// skip the Shoup product (one reduction instead of three multiplies):
// 31 of the 80 pass-0 butterflies at 32 coefficients per thread, 15 of 32 at
// 16.  Negacyclic tables have no unit twiddle; their keys leave the bit clear.
constexpr int gk_compat(int k) { return k | (1 << 14); }
constexpr bool gk_cp(int k) { return (k >> 14) & 1; }

// Pads for 32 coefficients per thread (tools/lab/lds_pads.py): i + (i >> (L-5))
// is conflict-free for every pass layout at L = 11..14.
// Fewer coefficients per thread (the low-latency blind rotation,
// ntt_br.hip) at N = 1024 with 64-bit words: (5, 6) for 8 per thread, (4, 5)
// for 4 (lds_pads.py --u64); other degrees take the 16-per-thread pads.
constexpr int pad_a(int L, int E) {
    return E == 5 ? 0 : (L == 10 && E == 3) ? 5 : (L == 10 && E == 2) ? 4 : kPadA[L];
}
constexpr int pad_b(int L, int E) {
    return E == 5 ? L - 5 : (L == 10 && E == 3) ? 6 : (L == 10 && E == 2) ? 5 : kPadB[L];
}
template <int K>
__host__ __device__ constexpr uint32_t pad_idx(uint32_t i) {
    constexpr int L = gk_logn(K);
    constexpr int A = pad_a(L, gk_loge(K));
    constexpr int B = pad_b(L, gk_loge(K));
    return i + (A ? (i >> A) : 0u) + (B ? (i >> B) : 0u);
}
// LDS words per polynomial
template <int K>
constexpr int lds_words() { return (int)pad_idx<K>((1u << gk_logn(K)) - 1) + 1; }

// Split exchange (64-bit words at N = 16384, 32 coefficients per thread):
// each pass exchange moves the
// low 32-bit halves of the words through the LDS buffer, then the high halves
// (store lo / sync / load lo / sync / store hi / sync / load hi), so the
// buffer is 64 KiB instead of 128 KiB and two workgroups fit per CU -- one's
// barriers and HBM waits overlap the other's butterflies.  Opt-in per
// translation unit (FHE_SPLIT_X64 before the includes).
#ifndef FHE_SPLIT_X64
#define FHE_SPLIT_X64 0
#endif
template <int K, typename W>
constexpr bool split_x() { return FHE_SPLIT_X64 && sizeof(W) == 8 && gk_logn(K) >= 14 && gk_loge(K) == 5; }
// W-typed elements of one polynomial's exchange buffer
template <int K, typename W>
constexpr int lds_elems() { return split_x<K, W>() ? (lds_words<K>() + 1) / 2 : lds_words<K>(); }

// ---------------------------------------------------------------- geometry
template <int LOGN>
struct Geo {
    static constexpr int L = gk_logn(LOGN);
    static constexpr int N = 1 << L;
    static constexpr int LOGE = gk_loge(LOGN);
    static constexpr int E = 1 << LOGE;
    static constexpr int LOGT = L - LOGE;
    static constexpr int T = 1 << LOGT;
    static constexpr int NP = (L + LOGE - 1) / LOGE;  // passes
    static constexpr int P = T >= 256 ? 1 : 256 / T;  // polynomials per workgroup
    static constexpr int THREADS = T * P;
    static constexpr int LW = lds_words<LOGN>();  // padded LDS words per polynomial
    static constexpr int S(int p) { return p * LOGE; }
    // Waves per SIMD the LDS footprint allows (160 KiB LDS, 2048 threads per
    // CU): used as __launch_bounds__' min-waves-per-EU so the register
    // allocation never costs a resident workgroup.
    template <typename W, int EXTRA_WORDS = 0>
    static constexpr int occ_waves() {
        const int by_lds = (160 * 1024) / ((P * lds_elems<LOGN, W>() + EXTRA_WORDS) * (int)sizeof(W));
        const int by_thr = 2048 / THREADS;
        const int wg = by_lds < by_thr ? by_lds : by_thr;
        const int w = wg * THREADS / 64 / 4;
#ifdef FHE_NO_OCC_BOUND
        return 1;
#else
        return w < 1 ? 1 : (w > 8 ? 8 : w);
#endif
    }
    static constexpr int R(int p) { return (L - p * LOGE) < LOGE ? (L - p * LOGE) : LOGE; }
};

// Polynomial index within the workgroup.  P == 1 must be the constant 0:
// otherwise the compiler cannot prove the polynomial's buffer resource
// wave-uniform (threadIdx.x >> LOGT is 0 only because of the launch size)
// and wraps every buffer access in a readfirstlane waterfall loop.
template <typename G>
__device__ __forceinline__ uint32_t wg_poly() {
    if constexpr (G::P == 1) return 0u;
    else return threadIdx.x >> G::LOGT;
}

// Lane index rebuilt on demand from the wave index (an SGPR) and mbcnt, for
// kernels that need threadIdx.x again after a register-heavy stretch: no
// VGPR holds it across the stretch (asm volatile: never hoisted or merged).
// Valid for workgroups of whole waves.
struct TidSource {
    uint32_t wave;
    __device__ TidSource() : wave(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {}
    __device__ uint32_t operator()() const {
        uint32_t t;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(t));
        return (wave << 6) | t;
    }
};

// A wave-uniform pointer the compiler may not relate to its other uses
// (FHE_OPAQUE_TW): each transform then re-loads its wave-uniform (scalar)
// twiddles through the constant cache instead of the compiler keeping one
// transform's SGPR copies live across the next ones -- in kernels with
// several transforms that CSE is what spilled SGPRs (k_ct_mul2: 142).
#ifndef FHE_OPAQUE_TW
#define FHE_OPAQUE_TW 0
#endif
// 1: every word size; 2: 32-bit words only (Tw<uint32_t>, 8 bytes).
template <typename T>
__device__ __forceinline__ const T *opaque_tw(const T *p) {
    if constexpr (FHE_OPAQUE_TW == 1 || (FHE_OPAQUE_TW == 2 && sizeof(T) == 8)) asm volatile("" : "+s"(p));
    return p;
}

__host__ __device__ constexpr uint32_t cbrv(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

// Position of element (g, t) in pass layout (S, R): t occupies bits
// [S, S+R), g the remaining bits.
template <int S, int R>
__device__ __forceinline__ uint32_t lay(uint32_t g) {
    return (g & ((1u << S) - 1)) | ((g >> S) << (S + R));
}

// g for slot-group u of pass p: pass 0 uses g = brv(tau) (bit-reversed HBM
// load), every other pass g = tau + u*T.
template <int LOGN, int PASS>
__device__ __forceinline__ uint32_t g_of(uint32_t tau, int u) {
    using G = Geo<LOGN>;
    if constexpr (PASS == 0) return cbrv(tau, G::LOGT);
    else return tau + uint32_t(u) * G::T;
}

// ---------------------------------------------------------------- LDS I/O
template <int LOGN, int PASS, typename W>
__device__ __forceinline__ void lds_store(W *lds, const W (&v)[Geo<LOGN>::E], uint32_t tau) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS), R = G::R(PASS), NU = G::E >> R;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const uint32_t base = pad_idx<LOGN>(lay<S, R>(g_of<LOGN, PASS>(tau, u)));
#pragma unroll
        for (int t = 0; t < (1 << R); ++t) lds[base + pad_idx<LOGN>(uint32_t(t) << S)] = v[t + (u << R)];
    }
}
template <int LOGN, int PASS, typename W>
__device__ __forceinline__ void lds_load(const W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS), R = G::R(PASS), NU = G::E >> R;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const uint32_t base = pad_idx<LOGN>(lay<S, R>(g_of<LOGN, PASS>(tau, u)));
#pragma unroll
        for (int t = 0; t < (1 << R); ++t) v[t + (u << R)] = lds[base + pad_idx<LOGN>(uint32_t(t) << S)];
    }
}
// Lab-only timing bound (FHE_LAB_NOBAR=1, never in a shipped build: the
// results are WRONG): the exchanges between passes >= 1 run without their
// workgroup barriers, i.e. as if each were confined to one wave (a layout
// whose wave bits avoid the pass digits of both passes).  Measures what
// barrier-free exchanges could buy before any layout is redesigned.
#ifndef FHE_LAB_NOBAR
#define FHE_LAB_NOBAR 0
#endif
template <bool LOCAL>
__device__ __forceinline__ void xbar() {
    if constexpr (LOCAL) asm volatile("" ::: "memory");
    else __syncthreads();
}
template <int PA, int PB>
constexpr bool lab_local() { return FHE_LAB_NOBAR && PA >= 1 && PB >= 1; }

// One pass exchange: registers in layout PA -> LDS -> registers in layout PB.
// The caller's next exchange stores to the positions this one loaded from
// (same thread, same layout), so no barrier is needed after the load.
template <int LOGN, int PA, int PB, typename W>
__device__ __forceinline__ void exchange(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau) {
    constexpr int E = Geo<LOGN>::E;
    constexpr bool LOC = lab_local<PA, PB>();
    if constexpr (split_x<LOGN, W>()) {
        uint32_t *l32 = reinterpret_cast<uint32_t *>(lds);
        uint32_t h[E];
#pragma unroll
        for (int e = 0; e < E; ++e) h[e] = (uint32_t)v[e];
        lds_store<LOGN, PA>(l32, h, tau);
#pragma unroll
        for (int e = 0; e < E; ++e) h[e] = (uint32_t)(v[e] >> 32);
        xbar<LOC>();
        uint32_t lo[E];
        lds_load<LOGN, PB>(l32, lo, tau);
        xbar<LOC>();  // every lane's low halves read before the high halves overwrite them
        lds_store<LOGN, PA>(l32, h, tau);
        xbar<LOC>();
        lds_load<LOGN, PB>(l32, h, tau);
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = (W)lo[e] | ((W)h[e] << 32);
    } else {
        lds_store<LOGN, PA>(lds, v, tau);
        xbar<LOC>();
        lds_load<LOGN, PB>(lds, v, tau);
    }
}

// Global (natural-order) index of slot e in pass layout PASS (PASS > 0, or
// the last pass): coalesced across tau.
template <int LOGN, int PASS>
__device__ __forceinline__ uint32_t gidx(uint32_t tau, int e) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS), R = G::R(PASS);
    int t = e & ((1 << R) - 1), u = e >> R;
    return lay<S, R>(g_of<LOGN, PASS>(tau, u)) | (uint32_t(t) << S);
}

// gidx = gidx_var(tau) + gidx_const(e) for PASS > 0: g = tau | (u << LOGT)
// has disjoint bit fields and lay() only moves bit fields, so the lane part
// and the slot part add without carries.
template <int LOGN, int PASS>
__device__ __forceinline__ uint32_t gidx_var(uint32_t tau) {
    static_assert(PASS > 0, "pass 0 is bit-reversed");
    using G = Geo<LOGN>;
    return lay<G::S(PASS), G::R(PASS)>(tau);
}
template <int LOGN, int PASS>
__host__ __device__ constexpr uint32_t gidx_const(int e) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS), R = G::R(PASS);
    const uint32_t t = uint32_t(e) & ((1u << R) - 1), u = uint32_t(e) >> R;
    const uint32_t g = u << G::LOGT;
    return ((g & ((1u << S) - 1)) | ((g >> S) << (S + R))) | (t << S);
}

// ---------------------------------------------------------------- HBM I/O
// Buffer loads/stores through a workgroup-uniform resource (used when a
// workgroup owns one polynomial, P == 1): the lane's byte offset is shared by
// all E accesses of a layout and each access adds a compile-time constant in
// an SGPR, so no 64-bit VALU address arithmetic is issued per access.
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
constexpr int kAuxNT = 2;  // gfx950 cache policy bit 'nt': streamed once
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)0xFFFFFFFF, 0x00020000);
}
template <int AUX = kAuxNT>
__device__ __forceinline__ uint64_t bload(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, AUX));
}
template <int AUX = kAuxNT>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so, uint64_t x) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, x), r, vo, so, AUX);
}
template <typename W>
__device__ __forceinline__ Tw<W> bload_tw(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    if constexpr (sizeof(W) == 4)
        return __builtin_bit_cast(Tw<W>, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
    else
        return __builtin_bit_cast(Tw<W>, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}
// Last-pass (natural order) coefficient access of a P == 1 polynomial.
template <int LOGN>
struct LastIO {
    static constexpr int PASS = Geo<LOGN>::NP - 1;
    __device__ static uint32_t vo(uint32_t tau) { return gidx_var<LOGN, PASS>(tau) * 8u; }
    static constexpr uint32_t so(int e) { return gidx_const<LOGN, PASS>(e) * 8u; }
};

// ---------------------------------------------------------------- twiddles
// Twiddles of one pass, loaded into VGPRs ahead of use: slot (k, u, tl) is
// butterfly group tl of global stage S+k for slot-group u.  The loads of
// pass p+1 are issued before the LDS exchange + barrier that precede it, so
// their L2 latency overlaps the exchange.
template <int LOGN, int PASS>
struct PassTw {
    using G = Geo<LOGN>;
    static constexpr int S = G::S(PASS), R = G::R(PASS), NU = G::E >> R;
    static constexpr int PER_U = (1 << R) - 1;
    static constexpr int COUNT = NU * PER_U;
    static constexpr int slot(int k, int u, int tl) { return u * PER_U + ((1 << k) - 1) + tl; }
};

// PF = stages of a pass whose twiddles are loaded before the LDS exchange
// (the rest right after it): trades VGPRs for hidden L2 latency.  Measured
// on MI355X: 2 for the single-transform kernels (64-VGPR budget at two
// workgroups per CU), 4 for polymul (one workgroup per CU).
constexpr int kPfSingle = 2;
#ifndef FHE_PF_POLYMUL
#define FHE_PF_POLYMUL 4
#endif
constexpr int kPfPolymul = FHE_PF_POLYMUL;

template <int LOGN, int PASS, typename W, int K0 = 0, int K1 = 8>
__device__ __forceinline__ void load_tw(uint32_t tau, const Tw<W> *__restrict__ tw,
                                        Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT]) {
    using P = PassTw<LOGN, PASS>;
    using G = Geo<LOGN>;
    constexpr int S = P::S, R = P::R, NU = P::NU;
    constexpr int KE = K1 < R ? K1 : R;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const uint32_t jlo = g_of<LOGN, PASS>(tau, u) & ((1u << S) - 1);
#pragma unroll
        for (int k = K0; k < KE; ++k)
#pragma unroll
            for (int tl = 0; tl < (1 << k); ++tl) {
                const uint32_t idx = (1u << (S + k)) + (jlo | (uint32_t(tl) << S));
                if constexpr (PASS == 0) {  // wave-uniform: scalar loads through the constant cache
                    typedef const __attribute__((address_space(4))) W cw_t;
                    const cw_t *cp = (const cw_t *)(const void *)tw;
                    t[P::slot(k, u, tl)] = Tw<W>{cp[2 * idx], cp[2 * idx + 1]};
                } else if constexpr (G::P == 1) {
                    // idx = (tau & m) + const: jlo = (tau | u << LOGT) & m, disjoint fields
                    constexpr uint32_t m = (1u << S) - 1;
                    const uint32_t cst = (1u << (S + k)) + ((uint32_t(u) << G::LOGT) & m) + (uint32_t(tl) << S);
                    t[P::slot(k, u, tl)] = bload_tw<W>(brsrc(tw), (tau & m) * (uint32_t)sizeof(Tw<W>),
                                                       cst * (uint32_t)sizeof(Tw<W>));
                } else
                    t[P::slot(k, u, tl)] = tw[idx];
            }
    }
}

// ---------------------------------------------------------------- passes
// One stage (K) of a pass, forward (CT) / inverse (GS).  RS (pass 0, stage
// 0 only): multiply by R (ct_rscale) instead of the twiddle.
template <int LOGN, int PASS, int K, bool LAZY, typename W, bool RS = false>
__device__ __forceinline__ void fwd_stage(W (&v)[Geo<LOGN>::E], const Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                          const Arith<W> &ar, Scale<W> rmod = Scale<W>{}) {
    using P = PassTw<LOGN, PASS>;
    constexpr int R = P::R, NU = P::NU;
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int tt = 0; tt < (1 << R); ++tt) {
            if (tt & (1 << K)) continue;
            const int e = tt + (u << R), e2 = e + (1 << K);
            // unit twiddle (gk_cp): pass 0, butterfly group 0; a lazy stage
            // above 0 keeps the Shoup form (its inputs exceed 4q)
            constexpr bool UNIT = gk_cp(LOGN) && PASS == 0 && (!LAZY || K == 0);
            if constexpr (RS && PASS == 0 && K == 0) ar.template ct_rscale<gk_sp(LOGN)>(v[e], v[e2], rmod);
            else if (UNIT && (tt & ((1 << K) - 1)) == 0) ar.ct_unit(v[e], v[e2]);
            else {
                const Tw<W> w = t[P::slot(K, u, tt & ((1 << K) - 1))];
                if constexpr (LAZY) ar.template ct_lazy<gk_sp(LOGN)>(v[e], v[e2], w);
                else ar.template ct<gk_sp(LOGN)>(v[e], v[e2], w);
            }
        }
}
template <int LOGN, int PASS, int K, bool FOLD, typename W>
__device__ __forceinline__ void inv_stage(W (&v)[Geo<LOGN>::E], const Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                          const Arith<W> &ar, Scale<W> scale) {
    using P = PassTw<LOGN, PASS>;
    constexpr int S = P::S, R = P::R, NU = P::NU;
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int tt = 0; tt < (1 << R); ++tt) {
            if (tt & (1 << K)) continue;
            const int e = tt + (u << R), e2 = e + (1 << K);
            if constexpr (FOLD && S + K == 0) ar.template gs_scaled<gk_sp(LOGN)>(v[e], v[e2], scale);
            else if (gk_cp(LOGN) && PASS == 0 && (tt & ((1 << K) - 1)) == 0) ar.gs_unit(v[e], v[e2]);
            else ar.template gs<gk_sp(LOGN)>(v[e], v[e2], t[P::slot(K, u, tt & ((1 << K) - 1))]);
        }
}
// Whole passes as compile-time stage sequences (a runtime stage loop that
// the unroller gives up on indexes the twiddle and coefficient arrays
// dynamically: scratch and s_set_gpr_idx).
template <int LOGN, int PASS, int K, bool LAZY, bool RS, typename W>
__device__ __forceinline__ void fwd_stages_from(W (&v)[Geo<LOGN>::E], const Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                                const Arith<W> &ar, Scale<W> rmod) {
    if constexpr (K < PassTw<LOGN, PASS>::R) {
        fwd_stage<LOGN, PASS, K, LAZY, W, RS>(v, t, ar, rmod);
        fwd_stages_from<LOGN, PASS, K + 1, LAZY, RS>(v, t, ar, rmod);
    }
}
template <int LOGN, int PASS, int K, bool FOLD, typename W>
__device__ __forceinline__ void inv_stages_from(W (&v)[Geo<LOGN>::E], const Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                                const Arith<W> &ar, Scale<W> scale) {
    if constexpr (K >= 0) {
        inv_stage<LOGN, PASS, K, FOLD>(v, t, ar, scale);
        inv_stages_from<LOGN, PASS, K - 1, FOLD>(v, t, ar, scale);
    }
}
// Forward (CT) butterflies of pass PASS: stages S..S+R-1 ascending.  LAZY:
// no intermediate reduction (values grow by 2q per stage; valid when
// (4 + 2L) q <= 2^W).
// RS (pass 0 only): global stage 0 multiplies by R (ct_rscale).
template <int LOGN, int PASS, bool LAZY, typename W, bool RS = false>
__device__ __forceinline__ void fwd_pass(W (&v)[Geo<LOGN>::E], const Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                         const Arith<W> &ar, Scale<W> rmod = Scale<W>{}) {
    fwd_stages_from<LOGN, PASS, 0, LAZY, RS>(v, t, ar, rmod);
}
// Inverse (GS) butterflies of pass PASS: stages S+R-1..S descending.  When
// FOLD, global stage 0 (w = 1) applies the N^-1 (or N^-1 * R) scaling.
template <int LOGN, int PASS, bool FOLD, typename W>
__device__ __forceinline__ void inv_pass(W (&v)[Geo<LOGN>::E], const Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                         const Arith<W> &ar, Scale<W> scale) {
    inv_stages_from<LOGN, PASS, PassTw<LOGN, PASS>::R - 1, FOLD>(v, t, ar, scale);
}

struct NoHook {
    __device__ void operator()() const {}
};

// Staged twiddles (32 coefficients per thread, where a pass holds 31 twiddle
// pairs per slot group): the twiddles of stage K+LA are issued while stage K
// computes (LA = the stages issued before the exchange), and a scheduling
// barrier per stage stops the compiler from hoisting every load to the top
// of the pass (which costs ~60 VGPRs and spills beside two 32-word spectra).
template <int LOGN, int PASS, int K, int LOOK, bool LAZY, typename W>
__device__ __forceinline__ void fwd_stages(uint32_t tau, W (&v)[Geo<LOGN>::E], Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                           const Tw<W> *__restrict__ tw, const Arith<W> &ar) {
    constexpr int R = PassTw<LOGN, PASS>::R;
    if constexpr (K < R) {
        if constexpr (K + LOOK < R) load_tw<LOGN, PASS, W, K + LOOK, K + LOOK + 1>(tau, tw, t);
        fwd_stage<LOGN, PASS, K, LAZY>(v, t, ar);
        __builtin_amdgcn_sched_barrier(0);
        fwd_stages<LOGN, PASS, K + 1, LOOK, LAZY>(tau, v, t, tw, ar);
    }
}
template <int LOGN, int PASS, int K, int LOOK, bool FOLD, typename W>
__device__ __forceinline__ void inv_stages(uint32_t tau, W (&v)[Geo<LOGN>::E], Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT],
                                           const Tw<W> *__restrict__ tw, const Arith<W> &ar, Scale<W> scale) {
    if constexpr (K >= 0) {
        if constexpr (K - LOOK >= 0) load_tw<LOGN, PASS, W, K - LOOK, K - LOOK + 1>(tau, tw, t);
        inv_stage<LOGN, PASS, K, FOLD>(v, t, ar, scale);
        __builtin_amdgcn_sched_barrier(0);
        inv_stages<LOGN, PASS, K - 1, LOOK, FOLD>(tau, v, t, tw, ar, scale);
    }
}
template <int LOGN>
constexpr bool staged_tw() { return Geo<LOGN>::LOGE >= 5; }

// Streamed twiddles (64-bit words, 32 coefficients per thread): a radix-32
// pass needs 31 Shoup pairs (124 VGPRs) per thread, which cannot sit beside a
// 64-VGPR spectrum at two workgroups per CU.  The pass is instead walked as a
// stream of its 31 butterfly groups (stage K, group tl: the 16 >> K
// butterflies sharing twiddle slot 2^K - 1 + tl), each twiddle loaded SD
// groups ahead of its single use, so only SD pairs are live.  The first SD
// loads are issued before the pass's LDS exchange.
#ifndef FHE_STREAM_TW
#define FHE_STREAM_TW 1
#endif
#ifndef FHE_STREAM_DEPTH
#define FHE_STREAM_DEPTH 4
#endif
template <int LOGN, typename W>
constexpr bool stream_tw() { return FHE_STREAM_TW && sizeof(W) == 8 && Geo<LOGN>::LOGE == 5; }
// Paired transforms (fwd_poly2 / inv_poly2) at 32 coefficients per thread
// may stream their twiddles too (two 32-word spectra leave little room for
// whole-stage twiddle sets).  Per translation unit: measured +1.3 % on the
// ciphertext multiply (ntt_cipher.hip turns it on), -2 % on polymul.
#ifndef FHE_STREAM_TW2
#define FHE_STREAM_TW2 0
#endif
template <int LOGN, typename W>
constexpr bool stream_tw2() { return FHE_STREAM_TW2 && Geo<LOGN>::LOGE == 5; }
constexpr int kStreamDepth = FHE_STREAM_DEPTH;
// 1: a pass's first SD twiddle loads are issued before its LDS exchange
#ifndef FHE_STREAM_PRE
#define FHE_STREAM_PRE 1
#endif

// Stream item i -> (stage k, slot group u, butterfly group tl): forward
// items run stages 0..R-1, inverse items R-1..0; within a stage, slot group
// then group ascending.
struct SItem { int k, u, tl; };
__host__ __device__ constexpr SItem stream_item(int R, int NU, bool inv, int i) {
    for (int s = 0; s < R; ++s) {
        const int k = inv ? R - 1 - s : s;
        if (i < NU << k) return SItem{k, i >> k, i & ((1 << k) - 1)};
        i -= NU << k;
    }
    return SItem{0, 0, 0};
}

// Twiddle (stage k, slot group u, group tl) for this lane (load_tw's
// addressing for one slot).
template <int LOGN, int PASS, typename W>
__device__ __forceinline__ Tw<W> tw_one(uint32_t tau, const Tw<W> *__restrict__ tw, SItem it) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS);
    if constexpr (PASS == 0) {  // S = 0: wave-uniform
        typedef const __attribute__((address_space(4))) W cw_t;
        const cw_t *cp = (const cw_t *)(const void *)tw;
        const uint32_t idx = (1u << it.k) + uint32_t(it.tl);
        return Tw<W>{cp[2 * idx], cp[2 * idx + 1]};
    } else {
        static_assert(G::P == 1, "streamed twiddles: one polynomial per workgroup");
        constexpr uint32_t m = (1u << S) - 1;
        const uint32_t cst = (1u << (S + it.k)) + ((uint32_t(it.u) << G::LOGT) & m) + (uint32_t(it.tl) << S);
        return bload_tw<W>(brsrc(tw), (tau & m) * (uint32_t)sizeof(Tw<W>), cst * (uint32_t)sizeof(Tw<W>));
    }
}

// Every item index is a template argument (compile-time twiddle slot and
// register indices: a runtime index would put the arrays in scratch).
template <int LOGN, int PASS, bool INV, bool SKIP0, int I, typename W>
__device__ __forceinline__ void stream_load(uint32_t tau, const Tw<W> *__restrict__ tw,
                                            Tw<W> (&b)[PassTw<LOGN, PASS>::COUNT]) {
    using P = PassTw<LOGN, PASS>;
    if constexpr (I < P::COUNT) {
        constexpr SItem it = stream_item(P::R, P::NU, INV, I);
        if constexpr (!(SKIP0 && it.k == 0))  // stage 0 of the transform: no twiddle (R-scaling / N^-1 folding)
            b[I] = tw_one<LOGN, PASS>(tau, tw, it);
    }
}
template <int LOGN, int PASS, bool INV, bool SKIP0, int I = 0, typename W>
__device__ __forceinline__ void stream_begin(uint32_t tau, const Tw<W> *__restrict__ tw,
                                             Tw<W> (&b)[PassTw<LOGN, PASS>::COUNT]) {
    if constexpr (I < kStreamDepth) {
        stream_load<LOGN, PASS, INV, SKIP0, I>(tau, tw, b);
        stream_begin<LOGN, PASS, INV, SKIP0, I + 1>(tau, tw, b);
    }
}
// Forward pass over the stream (stream_begin already issued).  RS: pass 0's
// stage 0 multiplies by R (ct_rscale) instead of a twiddle.  D2: a second
// spectrum *v2 takes the same butterflies (paired transforms, one twiddle
// stream).
template <int LOGN, int PASS, bool LAZY, bool RS, bool D2 = false, int I = 0, typename W>
__device__ __forceinline__ void fwd_pass_stream(uint32_t tau, W (&v)[Geo<LOGN>::E], Tw<W> (&b)[PassTw<LOGN, PASS>::COUNT],
                                                const Tw<W> *__restrict__ tw, const Arith<W> &ar, Scale<W> rmod = Scale<W>{},
                                                W (*v2)[Geo<LOGN>::E] = nullptr) {
    using P = PassTw<LOGN, PASS>;
    constexpr int R = P::R;
    constexpr bool SK = RS && PASS == 0;
    if constexpr (I < P::COUNT) {
        stream_load<LOGN, PASS, false, SK, I + kStreamDepth>(tau, tw, b);
        constexpr SItem it = stream_item(R, P::NU, false, I);
        constexpr int k = it.k;
#pragma unroll
        for (int h = 0; h < (D2 ? 2 : 1); ++h) {
            W (&x)[Geo<LOGN>::E] = h ? *v2 : v;
#pragma unroll
            for (int tt = 0; tt < (1 << R); ++tt) {
                if ((tt & (1 << k)) || (tt & ((1 << k) - 1)) != it.tl) continue;
                const int e = tt + (it.u << R), e2 = e + (1 << k);
                if constexpr (SK && k == 0) ar.template ct_rscale<gk_sp(LOGN)>(x[e], x[e2], rmod);
                else if constexpr (LAZY) ar.template ct_lazy<gk_sp(LOGN)>(x[e], x[e2], b[I]);
                else ar.template ct<gk_sp(LOGN)>(x[e], x[e2], b[I]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        fwd_pass_stream<LOGN, PASS, LAZY, RS, D2, I + 1>(tau, v, b, tw, ar, rmod, v2);
    }
}
// Inverse pass over the stream; FOLD: global stage 0 applies `scale`.
template <int LOGN, int PASS, bool FOLD, bool D2 = false, int I = 0, typename W>
__device__ __forceinline__ void inv_pass_stream(uint32_t tau, W (&v)[Geo<LOGN>::E], Tw<W> (&b)[PassTw<LOGN, PASS>::COUNT],
                                                const Tw<W> *__restrict__ tw, const Arith<W> &ar, Scale<W> scale,
                                                W (*v2)[Geo<LOGN>::E] = nullptr) {
    using P = PassTw<LOGN, PASS>;
    constexpr int R = P::R;
    constexpr bool SK = FOLD && PASS == 0;
    if constexpr (I < P::COUNT) {
        stream_load<LOGN, PASS, true, SK, I + kStreamDepth>(tau, tw, b);
        constexpr SItem it = stream_item(R, P::NU, true, I);
        constexpr int k = it.k;
#pragma unroll
        for (int h = 0; h < (D2 ? 2 : 1); ++h) {
            W (&x)[Geo<LOGN>::E] = h ? *v2 : v;
#pragma unroll
            for (int tt = 0; tt < (1 << R); ++tt) {
                if ((tt & (1 << k)) || (tt & ((1 << k) - 1)) != it.tl) continue;
                const int e = tt + (it.u << R), e2 = e + (1 << k);
                if constexpr (SK && k == 0) ar.template gs_scaled<gk_sp(LOGN)>(x[e], x[e2], scale);
                else ar.template gs<gk_sp(LOGN)>(x[e], x[e2], b[I]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        inv_pass_stream<LOGN, PASS, FOLD, D2, I + 1>(tau, v, b, tw, ar, scale, v2);
    }
}

// Passes PASS..NP-1 of the forward transform, exchanging through LDS.
// hook() runs once, in the last pass after its twiddle loads are issued: the
// place to start HBM loads for what follows the transform (VMEM counters
// retire in order, so loads issued earlier would make every later twiddle
// wait for them).
template <int LOGN, int PASS, bool LAZY, int PF, typename W, typename H = NoHook>
__device__ __forceinline__ void fwd_rest(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, const Tw<W> *__restrict__ tw,
                                         const Arith<W> &ar, H &&hook = NoHook{}) {
    using G = Geo<LOGN>;
    if constexpr (PASS < G::NP) {
        Tw<W> t[PassTw<LOGN, PASS>::COUNT];
        if constexpr (stream_tw<LOGN, W>()) {
            if constexpr (FHE_STREAM_PRE) stream_begin<LOGN, PASS, false, false>(tau, tw, t);  // in flight across the exchange
            exchange<LOGN, PASS - 1, PASS>(lds, v, tau);
            if constexpr (!FHE_STREAM_PRE) stream_begin<LOGN, PASS, false, false>(tau, tw, t);
            if constexpr (PASS == G::NP - 1) hook();
            fwd_pass_stream<LOGN, PASS, LAZY, false>(tau, v, t, tw, ar);
            fwd_rest<LOGN, PASS + 1, LAZY, PF>(lds, v, tau, tw, ar, hook);
            return;
        }
        load_tw<LOGN, PASS, W, 0, PF>(tau, tw, t);  // in flight across the exchange
        exchange<LOGN, PASS - 1, PASS>(lds, v, tau);
        if constexpr (staged_tw<LOGN>()) {
            // stages 0..PF-1 issued before the exchange; stage K issues K+PF
            if constexpr (PASS == G::NP - 1) hook();
            fwd_stages<LOGN, PASS, 0, PF, LAZY>(tau, v, t, tw, ar);
        } else {
            load_tw<LOGN, PASS, W, PF, 8>(tau, tw, t);
            if constexpr (PASS == G::NP - 1) hook();
            fwd_pass<LOGN, PASS, LAZY>(v, t, ar);
        }
        fwd_rest<LOGN, PASS + 1, LAZY, PF>(lds, v, tau, tw, ar, hook);
    }
}

// ---------------------------------------------------------------- dual
// Two forward transforms in lockstep (polymul's fwd(a) and fwd(b)): every
// twiddle is loaded once and applied to both, the butterflies of the two
// are independent (twice the ILP of one transform), and no spectrum has to
// be parked while the other runs.  One LDS exchange buffer serves both in
// turn (store a / sync / load a / sync / store b / sync / load b).
template <int LOGN, int PASS, int K, int LOOK, bool LAZY, typename W>
__device__ __forceinline__ void fwd_stages2(uint32_t tau, W (&v)[Geo<LOGN>::E], W (&v2)[Geo<LOGN>::E],
                                            Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT], const Tw<W> *__restrict__ tw,
                                            const Arith<W> &ar) {
    constexpr int R = PassTw<LOGN, PASS>::R;
    if constexpr (K < R) {
        if constexpr (K + LOOK < R) load_tw<LOGN, PASS, W, K + LOOK, K + LOOK + 1>(tau, tw, t);
        fwd_stage<LOGN, PASS, K, LAZY>(v, t, ar);
        fwd_stage<LOGN, PASS, K, LAZY>(v2, t, ar);
        __builtin_amdgcn_sched_barrier(0);
        fwd_stages2<LOGN, PASS, K + 1, LOOK, LAZY>(tau, v, v2, t, tw, ar);
    }
}
template <int LOGN, int PASS, bool LAZY, int PF, typename W>
__device__ __forceinline__ void fwd_rest2(W *lds, W (&v)[Geo<LOGN>::E], W (&v2)[Geo<LOGN>::E], uint32_t tau,
                                          const Tw<W> *__restrict__ tw, const Arith<W> &ar) {
    using G = Geo<LOGN>;
    if constexpr (PASS < G::NP) {
        Tw<W> t[PassTw<LOGN, PASS>::COUNT];
        if constexpr (stream_tw2<LOGN, W>()) {
            stream_begin<LOGN, PASS, false, false>(tau, tw, t);
            exchange<LOGN, PASS - 1, PASS>(lds, v, tau);
            xbar<lab_local<PASS - 1, PASS>()>();
            exchange<LOGN, PASS - 1, PASS>(lds, v2, tau);
            fwd_pass_stream<LOGN, PASS, LAZY, false, true>(tau, v, t, tw, ar, Scale<W>{}, &v2);
            fwd_rest2<LOGN, PASS + 1, LAZY, PF>(lds, v, v2, tau, tw, ar);
            return;
        }
        load_tw<LOGN, PASS, W, 0, PF>(tau, tw, t);
        exchange<LOGN, PASS - 1, PASS>(lds, v, tau);
        xbar<lab_local<PASS - 1, PASS>()>();
        exchange<LOGN, PASS - 1, PASS>(lds, v2, tau);
        fwd_stages2<LOGN, PASS, 0, PF, LAZY>(tau, v, v2, t, tw, ar);
        fwd_rest2<LOGN, PASS + 1, LAZY, PF>(lds, v, v2, tau, tw, ar);
    }
}

// Passes PASS..0 of the inverse transform (PASS+1 already in registers).
template <int LOGN, int PASS, bool FOLD, int PF, typename W>
__device__ __forceinline__ void inv_rest(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, const Tw<W> *__restrict__ tw,
                                         const Arith<W> &ar, Scale<W> scale) {
    if constexpr (PASS >= 0) {
        Tw<W> t[PassTw<LOGN, PASS>::COUNT];
        if constexpr (stream_tw<LOGN, W>()) {
            if constexpr (FHE_STREAM_PRE) stream_begin<LOGN, PASS, true, FOLD && PASS == 0>(tau, tw, t);
            exchange<LOGN, PASS + 1, PASS>(lds, v, tau);
            if constexpr (!FHE_STREAM_PRE) stream_begin<LOGN, PASS, true, FOLD && PASS == 0>(tau, tw, t);
            inv_pass_stream<LOGN, PASS, FOLD>(tau, v, t, tw, ar, scale);
            inv_rest<LOGN, PASS - 1, FOLD, PF>(lds, v, tau, tw, ar, scale);
            return;
        }
        // inverse stages run k = R-1 .. 0: prefetch the top ones
        constexpr int R = PassTw<LOGN, PASS>::R;
        constexpr int KS = R - PF < 0 ? 0 : R - PF;
        load_tw<LOGN, PASS, W, KS, 8>(tau, tw, t);
        exchange<LOGN, PASS + 1, PASS>(lds, v, tau);
        if constexpr (staged_tw<LOGN>()) {
            // stages R-1..KS issued before the exchange; stage K issues K-PF
            inv_stages<LOGN, PASS, R - 1, R - KS, FOLD>(tau, v, t, tw, ar, scale);
        } else {
            load_tw<LOGN, PASS, W, 0, KS>(tau, tw, t);
            inv_pass<LOGN, PASS, FOLD>(v, t, ar, scale);
        }
        inv_rest<LOGN, PASS - 1, FOLD, PF>(lds, v, tau, tw, ar, scale);
    }
}

// Per-launch constants.
template <typename W>
struct NttArgs {
    const Tw<W> *twf;      // forward stage table
    const Tw<W> *twi;      // inverse stage table
    Arith<W> ar;
    uint64_t q64, mu64;    // exact slow-path reduction of out-of-range inputs
    // Stage-0 multipliers (Scale): the inverse folds N^-1 into its last GS
    // stage and the R-scaled forward multiplies by R in its first CT stage,
    // each in place of that stage's twiddle w0 -- 1 in compat mode, psi^(N/2)
    // in negacyclic mode (merged stage tables), so .b carries w0 (or w0^-1).
    Scale<W> ninv;         // {N^-1, N^-1 w0^-1}
    Scale<W> ninv_r;       // {N^-1 R, N^-1 R w0^-1}  (after a Montgomery pointwise product)
    Scale<W> rs;           // {R, R w0}  (fwd * R, Montgomery form)
    Tw<W> rmod;            // R mod q  (to Montgomery form)
    Tw<W> one;             // {1, floor(2^W / q)}: shoup(x, one) = x mod q in [0, 2q)
};

// Any forward-transform output (< (4+2L) q when LAZY, < 4q otherwise) to
// [0, 2q) / to canonical.
template <bool LAZY, typename W>
__device__ __forceinline__ W fwd_to_2q(W x, const NttArgs<W> &A) {
    if constexpr (LAZY) return A.ar.shoup(x, A.one);
    else return A.ar.red2q(x);
}
template <bool LAZY, typename W>
__device__ __forceinline__ W fwd_to_canon(W x, const NttArgs<W> &A) {
    return A.ar.red1q(fwd_to_2q<LAZY>(x, A));
}

// Exact reduction of an out-of-range input word (any u64 behaves as x mod q).
// 32-bit lanes: x = hi 2^32 + lo -> shoup(hi, 2^32 mod q) + shoup(lo, 1),
// then canonical -- 32-bit multiplies only, a few registers (the 64-bit
// Barrett step of mod64_slow spilled in the cold paths of the 32-coefficient
// kernels).  64-bit lanes: mod64_slow.
template <typename W>
struct SlowRed {
    const NttArgs<W> &A;
    __device__ __forceinline__ uint64_t operator()(uint64_t x) const {
        if constexpr (sizeof(W) == 4) {
            const W r = A.ar.shoup((W)(x >> 32), A.rmod) + A.ar.shoup((W)x, A.one);  // [0, 4q)
            return (uint64_t)A.ar.canon4(r);
        } else {
            return mod64_slow(x, A.q64, A.mu64);
        }
    }
};
struct Mod64Red {
    uint64_t q, mu;
    __device__ __forceinline__ uint64_t operator()(uint64_t x) const { return mod64_slow(x, q, mu); }
};

// E coefficients of one polynomial from HBM into the lazy range [0, lim) of
// word W.  Out-of-range inputs take one divergent slow path for the whole
// thread, one element at a time (a scheduling barrier each: no spills).
template <int E, typename W, typename RD>
__device__ __forceinline__ void coeffs_from_raw(W (&v)[E], uint64_t (&raw)[E], uint64_t lim, RD &&red) {
    bool bad = false;
#pragma unroll
    for (int t = 0; t < E; ++t) bad |= raw[t] >= lim;
    if (__builtin_expect(bad, 0)) {
#pragma unroll
        for (int t = 0; t < E; ++t) {
            if (raw[t] >= lim) raw[t] = red(raw[t]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int t = 0; t < E; ++t) v[t] = W(raw[t]);
}
template <int E, typename W>
__device__ __forceinline__ void coeffs_from_raw(W (&v)[E], uint64_t (&raw)[E], uint64_t lim, uint64_t q, uint64_t mu) {
    coeffs_from_raw<E>(v, raw, lim, Mod64Red{q, mu});
}
// The raw words are narrowed as soon as they are checked; an out-of-range
// word is loaded again in the (cold) slow path, so no 64-bit word stays live
// across it (that is what spilled).
template <int E, typename W, typename RD, typename F>
__device__ __forceinline__ void load_coeffs_r(W (&v)[E], uint64_t lim, RD &&red, F &&addr_of) {
    uint64_t raw[E];
#pragma unroll
    for (int t = 0; t < E; ++t) raw[t] = addr_of(t);
    uint32_t bad = 0;
#pragma unroll
    for (int t = 0; t < E; ++t) {
        bad |= uint32_t(raw[t] >= lim) << t;
        v[t] = W(raw[t]);
    }
    if (__builtin_expect(bad != 0, 0)) {
#pragma unroll
        for (int t = 0; t < E; ++t)
            if ((bad >> t) & 1) v[t] = W(red(addr_of(t)));
    }
}
// Computed digit loads (k_dmac): no reload (the lambda is not a plain load).
template <int E, typename W, typename F>
__device__ __forceinline__ void load_coeffs(W (&v)[E], uint64_t lim, uint64_t q, uint64_t mu, F &&addr_of) {
    uint64_t raw[E];
#pragma unroll
    for (int t = 0; t < E; ++t) raw[t] = addr_of(t);
    coeffs_from_raw<E>(v, raw, lim, Mod64Red{q, mu});
}

#ifndef FHE_LOAD_INFLIGHT
#define FHE_LOAD_INFLIGHT 1
#endif
// coefficients per load chunk of the paired transforms (fwd_poly2)
#ifndef FHE_POLY2_CH
#define FHE_POLY2_CH 8
#endif
// As load_coeffs, for 32 coefficients per thread: raw u64 words are 2 VGPRs
// each, so only IN chunks of CH are in flight at once and each chunk is
// narrowed before the next is issued (scheduling barriers keep the compiler
// from hoisting all 32 loads, which spills beside a parked spectrum).
template <int E, int CH, int IN, typename W, typename RD, typename F>
__device__ __forceinline__ void load_coeffs_chunked(W (&v)[E], uint64_t lim, RD &&red, F &&addr_of) {
    constexpr int NC = E / CH;
    uint64_t raw[E];
#pragma unroll
    for (int c = 0; c < IN && c < NC; ++c)
#pragma unroll
        for (int t = c * CH; t < c * CH + CH; ++t) raw[t] = addr_of(t);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (c + IN < NC) {
#pragma unroll
            for (int t = (c + IN) * CH; t < (c + IN) * CH + CH; ++t) raw[t] = addr_of(t);
        }
        __builtin_amdgcn_sched_barrier(0);
        uint32_t bad = 0;
#pragma unroll
        for (int t = c * CH; t < c * CH + CH; ++t) {
            bad |= uint32_t(raw[t] >= lim) << (t - c * CH);
            v[t] = W(raw[t]);
        }
        if (__builtin_expect(bad != 0, 0)) {  // reload and reduce (see load_coeffs_r)
#pragma unroll
            for (int t = c * CH; t < c * CH + CH; ++t)
                if ((bad >> (t - c * CH)) & 1) v[t] = W(red(addr_of(t)));
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Forward transform of one polynomial held by this thread group: HBM load
// (bit-reversed, coalesced), all passes; result left in v (last layout,
// values in [0, 4q), or [0, (4+2L)q) when LAZY; every bound is <= R, so a
// raw output times a canonical residue is a valid Montgomery operand pair).
// RS: the result is the transform times R (Montgomery form).
//
// Sub-transform use (N > 16384, ntt_big.hip): the 2^LOGN coefficients are
// the strided subsequence src[i << sh] of a larger polynomial; the prefix
// stages of the big transform use the same stage-major twiddles.
// Raw pass-0 coefficients of a P == 1 polynomial (bit-reversed order), for
// prefetching through a fwd_rest hook.
template <int LOGN>
__device__ __forceinline__ void load_raw(uint64_t (&raw)[Geo<LOGN>::E], uint32_t tau, const uint64_t *src) {
    using G = Geo<LOGN>;
    const auto r = brsrc(src);
#pragma unroll
    for (int t = 0; t < G::E; ++t) raw[t] = bload(r, tau * 8u, cbrv(t, G::LOGE) * G::T * 8u);
}
template <int LOGN, bool LAZY, int PF = kPfSingle, bool RS = false, typename W, typename H = NoHook>
__device__ __forceinline__ void fwd_poly(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, const uint64_t *__restrict__ src,
                                         bool valid, const NttArgs<W> &A, uint32_t sh = 0, H &&hook = NoHook{}, uint64_t (*pre)[Geo<LOGN>::E] = nullptr) {
    using G = Geo<LOGN>;
    constexpr bool ST = stream_tw<LOGN, W>();
    const Tw<W> *const twf = opaque_tw(A.twf);
    Tw<W> t0[PassTw<LOGN, 0>::COUNT];
    if constexpr (!ST) load_tw<LOGN, 0>(tau, twf, t0);
    // a Shoup-based first step (R-scaling) accepts any word
    const uint64_t lim = RS ? (uint64_t)(W)~W(0) : (uint64_t)(A.ar.q2 * 2);
    if (pre) {  // prefetched by the caller (load_raw)
        coeffs_from_raw<G::E>(v, *pre, lim, SlowRed<W>{A});
    } else if constexpr (G::P == 1) {  // the caller has returned early if !valid
        const auto r = brsrc(src);
        const uint32_t vo = (tau << sh) * 8u;
        auto at = [&](int t) -> uint64_t { return bload(r, vo, ((cbrv(t, G::LOGE) * G::T) << sh) * 8u); };
        if constexpr (G::LOGE == 5) load_coeffs_chunked<G::E, 8, FHE_LOAD_INFLIGHT>(v, lim, SlowRed<W>{A}, at);
        else load_coeffs_r<G::E>(v, lim, SlowRed<W>{A}, at);
    } else {
        load_coeffs_r<G::E>(v, lim, SlowRed<W>{A}, [&](int t) -> uint64_t {
            return valid ? __builtin_nontemporal_load(src + ((tau + cbrv(t, G::LOGE) * G::T) << sh)) : 0;
        });
    }
    if constexpr (ST) {
        stream_begin<LOGN, 0, false, RS>(tau, twf, t0);
        fwd_pass_stream<LOGN, 0, LAZY, RS>(tau, v, t0, twf, A.ar, A.rs);
    } else {
        fwd_pass<LOGN, 0, LAZY, W, RS>(v, t0, A.ar, A.rs);
    }
    fwd_rest<LOGN, 1, LAZY, PF>(lds, v, tau, twf, A.ar, hook);
}

// fwd_poly for two polynomials at once (P == 1, no sub-transform offsets):
// results in v (from src) and v2 (from src2), last-pass layout.
template <int LOGN, bool LAZY, int PF, typename W>
__device__ __forceinline__ void fwd_poly2(W *lds, W (&v)[Geo<LOGN>::E], W (&v2)[Geo<LOGN>::E], uint32_t tau,
                                          const uint64_t *__restrict__ src, const uint64_t *__restrict__ src2,
                                          const NttArgs<W> &A) {
    using G = Geo<LOGN>;
    static_assert(G::P == 1, "dual transform: one polynomial pair per workgroup");
    constexpr bool ST = stream_tw2<LOGN, W>();
    const Tw<W> *const twf = opaque_tw(A.twf);
    Tw<W> t0[PassTw<LOGN, 0>::COUNT];
    if constexpr (!ST) load_tw<LOGN, 0>(tau, twf, t0);
    const uint64_t lim = (uint64_t)(A.ar.q2 * 2);
    const uint32_t vo = tau * 8u;
    {
        const auto r = brsrc(src);
        load_coeffs_chunked<G::E, FHE_POLY2_CH, FHE_LOAD_INFLIGHT>(v, lim, SlowRed<W>{A}, [&](int t) -> uint64_t {
            return bload(r, vo, cbrv(t, G::LOGE) * G::T * 8u);
        });
    }
    {
        const auto r = brsrc(src2);
        load_coeffs_chunked<G::E, FHE_POLY2_CH, FHE_LOAD_INFLIGHT>(v2, lim, SlowRed<W>{A}, [&](int t) -> uint64_t {
            return bload(r, vo, cbrv(t, G::LOGE) * G::T * 8u);
        });
    }
    if constexpr (ST) {
        stream_begin<LOGN, 0, false, false>(tau, twf, t0);
        fwd_pass_stream<LOGN, 0, LAZY, false, true>(tau, v, t0, twf, A.ar, Scale<W>{}, &v2);
    } else {
        fwd_pass<LOGN, 0, LAZY, W>(v, t0, A.ar);
        fwd_pass<LOGN, 0, LAZY, W>(v2, t0, A.ar);
    }
    fwd_rest2<LOGN, 1, LAZY, PF>(lds, v, v2, tau, twf, A.ar);
}

// Inverse transform from v (last-pass layout, values in [0, 2q)) to HBM
// (bit-reversed store, coalesced), canonical output.  scale = N^-1 or
// N^-1 * R, folded into the last stage.
// Sub-transform use (ntt_big.hip): output i goes to dst[i << sh].
// fin(gi, x): final map of canonical output x at global index gi (an
// epilogue fused into the store, e.g. "+ c0" of a relinearisation).
struct NoFin {
    __device__ uint64_t operator()(uint32_t, uint64_t x) const { return x; }
};
// STORE = false: fin() does every store itself (dst unused).
template <int LOGN, int PF = kPfSingle, bool STORE = true, typename W, typename F = NoFin>
__device__ __forceinline__ void inv_poly_from_regs(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, uint64_t *__restrict__ dst,
                                                   bool valid, const NttArgs<W> &A, Scale<W> scale, uint32_t sh = 0,
                                                   F &&fin = NoFin{}) {
    using G = Geo<LOGN>;
    constexpr int LAST = G::NP - 1;
    const Tw<W> *const twi = opaque_tw(A.twi);
    {
        Tw<W> t[PassTw<LOGN, LAST>::COUNT];
        if constexpr (stream_tw<LOGN, W>()) {
            stream_begin<LOGN, LAST, true, false>(tau, twi, t);
            inv_pass_stream<LOGN, LAST, true>(tau, v, t, twi, A.ar, scale);
        } else {
            load_tw<LOGN, LAST>(tau, twi, t);
            inv_pass<LOGN, LAST, true>(v, t, A.ar, scale);
        }
    }
    inv_rest<LOGN, LAST - 1, true, PF>(lds, v, tau, twi, A.ar, scale);
#pragma unroll
    for (int t = 0; t < G::E; ++t) {
        const uint32_t gi = (tau + cbrv(t, G::LOGE) * G::T) << sh;
        const uint64_t y = fin(gi, (uint64_t)A.ar.red1q(v[t]));
        if constexpr (!STORE) (void)y;
        else if constexpr (G::P == 1)
            bstore(brsrc(dst), (tau << sh) * 8u, ((cbrv(t, G::LOGE) * G::T) << sh) * 8u, y);
        else if (valid)
            __builtin_nontemporal_store(y, dst + gi);
    }
}

// Two inverse transforms in lockstep (shared twiddles, two butterfly
// streams), every pass staged (the last pass too: two 32-word spectra leave
// no room for a whole pass of twiddles).  Inputs in [0, 2q), last-pass
// layout; canonical outputs stored to dst / dst2 (P == 1).
template <int LOGN, int PASS, int K, int LOOK, bool FOLD, typename W>
__device__ __forceinline__ void inv_stages2(uint32_t tau, W (&v)[Geo<LOGN>::E], W (&v2)[Geo<LOGN>::E],
                                            Tw<W> (&t)[PassTw<LOGN, PASS>::COUNT], const Tw<W> *__restrict__ tw,
                                            const Arith<W> &ar, Scale<W> scale) {
    if constexpr (K >= 0) {
        if constexpr (K - LOOK >= 0) load_tw<LOGN, PASS, W, K - LOOK, K - LOOK + 1>(tau, tw, t);
        inv_stage<LOGN, PASS, K, FOLD>(v, t, ar, scale);
        inv_stage<LOGN, PASS, K, FOLD>(v2, t, ar, scale);
        __builtin_amdgcn_sched_barrier(0);
        inv_stages2<LOGN, PASS, K - 1, LOOK, FOLD>(tau, v, v2, t, tw, ar, scale);
    }
}
template <int LOGN, int PASS, bool FOLD, int PF, typename W>
__device__ __forceinline__ void inv_rest2(W *lds, W (&v)[Geo<LOGN>::E], W (&v2)[Geo<LOGN>::E], uint32_t tau,
                                          const Tw<W> *__restrict__ tw, const Arith<W> &ar, Scale<W> scale) {
    if constexpr (PASS >= 0) {
        Tw<W> t[PassTw<LOGN, PASS>::COUNT];
        if constexpr (stream_tw2<LOGN, W>()) {
            stream_begin<LOGN, PASS, true, FOLD && PASS == 0>(tau, tw, t);
            exchange<LOGN, PASS + 1, PASS>(lds, v, tau);
            xbar<lab_local<PASS + 1, PASS>()>();
            exchange<LOGN, PASS + 1, PASS>(lds, v2, tau);
            inv_pass_stream<LOGN, PASS, FOLD, true>(tau, v, t, tw, ar, scale, &v2);
            inv_rest2<LOGN, PASS - 1, FOLD, PF>(lds, v, v2, tau, tw, ar, scale);
            return;
        }
        constexpr int R = PassTw<LOGN, PASS>::R;
        constexpr int KS = R - PF < 0 ? 0 : R - PF;
        load_tw<LOGN, PASS, W, KS, 8>(tau, tw, t);
        exchange<LOGN, PASS + 1, PASS>(lds, v, tau);
        xbar<lab_local<PASS + 1, PASS>()>();
        exchange<LOGN, PASS + 1, PASS>(lds, v2, tau);
        inv_stages2<LOGN, PASS, R - 1, R - KS, FOLD>(tau, v, v2, t, tw, ar, scale);
        inv_rest2<LOGN, PASS - 1, FOLD, PF>(lds, v, v2, tau, tw, ar, scale);
    }
}
template <int LOGN, int PF, typename W, typename F1 = NoFin, typename F2 = NoFin>
__device__ __forceinline__ void inv_poly2(W *lds, W (&v)[Geo<LOGN>::E], W (&v2)[Geo<LOGN>::E], uint32_t tau,
                                          uint64_t *__restrict__ dst, uint64_t *__restrict__ dst2,
                                          const NttArgs<W> &A, Scale<W> scale, F1 &&fin1 = NoFin{}, F2 &&fin2 = NoFin{}) {
    using G = Geo<LOGN>;
    static_assert(G::P == 1, "dual transform: one polynomial pair per workgroup");
    constexpr int LAST = G::NP - 1;
    const Tw<W> *const twi = opaque_tw(A.twi);
    {
        Tw<W> t[PassTw<LOGN, LAST>::COUNT];
        if constexpr (stream_tw2<LOGN, W>()) {
            stream_begin<LOGN, LAST, true, false>(tau, twi, t);
            inv_pass_stream<LOGN, LAST, true, true>(tau, v, t, twi, A.ar, scale, &v2);
        } else {
            constexpr int R = PassTw<LOGN, LAST>::R;
            constexpr int KS = R - PF < 0 ? 0 : R - PF;
            load_tw<LOGN, LAST, W, KS, 8>(tau, twi, t);
            inv_stages2<LOGN, LAST, R - 1, R - KS, true>(tau, v, v2, t, twi, A.ar, scale);
        }
    }
    inv_rest2<LOGN, LAST - 1, true, PF>(lds, v, v2, tau, twi, A.ar, scale);
    const auto r1 = brsrc(dst), r2 = brsrc(dst2);
#pragma unroll
    for (int t = 0; t < G::E; ++t) {
        const uint32_t gi = tau + cbrv(t, G::LOGE) * G::T;
        bstore(r1, tau * 8u, cbrv(t, G::LOGE) * G::T * 8u, fin1(gi, (uint64_t)A.ar.red1q(v[t])));
        bstore(r2, tau * 8u, cbrv(t, G::LOGE) * G::T * 8u, fin2(gi, (uint64_t)A.ar.red1q(v2[t])));
    }
}

}  // namespace FHE_NS
