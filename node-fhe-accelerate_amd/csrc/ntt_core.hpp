// ntt_core.hpp -- one-workgroup-per-polynomial fused NTT building blocks.
//
// Transform reproduced (ntt_processor.cpp:262-380):
//   forward:  bit-reverse, then for stage s = 0..L-1 (m = 2^s), pairs
//             (k+j, k+j+m) with twiddle psi^(j*N/2m)  (compat mode), or
//             psi^(j*N/m) after a psi^i pre-twist (negacyclic mode);
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
//   * LDS addresses are XOR-swizzled per degree so every ds_read/ds_write
//     of the pass layouts is bank-conflict free (masks found by exhaustive
//     simulation of the access patterns).
#pragma once
#include "fhe_arith.hpp"

namespace fhe {

// ---------------------------------------------------------------- geometry
template <int LOGN>
struct Geo {
    static constexpr int L = LOGN;
    static constexpr int N = 1 << L;
    static constexpr int LOGE = L < 4 ? L : 4;
    static constexpr int E = 1 << LOGE;
    static constexpr int LOGT = L - LOGE;
    static constexpr int T = 1 << LOGT;
    static constexpr int NP = (L + LOGE - 1) / LOGE;  // passes
    static constexpr int P = T >= 256 ? 1 : 256 / T;  // polynomials per workgroup
    static constexpr int THREADS = T * P;
    static constexpr int S(int p) { return p * LOGE; }
    static constexpr int R(int p) { return (L - p * LOGE) < LOGE ? (L - p * LOGE) : LOGE; }
};

__host__ __device__ constexpr uint32_t cbrv(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

// XOR swizzle masks: bit b (b >= 5) of a coefficient index flips these low
// bits.  kSwz[L][b].  Zero-conflict for L >= 9 under the pass layouts.
constexpr uint32_t kSwz[17][17] = {
    {}, {}, {}, {}, {}, {},
    /* 6 */ {0, 0, 0, 0, 0, 11},
    /* 7 */ {0, 0, 0, 0, 0, 3, 6},
    /* 8 */ {0, 0, 0, 0, 0, 24, 2, 28},
    /* 9 */ {0, 0, 0, 0, 0, 7, 1, 28, 21},
    /*10 */ {0, 0, 0, 0, 0, 2, 27, 30, 31, 13},
    /*11 */ {0, 0, 0, 0, 0, 2, 15, 9, 20, 1, 30},
    /*12 */ {0, 0, 0, 0, 0, 30, 17, 22, 17, 24, 29, 23},
    /*13 */ {0, 0, 0, 0, 0, 17, 22, 4, 31, 10, 14, 23, 28},
    /*14 */ {0, 0, 0, 0, 0, 10, 17, 24, 31, 18, 11, 26, 29, 5},
    /*15 */ {0, 0, 0, 0, 0, 13, 21, 2, 19, 22, 1, 3, 9, 23, 15},
    {},
};

template <int L>
__host__ __device__ constexpr uint32_t swz_c(uint32_t i) {
    uint32_t a = i;
    for (int b = 5; b < L; ++b)
        if ((i >> b) & 1) a ^= kSwz[L][b];
    return a;
}
template <int L>
__device__ __forceinline__ uint32_t swz_rt(uint32_t i) {
    uint32_t a = i;
#pragma unroll
    for (int b = 5; b < L; ++b) a ^= ((i >> b) & 1) ? kSwz[L][b] : 0u;
    return a;
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
        uint32_t base = swz_rt<LOGN>(lay<S, R>(g_of<LOGN, PASS>(tau, u)));
#pragma unroll
        for (int t = 0; t < (1 << R); ++t)
            lds[base ^ swz_c<LOGN>(uint32_t(t) << S)] = v[t + (u << R)];
    }
}
template <int LOGN, int PASS, typename W>
__device__ __forceinline__ void lds_load(const W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS), R = G::R(PASS), NU = G::E >> R;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        uint32_t base = swz_rt<LOGN>(lay<S, R>(g_of<LOGN, PASS>(tau, u)));
#pragma unroll
        for (int t = 0; t < (1 << R); ++t)
            v[t + (u << R)] = lds[base ^ swz_c<LOGN>(uint32_t(t) << S)];
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

// ---------------------------------------------------------------- passes
// Forward (CT) butterflies of pass PASS: stages S..S+R-1 ascending.
template <int LOGN, int PASS, typename W>
__device__ __forceinline__ void fwd_pass(W (&v)[Geo<LOGN>::E], uint32_t tau, const Tw<W> *__restrict__ tw,
                                         const Arith<W> &ar) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS), R = G::R(PASS), NU = G::E >> R;
#pragma unroll
    for (int k = 0; k < R; ++k) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const uint32_t jlo = g_of<LOGN, PASS>(tau, u) & ((1u << S) - 1);
#pragma unroll
            for (int t = 0; t < (1 << R); ++t) {
                if (t & (1 << k)) continue;
                const int e = t + (u << R), e2 = e + (1 << k);
                const uint32_t j = jlo | (uint32_t(t & ((1 << k) - 1)) << S);
                const Tw<W> w = tw[(1u << (S + k)) + j];
                ar.ct(v[e], v[e2], w);
            }
        }
    }
}

// Inverse (GS) butterflies of pass PASS: stages S+R-1..S descending.  When
// FOLD, global stage 0 (w = 1) applies the N^-1 (or N^-1 * R) scaling.
template <int LOGN, int PASS, bool FOLD, typename W>
__device__ __forceinline__ void inv_pass(W (&v)[Geo<LOGN>::E], uint32_t tau, const Tw<W> *__restrict__ tw,
                                         const Arith<W> &ar, Tw<W> scale) {
    using G = Geo<LOGN>;
    constexpr int S = G::S(PASS), R = G::R(PASS), NU = G::E >> R;
#pragma unroll
    for (int k = R - 1; k >= 0; --k) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const uint32_t jlo = g_of<LOGN, PASS>(tau, u) & ((1u << S) - 1);
#pragma unroll
            for (int t = 0; t < (1 << R); ++t) {
                if (t & (1 << k)) continue;
                const int e = t + (u << R), e2 = e + (1 << k);
                if (FOLD && S + k == 0) {
                    ar.gs_scaled(v[e], v[e2], scale);
                } else {
                    const uint32_t j = jlo | (uint32_t(t & ((1 << k) - 1)) << S);
                    const Tw<W> w = tw[(1u << (S + k)) + j];
                    ar.gs(v[e], v[e2], w);
                }
            }
        }
    }
}

// Passes 1..NP-1 of the forward transform, exchanging through LDS.
template <int LOGN, int PASS, typename W>
__device__ __forceinline__ void fwd_rest(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, const Tw<W> *__restrict__ tw,
                                         const Arith<W> &ar) {
    using G = Geo<LOGN>;
    if constexpr (PASS < G::NP) {
        lds_store<LOGN, PASS - 1>(lds, v, tau);
        __syncthreads();
        lds_load<LOGN, PASS>(lds, v, tau);
        fwd_pass<LOGN, PASS>(v, tau, tw, ar);
        fwd_rest<LOGN, PASS + 1>(lds, v, tau, tw, ar);
    }
}

// Passes PASS..0 of the inverse transform (PASS+1 already in registers).
template <int LOGN, int PASS, bool FOLD, typename W>
__device__ __forceinline__ void inv_rest(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, const Tw<W> *__restrict__ tw,
                                         const Arith<W> &ar, Tw<W> scale) {
    if constexpr (PASS >= 0) {
        lds_store<LOGN, PASS + 1>(lds, v, tau);
        __syncthreads();
        lds_load<LOGN, PASS>(lds, v, tau);
        inv_pass<LOGN, PASS, FOLD>(v, tau, tw, ar, scale);
        inv_rest<LOGN, PASS - 1, FOLD>(lds, v, tau, tw, ar, scale);
    }
}

// Per-launch constants.
template <typename W>
struct NttArgs {
    const Tw<W> *twf;      // forward stage table
    const Tw<W> *twi;      // inverse stage table
    const Tw<W> *twist;    // psi^i          (negacyclic pre-twist)
    const Tw<W> *untwist;  // psi^-i * N^-1  (negacyclic post-twist)
    const Tw<W> *untwist_r;// psi^-i * N^-1 * R (post-twist after a Montgomery product)
    Arith<W> ar;
    uint64_t q64, mu64;    // exact slow-path reduction of out-of-range inputs
    Tw<W> ninv;            // N^-1
    Tw<W> ninv_r;          // N^-1 * R  (after a Montgomery pointwise product)
    Tw<W> rmod;            // R mod q  (to Montgomery form)
};

// Forward transform of one polynomial held by this thread group: HBM load
// (bit-reversed, coalesced), all passes; result left in v (last layout,
// values in [0, 4q)).
template <int LOGN, bool NEGA, typename W>
__device__ __forceinline__ void fwd_poly(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, const uint64_t *__restrict__ src,
                                         bool valid, const NttArgs<W> &A) {
    using G = Geo<LOGN>;
    const uint64_t lim = NEGA ? (uint64_t)(W)~W(0) : (uint64_t)(A.ar.q2 * 2);
#pragma unroll
    for (int t = 0; t < G::E; ++t) {
        const uint32_t gi = tau + cbrv(t, G::LOGE) * G::T;
        uint64_t x = valid ? __builtin_nontemporal_load(src + gi) : 0;
        v[t] = load_lazy<W>(x, lim, A.q64, A.mu64);
        if constexpr (NEGA) v[t] = A.ar.shoup(v[t], A.twist[gi]);
    }
    fwd_pass<LOGN, 0>(v, tau, A.twf, A.ar);
    fwd_rest<LOGN, 1>(lds, v, tau, A.twf, A.ar);
}

// Inverse transform from v (last-pass layout, values in [0, 2q)) to HBM
// (bit-reversed store, coalesced), canonical output.  scale = N^-1 or
// N^-1 * R; post = the matching negacyclic post-twist table.
template <int LOGN, bool NEGA, typename W>
__device__ __forceinline__ void inv_poly_from_regs(W *lds, W (&v)[Geo<LOGN>::E], uint32_t tau, uint64_t *__restrict__ dst,
                                                   bool valid, const NttArgs<W> &A, Tw<W> scale,
                                                   const Tw<W> *__restrict__ post) {
    using G = Geo<LOGN>;
    constexpr int LAST = G::NP - 1;
    inv_pass<LOGN, LAST, !NEGA>(v, tau, A.twi, A.ar, scale);
    inv_rest<LOGN, LAST - 1, !NEGA>(lds, v, tau, A.twi, A.ar, scale);
#pragma unroll
    for (int t = 0; t < G::E; ++t) {
        const uint32_t gi = tau + cbrv(t, G::LOGE) * G::T;
        W x = v[t];
        if constexpr (NEGA) x = A.ar.shoup(x, post[gi]);
        if (valid) __builtin_nontemporal_store((uint64_t)A.ar.red1q(x), dst + gi);
    }
}

}  // namespace fhe
