// ntt_fwd.hip -- forward NTT kernels: plain (NTTProcessor::forward_ntt,
// ntt_processor.cpp:262-311), Montgomery-prepared, and forward + pointwise
// modmul (config C3: to_ntt then PolynomialRing::pointwise_multiply,
// polynomial_ring.cpp:104-116, 493-530).
// Flag-free 64-bit arithmetic (fhe_arith.hpp FHE_U64_NOVCC) in this
// translation unit: q62 C3 8.75 -> 8.15 ms per 65,536 polys on MI355X
// (profiles/r3b/ab_novcc.txt; parity tests green).  Each .hip file is its own
// device code object, so other files keep their own choice.
#ifndef FHE_U64_NOVCC
#define FHE_U64_NOVCC 1
#endif
#ifndef FHE_SPLIT_X64
#define FHE_SPLIT_X64 1
#endif
// streamed twiddles one group ahead: depth 2+ spills 8-12 B at 128 VGPRs
#ifndef FHE_STREAM_DEPTH
#define FHE_STREAM_DEPTH 1
#endif
#include "fhe_internal.hpp"

namespace FHE_NS {

template <int LOGN, typename W, bool LAZY, int EPI>
__device__ __forceinline__ void ntt_fwd_body(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch,
                                             const NttArgs<W> &A) {
    using G = Geo<LOGN>;
    __shared__ W lds_all[G::P * lds_elems<LOGN, W>()];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < batch;
    W *lds = lds_all + pl * lds_elems<LOGN, W>();
    if (G::P == 1 && !valid) return;  // whole workgroup: no barrier is skipped
    W v[G::E];
    // EPI 1: transform times R (Montgomery form), folded into stage 0
    fwd_poly<LOGN, LAZY, kPfSingle, EPI == 1>(lds, v, tau, in + poly * G::N, valid, A);
    if (!valid) return;
    uint64_t *dst = out + poly * G::N;
    if constexpr (G::P == 1) {
        const auto r = brsrc(dst);
        const uint32_t vo = LastIO<LOGN>::vo(tau);
#pragma unroll
        for (int e = 0; e < G::E; ++e) bstore(r, vo, LastIO<LOGN>::so(e), (uint64_t)fwd_to_canon<LAZY>(v[e], A));
    } else {
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const W x = fwd_to_canon<LAZY>(v[e], A);
            __builtin_nontemporal_store((uint64_t)x, dst + gidx<LOGN, G::NP - 1>(tau, e));
        }
    }
}
template <int LOGN, typename W, bool LAZY, int EPI>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, Geo<LOGN>::template occ_waves<W>())
k_ntt_fwd(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch, NttArgs<W> A) {
    ntt_fwd_body<LOGN, W, LAZY, EPI>(in, out, batch, A);
}
// RNS ring (polynomial_ring.cpp:224-237) in one launch: limb blockIdx.y of
// [limbs][batch][N], with that limb's transform constants from a table.
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS)  // no occupancy floor: RNS calls are small
k_ntt_fwd_limbs(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch,
                const NttArgs<W> *__restrict__ tab) {
    const size_t o = (size_t)blockIdx.y * batch * Geo<LOGN>::N;
    const NttArgs<W> A = tab[blockIdx.y];
    ntt_fwd_body<LOGN, W, LAZY, 0>(in + o, out + o, batch, A);
}

#ifndef FHE_FWDMUL_PREFETCH
#define FHE_FWDMUL_PREFETCH 1
#endif
// 32 words per thread: w in chunks of FHE_FWDMUL_CH words, FHE_FWDMUL_PD
// chunks in flight ahead of their use, the first FHE_FWDMUL_HOOK of them
// issued inside the transform's last pass
#ifndef FHE_FWDMUL_CH
#define FHE_FWDMUL_CH 4
#endif
#ifndef FHE_FWDMUL_PD
#define FHE_FWDMUL_PD 1
#endif
#ifndef FHE_FWDMUL_HOOK
#define FHE_FWDMUL_HOOK 1
#endif
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, Geo<LOGN>::template occ_waves<W>())
k_ntt_fwd_mul(const uint64_t *__restrict__ in, const uint64_t *__restrict__ wv, uint64_t *__restrict__ out,
              size_t batch, NttArgs<W> A) {
    using G = Geo<LOGN>;
    __shared__ W lds_all[G::P * lds_elems<LOGN, W>()];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < batch;
    W *lds = lds_all + pl * lds_elems<LOGN, W>();
    if (G::P == 1 && !valid) return;
    W v[G::E];
    // fwd(a) * R (stage 0 scaled), so mont(fwd(a)R, w) = fwd(a) w; the raw
    // lazy output (< (4+2L)q <= R) times a canonical w is a valid
    // Montgomery pair.
    const uint64_t *wp = wv + poly * G::N;
    uint64_t *dst = out + poly * G::N;
#if FHE_FWDMUL_PREFETCH
    if constexpr (G::P == 1 && G::E <= 16) {  // 32 raw u64 words would not fit beside the spectrum
        // w is loaded during the last pass (its HBM latency overlaps it)
        uint64_t rw[G::E];
        const uint32_t vo = LastIO<LOGN>::vo(tau);
        auto hook = [&] {
            const auto r = brsrc(wp);
#pragma unroll
            for (int e = 0; e < G::E; ++e) rw[e] = bload(r, vo, LastIO<LOGN>::so(e));
        };
        fwd_poly<LOGN, LAZY, kPfSingle, true>(lds, v, tau, in + poly * G::N, valid, A, 0, hook);
        W w[G::E];
        coeffs_from_raw<G::E>(w, rw, A.q64, SlowRed<W>{A});
        const auto ro = brsrc(dst);
#pragma unroll
        for (int e = 0; e < G::E; ++e) bstore(ro, vo, LastIO<LOGN>::so(e), (uint64_t)A.ar.red1q(A.ar.mont(v[e], w[e])));
        return;
    }
#endif
#if FHE_FWDMUL_PREFETCH
    if constexpr (G::P == 1 && G::E == 32) {
        // 32 words per thread (64-bit lanes): w streams in chunks of 8 --
        // the first FHE_FWDMUL_PD chunks are issued in the last pass (hook),
        // then chunk c + IN is issued before chunk c is consumed, so the
        // loads of w overlap the transform's tail and each other instead of
        // one round trip per chunk after the transform.
        constexpr int CH = FHE_FWDMUL_CH, NC = G::E / CH;
        uint64_t rw[G::E];
        const uint32_t vo = LastIO<LOGN>::vo(tau);
        const auto rwr = brsrc(wp);
        auto issue = [&](int c) {
#pragma unroll
            for (int e = c * CH; e < c * CH + CH; ++e) rw[e] = bload(rwr, vo, LastIO<LOGN>::so(e));
        };
        auto hook = [&] {
#pragma unroll
            for (int c = 0; c < FHE_FWDMUL_HOOK && c < NC; ++c) issue(c);
        };
        fwd_poly<LOGN, LAZY, kPfSingle, true>(lds, v, tau, in + poly * G::N, valid, A, 0, hook);
        const auto ro = brsrc(dst);
#pragma unroll
        for (int c = FHE_FWDMUL_HOOK; c < FHE_FWDMUL_PD && c < NC; ++c) issue(c);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c + FHE_FWDMUL_PD < NC) issue(c + FHE_FWDMUL_PD);
            __builtin_amdgcn_sched_barrier(0);
            W w[CH];
            uint64_t r8[CH];
#pragma unroll
            for (int e = 0; e < CH; ++e) r8[e] = rw[c * CH + e];
            coeffs_from_raw<CH>(w, r8, A.q64, SlowRed<W>{A});
#pragma unroll
            for (int e = 0; e < CH; ++e)
                bstore(ro, vo, LastIO<LOGN>::so(c * CH + e), (uint64_t)A.ar.red1q(A.ar.mont(v[c * CH + e], w[e])));
            __builtin_amdgcn_sched_barrier(0);
        }
        return;
    }
#endif
    fwd_poly<LOGN, LAZY, kPfSingle, true>(lds, v, tau, in + poly * G::N, valid, A);
    if (!valid) return;
    // two chunks: 16 raw u64 w in flight at once would exceed 64 VGPRs
    constexpr int CH = G::E >= 8 ? G::E / 8 : G::E;
#pragma unroll
    for (int c0 = 0; c0 < G::E; c0 += CH) {
        W w[CH];
        if constexpr (G::P == 1) {
            const auto rw = brsrc(wp), ro = brsrc(dst);
            const uint32_t vo = LastIO<LOGN>::vo(tau);
            load_coeffs_r<CH>(w, A.q64, SlowRed<W>{A},
                            [&](int e) -> uint64_t { return bload(rw, vo, LastIO<LOGN>::so(c0 + e)); });
#pragma unroll
            for (int e = 0; e < CH; ++e)
                bstore(ro, vo, LastIO<LOGN>::so(c0 + e), (uint64_t)A.ar.red1q(A.ar.mont(v[c0 + e], w[e])));
        } else {
            load_coeffs_r<CH>(w, A.q64, SlowRed<W>{A}, [&](int e) -> uint64_t {
                return __builtin_nontemporal_load(wp + gidx<LOGN, G::NP - 1>(tau, c0 + e));
            });
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                const W x = A.ar.red1q(A.ar.mont(v[c0 + e], w[e]));
                __builtin_nontemporal_store((uint64_t)x, dst + gidx<LOGN, G::NP - 1>(tau, c0 + e));
            }
        }
    }
}

// 64-bit words at N = 16384: 32 coefficients per thread (512 threads,
// radix-32 passes: 2 exchanges instead of 3) and the split exchange, so two
// workgroups share a CU at <= 128 VGPRs each.
#ifndef FHE_FWD64_E32
#define FHE_FWD64_E32 1
#endif
template <int LOGN, typename W>
constexpr int fwd_key() { return (FHE_FWD64_E32 && sizeof(W) == 8 && LOGN == 14) ? gk(LOGN, 5) : LOGN; }

template <int LOGN0, typename W, bool LAZY>
static hipError_t fwd_one(const NttArgs<W> &A, hipStream_t s, const uint64_t *in, uint64_t *out, size_t batch,
                          int epi, const uint64_t *wv) {
    constexpr int LOGN = fwd_key<LOGN0, W>();
    using G = Geo<LOGN>;
    const size_t blocks = (batch + G::P - 1) / G::P;
    // (unit twiddles, ntt_core.hpp gk_compat: 7.29 vs 7.30 ms for the q62 C3
    // kernel, round 5 -- not instantiated)
    if (wv)
        hipLaunchKernelGGL((k_ntt_fwd_mul<LOGN, W, LAZY>), dim3(blocks), dim3(G::THREADS), 0, s, in, wv, out,
                           batch, A);
    else if (epi == 1)
        hipLaunchKernelGGL((k_ntt_fwd<LOGN, W, LAZY, 1>), dim3(blocks), dim3(G::THREADS), 0, s, in, out, batch, A);
    else
        hipLaunchKernelGGL((k_ntt_fwd<LOGN, W, LAZY, 0>), dim3(blocks), dim3(G::THREADS), 0, s, in, out, batch, A);
    return hipGetLastError();
}
template <int LOGN, typename W>
static hipError_t fwd_lazy(const Plan &p, const NttArgs<W> &A, const uint64_t *in, uint64_t *out, size_t batch,
                           int epi, const uint64_t *wv) {
    if constexpr (sizeof(W) == 4)
        if (p.lazy) return fwd_one<LOGN, W, true>(A, p.stream, in, out, batch, epi, wv);
    return fwd_one<LOGN, W, false>(A, p.stream, in, out, batch, epi, wv);
}

template <typename W>
static hipError_t fwd_dispatch(const Plan &p, const NttArgs<W> &A, const uint64_t *in, uint64_t *out, size_t batch,
                               int epi, const uint64_t *wv) {
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return fwd_lazy<L, W>(p, A, in, out, batch, epi, wv);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}

static hipError_t fwd_any(const Plan &p, const uint64_t *in, uint64_t *out, size_t batch, int epi,
                          const uint64_t *wv) {
    if (batch == 0) return hipSuccess;
    if (p.word == 32)
        return fwd_dispatch<uint32_t>(p, p.a32, in, out, batch, epi, wv);
    return fwd_dispatch<uint64_t>(p, p.a64, in, out, batch, epi, wv);
}

template <int LOGN0, typename W, bool LAZY>
static hipError_t fwd_limbs_one(const Plan &p, const void *tab, int limbs, const uint64_t *in, uint64_t *out,
                                size_t batch) {
    constexpr int LOGN = fwd_key<LOGN0, W>();
    using G = Geo<LOGN>;
    const size_t blocks = (batch + G::P - 1) / G::P;
    hipLaunchKernelGGL((k_ntt_fwd_limbs<LOGN, W, LAZY>), dim3(blocks, limbs), dim3(G::THREADS), 0, p.stream, in, out,
                       batch, static_cast<const NttArgs<W> *>(tab));
    return hipGetLastError();
}
template <int LOGN, typename W>
static hipError_t fwd_limbs_lazy(const Plan &p, const void *tab, int limbs, const uint64_t *in, uint64_t *out,
                                 size_t batch) {
    if constexpr (sizeof(W) == 4)
        if (p.lazy) return fwd_limbs_one<LOGN, W, true>(p, tab, limbs, in, out, batch);
    return fwd_limbs_one<LOGN, W, false>(p, tab, limbs, in, out, batch);
}
template <typename W>
static hipError_t fwd_limbs_dispatch(const Plan &p, const void *tab, int limbs, const uint64_t *in, uint64_t *out,
                                     size_t batch) {
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return fwd_limbs_lazy<L, W>(p, tab, limbs, in, out, batch);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}
hipError_t launch_fwd_limbs(const Plan &p, const void *tab, int limbs, const uint64_t *in, uint64_t *out,
                            size_t batch) {
    if (p.wide || p.logn > kMaxFusedLogN || limbs < 1 || limbs > 65535) return hipErrorInvalidValue;
    if (batch == 0) return hipSuccess;
    return p.word == 32 ? fwd_limbs_dispatch<uint32_t>(p, tab, limbs, in, out, batch)
                        : fwd_limbs_dispatch<uint64_t>(p, tab, limbs, in, out, batch);
}

hipError_t launch_fwd(const Plan &p, const uint64_t *in, uint64_t *out, size_t batch, int epi) {
    if (p.wide) return launch_wide(p, epi == 1 ? 1 : 0, in, nullptr, out, batch);
    if (p.logn > kMaxFusedLogN) return launch_big(p, epi == 1 ? 1 : 0, in, nullptr, out, batch);
    return fwd_any(p, in, out, batch, epi, nullptr);
}
hipError_t launch_fwd_mul(const Plan &p, const uint64_t *a, const uint64_t *w, uint64_t *out, size_t batch) {
    if (p.wide) return launch_wide(p, 2, a, w, out, batch);
    if (p.logn > kMaxFusedLogN) return launch_big(p, 2, a, w, out, batch);
    return fwd_any(p, a, out, batch, 0, w);
}

}  // namespace FHE_NS
