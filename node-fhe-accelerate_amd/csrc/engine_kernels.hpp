// engine_kernels.hpp -- the EncryptionEngine entry points around the transform:
// encrypt (encryption.cpp:171-205), decrypt + decode + noise measure
// (:234-300, :150-163, :364-400) and add_plain (:638-665), one workgroup
// per ciphertext (several for N < 1024), batched.
//
// Keys are prepared once in the NTT domain times R (Montgomery form):
//   pk_prep = (fwd(pk.a) R, fwd(pk.b) R), sk_prep = (fwd(s) R, fwd(s)^2 R),
// so mont(raw transform, key) is the plain pointwise product and the inverse
// uses the plain N^-1 (as k_dmac does).  Because the inverse transform is
// linear over Z_q and every intermediate is a canonical residue, the
// reference's sequence of separate inverse transforms and mod_add/mod_sub
// passes is reproduced bit for bit with fewer transforms:
//   encrypt  c0 = inv(U Pb) + e1 + m,  c1 = inv(U Pa) + e2      (1 fwd + 2 inv)
//   decrypt  is_ntt: phase = inv(C0 - C1 S [- C2 S^2])          (1 inv)
//            else    phase = c0 - inv(fwd(c1) S) [- inv(fwd(c2) S^2)]
//   add_plain        c0 + m, or c0 + fwd(m) for NTT-domain ciphertexts
// with m = encode(values) = (v * delta mod 2^64) mod q, delta = q / t.
// decrypt's epilogue decodes every coefficient (round(p t / q) mod t) and
// reduces the reference's max noise |p - round(p t / q) delta| per
// ciphertext, all in the inverse transform's store loop.
#pragma once
#include "fhe_internal.hpp"
#include "lwe_ops.hpp"

namespace FHE_NS {

// floor((hi:lo) / q) for a quotient known to be < 2^64 (exact): a double
// estimate, then steps of (remainder / q) until the remainder is in [0, q).
__device__ __forceinline__ uint64_t div128(uint64_t hi, uint64_t lo, uint64_t q, double qinv) {
    constexpr double k2_64 = 18446744073709551616.0;
    const double qd = ((double)hi * k2_64 + (double)lo) * qinv;
    uint64_t qe = qd >= k2_64 ? ~0ull : (uint64_t)qd;
    for (int it = 0; it < 8; ++it) {
        const uint64_t pl = qe * q, ph = __umul64hi(qe, q);
        const bool over = ph > hi || (ph == hi && pl > lo);  // q * qe > num
        const uint64_t rl = over ? pl - lo : lo - pl;
        const uint64_t rh = over ? ph - hi - (pl < lo ? 1 : 0) : hi - ph - (lo < pl ? 1 : 0);
        if (!over && rh == 0 && rl < q) break;
        uint64_t step = (uint64_t)(((double)rh * k2_64 + (double)rl) * qinv);
        step = step ? step : 1;
        qe = over ? qe - step : qe + step;
    }
    return qe;
}

// decode_packed's round(p t / q) mod t and compute_noise_budget's distance,
// for a canonical phase p < q.
struct Decoder {
    uint64_t q, mu, t, delta, half;
    double qinv;
    __device__ __forceinline__ uint64_t rounded(uint64_t p) const {
        const uint64_t lo = p * t, hi = __umul64hi(p, t);
        const uint64_t l2 = lo + half;
        return div128(hi + (l2 < lo ? 1 : 0), l2, q, qinv);
    }
    __device__ __forceinline__ uint64_t noise(uint64_t p, uint64_t r) const {
        const uint64_t expected = mod64_slow(r * delta, q, mu);  // (rounded * delta_) % modulus, u64 product
        uint64_t d = p >= expected ? p - expected : expected - p;
        if ((int64_t)d > (int64_t)half) d = q - d;
        return d;
    }
};

struct EngArgs {
    const uint64_t *ct;     // decrypt: [batch][comps][N]; add_plain: [batch][2][N]
    const uint64_t *key;    // prepared key rows [2][N]
    const uint64_t *vals;   // plaintext slots [batch][N]
    const uint64_t *u, *e1, *e2;  // encrypt randomness [batch][N]
    uint64_t *out;          // encrypt / add_plain: [batch][2][N]; decrypt: phase [batch][N] (or workspace)
    uint64_t *dec;          // decrypt: decoded slots [batch][N] (nullable)
    uint64_t *noise;        // decrypt: max noise [batch] (nullable)
    size_t batch;
    int comps, is_ntt, store_phase;
    Decoder D;
};

__device__ __forceinline__ uint64_t encode1(uint64_t v, const Decoder &D) {
    return mod64_slow(v * D.delta, D.q, D.mu);  // encode_packed (:117-131)
}

// Where the second product waits during the first inverse transform:
// 0 VGPRs (small N), 1 a second LDS region, 2 the c1 output row (own
// positions, W-typed) -- k_polymul's policy.
template <int LOGN, typename W>
constexpr int eng_stash() {
    using G = Geo<LOGN>;
    if (LOGN < 5) return 0;
    return G::P * (G::LW + G::N) * (int)sizeof(W) <= 160 * 1024 ? 1 : 2;
}
template <int LOGN, typename W>
constexpr int eng_occ() {
    return Geo<LOGN>::template occ_waves<W, eng_stash<LOGN, W>() == 1 ? Geo<LOGN>::P * Geo<LOGN>::N : 0>();
}

template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (eng_occ<LOGN, W>()))
k_encrypt(EngArgs E, NttArgs<W> A) {
    using G = Geo<LOGN>;
    constexpr int STASH = eng_stash<LOGN, W>();
    __shared__ W lds_all[G::P * G::LW + (STASH == 1 ? G::P * G::N : 0)];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < E.batch;
    if (G::P == 1 && !valid) return;
    W *lds = lds_all + pl * G::LW;
    W *st = lds_all + G::P * G::LW + pl * G::N;
    const size_t row = (valid ? poly : 0) * G::N;
    uint64_t *c0 = E.out + 2 * row, *c1 = c0 + G::N;
    const uint64_t q = A.q64, mu = A.mu64;
    W v[G::E];
    W va[STASH == 0 ? G::E : 1];
    fwd_poly<LOGN, LAZY>(lds, v, tau, E.u + row, valid, A);
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tau, e);
        // key rows: (pk.a, pk.b) (PublicKey field order, key_manager.h:70-76)
        const W a = valid ? A.ar.mont(v[e], (W)E.key[gi]) : W(0);          // U . pk.a
        if constexpr (STASH == 0) va[e] = a;
        else if constexpr (STASH == 1) st[gi] = a;
        else if (valid) reinterpret_cast<W *>(c1)[gi] = a;
        v[e] = valid ? A.ar.mont(v[e], (W)E.key[G::N + gi]) : W(0);        // U . pk.b
    }
    if constexpr (G::NP > 1) __syncthreads();
    {
        uint32_t tr = tau;
        asm volatile("" : "+v"(tr));
        auto fin0 = [&](uint32_t gi, uint64_t x) -> uint64_t {  // + e1 (mod_add), + m (mod_add)
            if (!valid) return 0;
            return addq(addq(x, red_q(E.e1[row + gi], q, mu), q), encode1(E.vals[row + gi], E.D), q);
        };
        inv_poly_from_regs<LOGN>(lds, v, tr, c0, valid, A, A.ninv, 0, fin0);
    }
    if constexpr (G::NP > 1) __syncthreads();
    uint32_t tb = tau;
    asm volatile("" : "+v"(tb));
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tb, e);
        if constexpr (STASH == 0) v[e] = va[e];
        else if constexpr (STASH == 1) v[e] = st[gi];
        else v[e] = valid ? reinterpret_cast<const W *>(c1)[gi] : W(0);
    }
    if constexpr (STASH == 2) __syncthreads();  // every stash read precedes the c1 stores
    auto fin1 = [&](uint32_t gi, uint64_t x) -> uint64_t {
        return valid ? addq(x, red_q(E.e2[row + gi], q, mu), q) : 0;
    };
    inv_poly_from_regs<LOGN>(lds, v, tb, c1, valid, A, A.ninv, 0, fin1);
}

// decrypt and add_plain: at most 4 waves per SIMD (128 VGPRs): the
// decode's 128-bit division and the three code paths of k_decrypt spill
// heavily at the 64-VGPR budget of 8 waves
template <int LOGN, typename W>
constexpr int eng_occ4() {
    constexpr int w = Geo<LOGN>::template occ_waves<W>();
    return w < 4 ? w : 4;
}

// decrypt at 64-bit words and N = 256..2048 (several polynomials per
// 256-thread workgroup): 2 waves per SIMD -- the decode epilogue beside a
// 16-word u64 spectrum does not fit 128 VGPRs there
template <int LOGN, typename W>
constexpr int dec_occ() {
    return (sizeof(W) == 8 && Geo<LOGN>::L >= 8 && Geo<LOGN>::L <= 11) ? 2 : eng_occ4<LOGN, W>();
}

template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (dec_occ<LOGN, W>()))
k_decrypt(EngArgs E, NttArgs<W> A) {
    using G = Geo<LOGN>;
    __shared__ W lds_all[G::P * G::LW];
    __shared__ unsigned long long nmax[G::P];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < E.batch;
    if (G::P == 1 && !valid) return;
    W *lds = lds_all + pl * G::LW;
    const size_t row = (valid ? poly : 0) * G::N;
    const uint64_t *ct = E.ct + (size_t)E.comps * row;
    uint64_t *phase = E.out ? E.out + row : nullptr;
    const uint64_t q = A.q64, mu = A.mu64;
    if (tau == 0) nmax[pl] = 0;
    uint64_t local_max = 0;
    // decode + noise of the final phase p at global index gi
    auto final_fin = [&](uint32_t gi, uint64_t p) -> uint64_t {
        if (!valid) return 0;
        const uint64_t r = E.D.rounded(p);
        if (E.dec) E.dec[row + gi] = r >= E.D.t ? r - E.D.t : r;
        const uint64_t d = E.D.noise(p, r);
        local_max = d > local_max ? d : local_max;
        if (E.store_phase) phase[gi] = p;
        return p;
    };
    W v[G::E];
    if (E.is_ntt) {
        // everything pointwise: X = C0 - C1 S (- C2 S^2), one inverse
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const uint32_t gi = gidx<LOGN, G::NP - 1>(tau, e);
            if (!valid) { v[e] = 0; continue; }
            W x = A.ar.red1q(A.ar.mont((W)red_q(ct[G::N + gi], q, mu), (W)E.key[gi]));
            if (E.comps == 3)
                x = A.ar.red1q(A.ar.red2q(x + A.ar.mont((W)red_q(ct[2 * G::N + gi], q, mu), (W)E.key[G::N + gi])));
            v[e] = (W)subq(red_q(ct[gi], q, mu), (uint64_t)x, q);
        }
    } else {
        // c0 - inv(fwd(c1) S) [- inv(fwd(c2) S^2)] == c0 - inv(fwd(c1) S [+ fwd(c2) S^2]):
        // the inverse is linear over Z_q and the phase is taken canonical, so
        // one inverse serves both components (bit-exact).  One forward
        // instance in a runtime loop; the c1 product waits in this thread's
        // own positions of the phase row (W words) while fwd(c2) runs.
        W *stash = reinterpret_cast<W *>(phase);
        for (int c = 1; c < E.comps; ++c) {
            uint32_t tc = tau;
            asm volatile("" : "+v"(tc));
            fwd_poly<LOGN, LAZY>(lds, v, tc, ct + (size_t)c * G::N, valid, A);
            const bool last = c + 1 == E.comps;
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const uint32_t gi = gidx<LOGN, G::NP - 1>(tc, e);
                W x = valid ? A.ar.mont(v[e], (W)E.key[(size_t)(c - 1) * G::N + gi]) : W(0);  // [0, 2q)
                if (c == 2 && valid) x = A.ar.red2q(x + stash[gi]);
                if (!last && valid) stash[gi] = x;
                v[e] = x;
            }
            if constexpr (G::NP > 1) __syncthreads();  // exchange buffer reuse; stash reads before the final stores
        }
    }
    {
        uint32_t tr = tau;
        asm volatile("" : "+v"(tr));
        const bool ntt = E.is_ntt;
        auto fin = [&](uint32_t gi, uint64_t x) -> uint64_t {
            return final_fin(gi, ntt ? x : (valid ? subq(red_q(ct[gi], q, mu), x, q) : 0));
        };
        inv_poly_from_regs<LOGN, kPfSingle, false>(lds, v, tr, phase, valid, A, A.ninv, 0, fin);
    }
    if (E.noise) {
        // max over the polynomial's lanes within the wave (a polynomial owns
        // T aligned lanes), then one LDS atomic per wave and polynomial
        constexpr int LANES = G::T < 64 ? G::T : 64;
#pragma unroll
        for (int o = LANES / 2; o >= 1; o >>= 1) {
            const uint64_t w = __shfl_xor(local_max, o, 64);
            local_max = w > local_max ? w : local_max;
        }
        __syncthreads();
        if ((threadIdx.x & (LANES - 1)) == 0) atomicMax(&nmax[pl], (unsigned long long)local_max);
        __syncthreads();
        if (valid && tau == 0) E.noise[poly] = nmax[pl];
    }
}

// add_plain on NTT-domain ciphertexts: c0 + fwd(encode(values)), c1 copied.
template <int LOGN, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (eng_occ4<LOGN, W>()))
k_add_plain_ntt(EngArgs E, NttArgs<W> A) {
    using G = Geo<LOGN>;
    __shared__ W lds_all[G::P * G::LW];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < E.batch;
    if (G::P == 1 && !valid) return;
    W *lds = lds_all + pl * G::LW;
    const size_t row = (valid ? poly : 0) * G::N;
    const uint64_t q = A.q64, mu = A.mu64;
    uint64_t raw[G::E];
#pragma unroll
    for (int t = 0; t < G::E; ++t)
        raw[t] = valid ? encode1(E.vals[row + tau + cbrv(t, G::LOGE) * G::T], E.D) : 0;
    W v[G::E];
    fwd_poly<LOGN, LAZY>(lds, v, tau, nullptr, valid, A, 0, NoHook{}, &raw);
    if (!valid) return;
    const uint64_t *c = E.ct + 2 * row;
    uint64_t *o = E.out + 2 * row;
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const uint32_t gi = gidx<LOGN, G::NP - 1>(tau, e);
        o[gi] = addq(red_q(c[gi], q, mu), (uint64_t)fwd_to_canon<LAZY>(v[e], A), q);
        o[G::N + gi] = c[G::N + gi];
    }
}

// Template dispatch over (logN, word, mode, lazy) for one kernel family;
// each ntt_engine_*.hip instantiates one family (parallel compile units).
template <int OP, int LOGN, typename W, bool LAZY>
static hipError_t eng_one(const NttArgs<W> &A, hipStream_t s, const EngArgs &E) {
    using G = Geo<LOGN>;
    const size_t blocks = (E.batch + G::P - 1) / G::P;
    if constexpr (OP == 0)
        hipLaunchKernelGGL((k_encrypt<LOGN, W, LAZY>), dim3(blocks), dim3(G::THREADS), 0, s, E, A);
    else if constexpr (OP == 1)
        hipLaunchKernelGGL((k_decrypt<LOGN, W, LAZY>), dim3(blocks), dim3(G::THREADS), 0, s, E, A);
    else
        hipLaunchKernelGGL((k_add_plain_ntt<LOGN, W, LAZY>), dim3(blocks), dim3(G::THREADS), 0, s, E, A);
    return hipGetLastError();
}
template <int OP, int LOGN, typename W>
static hipError_t eng_lazy(const Plan &p, const NttArgs<W> &A, const EngArgs &E) {
    if constexpr (sizeof(W) == 4)
        if (p.lazy) return eng_one<OP, LOGN, W, true>(A, p.stream, E);
    return eng_one<OP, LOGN, W, false>(A, p.stream, E);
}
template <int OP, typename W>
static hipError_t eng_dispatch(const Plan &p, const NttArgs<W> &A, const EngArgs &E) {
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return eng_lazy<OP, L, W>(p, A, E);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}
template <int OP>
static hipError_t eng_any(const Plan &p, const EngArgs &E) {
    if (E.batch == 0) return hipSuccess;
    if (p.word == 32)
        return eng_dispatch<OP, uint32_t>(p, p.a32, E);
    return eng_dispatch<OP, uint64_t>(p, p.a64, E);
}

static inline Decoder make_decoder(uint64_t q, uint64_t t) {
    Decoder D;
    D.q = q;
    D.mu = (uint64_t)((((unsigned __int128)1) << 64) / q);
    D.t = t ? t : 4;
    D.delta = q / D.t;
    D.half = q / 2;
    D.qinv = 1.0 / (double)q;
    return D;
}
static inline uint64_t plan_q(const Plan &p) { return p.word == 32 ? p.a32.q64 : p.a64.q64; }

}  // namespace FHE_NS
