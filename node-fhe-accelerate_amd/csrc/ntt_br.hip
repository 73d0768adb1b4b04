// ntt_br.hip -- low-latency blind rotation (BootstrapEngine::blind_rotate,
// bootstrap_engine.cpp:547-577: the initial rotation by -round(b 2N / q),
// then for every LWE mask coefficient a_i the CMux step
//   rot = (int32)((a_i * 2N + q/2) / q);  rot == 0: skip
//   acc = acc + ExtProd(X^rot * acc - acc, bsk[i])          (cmux :520-540)
// as ONE launch for the whole loop.
//
// The multi-launch path (k_dmac MODE 2, one launch per step over the batch,
// one wave per ciphertext) is throughput-shaped: at batch 64 it leaves the
// chip nearly idle and every step is the latency of 4 dependent transforms
// by a single wave, plus an HBM/L2 round trip of the accumulators.  Here one
// workgroup owns one ciphertext for all steps:
//   * the (k+1) = 2 accumulators live in LDS (raw u64, exactly the values the
//     multi-launch path would hold in HBM between steps);
//   * the two digit polynomials of a decomposition level are transformed in
//     parallel, each by 128 threads with N/128 coefficients per thread
//     (geometry gk(logN, logN - 7): P = 2 polynomials per workgroup);
//   * the MAC with the step's GGSW (NTT x R, Montgomery) accumulates in
//     registers; the two halves swap their cross terms through LDS, so half j
//     ends holding output component j and inverts it;
//   * the inverse's epilogue adds the old accumulator (mod_add) back into LDS.
// Same arithmetic as MODE 2 (digit load, red_q / subq / addq, Montgomery MAC,
// canonical inverse), so results are bit-identical to the multi-launch path
// and to the oracle.
// flag-free 64-bit arithmetic (fhe_arith.hpp): 19.0 vs 20.5 ms for the
// N = 2048 preset, 94.9 vs 100.9 ms for the N = 1024 batch (round 4)
#ifndef FHE_U64_NOVCC
#define FHE_U64_NOVCC 1
#endif
#ifndef FHE_BR_STAMPS
#define FHE_BR_STAMPS 0
#endif
#include "fhe_internal.hpp"
#include "lwe_ops.hpp"
#if FHE_BR_STAMPS
#include <cstdio>
#include <cstdlib>
#include <vector>
#endif

namespace FHE_NS {

struct BrArgs {
    uint64_t *acc;          // [batch][2][N], in/out
    const uint64_t *bsk;    // [lwe_dim][2L][2][N] prepared GGSWs
    const uint64_t *lwe_a;  // [batch][lwe_dim]
    const uint64_t *lwe_b;  // [batch]
    uint64_t lwe_q;
    uint32_t lwe_dim;
    int level, base_log;
    // input accumulators when they are not read from acc (k_br_pair's saved
    // copy, for its repair pass)
    const uint64_t *acc_in = nullptr;
    // repair pass of k_br_pair (k_br_persist only): ciphertexts with
    // only[ct] == 0 are skipped; each one run adds 1 to *repairs
    const uint32_t *only = nullptr;
    unsigned long long *repairs = nullptr;
};

// 8 coefficients per thread (N / 8 threads per half) from N = 1024, fewer
// below: the transforms are throughput-bound on the one CU, and 16 per thread
// (half the waves) measured 31.2 vs 20.7 ms (N = 2048, L = 2) and 70.7 vs
// 58.6 ms (N = 4096, L = 3) per batch-64 blind rotation (round 4).
#ifndef FHE_BR_LOGE
#define FHE_BR_LOGE 3
#endif
#ifndef FHE_BR_XACC
#define FHE_BR_XACC 1
#endif
#ifndef FHE_BR_LOGE_SMALL
#define FHE_BR_LOGE_SMALL FHE_BR_LOGE
#endif
template <int LOGN>
constexpr int br_key() {  // LOGN may carry key bits (gk_compat)
    constexpr int L = gk_logn(LOGN);
    return L >= 12 ? gk(LOGN, FHE_BR_LOGE) : gk(LOGN, L - 7 < FHE_BR_LOGE_SMALL ? L - 7 : FHE_BR_LOGE_SMALL);
}
template <int LOGN>
constexpr int br_threads() { return 2 * Geo<br_key<LOGN>()>::T; }
// The cross-half MAC terms share the exchange regions when the accumulators,
// two exchange regions and a separate cross buffer exceed the LDS (N = 4096
// with 64-bit words: 64 + 66 + 64 KiB): one more barrier per row.
template <int LOGN, typename W>
constexpr bool br_alias_x() {
    using G = Geo<br_key<LOGN>()>;
    return 2 * G::N * 8 + 2 * G::LW * (int)sizeof(W) + 2 * G::N * (int)sizeof(W) > 160 * 1024;
}

template <int LOGN, typename W>
__global__ void __launch_bounds__(br_threads<LOGN>()) k_br_persist(BrArgs D, NttArgs<W> A) {
    constexpr int K = br_key<LOGN>();
    using G = Geo<K>;
    constexpr int THREADS = br_threads<LOGN>();
    constexpr bool ALIAS = br_alias_x<LOGN, W>();
    // the per-step difference held in VGPRs (2 E of them): spills beside
    // 16-word spectra and at 1024 threads (128 VGPRs)
    constexpr bool CV = G::E <= 8 && THREADS <= 512;
    // the other half's MAC terms summed over the levels in VGPRs and
    // exchanged once per step (else once per level through LDS)
    constexpr bool XACC = FHE_BR_XACC && G::E <= 8 && (THREADS <= 512 || FHE_BR_XACC == 2);
    static_assert(G::LW >= G::N, "cross terms fit an exchange region");
    constexpr int N = G::N;
    __shared__ uint64_t accs[2][N];   // raw accumulators (component j)
    __shared__ W xlds[2 * G::LW];     // NTT exchange, one region per half
    __shared__ W xsep[ALIAS ? 1 : 2 * N];
    // cross-half MAC terms: own buffer, or half h's exchange region
    auto xb = [&](uint32_t h) -> W * { return ALIAS ? xlds + h * G::LW : xsep + h * N; };
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = threadIdx.x >> G::LOGT;
    const size_t ct = blockIdx.x;
    if (D.only) {  // repair pass: only the ciphertexts k_br_pair gave up on
        if (D.only[ct] == 0) return;  // workgroup-uniform, before any barrier
        if (threadIdx.x == 0) atomicAdd(D.repairs, 1ull);
    }
    const uint64_t q = A.q64, mu = A.mu64;
    W *lds = xlds + pl * G::LW;
    uint64_t *gacc = D.acc + ct * 2 * N;
    {
        // acc <- X^-round(b 2N/q) acc   (k_rotate's map)
        const uint64_t *gin = (D.acc_in ? D.acc_in : D.acc) + ct * 2 * N;
        const uint32_t r0 = rot_norm(-rot_amount(D.lwe_b[ct], N, D.lwe_q), N);
        for (uint32_t i = threadIdx.x; i < 2u * N; i += THREADS) {
            const uint32_t j = i / N, p = i % N;
            accs[j][p] = rotated_at(gin + (size_t)j * N, p, r0, N, q, mu);
        }
    }
    __syncthreads();
    const int level = D.level;
    const uint64_t base = 1ull << D.base_log, mask = base - 1, half = base / 2;
    // a negative digit's q - (base - d) is already below q
    const bool small_base = base <= q;
    const size_t ggsw_words = (size_t)2 * level * 2 * N;
    const uint64_t *lwe_a = D.lwe_a + ct * D.lwe_dim;
    bool canon = false;
    for (uint32_t step = 0; step < D.lwe_dim; ++step) {
        const int32_t r = rot_amount(lwe_a[step], N, D.lwe_q);  // workgroup-uniform
        if (r == 0) continue;
        const uint32_t rot = rot_norm(r, N);
        const uint64_t *key = D.bsk + ggsw_words * step;
        W oacc[G::E], xacc[XACC ? G::E : 1];
        // X^rot acc_pl - acc_pl at the lane's pass-0 positions: once per step
        // into VGPRs where they fit (every level's digits come from it),
        // else again for each level from the LDS accumulator.  After the
        // first executed step every accumulator word is canonical (the
        // mod_add below), and red_q / the wrap of (q - x) % q are the identity
        // on it: the reductions are skipped (workgroup-uniform).
        const uint64_t *ac = accs[pl];
        auto diff_at = [&](uint32_t tr, int t) -> uint64_t {
            const uint32_t p = tr + cbrv(t, G::LOGE) * G::T;
            const uint32_t j = (p + 2 * N - rot) & (2 * N - 1);
            if (canon) {
                const uint64_t a = ac[j < (uint32_t)N ? j : j - N];
                const uint64_t xr = j < (uint32_t)N || a == 0 ? a : q - a;
                return subq(xr, ac[p], q);
            }
            const uint64_t xr = j < (uint32_t)N ? ac[j] : red_q(q - ac[j - N], q, mu);
            return subq(red_q(xr, q, mu), red_q(ac[p], q, mu), q);
        };
        uint64_t cv[CV ? G::E : 1];
        if constexpr (CV) {
#pragma unroll
            for (int t = 0; t < G::E; ++t) cv[t] = diff_at(tau, t);
        }
        for (int g = 0; g < level; ++g) {
            // row (pl, g): digit g of X^rot acc_pl - acc_pl (MSB digit first)
            const int row = pl * level + g;
            const uint32_t shift = uint32_t(level - 1 - g) * uint32_t(D.base_log);
            // this row's key terms for both output components, in flight
            // across the transform
            uint64_t kv[2][G::E];
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const uint32_t gi = gidx<K, G::NP - 1>(tau, e);
                kv[0][e] = key[((size_t)row * 2 + pl) * N + gi];
                kv[1][e] = key[((size_t)row * 2 + (1 - pl)) * N + gi];
            }
            uint32_t tr = tau;
            asm volatile("" : "+v"(tr));
            W v[G::E];
            Tw<W> t0[PassTw<K, 0>::COUNT];
            load_tw<K, 0>(tr, A.twf, t0);
            load_coeffs<G::E>(v, (uint64_t)A.ar.q2 * 2, q, mu, [&](int t) -> uint64_t {
                uint64_t d = ((CV ? cv[CV ? t : 0] : diff_at(tr, t)) >> shift) & mask;
                if (d > half) d = small_base ? q - (base - d) : red_q(q - (base - d), q, mu);
                return d;
            });
            fwd_pass<K, 0, false>(v, t0, A.ar);
            fwd_rest<K, 1, false, kPfSingle>(lds, v, tr, A.twf, A.ar);
            // raw output (< 4q) times a canonical key: a valid Montgomery pair
            if constexpr (XACC) {
                // the other half's terms accumulate here and cross once per step
#pragma unroll
                for (int e = 0; e < G::E; ++e) {
                    const W own = A.ar.mont(v[e], (W)kv[0][e]), oth = A.ar.mont(v[e], (W)kv[1][e]);
                    oacc[e] = g == 0 ? own : A.ar.red2q(oacc[e] + own);
                    xacc[e] = g == 0 ? oth : A.ar.red2q(xacc[e] + oth);
                }
                if (g + 1 < level) __syncthreads();  // the exchange region is reused by the next level
            } else {
                // the other half may still read its exchange region (last pass)
                if constexpr (ALIAS) __syncthreads();
                W *const xo = xb(1 - pl);
#pragma unroll
                for (int e = 0; e < G::E; ++e) {
                    const uint32_t gi = gidx<K, G::NP - 1>(tr, e);
                    const W own = A.ar.mont(v[e], (W)kv[0][e]);
                    xo[gi] = A.ar.mont(v[e], (W)kv[1][e]);
                    oacc[e] = g == 0 ? own : A.ar.red2q(oacc[e] + own);
                }
                __syncthreads();
                const W *const xi = xb(pl);
#pragma unroll
                for (int e = 0; e < G::E; ++e) oacc[e] = A.ar.red2q(oacc[e] + xi[gidx<K, G::NP - 1>(tr, e)]);
                __syncthreads();  // the cross terms and the exchange regions are reused
            }
        }
        if constexpr (XACC) {
            uint32_t tx = tau;
            asm volatile("" : "+v"(tx));
            // the other half may still read its exchange region (last pass)
            if constexpr (ALIAS) __syncthreads();
            W *const xo = xb(1 - pl);
#pragma unroll
            for (int e = 0; e < G::E; ++e) xo[gidx<K, G::NP - 1>(tx, e)] = xacc[e];
            __syncthreads();
            const W *const xi = xb(pl);
#pragma unroll
            for (int e = 0; e < G::E; ++e) oacc[e] = A.ar.red2q(oacc[e] + xi[gidx<K, G::NP - 1>(tx, e)]);
            __syncthreads();  // the cross terms and the exchange regions are reused
        }
        // component pl: inverse, then acc_pl = mod_add(inv, red_q(acc_pl))
        uint32_t ti = tau;
        asm volatile("" : "+v"(ti));
        uint64_t *ap = accs[pl];
        inv_poly_from_regs<K, kPfSingle, false>(lds, oacc, ti, nullptr, true, A, A.ninv, 0,
                                                      [&](uint32_t gi, uint64_t x) -> uint64_t {
                                                          const uint64_t a = ap[gi];
                                                          ap[gi] = addq(x, canon ? a : red_q(a, q, mu), q);
                                                          return 0;
                                                      });
        __syncthreads();
        canon = true;
    }
    for (uint32_t i = threadIdx.x; i < 2u * N; i += THREADS) gacc[i] = accs[i / N][i % N];
}

// LB forward transforms in lockstep (the digit rows of one decomposition
// chunk): every twiddle is loaded once for all LB, the butterflies of the LB
// transforms are independent (LB times the ILP), and one barrier per pass
// exchange serves all of them (each has its own LDS region).  From pass PASS
// on; the caller ran pass 0.
template <int LOGN, int PASS, int LB, int PF, typename W>
__device__ __forceinline__ void fwd_rest_lb(W *lds, W (&v)[LB][Geo<LOGN>::E], uint32_t tau,
                                            const Tw<W> *__restrict__ tw, const Arith<W> &ar) {
    using G = Geo<LOGN>;
    if constexpr (PASS < G::NP) {
        Tw<W> t[PassTw<LOGN, PASS>::COUNT];
        load_tw<LOGN, PASS, W, 0, PF>(tau, tw, t);  // in flight across the exchange
#pragma unroll
        for (int l = 0; l < LB; ++l) lds_store<LOGN, PASS - 1>(lds + l * G::LW, v[l], tau);
        xbar<lab_local<PASS - 1, PASS>()>();
#pragma unroll
        for (int l = 0; l < LB; ++l) lds_load<LOGN, PASS>(lds + l * G::LW, v[l], tau);
        load_tw<LOGN, PASS, W, PF, 8>(tau, tw, t);
#pragma unroll
        for (int l = 0; l < LB; ++l) fwd_pass<LOGN, PASS, false>(v[l], t, ar);
        fwd_rest_lb<LOGN, PASS + 1, LB, PF>(lds, v, tau, tw, ar);
    }
}

// k = 1 on two CUs per ciphertext (small batches: the one-workgroup kernel
// above leaves most CUs idle and is bound by its one CU's VALU).  Workgroup
// (ct, h) owns accumulator component h: it transforms the L digit rows of
// X^rot acc_h - acc_h, accumulates their MAC terms for its own output
// component (oacc) and for the partner's (xacc), hands xacc to the partner
// through global memory, adds the partner's terms into oacc, inverts, and
// updates acc_h in LDS.  One hand-off per step per direction.
// Hand-off (MI355X_MICROARCH.md "inter-workgroup visibility", the sc1 form):
// payload stored write-through (sc1, 8 B per lane), every storing wave
// drains (vmcnt(0)), a workgroup barrier, ONE lane stores the flag (sc1) =
// executed step + 1; the consumer's wave 0 polls that word (bounded,
// s_sleep), a barrier, then every payload load is an sc1 load.  Payload
// double-buffered by step parity: a workgroup rewrites parity p only after
// the partner has published the next step, i.e. finished reading p.
// Placement: partners are blocks b and b + 8 (the same XCD when blocks are
// dealt round-robin over the 8 XCDs: speed only, not correctness).
//
// Co-residency is what the hand-off needs, and nothing on the device can
// promise it once other work shares the GPU (another context's stream, a
// second process).  So a partner that does not answer within the timeout
// (s_memrealtime, 100 MHz) is never waited for: the workgroup publishes an
// ABORT flag (its partner, if it ever runs, stops at its next poll), marks the
// ciphertext in fail[], and stores nothing.  The kernel reads its input from a
// saved copy (acc_in) and the host enqueues a repair pass right behind it
// (k_br_persist, one workgroup per ciphertext, `only` = fail[]) that recomputes
// every marked ciphertext from that copy -- so the result is exact whatever
// the residency, and the repairs are counted (fhe_br_repair_count).
typedef __attribute__((address_space(1))) uint64_t g64;
typedef __attribute__((address_space(1))) uint32_t g32;
typedef uint64_t u64x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64x2v pair128(uint64_t a, uint64_t b) {
    u64x2v v;
    v.x = a;
    v.y = b;
    return v;
}
// 1: the hand-off payload as 16-byte sc1 stores / loads (lane-contiguous
// word pairs); 0: 8-byte agent-scope atomics at the words' own positions
#ifndef FHE_BR_PAIR_X16
#define FHE_BR_PAIR_X16 1
#endif
struct BrPairX {
    uint32_t *flag;     // [batch][2] executed-step epochs (zeroed before each launch)
    uint32_t *fail;     // [batch] set by a workgroup that gave up (zeroed before each launch)
    uint64_t *buf;      // [batch][2 halves][2 parities][N] partner MAC terms (W words)
    uint64_t timeout;   // poll budget per hand-off, s_memrealtime ticks (100 MHz)
    uint64_t *stamps = nullptr;  // lab stamp build only: [grid][8] phase cycle sums
};
constexpr uint32_t kBrAbort = 0x80000000u;
// Flag store / poll memory order.  0: relaxed agent-scope atomics ordered by
// the drained write-through payload (the MICROARCH "sc1" form); 1: the flag
// stored with release and polled with acquire semantics (agent scope) -- the
// formal HIP memory-model form, which adds an L2 write-back per step.
#ifndef FHE_BR_PAIR_ACQREL
#define FHE_BR_PAIR_ACQREL 0
#endif
// 4 coefficients per thread (N / 4 threads per workgroup): 12.0 / 29.6 ms for
// the two presets and 4.3 ms for 64 ciphertexts at N = 1024, vs 14.0 / 31.9 /
// 6.1 ms at 8 per thread (round 4).
#ifndef FHE_BR_PAIR_LOGE
#define FHE_BR_PAIR_LOGE 2
#endif
#ifndef FHE_BR_PAIR_LOGE_SMALL
#define FHE_BR_PAIR_LOGE_SMALL 2
#endif
template <int LOGN>
constexpr int br_pair_key() { return gk(LOGN, gk_logn(LOGN) >= 12 ? FHE_BR_PAIR_LOGE : FHE_BR_PAIR_LOGE_SMALL); }
// Levels transformed in lockstep: up to 4, as many LDS exchange regions as
// fit beside the accumulator (tfhe-256-secure, N = 4096 with 64-bit words:
// 3 = its whole L).  Levels beyond LB run in further chunks of LB.
#ifndef FHE_BR_PAIR_LB
#define FHE_BR_PAIR_LB 4
#endif
template <int LOGN, typename W>
constexpr int br_pair_lb() {
    using G = Geo<br_pair_key<LOGN>()>;
    // 128 VGPRs at 16 waves: LB = 4 spills; LB = 3 with 64-bit words spills
    // 4 VGPRs and still measured 29.6 vs 31.0 ms (LB = 1) at
    // tfhe-256-secure (round 5)
    const int cap = G::T >= 1024 ? 3 : 4;
    int lb = FHE_BR_PAIR_LB < cap ? FHE_BR_PAIR_LB : cap;
    while (lb > 1 && G::N * 8 + lb * G::LW * (int)sizeof(W) > 150 * 1024) --lb;
    return lb;
}
// One workgroup per CU: the static LDS plus this dynamic pad exceeds half
// the CU's 160 KiB.
template <int LOGN, typename W, int LB>
constexpr int br_pair_pad_lds() {
    using G = Geo<br_pair_key<LOGN>()>;
    const int st = G::N * 8 + LB * G::LW * (int)sizeof(W) + 16;
    return st > 82 * 1024 ? 0 : 82 * 1024 - st;
}
// Lab diagnostic build (tools/lab/quick_variant2.sh ... -DFHE_BR_STAMPS=1):
// wave 0 of every workgroup sums s_memtime differences per step phase and
// the host prints the shares (FHE_BR_STAMPS=1 at run time).  Read shares,
// never that build's run time.
#ifndef FHE_BR_STAMPS
#define FHE_BR_STAMPS 0
#endif
#if FHE_BR_STAMPS
constexpr int kBrStampPhases = 8;
__device__ __forceinline__ uint64_t br_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define BR_STAMP(ph)                                \
    do {                                            \
        const uint64_t t_ = br_stamp();             \
        st_sum[ph] += t_ - st_last;                 \
        st_last = t_;                               \
    } while (0)
#else
#define BR_STAMP(ph) \
    do {             \
    } while (0)
#endif
// (Prime-specialised arithmetic, ntt_core.hpp gk_sparse, measured 0 to +2 %
// on the three presets, round 5: not used here.)
template <int LOGN, typename W, int LB>
__global__ void __launch_bounds__(Geo<br_pair_key<LOGN>()>::T) k_br_pair(BrArgs D, NttArgs<W> A, BrPairX X,
                                                                        uint32_t batch) {
    constexpr int K = br_pair_key<LOGN>();
    using G = Geo<K>;
    constexpr int N = G::N, T = G::T;
    constexpr bool CV = G::E <= 8;
    __shared__ uint64_t acc[N];      // raw accumulator component h
    __shared__ W lds[LB * G::LW];    // NTT exchange, one region per lockstep level
    __shared__ uint32_t fail;
    const uint32_t b = blockIdx.x, ct = (b >> 4) * 8 + (b & 7), pl = (b >> 3) & 1;
    if (ct >= batch) return;  // whole workgroup (and its partner: same ct)
    const uint32_t tau = threadIdx.x;
    const uint64_t q = A.q64, mu = A.mu64;
    uint64_t *gacc = D.acc + ((size_t)ct * 2 + pl) * N;
    {
        const uint64_t *gin = D.acc_in + ((size_t)ct * 2 + pl) * N;
        const uint32_t r0 = rot_norm(-rot_amount(D.lwe_b[ct], N, D.lwe_q), N);
        for (uint32_t i = tau; i < (uint32_t)N; i += T) acc[i] = rotated_at(gin, i, r0, N, q, mu);
    }
    if (tau == 0) fail = 0;
    __syncthreads();
    const int level = D.level;
    const uint64_t base = 1ull << D.base_log, mask = base - 1, half = base / 2;
    const bool small_base = base <= q;
    const size_t ggsw_words = (size_t)2 * level * 2 * N;
    const uint64_t *lwe_a = D.lwe_a + (size_t)ct * D.lwe_dim;
    g32 *const myflag = (g32 *)(X.flag + (size_t)ct * 2 + pl);
    g32 *const peerflag = (g32 *)(X.flag + (size_t)ct * 2 + (1 - pl));
    g64 *const mybuf = (g64 *)(X.buf + ((size_t)ct * 2 + pl) * 2 * N);
    g64 *const peerbuf = (g64 *)(X.buf + ((size_t)ct * 2 + (1 - pl)) * 2 * N);
    bool canon = false;
    uint32_t epoch = 0;
#if FHE_BR_STAMPS
    uint64_t st_sum[kBrStampPhases] = {}, st_last = br_stamp();
#endif
    for (uint32_t step = 0; step < D.lwe_dim; ++step) {
        const int32_t r = rot_amount(lwe_a[step], N, D.lwe_q);  // uniform, and equal in both halves
        if (r == 0) continue;
        const uint32_t rot = rot_norm(r, N);
        const uint64_t *key = D.bsk + ggsw_words * step;
        W oacc[G::E], xacc[G::E];
        BR_STAMP(7);
        auto diff_at = [&](uint32_t tr, int t) -> uint64_t {  // as in k_br_persist
            const uint32_t p = tr + cbrv(t, G::LOGE) * T;
            const uint32_t j = (p + 2 * N - rot) & (2 * N - 1);
            if (canon) {
                const uint64_t a = acc[j < (uint32_t)N ? j : j - N];
                const uint64_t xr = j < (uint32_t)N || a == 0 ? a : q - a;
                return subq(xr, acc[p], q);
            }
            const uint64_t xr = j < (uint32_t)N ? acc[j] : red_q(q - acc[j - N], q, mu);
            return subq(red_q(xr, q, mu), red_q(acc[p], q, mu), q);
        };
        uint64_t cv[CV ? G::E : 1];
        if constexpr (CV) {
#pragma unroll
            for (int t = 0; t < G::E; ++t) cv[t] = diff_at(tau, t);
        }
        BR_STAMP(0);
        for (int g0 = 0; g0 < level; g0 += LB) {
            // rows g0 .. g0 + LB - 1 of this half (digits MSB first); rows
            // past `level` transform zeros and add nothing
            uint64_t kv[LB][2][G::E];
#pragma unroll
            for (int l = 0; l < LB; ++l) {
                const int row = pl * level + (g0 + l < level ? g0 + l : level - 1);
#pragma unroll
                for (int e = 0; e < G::E; ++e) {
                    const uint32_t gi = gidx<K, G::NP - 1>(tau, e);
                    kv[l][0][e] = key[((size_t)row * 2 + pl) * N + gi];
                    kv[l][1][e] = key[((size_t)row * 2 + (1 - pl)) * N + gi];
                }
            }
            uint32_t tr = tau;
            asm volatile("" : "+v"(tr));
            W v[LB][G::E];
            Tw<W> t0[PassTw<K, 0>::COUNT];
            load_tw<K, 0>(tr, A.twf, t0);
#pragma unroll
            for (int l = 0; l < LB; ++l) {
                const int g = g0 + l;
                const uint32_t shift = g < level ? uint32_t(level - 1 - g) * uint32_t(D.base_log) : 0u;
                load_coeffs<G::E>(v[l], (uint64_t)A.ar.q2 * 2, q, mu, [&](int t) -> uint64_t {
                    if (g >= level) return 0;
                    uint64_t d = ((CV ? cv[CV ? t : 0] : diff_at(tr, t)) >> shift) & mask;
                    if (d > half) d = small_base ? q - (base - d) : red_q(q - (base - d), q, mu);
                    return d;
                });
                fwd_pass<K, 0, false>(v[l], t0, A.ar);
            }
            fwd_rest_lb<K, 1, LB, kPfSingle>(lds, v, tr, A.twf, A.ar);
            BR_STAMP(1);
#pragma unroll
            for (int l = 0; l < LB; ++l) {
                if (g0 + l >= level) break;  // uniform
#pragma unroll
                for (int e = 0; e < G::E; ++e) {
                    const W own = A.ar.mont(v[l][e], (W)kv[l][0][e]), oth = A.ar.mont(v[l][e], (W)kv[l][1][e]);
                    oacc[e] = g0 + l == 0 ? own : A.ar.red2q(oacc[e] + own);
                    xacc[e] = g0 + l == 0 ? oth : A.ar.red2q(xacc[e] + oth);
                }
            }
            if (g0 + LB < level) __syncthreads();  // the exchange regions are reused by the next chunk
            BR_STAMP(2);
        }
        // publish xacc (parity of this step), then take the partner's.
        // (Publishing it before the own terms are accumulated measured 5 %
        // slower at tfhe-256-secure, round 5.)
        ++epoch;
        const uint32_t par = (epoch & 1) * N;
        // (Data-tagged granules -- each word canonical with epoch mod 4 in its
        // top bits, polled by the lane that needs it, no drain or flag --
        // measured 3-5 % slower on all three presets, round 5: the partner's
        // stores take as long to become visible either way, and 16 waves
        // polling four words per lane load the CU's memory queue.)
        {
            uint32_t tx = tau;
            asm volatile("" : "+v"(tx));
            if constexpr (FHE_BR_PAIR_X16 && G::E >= 2 && G::E <= 8) {
                // 16-byte sc1 stores, lane-contiguous pairs (the partner's lane
                // tau reads exactly these words).  The s_nop 1 inside the asm:
                // a store of more than 8 bytes reads its data VGPRs after
                // issue, and the compiler's next VALU may already overwrite
                // them (its hazard pass does not pad inline asm) -- without it
                // a partner received an address word instead of a MAC term
                // now and then (round 6: the intermittent pair-vs-step test
                // failure at N = 2048, and every 64-bit k_br_multi result)
#pragma unroll
                for (int e = 0; e < G::E; e += 2) {
                    g64 *p = mybuf + par + 2 * ((e / 2) * T + tx);
                    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(pair128((uint64_t)xacc[e], (uint64_t)xacc[e + 1]))
                                 : "memory");
                }
            } else {
#pragma unroll
                for (int e = 0; e < G::E; ++e)
                    __hip_atomic_store(mybuf + par + gidx<K, G::NP - 1>(tx, e), (uint64_t)xacc[e], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        BR_STAMP(3);
        if (tau == 0)
            __hip_atomic_store(myflag, epoch, FHE_BR_PAIR_ACQREL ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (tau < 64) {  // wave 0 polls the partner's flag, for at most X.timeout
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            bool ok = false;
            for (;;) {
                const uint32_t f = __hip_atomic_load(peerflag, FHE_BR_PAIR_ACQREL ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                if (f & kBrAbort) break;  // the partner gave up
                if (f >= epoch && X.timeout != 0) {  // zero budget: the test's never-answering partner
                    ok = true;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 >= X.timeout) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (!ok && tau == 0) {
                fail = 1;
                __hip_atomic_store(myflag, kBrAbort | epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((g32 *)(X.fail + ct), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (fail) return;  // workgroup-uniform: nothing stored, the repair pass recomputes ct
        BR_STAMP(4);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
        uint32_t ti = tau;
        asm volatile("" : "+v"(ti));
        if constexpr (FHE_BR_PAIR_X16 && G::E >= 2 && G::E <= 8) {
            // the loads and their wait in ONE asm statement: the outputs exist
            // for the compiler only once they have landed (an output the
            // compiler spills between a load and a separate wait would be
            // stored before it arrives)
            u64x2v x[G::E / 2];
            const g64 *p0 = peerbuf + par + 2 * ti;
            if constexpr (G::E == 2) {
                asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(x[0]) : "v"(p0) : "memory");
            } else if constexpr (G::E == 4) {
                asm volatile("global_load_dwordx4 %0, %2, off sc1\n\tglobal_load_dwordx4 %1, %3, off sc1\n\t"
                             "s_waitcnt vmcnt(0)"
                             : "=&v"(x[0]), "=&v"(x[1]) : "v"(p0), "v"(p0 + 2 * T) : "memory");
            } else {
                static_assert(G::E == 8, "2, 4 or 8 words per lane");
                asm volatile("global_load_dwordx4 %0, %4, off sc1\n\tglobal_load_dwordx4 %1, %5, off sc1\n\t"
                             "global_load_dwordx4 %2, %6, off sc1\n\tglobal_load_dwordx4 %3, %7, off sc1\n\t"
                             "s_waitcnt vmcnt(0)"
                             : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
                             : "v"(p0), "v"(p0 + 2 * T), "v"(p0 + 4 * T), "v"(p0 + 6 * T) : "memory");
            }
#pragma unroll
            for (int e = 0; e < G::E; e += 2) {
                oacc[e] = A.ar.red2q(oacc[e] + (W)x[e / 2].x);
                oacc[e + 1] = A.ar.red2q(oacc[e + 1] + (W)x[e / 2].y);
            }
        } else {
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const W x = (W)__hip_atomic_load(peerbuf + par + gidx<K, G::NP - 1>(ti, e), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
                oacc[e] = A.ar.red2q(oacc[e] + x);
            }
        }
        BR_STAMP(5);
        // component h: inverse, then acc_h = mod_add(inv, red_q(acc_h))
        inv_poly_from_regs<K, kPfSingle, false>(lds, oacc, ti, nullptr, true, A, A.ninv, 0,
                                                [&](uint32_t gi, uint64_t x) -> uint64_t {
                                                    const uint64_t a = acc[gi];
                                                    acc[gi] = addq(x, canon ? a : red_q(a, q, mu), q);
                                                    return 0;
                                                });
        __syncthreads();
        canon = true;
        BR_STAMP(6);
    }
#if FHE_BR_STAMPS
    if (tau == 0 && X.stamps)
        for (int ph = 0; ph < kBrStampPhases; ++ph) X.stamps[(size_t)b * kBrStampPhases + ph] = st_sum[ph];
#endif
    for (uint32_t i = tau; i < (uint32_t)N; i += T) gacc[i] = acc[i];
}

// Blind rotation on M = 2L CUs per ciphertext (k = 1, L = level = 2 or 3):
// member m = (row, digit level) = (m / L, m % L) transforms ONE digit row per
// step (k_br_pair transforms L of them), multiplies it by both key
// components, and publishes both products; every member of row h then sums
// component h over all M members and runs the inverse of component h itself
// (the L members of a row hold the same accumulator row, so the inverse is
// computed L times instead of handed out: one hand-off per step, as in the
// pair).  The critical path of a step is one forward transform instead of L.
// Same hand-off protocol as k_br_pair (write-through payload, drain, barrier,
// relaxed epoch flag; bounded poll of the M - 1 partner flags by wave 0;
// ABORT + fail[] + the host's repair pass when a partner does not answer).
// The M workgroups of a ciphertext are blocks b, b + 8, ..., b + 8 (M - 1):
// one XCD.  Payload per (ciphertext, member): [2 parities][2 components][N].
// Dense form (DN): two workgroups per CU (8 coefficients per thread, no LDS
// pad), for batches whose M workgroups per ciphertext exceed one per CU.
template <int LOGN, bool DN>
constexpr int br_multi_key() { return DN ? gk(LOGN, 3) : br_pair_key<LOGN>(); }
template <int LOGN, bool DN>
constexpr int br_multi_threads() { return Geo<br_multi_key<LOGN, DN>()>::T; }
template <int LOGN, bool DN>
constexpr int br_multi_waves() { return DN ? 2 * br_multi_threads<LOGN, DN>() / 256 : 1; }
template <int LOGN, typename W, int M, bool DN>
__global__ void __launch_bounds__((br_multi_threads<LOGN, DN>()), (br_multi_waves<LOGN, DN>()))
    k_br_multi(BrArgs D, NttArgs<W> A, BrPairX X, uint32_t batch) {
    constexpr int K = br_multi_key<LOGN, DN>();
    using G = Geo<K>;
    constexpr int N = G::N, T = G::T, L = M / 2;
    static_assert(M == 4 || M == 6, "two or three digit levels");
    static_assert(G::E >= 2 && G::E <= 8, "2, 4 or 8 words per lane");
    __shared__ uint64_t acc[N];  // raw accumulator component h
    __shared__ W lds[G::LW];     // NTT exchange
    __shared__ uint32_t fail;
    const uint32_t b = blockIdx.x, ct = (b / (8 * M)) * 8 + (b & 7), m = (b >> 3) % M;
    if (ct >= batch) return;  // every member of ct takes the same branch
    const uint32_t pl = m / L, lv = m % L;
    const uint32_t tau = threadIdx.x;
    const uint64_t q = A.q64, mu = A.mu64;
    {
        const uint64_t *gin = D.acc_in + ((size_t)ct * 2 + pl) * N;
        const uint32_t r0 = rot_norm(-rot_amount(D.lwe_b[ct], N, D.lwe_q), N);
        for (uint32_t i = tau; i < (uint32_t)N; i += T) acc[i] = rotated_at(gin, i, r0, N, q, mu);
    }
    if (tau == 0) fail = 0;
    __syncthreads();
    const uint64_t base = 1ull << D.base_log, mask = base - 1, half = base / 2;
    const bool small_base = base <= q;
    const uint32_t shift = uint32_t(L - 1 - lv) * uint32_t(D.base_log);
    const size_t ggsw_words = (size_t)2 * L * 2 * N;
    const size_t row = (size_t)pl * L + lv;
    const uint64_t *lwe_a = D.lwe_a + (size_t)ct * D.lwe_dim;
    g32 *const flags = (g32 *)(X.flag + (size_t)ct * M);
    g64 *const mybuf = (g64 *)(X.buf + ((size_t)ct * M + m) * 4 * N);
    bool canon = false;
    uint32_t epoch = 0;
    for (uint32_t step = 0; step < D.lwe_dim; ++step) {
        const int32_t r = rot_amount(lwe_a[step], N, D.lwe_q);  // uniform, and equal in every member
        if (r == 0) continue;
        const uint32_t rot = rot_norm(r, N);
        const uint64_t *key = D.bsk + ggsw_words * step;
        W oacc[G::E], xacc[G::E];
        {
            uint64_t kv[2][G::E];
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const uint32_t gi = gidx<K, G::NP - 1>(tau, e);
                kv[0][e] = key[(row * 2 + pl) * N + gi];
                kv[1][e] = key[(row * 2 + (1 - pl)) * N + gi];
            }
            uint32_t tr = tau;
            asm volatile("" : "+v"(tr));
            W v[1][G::E];
            Tw<W> t0[PassTw<K, 0>::COUNT];
            load_tw<K, 0>(tr, A.twf, t0);
            load_coeffs<G::E>(v[0], (uint64_t)A.ar.q2 * 2, q, mu, [&](int t) -> uint64_t {
                const uint32_t p = tr + cbrv(t, G::LOGE) * T;
                const uint32_t j = (p + 2 * N - rot) & (2 * N - 1);
                uint64_t df;
                if (canon) {
                    const uint64_t a = acc[j < (uint32_t)N ? j : j - N];
                    const uint64_t xr = j < (uint32_t)N || a == 0 ? a : q - a;
                    df = subq(xr, acc[p], q);
                } else {
                    const uint64_t xr = j < (uint32_t)N ? acc[j] : red_q(q - acc[j - N], q, mu);
                    df = subq(red_q(xr, q, mu), red_q(acc[p], q, mu), q);
                }
                uint64_t d = (df >> shift) & mask;
                if (d > half) d = small_base ? q - (base - d) : red_q(q - (base - d), q, mu);
                return d;
            });
            fwd_pass<K, 0, false>(v[0], t0, A.ar);
            fwd_rest_lb<K, 1, 1, kPfSingle>(lds, v, tr, A.twf, A.ar);
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                oacc[e] = A.ar.mont(v[0][e], (W)kv[0][e]);
                xacc[e] = A.ar.mont(v[0][e], (W)kv[1][e]);
            }
        }
#ifndef FHE_BR_MULTI_INVPF
#define FHE_BR_MULTI_INVPF 1
#endif
        // the inverse's first-pass twiddles, in flight across the hand-off
        // (inv_poly_from_regs would load them after it)
        constexpr int LAST = G::NP - 1;
        Tw<W> tl[PassTw<K, LAST>::COUNT];
        if constexpr (FHE_BR_MULTI_INVPF) load_tw<K, LAST>(tau, A.twi, tl);
        ++epoch;
        const uint32_t par = (epoch & 1) * 2 * N;
        {
            // slot c of this member = its product for output component c
            uint32_t tx = tau;
            asm volatile("" : "+v"(tx));
#pragma unroll
            for (int e = 0; e < G::E; e += 2) {
                g64 *p0 = mybuf + par + pl * N + 2 * ((e / 2) * T + tx);
                g64 *p1 = mybuf + par + (1 - pl) * N + 2 * ((e / 2) * T + tx);
                asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p0), "v"(pair128((uint64_t)oacc[e], (uint64_t)oacc[e + 1]))
                             : "memory");
                asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p1), "v"(pair128((uint64_t)xacc[e], (uint64_t)xacc[e + 1]))
                             : "memory");
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        if (tau == 0) __hip_atomic_store(flags + m, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tau < 64) {  // wave 0: lane i polls member i, for at most X.timeout
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            bool ok = false;
            for (;;) {
                uint32_t f = epoch;
                if (tau < (uint32_t)M && tau != m)
                    f = __hip_atomic_load(flags + tau, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool ab = (f & kBrAbort) != 0;
                if (__ballot(ab)) break;  // a member gave up
                if (__ballot(f < epoch) == 0 && X.timeout != 0) {  // zero budget: the tests' never-answering partner
                    ok = true;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 >= X.timeout) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (!ok && tau == 0) {
                fail = 1;
                __hip_atomic_store(flags + m, kBrAbort | epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((g32 *)(X.fail + ct), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (fail) return;  // workgroup-uniform: nothing stored, the repair pass recomputes ct
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
        uint32_t ti = tau;
        asm volatile("" : "+v"(ti));
#pragma unroll
        for (int o = 1; o < M; ++o) {
            const uint32_t pm = (m + o) % M;
            const g64 *src = (const g64 *)(X.buf + ((size_t)ct * M + pm) * 4 * N) + par + pl * N;
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const W x = (W)__hip_atomic_load(src + 2 * ((e / 2) * T + ti) + (e & 1), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
                oacc[e] = A.ar.red2q(oacc[e] + x);
            }
        }
        // component h: inverse, then acc_h = mod_add(inv, red_q(acc_h))
        if constexpr (FHE_BR_MULTI_INVPF && !stream_tw<K, W>()) {
            inv_pass<K, LAST, true>(oacc, tl, A.ar, A.ninv);
            inv_rest<K, LAST - 1, true, kPfSingle>(lds, oacc, ti, A.twi, A.ar, A.ninv);
#pragma unroll
            for (int t = 0; t < G::E; ++t) {
                const uint32_t gi = ti + cbrv(t, G::LOGE) * T;
                const uint64_t a = acc[gi];
                acc[gi] = addq((uint64_t)A.ar.red1q(oacc[t]), canon ? a : red_q(a, q, mu), q);
            }
        } else {
            inv_poly_from_regs<K, kPfSingle, false>(lds, oacc, ti, nullptr, true, A, A.ninv, 0,
                                                    [&](uint32_t gi, uint64_t x) -> uint64_t {
                                                        const uint64_t a = acc[gi];
                                                        acc[gi] = addq(x, canon ? a : red_q(a, q, mu), q);
                                                        return 0;
                                                    });
        }
        __syncthreads();
        canon = true;
    }
    if (lv == 0) {
        uint64_t *gacc = D.acc + ((size_t)ct * 2 + pl) * N;
        for (uint32_t i = tau; i < (uint32_t)N; i += T) gacc[i] = acc[i];
    }
}

// GLWE dimension k >= 2 (K1 = k + 1 >= 3 accumulators): the same one-launch
// structure, generic in K1.  A step has K1 L digit rows; P thread groups
// transform them P at a time (row r0 + group), and every row's product with
// the step's GGSW goes to all K1 output components, so each group
// accumulates its rows' contributions for all K1 components in its own
// NTT-domain LDS region (oacc[group][j], own positions: no barrier).  The
// K1 inverses then run P at a time, each from the sum of the groups'
// partials, and their epilogue adds the old accumulator (cmux :537).  Rows
// and components past the end leave that group idle for the round (it still
// runs the transform on zeros: the exchange barriers are workgroup-wide).
// 2^LOGP transforms at a time (groups of 256 >> LOGP threads).  Four groups
// (fewer, longer rounds: 2 forward and 1 inverse round per step at K1 L = 6
// instead of 3 and 2) measured slower on MI355X -- 25.2 vs 20.1 ms for one
// k = 2, N = 1024 blind rotation (profiles/r3j) -- so two (FHE_BRK_P4=1
// keeps the four-group build for A/B).
#ifndef FHE_BRK_P4
#define FHE_BRK_P4 0
#endif
template <int LOGN, int LOGP>
constexpr int br_k_key() { return gk(LOGN, LOGN - 8 + LOGP); }
template <int LOGN, typename W, int K1, int LOGP>
constexpr int br_k_lds_bytes() {
    using G = Geo<br_k_key<LOGN, LOGP>()>;
    return K1 * G::N * 8 + (1 << LOGP) * G::LW * (int)sizeof(W) + (1 << LOGP) * K1 * G::N * (int)sizeof(W);
}
template <int LOGN, typename W, int K1>
constexpr int br_k_logp() { return FHE_BRK_P4 && br_k_lds_bytes<LOGN, W, K1, 2>() <= 160 * 1024 ? 2 : 1; }
// twiddle stages issued ahead in the k >= 2 kernel's transforms
#ifndef FHE_BRK_PF
#define FHE_BRK_PF 4
#endif
template <int LOGN, typename W, int K1, int LOGP>
__global__ void __launch_bounds__(256) k_br_persist_k(BrArgs D, NttArgs<W> A) {
    constexpr int K = br_k_key<LOGN, LOGP>();
    using G = Geo<K>;
    constexpr int P = 1 << LOGP;
    static_assert(G::P == P && G::THREADS == 256, "P thread groups per workgroup");
    static_assert(br_k_lds_bytes<LOGN, W, K1, LOGP>() <= 160 * 1024, "LDS");
    constexpr int N = G::N;
    __shared__ uint64_t accs[K1][N];   // raw accumulators (component j)
    __shared__ W xlds[P * G::LW];      // NTT exchange, one region per group
    __shared__ W oacc[P][K1][N];       // NTT-domain partial sums per group
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = threadIdx.x >> G::LOGT;
    const size_t ct = blockIdx.x;
    const uint64_t q = A.q64, mu = A.mu64;
    W *lds = xlds + pl * G::LW;
    uint64_t *gacc = D.acc + ct * K1 * N;
    {
        const uint32_t r0 = rot_norm(-rot_amount(D.lwe_b[ct], N, D.lwe_q), N);
        for (uint32_t i = threadIdx.x; i < (uint32_t)(K1 * N); i += G::THREADS) {
            const uint32_t j = i / N, p = i % N;
            accs[j][p] = rotated_at(gacc + (size_t)j * N, p, r0, N, q, mu);
        }
    }
    __syncthreads();
    const int level = D.level, rows = K1 * level;
    const uint64_t base = 1ull << D.base_log, mask = base - 1, half = base / 2;
    const size_t ggsw_words = (size_t)rows * K1 * N;
    const uint64_t *lwe_a = D.lwe_a + ct * D.lwe_dim;
    for (uint32_t step = 0; step < D.lwe_dim; ++step) {
        const int32_t r = rot_amount(lwe_a[step], N, D.lwe_q);  // workgroup-uniform
        if (r == 0) continue;
        const uint32_t rot = rot_norm(r, N);
        const uint64_t *key = D.bsk + ggsw_words * step;
        for (int rb = 0; rb < rows; rb += P) {
            const int row = rb + (int)pl;
            const bool active = row < rows;
            const int comp = active ? row / level : 0, g = active ? row % level : 0;
            const uint32_t shift = uint32_t(level - 1 - g) * uint32_t(D.base_log);
            uint32_t tr = tau;
            asm volatile("" : "+v"(tr));
            // this row's key terms for all K1 components, in flight across
            // the transform (issued first: loads retire in order)
            const uint64_t *kr = key + (size_t)(active ? row : 0) * K1 * N;
            uint64_t kv[K1][G::E];
#pragma unroll
            for (int j = 0; j < K1; ++j)
#pragma unroll
                for (int e = 0; e < G::E; ++e) kv[j][e] = kr[(size_t)j * N + gidx<K, G::NP - 1>(tr, e)];
            W v[G::E];
            Tw<W> t0[PassTw<K, 0>::COUNT];
            load_tw<K, 0>(tr, A.twf, t0);
            const uint64_t *ac = accs[comp];
            load_coeffs<G::E>(v, (uint64_t)A.ar.q2 * 2, q, mu, [&](int t) -> uint64_t {
                if (!active) return 0;
                const uint32_t p = tr + cbrv(t, G::LOGE) * G::T;
                const uint32_t j = (p + 2 * N - rot) & (2 * N - 1);
                const uint64_t xr = j < (uint32_t)N ? ac[j] : red_q(q - ac[j - N], q, mu);
                const uint64_t c = subq(red_q(xr, q, mu), red_q(ac[p], q, mu), q);
                uint64_t d = (c >> shift) & mask;
                if (d > half) d = red_q(q - (base - d), q, mu);
                return d;
            });
            fwd_pass<K, 0, false>(v, t0, A.ar);
            fwd_rest<K, 1, false, FHE_BRK_PF>(lds, v, tr, A.twf, A.ar);
            if (active) {
                // raw output (< 4q) times canonical keys: valid Montgomery pairs
#pragma unroll
                for (int j = 0; j < K1; ++j) {
#pragma unroll
                    for (int e = 0; e < G::E; ++e) {
                        const uint32_t gi = gidx<K, G::NP - 1>(tr, e);
                        const W m = A.ar.mont(v[e], (W)kv[j][e]);
                        oacc[pl][j][gi] = rb < P ? m : A.ar.red2q(oacc[pl][j][gi] + m);
                    }
                }
            }
            __syncthreads();  // the exchange regions are reused by the next round
        }
        // components j0 + pl: inverse of the two halves' sum, then
        // acc_j = mod_add(inv, red_q(acc_j))
        for (int j0 = 0; j0 < K1; j0 += P) {
            const int j = j0 + (int)pl;
            const bool active = j < K1;
            uint32_t ti = tau;
            asm volatile("" : "+v"(ti));
            W v[G::E];
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const uint32_t gi = gidx<K, G::NP - 1>(ti, e);
                W x = 0;
                if (active) {
                    // groups that ran no row of this step hold stale partials
#pragma unroll
                    for (int h = 0; h < P; ++h)
                        if (h < rows) x = A.ar.red2q(x + oacc[h][j][gi]);
                }
                v[e] = x;
            }
            uint64_t *ap = accs[active ? j : 0];
            inv_poly_from_regs<K, FHE_BRK_PF, false>(lds, v, ti, nullptr, true, A, A.ninv, 0,
                                                     [&](uint32_t gi, uint64_t x) -> uint64_t {
                                                         if (active) ap[gi] = addq(x, red_q(ap[gi], q, mu), q);
                                                        return 0;
                                                    });
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < (uint32_t)(K1 * N); i += G::THREADS) gacc[i] = accs[i / N][i % N];
}

// k1 == 2: N = 512..4096; k1 = 3..5 (GLWE dimension 2..4): N = 512..2048
// wherever the K1 accumulators, the exchange regions and both groups'
// partial sums fit in LDS (u64: k = 2..4 at N <= 1024; u32: k = 2, 3 at
// N = 2048 too).
constexpr int kBrK1Max = 5;
template <int LOGN, typename W, int K1>
constexpr bool brk_fits() {
    return LOGN >= 9 && LOGN <= 11 && br_k_lds_bytes<LOGN, W, K1, br_k_logp<LOGN, W, K1>()>() <= 160 * 1024;
}
template <int LOGN, typename W>
static bool brk_fits_rt(int k1) {
    switch (k1) {
    case 3: return brk_fits<LOGN, W, 3>();
    case 4: return brk_fits<LOGN, W, 4>();
    case 5: return brk_fits<LOGN, W, 5>();
    default: return false;
    }
}
bool br_persist_supported(const Plan &p, int k1) {
    if (p.wide) return false;
    if (k1 == 2) return p.logn >= 9 && p.logn <= 12;
    if (k1 < 3 || k1 > kBrK1Max) return false;
    switch (p.logn) {
    case 9: return p.word == 32 ? brk_fits_rt<9, uint32_t>(k1) : brk_fits_rt<9, uint64_t>(k1);
    case 10: return p.word == 32 ? brk_fits_rt<10, uint32_t>(k1) : brk_fits_rt<10, uint64_t>(k1);
    case 11: return p.word == 32 ? brk_fits_rt<11, uint32_t>(k1) : brk_fits_rt<11, uint64_t>(k1);
    default: return false;
    }
}

template <int LOGN, typename W, int K1>
static hipError_t brk_launch(const Plan &p, const BrArgs &D, size_t batch, const NttArgs<W> &A) {
    if constexpr (brk_fits<LOGN, W, K1>()) {
        constexpr int LP = br_k_logp<LOGN, W, K1>();
        hipLaunchKernelGGL((k_br_persist_k<LOGN, W, K1, LP>), dim3((unsigned)batch), dim3(256), 0, p.stream, D, A);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}
template <int LOGN, typename W>
static hipError_t br_one(const Plan &p, int k1, const BrArgs &D, size_t batch, const NttArgs<W> &A) {
    switch (k1) {
    case 2:
        hipLaunchKernelGGL((k_br_persist<LOGN, W>), dim3((unsigned)batch), dim3(br_threads<LOGN>()), 0, p.stream, D,
                           A);
        return hipGetLastError();
    case 3: return brk_launch<LOGN, W, 3>(p, D, batch, A);
    case 4: return brk_launch<LOGN, W, 4>(p, D, batch, A);
    case 5: return brk_launch<LOGN, W, 5>(p, D, batch, A);
    default: return hipErrorInvalidValue;
    }
}
template <typename W>
static hipError_t br_dispatch(const Plan &p, int k1, const BrArgs &D, size_t batch, const NttArgs<W> &A) {
    // k = 1 with 64-bit words in compat mode: unit twiddles in pass 0
    // (ntt_core.hpp gk_compat), as in the two-CU kernel
    if constexpr (sizeof(W) == 8) {
        if (p.compat && k1 == 2 && p.logn >= 10) {
            const auto go = [&](auto K) -> hipError_t {
                constexpr int L = decltype(K)::value;
                hipLaunchKernelGGL((k_br_persist<L, W>), dim3((unsigned)batch), dim3(br_threads<L>()), 0, p.stream,
                                   D, A);
                return hipGetLastError();
            };
            switch (p.logn) {
            case 10: return go(std::integral_constant<int, gk_compat(10)>{});
            case 11: return go(std::integral_constant<int, gk_compat(11)>{});
            case 12: return go(std::integral_constant<int, gk_compat(12)>{});
            default: break;
            }
        }
    }
    switch (p.logn) {
    case 9: return br_one<9, W>(p, k1, D, batch, A);
    case 10: return br_one<10, W>(p, k1, D, batch, A);
    case 11: return br_one<11, W>(p, k1, D, batch, A);
    case 12: return br_one<12, W>(p, k1, D, batch, A);
    default: return hipErrorInvalidValue;
    }
}

// Two-CU blind rotation (k = 1, N = 1024..4096): grid of 16 ceil(batch / 8)
// blocks, taken only when that grid fits one block per CU.
bool br_pair_supported(const Plan &p, int k1, size_t batch) {
    if (p.wide || k1 != 2 || p.logn < 10 || p.logn > 12 || batch == 0) return false;
    return 16 * ((batch + 7) / 8) <= (size_t)p.cus;
}
// M = 2 level CUs per ciphertext (k_br_multi) when every ciphertext's M
// workgroups fit one XCD beside the others dealt to it: 8 ceil(batch / 8)
// ciphertexts' worth of blocks, M ceil(batch / 8) per XCD, one per CU; up to
// twice that in the dense form (two per CU, kBrMultiDense bit); 0 = the pair.
// (The dense form measured slower than the pair: tfhe-256-secure at batch 64
// 32.6 vs 28.2 ms, round 6, profiles/r6r; lab FHE_BR_MULTI_DENSE=1, parity
// green in the blind-rotation suite.)
#ifndef FHE_BR_MULTI_DENSE
#define FHE_BR_MULTI_DENSE 0
#endif
constexpr int kBrMultiDense = 0x100;
int br_multi_members(const Plan &p, int level, size_t batch) {
    if (p.wide || level < 2 || level > 3 || p.logn < 10 || p.logn > 12 || batch == 0) return 0;
    const int M = 2 * level;
    const size_t per_xcd = (size_t)M * ((batch + 7) / 8), cus = (size_t)p.cus / 8;
    if (per_xcd <= cus) return M;
    return FHE_BR_MULTI_DENSE && per_xcd <= 2 * cus ? (M | kBrMultiDense) : 0;
}
// scratch: flags [batch][M] u32 + fail [batch] u32 (16-byte aligned), the
// saved input accumulators [batch][2][N], the hand-off buffers
// [batch][M][2 parities][2 components][N] (pair: [batch][2][2][N])
static size_t br_pair_flag_bytes(size_t batch, int members) {
    return ((batch * (members + 1) * 4 + 15) / 16) * 16;
}
size_t br_pair_scratch_bytes(const Plan &p, size_t batch, int level, bool multi) {
    const size_t n = (size_t)1 << p.logn;
    const int M = multi ? br_multi_members(p, level, batch) & 0xff : 0;
    const size_t xbuf = M ? batch * M * 4 * n * 8 : batch * 2 * 2 * n * 8;
    return br_pair_flag_bytes(batch, M ? M : 2) + batch * 2 * n * 8 + xbuf;
}
template <int LOGN, typename W, int LB>
static hipError_t br_pair_lb_one(const Plan &p, const BrArgs &D, const BrPairX &X, size_t batch, const NttArgs<W> &A,
                                bool coop) {
    constexpr int PAD = br_pair_pad_lds<LOGN, W, LB>();
    const unsigned grid = (unsigned)(16 * ((batch + 7) / 8));
    const dim3 block(Geo<br_pair_key<LOGN>()>::T);
    if (!coop) {
        hipLaunchKernelGGL((k_br_pair<LOGN, W, LB>), dim3(grid), block, PAD, p.stream, D, A, X, (uint32_t)batch);
        return hipGetLastError();
    }
    // cooperative launch: the runtime checks the whole grid against the
    // device's occupancy before it starts (hipErrorCooperativeLaunchTooLarge
    // instead of a grid that can never be co-resident)
    BrArgs d = D;
    NttArgs<W> a = A;
    BrPairX x = X;
    uint32_t nb = (uint32_t)batch;
    void *args[] = {&d, &a, &x, &nb};
    return hipLaunchCooperativeKernel((const void *)k_br_pair<LOGN, W, LB>, dim3(grid), block, args, PAD,
                                      p.stream);
}
template <int LOGN, typename W, int M, bool DN>
static hipError_t br_multi_one(const Plan &p, const BrArgs &D, const BrPairX &X, size_t batch, const NttArgs<W> &A) {
    constexpr int PAD = DN ? 0 : br_pair_pad_lds<LOGN, W, 1>();
    const unsigned grid = (unsigned)(8 * M * ((batch + 7) / 8));
    hipLaunchKernelGGL((k_br_multi<LOGN, W, M, DN>), dim3(grid), dim3(br_multi_threads<LOGN, DN>()), PAD,
                       p.stream, D, A, X, (uint32_t)batch);
    return hipGetLastError();
}
// Lockstep width for `level` levels: the LB <= br_pair_lb() with the fewest
// idle (zero) transforms, the widest among equals.
template <int LOGN, typename W>
static hipError_t br_pair_one(const Plan &p, const BrArgs &D, const BrPairX &X, size_t batch, const NttArgs<W> &A,
                              bool coop, int members) {
    switch (members) {
    case 4: return br_multi_one<LOGN, W, 4, false>(p, D, X, batch, A);
    case 6: return br_multi_one<LOGN, W, 6, false>(p, D, X, batch, A);
    case 4 | kBrMultiDense: return br_multi_one<LOGN, W, 4, true>(p, D, X, batch, A);
    case 6 | kBrMultiDense: return br_multi_one<LOGN, W, 6, true>(p, D, X, batch, A);
    default: break;
    }
    constexpr int LM = br_pair_lb<LOGN, W>();
    int lb = 1, best = 1 << 30;
    for (int c = 1; c <= LM; ++c) {
        const int work = (D.level + c - 1) / c * c;
        if (work <= best) best = work, lb = c;
    }
    switch (lb) {
    case 4: if constexpr (LM >= 4) return br_pair_lb_one<LOGN, W, 4>(p, D, X, batch, A, coop); else break;
    case 3: if constexpr (LM >= 3) return br_pair_lb_one<LOGN, W, 3>(p, D, X, batch, A, coop); else break;
    case 2: if constexpr (LM >= 2) return br_pair_lb_one<LOGN, W, 2>(p, D, X, batch, A, coop); else break;
    default: break;
    }
    return br_pair_lb_one<LOGN, W, 1>(p, D, X, batch, A, coop);
}
template <typename W>
static hipError_t br_pair_dispatch(const Plan &p, const BrArgs &D, const BrPairX &X, size_t batch,
                                   const NttArgs<W> &A, bool coop, int members) {
    // 64-bit words in compat mode (the TFHE presets' moduli): unit twiddles
    // in pass 0 (ntt_core.hpp gk_compat)
    if constexpr (sizeof(W) == 8) {
        if (p.compat) {
            switch (p.logn) {
            case 10: return br_pair_one<gk_compat(10), W>(p, D, X, batch, A, coop, members);
            case 11: return br_pair_one<gk_compat(11), W>(p, D, X, batch, A, coop, members);
            case 12: return br_pair_one<gk_compat(12), W>(p, D, X, batch, A, coop, members);
            default: return hipErrorInvalidValue;
            }
        }
    }
    switch (p.logn) {
    case 10: return br_pair_one<10, W>(p, D, X, batch, A, coop, members);
    case 11: return br_pair_one<11, W>(p, D, X, batch, A, coop, members);
    case 12: return br_pair_one<12, W>(p, D, X, batch, A, coop, members);
    default: return hipErrorInvalidValue;
    }
}
hipError_t launch_br_pair(const Plan &p, int level, int base_log, uint64_t *acc, const uint64_t *bsk,
                          const uint64_t *lwe_a, const uint64_t *lwe_b, uint32_t lwe_dim, uint64_t lwe_q, size_t batch,
                          void *scratch, const BrPairOpts &o) {
    if (!br_pair_supported(p, 2, batch)) return hipErrorInvalidValue;
    const int members = o.multi ? br_multi_members(p, level, batch) : 0, nm = members ? members & 0xff : 2;
    const size_t n = (size_t)1 << p.logn, fbytes = br_pair_flag_bytes(batch, nm), abytes = batch * 2 * n * 8;
    uint32_t *flag = (uint32_t *)scratch, *failw = flag + batch * nm;
    uint64_t *acc_in = (uint64_t *)((char *)scratch + fbytes);
    uint64_t *buf = acc_in + batch * 2 * n;
    hipError_t e = hipMemsetAsync(scratch, 0, fbytes, p.stream);  // flags and fail words, every launch
    if (e == hipSuccess) e = hipMemcpyAsync(acc_in, acc, abytes, hipMemcpyDeviceToDevice, p.stream);
    if (e != hipSuccess) return e;
    BrArgs D{acc, bsk, lwe_a, lwe_b, lwe_q, lwe_dim, level, base_log};
    D.acc_in = acc_in;
    BrPairX X{flag, failw, buf, o.timeout_ticks};
#if FHE_BR_STAMPS
    const size_t grid = 16 * ((batch + 7) / 8);
    const char *sv = std::getenv("FHE_BR_STAMPS");
    if (sv && sv[0] == '1' && hipMalloc(&X.stamps, grid * kBrStampPhases * 8) == hipSuccess)
        (void)hipMemsetAsync(X.stamps, 0, grid * kBrStampPhases * 8, p.stream);
#endif
    e = p.word == 32 ? br_pair_dispatch<uint32_t>(p, D, X, batch, p.a32, o.coop, members)
                     : br_pair_dispatch<uint64_t>(p, D, X, batch, p.a64, o.coop, members);
#if FHE_BR_STAMPS
    if (X.stamps) {
        std::vector<uint64_t> h(grid * kBrStampPhases);
        (void)hipStreamSynchronize(p.stream);
        (void)hipMemcpy(h.data(), X.stamps, h.size() * 8, hipMemcpyDeviceToHost);
        double sum[kBrStampPhases] = {}, tot = 0;
        size_t used = 0;
        for (size_t w = 0; w < grid; ++w) {
            if (h[w * kBrStampPhases + 6] == 0) continue;
            ++used;
            for (int ph = 0; ph < kBrStampPhases; ++ph) sum[ph] += (double)h[w * kBrStampPhases + ph];
        }
        for (int ph = 0; ph < kBrStampPhases; ++ph) tot += sum[ph];
        static const char *nm[kBrStampPhases] = {"diff", "fwd", "mac", "publish", "poll", "payload", "inverse", "step"};
        std::fprintf(stderr, "[br stamps] N=%u level=%d workgroups=%zu cycles/wg=%.0f:", 1u << p.logn, level, used,
                     used ? tot / used : 0.0);
        for (int ph = 0; ph < kBrStampPhases; ++ph) std::fprintf(stderr, " %s %.1f%%", nm[ph], tot ? 100 * sum[ph] / tot : 0.0);
        std::fprintf(stderr, "\n");
        (void)hipFree(X.stamps);
    }
#endif
    if (e == hipErrorCooperativeLaunchTooLarge) {
        // the grid cannot be co-resident on this device: every ciphertext
        // goes to the repair pass (the one-CU kernel)
        (void)hipGetLastError();
        e = hipMemsetAsync(failw, 0x01, batch * 4, p.stream);
    }
    if (e != hipSuccess) return e;
    // repair pass: the ciphertexts marked in fail[], from the saved input
    BrArgs R = D;
    R.only = failw;
    R.repairs = o.repairs;
    return p.word == 32 ? br_dispatch<uint32_t>(p, 2, R, batch, p.a32) : br_dispatch<uint64_t>(p, 2, R, batch, p.a64);
}

hipError_t launch_br_persist(const Plan &p, int k1, int level, int base_log, uint64_t *acc, const uint64_t *bsk,
                             const uint64_t *lwe_a, const uint64_t *lwe_b, uint32_t lwe_dim, uint64_t lwe_q,
                             size_t batch) {
    if (!br_persist_supported(p, k1)) return hipErrorInvalidValue;
    if (batch == 0) return hipSuccess;
    // grid.x <= 2^31 - 1 workgroups
    const size_t per = (size_t)1 << 30;
    for (size_t b0 = 0; b0 < batch; b0 += per) {
        const size_t nb = batch - b0 < per ? batch - b0 : per;
        BrArgs D{acc + b0 * (size_t)k1 * ((size_t)1 << p.logn), bsk, lwe_a + b0 * lwe_dim, lwe_b + b0, lwe_q, lwe_dim,
                 level, base_log};
        hipError_t e = p.word == 32 ? br_dispatch<uint32_t>(p, k1, D, nb, p.a32)
                                    : br_dispatch<uint64_t>(p, k1, D, nb, p.a64);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace FHE_NS
