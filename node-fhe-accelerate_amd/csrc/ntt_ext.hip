// ntt_ext.hip -- decompose / NTT / key-MAC / inverse kernels: the TFHE
// external product, BFV-style relinearisation and the blind-rotation CMux
// step share one kernel body (k_dmac) and differ only in where the digit
// polynomials come from and what the store epilogue adds.
//
// MODE 0  external product (BootstrapEngine::external_product,
//         bootstrap_engine.cpp:431-518): for each decomposition row r (mask
//         polynomials first, then the body; digit level inner, digits of
//         decompose_polynomial :152-185) and each output component j:
//           res_j = mod_add(res_j, inv( fwd(decomp_r) (.) fwd(ggsw[r][j]) )).
// MODE 1  relinearisation (EncryptionEngine::relinearize, encryption.cpp:
//         904-980): digit l of c2 is (c2 >> l*B) & (2^B - 1) (unsigned, LSB
//         first); c0' = c0 + sum_l inv(fwd(d_l) (.) fwd(b_l)),
//         c1' = c1 + sum_l inv(fwd(d_l) (.) fwd(a_l)), keys given as (a_l, b_l)
//         pairs (KeySwitchKey, key_manager.h:85-95; key_manager.cpp:296-324).
// MODE 2  one blind-rotation step (BootstrapEngine::blind_rotate :547-577 ->
//         cmux :520-540 -> multiply_glwe_by_monomial :249-261 ->
//         rotate_polynomial :122-145) for a batch of accumulators, each with
//         its own LWE mask coefficient a_i:
//           rot = (int32)((a_i * 2N + q/2) / q)   (u64 arithmetic)
//           rot == 0 : acc unchanged (the reference `continue`s)
//           else     : acc' = acc + ExtProd(X^rot * acc - acc, bsk[i])
//         The rotation and the subtraction are folded into the digit load.
// MODE 3  CMux with explicit inputs (cmux :520-540): out = ct0 +
//         ExtProd(ct1 - ct0, ggsw).
//
// Every intermediate is a canonical residue and the inverse transform is
// linear over Z_q, so  sum_r inv(X_r) == inv(sum_r X_r)  bit-exactly: keys are
// transformed once (fhe_ggsw_prepare / fhe_relin_key_prepare: NTT x R,
// Montgomery form), every digit polynomial is produced on its HBM load,
// transformed in registers/LDS, multiplied into K1 NTT-domain accumulators,
// and only K1 inverse transforms run at the end -- one kernel, one HBM pass
// over the ciphertext.
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
#include "lwe_ops.hpp"

namespace FHE_NS {

// Where the K1 NTT-domain accumulators live between rows: 1 = a second LDS
// region, 2 = the ciphertext's own output rows in HBM (read-modify-write of
// the thread's own positions; no synchronisation needed).  Holding them in
// VGPRs spilled 300-800 B/lane.
// LDS accumulators are used only while they leave at least kExtMinWaves
// waves per CU resident: at N = 1024 with u64 words they would cut the CU to
// one 4-wave workgroup (99 KB of LDS), and the HBM/L2 round trip of the
// output-row stash is cheaper than that loss of latency hiding.
#ifndef FHE_EXT_MINWAVES
#define FHE_EXT_MINWAVES 8
#endif
constexpr int kExtMinWaves = FHE_EXT_MINWAVES;
template <int LOGN, typename W, int K1, int MODE = 0>
constexpr int ext_stash() {
    using G = Geo<LOGN>;
    constexpr int bytes = G::P * (G::LW + K1 * G::N) * (int)sizeof(W);
    if (bytes <= 160 * 1024) {
        const int wg = (160 * 1024) / bytes < 2048 / G::THREADS ? (160 * 1024) / bytes : 2048 / G::THREADS;
        if (wg * G::THREADS / 64 >= kExtMinWaves) return 1;
    }
    // relinearisation (MODE 1): accumulator 0 in LDS, accumulator 1 and the
    // c2 words in VGPRs (one workgroup per CU); c2 is then read once instead
    // of once per digit level
#ifndef FHE_RELIN_REGS
#define FHE_RELIN_REGS 1
#endif
    if (FHE_RELIN_REGS && MODE == 1 && K1 == 2 && G::P == 1 && (G::LW + G::N) * (int)sizeof(W) <= 160 * 1024)
        return 3;
    return 2;
}
template <int LOGN, typename W, int K1, int MODE = 0>
constexpr int ext_extra_words() {
    constexpr int st = ext_stash<LOGN, W, K1, MODE>();
    return st == 1 ? Geo<LOGN>::P * K1 * Geo<LOGN>::N : (st == 3 ? Geo<LOGN>::N : 0);
}

template <int LOGN, typename W, int K1, int MODE = 0>
constexpr int ext_occ() {
    constexpr int extra = ext_extra_words<LOGN, W, K1, MODE>();
    return Geo<LOGN>::template occ_waves<W, extra>();
}

struct DmArgs {
    const uint64_t *src;    // MODE 0: glwe [batch][K1][N]; 1: ct [batch][3][N]; 2: acc [batch][K1][N]
    const uint64_t *key;    // prepared key rows (NTT x R): 0/2: [K1*L][K1][N]; 1: [L][2][N] (a_l, b_l)
    uint64_t *out;          // [batch][K1][N]
    size_t batch;
    int level, base_log;
    const uint64_t *lwe_a;  // MODE 2: LWE masks [batch][lwe_dim]
    uint64_t lwe_q;
    uint32_t lwe_dim, step;
    const uint64_t *src2;   // MODE 3: ct1 [batch][K1][N] (src = ct0)
};

// Relinearisation with 32-bit words loads the row's whole key (low words of
// the prepared u64 rows; canonical residues < q < 2^32) after the digit
// transform in one batch instead of two coefficients at a time: 8.14 vs 8.30 ms
// per 16,384 ciphertexts (round 5).  Issued before the transform (kept in
// flight across it) it spills 28 VGPRs and takes 10.4 ms.
#ifndef FHE_RELIN_KPF
#define FHE_RELIN_KPF 1
#endif
template <int LOGN, typename W, int K1, bool LAZY, int MODE>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (ext_occ<LOGN, W, K1, MODE>()))
k_dmac(DmArgs D, NttArgs<W> A) {
    using G = Geo<LOGN>;
    constexpr int STASH = ext_stash<LOGN, W, K1, MODE>();
    constexpr int KPF = (MODE == 1 && STASH == 3 && sizeof(W) == 4) ? FHE_RELIN_KPF : 0;
    constexpr int NIN = MODE == 1 ? 3 : K1;  // source polynomials per ciphertext
    __shared__ W lds_all[G::P * G::LW + ext_extra_words<LOGN, W, K1, MODE>()];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = wg_poly<G>();
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < D.batch;
    if (G::P == 1 && !valid) return;  // whole workgroup: no barrier is skipped
    W *lds = lds_all + pl * G::LW;
    uint64_t *orow = D.out + poly * K1 * G::N;
    const uint64_t *srow = D.src + (valid ? poly : 0) * NIN * G::N;
    // accumulator j of this ciphertext: LDS, or row j of the output
    // (STASH 3: j = 0 only; accumulator 1 is racc)
    auto acc = [&](int j) -> W * {
        if constexpr (STASH == 1) return lds_all + G::P * G::LW + (pl * K1 + j) * G::N;
        else if constexpr (STASH == 3) return lds_all + G::LW;
        else return reinterpret_cast<W *>(orow + (size_t)j * G::N);
    };
    W racc[STASH == 3 ? G::E : 1];
    uint64_t craw[STASH == 3 ? G::E : 1];  // c2 words at this lane's pass-0 positions
    if constexpr (STASH == 3) {
#pragma unroll
        for (int t = 0; t < G::E; ++t) craw[t] = valid ? srow[2 * G::N + tau + cbrv(t, G::LOGE) * G::T] : 0;
    }

    const int level = D.level;
    const uint64_t base = 1ull << D.base_log, mask = base - 1, half = base / 2;
    const uint64_t q = A.q64, mu = A.mu64, lim = (uint64_t)A.ar.q2 * 2;
    bool skip = false;   // MODE 2, rot == 0: output = input accumulator
    uint32_t rot = 0;
    if constexpr (MODE == 2) {
        const int32_t r = valid ? rot_amount(D.lwe_a[poly * D.lwe_dim + D.step], G::N, D.lwe_q) : 0;
        skip = r == 0;
        rot = rot_norm(r, G::N);
        if (G::P == 1 && skip) {  // workgroup-uniform: copy and leave
            for (uint32_t i = threadIdx.x; i < (uint32_t)(K1 * G::N); i += G::THREADS) orow[i] = srow[i];
            return;
        }
    }
    const int rows = MODE == 1 ? level : K1 * level;
    for (int r = 0; r < rows; ++r) {
        // opaque per-row copy of the lane index: keeps the (loop-invariant)
        // address arithmetic inside the loop instead of 100+ hoisted VGPRs
        uint32_t tr = tau;
        asm volatile("" : "+v"(tr));
        const int i = MODE == 1 ? 2 : r / level, l = MODE == 1 ? r : r % level;
        const uint32_t shift = MODE == 1 ? uint32_t(l) * uint32_t(D.base_log)
                                         : uint32_t(level - 1 - l) * uint32_t(D.base_log);
        const uint64_t *src = srow + (size_t)i * G::N;
        const uint64_t *src2 = MODE == 3 ? D.src2 + ((valid ? poly : 0) * K1 + i) * G::N : nullptr;
        if (r > 0 && G::NP > 1) __syncthreads();
        W v[G::E];
        Tw<W> t0[PassTw<LOGN, 0>::COUNT];
        load_tw<LOGN, 0>(tr, A.twf, t0);
        load_coeffs<G::E>(v, lim, q, mu, [&](int t) -> uint64_t {
            const uint32_t p = tr + cbrv(t, G::LOGE) * G::T;
            if (!valid || skip) return 0;
            uint64_t c;
            if constexpr (STASH == 3) c = craw[STASH == 3 ? t : 0];
            else if constexpr (MODE == 2) c = subq(red_q(rotated_at(src, p, rot, G::N, q, mu), q, mu), red_q(src[p], q, mu), q);
            else if constexpr (MODE == 3) c = subq(red_q(src2[p], q, mu), red_q(src[p], q, mu), q);
            else c = src[p];
            uint64_t d = (c >> shift) & mask;
            if constexpr (MODE != 1) {
                if (d > half) d = red_q(q - (base - d), q, mu);
            }
            return d;
        });
        // KPF: the row's key words loaded at once, before (2) or after (1)
        // the digit transform
        uint32_t kw[KPF ? G::E : 1][2];
        auto load_keys = [&]() {
            const uint32_t *g32 = reinterpret_cast<const uint32_t *>(D.key + (size_t)r * K1 * G::N);
#pragma unroll
            for (int e = 0; e < (KPF ? G::E : 1); ++e)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    kw[e][j] = g32[2 * ((size_t)(1 - j) * G::N + gidx<LOGN, G::NP - 1>(tr, e))];
        };
        if constexpr (KPF == 2) load_keys();
        fwd_pass<LOGN, 0, LAZY>(v, t0, A.ar);
        fwd_rest<LOGN, 1, LAZY, kPfSingle>(lds, v, tr, A.twf, A.ar);
        if constexpr (KPF == 1) load_keys();
        if (!valid) continue;
        if constexpr (KPF != 0) {
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const uint32_t gi = gidx<LOGN, G::NP - 1>(tr, e);
                const W p0 = r == 0 ? W(0) : acc(0)[gi];
                const W p1 = r == 0 ? W(0) : racc[STASH == 3 ? e : 0];
                acc(0)[gi] = A.ar.red2q(p0 + A.ar.mont(v[e], (W)kw[e][0]));
                racc[STASH == 3 ? e : 0] = A.ar.red2q(p1 + A.ar.mont(v[e], (W)kw[e][1]));
            }
            continue;
        }
        const uint64_t *g = D.key + (size_t)r * K1 * G::N;
        // chunks of 2 coefficients: all key + accumulator loads of the row in
        // flight at once would not fit the register budget
#pragma unroll
        for (int c0 = 0; c0 < G::E; c0 += 2) {
            uint64_t kv[2][K1];
            W pv[2][K1];
#pragma unroll
            for (int e = 0; e < 2; ++e)
#pragma unroll
                for (int j = 0; j < K1; ++j) {
                    const uint32_t gi = gidx<LOGN, G::NP - 1>(tr, c0 + e);
                    const int kj = MODE == 1 ? 1 - j : j;  // relin: c0' uses b_l, c1' uses a_l
                    kv[e][j] = g[(size_t)kj * G::N + gi];
                    if (STASH == 3 && j > 0) pv[e][j] = r == 0 ? W(0) : racc[STASH == 3 ? c0 + e : 0];
                    else pv[e][j] = r == 0 ? W(0) : acc(j)[gi];
                }
#pragma unroll
            for (int e = 0; e < 2; ++e)
#pragma unroll
                for (int j = 0; j < K1; ++j) {
                    // raw output (< R) times a canonical key: valid Montgomery pair
                    const W m = A.ar.mont(v[c0 + e], (W)kv[e][j]);
                    if (STASH == 3 && j > 0) racc[STASH == 3 ? c0 + e : 0] = A.ar.red2q(pv[e][j] + m);
                    else acc(j)[gidx<LOGN, G::NP - 1>(tr, c0 + e)] = A.ar.red2q(pv[e][j] + m);
                }
        }
    }
    auto out_row = [&](int j) {
        if (G::NP > 1) __syncthreads();
        uint32_t tr = tau;
        asm volatile("" : "+v"(tr));
        W v[G::E];
        if (STASH == 3 && j > 0) {
#pragma unroll
            for (int e = 0; e < G::E; ++e) v[e] = valid ? racc[STASH == 3 ? e : 0] : W(0);
        } else {
#pragma unroll
            for (int e = 0; e < G::E; ++e) v[e] = valid ? acc(j)[gidx<LOGN, G::NP - 1>(tr, e)] : W(0);
        }
        if constexpr (STASH == 2) {
            if (G::NP > 1) __syncthreads();  // every stash read of row j precedes its final stores
        }
        // MODE 1: + c_j (mod_add of encryption.cpp:953/958); MODE 2: + acc_j
        // (cmux's add_glwe_inplace, :537), or acc_j itself when skipped.
        const uint64_t *addend = srow + (size_t)j * G::N;
        auto fin = [&](uint32_t gi, uint64_t x) -> uint64_t {
            if constexpr (MODE == 0) return x;
            else {
                if (!valid) return 0;
                const uint64_t a = addend[gi];
                if (MODE == 2 && skip) return a;
                return addq(x, red_q(a, q, mu), q);
            }
        };
        inv_poly_from_regs<LOGN>(lds, v, tr, orow + (size_t)j * G::N, valid, A, A.ninv, 0, fin);
    };
    if constexpr (STASH == 3) {  // unrolled: racc is indexed by the row
#pragma unroll
        for (int j = 0; j < K1; ++j) out_row(j);
    } else {
#pragma nounroll
        for (int j = 0; j < K1; ++j) out_row(j);
    }
}

// Relinearisation at two workgroups per CU (lab build
// FHE_RELIN2=1, measured SLOWER and not dispatched: per 16,384 ciphertexts
// 9.11 ms with accumulator 1 in VGPRs (6 VGPRs spilled, FHE_RELIN2_ACC1G=0)
// and 10.11 ms with both accumulators in the output rows (spill-free), against
// 8.19 ms for k_dmac MODE 1; parity green, profiles/r6d).  k_dmac
// MODE 1 keeps accumulator 0 in LDS beside the 64 KiB exchange (133 KB: one
// 16-wave workgroup per CU).  Here one 512-thread workgroup per ciphertext
// holds 32 coefficients per thread; accumulator 1 stays in VGPRs and
// accumulator 0 lives in the ciphertext's own output row 0, used as [N] u32
// scratch (read-modify-write of the thread's own positions, L2-resident, no
// synchronisation) until that row's final stores -- so the LDS is the
// exchange alone (64 KiB) and two workgroups share a CU.  c2 is re-read per
// digit level (L2 / MALL) instead of held in VGPRs.  Same digit map,
// Montgomery MAC, red2q accumulation and N^-1 inverse + c_j epilogue as
// k_dmac MODE 1: bit-identical outputs.
#ifndef FHE_RELIN2
#define FHE_RELIN2 0
#endif
#ifndef FHE_RELIN2_MC
#define FHE_RELIN2_MC 2
#endif
#ifndef FHE_RELIN2_PF
#define FHE_RELIN2_PF 1
#endif
#ifndef FHE_RELIN2_ACC1G
#define FHE_RELIN2_ACC1G 0
#endif
constexpr int kRelin2Key = gk(14, 5);
__device__ __forceinline__ uint32_t bload32(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0);
}
__device__ __forceinline__ void bstore32(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so, uint32_t x) {
    __builtin_amdgcn_raw_buffer_store_b32(x, r, vo, so, 0);
}
template <int K>
__global__ void __launch_bounds__(Geo<K>::THREADS, Geo<K>::template occ_waves<uint32_t>())
k_relin2(DmArgs D, NttArgs<uint32_t> A) {
    using G = Geo<K>;
    using W = uint32_t;
    static_assert(G::P == 1 && G::E == 32, "one ciphertext per workgroup, 32 coefficients per thread");
    constexpr int N = G::N, E = G::E, MC = FHE_RELIN2_MC, NC = E / MC;
    __shared__ W lds[lds_elems<K, W>()];
    const TidSource lane;
    const size_t ct = blockIdx.x;
    if (ct >= D.batch) return;  // whole workgroup
    const uint64_t *srow = D.src + ct * 3 * N;
    uint64_t *orow = D.out + ct * 2 * N;
    const auto racc0 = brsrc(orow);  // accumulator 0: row 0 as u32 words at 4 gi
    const auto racc1 = brsrc(orow + N);  // FHE_RELIN2_ACC1G: accumulator 1 likewise in row 1
    const int level = D.level;
    const uint64_t mask = (1ull << D.base_log) - 1;
    const uint64_t q = A.q64, mu = A.mu64, lim = (uint64_t)A.ar.q2 * 2;
    W racc[FHE_RELIN2_ACC1G ? 1 : E];
    for (int l = 0; l < level; ++l) {
        const uint32_t tr = lane();
        const uint32_t shift = uint32_t(l) * uint32_t(D.base_log);
        W v[E];
        {
            const auto rs = brsrc(srow + 2 * N);
            // (SlowRed: the 32-bit-friendly exact reduction of out-of-range
            // digits; mod64_slow's 64-bit Barrett step spills here)
            load_coeffs_chunked<E, 8, 1>(v, lim, SlowRed<W>{A}, [&](int t) -> uint64_t {
                return (bload(rs, tr * 8u, cbrv(t, G::LOGE) * G::T * 8u) >> shift) & mask;
            });
        }
        if (l > 0) __syncthreads();  // the previous transform's last exchange reads precede these stores
        {
            Tw<W> t0[PassTw<K, 0>::COUNT];
            load_tw<K, 0>(tr, A.twf, t0);
            fwd_pass<K, 0, false>(v, t0, A.ar);
        }
        fwd_rest<K, 1, false, FHE_RELIN2_PF>(lds, v, tr, A.twf, A.ar);
        // key low words (canonical prepared residues < q < 2^32): c0' takes
        // b_l (row 1), c1' a_l (row 0); chunk c + 1 in flight while chunk c
        // is consumed
        const auto rb = brsrc(D.key + ((size_t)l * 2 + 1) * N), ra = brsrc(D.key + (size_t)l * 2 * N);
        const uint32_t vo = LastIO<K>::vo(lane());
        // one chunk in flight (nk*) while the previous one (ck*) is consumed
        uint32_t nkb[MC], nka[MC], na0[MC], na1[MC];
        auto issue = [&](int c) {
#pragma unroll
            for (int i = 0; i < MC; ++i) {
                const uint32_t so = LastIO<K>::so(c * MC + i);
                nkb[i] = bload32(rb, vo, so);
                nka[i] = bload32(ra, vo, so);
                if (l > 0) na0[i] = bload32(racc0, vo / 2u, so / 2u);
                if (FHE_RELIN2_ACC1G && l > 0) na1[i] = bload32(racc1, vo / 2u, so / 2u);
            }
        };
        issue(0);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint32_t ckb[MC], cka[MC], ca0[MC], ca1[MC];
#pragma unroll
            for (int i = 0; i < MC; ++i) ckb[i] = nkb[i], cka[i] = nka[i], ca0[i] = na0[i], ca1[i] = na1[i];
            if (c + 1 < NC) issue(c + 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < MC; ++i) {
                const int e = c * MC + i;
                const uint32_t so = LastIO<K>::so(e);
                // raw output (< 4q) times a canonical key: valid Montgomery pair
                const W m0 = A.ar.mont(v[e], ckb[i]), m1 = A.ar.mont(v[e], cka[i]);
                bstore32(racc0, vo / 2u, so / 2u, A.ar.red2q((l > 0 ? ca0[i] : W(0)) + m0));
                if constexpr (FHE_RELIN2_ACC1G)
                    bstore32(racc1, vo / 2u, so / 2u, A.ar.red2q((l > 0 ? ca1[i] : W(0)) + m1));
                else
                    racc[FHE_RELIN2_ACC1G ? 0 : e] = A.ar.red2q((l > 0 ? racc[FHE_RELIN2_ACC1G ? 0 : e] : W(0)) + m1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // c_j' = inv(acc_j) + c_j (encryption.cpp:953/958), row 0 first: its
    // scratch words are read into registers before the inverse's first
    // exchange barrier, its final stores come after the last one
    auto fin = [&](int j) {
        return [&, j](uint32_t gi, uint64_t x) -> uint64_t { return addq(x, red_q(srow[(size_t)j * N + gi], q, mu), q); };
    };
    __syncthreads();
    {
        const uint32_t ti = lane();
        const uint32_t vo = LastIO<K>::vo(ti);
        W v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = bload32(racc0, vo / 2u, LastIO<K>::so(e) / 2u);
        inv_poly_from_regs<K, FHE_RELIN2_PF>(lds, v, ti, orow, true, A, A.ninv, 0, fin(0));
    }
    __syncthreads();
    const uint32_t ti = lane();
    if constexpr (FHE_RELIN2_ACC1G) {
        const uint32_t vo = LastIO<K>::vo(ti);
        W v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = bload32(racc1, vo / 2u, LastIO<K>::so(e) / 2u);
        inv_poly_from_regs<K, FHE_RELIN2_PF>(lds, v, ti, orow + N, true, A, A.ninv, 0, fin(1));
    } else {
        inv_poly_from_regs<K, FHE_RELIN2_PF>(lds, racc, ti, orow + N, true, A, A.ninv, 0, fin(1));
    }
}

// External product with one decomposition level (level == 1, K1 == 2) for
// one polynomial per workgroup: the two digit polynomials are transformed in
// lockstep (shared twiddles), the key MAC turns (X0, X1) into the two
// NTT-domain outputs in place, and both inverses run in lockstep -- nothing
// is parked in HBM (k_dmac's output-row stash read and wrote every
// accumulator once per row: 2.2x the algorithmic traffic at N = 16384).
#ifndef FHE_EXT2_PF
#define FHE_EXT2_PF 0
#endif
#ifndef FHE_EXT2
#define FHE_EXT2 1
#endif
template <int LOGN, typename W>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, Geo<LOGN>::template occ_waves<W>())
k_extprod2(DmArgs D, NttArgs<W> A) {
    using G = Geo<LOGN>;
    static_assert(G::P == 1, "one ciphertext per workgroup");
    constexpr int PF = FHE_EXT2_PF;
    __shared__ W lds[G::LW];
    const TidSource tid;  // lane index per phase, not held across phases
    const uint32_t tau = tid();
    const size_t poly = blockIdx.x;
    if (poly >= D.batch) return;
    const uint64_t *srow = D.src + poly * 2 * G::N;
    uint64_t *orow = D.out + poly * 2 * G::N;
    const uint64_t base = 1ull << D.base_log, mask = base - 1, half = base / 2;
    const uint64_t q = A.q64, mu = A.mu64, lim = (uint64_t)A.ar.q2 * 2;
    W v0[G::E], v1[G::E];
    Tw<W> t0[PassTw<LOGN, 0>::COUNT];
    load_tw<LOGN, 0>(tau, A.twf, t0);
    // digit (level 0 of 1: shift 0) of glwe row i, signed (decompose_polynomial)
    auto digit = [&](const uint64_t *src, int t) -> uint64_t {
        uint64_t d = src[tau + cbrv(t, G::LOGE) * G::T] & mask;
        if (d > half) d = red_q(q - (base - d), q, mu);
        return d;
    };
    load_coeffs<G::E>(v0, lim, q, mu, [&](int t) { return digit(srow, t); });
    load_coeffs<G::E>(v1, lim, q, mu, [&](int t) { return digit(srow + G::N, t); });
    fwd_pass<LOGN, 0, false>(v0, t0, A.ar);
    fwd_pass<LOGN, 0, false>(v1, t0, A.ar);
    fwd_rest2<LOGN, 1, false, PF>(lds, v0, v1, tau, A.twf, A.ar);
    // (o0, o1) = (X0 G00 + X1 G10, X0 G01 + X1 G11); raw outputs (< 4q) times
    // canonical prepared keys: valid Montgomery pairs
    const uint64_t *g = D.key;
    const uint32_t tm = tid();
#pragma unroll
    for (int e0 = 0; e0 < G::E; e0 += 2) {
        uint64_t k[2][4];
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int j = 0; j < 4; ++j) k[e][j] = g[(size_t)j * G::N + gidx<LOGN, G::NP - 1>(tm, e0 + e)];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const W x0 = v0[e0 + e], x1 = v1[e0 + e];
            v0[e0 + e] = A.ar.red2q(A.ar.mont(x0, (W)k[e][0]) + A.ar.mont(x1, (W)k[e][2]));
            v1[e0 + e] = A.ar.red2q(A.ar.mont(x0, (W)k[e][1]) + A.ar.mont(x1, (W)k[e][3]));
        }
    }
    __syncthreads();
    const uint32_t ti = tid();
    inv_poly2<LOGN, PF>(lds, v0, v1, ti, orow, orow + G::N, A, A.ninv);
}

// Relinearisation takes k_dmac MODE 1.  Two 32-coefficient-per-thread
// kernels (c2 low words and accumulator 1 in VGPRs, accumulator 0 in LDS; 8
// waves per CU) measured slower on MI355X: single digit transforms 9.03 vs
// 8.29 ms per 16,384 ciphertexts (round 4), digit levels in lockstep pairs
// 4.67 vs 4.27 ms per 8,192 (round 5) -- the 16 waves of MODE 1 hide more of
// the exchange barriers than the shorter transforms save.

// FHE_EXT_ACC=0: multi-level external products at N = 16384 take k_dmac
// (lab A/B against ntt_ext2.hip).
#ifndef FHE_EXT_ACC
#define FHE_EXT_ACC 1
#endif
template <int LOGN, typename W, int MODE>
static hipError_t dmac_one(const NttArgs<W> &A, hipStream_t s, int k1, const DmArgs &D) {
    using G = Geo<LOGN>;
    const size_t blocks = (D.batch + G::P - 1) / G::P;
    if (k1 != 2) return hipErrorInvalidValue;
    if constexpr (MODE == 0 && G::P == 1 && FHE_EXT2 && sizeof(W) == 8 && LOGN >= 12) {
        if (D.level == 1) {
            if constexpr (LOGN == 14) {
                // a sparse prime (ntt_core.hpp gk_sparse): C5 (23, 1) 8.1 -> 7.7 ms
                // per 16,384 (round 5)
                if (A.ar.sp == 1 || A.ar.sp == 2) {
                    if (A.ar.sp == 1)
                        hipLaunchKernelGGL((k_extprod2<gk_sparse(LOGN, 1), W>), dim3((unsigned)D.batch),
                                           dim3(G::THREADS), 0, s, D, A);
                    else
                        hipLaunchKernelGGL((k_extprod2<gk_sparse(LOGN, 2), W>), dim3((unsigned)D.batch),
                                           dim3(G::THREADS), 0, s, D, A);
                    return hipGetLastError();
                }
            }
            hipLaunchKernelGGL((k_extprod2<LOGN, W>), dim3((unsigned)D.batch), dim3(G::THREADS), 0, s, D, A);
            return hipGetLastError();
        }
    }
    if constexpr (FHE_RELIN2 && MODE == 1 && LOGN == 14 && sizeof(W) == 4) {
        hipLaunchKernelGGL((k_relin2<kRelin2Key>), dim3((unsigned)D.batch), dim3(Geo<kRelin2Key>::THREADS), 0, s, D, A);
        return hipGetLastError();
    }
    // (unit twiddles, ntt_core.hpp gk_compat, measured 0 to +0.4 % here and in
    // the external-product kernels, round 5: not instantiated)
    hipLaunchKernelGGL((k_dmac<LOGN, W, 2, false, MODE>), dim3(blocks), dim3(G::THREADS), 0, s, D, A);
    return hipGetLastError();
}

template <typename W, int MODE>
static hipError_t dmac_dispatch(const Plan &p, const NttArgs<W> &A, int k1, const DmArgs &D) {
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return dmac_one<L, W, MODE>(A, p.stream, k1, D);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}

template <int MODE>
static hipError_t dmac(const Plan &p, int k1, const DmArgs &D) {
    if (D.batch == 0) return hipSuccess;
    if (p.word == 32)
        return dmac_dispatch<uint32_t, MODE>(p, p.a32, k1, D);
    return dmac_dispatch<uint64_t, MODE>(p, p.a64, k1, D);
}

hipError_t launch_extprod(const Plan &p, int k1, int level, int base_log, const uint64_t *glwe,
                          const uint64_t *ggsw, uint64_t *out, size_t batch) {
    if (FHE_EXT_ACC && extprod_acc_supported(p, k1, level, base_log))
        return launch_extprod_acc(p, level, base_log, glwe, ggsw, out, batch);
    DmArgs D{glwe, ggsw, out, batch, level, base_log, nullptr, 0, 0, 0, nullptr};
    return dmac<0>(p, k1, D);
}

hipError_t launch_relin(const Plan &p, int level, int base_log, const uint64_t *ct3, const uint64_t *rlk,
                        uint64_t *out, size_t batch) {
    DmArgs D{ct3, rlk, out, batch, level, base_log, nullptr, 0, 0, 0, nullptr};
    return dmac<1>(p, 2, D);
}

hipError_t launch_cmux_rotate(const Plan &p, int k1, int level, int base_log, const uint64_t *acc_in,
                              const uint64_t *ggsw, uint64_t *acc_out, size_t batch, const uint64_t *lwe_a,
                              uint32_t lwe_dim, uint32_t step, uint64_t lwe_q) {
    DmArgs D{acc_in, ggsw, acc_out, batch, level, base_log, lwe_a, lwe_q, lwe_dim, step, nullptr};
    return dmac<2>(p, k1, D);
}

hipError_t launch_cmux(const Plan &p, int k1, int level, int base_log, const uint64_t *ggsw, const uint64_t *ct0,
                       const uint64_t *ct1, uint64_t *out, size_t batch) {
    DmArgs D{ct0, ggsw, out, batch, level, base_log, nullptr, 0, 0, 0, ct1};
    return dmac<3>(p, k1, D);
}

}  // namespace FHE_NS
