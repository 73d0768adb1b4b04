// ntt_ext2.hip -- TFHE external product with several decomposition levels at
// N = 16384 and 64-bit words (config C5, (B, L) = (15, 2);
// BootstrapEngine::external_product, bootstrap_engine.cpp:431-518):
//   for each GLWE row i (mask first, then body) and digit level l (MSB digit
//   first, decompose_polynomial :152-185) and each output component j:
//     res_j = mod_add(res_j, inv( fwd(decomp_{i,l}) (.) fwd(ggsw[i L + l][j]) )).
//
// k_dmac (ntt_ext.hip) runs this shape at 16 coefficients per thread with
// the two NTT-domain accumulators parked in the output rows between rows
// (a read-modify-write of 2 x 8N bytes per digit row: 5.6x the algorithmic
// traffic at L = 2).  Here one workgroup of 512 threads owns one ciphertext
// and every thread owns 32 coefficients:
//   * both accumulators stay in VGPRs for the whole kernel (2 x 32 u64 =
//     128 VGPRs; one workgroup per CU, so 256 VGPRs per lane);
//   * a GLWE row is read from HBM once: its level-0 digits feed the first
//     transform and its level-1 digits wait in LDS as int32 (the signed
//     digit, at the lane's own pass-0 positions: no barrier), levels >= 2
//     (L >= 3) re-read the row;
//   * the transforms use the split 32-bit exchange (64 KiB) and streamed
//     twiddles of the 32-per-thread q62 forward;
//   * the two inverses run in lockstep (inv_poly2) straight from the
//     accumulators into the output rows.
// HBM traffic = the 32 N bytes of the GLWE in and out (the prepared GGSW
// rows, shared by the whole batch, stay in L2).  Same arithmetic as k_dmac
// (digit map, Montgomery MAC against NTT x R keys, red2q accumulation,
// plain N^-1 inverse): bit-identical results.
#ifndef FHE_U64_NOVCC
#define FHE_U64_NOVCC 1
#endif
#ifndef FHE_SPLIT_X64
#define FHE_SPLIT_X64 1
#endif
#ifndef FHE_STREAM_TW2
#define FHE_STREAM_TW2 1
#endif
#ifndef FHE_STREAM_DEPTH
#define FHE_STREAM_DEPTH 1
#endif
#include "fhe_internal.hpp"
#include "lwe_ops.hpp"
#ifndef FHE_EXTACC_MC
#define FHE_EXTACC_MC 4
#endif
// key chunks in flight ahead of their use; issue the first ones in the last pass
#ifndef FHE_EXTACC_PD
#define FHE_EXTACC_PD 1
#endif
#ifndef FHE_EXTACC_HOOK
#define FHE_EXTACC_HOOK 0
#endif
// lab: the 62-bit sparse prime compiled in (ntt_core.hpp gk_sparse), as in
// k_extprod2 for (23, 1): 0.4 % fewer static issue
// cycles, spill-free, but 13.33 vs 13.05 ms per 16,384 at (15, 2) (round 6,
// profiles/r6h): not dispatched
#ifndef FHE_EXTACC_SPARSE
#define FHE_EXTACC_SPARSE 0
#endif

namespace FHE_NS {

constexpr int kExtAccKey = gk(14, 5);

struct ExtAccArgs {
    const uint64_t *glwe;  // [batch][2][N]
    const uint64_t *key;   // [2L][2][N] prepared GGSW rows (NTT x R)
    uint64_t *out;         // [batch][2][N]
    int level, base_log;
};

template <int K>
__global__ void __launch_bounds__(Geo<K>::THREADS, 2) k_extprod_acc(ExtAccArgs D, NttArgs<uint64_t> A) {
    using G = Geo<K>;
    using W = uint64_t;
    static_assert(G::P == 1 && G::E == 32, "one ciphertext per workgroup, 32 coefficients per thread");
    constexpr int N = G::N, E = G::E, MC = FHE_EXTACC_MC;
    __shared__ W lds[lds_elems<K, W>()];
    __shared__ int32_t plane[N];  // level-1 digits of the current row (signed)
    // the lane index is rebuilt per row (TidSource): a VGPR holding it across
    // the loop is the one the 256-VGPR budget lacks
    const TidSource lane_index;
    const size_t ct = blockIdx.x;
    const uint64_t *srow = D.glwe + ct * 2 * N;
    uint64_t *orow = D.out + ct * 2 * N;
    const int level = D.level, B = D.base_log;
    const uint64_t base = 1ull << B, mask = base - 1, half = base / 2;
    const uint64_t q = A.q64, mu = A.mu64, lim = (uint64_t)A.ar.q2 * 2;
    W o0[E], o1[E];
#pragma unroll
    for (int e = 0; e < E; ++e) o0[e] = o1[e] = 0;
    for (int r = 0; r < 2 * level; ++r) {
        const int i = r / level, l = r % level;
        // opaque per-row lane index (keeps the address arithmetic inside the
        // loop instead of hoisted VGPRs)
        const uint32_t tr = lane_index();
        const uint64_t *src = srow + (size_t)i * N;
        const uint32_t shift = uint32_t(level - 1 - l) * uint32_t(B);
        W v[E];
        if (l == 1) {
            load_coeffs_chunked<E, 8, 1>(v, lim, Mod64Red{q, mu}, [&](int t) -> uint64_t {
                const int32_t s = plane[tr + cbrv(t, G::LOGE) * G::T];
                return s < 0 ? red_q(q - (uint64_t)(-(int64_t)s), q, mu) : (uint64_t)s;
            });
        } else {
            const bool park = l == 0 && level >= 2;
            const uint32_t shift1 = park ? uint32_t(level - 2) * uint32_t(B) : 0u;
            const auto rs = brsrc(src);
            load_coeffs_chunked<E, 8, 1>(v, lim, Mod64Red{q, mu}, [&](int t) -> uint64_t {
                const uint32_t p = tr + cbrv(t, G::LOGE) * G::T;
                const uint64_t c = bload(rs, tr * 8u, cbrv(t, G::LOGE) * G::T * 8u);
                if (park) {
                    const uint64_t d1 = (c >> shift1) & mask;
                    plane[p] = d1 > half ? (int32_t)(int64_t)(d1 - base) : (int32_t)d1;
                }
                uint64_t d = (c >> shift) & mask;
                if (d > half) d = red_q(q - (base - d), q, mu);
                return d;
            });
        }
        if (r > 0) __syncthreads();  // the previous transform's last exchange reads precede this one's stores
        {
            Tw<W> t0[PassTw<K, 0>::COUNT];
            stream_begin<K, 0, false, false>(tr, A.twf, t0);
            fwd_pass_stream<K, 0, false, false>(tr, v, t0, A.twf, A.ar);
        }
        // The row's key words stream in chunks of MC coefficients: the first
        // PD chunks are issued inside the transform's last pass (hook), then
        // chunk c + PD before chunk c is consumed -- the L2 round trips
        // overlap instead of following each other (they did, one per chunk).
        const auto rk = brsrc(D.key + (size_t)r * 2 * N);
        constexpr int NC = E / MC, PD = FHE_EXTACC_PD;
        uint64_t k0[E], k1[E];
        auto issue = [&](int c) {
            const uint32_t vo = LastIO<K>::vo(lane_index());
#pragma unroll
            for (int e = c * MC; e < c * MC + MC; ++e) {
                k0[e] = bload<0>(rk, vo, LastIO<K>::so(e));
                k1[e] = bload<0>(rk, vo, LastIO<K>::so(e) + N * 8u);
            }
        };
        auto hook = [&] {
#pragma unroll
            for (int c = 0; c < (FHE_EXTACC_HOOK ? PD : 0) && c < NC; ++c) issue(c);
        };
        fwd_rest<K, 1, false, kPfSingle>(lds, v, tr, A.twf, A.ar, hook);
#pragma unroll
        for (int c = FHE_EXTACC_HOOK ? PD : 0; c < PD && c < NC; ++c) issue(c);
        // raw outputs (< 4q) times canonical prepared keys: valid Montgomery pairs
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c + PD < NC) issue(c + PD);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int e = c * MC; e < c * MC + MC; ++e) {
                const W m0 = A.ar.mont(v[e], (W)k0[e]), m1 = A.ar.mont(v[e], (W)k1[e]);
                o0[e] = A.ar.red2q(o0[e] + m0);
                o1[e] = A.ar.red2q(o1[e] + m1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    __syncthreads();
    const uint32_t ti = lane_index();
    inv_poly2<K, kPfSingle>(lds, o0, o1, ti, orow, orow + N, A, A.ninv);
}

bool extprod_acc_supported(const Plan &p, int k1, int level, int base_log) {
    return p.word == 64 && p.logn == 14 && k1 == 2 && level >= 2 && base_log <= 31;
}

hipError_t launch_extprod_acc(const Plan &p, int level, int base_log, const uint64_t *glwe, const uint64_t *ggsw,
                              uint64_t *out, size_t batch) {
    if (!extprod_acc_supported(p, 2, level, base_log)) return hipErrorInvalidValue;
    if (batch == 0) return hipSuccess;
    const size_t per = (size_t)1 << 30;  // grid.x <= 2^31 - 1 workgroups
    for (size_t b0 = 0; b0 < batch; b0 += per) {
        const size_t nb = batch - b0 < per ? batch - b0 : per;
        ExtAccArgs D{glwe + b0 * 2 * ((size_t)1 << 14), ggsw, out + b0 * 2 * ((size_t)1 << 14), level, base_log};
        if (FHE_EXTACC_SPARSE && p.a64.ar.sp == 1)
            hipLaunchKernelGGL((k_extprod_acc<gk_sparse(kExtAccKey, 1)>), dim3((unsigned)nb),
                               dim3(Geo<kExtAccKey>::THREADS), 0, p.stream, D, p.a64);
        else
            hipLaunchKernelGGL((k_extprod_acc<kExtAccKey>), dim3((unsigned)nb), dim3(Geo<kExtAccKey>::THREADS), 0,
                               p.stream, D, p.a64);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace FHE_NS
