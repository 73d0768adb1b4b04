// ntt_ext.hip -- TFHE external product (BootstrapEngine::external_product,
// bootstrap_engine.cpp:431-518) for a batch of GLWE ciphertexts against one
// GGSW key.
//
// The reference computes, for each decomposition row r (mask polynomials
// first, then the body; digit level inner, decompose_polynomial :152-185)
// and each output component j:  res_j = mod_add(res_j,
//   inv( fwd(decomp_r) (.) fwd(ggsw[r][j]) ))
// i.e. (k+1)L + 2(k+1)^2 L transforms.  Because every intermediate is a
// canonical residue and the inverse transform is linear over Z_q,
//   sum_r inv(X_r) == inv(sum_r X_r)   (bit-exact),
// so here: the GGSW is transformed once (fhe_ggsw_prepare, kept in NTT +
// Montgomery form), every digit polynomial is decomposed on its HBM load,
// transformed in registers/LDS, multiplied into (k+1) NTT-domain
// accumulators held in VGPRs, and only (k+1) inverse transforms run at the
// end -- (k+1)L + (k+1) transforms, one kernel, one HBM pass over the GLWE.
#include "fhe_internal.hpp"

namespace FHE_NS {

// Where the (k+1) NTT-domain accumulators live between rows: 1 = a second
// LDS region, 2 = the ciphertext's own output rows in HBM (read-modify-write
// of the thread's own positions; no synchronisation needed).  Holding them
// in VGPRs spilled 300-800 B/lane.
template <int LOGN, typename W, int K1>
constexpr int ext_stash() {
    using G = Geo<LOGN>;
    return G::P * (G::LW + K1 * G::N) * (int)sizeof(W) <= 160 * 1024 ? 1 : 2;
}
template <int LOGN, typename W, int K1>
constexpr int ext_extra_words() {
    return ext_stash<LOGN, W, K1>() == 1 ? Geo<LOGN>::P * K1 * Geo<LOGN>::N : 0;
}

template <int LOGN, typename W, int K1>
constexpr int ext_occ() {
    constexpr int extra = ext_extra_words<LOGN, W, K1>();
    return Geo<LOGN>::template occ_waves<W, extra>();
}

template <int LOGN, typename W, bool NEGA, int K1, bool LAZY>
__global__ void __launch_bounds__(Geo<LOGN>::THREADS, (ext_occ<LOGN, W, K1>()))
k_extprod(const uint64_t *__restrict__ glwe, const uint64_t *__restrict__ ggsw, uint64_t *out,
          size_t batch, int level, int base_log, NttArgs<W> A) {
    using G = Geo<LOGN>;
    constexpr int STASH = ext_stash<LOGN, W, K1>();
    __shared__ W lds_all[G::P * G::LW + ext_extra_words<LOGN, W, K1>()];
    const uint32_t tau = threadIdx.x & (G::T - 1), pl = threadIdx.x >> G::LOGT;
    const size_t poly = (size_t)blockIdx.x * G::P + pl;
    const bool valid = poly < batch;
    if (G::P == 1 && !valid) return;  // whole workgroup: no barrier is skipped
    W *lds = lds_all + pl * G::LW;
    uint64_t *orow = out + poly * K1 * G::N;
    // accumulator j of this ciphertext: LDS, or row j of the output
    auto acc = [&](int j) -> W * {
        if constexpr (STASH == 1) return lds_all + G::P * G::LW + (pl * K1 + j) * G::N;
        else return reinterpret_cast<W *>(orow + (size_t)j * G::N);
    };

    const uint64_t base = 1ull << base_log, mask = base - 1, half = base / 2;
    const uint64_t q = A.q64, lim = (uint64_t)A.ar.q2 * 2;
    const int rows = K1 * level;
    for (int r = 0; r < rows; ++r) {
        // opaque per-row copy of the lane index: keeps the (loop-invariant)
        // address arithmetic inside the loop instead of 100+ hoisted VGPRs
        uint32_t tr = tau;
        asm volatile("" : "+v"(tr));
        const int i = r / level, l = r % level;
        const uint32_t shift = uint32_t(level - 1 - l) * uint32_t(base_log);
        const uint64_t *src = glwe + (poly * K1 + i) * G::N;
        if (r > 0 && G::NP > 1) __syncthreads();
        W v[G::E];
        Tw<W> t0[PassTw<LOGN, 0>::COUNT];
        load_tw<LOGN, 0>(tr, A.twf, t0);
        load_coeffs<G::E>(v, lim, q, A.mu64, [&](int t) -> uint64_t {
            const uint64_t c = valid ? src[tr + cbrv(t, G::LOGE) * G::T] : 0;
            uint64_t d = (c >> shift) & mask;
            if (d > half) {
                d = q - (base - d);
                if (d >= q) d = mod64_slow(d, q, A.mu64);
            }
            return d;
        });
        if constexpr (NEGA) {
#pragma unroll
            for (int t = 0; t < G::E; ++t) v[t] = A.ar.shoup(v[t], A.twist[tr + cbrv(t, G::LOGE) * G::T]);
        }
        fwd_pass<LOGN, 0, LAZY>(v, t0, A.ar);
        fwd_rest<LOGN, 1, LAZY, kPfSingle>(lds, v, tr, A.twf, A.ar);
        if (!valid) continue;
        const uint64_t *g = ggsw + (size_t)r * K1 * G::N;
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
                    kv[e][j] = g[(size_t)j * G::N + gi];
                    pv[e][j] = r == 0 ? W(0) : acc(j)[gi];
                }
#pragma unroll
            for (int e = 0; e < 2; ++e)
#pragma unroll
                for (int j = 0; j < K1; ++j) {
                    // raw output (< R) times a canonical key: valid Montgomery pair
                    const W m = A.ar.mont(v[c0 + e], (W)kv[e][j]);
                    acc(j)[gidx<LOGN, G::NP - 1>(tr, c0 + e)] = A.ar.red2q(pv[e][j] + m);
                }
        }
    }
#pragma nounroll
    for (int j = 0; j < K1; ++j) {
        if (G::NP > 1) __syncthreads();
        uint32_t tr = tau;
        asm volatile("" : "+v"(tr));
        W v[G::E];
#pragma unroll
        for (int e = 0; e < G::E; ++e) v[e] = valid ? acc(j)[gidx<LOGN, G::NP - 1>(tr, e)] : W(0);
        if constexpr (STASH == 2) {
            if (G::NP > 1) __syncthreads();  // every stash read of row j precedes its final stores
        }
        inv_poly_from_regs<LOGN, NEGA>(lds, v, tr, orow + (size_t)j * G::N, valid, A, A.ninv, A.untwist);
    }
}

template <int LOGN, typename W, bool NEGA>
static hipError_t ext_one(const NttArgs<W> &A, hipStream_t s, int k1, int level, int base_log, const uint64_t *glwe,
                          const uint64_t *ggsw, uint64_t *out, size_t batch) {
    using G = Geo<LOGN>;
    const size_t blocks = (batch + G::P - 1) / G::P;
    if (k1 != 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_extprod<LOGN, W, NEGA, 2, false>), dim3(blocks), dim3(G::THREADS), 0, s, glwe, ggsw, out,
                       batch, level, base_log, A);
    return hipGetLastError();
}

template <typename W, bool NEGA>
static hipError_t ext_dispatch(const Plan &p, const NttArgs<W> &A, int k1, int level, int base_log,
                               const uint64_t *glwe, const uint64_t *ggsw, uint64_t *out, size_t batch) {
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return ext_one<L, W, NEGA>(A, p.stream, k1, level, base_log, glwe, ggsw, out, batch);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_extprod(const Plan &p, int k1, int level, int base_log, const uint64_t *glwe,
                          const uint64_t *ggsw, uint64_t *out, size_t batch) {
    if (batch == 0) return hipSuccess;
    if (p.word == 32)
        return p.nega ? ext_dispatch<uint32_t, true>(p, p.a32, k1, level, base_log, glwe, ggsw, out, batch)
                      : ext_dispatch<uint32_t, false>(p, p.a32, k1, level, base_log, glwe, ggsw, out, batch);
    return p.nega ? ext_dispatch<uint64_t, true>(p, p.a64, k1, level, base_log, glwe, ggsw, out, batch)
                  : ext_dispatch<uint64_t, false>(p, p.a64, k1, level, base_log, glwe, ggsw, out, batch);
}

}  // namespace FHE_NS
