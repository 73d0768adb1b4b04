// ntt_big.hip -- degrees 32768 and 65536 (NTTProcessor accepts N up to
// 65536, ntt_processor.cpp:146-148; the TS round-trip suite runs N = 32768
// with the 62-bit prime, ntt-round-trip.prop.test.ts:43).
//
// A 2^L transform no longer fits one workgroup's LDS (2^L words > 160 KiB at
// u64), so it runs as two HBM passes over a row/column split with
// S = kBigS = 14 and M = L - S (1 or 2):
//
//   forward (bit-reverse, then DIT stages 0..L-1):
//     rows:  block b < 2^M of a polynomial is the bit-reversed subsequence
//            x[o + (i << M)], o = brv_M(b); stages 0..S-1 act on it exactly
//            like a 2^S transform (the stage-major twiddle tables are
//            prefix-compatible: entry 2^s + j is the same for N and 2^S),
//            so the fused one-workgroup kernel of ntt_core.hpp runs on the
//            strided view and writes block b contiguously at b*2^S;
//     cols:  stages S..L-1 pair positions c + 2^S k within column c < 2^S:
//            one thread per column, 2^M values, coalesced across c, with a
//            fused epilogue (canonical / *R / pointwise modmul / the whole
//            polymul middle: fwd(b) col (.) fwd(a) col, then the inverse's
//            column stages).
//   inverse (GS stages L-1..0, bit-reverse, N^-1): column stages first,
//            then the fused 2^S inverse per block, whose bit-reversed store
//            lands at o + (i << M) with the N^-1 (or N^-1 R) fold.
//
// Blocks of one polynomial are mapped to the same XCD, consecutive in
// dispatch order (workgroup i runs on XCD i mod 8), so the strided row reads
// of sibling blocks share that XCD's L2.  The split costs one extra HBM round
// trip per transform; a ctx-owned scratch of kBigChunk polynomials keeps
// every call alias-safe (out may equal any input).
#include "fhe_internal.hpp"

namespace FHE_NS {

constexpr int kBigS = 14;

template <int M>
__device__ __forceinline__ void big_map(size_t &poly, uint32_t &b) {
    const uint32_t i = blockIdx.x, xcd = i & 7u, slot = i >> 3;
    poly = (size_t)(slot >> M) * 8 + xcd;
    b = slot & ((1u << M) - 1);
}
static size_t big_blocks(size_t batch, int M) { return ((batch + 7) / 8) * 8 << M; }

// ---------------------------------------------------------------- rows
template <int M, typename W, bool LAZY>
__global__ void __launch_bounds__(Geo<kBigS>::THREADS, Geo<kBigS>::template occ_waves<W>())
k_big_fwd_rows(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch, NttArgs<W> A) {
    using G = Geo<kBigS>;
    static_assert(G::P == 1, "one polynomial block per workgroup");
    __shared__ W lds[G::LW];
    size_t poly;
    uint32_t b;
    big_map<M>(poly, b);
    const bool valid = poly < batch;
    if (!valid) return;  // whole workgroup (P == 1)
    const uint32_t tau = threadIdx.x, o = cbrv(b, M);
    W v[G::E];
    fwd_poly<kBigS, LAZY>(lds, v, tau, in + (poly << (kBigS + M)) + o, valid, A, M);
    const auto r = brsrc(out + (poly << (kBigS + M)) + ((size_t)b << kBigS));
    const uint32_t vo = LastIO<kBigS>::vo(tau);
#pragma unroll
    for (int e = 0; e < G::E; ++e) bstore(r, vo, LastIO<kBigS>::so(e), (uint64_t)fwd_to_canon<LAZY>(v[e], A));
}

template <int M, typename W, bool MONT>
__global__ void __launch_bounds__(Geo<kBigS>::THREADS, Geo<kBigS>::template occ_waves<W>())
k_big_inv_rows(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t batch, NttArgs<W> A) {
    using G = Geo<kBigS>;
    __shared__ W lds[G::LW];
    size_t poly;
    uint32_t b;
    big_map<M>(poly, b);
    const bool valid = poly < batch;
    if (!valid) return;  // whole workgroup (P == 1)
    const uint32_t tau = threadIdx.x, o = cbrv(b, M);
    const auto r = brsrc(in + (poly << (kBigS + M)) + ((size_t)b << kBigS));
    const uint32_t vo = LastIO<kBigS>::vo(tau);
    W v[G::E];
    load_coeffs_r<G::E>(v, (uint64_t)A.ar.q2, SlowRed<W>{A},
                      [&](int e) -> uint64_t { return bload(r, vo, LastIO<kBigS>::so(e)); });
    inv_poly_from_regs<kBigS>(lds, v, tau, out + (poly << (kBigS + M)) + o, valid, A,
                                    MONT ? A.ninv_r : A.ninv, M);
}

// ---------------------------------------------------------------- columns
// Twiddle of the butterfly pairing column slots (k, k + 2^s) at global
// stage S + s: stage-major index 2^(S+s) + c + 2^S (k mod 2^s).
template <int M, typename W>
__device__ __forceinline__ void col_fwd(W (&y)[1 << M], uint32_t c, const NttArgs<W> &A) {
#pragma unroll
    for (int s = 0; s < M; ++s)
#pragma unroll
        for (int k = 0; k < (1 << M); ++k) {
            if (k & (1 << s)) continue;
            const uint32_t j = c + (uint32_t(k & ((1 << s) - 1)) << kBigS);
            A.ar.ct(y[k], y[k + (1 << s)], A.twf[(1u << (kBigS + s)) + j]);
        }
}
template <int M, typename W>
__device__ __forceinline__ void col_inv(W (&y)[1 << M], uint32_t c, const NttArgs<W> &A) {
#pragma unroll
    for (int s = M - 1; s >= 0; --s)
#pragma unroll
        for (int k = 0; k < (1 << M); ++k) {
            if (k & (1 << s)) continue;
            const uint32_t j = c + (uint32_t(k & ((1 << s) - 1)) << kBigS);
            A.ar.gs(y[k], y[k + (1 << s)], A.twi[(1u << (kBigS + s)) + j]);
        }
}

// EPI 0: canonical; 1: times R (Montgomery form, GGSW preparation);
//     2: (.) w (C3 fwd + modmul, w any u64); 3: polymul middle -- (.) the
//     canonical a-spectrum in w with a Montgomery product (R^-1 folded into
//     the inverse rows' N^-1 R), then the inverse column stages.
template <int M, typename W, int EPI>
__global__ void __launch_bounds__(256) k_big_fwd_cols(const uint64_t *__restrict__ in, const uint64_t *__restrict__ w,
                                                      uint64_t *__restrict__ out, size_t batch, NttArgs<W> A) {
    constexpr int K = 1 << M;
    const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t poly = gid >> kBigS;
    const uint32_t c = (uint32_t)gid & ((1u << kBigS) - 1);
    if (poly >= batch) return;
    const size_t base = (poly << (kBigS + M)) + c;
    W y[K];
#pragma unroll
    for (int k = 0; k < K; ++k) y[k] = W(__builtin_nontemporal_load(in + base + ((size_t)k << kBigS)));  // canonical (rows)
    col_fwd<M>(y, c, A);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        W x = y[k];  // [0, 4q)
        if constexpr (EPI == 0) x = A.ar.canon4(x);
        else if constexpr (EPI == 1) x = A.ar.red1q(A.ar.shoup(x, A.rmod));
        else {
            const uint64_t wr = __builtin_nontemporal_load(w + base + ((size_t)k << kBigS));
            const W wq = load_lazy<W>(wr, A.q64, A.q64, A.mu64);  // canonical
            if constexpr (EPI == 2) x = A.ar.red1q(A.ar.mont(A.ar.shoup(x, A.rmod), wq));  // x R (< 2q) * w R^-1
            else x = A.ar.mont(A.ar.canon4(x), wq);                                          // [0, 2q)
        }
        y[k] = x;
    }
    if constexpr (EPI == 3) col_inv<M>(y, c, A);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const W x = EPI == 3 ? A.ar.red1q(y[k]) : y[k];
        __builtin_nontemporal_store((uint64_t)x, out + base + ((size_t)k << kBigS));
    }
}

template <int M, typename W>
__global__ void __launch_bounds__(256) k_big_inv_cols(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                      size_t batch, NttArgs<W> A) {
    constexpr int K = 1 << M;
    const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t poly = gid >> kBigS;
    const uint32_t c = (uint32_t)gid & ((1u << kBigS) - 1);
    if (poly >= batch) return;
    const size_t base = (poly << (kBigS + M)) + c;
    W y[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        y[k] = load_lazy<W>(__builtin_nontemporal_load(in + base + ((size_t)k << kBigS)), (uint64_t)A.ar.q2, A.q64,
                            A.mu64);  // GS inputs < 2q
    col_inv<M>(y, c, A);
#pragma unroll
    for (int k = 0; k < K; ++k) __builtin_nontemporal_store((uint64_t)A.ar.red1q(y[k]), out + base + ((size_t)k << kBigS));
}

// ---------------------------------------------------------------- host side
template <int M, typename W>
struct Big {
    static hipError_t rows_fwd(const Plan &p, const NttArgs<W> &A, const uint64_t *in, uint64_t *out, size_t nb) {
        const dim3 g(big_blocks(nb, M)), t(Geo<kBigS>::THREADS);
        if constexpr (sizeof(W) == 4)
            if (p.lazy) {
                hipLaunchKernelGGL((k_big_fwd_rows<M, W, true>), g, t, 0, p.stream, in, out, nb, A);
                return hipGetLastError();
            }
        hipLaunchKernelGGL((k_big_fwd_rows<M, W, false>), g, t, 0, p.stream, in, out, nb, A);
        return hipGetLastError();
    }
    template <int EPI>
    static hipError_t cols_fwd(const Plan &p, const NttArgs<W> &A, const uint64_t *in, const uint64_t *w, uint64_t *out,
                               size_t nb) {
        const dim3 g((unsigned)((nb << kBigS) / 256)), t(256);
        hipLaunchKernelGGL((k_big_fwd_cols<M, W, EPI>), g, t, 0, p.stream, in, w, out, nb, A);
        return hipGetLastError();
    }
    static hipError_t cols_inv(const Plan &p, const NttArgs<W> &A, const uint64_t *in, uint64_t *out, size_t nb) {
        const dim3 g((unsigned)((nb << kBigS) / 256)), t(256);
        hipLaunchKernelGGL((k_big_inv_cols<M, W>), g, t, 0, p.stream, in, out, nb, A);
        return hipGetLastError();
    }
    template <bool MONT>
    static hipError_t rows_inv(const Plan &p, const NttArgs<W> &A, const uint64_t *in, uint64_t *out, size_t nb) {
        const dim3 g(big_blocks(nb, M)), t(Geo<kBigS>::THREADS);
        hipLaunchKernelGGL((k_big_inv_rows<M, W, MONT>), g, t, 0, p.stream, in, out, nb, A);
        return hipGetLastError();
    }

    // op: 0 fwd, 1 fwd*R, 2 fwd (.) w, 3 inv, 4 polymul
    static hipError_t run(const Plan &p, const NttArgs<W> &A, int op, const uint64_t *a, const uint64_t *b,
                          uint64_t *c, size_t batch) {
        const size_t N = (size_t)1 << (kBigS + M);
        uint64_t *s0 = p.big_scratch[0], *s1 = p.big_scratch[1];
        if (!s0 || !s1) return hipErrorInvalidValue;
        hipError_t e = hipSuccess;
        for (size_t p0 = 0; p0 < batch && e == hipSuccess; p0 += p.big_chunk) {
            const size_t nb = batch - p0 < p.big_chunk ? batch - p0 : p.big_chunk;
            const uint64_t *ai = a + p0 * N, *bi = b ? b + p0 * N : nullptr;
            uint64_t *ci = c + p0 * N;
            switch (op) {
            case 0: case 1: case 2:
                e = rows_fwd(p, A, ai, s0, nb);
                if (e == hipSuccess)
                    e = op == 0 ? cols_fwd<0>(p, A, s0, nullptr, ci, nb)
                      : op == 1 ? cols_fwd<1>(p, A, s0, nullptr, ci, nb)
                                : cols_fwd<2>(p, A, s0, bi, ci, nb);
                break;
            case 3:
                e = cols_inv(p, A, ai, s0, nb);
                if (e == hipSuccess) e = rows_inv<false>(p, A, s0, ci, nb);
                break;
            default:  // polymul
                e = rows_fwd(p, A, ai, s0, nb);
                if (e == hipSuccess) e = cols_fwd<0>(p, A, s0, nullptr, s0, nb);
                if (e == hipSuccess) e = rows_fwd(p, A, bi, s1, nb);
                if (e == hipSuccess) e = cols_fwd<3>(p, A, s1, s0, s1, nb);
                if (e == hipSuccess) e = rows_inv<true>(p, A, s1, ci, nb);
            }
        }
        return e;
    }
};

template <typename W>
static hipError_t big_dispatch(const Plan &p, const NttArgs<W> &A, int op, const uint64_t *a, const uint64_t *b,
                               uint64_t *c, size_t batch) {
    if (p.logn == kBigS + 1) return Big<1, W>::run(p, A, op, a, b, c, batch);
    if (p.logn == kBigS + 2) return Big<2, W>::run(p, A, op, a, b, c, batch);
    return hipErrorInvalidValue;
}

hipError_t launch_big(const Plan &p, int op, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch) {
    if (batch == 0) return hipSuccess;
    if (!p.big_sync) return hipErrorInvalidValue;
    // The scratch pair is shared by every stream of the context: enqueue the
    // whole sequence under the lock, after the previous sequence if that ran
    // on another stream.
    BigSync &bs = *p.big_sync;
    std::lock_guard<std::mutex> lk(bs.mu);
    hipError_t e = hipSuccess;
    if (!bs.done) e = hipEventCreateWithFlags(&bs.done, hipEventDisableTiming);
    else if (bs.last != p.stream) e = hipStreamWaitEvent(p.stream, bs.done, 0);
    if (e != hipSuccess) return e;
    if (p.word == 32)
        e = big_dispatch<uint32_t>(p, p.a32, op, a, b, c, batch);
    else
        e = big_dispatch<uint64_t>(p, p.a64, op, a, b, c, batch);
    if (e != hipSuccess) return e;
    e = hipEventRecord(bs.done, p.stream);
    bs.last = p.stream;
    return e;
}

}  // namespace FHE_NS
