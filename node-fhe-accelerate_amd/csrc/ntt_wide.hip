// ntt_wide.hip -- transforms for moduli 2^62 <= q < 2^64 (any odd q the
// reference's NTTProcessor accepts: every product there is a
// `(__uint128_t)a * b % q`, ntt_processor.cpp:151-153, 298-307).
//
// The lazy Harvey butterflies of ntt_core.hpp keep values below 4q, which
// needs 4q <= 2^64; above 2^62 this family keeps every value canonical
// instead: mod_add / mod_sub with the carry-out of the 64-bit sum
// (ModularArithmetic::mod_add, modular_arithmetic.cpp:122-153), and products
// as Montgomery multiplications with R = 2^64 whose 65-bit intermediate sum
// is carried explicitly (wmont).  Twiddles are stored in Montgomery form
// (w R mod q), so wmont(x, w R) = x w mod q.
//
// N <= 16384: one workgroup per polynomial, the whole polynomial in LDS
// (128 KiB at N = 16384), radix-2 stages with a barrier each -- the
// reference's stage loop (ntt_processor.cpp:262-311, 325-380) with the
// bit reversal folded into the HBM load (forward) / store (inverse).
// N = 32768 / 65536: the same stages over HBM, one launch per stage, in
// chunks through the context's big-N scratch (ordered by BigSync as
// ntt_big.hip).  Canonical outputs are those of the reference bit for bit:
// every step is exact over Z_q.
#include "fhe_internal.hpp"

namespace FHE_NS {

__device__ __forceinline__ uint64_t wred(uint64_t x, const WideArgs &W) { return mod64_slow(x, W.q, W.mu); }

// final map of a forward output (op 0 canonical, 1 times R, 2 (.) w)
__device__ __forceinline__ uint64_t wide_fwd_epi(uint64_t x, int op, const uint64_t *w, size_t i, const WideArgs &W) {
    if (op == 1) return wmont(x, W.r2, W.q, W.qinv);
    if (op == 2) return wmont(wmont(x, wred(w[i], W), W.q, W.qinv), W.r2, W.q, W.qinv);
    return x;
}

// ---------------------------------------------------------------- N <= 16384
template <int LOGN>
__device__ __forceinline__ void wide_fwd_lds(uint64_t *s, const uint64_t *src, uint32_t tid, const WideArgs &W) {
    constexpr int N = 1 << LOGN, T = N / 2 < 1024 ? N / 2 : 1024;
    for (uint32_t i = tid; i < (uint32_t)N; i += T) s[cbrv(i, LOGN)] = wred(__builtin_nontemporal_load(src + i), W);
    __syncthreads();
#pragma unroll 1
    for (int st = 0; st < LOGN; ++st) {
        const uint32_t m = 1u << st;
        for (uint32_t b = tid; b < (uint32_t)N / 2; b += T) {
            const uint32_t j = b & (m - 1), k = ((b >> st) << (st + 1)) + j;
            const uint64_t t = wmont(s[k + m], W.twf[m + j], W.q, W.qinv), u = s[k];
            s[k] = wadd(u, t, W.q);
            s[k + m] = wsub(u, t, W.q);
        }
        __syncthreads();
    }
}
template <int LOGN>
__device__ __forceinline__ void wide_inv_stages_lds(uint64_t *s, uint32_t tid, const WideArgs &W) {
    constexpr int N = 1 << LOGN, T = N / 2 < 1024 ? N / 2 : 1024;
#pragma unroll 1
    for (int st = LOGN - 1; st >= 0; --st) {
        const uint32_t m = 1u << st;
        for (uint32_t b = tid; b < (uint32_t)N / 2; b += T) {
            const uint32_t j = b & (m - 1), k = ((b >> st) << (st + 1)) + j;
            const uint64_t u = s[k], v = s[k + m];
            s[k] = wadd(u, v, W.q);
            s[k + m] = wmont(wsub(u, v, W.q), W.twi[m + j], W.q, W.qinv);
        }
        __syncthreads();
    }
}

// op: 0 fwd, 1 fwd * R, 2 fwd (.) w, 3 inv, 4 polymul inv(fwd(a) (.) fwd(b))
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 2 < 1024 ? (1 << LOGN) / 2 : 1024)
k_wide(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *c, size_t batch, int op, WideArgs W) {
    constexpr int N = 1 << LOGN, T = N / 2 < 1024 ? N / 2 : 1024;
    __shared__ uint64_t s[N];
    const uint32_t tid = threadIdx.x;
    const size_t poly = blockIdx.x;
    if (poly >= batch) return;
    const uint64_t *ap = a + poly * N;
    uint64_t *cp = c + poly * N;
    if (op <= 2) {
        wide_fwd_lds<LOGN>(s, ap, tid, W);
        for (uint32_t i = tid; i < (uint32_t)N; i += T) cp[i] = wide_fwd_epi(s[i], op, b ? b + poly * N : nullptr, i, W);
        return;
    }
    uint64_t scale = W.ninv_m;  // N^-1 R: wmont(x, N^-1 R) = x N^-1
    if (op == 4) {
        // fwd(a) waits in c's row (own positions: no cross-thread order)
        wide_fwd_lds<LOGN>(s, ap, tid, W);
        for (uint32_t i = tid; i < (uint32_t)N; i += T) cp[i] = s[i];
        __syncthreads();
        wide_fwd_lds<LOGN>(s, b + poly * N, tid, W);
        for (uint32_t i = tid; i < (uint32_t)N; i += T) s[i] = wmont(cp[i], s[i], W.q, W.qinv);  // A B R^-1
        scale = W.ninv_r2;  // N^-1 R^2 restores the R
        __syncthreads();
    } else {
        for (uint32_t i = tid; i < (uint32_t)N; i += T) s[i] = wred(__builtin_nontemporal_load(ap + i), W);
        __syncthreads();
    }
    wide_inv_stages_lds<LOGN>(s, tid, W);
    for (uint32_t i = tid; i < (uint32_t)N; i += T) cp[i] = wmont(s[cbrv(i, LOGN)], scale, W.q, W.qinv);
}

// ---------------------------------------------------------------- N > 16384
// x[p][brv(i)] = src[p][i] mod q
__global__ void __launch_bounds__(256) k_wide_bitrev(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst,
                                                     uint32_t logn, size_t batch, WideArgs W) {
    const size_t total = batch << logn, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += stride) {
        const size_t p = g >> logn;
        const uint32_t i = (uint32_t)g & ((1u << logn) - 1);
        dst[(p << logn) + cbrv(i, (int)logn)] = wred(src[g], W);
    }
}
// one radix-2 stage over HBM: DIT (forward) or GS (inverse)
__global__ void __launch_bounds__(256) k_wide_stage(uint64_t *x, uint32_t logn, int st, int inv, size_t batch,
                                                    WideArgs W) {
    const size_t half = (size_t)1 << (logn - 1), total = batch * half, stride = (size_t)gridDim.x * blockDim.x;
    const uint32_t m = 1u << st;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += stride) {
        const size_t p = g >> (logn - 1);
        const uint32_t bf = (uint32_t)(g & (half - 1)), j = bf & (m - 1), k = ((bf >> st) << (st + 1)) + j;
        uint64_t *y = x + (p << logn);
        const uint64_t u = y[k], v = y[k + m];
        if (!inv) {
            const uint64_t t = wmont(v, W.twf[m + j], W.q, W.qinv);
            y[k] = wadd(u, t, W.q);
            y[k + m] = wsub(u, t, W.q);
        } else {
            y[k] = wadd(u, v, W.q);
            y[k + m] = wmont(wsub(u, v, W.q), W.twi[m + j], W.q, W.qinv);
        }
    }
}
// op 0/1/2: forward epilogue from x (natural order) to out; 3: out[i] =
// x[brv(i)] * scale; 5: out = wmont(x, y) (polymul middle); 6: out = x mod q
__global__ void __launch_bounds__(256) k_wide_finish(const uint64_t *x, const uint64_t *__restrict__ y, uint64_t *out,
                                                     uint32_t logn, size_t batch, int op, uint64_t scale, WideArgs W) {
    const size_t total = batch << logn, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += stride) {
        if (op == 3) {
            const size_t p = g >> logn;
            const uint32_t i = (uint32_t)g & ((1u << logn) - 1);
            out[g] = wmont(x[(p << logn) + cbrv(i, (int)logn)], scale, W.q, W.qinv);
        } else if (op == 5) {
            out[g] = wmont(x[g], y[g], W.q, W.qinv);
        } else if (op == 6) {
            out[g] = wred(x[g], W);
        } else {
            out[g] = wide_fwd_epi(x[g], op, y, g, W);
        }
    }
}

static dim3 wide_grid(size_t work) {
    size_t g = (work + 255) / 256;
    const size_t cap = 256 * 32;
    return dim3((unsigned)(g < 1 ? 1 : (g > cap ? cap : g)));
}

static hipError_t wide_big(const Plan &p, int op, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch) {
    const WideArgs &W = p.wa;
    const uint32_t logn = p.logn;
    const size_t N = (size_t)1 << logn;
    uint64_t *s0 = p.big_scratch[0], *s1 = p.big_scratch[1];
    if (!s0 || !s1 || !p.big_sync) return hipErrorInvalidValue;
    BigSync &bs = *p.big_sync;
    std::lock_guard<std::mutex> lk(bs.mu);
    hipError_t e = hipSuccess;
    if (!bs.done) e = hipEventCreateWithFlags(&bs.done, hipEventDisableTiming);
    else if (bs.last != p.stream) e = hipStreamWaitEvent(p.stream, bs.done, 0);
    if (e != hipSuccess) return e;
    auto fwd = [&](const uint64_t *src, uint64_t *x, size_t nb) -> hipError_t {
        hipLaunchKernelGGL(k_wide_bitrev, wide_grid(nb * N), dim3(256), 0, p.stream, src, x, logn, nb, W);
        for (int st = 0; st < (int)logn; ++st)
            hipLaunchKernelGGL(k_wide_stage, wide_grid(nb * N / 2), dim3(256), 0, p.stream, x, logn, st, 0, nb, W);
        return hipGetLastError();
    };
    auto inv_stages = [&](uint64_t *x, size_t nb) -> hipError_t {
        for (int st = (int)logn - 1; st >= 0; --st)
            hipLaunchKernelGGL(k_wide_stage, wide_grid(nb * N / 2), dim3(256), 0, p.stream, x, logn, st, 1, nb, W);
        return hipGetLastError();
    };
    for (size_t p0 = 0; p0 < batch && e == hipSuccess; p0 += p.big_chunk) {
        const size_t nb = batch - p0 < p.big_chunk ? batch - p0 : p.big_chunk;
        const uint64_t *ai = a + p0 * N, *bi = b ? b + p0 * N : nullptr;
        uint64_t *ci = c + p0 * N;
        if (op <= 2) {
            e = fwd(ai, s0, nb);
            if (e == hipSuccess)
                hipLaunchKernelGGL(k_wide_finish, wide_grid(nb * N), dim3(256), 0, p.stream, s0, bi, ci, logn, nb, op,
                                   0ull, W);
        } else if (op == 3) {
            hipLaunchKernelGGL(k_wide_finish, wide_grid(nb * N), dim3(256), 0, p.stream, ai, nullptr, s1, logn, nb, 6,
                               0ull, W);  // s1 = in mod q, natural order
            e = inv_stages(s1, nb);
            if (e == hipSuccess)
                hipLaunchKernelGGL(k_wide_finish, wide_grid(nb * N), dim3(256), 0, p.stream, s1, nullptr, ci, logn, nb,
                                   3, W.ninv_m, W);
        } else {
            e = fwd(ai, s0, nb);
            if (e == hipSuccess) e = fwd(bi, s1, nb);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_wide_finish, wide_grid(nb * N), dim3(256), 0, p.stream, s0, s1, s0, logn, nb, 5,
                                   0ull, W);
                e = inv_stages(s0, nb);
            }
            if (e == hipSuccess)
                hipLaunchKernelGGL(k_wide_finish, wide_grid(nb * N), dim3(256), 0, p.stream, s0, nullptr, ci, logn, nb,
                                   3, W.ninv_r2, W);
        }
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (e != hipSuccess) return e;
    e = hipEventRecord(bs.done, p.stream);
    bs.last = p.stream;
    return e;
}

template <int LOGN>
static hipError_t wide_one(const Plan &p, int op, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch) {
    constexpr int T = (1 << LOGN) / 2 < 1024 ? (1 << LOGN) / 2 : 1024;
    const size_t per = (size_t)1 << 30;  // grid.x <= 2^31 - 1
    for (size_t b0 = 0; b0 < batch; b0 += per) {
        const size_t nb = batch - b0 < per ? batch - b0 : per;
        const size_t off = b0 << LOGN;
        hipLaunchKernelGGL((k_wide<LOGN>), dim3((unsigned)nb), dim3(T), 0, p.stream, a + off, b ? b + off : nullptr,
                           c + off, nb, op, p.wa);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_wide(const Plan &p, int op, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch) {
    if (batch == 0) return hipSuccess;
    switch (p.logn) {
#define FHE_CASE(L) \
    case L: return wide_one<L>(p, op, a, b, c, batch);
        FHE_CASE(2) FHE_CASE(3) FHE_CASE(4) FHE_CASE(5) FHE_CASE(6) FHE_CASE(7) FHE_CASE(8)
        FHE_CASE(9) FHE_CASE(10) FHE_CASE(11) FHE_CASE(12) FHE_CASE(13) FHE_CASE(14)
#undef FHE_CASE
    case 15: case 16: return wide_big(p, op, a, b, c, batch);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace FHE_NS
