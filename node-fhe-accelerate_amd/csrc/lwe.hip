// lwe.hip -- the non-transform pieces of TFHE bootstrapping, batched over
// ciphertexts:
//
//   rotate         multiply_glwe_by_monomial / rotate_polynomial
//                  (bootstrap_engine.cpp:249-261, 122-145); also blind_rotate's
//                  initial rotation by -round(b * 2N / q) (:555-557)
//   sample_extract (:594-624)
//   key_switch     (:626-674): out_a = -sum_{i,l} d_il * ksk_a[i,l]  (mod q),
//                  out_b = b - sum_{i,l} d_il * ksk_b[i,l][0], with the
//                  reference's u64-wrapping digit * key products, its `digit
//                  == 0` skip and its raw (unreduced) body when every digit
//                  is zero.
//
// rotate / sample_extract are HBM gathers.  key_switch is a modular
// matrix-vector product per ciphertext over a key shared by the batch: a
// workgroup takes 256 output coefficients of CT ciphertexts, stages their
// digits in LDS chunk by chunk and streams the key rows (coalesced along the
// output index) once per CT ciphertexts.
#include "fhe_internal.hpp"
#include "lwe_ops.hpp"

namespace FHE_NS {

static constexpr int kLweBlock = 256;

static inline size_t lwe_grid(size_t work) {
    size_t g = (work + kLweBlock - 1) / kLweBlock;
    const size_t cap = 256 * 16;
    return g < 1 ? 1 : (g > cap ? cap : g);
}

__global__ void __launch_bounds__(kLweBlock)
k_rotate(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint32_t n, uint32_t k1, size_t batch,
         const int32_t *__restrict__ rot, const uint64_t *__restrict__ lwe_b, uint64_t lwe_q, uint64_t q,
         uint64_t mu) {
    const size_t total = (size_t)batch * k1 * n;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t poly = i / n, c = poly / k1;
        const uint32_t p = (uint32_t)(i % n);
        const int32_t r = rot ? rot[c] : -rot_amount(lwe_b[c], n, lwe_q);
        out[i] = rotated_at(in + poly * n, p, rot_norm(r, n), n, q, mu);
    }
}

// One composed blind-rotation step (GLWE dimension k > 1 or N > 16384, where
// no fused CMux kernel exists): blind_rotate :565-575 as
//   d   = X^r cur - cur            (k_br_diff)
//   nxt = cur + ExtProd(bsk_i, d)  (k_br_add; the external product runs
//                                   composed in between, fhe_gpu.cpp)
// with r = round(a_i 2N / q) per ciphertext; r == 0 skips the step (d = 0,
// nxt = cur word for word, as the reference's `continue`).  The add/sub
// reduce raw words first, as cmux's mod_sub / mod_add on the reduced inputs.
__device__ __forceinline__ uint64_t br_sub(uint64_t x, uint64_t y, uint64_t q, uint64_t mu) {
    return subq(red_q(x, q, mu), red_q(y, q, mu), q);
}
__global__ void __launch_bounds__(kLweBlock)
k_br_diff(const uint64_t *__restrict__ cur, uint64_t *__restrict__ d, uint32_t n, uint32_t k1, size_t batch,
          const uint64_t *__restrict__ lwe_a, uint32_t dim, uint32_t step, uint64_t lwe_q, uint64_t q, uint64_t mu) {
    const size_t total = (size_t)batch * k1 * n;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t poly = i / n, c = poly / k1;
        const int32_t r = rot_amount(lwe_a[c * dim + step], n, lwe_q);
        d[i] = r == 0 ? 0 : br_sub(rotated_at(cur + poly * n, (uint32_t)(i % n), rot_norm(r, n), n, q, mu), cur[i], q, mu);
    }
}
__global__ void __launch_bounds__(kLweBlock)
k_br_add(const uint64_t *__restrict__ cur, const uint64_t *__restrict__ ep, uint64_t *__restrict__ nxt, uint32_t n,
         uint32_t k1, size_t batch, const uint64_t *__restrict__ lwe_a, uint32_t dim, uint32_t step, uint64_t lwe_q,
         uint64_t q, uint64_t mu) {
    const size_t total = (size_t)batch * k1 * n;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t c = i / n / k1;
        const int32_t r = rot_amount(lwe_a[c * dim + step], n, lwe_q);
        nxt[i] = r == 0 ? cur[i] : addq(red_q(ep[i], q, mu), red_q(cur[i], q, mu), q);
    }
}

__global__ void __launch_bounds__(kLweBlock)
k_sample_extract(const uint64_t *__restrict__ glwe, uint64_t *__restrict__ lwe_a, uint64_t *__restrict__ lwe_b,
                 uint32_t n, uint32_t k, size_t batch, uint64_t q, uint64_t mu) {
    const size_t per = (size_t)k * n, total = batch * per;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const size_t c = x / per;
        const uint32_t i = (uint32_t)((x % per) / n), j = (uint32_t)(x % n);
        const uint64_t *mask = glwe + (c * (k + 1) + i) * n;
        lwe_a[x] = j == 0 ? mask[0] : red_q(q - mask[n - j], q, mu);
        if (i == 0 && j == 0) lwe_b[c] = glwe[(c * (k + 1) + k) * n];
    }
}

// ((d * key) mod 2^64) % q  -- key_switch's `(digit * ksk_entry.first[j]) % q`
__device__ __forceinline__ uint64_t ks_term(uint64_t d, uint64_t key, uint64_t q, uint64_t mu) {
    return mod64_slow(d * key, q, mu);
}

constexpr int kKsCt = 16;     // ciphertexts per workgroup (key rows read once per 16)
constexpr int kKsChunk = 256; // (i, l) entries staged per LDS round

__global__ void __launch_bounds__(kLweBlock)
k_key_switch_a(const uint64_t *__restrict__ ksk_a, const uint64_t *__restrict__ lwe_a, uint64_t *__restrict__ out_a,
               uint32_t in_dim, uint32_t out_dim, uint32_t level, uint32_t base_log, size_t batch, uint64_t q,
               uint64_t mu) {
    __shared__ uint64_t dig[kKsChunk][kKsCt];
    const uint32_t j = blockIdx.x * kLweBlock + threadIdx.x;
    const size_t c0 = (size_t)blockIdx.y * kKsCt;
    const uint64_t mask = (1ull << base_log) - 1;
    const uint32_t entries = in_dim * level;
    uint64_t acc[kKsCt];
#pragma unroll
    for (int c = 0; c < kKsCt; ++c) acc[c] = 0;
    for (uint32_t e0 = 0; e0 < entries; e0 += kKsChunk) {
        const uint32_t ne = entries - e0 < (uint32_t)kKsChunk ? entries - e0 : (uint32_t)kKsChunk;
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < ne * kKsCt; t += kLweBlock) {
            const uint32_t e = t / kKsCt, c = t % kKsCt;
            const uint32_t idx = e0 + e, i = idx / level, l = idx % level;
            const uint32_t shift = (level - 1 - l) * base_log;
            dig[e][c] = c0 + c < batch ? (lwe_a[(c0 + c) * in_dim + i] >> shift) & mask : 0;
        }
        __syncthreads();
        if (j < out_dim) {
            const uint64_t *krow = ksk_a + (size_t)e0 * out_dim + j;
            for (uint32_t e = 0; e < ne; ++e) {
                const uint64_t key = krow[(size_t)e * out_dim];
#pragma unroll
                for (int c = 0; c < kKsCt; ++c) {
                    const uint64_t d = dig[e][c];
                    if (d == 0) continue;  // uniform across the workgroup
                    acc[c] = addq(acc[c], ks_term(d, key, q, mu), q);
                }
            }
        }
    }
    if (j < out_dim) {
#pragma unroll
        for (int c = 0; c < kKsCt; ++c)
            if (c0 + c < batch) out_a[(c0 + c) * out_dim + j] = acc[c] == 0 ? 0 : q - acc[c];
    }
}

// One wavefront per ciphertext: sum of the body terms and the first
// non-zero digit (whose update also reduces the raw body).
__global__ void __launch_bounds__(64)
k_key_switch_b(const uint64_t *__restrict__ ksk_b, const uint64_t *__restrict__ lwe_a,
               const uint64_t *__restrict__ lwe_b, uint64_t *__restrict__ out_b, uint32_t in_dim, uint32_t level,
               uint32_t base_log, uint64_t q, uint64_t mu) {
    const size_t c = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const uint64_t mask = (1ull << base_log) - 1;
    const uint32_t entries = in_dim * level;
    uint64_t s = 0;
    uint32_t first = 0xFFFFFFFFu;
    for (uint32_t idx = lane; idx < entries; idx += 64) {
        const uint32_t i = idx / level, l = idx % level;
        const uint64_t d = (lwe_a[c * in_dim + i] >> ((level - 1 - l) * base_log)) & mask;
        if (d == 0) continue;
        s = addq(s, ks_term(d, ksk_b[idx], q, mu), q);
        first = first < idx ? first : idx;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t so = __shfl_xor(s, off, 64);
        const uint32_t fo = __shfl_xor(first, off, 64);
        s = addq(s, so, q);
        first = first < fo ? first : fo;
    }
    if (lane == 0) {
        const uint64_t b = lwe_b[c];
        if (first == 0xFFFFFFFFu) {
            out_b[c] = b;
        } else {
            const uint32_t i = first / level, l = first % level;
            const uint64_t d = (lwe_a[c * in_dim + i] >> ((level - 1 - l) * base_log)) & mask;
            const uint64_t t1 = ks_term(d, ksk_b[first], q, mu);
            const uint64_t b1 = mod64_slow(b + q - t1, q, mu);  // u64 wrap as in the reference
            out_b[c] = subq(b1, subq(s, t1, q), q);
        }
    }
}

// Key switch with a deferred reduction (q odd, q < 2^63, base_log <= 32).
// The reference's per-term `(result + q - (digit * key) % q) % q`
// (:645-660) stays canonical for q < 2^63, so its result is
// -(sum_{i,l} T_il) mod q with T = digit * key mod 2^64: the wrapped 64-bit
// products are summed exactly in 96 bits (two multiplies and a carry chain
// per term instead of a 64-bit remainder) and reduced once per output.
// grid: x = 256 outputs, y = CT ciphertexts, z = splits of the (i, l)
// entries (small batches: enough workgroups to stream the key at HBM rate);
// with one split the kernel writes -sum mod q, else its partial sum mod q
// to dst[z][batch][out_dim] for k_ks_sum.
constexpr uint32_t kKsSplitMin = 16;  // entries per split at least
template <int CT>
__global__ void __launch_bounds__(kLweBlock)
k_ks_acc(const uint64_t *__restrict__ ksk_a, const uint64_t *__restrict__ lwe_a, uint64_t *__restrict__ dst,
         uint32_t in_dim, uint32_t out_dim, uint32_t level, uint32_t base_log, size_t batch, uint32_t per_split,
         uint64_t q, uint64_t mu, uint64_t qinv, uint64_t r2, int neg) {
    __shared__ uint32_t dig[kKsChunk][CT];
    const uint32_t j = blockIdx.x * kLweBlock + threadIdx.x;
    const size_t c0 = (size_t)blockIdx.y * CT;
    const uint32_t entries = in_dim * level;
    const uint32_t e_lo = blockIdx.z * per_split;
    const uint32_t e_hi = entries - e_lo < per_split ? entries : e_lo + per_split;
    const uint64_t mask = (1ull << base_log) - 1;
    uint64_t lo[CT];
    uint32_t hi[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) lo[c] = 0, hi[c] = 0;
    for (uint32_t e0 = e_lo; e0 < e_hi; e0 += kKsChunk) {
        const uint32_t ne = e_hi - e0 < (uint32_t)kKsChunk ? e_hi - e0 : (uint32_t)kKsChunk;
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < ne * CT; t += kLweBlock) {
            const uint32_t e = t / CT, c = t % CT;
            const uint32_t idx = e0 + e, i = idx / level, l = idx % level;
            const uint32_t shift = (level - 1 - l) * base_log;
            dig[e][c] = c0 + c < batch ? (uint32_t)((lwe_a[(c0 + c) * in_dim + i] >> shift) & mask) : 0u;
        }
        __syncthreads();
        if (j < out_dim) {
            const uint64_t *krow = ksk_a + (size_t)e0 * out_dim + j;
#pragma unroll 4
            for (uint32_t e = 0; e < ne; ++e) {
                const uint64_t key = krow[(size_t)e * out_dim];
#pragma unroll
                for (int c = 0; c < CT; ++c) {
                    const uint64_t t = (uint64_t)dig[e][c] * key;  // mod 2^64, as the reference's u64 product
                    lo[c] += t;
                    hi[c] += lo[c] < t ? 1u : 0u;
                }
            }
        }
    }
    if (j >= out_dim) return;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        if (c0 + c >= batch) break;
        // (hi 2^64 + lo) mod q: hi 2^64 = wmont(hi, 2^128 mod q)
        const uint64_t h = wmont(mod64_slow(hi[c], q, mu), r2, q, qinv);
        const uint64_t r = wadd(h, mod64_slow(lo[c], q, mu), q);
        dst[((size_t)blockIdx.z * batch + c0 + c) * out_dim + j] = neg ? (r == 0 ? 0 : q - r) : r;
    }
}
// out[c][j] = -(sum over the splits) mod q
__global__ void __launch_bounds__(kLweBlock)
k_ks_sum(const uint64_t *__restrict__ part, uint64_t *__restrict__ out, size_t count, uint32_t splits, uint64_t q) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < count; x += stride) {
        uint64_t s = 0;
        for (uint32_t z = 0; z < splits; ++z) s = addq(s, part[(size_t)z * count + x], q);
        out[x] = s == 0 ? 0 : q - s;
    }
}

struct KsPlan {
    int ct;             // ciphertexts per workgroup
    uint32_t splits;    // entry splits (1: no partials)
    size_t chunk;       // ciphertexts per launch
};
static KsPlan ks_plan(const ModConsts &m, uint32_t base_log, uint32_t level, uint32_t in_dim, uint32_t out_dim,
                      size_t batch) {
    KsPlan p{0, 1, batch};
    if (!m.fast || base_log > 32 || out_dim == 0 || (uint64_t)in_dim * level == 0) return p;  // generic kernel
    p.ct = batch >= 16 ? 16 : batch >= 4 ? 4 : 1;
    p.chunk = (size_t)65535 * p.ct < batch ? (size_t)65535 * p.ct : batch;
    const size_t wgs = (size_t)((out_dim + kLweBlock - 1) / kLweBlock) * ((p.chunk + p.ct - 1) / p.ct);
    const uint32_t entries = in_dim * level;
    size_t s = (1024 + wgs - 1) / wgs;
    const size_t smax = (entries + kKsSplitMin - 1) / kKsSplitMin;
    p.splits = (uint32_t)(s < 1 ? 1 : s > smax ? smax : s);
    if (p.splits > 65535) p.splits = 65535;
    return p;
}
size_t key_switch_scratch_bytes(const ModConsts &m, uint32_t base_log, uint32_t level, uint32_t in_dim,
                                uint32_t out_dim, size_t batch) {
    const KsPlan p = ks_plan(m, base_log, level, in_dim, out_dim, batch);
    return p.ct && p.splits > 1 ? (size_t)p.splits * p.chunk * out_dim * 8 : 0;
}

hipError_t launch_rotate(const ModConsts &m, const uint64_t *in, uint64_t *out, uint32_t n, uint32_t k1, size_t batch,
                         const int32_t *rot, const uint64_t *lwe_b, uint64_t lwe_q, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rotate, dim3(lwe_grid((size_t)batch * k1 * n)), dim3(kLweBlock), 0, s, in, out, n, k1, batch,
                       rot, lwe_b, lwe_q, m.q, m.mu);
    return hipGetLastError();
}

hipError_t launch_br_diff(const ModConsts &m, const uint64_t *cur, uint64_t *d, uint32_t n, uint32_t k1, size_t batch,
                          const uint64_t *lwe_a, uint32_t dim, uint32_t step, uint64_t lwe_q, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_br_diff, dim3(lwe_grid((size_t)batch * k1 * n)), dim3(kLweBlock), 0, s, cur, d, n, k1, batch,
                       lwe_a, dim, step, lwe_q, m.q, m.mu);
    return hipGetLastError();
}
hipError_t launch_br_add(const ModConsts &m, const uint64_t *cur, const uint64_t *ep, uint64_t *nxt, uint32_t n,
                         uint32_t k1, size_t batch, const uint64_t *lwe_a, uint32_t dim, uint32_t step, uint64_t lwe_q,
                         hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_br_add, dim3(lwe_grid((size_t)batch * k1 * n)), dim3(kLweBlock), 0, s, cur, ep, nxt, n, k1,
                       batch, lwe_a, dim, step, lwe_q, m.q, m.mu);
    return hipGetLastError();
}

hipError_t launch_sample_extract(const ModConsts &m, const uint64_t *glwe, uint64_t *lwe_a, uint64_t *lwe_b,
                                 uint32_t n, uint32_t k, size_t batch, hipStream_t s) {
    if (batch == 0 || k == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sample_extract, dim3(lwe_grid((size_t)batch * k * n)), dim3(kLweBlock), 0, s, glwe, lwe_a,
                       lwe_b, n, k, batch, m.q, m.mu);
    return hipGetLastError();
}

template <int CT>
static hipError_t ks_acc_launch(const ModConsts &m, const KsPlan &P, uint32_t base_log, uint32_t level, uint32_t in_dim,
                                uint32_t out_dim, const uint64_t *ksk_a, const uint64_t *lwe_a, uint64_t *out_a,
                                size_t nb, void *scratch, hipStream_t s) {
    const uint32_t entries = in_dim * level;
    const uint32_t per = (entries + P.splits - 1) / P.splits;
    const uint32_t splits = (entries + per - 1) / per;
    const dim3 grid((out_dim + kLweBlock - 1) / kLweBlock, (unsigned)((nb + CT - 1) / CT), splits);
    uint64_t *dst = splits > 1 ? (uint64_t *)scratch : out_a;
    hipLaunchKernelGGL(k_ks_acc<CT>, grid, dim3(kLweBlock), 0, s, ksk_a, lwe_a, dst, in_dim, out_dim, level, base_log,
                       nb, per, m.q, m.mu, m.qinv, m.r2, splits > 1 ? 0 : 1);
    if (hipError_t e = hipGetLastError()) return e;
    if (splits > 1) {
        const size_t cnt = nb * out_dim;
        hipLaunchKernelGGL(k_ks_sum, dim3(lwe_grid(cnt)), dim3(kLweBlock), 0, s, dst, out_a, cnt, splits, m.q);
        return hipGetLastError();
    }
    return hipSuccess;
}

hipError_t launch_key_switch(const ModConsts &m, uint32_t base_log, uint32_t level, uint32_t in_dim, uint32_t out_dim,
                             const uint64_t *ksk_a, const uint64_t *ksk_b, const uint64_t *lwe_a,
                             const uint64_t *lwe_b, uint64_t *out_a, uint64_t *out_b, size_t batch, void *scratch,
                             hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const KsPlan P = ks_plan(m, base_log, level, in_dim, out_dim, batch);
    if (P.ct && (P.splits == 1 || scratch)) {
        for (size_t b0 = 0; b0 < batch; b0 += P.chunk) {
            const size_t nb = batch - b0 < P.chunk ? batch - b0 : P.chunk;
            const uint64_t *la = lwe_a + b0 * in_dim;
            uint64_t *oa = out_a + b0 * out_dim;
            hipError_t e = P.ct == 16 ? ks_acc_launch<16>(m, P, base_log, level, in_dim, out_dim, ksk_a, la, oa, nb, scratch, s)
                         : P.ct == 4 ? ks_acc_launch<4>(m, P, base_log, level, in_dim, out_dim, ksk_a, la, oa, nb, scratch, s)
                                     : ks_acc_launch<1>(m, P, base_log, level, in_dim, out_dim, ksk_a, la, oa, nb, scratch, s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_key_switch_b, dim3((unsigned)batch), dim3(64), 0, s, ksk_b, lwe_a, lwe_b, out_b, in_dim,
                           level, base_log, m.q, m.mu);
        return hipGetLastError();
    }
    // generic: any q >= 2, any base_log (64-bit remainder per term)
    // grid.y <= 65535 workgroups of kKsCt ciphertexts per launch
    const size_t per_launch = (size_t)65535 * kKsCt;
    for (size_t b0 = 0; out_dim > 0 && b0 < batch; b0 += per_launch) {
        const size_t nb = batch - b0 < per_launch ? batch - b0 : per_launch;
        const dim3 grid((out_dim + kLweBlock - 1) / kLweBlock, (unsigned)((nb + kKsCt - 1) / kKsCt));
        hipLaunchKernelGGL(k_key_switch_a, grid, dim3(kLweBlock), 0, s, ksk_a, lwe_a + b0 * in_dim,
                           out_a + b0 * out_dim, in_dim, out_dim, level, base_log, nb, m.q, m.mu);
        if (hipError_t e = hipGetLastError()) return e;
    }
    hipLaunchKernelGGL(k_key_switch_b, dim3((unsigned)batch), dim3(64), 0, s, ksk_b, lwe_a, lwe_b, out_b, in_dim, level,
                       base_log, m.q, m.mu);
    return hipGetLastError();
}

}  // namespace FHE_NS
