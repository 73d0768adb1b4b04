// engine_composed.hip -- EncryptionEngine encrypt / decrypt / add_plain for
// the contexts the fused engine kernels (engine_kernels.hpp) do not take:
// moduli 2^62 <= q < 2^64 (canonical arithmetic, ntt_wide.hip transforms)
// and degrees N > 16384 (two-pass transforms, ntt_big.hip).  The host
// (fhe_gpu.cpp) composes batched transforms, the exact broadcast modmul and
// the finishing kernels below, in the order of the reference:
//   encrypt_internal (encryption.cpp:171-205):
//     c0 = inv(fwd(pk.b) . fwd(u)) + e1 + encode(v),  c1 = inv(fwd(pk.a) . fwd(u)) + e2
//   decrypt (:234-300) + decode_packed (:150-163) + compute_noise_budget (:364-400):
//     phase = c0 - inv(fwd(c1) . fwd(s)) [- inv(fwd(c2) . fwd(s)^2)]
//   add_plain (:638-665): c0 + encode(v) (to_ntt'd for NTT-domain ciphertexts)
// Prepared keys of such contexts are canonical NTT-domain rows (no
// Montgomery factor): pk_prep = (fwd(pk.a), fwd(pk.b)), sk_prep = (fwd(s),
// fwd(s)^2).  Every kernel here is an HBM-streaming elementwise pass.
#include "engine_kernels.hpp"

namespace FHE_NS {

static constexpr int kEcBlock = 256;
static inline size_t ec_grid(size_t work) {
    size_t g = (work + kEcBlock - 1) / kEcBlock;
    return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}

// ct [batch][2][n]: c0 = t0 + e1 + encode(v), c1 = t1 + e2 (mod_add order of :186-196)
__global__ void __launch_bounds__(kEcBlock)
k_enc_finish(const uint64_t *__restrict__ t0, const uint64_t *__restrict__ t1, const uint64_t *__restrict__ e1,
             const uint64_t *__restrict__ e2, const uint64_t *__restrict__ vals, uint64_t *__restrict__ ct, uint32_t logn,
             size_t batch, Decoder D) {
    const size_t total = batch << logn, stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t q = D.q, mu = D.mu, mask = (1ull << logn) - 1;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const size_t o = ((x >> logn) << (logn + 1)) | (x & mask);
        ct[o] = addq(addq(red_q(t0[x], q, mu), red_q(e1[x], q, mu), q), encode1(vals[x], D), q);
        ct[o + mask + 1] = addq(red_q(t1[x], q, mu), red_q(e2[x], q, mu), q);
    }
}

// out[b][i] = src[b][row][i] - x[b][i] (src rows of `comps` polynomials)
__global__ void __launch_bounds__(kEcBlock)
k_sub_row(const uint64_t *__restrict__ src, uint32_t comps, const uint64_t *__restrict__ x, uint64_t *__restrict__ out,
          uint32_t logn, size_t batch, uint64_t q, uint64_t mu) {
    const size_t total = batch << logn, stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t mask = (1ull << logn) - 1;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const uint64_t c = red_q(src[((i >> logn) * comps << logn) | (i & mask)], q, mu);
        out[i] = subq(c, red_q(x[i], q, mu), q);
    }
}

// decode_packed + the noise distance of compute_noise_budget, literally with
// the reference's int64 arithmetic (wrapping where q >= 2^63), for the
// canonical phase; per-ciphertext maximum by a 64-bit atomic (noise zeroed
// by the host).
__global__ void __launch_bounds__(kEcBlock)
k_decode(const uint64_t *__restrict__ phase, uint64_t *__restrict__ dec, unsigned long long *__restrict__ noise,
         uint32_t logn, size_t batch, Decoder D) {
    const size_t total = batch << logn, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const uint64_t p = phase[i];
        const uint64_t r = D.rounded(p);
        if (dec) dec[i] = r % D.t;
        if (noise) {
            const uint64_t expected = mod64_slow(r * D.delta, D.q, D.mu);  // (rounded * delta_) % modulus
            uint64_t nz = p >= expected ? p - expected : expected - p;    // int64_t noise (two's complement)
            if ((int64_t)nz > (int64_t)D.half) nz = D.q - nz;            // (int64_t)q - noise
            const uint64_t a = (int64_t)nz < 0 ? 0ull - nz : nz;          // |noise|
            atomicMax(noise + (i >> logn), (unsigned long long)a);
        }
    }
}

// out[b] = (c0 + f, c1): add_plain with the (transformed) encoding f [batch][n]
__global__ void __launch_bounds__(kEcBlock)
k_add_plain_fin(const uint64_t *__restrict__ ct, const uint64_t *__restrict__ f, uint64_t *__restrict__ out, uint32_t logn,
                size_t batch, uint64_t q, uint64_t mu) {
    const size_t total = batch << logn, stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t mask = (1ull << logn) - 1;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const size_t o = ((x >> logn) << (logn + 1)) | (x & mask);
        out[o] = addq(red_q(ct[o], q, mu), red_q(f[x], q, mu), q);
        out[o + mask + 1] = ct[o + mask + 1];
    }
}

__global__ void __launch_bounds__(kEcBlock)
k_encode(const uint64_t *__restrict__ vals, uint64_t *__restrict__ out, size_t count, Decoder D) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) out[i] = encode1(vals[i], D);
}

static uint32_t log2u(uint32_t n) {
    uint32_t l = 0;
    while ((1u << l) < n) ++l;
    return l;
}

hipError_t launch_enc_finish(uint64_t q, uint64_t t, const uint64_t *t0, const uint64_t *t1, const uint64_t *e1,
                             const uint64_t *e2, const uint64_t *vals, uint64_t *ct, uint32_t n, size_t batch,
                             hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_enc_finish, dim3(ec_grid(batch * n)), dim3(kEcBlock), 0, s, t0, t1, e1, e2, vals, ct, log2u(n),
                       batch, make_decoder(q, t));
    return hipGetLastError();
}
hipError_t launch_sub_row(uint64_t q, const uint64_t *src, uint32_t comps, const uint64_t *x, uint64_t *out, uint32_t n,
                          size_t batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const Decoder D = make_decoder(q, 0);
    hipLaunchKernelGGL(k_sub_row, dim3(ec_grid(batch * n)), dim3(kEcBlock), 0, s, src, comps, x, out, log2u(n), batch,
                       D.q, D.mu);
    return hipGetLastError();
}
hipError_t launch_decode(uint64_t q, uint64_t t, const uint64_t *phase, uint64_t *dec, uint64_t *noise, uint32_t n,
                         size_t batch, hipStream_t s) {
    if (batch == 0 || (!dec && !noise)) return hipSuccess;
    if (noise) {
        hipError_t e = hipMemsetAsync(noise, 0, batch * 8, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_decode, dim3(ec_grid(batch * n)), dim3(kEcBlock), 0, s, phase, dec,
                       reinterpret_cast<unsigned long long *>(noise), log2u(n), batch, make_decoder(q, t));
    return hipGetLastError();
}
hipError_t launch_add_plain_fin(uint64_t q, const uint64_t *ct, const uint64_t *f, uint64_t *out, uint32_t n, size_t batch,
                                hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const Decoder D = make_decoder(q, 0);
    hipLaunchKernelGGL(k_add_plain_fin, dim3(ec_grid(batch * n)), dim3(kEcBlock), 0, s, ct, f, out, log2u(n), batch, D.q,
                       D.mu);
    return hipGetLastError();
}
hipError_t launch_encode(uint64_t q, uint64_t t, const uint64_t *vals, uint64_t *out, size_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode, dim3(ec_grid(count)), dim3(kEcBlock), 0, s, vals, out, count, make_decoder(q, t));
    return hipGetLastError();
}

}  // namespace FHE_NS
