// ntt_engine_add.hip -- EncryptionEngine::add_plain (encryption.cpp:638-665)
// and bootstrap's accumulator initialisation (bootstrap_engine.cpp:690-697).
#include "engine_kernels.hpp"

namespace FHE_NS {

// add_plain on coefficient-form ciphertexts: elementwise.
__global__ void k_add_plain(EngArgs E, uint32_t n) {
    const size_t total = E.batch * n, stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t q = E.D.q, mu = E.D.mu;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const size_t c = x / n, i = x % n;
        const uint64_t *src = E.ct + c * 2 * n;
        uint64_t *dst = E.out + c * 2 * n;
        dst[i] = addq(red_q(src[i], q, mu), encode1(E.vals[x], E.D), q);
        dst[n + i] = src[n + i];
    }
}

// bootstrap_with_test_poly's accumulator (bootstrap_engine.cpp:690-697):
// masks zero, body = the test polynomial, for every ciphertext.
__global__ void k_glwe_init(const uint64_t *__restrict__ tp, uint64_t *__restrict__ acc, uint32_t n, uint32_t k1,
                            size_t batch) {
    const size_t per = (size_t)k1 * n, total = batch * per, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const size_t r = x % per;
        acc[x] = r >= (size_t)(k1 - 1) * n ? tp[r - (size_t)(k1 - 1) * n] : 0;
    }
}
hipError_t launch_glwe_init(const uint64_t *test_poly, uint64_t *acc, uint32_t n, uint32_t k1, size_t batch,
                            hipStream_t s) {
    const size_t total = batch * k1 * n;
    if (total == 0) return hipSuccess;
    const size_t blocks = (total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536;
    hipLaunchKernelGGL(k_glwe_init, dim3(blocks), dim3(256), 0, s, test_poly, acc, n, k1, batch);
    return hipGetLastError();
}

hipError_t launch_add_plain(const Plan &p, uint64_t t, const uint64_t *ct, const uint64_t *vals, int is_ntt,
                            uint64_t *out, size_t batch) {
    EngArgs E{};
    E.ct = ct; E.vals = vals; E.out = out; E.batch = batch;
    E.D = make_decoder(plan_q(p), t);
    if (batch == 0) return hipSuccess;
    if (is_ntt) {
        if (p.logn > kMaxFusedLogN) return hipErrorInvalidValue;
        return eng_any<2>(p, E);
    }
    const uint32_t n = 1u << p.logn;
    const size_t total = batch * n;
    const size_t blocks = (total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536;
    hipLaunchKernelGGL(k_add_plain, dim3(blocks), dim3(256), 0, p.stream, E, n);
    return hipGetLastError();
}

}  // namespace FHE_NS
