// keygen.hip -- encryption randomness and key material on the device.
//
// The reference samples on the host with SecureRandom (key_manager.cpp:
// 24-115: random_u64_range's rejection sampling, sample_ternary,
// sample_gaussian's Box-Muller, sample_binary) and builds keys with ring
// operations (generate_public_key :218-246, generate_eval_key :252-333,
// BootstrapEngine::encrypt_ggsw / generate_key_switch_key,
// bootstrap_engine.cpp:268-306, 367-420).  Here the same draws come from a
// ChaCha20 keystream (RFC 8439 block function; 256-bit key, 64-bit block
// counter, 64-bit stream nonce), so a key or an encryption is reproducible
// from (seed, stream) and generated where the ciphertexts live:
//
//   element i of a stream of `count` elements takes its draws from blocks
//   i, i + count, i + 2 count, ... (8 u64 words per block, in order), so
//   every element is one independent lane and rejection sampling never
//   runs out of words.
//
// oracle/ref_cpu.c (oracle_sample) restates the same map on the CPU.
#include "engine_kernels.hpp"
#include "keygen.hpp"

namespace FHE_NS {

static constexpr int kKgBlock = 256;
static inline size_t kg_grid(size_t work) {
    size_t g = (work + kKgBlock - 1) / kKgBlock;
    const size_t cap = 256 * 16;
    return g < 1 ? 1 : (g > cap ? cap : g);
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define FHE_QR(a, b, c, d)                 \
    a += b; d ^= a; d = rotl32(d, 16);     \
    c += d; b ^= c; b = rotl32(b, 12);     \
    a += b; d ^= a; d = rotl32(d, 8);      \
    c += d; b ^= c; b = rotl32(b, 7);

// One 64-byte ChaCha20 block as 8 little-endian u64 words.
__device__ __forceinline__ void chacha_block(const ChaChaKey &key, uint64_t counter, uint64_t nonce, uint64_t (&o)[8]) {
    const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key.k[0], key.k[1], key.k[2], key.k[3],
                             key.k[4], key.k[5], key.k[6], key.k[7], (uint32_t)counter, (uint32_t)(counter >> 32),
                             (uint32_t)nonce, (uint32_t)(nonce >> 32)};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = in[i];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        FHE_QR(x[0], x[4], x[8], x[12]) FHE_QR(x[1], x[5], x[9], x[13])
        FHE_QR(x[2], x[6], x[10], x[14]) FHE_QR(x[3], x[7], x[11], x[15])
        FHE_QR(x[0], x[5], x[10], x[15]) FHE_QR(x[1], x[6], x[11], x[12])
        FHE_QR(x[2], x[7], x[8], x[13]) FHE_QR(x[3], x[4], x[9], x[14])
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
        o[i] = (uint64_t)(x[2 * i] + in[2 * i]) | ((uint64_t)(x[2 * i + 1] + in[2 * i + 1]) << 32);
}
#undef FHE_QR

// The draw sequence of one element.
struct Draws {
    const ChaChaKey &key;
    uint64_t nonce, idx, count;
    uint64_t blk = 0;
    int pos = 8;
    uint64_t buf[8];
    __device__ Draws(const ChaChaKey &k, uint64_t n, uint64_t i, uint64_t c) : key(k), nonce(n), idx(i), count(c) {}
    __device__ uint64_t next() {
        if (pos == 8) {
            chacha_block(key, idx + blk * count, nonce, buf);
            ++blk;
            pos = 0;
        }
        // a compare chain instead of buf[pos]: a dynamically indexed local
        // array lives in scratch (120 B per lane)
        uint64_t r = buf[0];
#pragma unroll
        for (int k = 1; k < 8; ++k)
            if (pos == k) r = buf[k];
        ++pos;
        return r;
    }
    // random_u64_range (key_manager.cpp:60-71): rejection below
    // (2^64 - max) % max, then % max
    __device__ uint64_t range(uint64_t max) {
        if (max == 0) return 0;
        const uint64_t thr = (0ull - max) % max;
        uint64_t r;
        do r = next();
        while (r < thr);
        return r % max;
    }
    // uniform_real_distribution<double>(0, 1): 53 random bits
    __device__ double unit() { return (double)(next() >> 11) * 0x1.0p-53; }
};

__device__ uint64_t sample_one(int kind, Draws &d, uint64_t q, double std_dev) {
    switch (kind) {
    case kUniform: return d.range(q);
    case kTernary: {  // sample_ternary (:73-83)
        const uint64_t r = d.range(3);
        return r == 0 ? q - 1 : (r == 1 ? 0 : 1);
    }
    case kGaussian: {  // sample_gaussian (:85-110)
        double u1 = d.unit();
        const double u2 = d.unit();
        while (u1 == 0.0) u1 = d.unit();
        const double z = sqrt(-2.0 * log(u1)) * cos(2.0 * 3.14159265358979323846 * u2);
        const double smp = round(z * std_dev);
        int64_t v = (int64_t)smp;
        if (v < 0) {
            if (q >> 63) {
                // (int64_t)q = q - 2^64 < 0: the reference loop adds it until
                // the sum wraps past INT64_MIN (signed overflow on its
                // platform, ~2^31 iterations at q = 2^64 - 2^32 + 1).  The
                // wrapped value in closed form: k = the first count with
                // v - k m < -2^63 (m = 2^64 - q), result v - k m + 2^64.
                const uint64_t m = 0ull - q;
                const uint64_t k = ((uint64_t)(v + INT64_MAX) + 1) / m + 1;
                return ((uint64_t)v - k * m) % q;
            }
            v = (int64_t)q + v;
            while (v < 0) v += (int64_t)q;
        }
        return (uint64_t)v % q;
    }
    case kBinary: return d.next() & 1;  // sample_binary (:112-114)
    default: return d.next();           // random_u64
    }
}

__global__ void __launch_bounds__(kKgBlock)
k_sample(int kind, ChaChaKey key, uint64_t nonce, uint64_t q, double std_dev, uint64_t *__restrict__ out, size_t count) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        Draws d(key, nonce, i, count);
        out[i] = sample_one(kind, d, q, std_dev);
    }
}

__device__ __forceinline__ uint64_t modmul_exact(uint64_t a, uint64_t b, uint64_t q, uint64_t mu, double qinv) {
    a = red_q(a, q, mu);
    b = red_q(b, q, mu);
    const uint64_t lo = a * b, hi = __umul64hi(a, b);
    return lo - div128(hi, lo, q, qinv) * q;
}

__global__ void __launch_bounds__(kKgBlock)
k_modmul_bcast(const uint64_t *__restrict__ x, const uint64_t *__restrict__ y, uint64_t *__restrict__ out, uint32_t n,
               size_t batch, uint64_t q, uint64_t mu, double qinv) {
    const size_t total = (size_t)n * batch, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride)
        out[i] = modmul_exact(x[i], y[i % n], q, mu, qinv);
}

// gadget term of encrypt_ggsw (:287-291): (|v| q) >> ((l + 1) B) with the
// u64 product, negated mod q for v < 0.  Shift counts of 64 or more take
// the count mod 64, as the shift instructions of the reference's targets do.
__device__ __forceinline__ uint64_t ggsw_gadget(int64_t v, uint64_t q, uint32_t l, uint32_t base_log) {
    const uint64_t av = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    uint64_t g = (av * q) >> (((l + 1) * base_log) & 63);
    if (v < 0) g = (q - g) % q;
    return g;
}

__global__ void __launch_bounds__(kKgBlock)
k_ggsw_finish(const uint64_t *__restrict__ prod, const uint64_t *__restrict__ masks, const uint64_t *__restrict__ err,
              const int64_t *__restrict__ values, uint64_t *__restrict__ out, uint32_t n, uint32_t k, uint32_t level,
              uint32_t base_log, size_t rows, uint64_t q, uint64_t mu) {
    const size_t total = rows * n, stride = (size_t)gridDim.x * blockDim.x;
    const uint32_t per_ct = (k + 1) * level;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const size_t r = x / n;
        const uint32_t j = (uint32_t)(x % n);
        const uint32_t rr = (uint32_t)(r % per_ct), grp = rr / level, l = rr % level;
        // encrypt_glwe_zero (:190-227): body = 0 + sum_i mask_i * sk, + e
        uint64_t body = 0;
        for (uint32_t i = 0; i < k; ++i) body = addq(body, red_q(prod[(r * k + i) * n + j], q, mu), q);
        body = addq(body, red_q(err[r * n + j], q, mu), q);
        const uint64_t g = j == 0 ? ggsw_gadget(values[r / per_ct], q, l, base_log) : 0;
        for (uint32_t i = 0; i < k; ++i) {
            uint64_t m = masks[(r * k + i) * n + j];
            if (j == 0 && grp == i) m = mod64_slow(m + g, q, mu);  // (mask[row][0] + gadget) % q
            out[(r * (k + 1) + i) * n + j] = m;
        }
        if (j == 0 && grp == k) body = mod64_slow(body + g, q, mu);
        out[(r * (k + 1) + k) * n + j] = body;
    }
}

// One wavefront per key-switching entry: the int64 inner product (wrapping,
// as the reference's int64_t accumulation) reduced across lanes.
__global__ void __launch_bounds__(64)
k_ksk_body(const uint64_t *__restrict__ glwe_sk, const int64_t *__restrict__ lwe_sk, const uint64_t *__restrict__ a,
           const uint64_t *__restrict__ err, uint64_t *__restrict__ b, uint32_t level, uint32_t base_log,
           uint32_t lwe_dim, uint64_t q, uint64_t mu) {
    const size_t e = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    uint64_t ip = 0;
    for (uint32_t j = lane; j < lwe_dim; j += 64) ip += a[e * lwe_dim + j] * (uint64_t)lwe_sk[j];
    for (int off = 32; off > 0; off >>= 1) ip += __shfl_xor(ip, off, 64);
    if (lane == 0) {
        const uint32_t i = (uint32_t)(e / level), l = (uint32_t)(e % level);
        int64_t ev = (int64_t)err[e];
        if (ev > (int64_t)(q / 2)) ev -= (int64_t)q;
        const uint64_t gadget = (glwe_sk[i] * q) >> (((l + 1) * base_log) & 63);
        const int64_t s = (int64_t)(ip + (uint64_t)ev);
        b[e] = mod64_slow((uint64_t)(s % (int64_t)q) + gadget, q, mu);
    }
}

// One wavefront per LWE ciphertext.
__global__ void __launch_bounds__(64)
k_lwe_decrypt(const int64_t *__restrict__ sk, uint32_t dim, const uint64_t *__restrict__ a, const uint64_t *__restrict__ b,
              uint64_t *__restrict__ m, uint64_t *__restrict__ phase, Decoder D) {
    const size_t c = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    uint64_t s = 0;
    for (uint32_t j = lane; j < dim; j += 64) {
        const int64_t kv = sk[j];
        const uint64_t mag = mod64_slow(kv < 0 ? (uint64_t)0 - (uint64_t)kv : (uint64_t)kv, D.q, D.mu);
        const uint64_t kq = kv < 0 && mag ? D.q - mag : mag;  // s_j mod q
        s = addq(s, modmul_exact(a[c * dim + j], kq, D.q, D.mu, D.qinv), D.q);
    }
    for (int off = 32; off > 0; off >>= 1) s = addq(s, __shfl_xor(s, off, 64), D.q);
    if (lane == 0) {
        const uint64_t p = subq(red_q(b[c], D.q, D.mu), s, D.q);
        if (phase) phase[c] = p;
        if (m) m[c] = D.rounded(p) % D.t;
    }
}

hipError_t launch_sample(int kind, const ChaChaKey &key, uint64_t nonce, uint64_t q, double std_dev, uint64_t *out,
                         size_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sample, dim3(kg_grid(count)), dim3(kKgBlock), 0, s, kind, key, nonce, q, std_dev, out, count);
    return hipGetLastError();
}
hipError_t launch_modmul_bcast(const ModConsts &m, const uint64_t *x, const uint64_t *y, uint64_t *out, uint32_t n,
                               size_t batch, hipStream_t s) {
    if (batch == 0 || n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_modmul_bcast, dim3(kg_grid((size_t)n * batch)), dim3(kKgBlock), 0, s, x, y, out, n, batch, m.q,
                       m.mu, 1.0 / (double)m.q);
    return hipGetLastError();
}
hipError_t launch_ggsw_finish(const ModConsts &m, const uint64_t *prod, const uint64_t *masks, const uint64_t *err,
                              const int64_t *values, uint64_t *out, uint32_t n, uint32_t k, uint32_t level,
                              uint32_t base_log, size_t count, hipStream_t s) {
    const size_t rows = count * (k + 1) * level;
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ggsw_finish, dim3(kg_grid(rows * n)), dim3(kKgBlock), 0, s, prod, masks, err, values, out, n, k,
                       level, base_log, rows, m.q, m.mu);
    return hipGetLastError();
}
hipError_t launch_ksk_body(const ModConsts &m, const uint64_t *glwe_sk, const int64_t *lwe_sk, const uint64_t *a,
                           const uint64_t *err, uint64_t *b, uint32_t n_in, uint32_t level, uint32_t base_log,
                           uint32_t lwe_dim, hipStream_t s) {
    const size_t entries = (size_t)n_in * level;
    if (entries == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ksk_body, dim3((unsigned)entries), dim3(64), 0, s, glwe_sk, lwe_sk, a, err, b, level, base_log,
                       lwe_dim, m.q, m.mu);
    return hipGetLastError();
}
hipError_t launch_lwe_decrypt(uint64_t q, uint64_t t, const int64_t *sk, uint32_t dim, const uint64_t *a,
                              const uint64_t *b, uint64_t *m, uint64_t *phase, size_t batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const Decoder D = make_decoder(q, t);
    hipLaunchKernelGGL(k_lwe_decrypt, dim3((unsigned)batch), dim3(64), 0, s, sk, dim, a, b, m, phase, D);
    return hipGetLastError();
}

}  // namespace FHE_NS
