// elementwise.hip -- HBM-streaming coefficient kernels.
//
//   modmul     : c = a*b mod q for any u64 a, b (BarrettReducer::barrett_mul
//                contract, modular_arithmetic.cpp:268-280; Metal
//                modmul_direct_batch, modmul_direct.metal:230-250;
//                PolynomialRing::pointwise_multiply, polynomial_ring.cpp:493-530)
//   add / sub  : ModularArithmetic::mod_add / mod_sub semantics
//                (modular_arithmetic.cpp:122-153) elementwise
//                (PolynomialRing::add/subtract, polynomial_ring.cpp:263-415)
//   neg        : PolynomialRing::negate (polynomial_ring.cpp:340-355)
//   mul_scalar : PolynomialRing::multiply_scalar (polynomial_ring.cpp:454-473)
//   ml_montmul : MultiLimbModularArithmetic::montgomery_mul, 2 limbs
//                (modular_arithmetic.cpp:525-625)
//   decompose  : BootstrapEngine::decompose_polynomial (bootstrap_engine.cpp:152-185)
//
// All are HBM-bound: 16-byte (2 x u64) loads/stores per lane, grid-stride.
#include "fhe_internal.hpp"

namespace FHE_NS {

static constexpr int kBlock = 256;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

static inline size_t grid_for(size_t work) {
    size_t g = (work + kBlock - 1) / kBlock;
    const size_t cap = 256 * 16;  // 256 CUs x 16 blocks: grid-stride beyond
    return g < 1 ? 1 : (g > cap ? cap : g);
}

__device__ __forceinline__ uint64_t red_any(uint64_t x, const ModConsts &m) {
    return x < m.q ? x : mod64_slow(x, m.q, m.mu);
}

// (hi:lo) mod q by restoring shift-subtract; any q >= 1.  Slow path only.
__device__ __noinline__ uint64_t mod128_slow(uint64_t hi, uint64_t lo, uint64_t q) {
    uint64_t r = 0;
    for (int i = 127; i >= 0; --i) {
        const uint64_t bit = i >= 64 ? (hi >> (i - 64)) & 1 : (lo >> i) & 1;
        const uint64_t c = r >> 63;
        r = (r << 1) | bit;
        if (c || r >= q) r -= q;
    }
    return r;
}

__device__ __forceinline__ uint64_t mont64(uint64_t a, uint64_t b, uint64_t q, uint64_t qinv) {
    const uint64_t lo = a * b, hi = __umul64hi(a, b);
    const uint64_t m = lo * qinv;
    return hi + __umul64hi(m, q) + (lo != 0);
}

__device__ __forceinline__ uint64_t modmul1(uint64_t a, uint64_t b, const ModConsts &m) {
    if (m.fast) {
        a = mod64_slow(a, m.q, m.mu);  // one Barrett step (q < 2^63)
        b = mod64_slow(b, m.q, m.mu);
        uint64_t t = mont64(a, b, m.q, m.qinv);  // a*b*R^-1 in [0, 2q)
        t = mont64(t, m.r2, m.q, m.qinv);        // a*b       in [0, 2q)
        return t >= m.q ? t - m.q : t;
    }
    return mod128_slow(__umul64hi(a, b), a * b, m.q);
}

__global__ void __launch_bounds__(kBlock)
k_modmul(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *__restrict__ c, size_t n,
         ModConsts m) {
    const size_t n2 = n / 2;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a) + i);
        const u64x2 y = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(b) + i);
        u64x2 z;
        z.x = modmul1(x.x, y.x, m);
        z.y = modmul1(x.y, y.y, m);
        __builtin_nontemporal_store(z, reinterpret_cast<u64x2 *>(c) + i);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) c[n - 1] = modmul1(a[n - 1], b[n - 1], m);
}

__device__ __forceinline__ uint64_t addsub1(uint64_t x, uint64_t y, int sub, const ModConsts &m) {
    x = red_any(x, m);
    y = red_any(y, m);
    if (sub) return x >= y ? x - y : m.q - (y - x);
    const uint64_t s = x + y;
    return (s < x || s >= m.q) ? s - m.q : s;
}

__global__ void __launch_bounds__(kBlock)
k_addsub(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *__restrict__ c, size_t n,
         int sub, ModConsts m) {
    const size_t n2 = n / 2;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a) + i);
        const u64x2 y = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(b) + i);
        u64x2 z;
        z.x = addsub1(x.x, y.x, sub, m);
        z.y = addsub1(x.y, y.y, sub, m);
        __builtin_nontemporal_store(z, reinterpret_cast<u64x2 *>(c) + i);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) c[n - 1] = addsub1(a[n - 1], b[n - 1], sub, m);
}

// RNS ring elementwise ops in one launch: limb blockIdx.y of [limbs][per]
// words with that limb's constants; op 0 = pointwise product, 1 = add, 2 = sub.
__global__ void __launch_bounds__(kBlock)
k_ew_limbs(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *__restrict__ c, size_t per,
           int op, const ModConsts *__restrict__ tab) {
    const ModConsts m = tab[blockIdx.y];
    const size_t o = (size_t)blockIdx.y * per, n2 = per / 2;  // per = batch N, even
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a + o) + i);
        const u64x2 y = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(b + o) + i);
        u64x2 z;
        z.x = op == 0 ? modmul1(x.x, y.x, m) : addsub1(x.x, y.x, op == 2, m);
        z.y = op == 0 ? modmul1(x.y, y.y, m) : addsub1(x.y, y.y, op == 2, m);
        __builtin_nontemporal_store(z, reinterpret_cast<u64x2 *>(c + o) + i);
    }
}

__global__ void __launch_bounds__(kBlock)
k_neg(const uint64_t *__restrict__ a, uint64_t *__restrict__ c, size_t n, uint64_t q) {
    const size_t n2 = n / 2;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a) + i);
        u64x2 z;
        z.x = x.x == 0 ? 0 : q - x.x;
        z.y = x.y == 0 ? 0 : q - x.y;
        __builtin_nontemporal_store(z, reinterpret_cast<u64x2 *>(c) + i);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) c[n - 1] = a[n - 1] == 0 ? 0 : q - a[n - 1];
}

__device__ __forceinline__ uint64_t mulsc1(uint64_t x, uint64_t s, uint64_t sp, const ModConsts &m) {
    if (m.q >> 63) return mod128_slow(__umul64hi(x, s), x * s, m.q);
    const uint64_t r = x * s - __umul64hi(x, sp) * m.q;  // Shoup, [0, 2q)
    return r >= m.q ? r - m.q : r;
}

__global__ void __launch_bounds__(kBlock)
k_mul_scalar(const uint64_t *__restrict__ a, uint64_t *__restrict__ c, size_t n, uint64_t s, uint64_t sp,
             ModConsts m) {
    const size_t n2 = n / 2;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a) + i);
        u64x2 z;
        z.x = mulsc1(x.x, s, sp, m);
        z.y = mulsc1(x.y, s, sp, m);
        __builtin_nontemporal_store(z, reinterpret_cast<u64x2 *>(c) + i);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) c[n - 1] = mulsc1(a[n - 1], s, sp, m);
}

// 2-limb Montgomery product exactly as MultiLimbModularArithmetic
// (schoolbook mul_limbs, word-serial reduce with its bounded carry
// propagation, one conditional subtraction).  c = [q0,q1,r0,r1,r2_0,r2_1,qinv]
struct MLConsts { uint64_t q0, q1, qinv; };

__device__ __forceinline__ void mac(uint64_t a, uint64_t b, uint64_t add, uint64_t &carry, uint64_t &out) {
    // out = lo(a*b + add + carry), carry = hi(...)
    const uint64_t lo = a * b, hi = __umul64hi(a, b);
    uint64_t s = lo + add;
    uint64_t c1 = s < lo;
    uint64_t s2 = s + carry;
    c1 += s2 < s;
    out = s2;
    carry = hi + c1;
}

__device__ __forceinline__ u64x2 ml_mont1(u64x2 a, u64x2 b, const MLConsts &c) {
    uint64_t t0, t1, t2, t3, carry;
    // mul_limbs
    carry = 0;
    mac(a.x, b.x, 0, carry, t0);
    mac(a.x, b.y, 0, carry, t1);
    t2 = carry;
    carry = 0;
    mac(a.y, b.x, t1, carry, t1);
    mac(a.y, b.y, t2, carry, t2);
    t3 = carry;
    // reduce, i = 0
    uint64_t m = t0 * c.qinv;
    carry = 0;
    mac(m, c.q0, t0, carry, t0);
    mac(m, c.q1, t1, carry, t1);
    if (carry) { uint64_t s = t2 + carry; carry = s < t2; t2 = s; }
    if (carry) { uint64_t s = t3 + carry; carry = s < t3; t3 = s; }
    // i = 1
    m = t1 * c.qinv;
    carry = 0;
    mac(m, c.q0, t1, carry, t1);
    mac(m, c.q1, t2, carry, t2);
    if (carry) { uint64_t s = t3 + carry; t3 = s; }
    u64x2 r;
    r.x = t2;
    r.y = t3;
    const bool lt = (t3 < c.q1) || (t3 == c.q1 && t2 < c.q0);
    if (!lt) {
        const uint64_t d0 = t2 - c.q0;
        const uint64_t borrow = t2 < c.q0;
        r.x = d0;
        r.y = t3 - c.q1 - borrow;
    }
    return r;
}

__global__ void __launch_bounds__(kBlock)
k_ml_montmul(const u64x2 *__restrict__ a, const u64x2 *__restrict__ b, u64x2 *__restrict__ c,
             size_t n, MLConsts k) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const u64x2 x = __builtin_nontemporal_load(a + i);
        const u64x2 y = __builtin_nontemporal_load(b + i);
        __builtin_nontemporal_store(ml_mont1(x, y, k), c + i);
    }
}

__global__ void __launch_bounds__(kBlock)
k_decompose(const uint64_t *__restrict__ poly, uint64_t *__restrict__ out, uint32_t n, size_t npoly,
            uint32_t base_log, uint32_t level, ModConsts m) {
    const size_t total = (size_t)n * npoly;
    const uint64_t base = 1ull << base_log, mask = base - 1, half = base / 2;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t p = i / n, x = i % n;
        const uint64_t c = poly[i];
        for (uint32_t l = 0; l < level; ++l) {
            const uint32_t shift = (level - 1 - l) * base_log;
            uint64_t d = (c >> shift) & mask;
            if (d > half) {
                d = m.q - (base - d);
                if (d >= m.q) d = mod64_slow(d, m.q, m.mu);
            }
            out[(p * level + l) * n + x] = d;
        }
    }
}

// EncryptionEngine::multiply for NTT-form ciphertexts (encryption.cpp:
// 762-780 without the transforms): c0 = x0 y0, c1 = x0 y1 + x1 y0, c2 = x1 y1
// with pointwise_multiply's exact (a*b) % q and mod_add.
__global__ void __launch_bounds__(kBlock)
k_tensor_ntt(const uint64_t *__restrict__ x, const uint64_t *__restrict__ y, uint64_t *__restrict__ out,
             uint32_t n, size_t batch, ModConsts m) {
    const size_t total = (size_t)n * batch;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t b = i / n, k = i % n;
        const uint64_t x0 = x[(2 * b) * n + k], x1 = x[(2 * b + 1) * n + k];
        const uint64_t y0 = y[(2 * b) * n + k], y1 = y[(2 * b + 1) * n + k];
        const uint64_t c0 = modmul1(x0, y0, m), c2 = modmul1(x1, y1, m);
        const uint64_t c1 = addsub1(modmul1(x0, y1, m), modmul1(x1, y0, m), 0, m);
        out[(3 * b) * n + k] = c0;
        out[(3 * b + 1) * n + k] = c1;
        out[(3 * b + 2) * n + k] = c2;
    }
}

// ---- composed external product / relinearisation (k > 1 or N > 16384) ----
// out[b][j] = sum_r X[b][r] (.) G[r][kj(j)], X canonical NTT-domain digit
// transforms, G prepared keys (NTT x R, R = 2^word): Montgomery products
// remove the R.  kj(j) = j (external product) or K1-1-j (relinearisation:
// c0' uses b_l, c1' uses a_l).  Canonical output.
__device__ __forceinline__ uint64_t mont_word(uint64_t a, uint64_t b, uint64_t q, uint64_t qinv, int word) {
    if (word == 32) {  // a, b < q < 2^30: a*b*2^-32 mod q in [0, 2q)
        const uint64_t p = a * b;
        const uint32_t m = (uint32_t)p * (uint32_t)qinv;
        return (p + (uint64_t)m * q) >> 32;
    }
    if (word == 65) return wmont(a, b, q, qinv);  // q >= 2^62: canonical
    return mont64(a, b, q, qinv);  // [0, 2q) for q < 2^62
}
__global__ void __launch_bounds__(kBlock)
k_mac_keys(const uint64_t *__restrict__ x, const uint64_t *__restrict__ g, uint64_t *__restrict__ out, uint32_t n,
           size_t batch, uint32_t rows, uint32_t k1, int swap, int word, ModConsts m) {
    const size_t total = (size_t)n * batch;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t b = i / n, c = i % n;
        for (uint32_t j = 0; j < k1; ++j) {
            const uint32_t kj = swap ? k1 - 1 - j : j;
            uint64_t acc = 0;
            for (uint32_t r = 0; r < rows; ++r) {
                const uint64_t t = mont_word(x[(b * rows + r) * n + c], g[((size_t)r * k1 + kj) * n + c], m.q, m.qinv, word);
                if (word == 65) {  // canonical terms; the sum may carry out of 64 bits
                    acc = wadd(acc, t, m.q);
                    continue;
                }
                acc += t;  // < 4q
                acc = acc >= 2 * m.q ? acc - 2 * m.q : acc;
            }
            out[(b * k1 + j) * n + c] = acc >= m.q ? acc - m.q : acc;
        }
    }
}
// relinearize's digits (encryption.cpp:920-925): d_l = (c2 >> l B) & (2^B - 1)
// of ct3 [batch][3][n] -> [batch][level][n]
__global__ void __launch_bounds__(kBlock)
k_relin_digits(const uint64_t *__restrict__ ct3, uint64_t *__restrict__ out, uint32_t n, size_t batch,
               uint32_t base_log, uint32_t level) {
    const size_t total = (size_t)n * batch;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t mask = (1ull << base_log) - 1;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t b = i / n, c = i % n;
        const uint64_t w = ct3[(3 * b + 2) * n + c];
        for (uint32_t l = 0; l < level; ++l) out[(b * level + l) * n + c] = (w >> (l * base_log)) & mask;
    }
}
// out[b][j] = mod_add(out[b][j], src[b][j] mod q) for j < rows; out rows
// [batch][rows][n], src rows [batch][src_rows][n]
__global__ void __launch_bounds__(kBlock)
k_add_rows(uint64_t *__restrict__ out, const uint64_t *__restrict__ src, uint32_t n, size_t batch, uint32_t rows,
           uint32_t src_rows, ModConsts m) {
    const size_t total = (size_t)n * batch * rows;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const size_t c = i % n, j = (i / n) % rows, b = i / ((size_t)n * rows);
        const uint64_t a = out[i] < m.q ? out[i] : mod64_slow(out[i], m.q, m.mu);
        const uint64_t y = red_any(src[(b * src_rows + j) * n + c], m);
        const uint64_t s = a + y;
        out[i] = (s < a || s >= m.q) ? s - m.q : s;
    }
}

hipError_t launch_mac_keys(const ModConsts &m, int word, const uint64_t *x, const uint64_t *g, uint64_t *out,
                           uint32_t n, size_t batch, uint32_t rows, uint32_t k1, int swap, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mac_keys, dim3(grid_for((size_t)n * batch)), dim3(kBlock), 0, s, x, g, out, n, batch, rows, k1,
                       swap, word, m);
    return hipGetLastError();
}
hipError_t launch_relin_digits(const uint64_t *ct3, uint64_t *out, uint32_t n, size_t batch, uint32_t base_log,
                               uint32_t level, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_relin_digits, dim3(grid_for((size_t)n * batch)), dim3(kBlock), 0, s, ct3, out, n, batch,
                       base_log, level);
    return hipGetLastError();
}
hipError_t launch_add_rows(const ModConsts &m, uint64_t *out, const uint64_t *src, uint32_t n, size_t batch,
                           uint32_t rows, uint32_t src_rows, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_add_rows, dim3(grid_for((size_t)n * batch * rows)), dim3(kBlock), 0, s, out, src, n, batch,
                       rows, src_rows, m);
    return hipGetLastError();
}

hipError_t launch_tensor_ntt(const ModConsts &m, const uint64_t *x, const uint64_t *y, uint64_t *out, uint32_t n,
                             size_t batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_tensor_ntt, dim3(grid_for((size_t)n * batch)), dim3(kBlock), 0, s, x, y, out, n, batch, m);
    return hipGetLastError();
}

hipError_t launch_modmul(const ModConsts &m, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t n,
                         hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_modmul, dim3(grid_for((n + 1) / 2)), dim3(kBlock), 0, s, a, b, c, n, m);
    return hipGetLastError();
}
hipError_t launch_addsub(const ModConsts &m, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t n, int sub,
                         hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_addsub, dim3(grid_for((n + 1) / 2)), dim3(kBlock), 0, s, a, b, c, n, sub, m);
    return hipGetLastError();
}
hipError_t launch_ew_limbs(const ModConsts *tab, int limbs, const uint64_t *a, const uint64_t *b, uint64_t *c,
                           size_t per, int op, hipStream_t s) {
    if (per == 0) return hipSuccess;
    if ((per & 1) || limbs < 1 || limbs > 65535) return hipErrorInvalidValue;
    const size_t g = grid_for(per / 2), gpl = (g + limbs - 1) / limbs;  // about the usual grid in total
    hipLaunchKernelGGL(k_ew_limbs, dim3((unsigned)(gpl < 1 ? 1 : gpl), (unsigned)limbs), dim3(kBlock), 0, s, a, b, c,
                       per, op, tab);
    return hipGetLastError();
}
hipError_t launch_neg(uint64_t q, const uint64_t *a, uint64_t *c, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_neg, dim3(grid_for((n + 1) / 2)), dim3(kBlock), 0, s, a, c, n, q);
    return hipGetLastError();
}
hipError_t launch_mul_scalar(const ModConsts &m, const uint64_t *a, uint64_t sc, uint64_t sc_shoup, uint64_t *c,
                             size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mul_scalar, dim3(grid_for((n + 1) / 2)), dim3(kBlock), 0, s, a, c, n, sc, sc_shoup, m);
    return hipGetLastError();
}
hipError_t launch_ml_montmul(const uint64_t consts[7], const uint64_t *a, const uint64_t *b, uint64_t *c, size_t n,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    MLConsts k{consts[0], consts[1], consts[6]};
    hipLaunchKernelGGL(k_ml_montmul, dim3(grid_for(n)), dim3(kBlock), 0, s, reinterpret_cast<const u64x2 *>(a),
                       reinterpret_cast<const u64x2 *>(b), reinterpret_cast<u64x2 *>(c), n, k);
    return hipGetLastError();
}
hipError_t launch_decompose(const ModConsts &m, const uint64_t *poly, uint64_t *out, uint32_t n, size_t npoly,
                            uint32_t base_log, uint32_t level, hipStream_t s) {
    if (n == 0 || npoly == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decompose, dim3(grid_for((size_t)n * npoly)), dim3(kBlock), 0, s, poly, out, n, npoly,
                       base_log, level, m);
    return hipGetLastError();
}

}  // namespace FHE_NS
