// lwe_ops.hpp -- scalar helpers shared by the TFHE kernels (ntt_ext.hip,
// lwe.hip): exact mod_add / mod_sub and the monomial rotation of
// BootstrapEngine (bootstrap_engine.cpp).
#pragma once
#include "fhe_arith.hpp"

namespace FHE_NS {

__device__ __forceinline__ uint64_t red_q(uint64_t x, uint64_t q, uint64_t mu) {
    return x < q ? x : mod64_slow(x, q, mu);
}
// ModularArithmetic::mod_add / mod_sub (modular_arithmetic.cpp:122-153) on
// inputs already reduced below q.
__device__ __forceinline__ uint64_t addq(uint64_t a, uint64_t b, uint64_t q) {
    const uint64_t s = a + b;
    return (s < a || s >= q) ? s - q : s;
}
__device__ __forceinline__ uint64_t subq(uint64_t a, uint64_t b, uint64_t q) { return a >= b ? a - b : q - (b - a); }

// blind_rotate's rotation amount (bootstrap_engine.cpp:560): u64 product
// (wraps like the reference), then the int32 cast.
__device__ __forceinline__ int32_t rot_amount(uint64_t a, uint32_t n, uint64_t q) {
    return (int32_t)(uint32_t)((a * (uint64_t)(2u * n) + q / 2) / q);
}
// rotate_polynomial's normalisation to [0, 2N) (bootstrap_engine.cpp:126-127)
__device__ __forceinline__ uint32_t rot_norm(int32_t r, uint32_t n) {
    const int32_t two_n = 2 * (int32_t)n;
    return (uint32_t)(((r % two_n) + two_n) % two_n);
}
// Coefficient p of X^rot * c (rot in [0, 2N)): c[(p - rot) mod 2N] with the
// sign flip of X^N = -1 as (q - x) % q on the raw u64 (rotate_polynomial
// :136-141).
__device__ __forceinline__ uint64_t rotated_at(const uint64_t *c, uint32_t p, uint32_t rot, uint32_t n, uint64_t q,
                                               uint64_t mu) {
    const uint32_t j = (p + 2 * n - rot) & (2 * n - 1);
    if (j < n) return c[j];
    return red_q(q - c[j - n], q, mu);
}

}  // namespace FHE_NS
