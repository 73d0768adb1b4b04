// fhe_arith.hpp -- modular arithmetic for the gfx950 kernels.
//
// Two word sizes share one interface (struct Arith<W>):
//   W = uint32_t : q < 2^30   (Harvey lazy butterflies need 4q < 2^32)
//   W = uint64_t : q < 2^62   (4q < 2^64)
// Coefficients stay in HBM as u64 in both cases (the reference's
// Polynomial layout, polynomial_ring.h:31-93); the 32-bit path only narrows
// registers and LDS.
//
// All reductions are exact over Z_q, so canonical outputs are bit-identical
// to the reference's "%"-based arithmetic (ntt_processor.cpp:298-307,
// polynomial_ring.cpp:512-526) even though the operation sequence differs.
#pragma once
// Kernel namespace; lab A/B builds override it so variants can share a process.
#ifndef FHE_NS
#define FHE_NS fhe
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace FHE_NS {

__device__ __forceinline__ uint32_t mulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }
// 64 x 64 -> high 64.  FHE_MULHI64=1: the middle partial products summed with
// a 65-bit carry (two full-width mads) instead of two zero-extended halves
// (the compiler builds those pairs with 3 v_mov per product).
#ifndef FHE_MULHI64
#define FHE_MULHI64 0
#endif
__device__ __forceinline__ uint64_t mulhi(uint64_t a, uint64_t b) {
#if FHE_MULHI64
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t m1 = (uint64_t)a1 * b0 + __umulhi(a0, b0);             // < 2^64
    const unsigned __int128 m2 = (unsigned __int128)((uint64_t)a0 * b1) + m1;  // < 2^65
    return (uint64_t)a1 * b1 + (uint64_t)(m2 >> 32);
#else
    return __umul64hi(a, b);
#endif
}
// unsigned min: x - k wraps above x when x < k, so min() keeps x.
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umin(uint64_t a, uint64_t b) { return a < b ? a : b; }

// Twiddle with its Shoup companion w' = floor(w * 2^W / q).
template <typename W> struct Tw { W w, wp; };

// 32-bit forward (CT) twiddle tables hold -w mod 2^32 in Tw::w (Arith::ct).
#ifndef FHE_NEG_FWD_TW
#define FHE_NEG_FWD_TW 1
#endif
constexpr bool kNegFwdTw = FHE_NEG_FWD_TW;

template <typename W>
struct Arith {
    W q, q2;      // q, 2q
    W qinv;       // -q^-1 mod 2^W (Montgomery)
    W r2;         // R^2 mod q, R = 2^W

    // x in [0, 2^W): x*w mod q, lazy result in [0, 2q)   (Shoup)
    __device__ __forceinline__ W shoup(W x, W w, W wp) const {
        W h = mulhi(x, wp);
#ifndef FHE_SHOUP_MAD
#define FHE_SHOUP_MAD 1
#endif
#ifndef FHE_SHOUP_ASM
#define FHE_SHOUP_ASM 1
#endif
#ifndef FHE_MAD_EARLYCLOBBER
#define FHE_MAD_EARLYCLOBBER 1
#endif
        if constexpr (sizeof(W) == 4 && FHE_SHOUP_ASM) {
            // One v_mad_u64_u32 for x*w - h*q (mod 2^32): LLVM narrows the
            // 64-bit form below to two v_mul_lo_u32 + v_sub.  Only the low
            // half of the addend matters, so its high half is left undefined
            // (no zeroing move).
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            // Early-clobber destination: with dst overlapping the addend the
            // hazard recognizer pads every such mad with an s_nop (measured:
            // 1 per butterfly).
            u32x2 c;
            c.x = x * w;
            uint64_t r, cy;
#if FHE_MAD_EARLYCLOBBER
            asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=&s"(cy) : "v"(h), "s"(0u - q), "v"(c));
#else
            asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cy) : "v"(h), "s"(0u - q), "v"(c));
#endif
            (void)cy;
            return (W)r;
        } else if constexpr (sizeof(W) == 4 && FHE_SHOUP_MAD) {
            // x*w - h*q (mod 2^32) as one v_mad_u64_u32: h*(2^32 - q) + x*w
            return (W)((uint64_t)h * (uint32_t)(0u - q) + (uint32_t)(x * w));
        } else {
            return x * w - h * q;
        }
    }
    __device__ __forceinline__ W shoup(W x, Tw<W> t) const { return shoup(x, t.w, t.wp); }

    // Montgomery: a*b*R^-1 mod q in [0, 2q); requires a*b < q*R.
    __device__ __forceinline__ W mont(W a, W b) const {
        W lo = a * b;
        W hi = mulhi(a, b);
        W m = lo * qinv;
        return hi + mulhi(m, q) + (lo != 0 ? W(1) : W(0));
    }

    __device__ __forceinline__ W red2q(W x) const { return umin(x, W(x - q2)); }  // [0,4q)->[0,2q)
    __device__ __forceinline__ W red1q(W x) const { return umin(x, W(x - q)); }   // [0,2q)->[0,q)
    __device__ __forceinline__ W canon4(W x) const { return red1q(red2q(x)); }     // [0,4q)->[0,q)

    // 32-bit forward twiddles are stored negated, {-w mod 2^32, w'}
    // (kNegFwdTw): one v_mad_u64_u32 then yields nb = h*q - y*w = -b (mod
    // 2^32), and the butterfly is x - nb, x + nb + 2q: a v_sub and a v_add3
    // instead of an add, a sub and an add.
    __device__ __forceinline__ W shoup_neg(W y, Tw<W> t) const {
        const W h = mulhi(y, t.wp);
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        u32x2 c;
        c.x = y * t.w;  // y * (-w)
        uint64_t r, cy;
        asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=&s"(cy) : "v"(h), "s"(q), "v"(c));
        (void)cy;
        return (W)r;
    }
    // Harvey forward (Cooley-Tukey) butterfly, values in [0, 4q).
    __device__ __forceinline__ void ct(W &x, W &y, Tw<W> t) const {
        W a = red2q(x);
        if constexpr (sizeof(W) == 4 && FHE_NEG_FWD_TW) {
            const W nb = shoup_neg(y, t);
            x = a - nb;
            y = a + nb + q2;
        } else {
            W b = shoup(y, t);
            x = a + b;
            y = a - b + q2;
        }
    }
    // Forward butterfly without reducing x: outputs grow by 2q per stage.
    __device__ __forceinline__ void ct_lazy(W &x, W &y, Tw<W> t) const {
        W a = x;
        if constexpr (sizeof(W) == 4 && FHE_NEG_FWD_TW) {
            const W nb = shoup_neg(y, t);
            x = a - nb;
            y = a + nb + q2;
        } else {
            W b = shoup(y, t);
            x = a + b;
            y = a - b + q2;
        }
    }
    // Stage-0 butterfly that also multiplies by R = 2^W (twiddle 1 -> R):
    // puts the transform in Montgomery form for a following pointwise
    // Montgomery product.  Outputs in [0, 4q) for any inputs < 2^W.
    __device__ __forceinline__ void ct_rscale(W &x, W &y, Tw<W> r) const {
        W a = shoup(x, r);
        W b = shoup(y, r);
        x = a + b;
        y = a - b + q2;
    }
    // Gentleman-Sande butterfly, values in [0, 2q).
    __device__ __forceinline__ void gs(W &x, W &y, Tw<W> t) const {
        W s = x + y;
        W d = x - y + q2;
        x = red2q(s);
        y = shoup(d, t);
    }
    // Last GS stage with the N^-1 scaling folded in (w = 1 at stage 0).
    __device__ __forceinline__ void gs_scaled(W &x, W &y, Tw<W> ninv) const {
        W s = x + y;
        W d = x - y + q2;
        x = shoup(s, ninv);
        y = shoup(d, ninv);
    }
};

// Exact 64-bit x mod q for any q >= 2 (slow path; taken only for inputs
// outside the lazy range).  mu = floor(2^64 / q).
__device__ __forceinline__ uint64_t mod64_slow(uint64_t x, uint64_t q, uint64_t mu) {
    if (q >> 63) return x >= q ? x - q : x;
    uint64_t r = x - __umul64hi(x, mu) * q;
    return r >= q ? r - q : r;
}

// Load a u64 coefficient into the lazy range [0, lim) of word W.
template <typename W>
__device__ __forceinline__ W load_lazy(uint64_t x, uint64_t lim, uint64_t q, uint64_t mu) {
    if (x >= lim) x = mod64_slow(x, q, mu);
    return W(x);
}

}  // namespace FHE_NS
