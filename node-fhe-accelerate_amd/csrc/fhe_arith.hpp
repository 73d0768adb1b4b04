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
// 64 x 64 -> high 64.  Variants (lab flag FHE_MULHI64): 0 = __umul64hi (the
// compiler splits the middle sum into two zero-extended halves: 3 v_mov + a
// 64-bit add per product); 1/2 = 65-bit middle sum in C (the compiler
// recomputes the carry with a 64-bit compare); 3 (default) = the carry-out of
// the v_mad_u64_u32 itself, added with one v_addc.  Measured statically on the
// q62 C3 kernel (k_ntt_fwd_mul<14, u64>): non-multiply VALU 3180 -> 2763 per
// wave, multiplies unchanged (1590), no new scratch anywhere.
#ifndef FHE_MULHI64
#define FHE_MULHI64 3
#endif
__device__ __forceinline__ uint64_t mulhi(uint64_t a, uint64_t b) {
#if FHE_MULHI64 == 4
    // carry-free: every partial sum stays below 2^64 (lo(m1) and hi(m1) are
    // added separately), so no carry flag is written or read
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t m1 = (uint64_t)a1 * b0 + (uint64_t)__umulhi(a0, b0);
    const uint64_t m2 = (uint64_t)a0 * b1 + (uint64_t)(uint32_t)m1;
    const uint64_t h = (uint64_t)a1 * b1 + (m1 >> 32);
    return h + (m2 >> 32);
#elif FHE_MULHI64 == 3
    // The middle sum x0*b1 + (x1*b0 + hi(x0*b0)) reaches 65 bits: its carry
    // comes out of the v_mad_u64_u32 (SGPR pair) and goes into the high word
    // through one v_addc (s_nop 1: VALU-written SGPR read by a VALU).
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t m1 = (uint64_t)a1 * b0 + __umulhi(a0, b0);  // < 2^64
    uint64_t m2, cy;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(m2), "=&s"(cy) : "v"(a0), "v"(b1), "v"(m1));
    const uint64_t h = (uint64_t)a1 * b1 + (m2 >> 32);
    uint32_t hh;
    uint64_t cy2;
    asm("s_nop 1\n\tv_addc_co_u32_e64 %0, %1, %2, 0, %3"
        : "=v"(hh), "=s"(cy2) : "v"((uint32_t)(h >> 32)), "s"(cy));
    (void)cy2;
    return (uint64_t)(uint32_t)h | ((uint64_t)hh << 32);
#elif FHE_MULHI64 == 2
    // middle sum to 65 bits through the carry-out of the 64-bit add
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t m1 = (uint64_t)a1 * b0 + __umulhi(a0, b0);  // < 2^64
    uint64_t m2;
    const bool c = __builtin_add_overflow((uint64_t)a0 * b1, m1, &m2);
    return (uint64_t)a1 * b1 + ((m2 >> 32) | ((uint64_t)c << 32));
#elif FHE_MULHI64
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

// 64-bit word arithmetic without carry / borrow / compare flags (FHE_U64_NOVCC).
// On gfx950 every VALU write of VCC (or of an SGPR pair) that a later VALU
// reads -- the borrow of v_sub_co -> v_subb_co, the v_cmp_lt_u64 -> 2 x
// v_cndmask of a select -- is padded by the hazard recognizer with s_nop
// wait states: 4-5 per 64-bit butterfly in the q62 kernels (653 s_nop in the
// C3 kernel, 1924 in polymul).  Here a 64-bit add is one v_lshl_add_u64, a
// subtraction a - b is a + ~b + 1 (two v_not_b32 + the add, the +1 folded
// into a constant), and the conditional subtraction of k (< 2^63) from
// x (< 2k) selects on the sign bit of x - k with two v_bfi_b32.
#ifndef FHE_U64_NOVCC
#define FHE_U64_NOVCC 0
#endif
// (m & a) | (~m & b) as gfx950's v_bitop3_b32 (LUT 0xe4 over (a, b, m)):
// measured at full rate (111 lane-ops/CU/clk) where v_bfi_b32 issues at
// half rate (63; tools/lab/valu_rates.hip, profiles/r6a/valu_rates_ext.txt).
// Inline asm: written in C, LLVM turns the select of redk64 back into
// compares and v_cndmask (more, half-rate instructions).  FHE_BFI_ASM=1:
// the v_bfi_b32 form.
#ifndef FHE_BFI_ASM
#define FHE_BFI_ASM 0
#endif
__device__ __forceinline__ uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
#if FHE_BFI_ASM
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
#else
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe4" : "=v"(r) : "v"(a), "v"(b), "v"(m));
#endif
    return r;
}
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
// (lo, hi) -> u64 as one register pair (a bit cast, not shifts and ors that
// the compiler may lower to two 64-bit adds)
__device__ __forceinline__ uint64_t pair64(uint32_t lo, uint32_t hi) {
    u32x2v v;
    v.x = lo;
    v.y = hi;
    return __builtin_bit_cast(uint64_t, v);
}
__device__ __forceinline__ uint64_t not64(uint64_t x) {
    uint32_t lo, hi;
    asm("v_not_b32 %0, %1" : "=v"(lo) : "v"((uint32_t)x));
    asm("v_not_b32 %0, %1" : "=v"(hi) : "v"((uint32_t)(x >> 32)));
    return pair64(lo, hi);
}
// A wave-uniform constant the compiler may no longer relate to its source
// (x + launder(-k) stays a v_lshl_add_u64 instead of being folded back into
// a borrow-chain subtraction x - k).
#ifndef FHE_LAUNDER_SGPR
#define FHE_LAUNDER_SGPR 1
#endif
__device__ __forceinline__ uint64_t launder(uint64_t c) {
#if FHE_LAUNDER_SGPR
    asm("" : "+s"(c));
#else
    asm("" : "+r"(c));
#endif
    return c;
}
// x < 2k, k < 2^63: x - k if x >= k else x
__device__ __forceinline__ uint64_t redk64(uint64_t x, uint64_t k) {
    const uint64_t t = x + launder(0ull - k);  // bit 63 set iff x < k
    const uint32_t m = (uint32_t)((int32_t)(uint32_t)(t >> 32) >> 31);
    return pair64(bfi32(m, (uint32_t)x, (uint32_t)t), bfi32(m, (uint32_t)(x >> 32), (uint32_t)(t >> 32)));
}
// a - b + c (mod 2^64) as a + ~b + (c + 1); c + 1 wave-uniform
__device__ __forceinline__ uint64_t sub_add64(uint64_t a, uint64_t b, uint64_t c1) { return a + not64(b) + c1; }

// Lab flags, off by default: the 64-bit Shoup remainder as one mad chain
// (Arith::lo_chain64; a further 2763 -> 2561 on the q62 C3 kernel, but 28 more
// kernels with scratch: negacyclic u64 transforms, k_extprod2, k_dmac), and
// red2q from the borrow of the subtraction (LLVM rebuilds the compare: no
// change).
#ifndef FHE_SHOUP64_CHAIN
#define FHE_SHOUP64_CHAIN 0
#endif
#ifndef FHE_RED64_BORROW
#define FHE_RED64_BORROW 0
#endif

// The reference's 64-bit primes, all of the form q = 2^k - d with d < 2^32
// (parameter_set.cpp:22-42, cpp/tests/test_harness.h:143-147).  A kernel
// instantiated for one of them (key bits 12-13) computes the Shoup remainder's
// h q mod 2^64 as (h << k) - h d: two 32-bit multiplies instead of three.
struct SparsePrime { uint64_t q; uint32_t d, k; };
constexpr SparsePrime kSparsePrimes[4] = {
    {0, 0, 0},
    {4611686018326724609ull, 3u * (1u << 25) - 1u, 62},  // 2^62 - (3 2^25 - 1)
    {1152921504606584833ull, (1u << 18) - 1u, 60},       // Q_60_1 = 2^60 - 2^18 + 1
    {1125899906826241ull, (1u << 14) - 1u, 50},          // Q_50_1 = 2^50 - 2^14 + 1
};

// Twiddle with its Shoup companion w' = floor(w * 2^W / q).
template <typename W> struct Tw { W w, wp; };
// Two Shoup multipliers of a stage-0 butterfly that folds a scaling into
// the stage (Arith::ct_rscale, Arith::gs_scaled): .a for the first
// operand / output, .b for the second (ntt_core.hpp NttArgs).
template <typename W> struct Scale { Tw<W> a, b; };

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
    // index into kSparsePrimes when q is one of them (0: none); read by the
    // host's dispatch only (ntt_core.hpp gk_sparse)
    uint32_t sp;

    // x in [0, 2^W): x*w mod q, lazy result in [0, 2q)   (Shoup)
    template <bool CHAIN = true, int SP = 0>
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
        } else if constexpr (sizeof(W) == 8 && SP != 0) {
            // q = 2^k - d (kSparsePrimes[SP]): -(h q) = h d - (h << k) =
            // h0 d + ((h1 d - (h0 << (k - 32))) << 32)  (mod 2^64)
            constexpr uint32_t d = kSparsePrimes[SP].d, sk = kSparsePrimes[SP].k - 32;
            const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32);
            // h0 d as one v_mad_u64_u32 (d in an SGPR): the C form lets LLVM
            // split it into a mul_lo / mul_hi pair (14194 vs 12999
            // instructions in the q62 polymul)
            uint64_t P, cy;
            asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=&v"(P), "=&s"(cy) : "v"(h0), "s"(d));
            (void)cy;
            const uint32_t ph = (uint32_t)(P >> 32) + h1 * d - (h0 << sk);
            return x * w + pair64((uint32_t)P, ph);
        } else if constexpr (sizeof(W) == 8 && FHE_SHOUP64_CHAIN && CHAIN) {
            return (W)lo_chain64(x, w, h);
        } else if constexpr (sizeof(W) == 8 && FHE_U64_NOVCC) {
            return x * w + h * (W)launder(W(0) - q);  // two low products and one v_lshl_add_u64: no borrow
        } else {
            return x * w - h * q;
        }
    }
    // 64-bit x*w - h*q (mod 2^64) as x*w + h*(2^64 - q): six v_mad_u64_u32
    // and no subtraction.  The two low-word products go through the 64-bit
    // adder of the mad; the four cross products only feed the high word, so
    // they accumulate in the low half of a mad (one instruction each instead
    // of v_mul_lo + v_add3 + the borrow chain of a 64-bit subtract).
    __device__ __forceinline__ uint64_t lo_chain64(uint64_t x, uint64_t w, uint64_t h) const {
        const uint64_t nq = 0ull - (uint64_t)q;
        const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
        const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32);
        const uint32_t n0 = (uint32_t)nq, n1 = (uint32_t)(nq >> 32);
        uint64_t p = (uint64_t)x0 * w0;
        p = (uint64_t)h0 * n0 + p;
        uint32_t acc = madlo(x0, w1, (uint32_t)(p >> 32));
        acc = madlo(x1, w0, acc);
        acc = madlo_s(h0, n1, acc);
        acc = madlo_s(h1, n0, acc);
        return (uint64_t)(uint32_t)p | ((uint64_t)acc << 32);
    }
    // a*b + c (mod 2^32) in one v_mad_u64_u32 (high half of the addend and
    // of the result unused); _s: b wave-uniform.
    static __device__ __forceinline__ uint32_t madlo(uint32_t a, uint32_t b, uint32_t c) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        u32x2 cc;
        cc.x = c;
        uint64_t r, cy;
        asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=&s"(cy) : "v"(a), "v"(b), "v"(cc));
        (void)cy;
        return (uint32_t)r;
    }
    static __device__ __forceinline__ uint32_t madlo_s(uint32_t a, uint32_t b, uint32_t c) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        u32x2 cc;
        cc.x = c;
        uint64_t r, cy;
        asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=&s"(cy) : "v"(a), "s"(b), "v"(cc));
        (void)cy;
        return (uint32_t)r;
    }
    template <int SP = 0>
    __device__ __forceinline__ W shoup(W x, Tw<W> t) const { return shoup<true, SP>(x, t.w, t.wp); }
    // Inverse butterflies keep the plain 64-bit form: with the mad chain the
    // compiler gives the non-negacyclic u64 inverse kernels a 256-byte stack
    // frame (k_ntt_inv / k_polymul <14, u64>).
    template <int SP = 0>
    __device__ __forceinline__ W shoup_inv(W x, Tw<W> t) const { return shoup<false, SP>(x, t.w, t.wp); }

    // Montgomery: a*b*R^-1 mod q in [0, 2q); requires a*b < q*R.
    // 64-bit words (FHE_U64_NOVCC): the signed form (a*b - m*q) / R + q with
    // m = lo(a*b) * q^-1, whose low halves cancel exactly -- no carry from
    // the low half (the `lo != 0` compare) and a flag-free subtraction; the
    // result is congruent and in (0, 2q) (it may differ from the unsigned
    // form by q; every caller reduces or accepts [0, 2q)).
    __device__ __forceinline__ W mont(W a, W b) const {
        W lo = a * b;
        W hi = mulhi(a, b);
        if constexpr (sizeof(W) == 8 && FHE_U64_NOVCC) {
            const W m = lo * (W(0) - qinv);  // qinv = -q^-1: m = lo * q^-1
            return (W)sub_add64(hi, mulhi(m, q), (uint64_t)q + 1);
        } else {
            W m = lo * qinv;
            return hi + mulhi(m, q) + (lo != 0 ? W(1) : W(0));
        }
    }

    __device__ __forceinline__ W red2q(W x) const { return redk(x, q2); }  // [0,4q)->[0,2q)
    __device__ __forceinline__ W red1q(W x) const { return redk(x, q); }   // [0,2q)->[0,q)
    static __device__ __forceinline__ W redk(W x, W k) {
        if constexpr (sizeof(W) == 8 && FHE_U64_NOVCC) {
            return (W)redk64(x, k);
        } else if constexpr (sizeof(W) == 8 && FHE_RED64_BORROW) {
            W d;
            return __builtin_sub_overflow(x, k, &d) ? x : d;
        } else {
            return umin(x, W(x - k));
        }
    }
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
    template <int SP = 0>
    __device__ __forceinline__ void ct(W &x, W &y, Tw<W> t) const {
        W a = red2q(x);
        if constexpr (sizeof(W) == 4 && FHE_NEG_FWD_TW) {
            const W nb = shoup_neg(y, t);
            x = a - nb;
            y = a + nb + q2;
        } else {
            W b = shoup<SP>(y, t);
            x = a + b;
            y = sub2q(a, b);
        }
    }
    // a - b + 2q (b <= 2q): flag-free for 64-bit words
    __device__ __forceinline__ W sub2q(W a, W b) const {
        if constexpr (sizeof(W) == 8 && FHE_U64_NOVCC) return (W)sub_add64(a, b, (uint64_t)q2 + 1);
        else return a - b + q2;
    }
    // Forward butterfly without reducing x: outputs grow by 2q per stage.
    template <int SP = 0>
    __device__ __forceinline__ void ct_lazy(W &x, W &y, Tw<W> t) const {
        W a = x;
        if constexpr (sizeof(W) == 4 && FHE_NEG_FWD_TW) {
            const W nb = shoup_neg(y, t);
            x = a - nb;
            y = a + nb + q2;
        } else {
            W b = shoup<SP>(y, t);
            x = a + b;
            y = a - b + q2;
        }
    }
    // Stage-0 butterfly that also multiplies by R = 2^W (twiddle 1 -> R):
    // puts the transform in Montgomery form for a following pointwise
    // Montgomery product.  Outputs in [0, 4q) for any inputs < 2^W.
    template <int SP = 0>
    __device__ __forceinline__ void ct_rscale(W &x, W &y, Scale<W> r) const {
        W a = shoup<SP>(x, r.a);
        W b = shoup<SP>(y, r.b);
        x = a + b;
        y = sub2q(a, b);
    }
    // Butterflies with twiddle 1 (compat mode, ntt_core.hpp gk_cp): inputs
    // in [0, 4q) (forward) / [0, 2q) (inverse), outputs in the same ranges as
    // ct / gs.
    __device__ __forceinline__ void ct_unit(W &x, W &y) const {
        const W a = red2q(x), b = red2q(y);
        x = a + b;
        y = sub2q(a, b);
    }
    __device__ __forceinline__ void gs_unit(W &x, W &y) const {
        const W s = x + y, d = sub2q(x, y);
        x = red2q(s);
        y = red2q(d);
    }
    // Gentleman-Sande butterfly, values in [0, 2q).
    template <int SP = 0>
    __device__ __forceinline__ void gs(W &x, W &y, Tw<W> t) const {
        W s = x + y;
        W d = sub2q(x, y);
        x = red2q(s);
        y = shoup_inv<SP>(d, t);
    }
    // Last GS stage with the N^-1 scaling folded in (w = 1 at stage 0).
    template <int SP = 0>
    __device__ __forceinline__ void gs_scaled(W &x, W &y, Scale<W> ninv) const {
        W s = x + y;
        W d = sub2q(x, y);
        x = shoup_inv<SP>(s, ninv.a);
        y = shoup_inv<SP>(d, ninv.b);
    }
};

// Exact 64-bit x mod q for any q >= 2 (slow path; taken only for inputs
// outside the lazy range).  mu = floor(2^64 / q).
__device__ __forceinline__ uint64_t mod64_slow(uint64_t x, uint64_t q, uint64_t mu) {
    if (q >> 63) return x >= q ? x - q : x;
    uint64_t r = x - __umul64hi(x, mu) * q;
    return r >= q ? r - q : r;
}

// Moduli up to 2^64 (ntt_wide.hip, the composed key MAC): a * b * 2^-64 mod q, canonical, for a, b < q and any odd q < 2^64:
// (a b + m q) / 2^64 < 2q, and its 65th bit is the carry of the high sum.
__device__ __forceinline__ uint64_t wmont(uint64_t a, uint64_t b, uint64_t q, uint64_t qinv) {
    const uint64_t lo = a * b, hi = __umul64hi(a, b);
    const uint64_t mh = __umul64hi(lo * qinv, q);
    const uint64_t s = hi + mh;
    const bool c1 = s < hi;
    const uint64_t s2 = s + (lo != 0);  // low words: lo + lo(m q) == 0 mod 2^64, carry iff lo != 0
    const bool c2 = s2 < s;
    return (c1 || c2 || s2 >= q) ? s2 - q : s2;
}
__device__ __forceinline__ uint64_t wadd(uint64_t a, uint64_t b, uint64_t q) {
    const uint64_t s = a + b;
    return (s < a || s >= q) ? s - q : s;
}
__device__ __forceinline__ uint64_t wsub(uint64_t a, uint64_t b, uint64_t q) { return a >= b ? a - b : a - b + q; }
// Load a u64 coefficient into the lazy range [0, lim) of word W.
template <typename W>
__device__ __forceinline__ W load_lazy(uint64_t x, uint64_t lim, uint64_t q, uint64_t mu) {
    if (x >= lim) x = mod64_slow(x, q, mu);
    return W(x);
}

}  // namespace FHE_NS
