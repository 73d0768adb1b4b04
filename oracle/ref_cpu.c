/*
 * oracle/ref_cpu.c -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * backend: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product library (node-fhe-accelerate_amd/csrc) never
 * links, calls or falls back to it.
 *
 * It restates, operation for operation, the reference C++ in
 * /root/reference/cpp/src (Digital-Defiance/node-fhe-accelerate):
 *   - NTTProcessor              ntt_processor.cpp
 *   - ModularArithmetic/Barrett modular_arithmetic.cpp
 *   - MultiLimbModularArithmetic modular_arithmetic.cpp:286-693
 *   - PolynomialRing            polynomial_ring.cpp
 *   - BootstrapEngine pieces    bootstrap_engine.cpp
 * including the reference's "%"-based mod_add/mod_sub and 128-bit "%"
 * products, so that its speed is representative of the reference CPU path
 * (it is the cpu_baseline of bench.py, kind "port").
 *
 * Pinning: the reference cannot be compiled here (modular_arithmetic.h:5
 * includes <arm_neon.h> unconditionally and the image has no such header; a
 * stand-in header is not allowed), so this restatement is pinned by the
 * reference's own known-answer tests and properties (tests/test_oracle.py),
 * the psi table of SURVEY.md section 8 (measured on the compiled reference
 * when the survey was written) and an independent big-integer restatement of
 * the reference's TypeScript restatement (oracle/pyref.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <math.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef uint32_t u32;

/* ------------------------------------------------------------------------
 * Error reporting (the reference throws std::invalid_argument; we return
 * negative codes whose strings match the reference messages).
 * ------------------------------------------------------------------------ */
static const char *k_msgs[] = {
    "ok",
    "Polynomial degree must be a power of 2",          /* ntt_processor.cpp:142 */
    "Polynomial degree must be between 4 and 65536",   /* ntt_processor.cpp:147 */
    "Modulus must be odd",                             /* ntt_processor.cpp:152 */
    "Modulus is not NTT-friendly: q \xe2\x89\xa2 1 (mod 2N)", /* :104 */
    "Coefficient count must equal polynomial degree",  /* ntt_processor.cpp:264 */
    "Could not find primitive root for given parameters", /* :127 */
    "Modulus must be odd and non-zero for Montgomery arithmetic", /* modular_arithmetic.cpp:54 */
    "Modulus must be non-zero for Barrett reduction",  /* modular_arithmetic.cpp:240 */
};
const char *oracle_strerror(int code) {
    int c = code < 0 ? -code : code;
    if (c >= (int)(sizeof(k_msgs) / sizeof(k_msgs[0]))) return "unknown";
    return k_msgs[c];
}

/* ------------------------------------------------------------------------
 * NTTProcessor static helpers (ntt_processor.cpp:25-128)
 * ------------------------------------------------------------------------ */
int oracle_is_power_of_two(u32 n) { return n > 0 && (n & (n - 1)) == 0; } /* :25-27 */

u32 oracle_log2_pow2(u32 n) { /* :29-36 */
    u32 l = 0;
    while (n > 1) { n >>= 1; l++; }
    return l;
}

u32 oracle_bit_reverse(u32 index, u32 bits) { /* :38-45 */
    u32 r = 0;
    for (u32 i = 0; i < bits; i++) { r = (r << 1) | (index & 1); index >>= 1; }
    return r;
}

u64 oracle_mod_pow(u64 base, u64 exp, u64 mod) { /* :47-62 */
    u64 result = 1;
    base %= mod;
    while (exp > 0) {
        if (exp & 1) result = (u64)(((u128)result * base) % mod);
        base = (u64)(((u128)base * base) % mod);
        exp >>= 1;
    }
    return result;
}

/* Signed extended Euclid of ntt_processor.cpp:64-90.  Division by zero (a
 * non-invertible a) traps on x86 in the reference; here it follows AArch64
 * semantics (x/0 = 0, x%0 = x), the platform the reference targets. */
static int64_t sdiv0(int64_t a, int64_t b) { return b == 0 ? 0 : a / b; }
static int64_t smod0(int64_t a, int64_t b) { return b == 0 ? a : a % b; }

int oracle_ntt_mod_inverse(u64 a, u64 m, u64 *out) {
    if (m == 0) return -8; /* "Modulus cannot be zero" */
    if (m == 1) { *out = 0; return 0; }
    int64_t m0 = (int64_t)m;
    int64_t x0 = 0, x1 = 1;
    int64_t as = (int64_t)(a % m);
    int64_t ms = (int64_t)m;
    while (as > 1) {
        int64_t q = sdiv0(as, ms);
        int64_t t = ms;
        ms = smod0(as, ms);
        as = t;
        t = x0;
        x0 = (int64_t)((u64)x1 - (u64)q * (u64)x0);
        x1 = t;
    }
    if (x1 < 0) x1 = (int64_t)((u64)x1 + (u64)m0);
    *out = (u64)x1;
    return 0;
}

/* find_primitive_root (ntt_processor.cpp:92-128): smallest g >= 2 with
 * psi = g^((q-1)/2N), psi^(2N) == 1 and psi^N == q-1. */
int oracle_find_primitive_root(u32 degree, u64 modulus, u64 *out) {
    u64 two_n = (u64)degree * 2;
    if ((modulus - 1) % two_n != 0) return -4;
    u64 e = (modulus - 1) / two_n;
    for (u64 g = 2; g < modulus; g++) {
        u64 w = oracle_mod_pow(g, e, modulus);
        u64 wn = oracle_mod_pow(w, degree, modulus);
        u64 w2n = oracle_mod_pow(w, two_n, modulus);
        if (w2n == 1 && wn == modulus - 1) { *out = w; return 0; }
    }
    return -6;
}

/* ------------------------------------------------------------------------
 * ModularArithmetic (modular_arithmetic.cpp:8-165), including the
 * reference's q_inv = -(q^-1 mod (2^64-1)) constant (modular_arithmetic.cpp:69)
 * ------------------------------------------------------------------------ */

/* modular_arithmetic.cpp:8-31: unsigned a, m; signed x0/x1; m0 = (int64)m.
 * AArch64 division-by-zero semantics as above. */
static u64 ma_mod_inverse(u64 a, u64 m) {
    if (m == 0) return 0;
    int64_t m0 = (int64_t)m;
    int64_t x0 = 0, x1 = 1;
    if (m == 1) return 0;
    while (a > 1) {
        int64_t q = (int64_t)(m == 0 ? 0 : a / m);
        int64_t t = (int64_t)m;
        m = (m == 0) ? a : a % m;
        a = (u64)t;
        t = x0;
        x0 = (int64_t)((u64)x1 - (u64)q * (u64)x0);
        x1 = t;
    }
    if (x1 < 0) x1 = (int64_t)((u64)x1 + (u64)m0);
    return (u64)x1;
}

typedef struct { u64 modulus, r_mod_q, r2_mod_q, q_inv; } mont_consts;

int oracle_mont_constants(u64 q, u64 out[4]) { /* :52-71 */
    if (q == 0 || (q & 1) == 0) return -7;
    u128 r = (u128)1 << 64;
    u64 rq = (u64)(r % q);
    u64 r2 = (u64)(((u128)rq * rq) % q);
    u64 inv = ma_mod_inverse(q, UINT64_MAX);
    out[0] = q; out[1] = rq; out[2] = r2; out[3] = (~inv) + 1;
    return 0;
}

static u64 mont_reduce(const u64 c[4], u64 hi, u64 lo) { /* :84-111 */
    u64 m = lo * c[3];
    u128 mq = (u128)m * c[0];
    u128 sum = ((u128)hi << 64) + lo + mq; /* wraps mod 2^128 like the reference */
    u64 t = (u64)(sum >> 64);
    if (t >= c[0]) t -= c[0];
    return t;
}

u64 oracle_mont_mul(const u64 c[4], u64 a, u64 b) { /* :113-120 */
    u128 p = (u128)a * b;
    return mont_reduce(c, (u64)(p >> 64), (u64)p);
}
u64 oracle_mont_reduce(const u64 c[4], u64 hi, u64 lo) { return mont_reduce(c, hi, lo); }
u64 oracle_to_mont(const u64 c[4], u64 a) { return oracle_mont_mul(c, a, c[2]); }   /* :155-159 */
u64 oracle_from_mont(const u64 c[4], u64 a) { return mont_reduce(c, 0, a); }       /* :161-165 */

/* mod_add / mod_sub (modular_arithmetic.cpp:122-153).  Kept out of line, as
 * in the reference, so the CPU baseline pays the same calls. */
__attribute__((noinline)) u64 oracle_mod_add(u64 q, u64 a, u64 b) {
    a %= q; b %= q;
    u64 s = a + b;
    if (s < a || s >= q) s -= q;
    return s;
}
__attribute__((noinline)) u64 oracle_mod_sub(u64 q, u64 a, u64 b) {
    a %= q; b %= q;
    return a >= b ? a - b : q - (b - a);
}

/* BarrettReducer (modular_arithmetic.cpp:238-280) */
int oracle_barrett_mu(u64 q, u64 *mu) {
    if (q == 0) return -8;
    *mu = (u64)(((u128)1 << 64) / q); /* truncated to 64 bits as in :245-246 */
    return 0;
}
u64 oracle_barrett_reduce(u64 q, u64 mu, u64 x) {
    u64 q2 = (u64)(((u128)x * mu) >> 64);
    u64 r = x - q2 * q;
    if (r >= q) r -= q;
    return r;
}
u64 oracle_barrett_mul(u64 q, u64 mu, u64 a, u64 b) {
    u128 p = (u128)a * b;
    if (p < ((u128)1 << 64)) return oracle_barrett_reduce(q, mu, (u64)p);
    return (u64)(p % q);
}
void oracle_modmul_batch(u64 q, const u64 *a, const u64 *b, u64 *c, size_t n) {
    u64 mu; oracle_barrett_mu(q, &mu);
    for (size_t i = 0; i < n; i++) c[i] = oracle_barrett_mul(q, mu, a[i], b[i]);
}

/* ------------------------------------------------------------------------
 * MultiLimbModularArithmetic with 2 limbs (modular_arithmetic.cpp:286-693)
 * ------------------------------------------------------------------------ */
#define ML_MAX 8
/* multi_limb_mod_proper (:361-429), including its truncated shifted modulus
 * and strict ">" comparison. */
static void ml_mod_proper(const u64 *a, size_t asz, const u64 *mod, size_t nl, u64 *out) {
    u64 rem[ML_MAX];
    size_t rs = asz < nl ? nl : asz;
    memset(rem, 0, sizeof(rem));
    memcpy(rem, a, asz * sizeof(u64));
    /* early return when a < modulus (a.size <= nl && a < modulus) */
    if (asz <= nl) {
        int lt = 0;
        for (size_t i = nl; i > 0; --i) {
            u64 x = (i - 1 < asz) ? a[i - 1] : 0, y = mod[i - 1];
            if (x < y) { lt = 1; break; }
            if (x > y) { lt = 0; break; }
        }
        if (lt) { memset(out, 0, nl * sizeof(u64)); memcpy(out, a, asz * sizeof(u64)); return; }
    }
    for (int bp = (int)(rs * 64) - 1; bp >= 0; --bp) {
        size_t ls = (size_t)bp / 64, bs = (size_t)bp % 64;
        u64 sh[ML_MAX];
        memset(sh, 0, sizeof(sh));
        for (size_t i = 0; i < nl && (i + ls) < rs; ++i) {
            u64 ml = mod[i];
            if (bs == 0) sh[i + ls] = ml;
            else {
                sh[i + ls] |= (ml << bs);
                if (i + ls + 1 < rs) sh[i + ls + 1] = (ml >> (64 - bs));
            }
        }
        int can = 0;
        for (int i = (int)rs - 1; i >= 0; --i) {
            if (rem[i] > sh[i]) { can = 1; break; }
            else if (rem[i] < sh[i]) break;
        }
        if (can) {
            u64 borrow = 0;
            for (size_t i = 0; i < rs; ++i) {
                u64 r = rem[i], s = sh[i];
                u64 d = r - s - borrow;
                borrow = (r < s + borrow) ? 1 : 0;
                rem[i] = d;
            }
        }
    }
    memcpy(out, rem, nl * sizeof(u64));
}

static u64 ml_q_inv_limb(u64 q0) { /* :347-358 */
    u64 x = q0;
    for (int i = 0; i < 5; ++i) x = x * (2 - q0 * x);
    return (~x) + 1;
}

/* out: [q0,q1, r0,r1, r2_0,r2_1, q_inv] */
int oracle_ml_constants(const u64 q[2], u64 out[7]) { /* :471-486 */
    if ((q[0] == 0 && q[1] == 0) || (q[0] & 1) == 0) return -7;
    u64 rl[3] = {0, 0, 1};
    u64 r[2];
    ml_mod_proper(rl, 3, q, 2, r);
    u64 prod[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < 2; ++i) { /* compute_r2_mod_q :443-468 */
        u64 carry = 0;
        for (size_t j = 0; j < 2; ++j) {
            u128 p = (u128)r[i] * r[j];
            p += prod[i + j];
            p += carry;
            prod[i + j] = (u64)p;
            carry = (u64)(p >> 64);
        }
        prod[i + 2] = carry;
    }
    u64 r2[2];
    ml_mod_proper(prod, 4, q, 2, r2);
    out[0] = q[0]; out[1] = q[1]; out[2] = r[0]; out[3] = r[1];
    out[4] = r2[0]; out[5] = r2[1]; out[6] = ml_q_inv_limb(q[0]);
    return 0;
}

/* montgomery_mul (:614-625) = mul_limbs (:525-545) + montgomery_reduce (:558-612) */
void oracle_ml_montmul(const u64 c[7], const u64 a[2], const u64 b[2], u64 r[2]) {
    u64 t[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < 2; ++i) {
        u64 carry = 0;
        for (size_t j = 0; j < 2; ++j) {
            u128 p = (u128)a[i] * b[j];
            p += t[i + j];
            p += carry;
            t[i + j] = (u64)p;
            carry = (u64)(p >> 64);
        }
        t[i + 2] = carry;
    }
    for (size_t i = 0; i < 2; ++i) {
        u64 m = t[i] * c[6];
        u64 carry = 0;
        for (size_t j = 0; j < 2; ++j) {
            u128 p = (u128)m * c[j];
            p += t[i + j];
            p += carry;
            t[i + j] = (u64)p;
            carry = (u64)(p >> 64);
        }
        for (size_t j = 2; j < 4 - i && carry; ++j) {
            u128 s = (u128)t[i + j] + carry;
            t[i + j] = (u64)s;
            carry = (u64)(s >> 64);
        }
    }
    u64 res[2] = {t[2], t[3]};
    int lt = (res[1] < c[1]) || (res[1] == c[1] && res[0] < c[0]);
    if (!lt) {
        u64 borrow = 0;
        for (size_t i = 0; i < 2; ++i) {
            u64 x = res[i], y = c[i];
            u64 d = x - y - borrow;
            borrow = (x < y + borrow) ? 1 : 0;
            res[i] = d;
        }
    }
    r[0] = res[0]; r[1] = res[1];
}

void oracle_ml_montmul_batch(const u64 c[7], const u64 *a, const u64 *b, u64 *r, size_t n) {
    for (size_t i = 0; i < n; i++) oracle_ml_montmul(c, a + 2 * i, b + 2 * i, r + 2 * i);
}

/* ------------------------------------------------------------------------
 * NTTProcessor instance (ntt_processor.cpp:134-208)
 * ------------------------------------------------------------------------ */
typedef struct {
    u32 n, logn;
    u64 q, psi, psi_inv, inv_n;
    u64 *fwd, *inv; /* psi^i, psi^-i for i < n (plain form, :188-205) */
} oracle_ntt;

int oracle_ntt_create(u32 n, u64 q, oracle_ntt **out) {
    if (!oracle_is_power_of_two(n)) return -1;
    if (n < 4 || n > 65536) return -2;
    if ((q & 1) == 0) return -3;
    u64 mc[4];
    if (oracle_mont_constants(q, mc)) return -7; /* ModularArithmetic ctor (:156) */
    oracle_ntt *t = (oracle_ntt *)calloc(1, sizeof(*t));
    t->n = n; t->logn = oracle_log2_pow2(n); t->q = q;
    int rc = oracle_find_primitive_root(n, q, &t->psi);
    if (rc) { free(t); return rc; }
    oracle_ntt_mod_inverse(t->psi, q, &t->psi_inv);
    oracle_ntt_mod_inverse(n, q, &t->inv_n);
    t->fwd = (u64 *)malloc(sizeof(u64) * n);
    t->inv = (u64 *)malloc(sizeof(u64) * n);
    t->fwd[0] = 1; t->inv[0] = 1;
    for (u32 i = 1; i < n; i++) {
        t->fwd[i] = (u64)(((u128)t->fwd[i - 1] * t->psi) % q);
        t->inv[i] = (u64)(((u128)t->inv[i - 1] * t->psi_inv) % q);
    }
    *out = t;
    return 0;
}
void oracle_ntt_destroy(oracle_ntt *t) { if (t) { free(t->fwd); free(t->inv); free(t); } }
u64 oracle_ntt_psi(const oracle_ntt *t) { return t->psi; }
u64 oracle_ntt_inv_n(const oracle_ntt *t) { return t->inv_n; }
void oracle_ntt_tables(const oracle_ntt *t, u64 *fwd, u64 *inv) {
    memcpy(fwd, t->fwd, sizeof(u64) * t->n);
    memcpy(inv, t->inv, sizeof(u64) * t->n);
}

static void bitrev_perm(u64 *c, u32 n) { /* :214-223 */
    u32 bits = oracle_log2_pow2(n);
    for (u32 i = 0; i < n; i++) {
        u32 j = oracle_bit_reverse(i, bits);
        if (i < j) { u64 x = c[i]; c[i] = c[j]; c[j] = x; }
    }
}

/* forward_ntt (ntt_processor.cpp:262-311) */
void oracle_ntt_forward(const oracle_ntt *t, u64 *c) {
    const u32 n = t->n; const u64 q = t->q;
    bitrev_perm(c, n);
    for (u32 s = 0; s < t->logn; s++) {
        u32 m = 1u << s, gs = 2 * m;
        for (u32 k = 0; k < n; k += gs)
            for (u32 j = 0; j < m; j++) {
                u64 w = t->fwd[j * (n / gs)];
                u64 a = c[k + j], b = c[k + j + m];
                u64 wb = (u64)(((u128)w * b) % q);
                c[k + j] = oracle_mod_add(q, a, wb);
                c[k + j + m] = oracle_mod_sub(q, a, wb);
            }
    }
}

/* inverse_ntt (ntt_processor.cpp:325-380) */
void oracle_ntt_inverse(const oracle_ntt *t, u64 *c) {
    const u32 n = t->n; const u64 q = t->q;
    for (int s = (int)t->logn - 1; s >= 0; s--) {
        u32 m = 1u << s, gs = 2 * m;
        for (u32 k = 0; k < n; k += gs)
            for (u32 j = 0; j < m; j++) {
                u64 wi = t->inv[j * (n / gs)];
                u64 a = c[k + j], b = c[k + j + m];
                u64 ap = oracle_mod_add(q, a, b);
                u64 am = oracle_mod_sub(q, a, b);
                c[k + j] = ap;
                c[k + j + m] = (u64)(((u128)am * wi) % q);
            }
    }
    bitrev_perm(c, n);
    for (u32 i = 0; i < n; i++) c[i] = (u64)(((u128)c[i] * t->inv_n) % q);
}

/* forward_ntt_batch / inverse_ntt_batch (:394-408) over a contiguous
 * [batch][n] buffer */
void oracle_ntt_forward_batch(const oracle_ntt *t, u64 *c, size_t batch) {
    for (size_t i = 0; i < batch; i++) oracle_ntt_forward(t, c + i * t->n);
}
void oracle_ntt_inverse_batch(const oracle_ntt *t, u64 *c, size_t batch) {
    for (size_t i = 0; i < batch; i++) oracle_ntt_inverse(t, c + i * t->n);
}

/* ------------------------------------------------------------------------
 * PolynomialRing (polynomial_ring.cpp)
 * ------------------------------------------------------------------------ */
/* pointwise_multiply (:493-530) */
void oracle_pointwise(u64 q, const u64 *a, const u64 *b, u64 *c, size_t n) {
    for (size_t i = 0; i < n; i++) c[i] = (u64)(((u128)a[i] * b[i]) % q);
}
/* add (:263-272, add_neon :372-393) / subtract (:306-315, :395-415) */
void oracle_poly_add(u64 q, const u64 *a, const u64 *b, u64 *c, size_t n) {
    for (size_t i = 0; i < n; i++) c[i] = oracle_mod_add(q, a[i], b[i]);
}
void oracle_poly_sub(u64 q, const u64 *a, const u64 *b, u64 *c, size_t n) {
    for (size_t i = 0; i < n; i++) c[i] = oracle_mod_sub(q, a[i], b[i]);
}
/* negate (:340-355): 0 -> 0, else q - a (u64 wrap for a > q) */
void oracle_poly_neg(u64 q, const u64 *a, u64 *c, size_t n) {
    for (size_t i = 0; i < n; i++) c[i] = a[i] == 0 ? 0 : q - a[i];
}
/* multiply_scalar (:454-473) */
void oracle_poly_mul_scalar(u64 q, const u64 *a, u64 s, u64 *c, size_t n) {
    s %= q;
    for (size_t i = 0; i < n; i++) c[i] = (u64)(((u128)a[i] * s) % q);
}
/* multiply (:421-447) for coefficient-form inputs:
 * inv( fwd(a) (.) fwd(b) ).  Clones a and b as the reference does. */
void oracle_polymul(const oracle_ntt *t, const u64 *a, const u64 *b, u64 *c) {
    const u32 n = t->n;
    u64 *ta = (u64 *)malloc(sizeof(u64) * n), *tb = (u64 *)malloc(sizeof(u64) * n);
    memcpy(ta, a, sizeof(u64) * n); memcpy(tb, b, sizeof(u64) * n);
    oracle_ntt_forward(t, ta);
    oracle_ntt_forward(t, tb);
    oracle_pointwise(t->q, ta, tb, c, n);
    oracle_ntt_inverse(t, c);
    free(ta); free(tb);
}
void oracle_polymul_batch(const oracle_ntt *t, const u64 *a, const u64 *b, u64 *c, size_t batch) {
    for (size_t i = 0; i < batch; i++) oracle_polymul(t, a + i * t->n, b + i * t->n, c + i * t->n);
}
/* to_ntt(a) then pointwise by w (config C3: forward NTT + modmul) */
void oracle_ntt_fwd_mul_batch(const oracle_ntt *t, const u64 *a, const u64 *w, u64 *out, size_t batch) {
    const u32 n = t->n;
    u64 *tmp = (u64 *)malloc(sizeof(u64) * n);
    for (size_t i = 0; i < batch; i++) {
        memcpy(tmp, a + i * n, sizeof(u64) * n);
        oracle_ntt_forward(t, tmp);
        oracle_pointwise(t->q, tmp, w + i * n, out + i * n, n);
    }
    free(tmp);
}

/* ------------------------------------------------------------------------
 * BootstrapEngine pieces (bootstrap_engine.cpp)
 * ------------------------------------------------------------------------ */
/* decompose_polynomial (:152-185): digit l of c; centred as (q-(base-d))%q */
void oracle_decompose(u64 q, const u64 *poly, u32 n, u32 base_log, u32 level, u64 *out /*[level][n]*/) {
    u64 base = 1ULL << base_log, mask = base - 1;
    for (u32 l = 0; l < level; ++l) {
        u32 shift = (level - 1 - l) * base_log;
        for (u32 i = 0; i < n; ++i) {
            u64 d = (poly[i] >> shift) & mask;
            out[(size_t)l * n + i] = d > base / 2 ? (q - (base - d)) % q : d;
        }
    }
}

/* external_product (:431-518), literally: for each row (mask polys first,
 * then body; digit level inner), for each component j (masks, then body):
 * res_j = mod_add(res_j, inv(fwd(decomp) (.) fwd(ggsw[row][j]))).
 * glwe: [(k+1)][n] (k masks then body); ggsw: [(k+1)*level][(k+1)][n] in
 * coefficient form; out: [(k+1)][n]. */
void oracle_external_product(const oracle_ntt *t, u32 k, u32 base_log, u32 level,
                             const u64 *glwe, const u64 *ggsw, u64 *out) {
    const u32 n = t->n; const u64 q = t->q;
    u64 *dec = (u64 *)malloc(sizeof(u64) * n * level);
    u64 *dn = (u64 *)malloc(sizeof(u64) * n);
    u64 *gn = (u64 *)malloc(sizeof(u64) * n);
    u64 *pr = (u64 *)malloc(sizeof(u64) * n);
    memset(out, 0, sizeof(u64) * n * (k + 1));
    u32 row = 0;
    for (u32 i = 0; i <= k; ++i) {
        oracle_decompose(q, glwe + (size_t)i * n, n, base_log, level, dec);
        for (u32 l = 0; l < level; ++l, ++row) {
            memcpy(dn, dec + (size_t)l * n, sizeof(u64) * n);
            oracle_ntt_forward(t, dn);
            for (u32 j = 0; j <= k; ++j) {
                memcpy(gn, ggsw + ((size_t)row * (k + 1) + j) * n, sizeof(u64) * n);
                oracle_ntt_forward(t, gn);
                oracle_pointwise(q, dn, gn, pr, n);
                oracle_ntt_inverse(t, pr);
                for (u32 x = 0; x < n; ++x) out[(size_t)j * n + x] = oracle_mod_add(q, out[(size_t)j * n + x], pr[x]);
            }
        }
    }
    free(dec); free(dn); free(gn); free(pr);
}

/* rotate_polynomial (:122-145): multiply by X^rotation mod X^N+1 */
void oracle_rotate(u64 q, const u64 *p, u32 n, int32_t rotation, u64 *out) {
    int32_t two_n = 2 * (int32_t)n;
    int32_t rot = ((rotation % two_n) + two_n) % two_n;
    memset(out, 0, sizeof(u64) * n);
    for (u32 i = 0; i < n; ++i) {
        int32_t ni = ((int32_t)i + rot) % two_n;
        if (ni < (int32_t)n) out[ni] = p[i];
        else out[ni - n] = (q - p[i]) % q;
    }
}

/* sample_extract (:594-624): a[i*N] = mask_i[0]; a[i*N+j] = (q-mask_i[N-j])%q */
void oracle_sample_extract(u64 q, u32 k, u32 n, const u64 *glwe, u64 *a, u64 *b) {
    for (u32 i = 0; i < k; ++i) {
        const u64 *m = glwe + (size_t)i * n;
        a[(size_t)i * n] = m[0];
        for (u32 j = 1; j < n; ++j) a[(size_t)i * n + j] = (q - m[n - j]) % q;
    }
    *b = glwe[(size_t)k * n];
}

/* cmux (:520-540): diff = ct1 - ct0 (subtract_glwe_inplace -> mod_sub),
 * product = external_product(diff, ggsw), product += ct0 (mod_add). */
void oracle_cmux(const oracle_ntt *t, u32 k, u32 base_log, u32 level, const u64 *ggsw,
                 const u64 *ct0, const u64 *ct1, u64 *out) {
    const size_t m = (size_t)(k + 1) * t->n;
    u64 *diff = (u64 *)calloc(m, sizeof(u64));
    for (size_t x = 0; x < m; ++x) diff[x] = oracle_mod_sub(t->q, ct1[x], ct0[x]);
    oracle_external_product(t, k, base_log, level, diff, ggsw, out);
    for (size_t x = 0; x < m; ++x) out[x] = oracle_mod_add(t->q, out[x], ct0[x]);
    free(diff);
}

/* multiply_glwe_by_monomial (:249-261): every polynomial rotated */
static void glwe_rotate(u64 q, u32 k, u32 n, const u64 *in, int32_t r, u64 *out) {
    for (u32 i = 0; i <= k; ++i) oracle_rotate(q, in + (size_t)i * n, n, r, out + (size_t)i * n);
}

/* blind_rotate (:547-577) of acc [(k+1)][n] in place; lwe_q = lwe_modulus_
 * (= glwe modulus, :39-40); bsk: lwe_dim GGSWs [(k+1)*level][(k+1)][n]. */
void oracle_blind_rotate(const oracle_ntt *t, u32 k, u32 base_log, u32 level, u32 lwe_dim,
                         const u64 *lwe_a, u64 lwe_b, u64 lwe_q, const u64 *bsk, u64 *acc) {
    const u32 n = t->n;
    const size_t m = (size_t)(k + 1) * n, gw = (size_t)(k + 1) * level * (k + 1) * n;
    u64 *rot = (u64 *)malloc(sizeof(u64) * m), *res = (u64 *)malloc(sizeof(u64) * m);
    int32_t b_rotation = -(int32_t)((lwe_b * 2 * n + lwe_q / 2) / lwe_q);
    glwe_rotate(t->q, k, n, acc, b_rotation, rot);
    memcpy(acc, rot, sizeof(u64) * m);
    for (u32 i = 0; i < lwe_dim; ++i) {
        int32_t a_rotation = (int32_t)((lwe_a[i] * 2 * n + lwe_q / 2) / lwe_q);
        if (a_rotation == 0) continue;
        glwe_rotate(t->q, k, n, acc, a_rotation, rot);
        oracle_cmux(t, k, base_log, level, bsk + gw * i, acc, rot, res);
        memcpy(acc, res, sizeof(u64) * m);
    }
    free(rot); free(res);
}

/* key_switch (:626-674): ksk_a [in_dim*level][out_dim] (keys[idx].first),
 * ksk_b [in_dim*level] (keys[idx].second[0]). */
void oracle_key_switch(u64 q, u32 base_log, u32 level, u32 in_dim, u32 out_dim, const u64 *ksk_a,
                       const u64 *ksk_b, const u64 *lwe_a, u64 lwe_b, u64 *out_a, u64 *out_b) {
    u64 base = 1ULL << base_log, mask = base - 1;
    memset(out_a, 0, sizeof(u64) * out_dim);
    u64 rb = lwe_b;
    size_t idx = 0;
    for (u32 i = 0; i < in_dim; ++i) {
        u64 coeff = lwe_a[i];
        for (u32 l = 0; l < level; ++l) {
            u32 shift = (level - 1 - l) * base_log;
            u64 digit = (coeff >> shift) & mask;
            if (digit == 0) { idx++; continue; }
            const u64 *ka = ksk_a + idx * out_dim;
            for (u32 j = 0; j < out_dim; ++j) out_a[j] = (out_a[j] + q - (digit * ka[j]) % q) % q;
            rb = (rb + q - (digit * ksk_b[idx]) % q) % q;
            idx++;
        }
    }
    *out_b = rb;
}

/* EncryptionEngine::multiply (encryption.cpp:737-798): ct [2][n] each;
 * out [3][n].  is_ntt: inputs already in the NTT domain (no transforms). */
void oracle_ct_multiply(const oracle_ntt *t, const u64 *ct1, const u64 *ct2, int is_ntt, u64 *out) {
    const u32 n = t->n; const u64 q = t->q;
    u64 *w = (u64 *)malloc(sizeof(u64) * n * 6);
    u64 *x0 = w, *x1 = w + n, *y0 = w + 2 * n, *y1 = w + 3 * n, *p = w + 4 * n, *r = w + 5 * n;
    memcpy(x0, ct1, 8 * n); memcpy(x1, ct1 + n, 8 * n);
    memcpy(y0, ct2, 8 * n); memcpy(y1, ct2 + n, 8 * n);
    if (!is_ntt) {
        oracle_ntt_forward(t, x0); oracle_ntt_forward(t, x1);
        oracle_ntt_forward(t, y0); oracle_ntt_forward(t, y1);
    }
    oracle_pointwise(q, x0, y0, out, n);                /* c0 */
    oracle_pointwise(q, x0, y1, p, n);                  /* c1 */
    oracle_pointwise(q, x1, y0, r, n);
    oracle_poly_add(q, p, r, out + n, n);
    oracle_pointwise(q, x1, y1, out + 2 * n, n);        /* c2 */
    if (!is_ntt) {
        oracle_ntt_inverse(t, out); oracle_ntt_inverse(t, out + n); oracle_ntt_inverse(t, out + 2 * n);
    }
    free(w);
}

/* EncryptionEngine::relinearize (:904-980) with num_levels key pairs:
 * ct3 [3][n]; rlk [level][2][n] as (a_l, b_l); out [2][n]. */
void oracle_relinearize(const oracle_ntt *t, u32 base_log, u32 level, const u64 *ct3, const u64 *rlk, u64 *out) {
    const u32 n = t->n; const u64 q = t->q;
    u64 base = 1ULL << base_log, mask = base - 1;
    u64 *d = (u64 *)malloc(sizeof(u64) * n * 4);
    u64 *ka = d + n, *kb = d + 2 * n, *pr = d + 3 * n;
    memcpy(out, ct3, 8 * (size_t)n * 2);
    for (u32 l = 0; l < level; ++l) {
        u64 shift = (u64)l * base_log;
        for (u32 i = 0; i < n; ++i) d[i] = (ct3[2 * (size_t)n + i] >> shift) & mask;
        memcpy(ka, rlk + (2 * (size_t)l) * n, 8 * n);
        memcpy(kb, rlk + (2 * (size_t)l + 1) * n, 8 * n);
        oracle_ntt_forward(t, d); oracle_ntt_forward(t, ka); oracle_ntt_forward(t, kb);
        oracle_pointwise(q, d, kb, pr, n);
        oracle_ntt_inverse(t, pr);
        oracle_poly_add(q, out, pr, out, n);
        oracle_pointwise(q, d, ka, pr, n);
        oracle_ntt_inverse(t, pr);
        oracle_poly_add(q, out + n, pr, out + n, n);
    }
    free(d);
}

/* ------------------------------------------------------------------------
 * EncryptionEngine encrypt / decrypt / add_plain (encryption.cpp) with the
 * sampled polynomials (u, e1, e2) supplied by the caller, so the function
 * is deterministic.
 * ------------------------------------------------------------------------ */
/* delta_ = q / t, t = plaintext_modulus or 4 when 0 (encryption.cpp:40-46) */
static u64 ee_t(u64 t) { return t ? t : 4; }
/* encode_packed (:117-131): coeffs[i] = (values[i] * delta) % q, u64 product
 * (wraps); encode_plaintext (:107-115) is the one-value case. */
void oracle_encode(u64 q, u64 t, const u64 *values, u32 n, u64 *out) {
    const u64 delta = q / ee_t(t);
    for (u32 i = 0; i < n; ++i) out[i] = (values[i] * delta) % q;
}
/* encrypt_internal (:171-205): c0 = from_ntt(to_ntt(pk.b) . to_ntt(u)) + e1
 * + m, c1 = from_ntt(to_ntt(pk.a) . to_ntt(u)) + e2 (add_inplace: mod_add).
 * pk [2][n] = (a, b) (PublicKey field order, key_manager.h:70-76);
 * ct out [2][n]. */
void oracle_encrypt(const oracle_ntt *t, u64 pt_mod, const u64 *pk, const u64 *values, const u64 *u,
                    const u64 *e1, const u64 *e2, u64 *ct) {
    const u32 n = t->n; const u64 q = t->q;
    u64 *w = (u64 *)malloc(sizeof(u64) * n * 4);
    u64 *un = w, *pb = w + n, *pa = w + 2 * n, *m = w + 3 * n;
    memcpy(un, u, 8 * (size_t)n); memcpy(pa, pk, 8 * (size_t)n); memcpy(pb, pk + n, 8 * (size_t)n);
    oracle_ntt_forward(t, un); oracle_ntt_forward(t, pa); oracle_ntt_forward(t, pb);
    oracle_encode(q, pt_mod, values, n, m);
    oracle_pointwise(q, pb, un, ct, n);
    oracle_ntt_inverse(t, ct);
    oracle_poly_add(q, ct, e1, ct, n);
    oracle_poly_add(q, ct, m, ct, n);
    oracle_pointwise(q, pa, un, ct + n, n);
    oracle_ntt_inverse(t, ct + n);
    oracle_poly_add(q, ct + n, e2, ct + n, n);
    free(w);
}
/* decrypt (:234-300) + decode_packed (:150-163) + compute_noise_budget
 * (:364-400).  ct [comps][n] (comps 2 or 3); is_ntt as Ciphertext::is_ntt.
 * phase [n] = c0 - c1 s (- c2 s^2); values [n] = round(phase * t / q) % t;
 * *max_noise = max_i |phase_i - round_i * delta| (wrapped at q/2), the
 * integer whose double the reference's budget log2(q / (2 max)) uses. */
void oracle_decrypt(const oracle_ntt *t, u64 pt_mod, const u64 *sk, const u64 *ct, u32 comps, int is_ntt,
                    u64 *values, u64 *phase, u64 *max_noise) {
    const u32 n = t->n; const u64 q = t->q, tt = ee_t(pt_mod), delta = q / tt;
    u64 *w = (u64 *)malloc(sizeof(u64) * n * 5);
    u64 *c1 = w, *s = w + n, *c1s = w + 2 * n, *c0 = w + 3 * n, *tmp = w + 4 * n;
    memcpy(c1, ct + n, 8 * (size_t)n);
    if (!is_ntt) oracle_ntt_forward(t, c1);
    memcpy(s, sk, 8 * (size_t)n);
    oracle_ntt_forward(t, s);
    oracle_pointwise(q, c1, s, c1s, n);
    oracle_ntt_inverse(t, c1s);
    memcpy(c0, ct, 8 * (size_t)n);
    if (is_ntt) oracle_ntt_inverse(t, c0);
    oracle_poly_sub(q, c0, c1s, phase, n);
    if (comps == 3) {
        u64 *s2 = c1, *c2 = c0;  /* reuse */
        oracle_pointwise(q, s, s, s2, n);
        memcpy(c2, ct + 2 * (size_t)n, 8 * (size_t)n);
        if (!is_ntt) oracle_ntt_forward(t, c2);
        oracle_pointwise(q, c2, s2, tmp, n);
        oracle_ntt_inverse(t, tmp);
        oracle_poly_sub(q, phase, tmp, phase, n);
    }
    u64 mx = 0;
    for (u32 i = 0; i < n; ++i) {
        const u64 c = phase[i];
        const u64 rounded = (u64)(((u128)c * tt + q / 2) / q);
        values[i] = rounded % tt;
        const u64 expected = (rounded * delta) % q;
        int64_t noise = c >= expected ? (int64_t)(c - expected) : (int64_t)(expected - c);
        if (noise > (int64_t)(q / 2)) noise = (int64_t)q - noise;
        const u64 a = (u64)(noise < 0 ? -noise : noise);
        if (a > mx) mx = a;
    }
    *max_noise = mx;
    free(w);
}
/* add_plain (:638-665): c0 + encode(values) (to_ntt'd first when the
 * ciphertext is in the NTT domain), c1 copied.  ct, out [2][n]. */
void oracle_add_plain(const oracle_ntt *t, u64 pt_mod, const u64 *ct, const u64 *values, int is_ntt, u64 *out) {
    const u32 n = t->n;
    u64 *m = (u64 *)malloc(sizeof(u64) * n);
    oracle_encode(t->q, pt_mod, values, n, m);
    if (is_ntt) oracle_ntt_forward(t, m);
    oracle_poly_add(t->q, ct, m, out, n);
    memcpy(out + n, ct + n, 8 * (size_t)n);
    free(m);
}
/* BootstrapEngine::bootstrap_with_test_poly (bootstrap_engine.cpp:684-708):
 * acc = (0, .., 0, test_poly); blind_rotate; sample_extract; key_switch
 * with the GLWE modulus.  Out: out_a [out_dim], *out_b. */
void oracle_bootstrap(const oracle_ntt *t, u32 k, u32 base_log, u32 level, u32 lwe_dim, const u64 *lwe_a,
                      u64 lwe_b, u64 lwe_q, const u64 *bsk, const u64 *test_poly, u32 ks_base_log,
                      u32 ks_level, u32 out_dim, const u64 *ksk_a, const u64 *ksk_b, u64 *out_a, u64 *out_b) {
    const u32 n = t->n;
    u64 *acc = (u64 *)calloc((size_t)(k + 1) * n, sizeof(u64));
    u64 *ea = (u64 *)malloc(sizeof(u64) * ((size_t)k * n + 1));
    u64 eb = 0;
    memcpy(acc + (size_t)k * n, test_poly, 8 * (size_t)n);
    oracle_blind_rotate(t, k, base_log, level, lwe_dim, lwe_a, lwe_b, lwe_q, bsk, acc);
    oracle_sample_extract(t->q, k, n, acc, ea, &eb);
    oracle_key_switch(t->q, ks_base_log, ks_level, k * n, out_dim, ksk_a, ksk_b, ea, eb, out_a, out_b);
    free(acc); free(ea);
}

/* ------------------------------------------------------------------------
 * Key material and encryption randomness (key_manager.cpp, bootstrap_engine.cpp)
 * SecureRandom's draws (key_manager.cpp:53-115) are restated over the
 * backend's seeded ChaCha20 stream (include/fhe_gpu.h, FHE_SAMPLE_*): RFC
 * 8439 block function, key = seed[4] as 8 little-endian words, 64-bit block
 * counter (words 12-13), 64-bit nonce = stream (words 14-15); element i of
 * a stream of `count` draws from blocks i, i + count, i + 2 count, ...
 * (8 u64 words per block).  The key formulas follow the reference lines
 * cited at each function, with the reference's u64 / int64 wrap-around.
 * ------------------------------------------------------------------------ */
static u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }
#define CC_QR(a, b, c, d) \
    a += b; d ^= a; d = rotl32(d, 16); c += d; b ^= c; b = rotl32(b, 12); \
    a += b; d ^= a; d = rotl32(d, 8);  c += d; b ^= c; b = rotl32(b, 7);
void oracle_chacha_block(const u64 seed[4], u64 counter, u64 nonce, u64 o[8]) {
    u32 in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int i = 0; i < 4; ++i) { in[4 + 2 * i] = (u32)seed[i]; in[5 + 2 * i] = (u32)(seed[i] >> 32); }
    in[12] = (u32)counter; in[13] = (u32)(counter >> 32); in[14] = (u32)nonce; in[15] = (u32)(nonce >> 32);
    u32 x[16];
    memcpy(x, in, sizeof x);
    for (int r = 0; r < 10; ++r) {
        CC_QR(x[0], x[4], x[8], x[12]) CC_QR(x[1], x[5], x[9], x[13])
        CC_QR(x[2], x[6], x[10], x[14]) CC_QR(x[3], x[7], x[11], x[15])
        CC_QR(x[0], x[5], x[10], x[15]) CC_QR(x[1], x[6], x[11], x[12])
        CC_QR(x[2], x[7], x[8], x[13]) CC_QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 8; ++i) o[i] = (u64)(x[2 * i] + in[2 * i]) | ((u64)(x[2 * i + 1] + in[2 * i + 1]) << 32);
}
#undef CC_QR
typedef struct { const u64 *seed; u64 nonce, idx, count, blk; int pos; u64 buf[8]; } draws_t;
static u64 dr_next(draws_t *d) {
    if (d->pos == 8) { oracle_chacha_block(d->seed, d->idx + d->blk * d->count, d->nonce, d->buf); d->blk++; d->pos = 0; }
    return d->buf[d->pos++];
}
static u64 dr_range(draws_t *d, u64 max) { /* random_u64_range (:60-71) */
    if (max == 0) return 0;
    const u64 thr = (0ULL - max) % max;
    u64 r;
    do r = dr_next(d); while (r < thr);
    return r % max;
}
static double dr_unit(draws_t *d) { return (double)(dr_next(d) >> 11) * 0x1.0p-53; }
/* kind: 0 uniform mod q, 1 ternary, 2 gaussian(std), 3 binary, 4 raw */
void oracle_sample(int kind, const u64 seed[4], u64 stream, u64 q, double std_dev, u64 *out, size_t count) {
    for (size_t i = 0; i < count; ++i) {
        draws_t d = {seed, stream, (u64)i, (u64)count, 0, 8, {0}};
        u64 v;
        switch (kind) {
        case 0: v = dr_range(&d, q); break;
        case 1: { const u64 r = dr_range(&d, 3); v = r == 0 ? q - 1 : (r == 1 ? 0 : 1); break; } /* :73-83 */
        case 2: { /* sample_gaussian (:85-110) */
            double u1 = dr_unit(&d);
            const double u2 = dr_unit(&d);
            while (u1 == 0.0) u1 = dr_unit(&d);
            const double z = sqrt(-2.0 * log(u1)) * cos(2.0 * 3.14159265358979323846 * u2);
            int64_t iv = (int64_t)round(z * std_dev);
            if (iv < 0 && (q >> 63)) {
                /* (int64_t)q < 0: the reference loop ends only when the sum
                 * wraps past INT64_MIN (two's complement wrap, the AArch64
                 * behaviour of its signed overflow); closed form of that
                 * wrapped value (the loop would run ~2^31 times) */
                const u64 m = 0ull - q;
                const u64 k = ((u64)(iv + INT64_MAX) + 1) / m + 1;
                v = ((u64)iv - k * m) % q;
                break;
            }
            if (iv < 0) { iv = (int64_t)q + iv; while (iv < 0) iv += (int64_t)q; }
            v = (u64)iv % q;
            break;
        }
        case 3: v = dr_next(&d) & 1; break;
        default: v = dr_next(&d);
        }
        out[i] = v;
    }
}
/* PolynomialRing product as the key code spells it: from_ntt(to_ntt(a) . to_ntt(b)) */
static void ring_product(const oracle_ntt *t, const u64 *a, const u64 *b, u64 *out) {
    const u32 n = t->n;
    u64 *x = (u64 *)malloc(8 * (size_t)n * 2), *y = x + n;
    memcpy(x, a, 8 * (size_t)n); memcpy(y, b, 8 * (size_t)n);
    oracle_ntt_forward(t, x); oracle_ntt_forward(t, y);
    oracle_pointwise(t->q, x, y, out, n);
    oracle_ntt_inverse(t, out);
    free(x);
}
/* generate_public_key (key_manager.cpp:218-246): pk [2][n] = (a, a*s + e);
 * a uniform (stream), e gaussian (stream + 1) */
void oracle_public_key_generate(const oracle_ntt *t, const u64 *sk, const u64 seed[4], u64 stream, double std_dev,
                                u64 *pk) {
    const u32 n = t->n;
    u64 *e = (u64 *)malloc(8 * (size_t)n);
    oracle_sample(0, seed, stream, t->q, 0, pk, n);
    oracle_sample(2, seed, stream + 1, t->q, std_dev, e, n);
    ring_product(t, pk, sk, pk + n);
    oracle_poly_add(t->q, pk + n, e, pk + n, n);
    free(e);
}
/* generate_eval_key (:252-333): s2 = s*s; level l: a uniform (stream + 2l),
 * e gaussian (stream + 2l + 1), b = a*s + e + multiply_scalar(s2, power),
 * power = (power * base) % q with the u64 product */
void oracle_eval_key_generate(const oracle_ntt *t, const u64 *sk, u32 base_log, u32 level, const u64 seed[4],
                              u64 stream, double std_dev, u64 *rlk) {
    const u32 n = t->n; const u64 q = t->q;
    u64 *w = (u64 *)malloc(8 * (size_t)n * 3), *s2 = w, *e = w + n, *sc = w + 2 * n;
    ring_product(t, sk, sk, s2);
    const u64 base = 1ULL << base_log;
    u64 power = 1;
    for (u32 l = 0; l < level; ++l) {
        u64 *a = rlk + (size_t)2 * l * n, *b = a + n;
        oracle_sample(0, seed, stream + 2 * l, q, 0, a, n);
        oracle_sample(2, seed, stream + 2 * l + 1, q, std_dev, e, n);
        ring_product(t, a, sk, b);
        oracle_poly_add(q, b, e, b, n);
        oracle_poly_mul_scalar(q, s2, power, sc, n);
        oracle_poly_add(q, b, sc, b, n);
        power = (power * base) % q;
    }
    free(w);
}
/* encrypt_ggsw (bootstrap_engine.cpp:268-306) for count values: out
 * [count][(k+1)L][k+1][n].  Row r = row*L + l of value c is
 * encrypt_glwe_zero (:190-227): masks uniform (stream, element
 * ((c (k+1)L + r) k + i) n + j), error (stream + 1, element (c (k+1)L + r) n
 * + j), body = 0 + sum_i mask_i * s (mod_add) + e; then the gadget
 * (|v| q) >> ((l+1) B) (negated mod q for v < 0) added (% q) to coefficient
 * 0 of mask[row] (row < k) or the body.  Shift counts mod 64. */
void oracle_ggsw_encrypt(const oracle_ntt *t, u32 k, u32 base_log, u32 level, const int64_t *values, size_t count,
                         const u64 *sk, const u64 seed[4], u64 stream, double std_dev, u64 *out) {
    const u32 n = t->n; const u64 q = t->q;
    const size_t rows = count * (k + 1) * level;
    u64 *masks = (u64 *)malloc(8 * rows * k * n), *err = (u64 *)malloc(8 * rows * n);
    u64 *prod = (u64 *)malloc(8 * (size_t)n);
    oracle_sample(0, seed, stream, q, 0, masks, rows * k * n);
    oracle_sample(2, seed, stream + 1, q, std_dev, err, rows * n);
    for (size_t r = 0; r < rows; ++r) {
        const size_t c = r / ((k + 1) * level);
        const u32 rr = (u32)(r % ((k + 1) * level)), grp = rr / level, l = rr % level;
        u64 *o = out + r * (k + 1) * n, *body = o + (size_t)k * n;
        memset(body, 0, 8 * (size_t)n);
        for (u32 i = 0; i < k; ++i) {
            memcpy(o + (size_t)i * n, masks + (r * k + i) * n, 8 * (size_t)n);
            ring_product(t, o + (size_t)i * n, sk, prod);
            oracle_poly_add(q, body, prod, body, n);
        }
        oracle_poly_add(q, body, err + r * n, body, n);
        const int64_t v = values[c];
        const u64 av = v < 0 ? (u64)0 - (u64)v : (u64)v;
        u64 g = (av * q) >> (((l + 1) * base_log) & 63);
        if (v < 0) g = (q - g) % q;
        if (grp < k) o[(size_t)grp * n] = (o[(size_t)grp * n] + g) % q;
        else body[0] = (body[0] + g) % q;
    }
    free(masks); free(err); free(prod);
}
/* generate_key_switch_key (:367-420): entry e = i L + l: a_e uniform
 * (stream, element e*lwe_dim + j), error (stream + 1, element e; std_dev 0
 * selects 3.2), b_e = ((u64)((ip + err) % (int64)q) + gadget) % q */
void oracle_ksk_generate(u64 q, u32 base_log, u32 level, const u64 *glwe_sk, u32 n_in, const int64_t *lwe_sk,
                         u32 lwe_dim, const u64 seed[4], u64 stream, double std_dev, u64 *ksk_a, u64 *ksk_b) {
    const size_t entries = (size_t)n_in * level;
    u64 *err = (u64 *)malloc(8 * (entries ? entries : 1));
    oracle_sample(0, seed, stream, q, 0, ksk_a, entries * lwe_dim);
    oracle_sample(2, seed, stream + 1, q, std_dev > 0 ? std_dev : 3.2, err, entries);
    for (size_t e = 0; e < entries; ++e) {
        const u32 i = (u32)(e / level), l = (u32)(e % level);
        u64 ip = 0; /* int64 accumulation, wrapping */
        for (u32 j = 0; j < lwe_dim; ++j) ip += ksk_a[e * lwe_dim + j] * (u64)lwe_sk[j];
        int64_t ev = (int64_t)err[e];
        if (ev > (int64_t)(q / 2)) ev -= (int64_t)q;
        const u64 gadget = (glwe_sk[i] * q) >> (((l + 1) * base_log) & 63);
        const int64_t sm = (int64_t)(ip + (u64)ev);
        ksk_b[e] = ((u64)(sm % (int64_t)q) + gadget) % q;
    }
    free(err);
}
/* LWE decryption: phase = b - sum_j a_j s_j mod q, value = round(phase t / q) % t */
void oracle_lwe_decrypt(u64 q, u64 t, const int64_t *sk, u32 dim, const u64 *a, u64 b, u64 *value, u64 *phase) {
    u64 s = 0;
    for (u32 j = 0; j < dim; ++j) {
        const u64 mag = (u64)(sk[j] < 0 ? -(u128)sk[j] : (u128)sk[j]) % q;
        const u64 kq = sk[j] < 0 && mag ? q - mag : mag;
        s = (u64)(((u128)s + (u64)((u128)(a[j] % q) * kq % q)) % q);
    }
    const u64 p = (b % q + q - s) % q;
    if (phase) *phase = p;
    if (value) *value = (u64)(((u128)p * ee_t(t) + q / 2) / q) % ee_t(t);
}

/* ------------------------------------------------------------------------
 * Test-input generators
 * ------------------------------------------------------------------------ */
/* std::mt19937_64 (used by TestRandom, cpp/tests/test_harness.h:29-73);
 * uniform_int_distribution<uint64_t>(0, UINT64_MAX) returns the raw draw. */
typedef struct { u64 mt[312]; int idx; } mt64;
static void mt64_seed(mt64 *s, u64 seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 312; i++)
        s->mt[i] = 6364136223846793005ULL * (s->mt[i - 1] ^ (s->mt[i - 1] >> 62)) + (u64)i;
    s->idx = 312;
}
static u64 mt64_next(mt64 *s) {
    if (s->idx >= 312) {
        for (int i = 0; i < 312; i++) {
            u64 x = (s->mt[i] & 0xFFFFFFFF80000000ULL) | (s->mt[(i + 1) % 312] & 0x7FFFFFFFULL);
            u64 xa = x >> 1;
            if (x & 1) xa ^= 0xB5026F5AA96619E9ULL;
            s->mt[i] = s->mt[(i + 156) % 312] ^ xa;
        }
        s->idx = 0;
    }
    u64 y = s->mt[s->idx++];
    y ^= (y >> 29) & 0x5555555555555555ULL;
    y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
    y ^= (y << 37) & 0xFFF7EEE000000000ULL;
    y ^= (y >> 43);
    return y;
}
/* TestRandom(seed).next_coefficient(q) repeated count times */
void oracle_testrandom_coeffs(u64 seed, u64 q, u64 *out, size_t count) {
    mt64 s; mt64_seed(&s, seed);
    for (size_t i = 0; i < count; i++) out[i] = q ? mt64_next(&s) % q : 0;
}
void oracle_mt19937_64_raw(u64 seed, u64 *out, size_t count) {
    mt64 s; mt64_seed(&s, seed);
    for (size_t i = 0; i < count; i++) out[i] = mt64_next(&s);
}
/* splitmix64(seed ^ index) % q (SURVEY.md 8(d) synthetic inputs) */
static inline u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
void oracle_splitmix_fill(u64 seed, u64 q, u64 *out, size_t count, size_t offset) {
    for (size_t i = 0; i < count; i++) {
        u64 v = splitmix64(seed ^ (u64)(offset + i));
        out[i] = q ? v % q : v;
    }
}

/* ------------------------------------------------------------------------
 * Multithreaded batch driver for the CPU baseline: contiguous chunks, one
 * std::thread-equivalent per core sharing the read-only processor, as in
 * encryption.cpp:472, 520-533.
 * op: 0 = forward, 1 = inverse, 2 = polymul, 3 = forward + pointwise by w
 * ------------------------------------------------------------------------ */
typedef struct {
    const oracle_ntt *t; int op;
    u64 *a; const u64 *b; u64 *c;
    size_t lo, hi;
} job_t;
static void *job_run(void *p) {
    job_t *j = (job_t *)p;
    const u32 n = j->t->n;
    for (size_t i = j->lo; i < j->hi; i++) {
        u64 *ai = j->a + i * n;
        switch (j->op) {
        case 0: oracle_ntt_forward(j->t, ai); break;
        case 1: oracle_ntt_inverse(j->t, ai); break;
        case 2: oracle_polymul(j->t, ai, j->b + i * n, j->c + i * n); break;
        case 3: oracle_ntt_fwd_mul_batch(j->t, ai, j->b + i * n, j->c + i * n, 1); break;
        }
    }
    return NULL;
}
int oracle_batch_threaded(const oracle_ntt *t, int op, u64 *a, const u64 *b, u64 *c,
                          size_t batch, int threads) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > batch) threads = (int)(batch ? batch : 1);
    pthread_t th[256];
    job_t jobs[256];
    if (threads > 256) threads = 256;
    size_t per = (batch + threads - 1) / threads;
    for (int i = 0; i < threads; i++) {
        jobs[i].t = t; jobs[i].op = op; jobs[i].a = a; jobs[i].b = b; jobs[i].c = c;
        jobs[i].lo = (size_t)i * per;
        jobs[i].hi = jobs[i].lo + per > batch ? batch : jobs[i].lo + per;
        if (jobs[i].lo > batch) jobs[i].lo = batch;
        pthread_create(&th[i], NULL, job_run, &jobs[i]);
    }
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    return 0;
}
