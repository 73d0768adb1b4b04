/*
 * fhe_gpu.h -- C ABI of the MI355X (gfx950) FHE polynomial-arithmetic
 * backend (libfhe_gpu.so).  Drop-in replacement for the compute path of
 * Digital-Defiance/node-fhe-accelerate: NTTProcessor, PolynomialRing,
 * ModularArithmetic / BarrettReducer / MultiLimbModularArithmetic and
 * BootstrapEngine::external_product, plus the N-API-visible
 * ModularArithmetic class and detectHardware().
 *
 * Conventions
 *   - Plain C: pointers + sizes, no C++ or torch types, no exceptions.
 *   - Every function returns FHE_OK (0) or a negative FHE_ERR_* code; the
 *     message (the reference's exception text where one exists) is
 *     available from fhe_last_error() (thread-local).
 *   - Polynomial data: contiguous row-major [batch][n] uint64 (the layout of
 *     the reference's Polynomial / Metal buffers, metal_compute.mm:400-410).
 *     Inputs may be any u64 and behave as x mod q (every reference path
 *     reduces); outputs are canonical residues in [0, q).
 *   - where = FHE_DEVICE: pointers are device (HBM) pointers of the context's
 *     device, work is enqueued on the context stream and NOT synchronised.
 *     where = FHE_HOST: pointers are host memory; the call stages through
 *     device scratch and returns after the result is back in host memory.
 *   - A context is immutable after creation (except its stream); concurrent
 *     calls on distinct buffers are safe, as with the reference's shared
 *     read-only NTTProcessor (encryption.cpp:520-533).
 */
#ifndef FHE_GPU_H
#define FHE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FHE_GPU_ABI_VERSION 1

/* ---- status codes (messages mirror the reference's std::invalid_argument) */
#define FHE_OK 0
#define FHE_ERR_DEGREE_POW2 (-1)     /* "Polynomial degree must be a power of 2"      ntt_processor.cpp:142 */
#define FHE_ERR_DEGREE_RANGE (-2)    /* "Polynomial degree must be between 4 and 65536" ntt_processor.cpp:147 */
#define FHE_ERR_MODULUS_EVEN (-3)    /* "Modulus must be odd"                          ntt_processor.cpp:152 */
#define FHE_ERR_NOT_NTT_FRIENDLY (-4) /* "Modulus is not NTT-friendly: q != 1 (mod 2N)" ntt_processor.cpp:104 */
#define FHE_ERR_COUNT (-5)           /* "Coefficient count must equal polynomial degree" ntt_processor.cpp:264 */
#define FHE_ERR_NO_ROOT (-6)         /* "Could not find primitive root ..."            ntt_processor.cpp:127 */
#define FHE_ERR_MONT_MODULUS (-7)    /* "Modulus must be odd and non-zero for Montgomery arithmetic" modular_arithmetic.cpp:54 */
#define FHE_ERR_ZERO_MODULUS (-8)    /* "Modulus must be non-zero for Barrett reduction" modular_arithmetic.cpp:240 */
#define FHE_ERR_INVALID_ARG (-9)
#define FHE_ERR_UNSUPPORTED (-10)    /* parameter outside what the GPU kernels implement */
#define FHE_ERR_DEVICE (-11)         /* HIP runtime error / no device */
#define FHE_ERR_OOM (-12)

#define FHE_MODE_COMPAT 0      /* the reference's transform, bit-exact */
#define FHE_MODE_NEGACYCLIC 1  /* psi-twisted cyclic NTT: polymul == a*b mod (X^N+1) */

#define FHE_HOST 0
#define FHE_DEVICE 1

typedef struct fhe_ctx fhe_ctx;

/* Thread-local message of the last failing call on this thread. */
const char *fhe_last_error(void);
const char *fhe_version(void);
/* Hash of the sources and flags this library was built from (16 hex
 * digits).  Profiles under profiles/ are stamped with it; bench.py uses a
 * PMC traffic figure only when it matches the loaded library.  No reference
 * counterpart (measurement plumbing). */
const char *fhe_build_id(void);

/* ---- hardware ------------------------------------------------------------
 * Replaces HardwareDetector::detect() (hardware_detector.mm; N-API
 * detectHardware(), src/native/lib.rs:123-127, index.d.ts:22-30).          */
typedef struct {
    int32_t device_count;
    int32_t compute_units;     /* of device 0 */
    int32_t wavefront_size;
    int32_t xcds;
    uint64_t hbm_bytes;        /* of device 0 */
    uint64_t lds_bytes_per_cu;
    char arch[32];             /* "gfx950" */
    char name[96];
} fhe_hw_caps;
int fhe_detect(fhe_hw_caps *caps);

/* ---- context: NTTProcessor(degree, modulus) + PolynomialRing(degree, q)
 * (ntt_processor.cpp:134-208, polynomial_ring.cpp:213-222).
 * Validation order and messages follow the reference constructor.  n must
 * be a power of two in [4, 65536]; the GPU kernels implement every such n
 * and every odd q whose root search succeeds: q < 2^62 in the lazy kernel
 * family, 2^62 <= q < 2^64 in the canonical one (ntt_wide.hip; there
 * encrypt / decrypt / add_plain are composed from batched transforms,
 * engine_composed.hip, as they are for n > 16384, and
 * compat mode keeps the reference's psi^-1 and N^-1, which are not inverses
 * at q >= 2^63, ntt_processor.cpp:63-89).  n > 16384 runs as a
 * two-pass row/column split and the context holds 512 MiB of device
 * scratch (every entry point takes such contexts: fused kernels up to
 * n = 16384, composed ones above).
 * device: HIP device ordinal.
 * Side effect: call temporaries come from the device's default
 * stream-ordered memory pool, and creating a context sets that pool's
 * release threshold to FHE_POOL_KEEP_MB MiB (environment, default 8192), so
 * up to that much freed memory stays cached across synchronisations.  The
 * pool is process-wide (other HIP users of the device share it);
 * FHE_POOL_KEEP_MB=0 leaves it unchanged.                                   */
int fhe_ctx_create(uint32_t n, uint64_t q, int mode, int device, fhe_ctx **out);
void fhe_ctx_destroy(fhe_ctx *ctx);
/* Multi-device context (SURVEY.md 8(b) `devices, ndev`): one transform
 * context per listed device (tables, scratch and stream replicated; a
 * device may be listed twice).  Every batch entry point below accepts it:
 *   FHE_HOST    the batch is cut into ndev contiguous balanced ranges, each
 *               staged through its own device by its own host thread (the
 *               reference's batch_encrypt chunks a batch over threads sharing
 *               one read-only NTTProcessor, encryption.cpp:472, 520-533);
 *               returns when every range is back in host memory;
 *   FHE_DEVICE  the pointers are device memory of one listed device and the
 *               call runs there (data stays where it lives; shard across
 *               devices by calling once per device-resident shard).
 * Key preparation (fhe_ggsw_prepare, fhe_relin_key_prepare, fhe_secret_key_prepare,
 * fhe_public_key_prepare) runs on the first device for FHE_HOST.
 * fhe_ctx_set_stream binds the stream to the sub-context of its device.     */
int fhe_ctx_create_multi(uint32_t n, uint64_t q, int mode, const int *devices, int ndev, fhe_ctx **out);
int fhe_ctx_device_count(const fhe_ctx *ctx, int *ndev);
/* The per-device context i (borrowed; owned by ctx).  A single-device
 * context returns itself for i = 0. */
int fhe_ctx_sub(const fhe_ctx *ctx, int i, fhe_ctx **out);
/* Enqueue all later work of this context on the given hipStream_t (e.g. the
 * caller's torch stream).  NULL selects the null (legacy default) stream,
 * which is torch's default stream.  A new context uses a private
 * non-blocking stream until this is called. */
int fhe_ctx_set_stream(fhe_ctx *ctx, void *hip_stream);
void *fhe_ctx_stream(const fhe_ctx *ctx);
int fhe_ctx_synchronize(fhe_ctx *ctx);

typedef struct {
    uint32_t n, log_n;
    uint64_t q;
    uint64_t psi;          /* primitive 2N-th root (smallest generator rule, ntt_processor.cpp:92-128) */
    uint64_t psi_inv;
    uint64_t inv_n;        /* N^-1 mod q */
    int32_t mode;
    int32_t word_bits;     /* 32 (q < 2^30) or 64 (q < 2^64) kernel arithmetic */
    int32_t device;
    int32_t polys_per_block;
    int32_t threads_per_block;
} fhe_ctx_info;
int fhe_ctx_get_info(const fhe_ctx *ctx, fhe_ctx_info *info);
/* The reference's twiddle vectors psi^i / psi^-i, i < n (ntt_processor.cpp:188-202). */
int fhe_ctx_get_twiddles(const fhe_ctx *ctx, uint64_t *forward, uint64_t *inverse);

/* ---- transforms (ntt_processor.cpp:262-408) -----------------------------
 * In place allowed (out == in).                                            */
int fhe_ntt_fwd_batch(fhe_ctx *ctx, const uint64_t *in, uint64_t *out, size_t batch, int where);
int fhe_ntt_inv_batch(fhe_ctx *ctx, const uint64_t *in, uint64_t *out, size_t batch, int where);
/* out = to_ntt(a) (.) w, per polynomial (config C3: NTT + modmul). */
int fhe_ntt_fwd_mul_batch(fhe_ctx *ctx, const uint64_t *a, const uint64_t *w, uint64_t *out, size_t batch,
                          int where);

/* ---- PolynomialRing (polynomial_ring.cpp) ------------------------------- */
/* multiply (:421-447) on coefficient-form inputs: inv(fwd(a) (.) fwd(b)). */
int fhe_polymul_batch(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch, int where);
/* pointwise_multiply (:493-530): c = a*b mod q over n*batch coefficients. */
int fhe_pointwise_batch(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch, int where);
int fhe_poly_add_batch(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch, int where);
int fhe_poly_sub_batch(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch, int where);
int fhe_poly_neg_batch(fhe_ctx *ctx, const uint64_t *a, uint64_t *c, size_t batch, int where);
int fhe_poly_mul_scalar_batch(fhe_ctx *ctx, const uint64_t *a, uint64_t scalar, uint64_t *c, size_t batch,
                              int where);

/* ---- TFHE external product (bootstrap_engine.cpp:152-185, 431-518) ------
 * glwe:  [batch][k+1][n] (k mask polynomials, then the body)
 * ggsw:  [(k+1)*level rows][k+1][n], rows ordered as the reference's
 *        ggsw.matrix (mask digit rows first, digit level inner).
 * fhe_ggsw_prepare turns a coefficient-form GGSW into the NTT-domain form
 * fhe_external_product_batch consumes (same shape).  GLWE dimension k = 1..16:
 * fused kernels for k = 1 and n <= 16384, composed (decompose, batched
 * transforms, key MAC, inverse) otherwise. */
int fhe_ggsw_prepare(fhe_ctx *ctx, uint32_t k, uint32_t level, const uint64_t *ggsw, uint64_t *ggsw_ntt, int where);
int fhe_external_product_batch(fhe_ctx *ctx, uint32_t k, uint32_t base_log, uint32_t level, const uint64_t *glwe,
                               const uint64_t *ggsw_ntt, uint64_t *out, size_t batch, int where);
/* decompose_polynomial (:152-185) for npoly polynomials: out [npoly][level][n]. */
int fhe_decompose_batch(fhe_ctx *ctx, uint32_t base_log, uint32_t level, const uint64_t *poly, uint64_t *out,
                        size_t npoly, int where);

/* ---- RNS multi-modulus ring (PolynomialRing(degree, moduli),
 * polynomial_ring.cpp:224-237): one transform context per modulus, all on
 * one stream.  RNS polynomials are modulus-major: [count][batch][n] (limb i
 * of every polynomial contiguous).  FHE_DEVICE calls run each operation as
 * ONE launch over all limbs (grid.y = limb, per-limb constants from device
 * tables built at creation) when every limb shares the kernel shape (n <=
 * 16384, q < 2^62, all limbs in 32-bit or all in 64-bit lanes, same
 * laziness); otherwise, and for FHE_HOST calls (staged limb by limb), one
 * launch per limb.  FHE_RNS_ONE_LAUNCH=0 forces one launch per limb.  The
 * reference's ring operations use moduli_[0] only; these apply the
 * operation to every limb. */
typedef struct fhe_rns_ctx fhe_rns_ctx;
int fhe_rns_ctx_create(uint32_t n, const uint64_t *moduli, uint32_t count, int mode, int device, fhe_rns_ctx **out);
void fhe_rns_ctx_destroy(fhe_rns_ctx *rns);
int fhe_rns_ctx_limb(const fhe_rns_ctx *rns, uint32_t i, fhe_ctx **out);
int fhe_rns_ntt_fwd_batch(fhe_rns_ctx *rns, const uint64_t *in, uint64_t *out, size_t batch, int where);
int fhe_rns_ntt_inv_batch(fhe_rns_ctx *rns, const uint64_t *in, uint64_t *out, size_t batch, int where);
int fhe_rns_polymul_batch(fhe_rns_ctx *rns, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch,
                          int where);
int fhe_rns_pointwise_batch(fhe_rns_ctx *rns, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch,
                            int where);
int fhe_rns_add_batch(fhe_rns_ctx *rns, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch, int where);
int fhe_rns_sub_batch(fhe_rns_ctx *rns, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch, int where);

/* ---- BFV-style ciphertext multiplication (encryption.cpp:737-980) -------
 * A ciphertext is its component polynomials, contiguous: ct [batch][2][n]
 * (c0, c1); a degree-2 product [batch][3][n] (c0, c1, c2).
 * fhe_ct_multiply_batch  EncryptionEngine::multiply (:737-798): is_ntt = 0
 *   for coefficient-form inputs (4 forward + 3 inverse transforms in one
 *   kernel), 1 when both inputs are already NTT-domain (tensor only).
 * fhe_relin_key_prepare  the KeySwitchKey pairs (a_l, b_l) of
 *   key_manager.cpp:296-324, rlk [level][2][n], into the NTT-domain form
 *   fhe_relinearize_batch consumes (same shape).
 * fhe_relinearize_batch  EncryptionEngine::relinearize (:904-980): digit l
 *   of c2 is (c2 >> l*base_log) & (2^base_log - 1); out [batch][2][n] =
 *   (c0 + sum_l d_l * b_l, c1 + sum_l d_l * a_l).  level = number of key
 *   pairs used (the reference's min(decomp_level, keys.size())); level 0
 *   copies c0, c1.  Requires (level - 1) * base_log < 64, 1 <= base_log <= 63.
 * fhe_ct_multiply_relin_batch  multiply_relin (:800-807): both steps. */
int fhe_ct_multiply_batch(fhe_ctx *ctx, const uint64_t *ct1, const uint64_t *ct2, uint64_t *out, size_t batch,
                          int is_ntt, int where);
int fhe_relin_key_prepare(fhe_ctx *ctx, uint32_t level, const uint64_t *rlk, uint64_t *rlk_ntt, int where);
int fhe_relinearize_batch(fhe_ctx *ctx, uint32_t base_log, uint32_t level, const uint64_t *ct3,
                          const uint64_t *rlk_ntt, uint64_t *out, size_t batch, int where);
int fhe_ct_multiply_relin_batch(fhe_ctx *ctx, uint32_t base_log, uint32_t level, const uint64_t *ct1,
                                const uint64_t *ct2, const uint64_t *rlk_ntt, uint64_t *out, size_t batch,
                                int where);

/* ---- TFHE bootstrapping pieces (bootstrap_engine.cpp) --------------------
 * GLWE [batch][k+1][n] as above; LWE masks [batch][dim], bodies [batch].
 * fhe_glwe_rotate_batch    multiply_glwe_by_monomial (:249-261) by X^rot[c].
 * fhe_cmux_batch           cmux (:520-540): ct0 + ggsw (x) (ct1 - ct0).
 * fhe_blind_rotate_batch   blind_rotate (:547-577) of acc in place, for each
 *   ciphertext c with its own LWE (lwe_a[c], lwe_b[c]) modulo lwe_q; bsk_ntt
 *   = lwe_dim prepared GGSWs ([lwe_dim][(k+1)*level][k+1][n]).  k = 1 with
 *   n <= 16384 runs fused: one launch for the whole loop at n = 512..4096
 *   (two CUs per ciphertext while 16 * ceil(batch / 8) <= CUs, else one;
 *   2 * level CUs at level 2 / 3 while 2 * level * ceil(batch / 8) <= the
 *   CUs of one XCD, FHE_BR_MULTI=0 keeps two; FHE_BR_PAIR=0 forces one),
 *   per-step CMux launches above; k = 2..4 run
 *   as one launch where the k + 1 accumulators fit in LDS (n = 512 / 1024
 *   with 64-bit words; n = 2048 for k <= 3 with 32-bit words); other
 *   k <= 16 and n = 32768 / 65536 run composed step by step (one digit
 *   buffer for the whole loop, stream-ordered, no host synchronisation).  The multi-CU
 *   launch needs the workgroups of a ciphertext co-resident.  It is never
 *   assumed: multi-CU launches of one process are serialised per device,
 *   and a workgroup whose partners do not answer within
 *   FHE_BR_PAIR_TIMEOUT_US (default 20000 us; 0 simulates a partner that
 *   never answers, for tests) gives its
 *   ciphertext up: a repair pass enqueued behind the launch recomputes every
 *   given-up ciphertext on one CU from a saved copy of its input, so the
 *   result is exact in every case (no host synchronisation either way).
 *   fhe_br_repair_count reports how many ciphertexts took the repair pass.
 *   fhe_bootstrap_batch takes the same shapes.
 * fhe_sample_extract_batch sample_extract (:594-624): lwe_a [batch][k*n].
 * fhe_key_switch_batch     key_switch (:626-674): ksk_a [in_dim*level][out_dim]
 *   (the `first` polynomials of ksk.keys, entry i*level + l), ksk_b
 *   [in_dim*level] (coefficient 0 of each `second` polynomial). */
int fhe_glwe_rotate_batch(fhe_ctx *ctx, uint32_t k, const int32_t *rot, const uint64_t *glwe, uint64_t *out,
                          size_t batch, int where);
int fhe_cmux_batch(fhe_ctx *ctx, uint32_t k, uint32_t base_log, uint32_t level, const uint64_t *ggsw_ntt,
                   const uint64_t *ct0, const uint64_t *ct1, uint64_t *out, size_t batch, int where);
int fhe_blind_rotate_batch(fhe_ctx *ctx, uint32_t k, uint32_t base_log, uint32_t level, uint32_t lwe_dim,
                           const uint64_t *lwe_a, const uint64_t *lwe_b, uint64_t lwe_q, const uint64_t *bsk_ntt,
                           uint64_t *acc, size_t batch, int where);
int fhe_sample_extract_batch(fhe_ctx *ctx, uint32_t k, const uint64_t *glwe, uint64_t *lwe_a, uint64_t *lwe_b,
                             size_t batch, int where);
/* Ciphertexts of this context's multi-CU blind rotations that were recomputed
 * by the repair pass since the context was created (a partner workgroup that
 * was not co-resident in time; see fhe_blind_rotate_batch).  Waits for the
 * context's stream.  No reference counterpart: blind_rotate
 * (bootstrap_engine.cpp:547-577) is a sequential CPU loop. */
int fhe_br_repair_count(fhe_ctx *ctx, uint64_t *count);
int fhe_key_switch_batch(uint64_t q, uint32_t base_log, uint32_t level, uint32_t in_dim, uint32_t out_dim,
                         const uint64_t *ksk_a, const uint64_t *ksk_b, const uint64_t *lwe_a, const uint64_t *lwe_b,
                         uint64_t *out_a, uint64_t *out_b, size_t batch, int where, int device, void *hip_stream);

/* ---- EncryptionEngine encrypt / decrypt / add_plain (encryption.cpp) ----
 * The reference's RLWE encryption with its encoding: t = plaintext modulus
 * (0 selects 4, encryption.cpp:40-46), delta = q / t, a plaintext is n slot
 * values per ciphertext encoded as (v * delta mod 2^64) mod q
 * (encode_packed :117-131; encode_plaintext is the one-slot case).
 * fhe_secret_key_prepare  sk [n] (SecretKey::poly) -> sk_prep [2][n]
 *   (NTT-domain s and s^2; decrypt :256-271).
 * fhe_public_key_prepare  pk [2][n] = (a, b) (PublicKey, key_manager.h:70-76)
 *   -> pk_prep [2][n] (NTT-domain).
 *   Prepared keys are opaque to the caller: Montgomery form for the fused
 *   kernels (q < 2^62, n <= 16384), canonical rows for the composed path
 *   (q >= 2^62 or n > 16384); pass them back to the context that made them.
 * fhe_encrypt_batch  encrypt_internal (:171-205) with the sampled
 *   polynomials supplied (u ternary, e1, e2 error; [batch][n] each, any u64
 *   as x mod q), so the call is deterministic: ct [batch][2][n] =
 *   (pk.b u + e1 + m, pk.a u + e2) under the context's transform product.
 * fhe_decrypt_batch  decrypt / decrypt_packed (:234-348) of ciphertexts
 *   [batch][components][n] (2: (c0, c1); 3: degree-2 (c0, c1, c2)); is_ntt
 *   as Ciphertext::is_ntt.  Outputs (each nullable): values [batch][n] =
 *   round(p t / q) mod t per coefficient of the phase p = c0 - c1 s
 *   (- c2 s^2) (decode_packed :150-163; slot 0 is decode_plaintext),
 *   phase [batch][n], max_noise [batch] = the integer whose double is the
 *   reference's max_noise (compute_noise_budget :364-400); its noise
 *   budget is log2(q / (2 max(max_noise, 1))), negative = the reference's
 *   "Noise budget exhausted" failure.
 * fhe_add_plain_batch  add_plain (:638-665): out = (c0 + m, c1), m
 *   transformed first when is_ntt.
 * Every degree and modulus the context takes: one fused kernel per call for
 * q < 2^62 and n <= 16384, batched transforms plus elementwise passes
 * otherwise (engine_composed.hip). */
int fhe_secret_key_prepare(fhe_ctx *ctx, const uint64_t *sk, uint64_t *sk_prep, int where);
int fhe_public_key_prepare(fhe_ctx *ctx, const uint64_t *pk, uint64_t *pk_prep, int where);
int fhe_encrypt_batch(fhe_ctx *ctx, uint64_t t, const uint64_t *pk_prep, const uint64_t *values, const uint64_t *u,
                      const uint64_t *e1, const uint64_t *e2, uint64_t *ct, size_t batch, int where);
int fhe_decrypt_batch(fhe_ctx *ctx, uint64_t t, const uint64_t *sk_prep, const uint64_t *ct, uint32_t components,
                      int is_ntt, uint64_t *values, uint64_t *phase, uint64_t *max_noise, size_t batch, int where);
int fhe_add_plain_batch(fhe_ctx *ctx, uint64_t t, const uint64_t *ct, const uint64_t *values, int is_ntt,
                        uint64_t *out, size_t batch, int where);

/* ---- BootstrapEngine::bootstrap_with_test_poly (bootstrap_engine.cpp:684-708)
 * For each LWE ciphertext c (lwe_a [batch][lwe_dim], lwe_b [batch] mod
 * lwe_q): acc = (0, .., 0, test_poly), blind_rotate (as
 * fhe_blind_rotate_batch), sample_extract, then key_switch modulo the GLWE
 * modulus with ksk_a [k*n*ks_level][out_dim], ksk_b [k*n*ks_level] (as
 * fhe_key_switch_batch): out_a [batch][out_dim], out_b [batch].
 * bootstrap() is the identity test polynomial; programmable_bootstrap
 * (:716-722) passes a lookup table's polynomial. */
int fhe_bootstrap_batch(fhe_ctx *ctx, uint32_t k, uint32_t base_log, uint32_t level, uint32_t lwe_dim,
                        const uint64_t *lwe_a, const uint64_t *lwe_b, uint64_t lwe_q, const uint64_t *bsk_ntt,
                        const uint64_t *test_poly, uint32_t ks_base_log, uint32_t ks_level, uint32_t out_dim,
                        const uint64_t *ksk_a, const uint64_t *ksk_b, uint64_t *out_a, uint64_t *out_b, size_t batch,
                        int where);

/* ---- device randomness and key material (key_manager.cpp, bootstrap_engine.cpp)
 * SecureRandom's draws (key_manager.cpp:53-115) come from a ChaCha20
 * keystream (RFC 8439 block function) keyed by seed[4] (256 bits, little-
 * endian words), with the 64-bit `stream` as the nonce: element i of a
 * stream of `count` elements draws from blocks i, i + count, i + 2 count, ..
 * (8 u64 words per block, in order).  The same (seed, stream, count) gives
 * the same values on every device and in the CPU oracle (oracle_sample), so
 * keys and encryptions are reproducible; the engine seeds from the OS CSPRNG.
 *   FHE_SAMPLE_UNIFORM   random_u64_range(q): rejection below (2^64 - q) % q, then % q (:60-71)
 *   FHE_SAMPLE_TERNARY   sample_ternary: range(3) -> {q-1, 0, 1} (:73-83)
 *   FHE_SAMPLE_GAUSSIAN  sample_gaussian(std_dev, q): Box-Muller on two 53-bit
 *                        uniforms, std::round, negatives as q + x (:85-110)
 *   FHE_SAMPLE_BINARY    sample_binary: random_u64() & 1
 *   FHE_SAMPLE_RAW       random_u64()
 * q is the context modulus.  Every keygen entry point names the streams it
 * takes; results follow the reference formulas under the context's
 * transform product (*).
 * fhe_encrypt_sampled_batch   encrypt_internal (encryption.cpp:171-205) with
 *   u ternary (stream), e1 (stream + 1), e2 (stream + 2) error, [batch][n]
 *   each; otherwise as fhe_encrypt_batch.
 * fhe_public_key_generate     generate_public_key (key_manager.cpp:218-246):
 *   pk [2][n] = (a, a (*) s + e), a uniform (stream), e error (stream + 1).
 * fhe_eval_key_generate       generate_eval_key (:252-333): rlk [level][2][n],
 *   a_l uniform (stream + 2l), e_l error (stream + 2l + 1),
 *   b_l = a_l (*) s + e_l + (s (*) s) * power_l, power_0 = 1,
 *   power_{l+1} = (power_l * 2^base_log) % q in u64 arithmetic (as the reference).
 * fhe_ggsw_encrypt_batch      encrypt_ggsw (bootstrap_engine.cpp:268-306) of
 *   count values (the LWE key of a bootstrapping key, :308-360): out
 *   [count][(k+1)*level][k+1][n] coefficient form, row (row, l) an
 *   encrypt_glwe_zero (:190-227; masks uniform (stream), error (stream + 1),
 *   body = sum_i mask_i (*) s + e) plus (|v| q) >> ((l+1) base_log) (negated
 *   mod q for v < 0) on coefficient 0 of mask `row` (row < k) or the body.
 * fhe_ksk_generate            generate_key_switch_key (:367-420): entry
 *   e = i*level + l (i < n_in, the GLWE key coefficients glwe_sk[i]):
 *   ksk_a [entries][lwe_dim] uniform (stream), error (stream + 1; std_dev 0
 *   selects 3.2), ksk_b[e] = ((u64)((<a_e, lwe_sk> + e) % (int64)q)
 *   + (glwe_sk[i] q) >> ((l+1) base_log)) % q with the reference's int64 /
 *   u64 wrap-around.  Shift counts >= 64 take the count mod 64.
 * fhe_lwe_decrypt_batch       LWE decryption under an integer key s [dim]:
 *   phase = b - sum_j a_j s_j (mod q), values = round(phase t / q) mod t
 *   (decode_plaintext's rounding, encryption.cpp:133-148).  Each output
 *   nullable. */
#define FHE_SAMPLE_UNIFORM 0
#define FHE_SAMPLE_TERNARY 1
#define FHE_SAMPLE_GAUSSIAN 2
#define FHE_SAMPLE_BINARY 3
#define FHE_SAMPLE_RAW 4
int fhe_sample_batch(fhe_ctx *ctx, int kind, const uint64_t seed[4], uint64_t stream, double std_dev, uint64_t *out,
                     size_t count, int where);
int fhe_encrypt_sampled_batch(fhe_ctx *ctx, uint64_t t, const uint64_t *pk_prep, const uint64_t *values,
                              const uint64_t seed[4], uint64_t stream, double std_dev, uint64_t *ct, size_t batch,
                              int where);
int fhe_public_key_generate(fhe_ctx *ctx, const uint64_t *sk, const uint64_t seed[4], uint64_t stream, double std_dev,
                            uint64_t *pk, int where);
int fhe_eval_key_generate(fhe_ctx *ctx, const uint64_t *sk, uint32_t base_log, uint32_t level, const uint64_t seed[4],
                          uint64_t stream, double std_dev, uint64_t *rlk, int where);
int fhe_ggsw_encrypt_batch(fhe_ctx *ctx, uint32_t k, uint32_t base_log, uint32_t level, const int64_t *values,
                           size_t count, const uint64_t *sk, const uint64_t seed[4], uint64_t stream, double std_dev,
                           uint64_t *out, int where);
int fhe_ksk_generate(fhe_ctx *ctx, uint32_t base_log, uint32_t level, const uint64_t *glwe_sk, uint32_t n_in,
                     const int64_t *lwe_sk, uint32_t lwe_dim, const uint64_t seed[4], uint64_t stream, double std_dev,
                     uint64_t *ksk_a, uint64_t *ksk_b, int where);
int fhe_lwe_decrypt_batch(uint64_t q, uint64_t t, const int64_t *sk, uint32_t dim, const uint64_t *lwe_a,
                          const uint64_t *lwe_b, uint64_t *values, uint64_t *phase, size_t batch, int where,
                          int device, void *hip_stream);

/* ---- context-free modular kernels --------------------------------------- */
/* BarrettReducer::barrett_mul contract (modular_arithmetic.cpp:268-280):
 * c[i] = a[i]*b[i] mod q for any u64 inputs, any q != 0. stream may be NULL. */
int fhe_modmul_batch(uint64_t q, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t count, int where,
                     int device, void *hip_stream);
/* MultiLimbModularArithmetic (2 limbs, modular_arithmetic.cpp:471-625).
 * q[2] little-endian limbs; a, b, c: count elements of 2 limbs each. */
int fhe_ml_constants(const uint64_t q[2], uint64_t out[7]); /* q0,q1,r0,r1,r2_0,r2_1,q_inv */
int fhe_ml_montmul_batch(const uint64_t q[2], const uint64_t *a, const uint64_t *b, uint64_t *c, size_t count,
                         int where, int device, void *hip_stream);

/* ---- N-API ModularArithmetic class (index.d.ts:32-44, lib.rs:42-121) -----
 * Scalar host functions with the reference's exact constants, including
 * q_inv = -(q^-1 mod (2^64-1)) (modular_arithmetic.cpp:69).  consts[4] =
 * {q, R mod q, R^2 mod q, q_inv}.                                            */
int fhe_mont_constants_compat(uint64_t q, uint64_t consts[4]);
uint64_t fhe_compat_montgomery_mul(const uint64_t consts[4], uint64_t a, uint64_t b);
uint64_t fhe_compat_to_montgomery(const uint64_t consts[4], uint64_t a);
uint64_t fhe_compat_from_montgomery(const uint64_t consts[4], uint64_t a);
uint64_t fhe_compat_mod_add(uint64_t q, uint64_t a, uint64_t b);
uint64_t fhe_compat_mod_sub(uint64_t q, uint64_t a, uint64_t b);

/* ---- context-owned device memory (resident ciphertexts and keys) -------
 * fhe_ctx_alloc / fhe_ctx_free: stream-ordered allocations on the context's
 * (first) device: a free is ordered after the work already enqueued on the
 * context stream, and the device pool keeps the memory warm (no device
 * synchronisation per call).  fhe_ctx_memcpy copies on the context stream:
 * FHE_COPY_H2D / FHE_COPY_D2H return when the copy is done (ordered after the
 * context's earlier work), FHE_COPY_D2D is enqueued. */
#define FHE_COPY_H2D 0
#define FHE_COPY_D2H 1
#define FHE_COPY_D2D 2
int fhe_ctx_alloc(fhe_ctx *ctx, size_t bytes, void **out);
int fhe_ctx_free(fhe_ctx *ctx, void *ptr);
int fhe_ctx_memcpy(fhe_ctx *ctx, void *dst, const void *src, size_t bytes, int kind);

/* ---- device memory helpers (for callers without their own allocator) --- */
int fhe_dev_alloc(int device, size_t bytes, void **out);
int fhe_dev_free(void *ptr);
int fhe_memcpy_h2d(void *dst, const void *src, size_t bytes);
int fhe_memcpy_d2h(void *dst, const void *src, size_t bytes);
int fhe_device_synchronize(int device);

/* Event timing on a stream (used by bench.py for HIP-event kernel timing). */
int fhe_event_create(void **ev);
int fhe_event_destroy(void *ev);
int fhe_event_record(void *ev, void *hip_stream);
int fhe_event_elapsed_ms(void *start, void *stop, float *ms);

#ifdef __cplusplus
}
#endif
#endif /* FHE_GPU_H */
