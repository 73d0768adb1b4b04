/*
 * fhe_napi.c -- plain node_api.h addon over libfhe_gpu.so.
 *
 * Replaces the napi-rs binding (src/native/lib.rs:22-133, bridge.rs:3-41)
 * with the same JS surface as index.d.ts:
 *   initialize(), detectHardware(), version(), class ModularArithmetic
 * plus the batched polynomial engine the TS FHEEngine needs (NttContext,
 * modmulBatch, mlMontgomeryMulBatch) over zero-copy BigUint64Array buffers
 * (napi_get_typedarray_info; FHE_HOST placement, the library stages the data
 * through HBM).  Errors become JS exceptions with the library's message --
 * the reference's cxx bridge aborted the process on a C++ exception instead.
 */
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fhe_gpu.h"

#define NAPI_CALL(env, call)                                        \
    do {                                                            \
        if ((call) != napi_ok) {                                    \
            napi_throw_error((env), "NATIVE_ERROR", "N-API call failed: " #call); \
            return NULL;                                            \
        }                                                           \
    } while (0)

static napi_value throw_fhe(napi_env env, int rc) {
    char code[32];
    snprintf(code, sizeof code, "FHE_%d", rc);
    napi_throw_error(env, code, fhe_last_error());
    return NULL;
}

static napi_value make_bool(napi_env env, int v) {
    napi_value r;
    napi_get_boolean(env, v != 0, &r);
    return r;
}
static napi_value make_i64(napi_env env, int64_t v) {
    napi_value r;
    napi_create_int64(env, v, &r);
    return r;
}
static napi_value make_str(napi_env env, const char *s) {
    napi_value r;
    napi_create_string_utf8(env, s, NAPI_AUTO_LENGTH, &r);
    return r;
}
static void set(napi_env env, napi_value obj, const char *k, napi_value v) { napi_set_named_property(env, obj, k, v); }

/* integer argument: JS number (as napi-rs i64) or BigInt */
static int get_u64(napi_env env, napi_value v, uint64_t *out, int *negative) {
    napi_valuetype t;
    napi_typeof(env, v, &t);
    *negative = 0;
    if (t == napi_bigint) {
        bool lossless;
        return napi_get_value_bigint_uint64(env, v, out, &lossless) == napi_ok ? 0 : -1;
    }
    if (t == napi_number) {
        int64_t x;
        if (napi_get_value_int64(env, v, &x) != napi_ok) return -1;
        if (x < 0) *negative = 1;
        *out = (uint64_t)x;
        return 0;
    }
    return -1;
}

/* BigUint64Array -> pointer + element count */
static int get_u64_array(napi_env env, napi_value v, uint64_t **data, size_t *count) {
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return -1;
    napi_typedarray_type type;
    size_t len, off;
    void *raw;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &len, &raw, &ab, &off) != napi_ok) return -1;
    if (type != napi_biguint64_array) return -1;
    *data = (uint64_t *)raw;
    *count = len;
    return 0;
}

/* ------------------------------------------------------------------ free functions */
static napi_value js_initialize(napi_env env, napi_callback_info info) {
    (void)info;
    fhe_hw_caps caps;
    int rc = fhe_detect(&caps);
    if (rc) return throw_fhe(env, rc);
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

static napi_value js_detect(napi_env env, napi_callback_info info) {
    (void)info;
    fhe_hw_caps caps;
    int rc = fhe_detect(&caps);
    if (rc) return throw_fhe(env, rc);
    napi_value o;
    NAPI_CALL(env, napi_create_object(env, &o));
    /* the reference's HardwareCapabilities fields (index.d.ts:22-29) ... */
    set(env, o, "hasSme", make_bool(env, 0));
    set(env, o, "hasMetal", make_bool(env, 0));
    set(env, o, "hasNeon", make_bool(env, 0));
    set(env, o, "hasAmx", make_bool(env, 0));
    set(env, o, "metalGpuCores", make_i64(env, 0));
    set(env, o, "unifiedMemorySize", make_i64(env, 0));
    /* ... and what this backend actually runs on */
    set(env, o, "hasHip", make_bool(env, caps.device_count > 0));
    set(env, o, "gpuDevices", make_i64(env, caps.device_count));
    set(env, o, "computeUnits", make_i64(env, caps.compute_units));
    set(env, o, "wavefrontSize", make_i64(env, caps.wavefront_size));
    set(env, o, "xcds", make_i64(env, caps.xcds));
    set(env, o, "hbmBytes", make_i64(env, (int64_t)caps.hbm_bytes));
    set(env, o, "arch", make_str(env, caps.arch));
    set(env, o, "deviceName", make_str(env, caps.name));
    return o;
}

static napi_value js_version(napi_env env, napi_callback_info info) {
    (void)info;
    return make_str(env, fhe_version());
}

/* modmulBatch(q, a, b, out?) -> out : BarrettReducer contract on the GPU */
static napi_value js_modmul_batch(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint64_t q, *a, *b, *c;
    size_t na, nb, nc;
    int neg;
    if (argc < 4 || get_u64(env, argv[0], &q, &neg) || neg || get_u64_array(env, argv[1], &a, &na) ||
        get_u64_array(env, argv[2], &b, &nb) || get_u64_array(env, argv[3], &c, &nc)) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "modmulBatch(q: bigint, a, b, out: BigUint64Array)");
        return NULL;
    }
    if (na != nb || na != nc) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "operand lengths differ");
        return NULL;
    }
    int rc = fhe_modmul_batch(q, a, b, c, na, FHE_HOST, 0, NULL);
    if (rc) return throw_fhe(env, rc);
    return argv[3];
}

/* mlMontgomeryMulBatch([q0, q1], a, b, out) : 2-limb Montgomery products */
static napi_value js_ml_montmul(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint64_t *qv, *a, *b, *c;
    size_t nq, na, nb, nc;
    if (argc < 4 || get_u64_array(env, argv[0], &qv, &nq) || nq != 2 || get_u64_array(env, argv[1], &a, &na) ||
        get_u64_array(env, argv[2], &b, &nb) || get_u64_array(env, argv[3], &c, &nc) || na % 2 || na != nb ||
        na != nc) {
        napi_throw_type_error(env, "INVALID_PARAMETERS",
                              "mlMontgomeryMulBatch(q: BigUint64Array(2), a, b, out: BigUint64Array of limb pairs)");
        return NULL;
    }
    int rc = fhe_ml_montmul_batch(qv, a, b, c, na / 2, FHE_HOST, 0, NULL);
    if (rc) return throw_fhe(env, rc);
    return argv[3];
}

/* ------------------------------------------------------------------ class ModularArithmetic */
typedef struct {
    uint64_t k[4];
} mod_arith;

static void ma_finalize(napi_env env, void *data, void *hint) {
    (void)env;
    (void)hint;
    free(data);
}

static napi_value ma_ctor(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], self;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, &self, NULL));
    int64_t m = 0;
    if (argc < 1 || napi_get_value_int64(env, argv[0], &m) != napi_ok) {
        napi_throw_type_error(env, NULL, "modulus must be a number");
        return NULL;
    }
    if (m <= 0) { /* lib.rs:53-55 */
        napi_throw_error(env, NULL, "Modulus must be positive");
        return NULL;
    }
    mod_arith *ma = (mod_arith *)calloc(1, sizeof *ma);
    int rc = fhe_mont_constants_compat((uint64_t)m, ma->k);
    if (rc) {
        free(ma);
        return throw_fhe(env, rc);
    }
    NAPI_CALL(env, napi_wrap(env, self, ma, ma_finalize, NULL, NULL));
    return self;
}

static mod_arith *ma_this(napi_env env, napi_callback_info info, size_t *argc, napi_value *argv) {
    napi_value self;
    if (napi_get_cb_info(env, info, argc, argv, &self, NULL) != napi_ok) return NULL;
    void *p = NULL;
    napi_unwrap(env, self, &p);
    return (mod_arith *)p;
}

/* number args as i64 (lib.rs: JS number <-> i64, negative rejected) */
static int ma_args(napi_env env, size_t argc, napi_value *argv, size_t need, int64_t *out, const char *neg_msg) {
    if (argc < need) {
        napi_throw_type_error(env, NULL, "missing argument");
        return -1;
    }
    for (size_t i = 0; i < need; ++i) {
        if (napi_get_value_int64(env, argv[i], &out[i]) != napi_ok) {
            napi_throw_type_error(env, NULL, "arguments must be numbers");
            return -1;
        }
        if (out[i] < 0) {
            napi_throw_error(env, NULL, neg_msg);
            return -1;
        }
    }
    return 0;
}

#define MA_BINARY(NAME, EXPR)                                                        \
    static napi_value NAME(napi_env env, napi_callback_info info) {                  \
        size_t argc = 2;                                                             \
        napi_value argv[2];                                                          \
        mod_arith *ma = ma_this(env, info, &argc, argv);                             \
        int64_t x[2];                                                                \
        if (!ma || ma_args(env, argc, argv, 2, x, "Inputs must be non-negative")) return NULL; \
        uint64_t a = (uint64_t)x[0], b = (uint64_t)x[1];                             \
        return make_i64(env, (int64_t)(EXPR));                                       \
    }
#define MA_UNARY(NAME, EXPR)                                                         \
    static napi_value NAME(napi_env env, napi_callback_info info) {                  \
        size_t argc = 1;                                                             \
        napi_value argv[1];                                                          \
        mod_arith *ma = ma_this(env, info, &argc, argv);                             \
        int64_t x[1];                                                                \
        if (!ma || ma_args(env, argc, argv, 1, x, "Input must be non-negative")) return NULL; \
        uint64_t a = (uint64_t)x[0];                                                 \
        return make_i64(env, (int64_t)(EXPR));                                       \
    }

MA_BINARY(ma_montgomery_mul, fhe_compat_montgomery_mul(ma->k, a, b))
MA_BINARY(ma_mod_add, fhe_compat_mod_add(ma->k[0], a, b))
MA_BINARY(ma_mod_sub, fhe_compat_mod_sub(ma->k[0], a, b))
MA_UNARY(ma_to_mont, fhe_compat_to_montgomery(ma->k, a))
MA_UNARY(ma_from_mont, fhe_compat_from_montgomery(ma->k, a))

static napi_value ma_get_modulus(napi_env env, napi_callback_info info) {
    size_t argc = 0;
    mod_arith *ma = ma_this(env, info, &argc, NULL);
    if (!ma) return NULL;
    return make_i64(env, (int64_t)ma->k[0]);
}

/* ------------------------------------------------------------------ class NttContext */
static void ctx_finalize(napi_env env, void *data, void *hint) {
    (void)env;
    (void)hint;
    fhe_ctx_destroy((fhe_ctx *)data);
}

static napi_value ctx_ctor(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4], self;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, &self, NULL));
    uint64_t n, q, mode = 0, dev = 0;
    int neg;
    if (argc < 2 || get_u64(env, argv[0], &n, &neg) || neg || get_u64(env, argv[1], &q, &neg) || neg ||
        (argc > 2 && (get_u64(env, argv[2], &mode, &neg) || neg)) ||
        (argc > 3 && (get_u64(env, argv[3], &dev, &neg) || neg))) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "NttContext(degree, modulus: bigint|number, mode?, device?)");
        return NULL;
    }
    fhe_ctx *c = NULL;
    int rc = fhe_ctx_create((uint32_t)n, q, (int)mode, (int)dev, &c);
    if (rc) return throw_fhe(env, rc);
    NAPI_CALL(env, napi_wrap(env, self, c, ctx_finalize, NULL, NULL));
    return self;
}

static fhe_ctx *ctx_this(napi_env env, napi_callback_info info, size_t *argc, napi_value *argv) {
    napi_value self;
    if (napi_get_cb_info(env, info, argc, argv, &self, NULL) != napi_ok) return NULL;
    void *p = NULL;
    napi_unwrap(env, self, &p);
    return (fhe_ctx *)p;
}

static int batch_of(napi_env env, fhe_ctx *c, size_t count, size_t *batch) {
    fhe_ctx_info ci;
    fhe_ctx_get_info(c, &ci);
    if (count % ci.n) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "Coefficient count must equal polynomial degree");
        return -1;
    }
    *batch = count / ci.n;
    return 0;
}

typedef int (*unary_fn)(fhe_ctx *, const uint64_t *, uint64_t *, size_t, int);
typedef int (*binary_fn)(fhe_ctx *, const uint64_t *, const uint64_t *, uint64_t *, size_t, int);

/* op(a, out?) ; out defaults to a (in place, like NTTProcessor::forward_ntt) */
static napi_value ctx_unary(napi_env env, napi_callback_info info, unary_fn fn) {
    size_t argc = 2;
    napi_value argv[2];
    fhe_ctx *c = ctx_this(env, info, &argc, argv);
    uint64_t *a, *o;
    size_t na, no, batch;
    if (!c || argc < 1 || get_u64_array(env, argv[0], &a, &na)) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "expected BigUint64Array");
        return NULL;
    }
    napi_value ret = argv[0];
    o = a;
    no = na;
    if (argc > 1) {
        napi_valuetype t;
        napi_typeof(env, argv[1], &t);
        if (t != napi_undefined) {
            if (get_u64_array(env, argv[1], &o, &no) || no != na) {
                napi_throw_type_error(env, "INVALID_PARAMETERS", "out must be a BigUint64Array of equal length");
                return NULL;
            }
            ret = argv[1];
        }
    }
    if (batch_of(env, c, na, &batch)) return NULL;
    int rc = fn(c, a, o, batch, FHE_HOST);
    if (rc) return throw_fhe(env, rc);
    return ret;
}

static napi_value ctx_binary(napi_env env, napi_callback_info info, binary_fn fn) {
    size_t argc = 3;
    napi_value argv[3];
    fhe_ctx *c = ctx_this(env, info, &argc, argv);
    uint64_t *a, *b, *o;
    size_t na, nb, no, batch;
    if (!c || argc < 3 || get_u64_array(env, argv[0], &a, &na) || get_u64_array(env, argv[1], &b, &nb) ||
        get_u64_array(env, argv[2], &o, &no) || na != nb || na != no) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "expected (a, b, out) BigUint64Arrays of equal length");
        return NULL;
    }
    if (batch_of(env, c, na, &batch)) return NULL;
    int rc = fn(c, a, b, o, batch, FHE_HOST);
    if (rc) return throw_fhe(env, rc);
    return argv[2];
}

static int neg_adapter(fhe_ctx *c, const uint64_t *a, uint64_t *o, size_t b, int w) {
    return fhe_poly_neg_batch(c, a, o, b, w);
}

#define CTX_U(NAME, FN) \
    static napi_value NAME(napi_env env, napi_callback_info info) { return ctx_unary(env, info, FN); }
#define CTX_B(NAME, FN) \
    static napi_value NAME(napi_env env, napi_callback_info info) { return ctx_binary(env, info, FN); }
CTX_U(ctx_forward, fhe_ntt_fwd_batch)
CTX_U(ctx_inverse, fhe_ntt_inv_batch)
CTX_U(ctx_negate, neg_adapter)
CTX_B(ctx_polymul, fhe_polymul_batch)
CTX_B(ctx_pointwise, fhe_pointwise_batch)
CTX_B(ctx_add, fhe_poly_add_batch)
CTX_B(ctx_sub, fhe_poly_sub_batch)
CTX_B(ctx_fwd_mul, fhe_ntt_fwd_mul_batch)

static napi_value ctx_mul_scalar(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    fhe_ctx *c = ctx_this(env, info, &argc, argv);
    uint64_t *a, *o, s;
    size_t na, no, batch;
    int neg;
    if (!c || argc < 3 || get_u64_array(env, argv[0], &a, &na) || get_u64(env, argv[1], &s, &neg) || neg ||
        get_u64_array(env, argv[2], &o, &no) || na != no) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "mulScalar(a, scalar, out)");
        return NULL;
    }
    if (batch_of(env, c, na, &batch)) return NULL;
    int rc = fhe_poly_mul_scalar_batch(c, a, s, o, batch, FHE_HOST);
    if (rc) return throw_fhe(env, rc);
    return argv[2];
}

/* externalProduct(glwe, ggswCoeff, baseLog, level, out): k = 1 */
static napi_value ctx_ext_product(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5];
    fhe_ctx *c = ctx_this(env, info, &argc, argv);
    uint64_t *g, *k, *o, bl, lv;
    size_t ng, nk, no;
    int neg;
    if (!c || argc < 5 || get_u64_array(env, argv[0], &g, &ng) || get_u64_array(env, argv[1], &k, &nk) ||
        get_u64(env, argv[2], &bl, &neg) || neg || get_u64(env, argv[3], &lv, &neg) || neg ||
        get_u64_array(env, argv[4], &o, &no) || ng != no) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "externalProduct(glwe, ggsw, baseLog, level, out)");
        return NULL;
    }
    fhe_ctx_info ci;
    fhe_ctx_get_info(c, &ci);
    const size_t per = 2 * (size_t)ci.n;
    if (ng % per || nk != (size_t)4 * lv * ci.n) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "shape mismatch (k = 1)");
        return NULL;
    }
    uint64_t *prep = (uint64_t *)malloc(nk * 8);
    int rc = fhe_ggsw_prepare(c, 1, (uint32_t)lv, k, prep, FHE_HOST);
    if (!rc) rc = fhe_external_product_batch(c, 1, (uint32_t)bl, (uint32_t)lv, g, prep, o, ng / per, FHE_HOST);
    free(prep);
    if (rc) return throw_fhe(env, rc);
    return argv[4];
}

/* ctMultiply(ct1, ct2, out, isNtt?): ct [batch][2][n] -> out [batch][3][n]
 * (EncryptionEngine::multiply, encryption.cpp:737-798) */
static napi_value ctx_ct_multiply(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    fhe_ctx *c = ctx_this(env, info, &argc, argv);
    uint64_t *x, *y, *o, is_ntt = 0;
    size_t nx, ny, no;
    int neg;
    if (!c || argc < 3 || get_u64_array(env, argv[0], &x, &nx) || get_u64_array(env, argv[1], &y, &ny) ||
        get_u64_array(env, argv[2], &o, &no) || nx != ny ||
        (argc > 3 && (get_u64(env, argv[3], &is_ntt, &neg) || neg))) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "ctMultiply(ct1, ct2, out, isNtt?)");
        return NULL;
    }
    fhe_ctx_info ci;
    fhe_ctx_get_info(c, &ci);
    const size_t per = 2 * (size_t)ci.n;
    if (nx % per || no != nx / 2 * 3) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "ciphertexts must be [batch][2][n], out [batch][3][n]");
        return NULL;
    }
    int rc = fhe_ct_multiply_batch(c, x, y, o, nx / per, (int)is_ntt, FHE_HOST);
    if (rc) return throw_fhe(env, rc);
    return argv[2];
}

/* relinearize(ct3, rlk, baseLog, out): rlk [level][2][n] (a_l, b_l) in
 * coefficient form (KeySwitchKey), out [batch][2][n]
 * (EncryptionEngine::relinearize, encryption.cpp:904-980) */
static napi_value ctx_relinearize(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    fhe_ctx *c = ctx_this(env, info, &argc, argv);
    uint64_t *ct, *k, *o, bl;
    size_t nc, nk, no;
    int neg;
    if (!c || argc < 4 || get_u64_array(env, argv[0], &ct, &nc) || get_u64_array(env, argv[1], &k, &nk) ||
        get_u64(env, argv[2], &bl, &neg) || neg || get_u64_array(env, argv[3], &o, &no)) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "relinearize(ct3, rlk, baseLog, out)");
        return NULL;
    }
    fhe_ctx_info ci;
    fhe_ctx_get_info(c, &ci);
    const size_t n = ci.n;
    if (nc % (3 * n) || nk % (2 * n) || no != nc / 3 * 2) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "ct3 [batch][3][n], rlk [level][2][n], out [batch][2][n]");
        return NULL;
    }
    const uint32_t level = (uint32_t)(nk / (2 * n));
    uint64_t *prep = level ? (uint64_t *)malloc(nk * 8) : NULL;
    int rc = level ? fhe_relin_key_prepare(c, level, k, prep, FHE_HOST) : 0;
    if (!rc) rc = fhe_relinearize_batch(c, bl ? (uint32_t)bl : 4, level, ct, prep, o, nc / (3 * n), FHE_HOST);
    free(prep);
    if (rc) return throw_fhe(env, rc);
    return argv[3];
}

/* blindRotate(acc, lweA, lweB, bsk, baseLog, level): k = 1, in place on acc
 * [batch][2][n]; lweA [batch][dim]; lweB [batch]; bsk [dim][2*level][2][n]
 * coefficient-form GGSWs (BootstrapEngine::blind_rotate :547-577) */
static napi_value ctx_blind_rotate(napi_env env, napi_callback_info info) {
    size_t argc = 6;
    napi_value argv[6];
    fhe_ctx *c = ctx_this(env, info, &argc, argv);
    uint64_t *acc, *la, *lb, *bsk, bl, lv;
    size_t nacc, nla, nlb, nbsk;
    int neg;
    if (!c || argc < 6 || get_u64_array(env, argv[0], &acc, &nacc) || get_u64_array(env, argv[1], &la, &nla) ||
        get_u64_array(env, argv[2], &lb, &nlb) || get_u64_array(env, argv[3], &bsk, &nbsk) ||
        get_u64(env, argv[4], &bl, &neg) || neg || get_u64(env, argv[5], &lv, &neg) || neg || lv == 0) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "blindRotate(acc, lweA, lweB, bsk, baseLog, level)");
        return NULL;
    }
    fhe_ctx_info ci;
    fhe_ctx_get_info(c, &ci);
    const size_t n = ci.n, ggsw = 4 * lv * n;
    if (nacc % (2 * n) || nlb != nacc / (2 * n) || (nlb && nla % nlb) || nbsk % ggsw ||
        (nlb && nbsk / ggsw != nla / nlb)) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "shape mismatch (k = 1)");
        return NULL;
    }
    const uint32_t dim = nlb ? (uint32_t)(nla / nlb) : 0;
    uint64_t *prep = (uint64_t *)malloc(nbsk ? nbsk * 8 : 8);
    int rc = nbsk ? fhe_ggsw_prepare(c, 1, (uint32_t)(lv * dim), bsk, prep, FHE_HOST) : 0;
    if (!rc) rc = fhe_blind_rotate_batch(c, 1, (uint32_t)bl, (uint32_t)lv, dim, la, lb, ci.q, prep, acc, nlb, FHE_HOST);
    free(prep);
    if (rc) return throw_fhe(env, rc);
    return argv[0];
}

static napi_value ctx_info(napi_env env, napi_callback_info info) {
    size_t argc = 0;
    fhe_ctx *c = ctx_this(env, info, &argc, NULL);
    if (!c) return NULL;
    fhe_ctx_info ci;
    int rc = fhe_ctx_get_info(c, &ci);
    if (rc) return throw_fhe(env, rc);
    napi_value o, v;
    NAPI_CALL(env, napi_create_object(env, &o));
    set(env, o, "degree", make_i64(env, ci.n));
    napi_create_bigint_uint64(env, ci.q, &v);
    set(env, o, "modulus", v);
    napi_create_bigint_uint64(env, ci.psi, &v);
    set(env, o, "primitiveRoot", v);
    napi_create_bigint_uint64(env, ci.inv_n, &v);
    set(env, o, "invN", v);
    set(env, o, "mode", make_str(env, ci.mode ? "negacyclic" : "compat"));
    set(env, o, "wordBits", make_i64(env, ci.word_bits));
    set(env, o, "device", make_i64(env, ci.device));
    return o;
}

/* ------------------------------------------------------------------ module */
static napi_value init(napi_env env, napi_value exports) {
    napi_property_descriptor fns[] = {
        {"initialize", NULL, js_initialize, NULL, NULL, NULL, napi_default, NULL},
        {"detectHardware", NULL, js_detect, NULL, NULL, NULL, napi_default, NULL},
        {"version", NULL, js_version, NULL, NULL, NULL, napi_default, NULL},
        {"modmulBatch", NULL, js_modmul_batch, NULL, NULL, NULL, napi_default, NULL},
        {"mlMontgomeryMulBatch", NULL, js_ml_montmul, NULL, NULL, NULL, napi_default, NULL},
    };
    for (size_t i = 0; i < sizeof fns / sizeof fns[0]; ++i) fns[i].attributes = napi_enumerable;
    NAPI_CALL(env, napi_define_properties(env, exports, sizeof fns / sizeof fns[0], fns));

    napi_property_descriptor ma_props[] = {
        {"montgomeryMul", NULL, ma_montgomery_mul, NULL, NULL, NULL, napi_default, NULL},
        {"modAdd", NULL, ma_mod_add, NULL, NULL, NULL, napi_default, NULL},
        {"modSub", NULL, ma_mod_sub, NULL, NULL, NULL, napi_default, NULL},
        {"toMontgomery", NULL, ma_to_mont, NULL, NULL, NULL, napi_default, NULL},
        {"fromMontgomery", NULL, ma_from_mont, NULL, NULL, NULL, napi_default, NULL},
        {"getModulus", NULL, ma_get_modulus, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_value ma_cls;
    NAPI_CALL(env, napi_define_class(env, "ModularArithmetic", NAPI_AUTO_LENGTH, ma_ctor, NULL,
                                     sizeof ma_props / sizeof ma_props[0], ma_props, &ma_cls));
    set(env, exports, "ModularArithmetic", ma_cls);

    napi_property_descriptor ctx_props[] = {
        {"forward", NULL, ctx_forward, NULL, NULL, NULL, napi_default, NULL},
        {"inverse", NULL, ctx_inverse, NULL, NULL, NULL, napi_default, NULL},
        {"polymul", NULL, ctx_polymul, NULL, NULL, NULL, napi_default, NULL},
        {"pointwise", NULL, ctx_pointwise, NULL, NULL, NULL, napi_default, NULL},
        {"add", NULL, ctx_add, NULL, NULL, NULL, napi_default, NULL},
        {"sub", NULL, ctx_sub, NULL, NULL, NULL, napi_default, NULL},
        {"negate", NULL, ctx_negate, NULL, NULL, NULL, napi_default, NULL},
        {"mulScalar", NULL, ctx_mul_scalar, NULL, NULL, NULL, napi_default, NULL},
        {"forwardMul", NULL, ctx_fwd_mul, NULL, NULL, NULL, napi_default, NULL},
        {"externalProduct", NULL, ctx_ext_product, NULL, NULL, NULL, napi_default, NULL},
        {"ctMultiply", NULL, ctx_ct_multiply, NULL, NULL, NULL, napi_default, NULL},
        {"relinearize", NULL, ctx_relinearize, NULL, NULL, NULL, napi_default, NULL},
        {"blindRotate", NULL, ctx_blind_rotate, NULL, NULL, NULL, napi_default, NULL},
        {"info", NULL, ctx_info, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_value ctx_cls;
    NAPI_CALL(env, napi_define_class(env, "NttContext", NAPI_AUTO_LENGTH, ctx_ctor, NULL,
                                     sizeof ctx_props / sizeof ctx_props[0], ctx_props, &ctx_cls));
    set(env, exports, "NttContext", ctx_cls);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
