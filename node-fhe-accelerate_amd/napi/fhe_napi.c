/*
 * fhe_napi.c -- plain node_api.h addon over libfhe_gpu.so.
 *
 * Replaces the napi-rs binding (src/native/lib.rs:22-133, bridge.rs:3-41)
 * with the same JS surface as index.d.ts:
 *   initialize(), detectHardware(), version(), class ModularArithmetic
 * plus what the TS FHEEngine needs (src/api/fhe-engine.ts:33-78, wired in
 * lib/engine.js):
 *   NttContext    one transform context (fhe_ctx) and every batched entry
 *                 point of include/fhe_gpu.h;
 *   DeviceBuffer  u64 words resident in HBM on a context's device (the
 *                 native object behind a Ciphertext / key `handle`), freed
 *                 stream-ordered when collected or free()d; view() slices.
 * Every NttContext compute method takes BigUint64Array / BigInt64Array host
 * buffers (zero-copy; FHE_HOST, the library stages them through HBM) or
 * DeviceBuffers (FHE_DEVICE: nothing crosses PCIe), one placement per call,
 * and has a synchronous form and an `...Async` form that runs as
 * napi_async_work on the libuv pool and returns a Promise.  Jobs on one
 * context are serialised on its stream; device jobs synchronise the stream
 * before they complete, so a resolved Promise means the result is in place.
 * Errors carry the library's message and a FHEErrorCode name
 * (src/api/types.ts:140-151) in `code`: INVALID_PARAMETERS for parameter
 * errors, HARDWARE_UNAVAILABLE without a device, NATIVE_ERROR otherwise; the
 * numeric status is in `status`.  The reference's cxx bridge aborted the
 * process on a C++ exception instead.
 */
#include <node_api.h>
#include <pthread.h>
#include <stdint.h>
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

/* FHEErrorCode (types.ts:140-151) of a library status */
static const char *code_name(int rc) {
    if (rc <= FHE_ERR_DEGREE_POW2 && rc >= FHE_ERR_UNSUPPORTED) return "INVALID_PARAMETERS";
    if (rc == FHE_ERR_DEVICE) return "HARDWARE_UNAVAILABLE";
    return "NATIVE_ERROR";
}
static napi_value make_error(napi_env env, int rc, const char *msg) {
    napi_value m, c, e, st;
    napi_create_string_utf8(env, msg, NAPI_AUTO_LENGTH, &m);
    napi_create_string_utf8(env, code_name(rc), NAPI_AUTO_LENGTH, &c);
    napi_create_error(env, c, m, &e);
    napi_create_int32(env, rc, &st);
    napi_set_named_property(env, e, "status", st);
    return e;
}
static napi_value throw_fhe(napi_env env, int rc) {
    napi_throw(env, make_error(env, rc, fhe_last_error()));
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

/* BigUint64Array / BigInt64Array -> pointer + element count */
static int get_u64_array(napi_env env, napi_value v, uint64_t **data, size_t *count) {
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return -1;
    napi_typedarray_type type;
    size_t len, off;
    void *raw;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &len, &raw, &ab, &off) != napi_ok) return -1;
    if (type != napi_biguint64_array && type != napi_bigint64_array) return -1;
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

/* ------------------------------------------------------------------ contexts and device memory */
/* A context is shared by its JS object and every DeviceBuffer allocated on
 * it (refcounted on the JS thread, where all finalizers run); `mu`
 * serialises the jobs of one context (each job's launches and its final
 * stream synchronisation form one unit). */
typedef struct {
    fhe_ctx *c;
    int refs;
    pthread_mutex_t mu;
} nctx;
static void nctx_release(nctx *k) {
    if (--k->refs == 0) {
        fhe_ctx_destroy(k->c);
        pthread_mutex_destroy(&k->mu);
        free(k);
    }
}

/* Device memory block (refcounted: a view shares its parent's block). */
typedef struct {
    nctx *owner;
    void *base;
    int refs;
} dblock;
typedef struct {
    dblock *blk;
    size_t off, words;  /* in u64 words */
} dbuf;
static void dblock_release(dblock *b) {
    if (--b->refs == 0) {
        if (b->base) fhe_ctx_free(b->owner->c, b->base);
        nctx_release(b->owner);
        free(b);
    }
}
static void dbuf_finalize(napi_env env, void *data, void *hint) {
    (void)env;
    (void)hint;
    dbuf *d = (dbuf *)data;
    if (d->blk) dblock_release(d->blk);
    free(d);
}

static napi_ref g_ctx_ctor, g_buf_ctor;

static nctx *unwrap_ctx(napi_env env, napi_value v) {
    bool is = false;
    napi_value ctor;
    if (!g_ctx_ctor || napi_get_reference_value(env, g_ctx_ctor, &ctor) != napi_ok) return NULL;
    if (napi_instanceof(env, v, ctor, &is) != napi_ok || !is) return NULL;
    void *p = NULL;
    napi_unwrap(env, v, &p);
    return (nctx *)p;
}
static dbuf *unwrap_buf(napi_env env, napi_value v) {
    napi_valuetype t;
    if (napi_typeof(env, v, &t) != napi_ok || t != napi_object) return NULL;
    bool is = false;
    napi_value ctor;
    if (!g_buf_ctor || napi_get_reference_value(env, g_buf_ctor, &ctor) != napi_ok) return NULL;
    if (napi_instanceof(env, v, ctor, &is) != napi_ok || !is) return NULL;
    void *p = NULL;
    napi_unwrap(env, v, &p);
    return (dbuf *)p;
}
static uint64_t *dbuf_ptr(const dbuf *d) { return (uint64_t *)d->blk->base + d->off; }

/* ------------------------------------------------------------------ class NttContext */
static void ctx_finalize(napi_env env, void *data, void *hint) {
    (void)env;
    (void)hint;
    nctx_release((nctx *)data);
}

/* NttContext(degree, modulus, mode?, device? | devices[]?) -- an array of
 * device ordinals makes a multi-device context (fhe_ctx_create_multi):
 * every host-buffer batch is split across the devices. */
static napi_value ctx_ctor(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4], self;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, &self, NULL));
    uint64_t n, q, mode = 0, dev = 0;
    int neg;
    bool is_arr = false;
    if (argc > 3) napi_is_array(env, argv[3], &is_arr);
    if (argc < 2 || get_u64(env, argv[0], &n, &neg) || neg || get_u64(env, argv[1], &q, &neg) || neg ||
        (argc > 2 && (get_u64(env, argv[2], &mode, &neg) || neg)) ||
        (argc > 3 && !is_arr && (get_u64(env, argv[3], &dev, &neg) || neg))) {
        napi_throw_type_error(env, "INVALID_PARAMETERS",
                              "NttContext(degree, modulus: bigint|number, mode?, device?: number|number[])");
        return NULL;
    }
    fhe_ctx *c = NULL;
    int rc;
    if (is_arr) {
        uint32_t len = 0;
        napi_get_array_length(env, argv[3], &len);
        int devs[64];
        if (len == 0 || len > 64) {
            napi_throw_range_error(env, "INVALID_PARAMETERS", "1 to 64 devices");
            return NULL;
        }
        for (uint32_t i = 0; i < len; ++i) {
            napi_value e;
            uint64_t d;
            napi_get_element(env, argv[3], i, &e);
            if (get_u64(env, e, &d, &neg) || neg) {
                napi_throw_type_error(env, "INVALID_PARAMETERS", "devices must be non-negative integers");
                return NULL;
            }
            devs[i] = (int)d;
        }
        rc = fhe_ctx_create_multi((uint32_t)n, q, (int)mode, devs, (int)len, &c);
    } else {
        rc = fhe_ctx_create((uint32_t)n, q, (int)mode, (int)dev, &c);
    }
    if (rc) return throw_fhe(env, rc);
    nctx *k = (nctx *)calloc(1, sizeof *k);
    k->c = c;
    k->refs = 1;
    pthread_mutex_init(&k->mu, NULL);
    NAPI_CALL(env, napi_wrap(env, self, k, ctx_finalize, NULL, NULL));
    return self;
}

/* ------------------------------------------------------------------ class DeviceBuffer */
/* new DeviceBuffer(ctx: NttContext, words: number) -- uninitialised words
 * new DeviceBuffer(parent: DeviceBuffer, offsetWords, words) -- a view */
static napi_value buf_ctor(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], self;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, &self, NULL));
    dbuf *parent = argc > 0 ? unwrap_buf(env, argv[0]) : NULL;
    uint64_t words, off = 0;
    int neg;
    if (parent) {
        if (!parent->blk || argc < 3 || get_u64(env, argv[1], &off, &neg) || neg ||
            get_u64(env, argv[2], &words, &neg) || neg || off > parent->words || words > parent->words - off) {
            napi_throw_range_error(env, "INVALID_PARAMETERS", "DeviceBuffer(parent, offsetWords, words) out of range");
            return NULL;
        }
        dbuf *v = (dbuf *)calloc(1, sizeof *v);
        v->blk = parent->blk;
        v->blk->refs++;
        v->off = parent->off + off;
        v->words = (size_t)words;
        NAPI_CALL(env, napi_wrap(env, self, v, dbuf_finalize, NULL, NULL));
        return self;
    }
    nctx *k = argc > 0 ? unwrap_ctx(env, argv[0]) : NULL;
    if (!k || argc < 2 || get_u64(env, argv[1], &words, &neg) || neg) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "DeviceBuffer(ctx: NttContext, words: number)");
        return NULL;
    }
    dblock *b = (dblock *)calloc(1, sizeof *b);
    int rc = fhe_ctx_alloc(k->c, (size_t)words * 8, &b->base);
    if (rc) {
        free(b);
        return throw_fhe(env, rc);
    }
    b->owner = k;
    b->refs = 1;
    k->refs++;
    dbuf *d = (dbuf *)calloc(1, sizeof *d);
    d->blk = b;
    d->words = (size_t)words;
    NAPI_CALL(env, napi_wrap(env, self, d, dbuf_finalize, NULL, NULL));
    return self;
}
static dbuf *buf_this(napi_env env, napi_callback_info info, size_t *argc, napi_value *argv, napi_value *self) {
    napi_value s;
    if (napi_get_cb_info(env, info, argc, argv, &s, NULL) != napi_ok) return NULL;
    if (self) *self = s;
    dbuf *d = unwrap_buf(env, s);
    if (!d || !d->blk) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "not a live DeviceBuffer");
        return NULL;
    }
    return d;
}
static napi_value buf_words(napi_env env, napi_callback_info info) {
    size_t argc = 0;
    dbuf *d = buf_this(env, info, &argc, NULL, NULL);
    return d ? make_i64(env, (int64_t)d->words) : NULL;
}
/* handle: the device address as a bigint (an opaque id for the TS handle types) */
static napi_value buf_handle(napi_env env, napi_callback_info info) {
    size_t argc = 0;
    dbuf *d = buf_this(env, info, &argc, NULL, NULL);
    if (!d) return NULL;
    napi_value v;
    napi_create_bigint_uint64(env, (uint64_t)(uintptr_t)dbuf_ptr(d), &v);
    return v;
}
/* upload(src: BigUint64Array|BigInt64Array, offsetWords = 0) -> this */
static napi_value buf_upload(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], self;
    dbuf *d = buf_this(env, info, &argc, argv, &self);
    if (!d) return NULL;
    uint64_t *src, off = 0;
    size_t n;
    int neg;
    if (argc < 1 || get_u64_array(env, argv[0], &src, &n) || (argc > 1 && (get_u64(env, argv[1], &off, &neg) || neg)) ||
        off + n > d->words) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "upload(src: BigUint64Array, offsetWords?) out of range");
        return NULL;
    }
    pthread_mutex_lock(&d->blk->owner->mu);
    int rc = fhe_ctx_memcpy(d->blk->owner->c, dbuf_ptr(d) + off, src, n * 8, FHE_COPY_H2D);
    pthread_mutex_unlock(&d->blk->owner->mu);
    if (rc) return throw_fhe(env, rc);
    return self;
}
/* download(dst?: BigUint64Array, offsetWords = 0, words = rest) -> dst */
static napi_value buf_download(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], self;
    dbuf *d = buf_this(env, info, &argc, argv, &self);
    if (!d) return NULL;
    uint64_t off = 0, cnt;
    int neg;
    if (argc > 1 && (get_u64(env, argv[1], &off, &neg) || neg)) off = ~0ull;
    cnt = off <= d->words ? d->words - off : 0;
    if (argc > 2 && (get_u64(env, argv[2], &cnt, &neg) || neg)) cnt = ~0ull;
    if (off > d->words || cnt > d->words - off) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "download(dst?, offsetWords?, words?) out of range");
        return NULL;
    }
    napi_value dst;
    uint64_t *p;
    size_t n;
    napi_valuetype t = napi_undefined;
    if (argc > 0) napi_typeof(env, argv[0], &t);
    if (argc > 0 && t != napi_undefined && t != napi_null) {
        dst = argv[0];
        if (get_u64_array(env, dst, &p, &n) || n != cnt) {
            napi_throw_range_error(env, "INVALID_PARAMETERS", "dst must be a BigUint64Array of the copied length");
            return NULL;
        }
    } else {
        napi_value ab;
        void *raw;
        NAPI_CALL(env, napi_create_arraybuffer(env, cnt * 8, &raw, &ab));
        NAPI_CALL(env, napi_create_typedarray(env, napi_biguint64_array, cnt, ab, 0, &dst));
        p = (uint64_t *)raw;
    }
    pthread_mutex_lock(&d->blk->owner->mu);
    int rc = fhe_ctx_memcpy(d->blk->owner->c, p, dbuf_ptr(d) + off, cnt * 8, FHE_COPY_D2H);
    pthread_mutex_unlock(&d->blk->owner->mu);
    if (rc) return throw_fhe(env, rc);
    return dst;
}
/* copyFrom(src: DeviceBuffer, dstOffset = 0, srcOffset = 0, words = src rest) -> this (device to device) */
static napi_value buf_copy_from(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4], self;
    dbuf *d = buf_this(env, info, &argc, argv, &self);
    if (!d) return NULL;
    dbuf *s = argc > 0 ? unwrap_buf(env, argv[0]) : NULL;
    uint64_t doff = 0, soff = 0, cnt;
    int neg, bad = !s || !s->blk || s->blk->owner != d->blk->owner;
    if (!bad && argc > 1 && (get_u64(env, argv[1], &doff, &neg) || neg)) bad = 1;
    if (!bad && argc > 2 && (get_u64(env, argv[2], &soff, &neg) || neg)) bad = 1;
    cnt = !bad && soff <= s->words ? s->words - soff : 0;
    if (!bad && argc > 3 && (get_u64(env, argv[3], &cnt, &neg) || neg)) bad = 1;
    if (bad || soff > s->words || cnt > s->words - soff || doff > d->words || cnt > d->words - doff) {
        napi_throw_range_error(env, "INVALID_PARAMETERS",
                               "copyFrom(src: DeviceBuffer of the same context, dstOffset?, srcOffset?, words?)");
        return NULL;
    }
    pthread_mutex_lock(&d->blk->owner->mu);
    int rc = fhe_ctx_memcpy(d->blk->owner->c, dbuf_ptr(d) + doff, dbuf_ptr(s) + soff, cnt * 8, FHE_COPY_D2D);
    pthread_mutex_unlock(&d->blk->owner->mu);
    if (rc) return throw_fhe(env, rc);
    return self;
}
/* view(offsetWords, words) -> DeviceBuffer sharing this memory */
static napi_value buf_view(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], self;
    dbuf *d = buf_this(env, info, &argc, argv, &self);
    if (!d) return NULL;
    napi_value ctor, obj, a[3] = {self, argc > 0 ? argv[0] : NULL, argc > 1 ? argv[1] : NULL};
    if (argc < 2) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "view(offsetWords, words)");
        return NULL;
    }
    NAPI_CALL(env, napi_get_reference_value(env, g_buf_ctor, &ctor));
    if (napi_new_instance(env, ctor, 3, a, &obj) != napi_ok) return NULL;
    return obj;
}
/* free(): release this handle's reference now (the memory goes when no view holds it) */
static napi_value buf_free(napi_env env, napi_callback_info info) {
    size_t argc = 0;
    napi_value self;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, NULL, &self, NULL));
    dbuf *d = unwrap_buf(env, self);
    if (d && d->blk) {
        dblock_release(d->blk);
        d->blk = NULL;
        d->words = 0;
    }
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

/* ---- jobs: every compute method runs either synchronously on the JS
 * thread (`name`) or as napi_async_work on the libuv pool (`nameAsync`,
 * returns a Promise of the output).  A job holds references to its buffers
 * and to the context object until it completes. */
#define MAXP 12
typedef struct job job;
typedef int (*job_fn)(job *);
struct job {
    job_fn fn;
    void *op;           /* the library entry point for the generic runners */
    nctx *k;
    fhe_ctx *c;
    int where;          /* FHE_HOST or FHE_DEVICE */
    uint64_t *p[MAXP];
    uint64_t v[10];
    double d;
    size_t batch;
    uint64_t *owned;    /* host scratch (prepared keys), freed on completion */
    int rc;
    char err[512];
    napi_ref refs[MAXP + 2];
    int nref;
    dblock *blks[MAXP]; /* async path: device blocks pinned until completion */
    int nblk;
    napi_ref ret;       /* async path */
    napi_deferred def;
    napi_async_work work;
};

typedef struct {
    nctx *k;
    fhe_ctx *c;
    napi_value self;
    napi_value argv[14];
    size_t argc;
    int async;
    int where;          /* -1 until the first buffer argument */
    size_t n;
    uint64_t q;
    dblock *blks[MAXP]; /* device blocks of the buffer arguments (arr_arg) */
    int nblk;
} call;

static int call_begin(napi_env env, napi_callback_info info, size_t want, call *k) {
    k->argc = want;
    void *data = NULL;
    if (napi_get_cb_info(env, info, &k->argc, k->argv, &k->self, &data) != napi_ok) return -1;
    k->async = data != NULL;
    k->where = -1;
    k->nblk = 0;
    k->k = unwrap_ctx(env, k->self);
    if (!k->k) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "not an NttContext");
        return -1;
    }
    k->c = k->k->c;
    fhe_ctx_info ci;
    fhe_ctx_get_info(k->c, &ci);
    k->n = ci.n;
    k->q = ci.q;
    return 0;
}

static job *job_new(const call *k, job_fn fn, void *op) {
    job *j = (job *)calloc(1, sizeof *j);
    j->fn = fn;
    j->op = op;
    j->k = k->k;
    j->c = k->c;
    j->where = k->where < 0 ? FHE_HOST : k->where;
    return j;
}

static void job_free(napi_env env, job *j) {
    for (int i = 0; i < j->nref; ++i) napi_delete_reference(env, j->refs[i]);
    /* after the job's final stream synchronisation: a buffer freed by the
     * caller meanwhile is returned to the pool only now */
    for (int i = 0; i < j->nblk; ++i) dblock_release(j->blks[i]);
    if (j->ret) napi_delete_reference(env, j->ret);
    free(j->owned);
    free(j);
}

/* run the job under the context lock; device jobs end with a stream
 * synchronisation (results in place, kernel errors reported here) */
static int job_run(job *j) {
    pthread_mutex_lock(&j->k->mu);
    int rc = j->fn(j);
    if (!rc && j->where == FHE_DEVICE) rc = fhe_ctx_synchronize(j->c);
    pthread_mutex_unlock(&j->k->mu);
    return rc;
}

static void job_exec(napi_env env, void *data) {
    (void)env;
    job *j = (job *)data;
    j->rc = job_run(j);
    if (j->rc) snprintf(j->err, sizeof j->err, "%s", fhe_last_error()); /* thread-local: read on this thread */
}

static void job_done(napi_env env, napi_status status, void *data) {
    job *j = (job *)data;
    napi_value v;
    if (status != napi_ok || j->rc) {
        napi_value e = make_error(env, j->rc ? j->rc : FHE_ERR_DEVICE,
                                  status != napi_ok ? "async work cancelled" : j->err);
        napi_reject_deferred(env, j->def, e);
    } else {
        napi_get_reference_value(env, j->ret, &v);
        napi_resolve_deferred(env, j->def, v);
    }
    napi_delete_async_work(env, j->work);
    job_free(env, j);
}

/* Run or queue the job; `ret` is what the call returns / resolves with.
 * keep[] are the JS values the work reads or writes (kept alive). */
static napi_value job_go(napi_env env, const call *k, job *j, napi_value ret, napi_value *keep, int nkeep) {
    if (!k->async) {
        int rc = job_run(j);
        free(j->owned);
        free(j);
        if (rc) return throw_fhe(env, rc);
        return ret;
    }
    for (int i = 0; i < nkeep && j->nref < MAXP + 1; ++i) napi_create_reference(env, keep[i], 1, &j->refs[j->nref++]);
    /* Each device block the job reads or writes is pinned by a block
     * reference (not only its JS object): buf.free() while the job is queued
     * must not let fhe_ctx_free enqueue the release ahead of the job's
     * kernels, where a later allocation could reuse the memory. */
    for (int i = 0; i < k->nblk; ++i) {
        k->blks[i]->refs++;
        j->blks[j->nblk++] = k->blks[i];
    }
    napi_create_reference(env, k->self, 1, &j->refs[j->nref++]);
    napi_create_reference(env, ret, 1, &j->ret);
    napi_value promise, name;
    napi_create_promise(env, &j->def, &promise);
    napi_create_string_utf8(env, "fhe_gpu", NAPI_AUTO_LENGTH, &name);
    if (napi_create_async_work(env, NULL, name, job_exec, job_done, j, &j->work) != napi_ok ||
        napi_queue_async_work(env, j->work) != napi_ok) {
        job_free(env, j);
        napi_throw_error(env, "NATIVE_ERROR", "could not queue async work");
        return NULL;
    }
    return promise;
}

static int bad_args(napi_env env, const char *usage) {
    napi_throw_type_error(env, "INVALID_PARAMETERS", usage);
    return -1;
}
/* Buffer argument i: a host typed array or a DeviceBuffer of this context;
 * every buffer of one call has the same placement. */
static int arr_arg(napi_env env, call *k, size_t i, uint64_t **p, size_t *cnt) {
    if (i >= k->argc) return -1;
    int w;
    dbuf *d = unwrap_buf(env, k->argv[i]);
    if (d) {
        if (!d->blk || d->blk->owner != k->k) return -1;
        int seen = 0;
        for (int b = 0; b < k->nblk; ++b) seen |= k->blks[b] == d->blk;
        if (!seen) {
            if (k->nblk >= MAXP) return -1;
            k->blks[k->nblk++] = d->blk;
        }
        *p = dbuf_ptr(d);
        *cnt = d->words;
        w = FHE_DEVICE;
    } else {
        if (get_u64_array(env, k->argv[i], p, cnt)) return -1;
        w = FHE_HOST;
    }
    if (k->where >= 0 && k->where != w) return -1;
    k->where = w;
    return 0;
}
static int num_arg(napi_env env, const call *k, size_t i, uint64_t *v) {
    int neg;
    if (i >= k->argc || get_u64(env, k->argv[i], v, &neg) || neg) return -1;
    return 0;
}
static int dbl_arg(napi_env env, const call *k, size_t i, double *v) {
    if (i >= k->argc) return -1;
    return napi_get_value_double(env, k->argv[i], v) == napi_ok ? 0 : -1;
}
static int undef_arg(napi_env env, const call *k, size_t i) {
    if (i >= k->argc) return 1;
    napi_valuetype t;
    napi_typeof(env, k->argv[i], &t);
    return t == napi_undefined || t == napi_null;
}
/* seed argument: BigUint64Array(4) (256-bit ChaCha20 key), host memory */
static int seed_arg(napi_env env, const call *k, size_t i, uint64_t seed[4]) {
    uint64_t *p;
    size_t n;
    if (i >= k->argc || get_u64_array(env, k->argv[i], &p, &n) || n != 4) return -1;
    memcpy(seed, p, 32);
    return 0;
}
/* ------------------------------------------------------------------ compute methods */
typedef int (*unary_fn)(fhe_ctx *, const uint64_t *, uint64_t *, size_t, int);
typedef int (*binary_fn)(fhe_ctx *, const uint64_t *, const uint64_t *, uint64_t *, size_t, int);
static int run_unary(job *j) { return ((unary_fn)j->op)(j->c, j->p[0], j->p[1], j->batch, j->where); }
static int run_binary(job *j) { return ((binary_fn)j->op)(j->c, j->p[0], j->p[1], j->p[2], j->batch, j->where); }

static napi_value range_err(napi_env env, const char *msg) {
    napi_throw_range_error(env, "INVALID_PARAMETERS", msg);
    return NULL;
}

/* op(a, out?) ; out defaults to a (in place, like NTTProcessor::forward_ntt) */
static napi_value ctx_unary(napi_env env, napi_callback_info info, unary_fn fn) {
    call k;
    if (call_begin(env, info, 2, &k)) return NULL;
    uint64_t *a, *o;
    size_t na, no;
    if (arr_arg(env, &k, 0, &a, &na)) return bad_args(env, "expected BigUint64Array or DeviceBuffer"), NULL;
    napi_value ret = k.argv[0];
    o = a;
    no = na;
    if (!undef_arg(env, &k, 1)) {
        if (arr_arg(env, &k, 1, &o, &no) || no != na)
            return bad_args(env, "out must be a buffer of equal length and placement"), NULL;
        ret = k.argv[1];
    }
    if (na % k.n) return range_err(env, "Coefficient count must equal polynomial degree");
    job *j = job_new(&k, run_unary, (void *)fn);
    j->p[0] = a; j->p[1] = o; j->batch = na / k.n;
    return job_go(env, &k, j, ret, k.argv, (int)(k.argc < 2 ? k.argc : 2));
}

static napi_value ctx_binary(napi_env env, napi_callback_info info, binary_fn fn) {
    call k;
    if (call_begin(env, info, 3, &k)) return NULL;
    uint64_t *a, *b, *o;
    size_t na, nb, no;
    if (arr_arg(env, &k, 0, &a, &na) || arr_arg(env, &k, 1, &b, &nb) || arr_arg(env, &k, 2, &o, &no) || na != nb ||
        na != no)
        return bad_args(env, "expected (a, b, out) buffers of equal length and placement"), NULL;
    if (na % k.n) return range_err(env, "Coefficient count must equal polynomial degree");
    job *j = job_new(&k, run_binary, (void *)fn);
    j->p[0] = a; j->p[1] = b; j->p[2] = o; j->batch = na / k.n;
    return job_go(env, &k, j, k.argv[2], k.argv, 3);
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

static int run_mul_scalar(job *j) { return fhe_poly_mul_scalar_batch(j->c, j->p[0], j->v[0], j->p[1], j->batch, j->where); }
static napi_value ctx_mul_scalar(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 3, &k)) return NULL;
    uint64_t *a, *o, s;
    size_t na, no;
    if (arr_arg(env, &k, 0, &a, &na) || num_arg(env, &k, 1, &s) || arr_arg(env, &k, 2, &o, &no) || na != no ||
        na % k.n)
        return bad_args(env, "mulScalar(a, scalar, out)"), NULL;
    job *j = job_new(&k, run_mul_scalar, NULL);
    j->p[0] = a; j->p[1] = o; j->v[0] = s; j->batch = na / k.n;
    return job_go(env, &k, j, k.argv[2], k.argv, 3);
}

/* externalProduct(glwe, ggswCoeff, baseLog, level, out): k = 1, the key
 * prepared per call (host buffers: into host scratch; device: in place of
 * a stream-ordered temporary is not available here, so device callers use
 * prepareGgsw + externalProductPrepared) */
static int run_ext_product(job *j) {
    const size_t nk = j->v[2];
    if (j->where == FHE_DEVICE) return FHE_ERR_INVALID_ARG;
    j->owned = (uint64_t *)malloc(nk * 8);
    int rc = fhe_ggsw_prepare(j->c, 1, (uint32_t)j->v[1], j->p[1], j->owned, FHE_HOST);
    if (!rc) rc = fhe_external_product_batch(j->c, 1, (uint32_t)j->v[0], (uint32_t)j->v[1], j->p[0], j->owned, j->p[2],
                                             j->batch, FHE_HOST);
    return rc;
}
static napi_value ctx_ext_product(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 5, &k)) return NULL;
    uint64_t *g, *kk, *o, bl, lv;
    size_t ng, nk, no;
    if (arr_arg(env, &k, 0, &g, &ng) || arr_arg(env, &k, 1, &kk, &nk) || num_arg(env, &k, 2, &bl) ||
        num_arg(env, &k, 3, &lv) || arr_arg(env, &k, 4, &o, &no) || ng != no || k.where != FHE_HOST)
        return bad_args(env, "externalProduct(glwe, ggsw, baseLog, level, out): host buffers "
                             "(device buffers: prepareGgsw + externalProductPrepared)"), NULL;
    const size_t per = 2 * k.n;
    if (ng % per || nk != (size_t)4 * lv * k.n) return range_err(env, "shape mismatch (k = 1)");
    job *j = job_new(&k, run_ext_product, NULL);
    j->p[0] = g; j->p[1] = kk; j->p[2] = o; j->v[0] = bl; j->v[1] = lv; j->v[2] = nk; j->batch = ng / per;
    return job_go(env, &k, j, k.argv[4], k.argv, 5);
}

/* prepareGgsw(ggsw [(k+1)L][k+1][n], k, level, out): NTT x R form */
static int run_prep_ggsw(job *j) {
    return fhe_ggsw_prepare(j->c, (uint32_t)j->v[0], (uint32_t)j->v[1], j->p[0], j->p[1], j->where);
}
static napi_value ctx_prep_ggsw(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 4, &k)) return NULL;
    uint64_t *g, *o, kd, lv;
    size_t ng, no;
    if (arr_arg(env, &k, 0, &g, &ng) || num_arg(env, &k, 1, &kd) || num_arg(env, &k, 2, &lv) ||
        arr_arg(env, &k, 3, &o, &no) || ng != no || kd == 0 || lv == 0)
        return bad_args(env, "prepareGgsw(ggsw, k, level, out)"), NULL;
    if (ng % ((kd + 1) * lv * (kd + 1) * k.n)) return range_err(env, "ggsw must be [count][(k+1)L][k+1][n]");
    job *j = job_new(&k, run_prep_ggsw, NULL);
    j->p[0] = g; j->p[1] = o; j->v[0] = kd; j->v[1] = lv * (ng / ((kd + 1) * lv * (kd + 1) * k.n));
    return job_go(env, &k, j, k.argv[3], k.argv, 4);
}
/* externalProductPrepared(glwe [batch][k+1][n], ggswPrep, k, baseLog, level, out) */
static int run_ext_prepared(job *j) {
    return fhe_external_product_batch(j->c, (uint32_t)j->v[0], (uint32_t)j->v[1], (uint32_t)j->v[2], j->p[0], j->p[1],
                                      j->p[2], j->batch, j->where);
}
static napi_value ctx_ext_prepared(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 6, &k)) return NULL;
    uint64_t *g, *kk, *o, kd, bl, lv;
    size_t ng, nk, no;
    if (arr_arg(env, &k, 0, &g, &ng) || arr_arg(env, &k, 1, &kk, &nk) || num_arg(env, &k, 2, &kd) ||
        num_arg(env, &k, 3, &bl) || num_arg(env, &k, 4, &lv) || arr_arg(env, &k, 5, &o, &no) || ng != no || kd == 0)
        return bad_args(env, "externalProductPrepared(glwe, ggswPrep, k, baseLog, level, out)"), NULL;
    if (ng % ((kd + 1) * k.n) || nk != (kd + 1) * lv * (kd + 1) * k.n) return range_err(env, "shape mismatch");
    job *j = job_new(&k, run_ext_prepared, NULL);
    j->p[0] = g; j->p[1] = kk; j->p[2] = o; j->v[0] = kd; j->v[1] = bl; j->v[2] = lv; j->batch = ng / ((kd + 1) * k.n);
    return job_go(env, &k, j, k.argv[5], k.argv, 6);
}

/* ctMultiply(ct1, ct2, out, isNtt?): ct [batch][2][n] -> out [batch][3][n]
 * (EncryptionEngine::multiply, encryption.cpp:737-798) */
static int run_ct_multiply(job *j) {
    return fhe_ct_multiply_batch(j->c, j->p[0], j->p[1], j->p[2], j->batch, (int)j->v[0], j->where);
}
static napi_value ctx_ct_multiply(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 4, &k)) return NULL;
    uint64_t *x, *y, *o, is_ntt = 0;
    size_t nx, ny, no;
    if (arr_arg(env, &k, 0, &x, &nx) || arr_arg(env, &k, 1, &y, &ny) || arr_arg(env, &k, 2, &o, &no) || nx != ny ||
        (!undef_arg(env, &k, 3) && num_arg(env, &k, 3, &is_ntt)))
        return bad_args(env, "ctMultiply(ct1, ct2, out, isNtt?)"), NULL;
    const size_t per = 2 * k.n;
    if (nx % per || no != nx / 2 * 3) return range_err(env, "ciphertexts must be [batch][2][n], out [batch][3][n]");
    job *j = job_new(&k, run_ct_multiply, NULL);
    j->p[0] = x; j->p[1] = y; j->p[2] = o; j->v[0] = is_ntt; j->batch = nx / per;
    return job_go(env, &k, j, k.argv[2], k.argv, 3);
}

/* relinearize(ct3, rlk, baseLog, out): rlk [level][2][n] (a_l, b_l) in
 * coefficient form (KeySwitchKey), prepared per call; host buffers
 * (EncryptionEngine::relinearize, encryption.cpp:904-980) */
static int run_relinearize(job *j) {
    const uint32_t level = (uint32_t)j->v[1];
    int rc = 0;
    if (level) {
        j->owned = (uint64_t *)malloc(j->v[2] * 8);
        rc = fhe_relin_key_prepare(j->c, level, j->p[1], j->owned, FHE_HOST);
    }
    if (!rc) rc = fhe_relinearize_batch(j->c, (uint32_t)j->v[0], level, j->p[0], j->owned, j->p[2], j->batch, FHE_HOST);
    return rc;
}
static napi_value ctx_relinearize(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 4, &k)) return NULL;
    uint64_t *ct, *kk, *o, bl;
    size_t nc, nk, no;
    if (arr_arg(env, &k, 0, &ct, &nc) || arr_arg(env, &k, 1, &kk, &nk) || num_arg(env, &k, 2, &bl) ||
        arr_arg(env, &k, 3, &o, &no) || k.where != FHE_HOST)
        return bad_args(env, "relinearize(ct3, rlk, baseLog, out): host buffers "
                             "(device buffers: prepareRelinKey + relinearizePrepared)"), NULL;
    const size_t n = k.n;
    if (nc % (3 * n) || nk % (2 * n) || no != nc / 3 * 2)
        return range_err(env, "ct3 [batch][3][n], rlk [level][2][n], out [batch][2][n]");
    job *j = job_new(&k, run_relinearize, NULL);
    j->p[0] = ct; j->p[1] = kk; j->p[2] = o;
    j->v[0] = bl ? bl : 4; j->v[1] = nk / (2 * n); j->v[2] = nk; j->batch = nc / (3 * n);
    return job_go(env, &k, j, k.argv[3], k.argv, 4);
}
/* prepareRelinKey(rlk [level][2][n], out) */
static int run_prep_rlk(job *j) { return fhe_relin_key_prepare(j->c, (uint32_t)j->v[0], j->p[0], j->p[1], j->where); }
static napi_value ctx_prep_rlk(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 2, &k)) return NULL;
    uint64_t *r, *o;
    size_t nr, no;
    if (arr_arg(env, &k, 0, &r, &nr) || arr_arg(env, &k, 1, &o, &no) || nr != no || nr % (2 * k.n))
        return bad_args(env, "prepareRelinKey(rlk [level][2][n], out)"), NULL;
    job *j = job_new(&k, run_prep_rlk, NULL);
    j->p[0] = r; j->p[1] = o; j->v[0] = nr / (2 * k.n);
    return job_go(env, &k, j, k.argv[1], k.argv, 2);
}
/* relinearizePrepared(ct3, rlkPrep [level][2][n], baseLog, out) */
static int run_relin_prepared(job *j) {
    return fhe_relinearize_batch(j->c, (uint32_t)j->v[0], (uint32_t)j->v[1], j->p[0], j->v[1] ? j->p[1] : NULL, j->p[2],
                                 j->batch, j->where);
}
static napi_value ctx_relin_prepared(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 4, &k)) return NULL;
    uint64_t *ct, *kk, *o, bl;
    size_t nc, nk, no;
    if (arr_arg(env, &k, 0, &ct, &nc) || arr_arg(env, &k, 1, &kk, &nk) || num_arg(env, &k, 2, &bl) ||
        arr_arg(env, &k, 3, &o, &no))
        return bad_args(env, "relinearizePrepared(ct3, rlkPrep, baseLog, out)"), NULL;
    const size_t n = k.n;
    if (nc % (3 * n) || nk % (2 * n) || no != nc / 3 * 2)
        return range_err(env, "ct3 [batch][3][n], rlk [level][2][n], out [batch][2][n]");
    job *j = job_new(&k, run_relin_prepared, NULL);
    j->p[0] = ct; j->p[1] = kk; j->p[2] = o; j->v[0] = bl ? bl : 4; j->v[1] = nk / (2 * n); j->batch = nc / (3 * n);
    return job_go(env, &k, j, k.argv[3], k.argv, 4);
}

/* blindRotate(acc, lweA, lweB, bsk, baseLog, level): k = 1, in place on acc
 * [batch][2][n]; lweA [batch][dim]; lweB [batch]; bsk [dim][2*level][2][n]
 * coefficient-form GGSWs, host buffers (BootstrapEngine::blind_rotate :547-577) */
static int run_blind_rotate(job *j) {
    const size_t nbsk = j->v[2];
    const uint32_t lv = (uint32_t)j->v[1], dim = (uint32_t)j->v[3];
    j->owned = (uint64_t *)malloc(nbsk ? nbsk * 8 : 8);
    int rc = nbsk ? fhe_ggsw_prepare(j->c, 1, lv * dim, j->p[3], j->owned, FHE_HOST) : 0;
    if (!rc)
        rc = fhe_blind_rotate_batch(j->c, 1, (uint32_t)j->v[0], lv, dim, j->p[1], j->p[2], j->v[4], j->owned, j->p[0],
                                    j->batch, FHE_HOST);
    return rc;
}
static napi_value ctx_blind_rotate(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 6, &k)) return NULL;
    uint64_t *acc, *la, *lb, *bsk, bl, lv;
    size_t nacc, nla, nlb, nbsk;
    if (arr_arg(env, &k, 0, &acc, &nacc) || arr_arg(env, &k, 1, &la, &nla) || arr_arg(env, &k, 2, &lb, &nlb) ||
        arr_arg(env, &k, 3, &bsk, &nbsk) || num_arg(env, &k, 4, &bl) || num_arg(env, &k, 5, &lv) || lv == 0 ||
        k.where != FHE_HOST)
        return bad_args(env, "blindRotate(acc, lweA, lweB, bsk, baseLog, level): host buffers"), NULL;
    const size_t n = k.n, ggsw = 4 * lv * n;
    if (nacc % (2 * n) || nlb != nacc / (2 * n) || (nlb && nla % nlb) || nbsk % ggsw ||
        (nlb && nbsk / ggsw != nla / nlb))
        return range_err(env, "shape mismatch (k = 1)");
    job *j = job_new(&k, run_blind_rotate, NULL);
    j->p[0] = acc; j->p[1] = la; j->p[2] = lb; j->p[3] = bsk;
    j->v[0] = bl; j->v[1] = lv; j->v[2] = nbsk; j->v[3] = nlb ? nla / nlb : 0; j->v[4] = k.q; j->batch = nlb;
    return job_go(env, &k, j, k.argv[0], k.argv, 4);
}

/* preparePublicKey(pk [2][n] = (a, b), out [2][n]) / prepareSecretKey(sk [n],
 * out [2][n]): NTT-domain key forms for encrypt / decrypt */
static int run_pk_prep(job *j) { return fhe_public_key_prepare(j->c, j->p[0], j->p[1], j->where); }
static int run_sk_prep(job *j) { return fhe_secret_key_prepare(j->c, j->p[0], j->p[1], j->where); }
static napi_value key_prep(napi_env env, napi_callback_info info, int secret) {
    call k;
    if (call_begin(env, info, 2, &k)) return NULL;
    uint64_t *a, *o;
    size_t na, no;
    if (arr_arg(env, &k, 0, &a, &na) || arr_arg(env, &k, 1, &o, &no) || no != 2 * k.n || na != (secret ? 1 : 2) * k.n)
        return bad_args(env, secret ? "prepareSecretKey(sk [n], out [2n])" : "preparePublicKey(pk [2n], out [2n])"),
               NULL;
    job *j = job_new(&k, secret ? run_sk_prep : run_pk_prep, NULL);
    j->p[0] = a; j->p[1] = o;
    return job_go(env, &k, j, k.argv[1], k.argv, 2);
}
static napi_value ctx_pk_prep(napi_env env, napi_callback_info info) { return key_prep(env, info, 0); }
static napi_value ctx_sk_prep(napi_env env, napi_callback_info info) { return key_prep(env, info, 1); }

/* encrypt(t, pkPrep, values, u, e1, e2, out): EncryptionEngine::encrypt_internal
 * (encryption.cpp:171-205) with the sampled polynomials supplied */
static int run_encrypt(job *j) {
    return fhe_encrypt_batch(j->c, j->v[0], j->p[0], j->p[1], j->p[2], j->p[3], j->p[4], j->p[5], j->batch, j->where);
}
static napi_value ctx_encrypt(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 7, &k)) return NULL;
    uint64_t t, *pk, *v, *u, *e1, *e2, *o;
    size_t npk, nv, nu, n1, n2, no;
    if (num_arg(env, &k, 0, &t) || arr_arg(env, &k, 1, &pk, &npk) || arr_arg(env, &k, 2, &v, &nv) ||
        arr_arg(env, &k, 3, &u, &nu) || arr_arg(env, &k, 4, &e1, &n1) || arr_arg(env, &k, 5, &e2, &n2) ||
        arr_arg(env, &k, 6, &o, &no) || npk != 2 * k.n || nv != nu || n1 != nu || n2 != nu || nu % k.n ||
        no != 2 * nu)
        return bad_args(env, "encrypt(t, pkPrep [2n], values, u, e1, e2 [batch*n], out [batch*2n])"), NULL;
    job *j = job_new(&k, run_encrypt, NULL);
    j->p[0] = pk; j->p[1] = v; j->p[2] = u; j->p[3] = e1; j->p[4] = e2; j->p[5] = o;
    j->v[0] = t; j->batch = nu / k.n;
    return job_go(env, &k, j, k.argv[6], k.argv + 1, 6);
}

/* encryptSampled(t, pkPrep, values, seed: BigUint64Array(4), stream, noiseStd, out):
 * u / e1 / e2 drawn on the device (fhe_encrypt_sampled_batch) */
static int run_encrypt_sampled(job *j) {
    return fhe_encrypt_sampled_batch(j->c, j->v[0], j->p[0], j->p[1], j->v + 6, j->v[1], j->d, j->p[2], j->batch,
                                     j->where);
}
static napi_value ctx_encrypt_sampled(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 7, &k)) return NULL;
    uint64_t t, *pk, *v, *o, stream, seed[4];
    size_t npk, nv, no;
    double sd;
    if (num_arg(env, &k, 0, &t) || arr_arg(env, &k, 1, &pk, &npk) || arr_arg(env, &k, 2, &v, &nv) ||
        seed_arg(env, &k, 3, seed) || num_arg(env, &k, 4, &stream) || dbl_arg(env, &k, 5, &sd) ||
        arr_arg(env, &k, 6, &o, &no) || npk != 2 * k.n || nv % k.n || no != 2 * nv)
        return bad_args(env, "encryptSampled(t, pkPrep [2n], values [batch*n], seed (BigUint64Array 4), stream, "
                             "noiseStd, out [batch*2n])"), NULL;
    job *j = job_new(&k, run_encrypt_sampled, NULL);
    j->p[0] = pk; j->p[1] = v; j->p[2] = o; j->v[0] = t; j->v[1] = stream; j->d = sd;
    memcpy(j->v + 6, seed, 32);
    j->batch = nv / k.n;
    napi_value keep[4] = {k.argv[1], k.argv[2], k.argv[6], k.argv[3]};
    return job_go(env, &k, j, k.argv[6], keep, 4);
}

/* decrypt(t, skPrep, ct, components, isNtt, values, maxNoise, phase?) ->
 * values (decode_packed slots); maxNoise [batch] per ciphertext */
static int run_decrypt(job *j) {
    return fhe_decrypt_batch(j->c, j->v[0], j->p[0], j->p[1], (uint32_t)j->v[1], (int)j->v[2], j->p[2], j->p[4],
                             j->p[3], j->batch, j->where);
}
static napi_value ctx_decrypt(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 8, &k)) return NULL;
    uint64_t t, comps, is_ntt, *sk, *ct, *v, *mx, *ph = NULL;
    size_t nsk, nct, nv, nmx, nph = 0;
    if (num_arg(env, &k, 0, &t) || arr_arg(env, &k, 1, &sk, &nsk) || arr_arg(env, &k, 2, &ct, &nct) ||
        num_arg(env, &k, 3, &comps) || num_arg(env, &k, 4, &is_ntt) || arr_arg(env, &k, 5, &v, &nv) ||
        arr_arg(env, &k, 6, &mx, &nmx) || (!undef_arg(env, &k, 7) && arr_arg(env, &k, 7, &ph, &nph)) ||
        (comps != 2 && comps != 3) || nsk != 2 * k.n || nct % (comps * k.n))
        return bad_args(env, "decrypt(t, skPrep [2n], ct [batch*comps*n], comps, isNtt, values, maxNoise, phase?)"),
               NULL;
    const size_t batch = nct / (comps * k.n);
    if (nv != batch * k.n || nmx != batch || (ph && nph != batch * k.n))
        return range_err(env, "values [batch*n], maxNoise [batch], phase [batch*n]");
    job *j = job_new(&k, run_decrypt, NULL);
    j->p[0] = sk; j->p[1] = ct; j->p[2] = v; j->p[3] = mx; j->p[4] = ph;
    j->v[0] = t; j->v[1] = comps; j->v[2] = is_ntt; j->batch = batch;
    return job_go(env, &k, j, k.argv[5], k.argv + 1, ph ? 7 : 6);
}

/* addPlain(t, ct, values, isNtt, out): EncryptionEngine::add_plain (:638-665) */
static int run_add_plain(job *j) {
    return fhe_add_plain_batch(j->c, j->v[0], j->p[0], j->p[1], (int)j->v[1], j->p[2], j->batch, j->where);
}
static napi_value ctx_add_plain(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 5, &k)) return NULL;
    uint64_t t, is_ntt, *ct, *v, *o;
    size_t nct, nv, no;
    if (num_arg(env, &k, 0, &t) || arr_arg(env, &k, 1, &ct, &nct) || arr_arg(env, &k, 2, &v, &nv) ||
        num_arg(env, &k, 3, &is_ntt) || arr_arg(env, &k, 4, &o, &no) || nct % (2 * k.n) || nv != nct / 2 ||
        no != nct)
        return bad_args(env, "addPlain(t, ct [batch*2n], values [batch*n], isNtt, out [batch*2n])"), NULL;
    job *j = job_new(&k, run_add_plain, NULL);
    j->p[0] = ct; j->p[1] = v; j->p[2] = o; j->v[0] = t; j->v[1] = is_ntt; j->batch = nct / (2 * k.n);
    return job_go(env, &k, j, k.argv[4], k.argv + 1, 4);
}

/* bootstrap(lweA, lweB, bsk, testPoly, kskA, kskB, baseLog, level, ksBaseLog,
 * ksLevel, outA, outB): BootstrapEngine::bootstrap_with_test_poly
 * (bootstrap_engine.cpp:684-708), k = 1, bsk in coefficient form
 * [dim][2*level][2][n] prepared per call (host buffers), LWE modulus = the
 * ring modulus.  bootstrapPrepared takes the prepared key (either placement). */
static int run_bootstrap(job *j) {
    const uint32_t lv = (uint32_t)j->v[1], dim = (uint32_t)j->v[4];
    const size_t nbsk = j->v[5];
    const uint64_t *bsk = j->p[2];
    int rc = 0;
    if (!j->v[8]) {
        j->owned = (uint64_t *)malloc(nbsk ? nbsk * 8 : 8);
        rc = nbsk ? fhe_ggsw_prepare(j->c, 1, lv * dim, j->p[2], j->owned, FHE_HOST) : 0;
        bsk = j->owned;
    }
    if (!rc)
        rc = fhe_bootstrap_batch(j->c, 1, (uint32_t)j->v[0], lv, dim, j->p[0], j->p[1], j->v[7], bsk, j->p[3],
                                 (uint32_t)j->v[2], (uint32_t)j->v[3], (uint32_t)j->v[6], j->p[4], j->p[5], j->p[6],
                                 j->p[7], j->batch, j->where);
    return rc;
}
static napi_value bootstrap_call(napi_env env, napi_callback_info info, int prepared) {
    call k;
    if (call_begin(env, info, 12, &k)) return NULL;
    uint64_t *la, *lb, *bsk, *tp, *ka, *kb, *oa, *ob, bl, lv, kbl, klv;
    size_t nla, nlb, nbsk, ntp, nka, nkb, noa, nob;
    if (arr_arg(env, &k, 0, &la, &nla) || arr_arg(env, &k, 1, &lb, &nlb) || arr_arg(env, &k, 2, &bsk, &nbsk) ||
        arr_arg(env, &k, 3, &tp, &ntp) || arr_arg(env, &k, 4, &ka, &nka) || arr_arg(env, &k, 5, &kb, &nkb) ||
        num_arg(env, &k, 6, &bl) || num_arg(env, &k, 7, &lv) || num_arg(env, &k, 8, &kbl) ||
        num_arg(env, &k, 9, &klv) || arr_arg(env, &k, 10, &oa, &noa) || arr_arg(env, &k, 11, &ob, &nob) || lv == 0 ||
        (!prepared && k.where != FHE_HOST))
        return bad_args(env, prepared ? "bootstrapPrepared(lweA, lweB, bskPrep, testPoly, kskA, kskB, baseLog, level, "
                                        "ksBaseLog, ksLevel, outA, outB)"
                                      : "bootstrap(lweA, lweB, bsk, testPoly, kskA, kskB, baseLog, level, ksBaseLog, "
                                        "ksLevel, outA, outB): host buffers"), NULL;
    const size_t n = k.n, ggsw = 4 * lv * n, batch = nlb;
    const size_t dim = batch ? nla / batch : 0, entries = n * klv, out_dim = entries ? nka / entries : 0;
    if ((batch && nla % batch) || nbsk != dim * ggsw || ntp != n || nkb != entries || nka != entries * out_dim ||
        nob != batch || noa != batch * out_dim)
        return range_err(env, "shape mismatch (k = 1)");
    job *j = job_new(&k, run_bootstrap, NULL);
    j->p[0] = la; j->p[1] = lb; j->p[2] = bsk; j->p[3] = tp; j->p[4] = ka; j->p[5] = kb; j->p[6] = oa; j->p[7] = ob;
    j->v[0] = bl; j->v[1] = lv; j->v[2] = kbl; j->v[3] = klv; j->v[4] = dim; j->v[5] = nbsk; j->v[6] = out_dim;
    j->v[7] = k.q; j->v[8] = (uint64_t)prepared; j->batch = batch;
    napi_value keep[8] = {k.argv[0], k.argv[1], k.argv[2], k.argv[3], k.argv[4], k.argv[5], k.argv[10], k.argv[11]};
    return job_go(env, &k, j, k.argv[10], keep, 8);
}
static napi_value ctx_bootstrap(napi_env env, napi_callback_info info) { return bootstrap_call(env, info, 0); }
static napi_value ctx_bootstrap_prepared(napi_env env, napi_callback_info info) { return bootstrap_call(env, info, 1); }

/* sampleExtract(k, glwe [batch][k+1][n], lweA [batch][k n], lweB [batch]) (:594-624) */
static int run_sample_extract(job *j) {
    return fhe_sample_extract_batch(j->c, (uint32_t)j->v[0], j->p[0], j->p[1], j->p[2], j->batch, j->where);
}
static napi_value ctx_sample_extract(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 4, &k)) return NULL;
    uint64_t kd, *g, *a, *b;
    size_t ng, na, nb;
    if (num_arg(env, &k, 0, &kd) || arr_arg(env, &k, 1, &g, &ng) || arr_arg(env, &k, 2, &a, &na) ||
        arr_arg(env, &k, 3, &b, &nb) || ng % ((kd + 1) * k.n) || nb != ng / ((kd + 1) * k.n) || na != nb * kd * k.n)
        return bad_args(env, "sampleExtract(k, glwe [batch][k+1][n], lweA [batch][k n], lweB [batch])"), NULL;
    job *j = job_new(&k, run_sample_extract, NULL);
    j->p[0] = g; j->p[1] = a; j->p[2] = b; j->v[0] = kd; j->batch = nb;
    return job_go(env, &k, j, k.argv[2], k.argv + 1, 3);
}

/* keySwitch(baseLog, level, kskA [inDim L][outDim], kskB [inDim L], lweA [batch][inDim],
 * lweB [batch], outA [batch][outDim], outB [batch]) modulo the ring modulus (:626-674) */
static int run_key_switch(job *j) {
    fhe_ctx_info ci;
    fhe_ctx_get_info(j->c, &ci);
    return fhe_key_switch_batch(ci.q, (uint32_t)j->v[0], (uint32_t)j->v[1], (uint32_t)j->v[2], (uint32_t)j->v[3],
                                j->p[0], j->p[1], j->p[2], j->p[3], j->p[4], j->p[5], j->batch, j->where, ci.device,
                                fhe_ctx_stream(j->c));
}
static napi_value ctx_key_switch(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 8, &k)) return NULL;
    uint64_t bl, lv, *ka, *kb, *la, *lb, *oa, *ob;
    size_t nka, nkb, nla, nlb, noa, nob;
    if (num_arg(env, &k, 0, &bl) || num_arg(env, &k, 1, &lv) || arr_arg(env, &k, 2, &ka, &nka) ||
        arr_arg(env, &k, 3, &kb, &nkb) || arr_arg(env, &k, 4, &la, &nla) || arr_arg(env, &k, 5, &lb, &nlb) ||
        arr_arg(env, &k, 6, &oa, &noa) || arr_arg(env, &k, 7, &ob, &nob) || lv == 0 || nlb == 0 || nla % nlb ||
        nob != nlb || noa % nlb || nkb != (nla / nlb) * lv || nka != nkb * (noa / nlb))
        return bad_args(env, "keySwitch(baseLog, level, kskA, kskB, lweA, lweB, outA, outB)"), NULL;
    job *j = job_new(&k, run_key_switch, NULL);
    j->p[0] = ka; j->p[1] = kb; j->p[2] = la; j->p[3] = lb; j->p[4] = oa; j->p[5] = ob;
    j->v[0] = bl; j->v[1] = lv; j->v[2] = nla / nlb; j->v[3] = noa / nlb; j->batch = nlb;
    return job_go(env, &k, j, k.argv[6], k.argv + 2, 6);
}

/* ---- randomness and key material (fhe_sample_batch, fhe_*_generate) ---- */
/* sample(kind, seed, stream, noiseStd, out) */
static int run_sample(job *j) {
    return fhe_sample_batch(j->c, (int)j->v[0], j->v + 6, j->v[1], j->d, j->p[0], j->batch, j->where);
}
static napi_value ctx_sample(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 5, &k)) return NULL;
    uint64_t kind, seed[4], stream, *o;
    size_t no;
    double sd;
    if (num_arg(env, &k, 0, &kind) || seed_arg(env, &k, 1, seed) || num_arg(env, &k, 2, &stream) ||
        dbl_arg(env, &k, 3, &sd) || arr_arg(env, &k, 4, &o, &no))
        return bad_args(env, "sample(kind, seed (BigUint64Array 4), stream, noiseStd, out)"), NULL;
    job *j = job_new(&k, run_sample, NULL);
    j->p[0] = o; j->v[0] = kind; j->v[1] = stream; j->d = sd; memcpy(j->v + 6, seed, 32); j->batch = no;
    return job_go(env, &k, j, k.argv[4], k.argv + 4, 1);
}
/* publicKeyGenerate(sk [n], seed, stream, noiseStd, out [2n]) */
static int run_pk_gen(job *j) { return fhe_public_key_generate(j->c, j->p[0], j->v + 6, j->v[1], j->d, j->p[1], j->where); }
static napi_value ctx_pk_gen(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 5, &k)) return NULL;
    uint64_t seed[4], stream, *sk, *o;
    size_t ns, no;
    double sd;
    if (arr_arg(env, &k, 0, &sk, &ns) || seed_arg(env, &k, 1, seed) || num_arg(env, &k, 2, &stream) ||
        dbl_arg(env, &k, 3, &sd) || arr_arg(env, &k, 4, &o, &no) || ns != k.n || no != 2 * k.n)
        return bad_args(env, "publicKeyGenerate(sk [n], seed, stream, noiseStd, out [2n])"), NULL;
    job *j = job_new(&k, run_pk_gen, NULL);
    j->p[0] = sk; j->p[1] = o; j->v[1] = stream; j->d = sd; memcpy(j->v + 6, seed, 32);
    napi_value keep[2] = {k.argv[0], k.argv[4]};
    return job_go(env, &k, j, k.argv[4], keep, 2);
}
/* evalKeyGenerate(sk [n], baseLog, level, seed, stream, noiseStd, out [level][2][n]) */
static int run_ek_gen(job *j) {
    return fhe_eval_key_generate(j->c, j->p[0], (uint32_t)j->v[2], (uint32_t)j->v[3], j->v + 6, j->v[1], j->d,
                                 j->p[1], j->where);
}
static napi_value ctx_ek_gen(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 7, &k)) return NULL;
    uint64_t seed[4], stream, bl, lv, *sk, *o;
    size_t ns, no;
    double sd;
    if (arr_arg(env, &k, 0, &sk, &ns) || num_arg(env, &k, 1, &bl) || num_arg(env, &k, 2, &lv) ||
        seed_arg(env, &k, 3, seed) || num_arg(env, &k, 4, &stream) || dbl_arg(env, &k, 5, &sd) ||
        arr_arg(env, &k, 6, &o, &no) || ns != k.n || no != lv * 2 * k.n)
        return bad_args(env, "evalKeyGenerate(sk [n], baseLog, level, seed, stream, noiseStd, out [level][2][n])"),
               NULL;
    job *j = job_new(&k, run_ek_gen, NULL);
    j->p[0] = sk; j->p[1] = o; j->v[1] = stream; j->v[2] = bl; j->v[3] = lv; j->d = sd; memcpy(j->v + 6, seed, 32);
    napi_value keep[2] = {k.argv[0], k.argv[6]};
    return job_go(env, &k, j, k.argv[6], keep, 2);
}
/* ggswEncrypt(values: BigInt64Array [count], sk [n], k, baseLog, level, seed, stream, noiseStd,
 * out [count][(k+1)L][k+1][n]) */
static int run_ggsw_enc(job *j) {
    return fhe_ggsw_encrypt_batch(j->c, (uint32_t)j->v[2], (uint32_t)j->v[3], (uint32_t)j->v[4], (const int64_t *)j->p[0],
                                  j->batch, j->p[1], j->v + 6, j->v[1], j->d, j->p[2], j->where);
}
static napi_value ctx_ggsw_enc(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 9, &k)) return NULL;
    uint64_t seed[4], stream, kd, bl, lv, *vals, *sk, *o;
    size_t nv, ns, no;
    double sd;
    if (arr_arg(env, &k, 0, &vals, &nv) || arr_arg(env, &k, 1, &sk, &ns) || num_arg(env, &k, 2, &kd) ||
        num_arg(env, &k, 3, &bl) || num_arg(env, &k, 4, &lv) || seed_arg(env, &k, 5, seed) ||
        num_arg(env, &k, 6, &stream) || dbl_arg(env, &k, 7, &sd) || arr_arg(env, &k, 8, &o, &no) || ns != k.n ||
        no != nv * (kd + 1) * lv * (kd + 1) * k.n)
        return bad_args(env, "ggswEncrypt(values (BigInt64Array), sk [n], k, baseLog, level, seed, stream, noiseStd, "
                             "out [count][(k+1)L][k+1][n])"), NULL;
    job *j = job_new(&k, run_ggsw_enc, NULL);
    j->p[0] = vals; j->p[1] = sk; j->p[2] = o; j->v[1] = stream; j->v[2] = kd; j->v[3] = bl; j->v[4] = lv; j->d = sd;
    memcpy(j->v + 6, seed, 32);
    j->batch = nv;
    napi_value keep[3] = {k.argv[0], k.argv[1], k.argv[8]};
    return job_go(env, &k, j, k.argv[8], keep, 3);
}
/* kskGenerate(glweSk [nIn], lweSk: BigInt64Array [dim], baseLog, level, seed, stream, noiseStd,
 * outA [nIn L][dim], outB [nIn L]) */
static int run_ksk_gen(job *j) {
    return fhe_ksk_generate(j->c, (uint32_t)j->v[2], (uint32_t)j->v[3], j->p[0], (uint32_t)j->v[4],
                            (const int64_t *)j->p[1], (uint32_t)j->v[5], j->v + 6, j->v[1], j->d, j->p[2], j->p[3],
                            j->where);
}
static napi_value ctx_ksk_gen(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 9, &k)) return NULL;
    uint64_t seed[4], stream, bl, lv, *g, *ls, *oa, *ob;
    size_t ng, nl, noa, nob;
    double sd;
    if (arr_arg(env, &k, 0, &g, &ng) || arr_arg(env, &k, 1, &ls, &nl) || num_arg(env, &k, 2, &bl) ||
        num_arg(env, &k, 3, &lv) || seed_arg(env, &k, 4, seed) || num_arg(env, &k, 5, &stream) ||
        dbl_arg(env, &k, 6, &sd) || arr_arg(env, &k, 7, &oa, &noa) || arr_arg(env, &k, 8, &ob, &nob) ||
        nob != ng * lv || noa != nob * nl)
        return bad_args(env, "kskGenerate(glweSk, lweSk (BigInt64Array), baseLog, level, seed, stream, noiseStd, "
                             "outA [nIn L][dim], outB [nIn L])"), NULL;
    job *j = job_new(&k, run_ksk_gen, NULL);
    j->p[0] = g; j->p[1] = ls; j->p[2] = oa; j->p[3] = ob;
    j->v[1] = stream; j->v[2] = bl; j->v[3] = lv; j->v[4] = ng; j->v[5] = nl; j->d = sd; memcpy(j->v + 6, seed, 32);
    napi_value keep[4] = {k.argv[0], k.argv[1], k.argv[7], k.argv[8]};
    return job_go(env, &k, j, k.argv[8], keep, 4);
}
/* lweDecrypt(t, sk: BigInt64Array [dim], lweA [batch][dim], lweB [batch], values [batch], phase?) */
static int run_lwe_dec(job *j) {
    fhe_ctx_info ci;
    fhe_ctx_get_info(j->c, &ci);
    return fhe_lwe_decrypt_batch(ci.q, j->v[0], (const int64_t *)j->p[0], (uint32_t)j->v[1], j->p[1], j->p[2], j->p[3],
                                 j->p[4], j->batch, j->where, ci.device, fhe_ctx_stream(j->c));
}
static napi_value ctx_lwe_dec(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 6, &k)) return NULL;
    uint64_t t, *s, *a, *b, *v, *ph = NULL;
    size_t ns, na, nb, nv, nph = 0;
    if (num_arg(env, &k, 0, &t) || arr_arg(env, &k, 1, &s, &ns) || arr_arg(env, &k, 2, &a, &na) ||
        arr_arg(env, &k, 3, &b, &nb) || arr_arg(env, &k, 4, &v, &nv) ||
        (!undef_arg(env, &k, 5) && arr_arg(env, &k, 5, &ph, &nph)) || nb == 0 || na != nb * ns || nv != nb ||
        (ph && nph != nb))
        return bad_args(env, "lweDecrypt(t, sk (BigInt64Array), lweA [batch][dim], lweB [batch], values, phase?)"), NULL;
    job *j = job_new(&k, run_lwe_dec, NULL);
    j->p[0] = s; j->p[1] = a; j->p[2] = b; j->p[3] = v; j->p[4] = ph; j->v[0] = t; j->v[1] = ns; j->batch = nb;
    return job_go(env, &k, j, k.argv[4], k.argv + 1, ph ? 5 : 4);
}

static napi_value ctx_synchronize(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 0, &k)) return NULL;
    pthread_mutex_lock(&k.k->mu);
    int rc = fhe_ctx_synchronize(k.c);
    pthread_mutex_unlock(&k.k->mu);
    if (rc) return throw_fhe(env, rc);
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

/* ciphertexts of two-CU blind rotations recomputed by the repair pass (a
   partner workgroup was not co-resident); synchronises the context */
static napi_value ctx_br_repairs(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 0, &k)) return NULL;
    uint64_t n = 0;
    pthread_mutex_lock(&k.k->mu);
    int rc = fhe_br_repair_count(k.c, &n);
    pthread_mutex_unlock(&k.k->mu);
    if (rc) return throw_fhe(env, rc);
    return make_i64(env, (int64_t)n);
}

static napi_value ctx_info(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 0, &k)) return NULL;
    fhe_ctx_info ci;
    int rc = fhe_ctx_get_info(k.c, &ci);
    if (rc) return throw_fhe(env, rc);
    int nd = 1;
    fhe_ctx_device_count(k.c, &nd);
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
    set(env, o, "devices", make_i64(env, nd));
    return o;
}

/* ------------------------------------------------------------------ module */
static int g_async_tag;
#define M(NAME, FN)                                                                \
    {NAME, NULL, FN, NULL, NULL, NULL, napi_default, NULL},                        \
    {NAME "Async", NULL, FN, NULL, NULL, NULL, napi_default, &g_async_tag}

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
        M("forward", ctx_forward),
        M("inverse", ctx_inverse),
        M("polymul", ctx_polymul),
        M("pointwise", ctx_pointwise),
        M("add", ctx_add),
        M("sub", ctx_sub),
        M("negate", ctx_negate),
        M("mulScalar", ctx_mul_scalar),
        M("forwardMul", ctx_fwd_mul),
        M("externalProduct", ctx_ext_product),
        M("prepareGgsw", ctx_prep_ggsw),
        M("externalProductPrepared", ctx_ext_prepared),
        M("ctMultiply", ctx_ct_multiply),
        M("relinearize", ctx_relinearize),
        M("prepareRelinKey", ctx_prep_rlk),
        M("relinearizePrepared", ctx_relin_prepared),
        M("blindRotate", ctx_blind_rotate),
        M("preparePublicKey", ctx_pk_prep),
        M("prepareSecretKey", ctx_sk_prep),
        M("encrypt", ctx_encrypt),
        M("encryptSampled", ctx_encrypt_sampled),
        M("decrypt", ctx_decrypt),
        M("addPlain", ctx_add_plain),
        M("bootstrap", ctx_bootstrap),
        M("bootstrapPrepared", ctx_bootstrap_prepared),
        M("sampleExtract", ctx_sample_extract),
        M("keySwitch", ctx_key_switch),
        M("sample", ctx_sample),
        M("publicKeyGenerate", ctx_pk_gen),
        M("evalKeyGenerate", ctx_ek_gen),
        M("ggswEncrypt", ctx_ggsw_enc),
        M("kskGenerate", ctx_ksk_gen),
        M("lweDecrypt", ctx_lwe_dec),
        {"synchronize", NULL, ctx_synchronize, NULL, NULL, NULL, napi_default, NULL},
        {"info", NULL, ctx_info, NULL, NULL, NULL, napi_default, NULL},
        {"brRepairCount", NULL, ctx_br_repairs, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_value ctx_cls;
    NAPI_CALL(env, napi_define_class(env, "NttContext", NAPI_AUTO_LENGTH, ctx_ctor, NULL,
                                     sizeof ctx_props / sizeof ctx_props[0], ctx_props, &ctx_cls));
    NAPI_CALL(env, napi_create_reference(env, ctx_cls, 1, &g_ctx_ctor));
    set(env, exports, "NttContext", ctx_cls);

    napi_property_descriptor buf_props[] = {
        {"words", NULL, NULL, buf_words, NULL, NULL, napi_default, NULL},
        {"handle", NULL, NULL, buf_handle, NULL, NULL, napi_default, NULL},
        {"upload", NULL, buf_upload, NULL, NULL, NULL, napi_default, NULL},
        {"download", NULL, buf_download, NULL, NULL, NULL, napi_default, NULL},
        {"copyFrom", NULL, buf_copy_from, NULL, NULL, NULL, napi_default, NULL},
        {"view", NULL, buf_view, NULL, NULL, NULL, napi_default, NULL},
        {"free", NULL, buf_free, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_value buf_cls;
    NAPI_CALL(env, napi_define_class(env, "DeviceBuffer", NAPI_AUTO_LENGTH, buf_ctor, NULL,
                                     sizeof buf_props / sizeof buf_props[0], buf_props, &buf_cls));
    NAPI_CALL(env, napi_create_reference(env, buf_cls, 1, &g_buf_ctor));
    set(env, exports, "DeviceBuffer", buf_cls);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
