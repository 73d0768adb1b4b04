/*
 * fhe_napi.c -- plain node_api.h addon over libfhe_gpu.so.
 *
 * Replaces the napi-rs binding (src/native/lib.rs:22-133, bridge.rs:3-41)
 * with the same JS surface as index.d.ts:
 *   initialize(), detectHardware(), version(), class ModularArithmetic
 * plus the batched polynomial engine the TS FHEEngine needs (NttContext,
 * modmulBatch, mlMontgomeryMulBatch) over zero-copy BigUint64Array buffers
 * (napi_get_typedarray_info; FHE_HOST placement, the library stages the data
 * through HBM).  Every NttContext compute method has a synchronous form and
 * an `...Async` form that runs as napi_async_work on the libuv pool and
 * returns a Promise, so the JS event loop is never blocked by a transfer or
 * a kernel.  Errors become JS exceptions / rejections with the library's
 * message -- the reference's cxx bridge aborted the process on a C++
 * exception instead.
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
    NAPI_CALL(env, napi_wrap(env, self, c, ctx_finalize, NULL, NULL));
    return self;
}

/* ---- jobs: every compute method runs either synchronously on the JS
 * thread (`name`) or as napi_async_work on the libuv pool (`nameAsync`,
 * returns a Promise of the output array).  A job holds references to its
 * typed arrays and to the context object until it completes. */
#define MAXP 12
typedef struct job job;
typedef int (*job_fn)(job *);
struct job {
    job_fn fn;
    void *op;           /* the library entry point for the generic runners */
    fhe_ctx *c;
    uint64_t *p[MAXP];
    uint64_t v[8];
    size_t batch;
    uint64_t *owned;    /* scratch (prepared keys), freed on completion */
    int rc;
    char err[512];
    napi_ref refs[MAXP + 2];
    int nref;
    napi_value ret_now; /* sync path */
    napi_ref ret;       /* async path */
    napi_deferred def;
    napi_async_work work;
};

typedef struct {
    fhe_ctx *c;
    napi_value self;
    napi_value argv[12];
    size_t argc;
    int async;
    size_t n;
    uint64_t q;
} call;

static int call_begin(napi_env env, napi_callback_info info, size_t want, call *k) {
    k->argc = want;
    void *data = NULL;
    if (napi_get_cb_info(env, info, &k->argc, k->argv, &k->self, &data) != napi_ok) return -1;
    k->async = data != NULL;
    void *p = NULL;
    napi_unwrap(env, k->self, &p);
    k->c = (fhe_ctx *)p;
    if (!k->c) {
        napi_throw_type_error(env, "INVALID_PARAMETERS", "not an NttContext");
        return -1;
    }
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
    j->c = k->c;
    return j;
}

static void job_free(napi_env env, job *j) {
    for (int i = 0; i < j->nref; ++i) napi_delete_reference(env, j->refs[i]);
    if (j->ret) napi_delete_reference(env, j->ret);
    free(j->owned);
    free(j);
}

static void job_exec(napi_env env, void *data) {
    (void)env;
    job *j = (job *)data;
    j->rc = j->fn(j);
    if (j->rc) snprintf(j->err, sizeof j->err, "%s", fhe_last_error()); /* thread-local: read on this thread */
}

static void job_done(napi_env env, napi_status status, void *data) {
    job *j = (job *)data;
    napi_value v;
    if (status != napi_ok || j->rc) {
        napi_value msg, code, e;
        char cs[32];
        snprintf(cs, sizeof cs, "FHE_%d", j->rc ? j->rc : -11);
        napi_create_string_utf8(env, status != napi_ok ? "async work cancelled" : j->err, NAPI_AUTO_LENGTH, &msg);
        napi_create_string_utf8(env, cs, NAPI_AUTO_LENGTH, &code);
        napi_create_error(env, code, msg, &e);
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
        int rc = j->fn(j);
        free(j->owned);
        free(j);
        if (rc) return throw_fhe(env, rc);
        return ret;
    }
    for (int i = 0; i < nkeep && j->nref < MAXP + 1; ++i) napi_create_reference(env, keep[i], 1, &j->refs[j->nref++]);
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
static int arr_arg(napi_env env, const call *k, size_t i, uint64_t **p, size_t *cnt) {
    if (i >= k->argc || get_u64_array(env, k->argv[i], p, cnt)) return -1;
    return 0;
}
static int num_arg(napi_env env, const call *k, size_t i, uint64_t *v) {
    int neg;
    if (i >= k->argc || get_u64(env, k->argv[i], v, &neg) || neg) return -1;
    return 0;
}
static int undef_arg(napi_env env, const call *k, size_t i) {
    if (i >= k->argc) return 1;
    napi_valuetype t;
    napi_typeof(env, k->argv[i], &t);
    return t == napi_undefined || t == napi_null;
}

typedef int (*unary_fn)(fhe_ctx *, const uint64_t *, uint64_t *, size_t, int);
typedef int (*binary_fn)(fhe_ctx *, const uint64_t *, const uint64_t *, uint64_t *, size_t, int);
static int run_unary(job *j) { return ((unary_fn)j->op)(j->c, j->p[0], j->p[1], j->batch, FHE_HOST); }
static int run_binary(job *j) { return ((binary_fn)j->op)(j->c, j->p[0], j->p[1], j->p[2], j->batch, FHE_HOST); }

/* op(a, out?) ; out defaults to a (in place, like NTTProcessor::forward_ntt) */
static napi_value ctx_unary(napi_env env, napi_callback_info info, unary_fn fn) {
    call k;
    if (call_begin(env, info, 2, &k)) return NULL;
    uint64_t *a, *o;
    size_t na, no;
    if (arr_arg(env, &k, 0, &a, &na)) return bad_args(env, "expected BigUint64Array"), NULL;
    napi_value ret = k.argv[0];
    o = a;
    no = na;
    if (!undef_arg(env, &k, 1)) {
        if (arr_arg(env, &k, 1, &o, &no) || no != na)
            return bad_args(env, "out must be a BigUint64Array of equal length"), NULL;
        ret = k.argv[1];
    }
    if (na % k.n) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "Coefficient count must equal polynomial degree");
        return NULL;
    }
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
        return bad_args(env, "expected (a, b, out) BigUint64Arrays of equal length"), NULL;
    if (na % k.n) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "Coefficient count must equal polynomial degree");
        return NULL;
    }
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

static int run_mul_scalar(job *j) { return fhe_poly_mul_scalar_batch(j->c, j->p[0], j->v[0], j->p[1], j->batch, FHE_HOST); }
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

/* externalProduct(glwe, ggswCoeff, baseLog, level, out): k = 1 */
static int run_ext_product(job *j) {
    const size_t nk = j->v[2];
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
        num_arg(env, &k, 3, &lv) || arr_arg(env, &k, 4, &o, &no) || ng != no)
        return bad_args(env, "externalProduct(glwe, ggsw, baseLog, level, out)"), NULL;
    const size_t per = 2 * k.n;
    if (ng % per || nk != (size_t)4 * lv * k.n) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "shape mismatch (k = 1)");
        return NULL;
    }
    job *j = job_new(&k, run_ext_product, NULL);
    j->p[0] = g; j->p[1] = kk; j->p[2] = o; j->v[0] = bl; j->v[1] = lv; j->v[2] = nk; j->batch = ng / per;
    return job_go(env, &k, j, k.argv[4], k.argv, 5);
}

/* ctMultiply(ct1, ct2, out, isNtt?): ct [batch][2][n] -> out [batch][3][n]
 * (EncryptionEngine::multiply, encryption.cpp:737-798) */
static int run_ct_multiply(job *j) {
    return fhe_ct_multiply_batch(j->c, j->p[0], j->p[1], j->p[2], j->batch, (int)j->v[0], FHE_HOST);
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
    if (nx % per || no != nx / 2 * 3) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "ciphertexts must be [batch][2][n], out [batch][3][n]");
        return NULL;
    }
    job *j = job_new(&k, run_ct_multiply, NULL);
    j->p[0] = x; j->p[1] = y; j->p[2] = o; j->v[0] = is_ntt; j->batch = nx / per;
    return job_go(env, &k, j, k.argv[2], k.argv, 3);
}

/* relinearize(ct3, rlk, baseLog, out): rlk [level][2][n] (a_l, b_l) in
 * coefficient form (KeySwitchKey), out [batch][2][n]
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
        arr_arg(env, &k, 3, &o, &no))
        return bad_args(env, "relinearize(ct3, rlk, baseLog, out)"), NULL;
    const size_t n = k.n;
    if (nc % (3 * n) || nk % (2 * n) || no != nc / 3 * 2) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "ct3 [batch][3][n], rlk [level][2][n], out [batch][2][n]");
        return NULL;
    }
    job *j = job_new(&k, run_relinearize, NULL);
    j->p[0] = ct; j->p[1] = kk; j->p[2] = o;
    j->v[0] = bl ? bl : 4; j->v[1] = nk / (2 * n); j->v[2] = nk; j->batch = nc / (3 * n);
    return job_go(env, &k, j, k.argv[3], k.argv, 4);
}

/* blindRotate(acc, lweA, lweB, bsk, baseLog, level): k = 1, in place on acc
 * [batch][2][n]; lweA [batch][dim]; lweB [batch]; bsk [dim][2*level][2][n]
 * coefficient-form GGSWs (BootstrapEngine::blind_rotate :547-577) */
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
        arr_arg(env, &k, 3, &bsk, &nbsk) || num_arg(env, &k, 4, &bl) || num_arg(env, &k, 5, &lv) || lv == 0)
        return bad_args(env, "blindRotate(acc, lweA, lweB, bsk, baseLog, level)"), NULL;
    const size_t n = k.n, ggsw = 4 * lv * n;
    if (nacc % (2 * n) || nlb != nacc / (2 * n) || (nlb && nla % nlb) || nbsk % ggsw ||
        (nlb && nbsk / ggsw != nla / nlb)) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "shape mismatch (k = 1)");
        return NULL;
    }
    job *j = job_new(&k, run_blind_rotate, NULL);
    j->p[0] = acc; j->p[1] = la; j->p[2] = lb; j->p[3] = bsk;
    j->v[0] = bl; j->v[1] = lv; j->v[2] = nbsk; j->v[3] = nlb ? nla / nlb : 0; j->v[4] = k.q; j->batch = nlb;
    return job_go(env, &k, j, k.argv[0], k.argv, 4);
}

/* preparePublicKey(pk [2][n] = (a, b), out [2][n]) / prepareSecretKey(sk [n],
 * out [2][n]): NTT-domain key forms for encrypt / decrypt */
static int run_pk_prep(job *j) { return fhe_public_key_prepare(j->c, j->p[0], j->p[1], FHE_HOST); }
static int run_sk_prep(job *j) { return fhe_secret_key_prepare(j->c, j->p[0], j->p[1], FHE_HOST); }
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
    return fhe_encrypt_batch(j->c, j->v[0], j->p[0], j->p[1], j->p[2], j->p[3], j->p[4], j->p[5], j->batch, FHE_HOST);
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

/* decrypt(t, skPrep, ct, components, isNtt, values, maxNoise, phase?) ->
 * values (decode_packed slots); maxNoise [batch] per ciphertext */
static int run_decrypt(job *j) {
    return fhe_decrypt_batch(j->c, j->v[0], j->p[0], j->p[1], (uint32_t)j->v[1], (int)j->v[2], j->p[2], j->p[4],
                             j->p[3], j->batch, FHE_HOST);
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
    if (nv != batch * k.n || nmx != batch || (ph && nph != batch * k.n)) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "values [batch*n], maxNoise [batch], phase [batch*n]");
        return NULL;
    }
    job *j = job_new(&k, run_decrypt, NULL);
    j->p[0] = sk; j->p[1] = ct; j->p[2] = v; j->p[3] = mx; j->p[4] = ph;
    j->v[0] = t; j->v[1] = comps; j->v[2] = is_ntt; j->batch = batch;
    return job_go(env, &k, j, k.argv[5], k.argv + 1, ph ? 7 : 6);
}

/* addPlain(t, ct, values, isNtt, out): EncryptionEngine::add_plain (:638-665) */
static int run_add_plain(job *j) {
    return fhe_add_plain_batch(j->c, j->v[0], j->p[0], j->p[1], (int)j->v[1], j->p[2], j->batch, FHE_HOST);
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
 * [dim][2*level][2][n], LWE modulus = the ring modulus */
static int run_bootstrap(job *j) {
    const uint32_t lv = (uint32_t)j->v[1], dim = (uint32_t)j->v[4];
    const size_t nbsk = j->v[5];
    j->owned = (uint64_t *)malloc(nbsk ? nbsk * 8 : 8);
    int rc = nbsk ? fhe_ggsw_prepare(j->c, 1, lv * dim, j->p[2], j->owned, FHE_HOST) : 0;
    if (!rc)
        rc = fhe_bootstrap_batch(j->c, 1, (uint32_t)j->v[0], lv, dim, j->p[0], j->p[1], j->v[7], j->owned, j->p[3],
                                 (uint32_t)j->v[2], (uint32_t)j->v[3], (uint32_t)j->v[6], j->p[4], j->p[5], j->p[6],
                                 j->p[7], j->batch, FHE_HOST);
    return rc;
}
static napi_value ctx_bootstrap(napi_env env, napi_callback_info info) {
    call k;
    if (call_begin(env, info, 12, &k)) return NULL;
    uint64_t *la, *lb, *bsk, *tp, *ka, *kb, *oa, *ob, bl, lv, kbl, klv;
    size_t nla, nlb, nbsk, ntp, nka, nkb, noa, nob;
    if (arr_arg(env, &k, 0, &la, &nla) || arr_arg(env, &k, 1, &lb, &nlb) || arr_arg(env, &k, 2, &bsk, &nbsk) ||
        arr_arg(env, &k, 3, &tp, &ntp) || arr_arg(env, &k, 4, &ka, &nka) || arr_arg(env, &k, 5, &kb, &nkb) ||
        num_arg(env, &k, 6, &bl) || num_arg(env, &k, 7, &lv) || num_arg(env, &k, 8, &kbl) ||
        num_arg(env, &k, 9, &klv) || arr_arg(env, &k, 10, &oa, &noa) || arr_arg(env, &k, 11, &ob, &nob) || lv == 0)
        return bad_args(env, "bootstrap(lweA, lweB, bsk, testPoly, kskA, kskB, baseLog, level, ksBaseLog, ksLevel, "
                             "outA, outB)"), NULL;
    const size_t n = k.n, ggsw = 4 * lv * n, batch = nlb;
    const size_t dim = batch ? nla / batch : 0, entries = n * klv, out_dim = entries ? nka / entries : 0;
    if ((batch && nla % batch) || nbsk != dim * ggsw || ntp != n || nkb != entries || nka != entries * out_dim ||
        nob != batch || noa != batch * out_dim) {
        napi_throw_range_error(env, "INVALID_PARAMETERS", "shape mismatch (k = 1)");
        return NULL;
    }
    job *j = job_new(&k, run_bootstrap, NULL);
    j->p[0] = la; j->p[1] = lb; j->p[2] = bsk; j->p[3] = tp; j->p[4] = ka; j->p[5] = kb; j->p[6] = oa; j->p[7] = ob;
    j->v[0] = bl; j->v[1] = lv; j->v[2] = kbl; j->v[3] = klv; j->v[4] = dim; j->v[5] = nbsk; j->v[6] = out_dim;
    j->v[7] = k.q; j->batch = batch;
    napi_value keep[8] = {k.argv[0], k.argv[1], k.argv[2], k.argv[3], k.argv[4], k.argv[5], k.argv[10], k.argv[11]};
    return job_go(env, &k, j, k.argv[10], keep, 8);
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
        M("ctMultiply", ctx_ct_multiply),
        M("relinearize", ctx_relinearize),
        M("blindRotate", ctx_blind_rotate),
        M("preparePublicKey", ctx_pk_prep),
        M("prepareSecretKey", ctx_sk_prep),
        M("encrypt", ctx_encrypt),
        M("decrypt", ctx_decrypt),
        M("addPlain", ctx_add_plain),
        M("bootstrap", ctx_bootstrap),
        {"info", NULL, ctx_info, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_value ctx_cls;
    NAPI_CALL(env, napi_define_class(env, "NttContext", NAPI_AUTO_LENGTH, ctx_ctor, NULL,
                                     sizeof ctx_props / sizeof ctx_props[0], ctx_props, &ctx_cls));
    set(env, exports, "NttContext", ctx_cls);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
