// fhe_gpu.cpp -- host side of libfhe_gpu.so: the C ABI of include/fhe_gpu.h.
//
// Owns per-context twiddle tables in HBM, parameter validation with the
// reference's messages, host<->device staging for FHE_HOST calls, and the
// scalar N-API ModularArithmetic helpers.  All arithmetic on coefficient
// vectors runs in the HIP kernels (ntt_*.hip, elementwise.hip); there is no
// CPU fallback: without a usable device every compute entry point fails
// with FHE_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/fhe_gpu.h"
#include "fhe_internal.hpp"
#include "keygen.hpp"

using u64 = uint64_t;
using u32 = uint32_t;
using u128 = unsigned __int128;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char *what) {
    return fail(FHE_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr, what)                      \
    do {                                         \
        hipError_t _e = (expr);                  \
        if (_e != hipSuccess) return hip_fail(_e, what); \
    } while (0)

// ---------------------------------------------------------------- number theory (host)
u64 mulmod(u64 a, u64 b, u64 q) { return (u64)((u128)a * b % q); }
u64 powmod(u64 b, u64 e, u64 q) {
    u64 r = 1 % q;
    b %= q;
    while (e) {
        if (e & 1) r = mulmod(r, b, q);
        b = mulmod(b, b, q);
        e >>= 1;
    }
    return r;
}
// a^-1 mod q by extended Euclid on 128-bit signed values (exact for any q).
bool invmod(u64 a, u64 q, u64 &out) {
    __int128 t = 0, nt = 1, r = q, nr = a % q;
    while (nr != 0) {
        __int128 quo = r / nr, tmp;
        tmp = t - quo * nt; t = nt; nt = tmp;
        tmp = r - quo * nr; r = nr; nr = tmp;
    }
    if (r != 1) return false;
    if (t < 0) t += q;
    out = (u64)t;
    return true;
}
// NTTProcessor::mod_inverse (ntt_processor.cpp:63-89) as the reference
// computes it: a signed extended Euclid on int64 casts of a % m and m, so
// for m >= 2^63 (negative as int64) the loop stops at once and the result is
// not an inverse (1 for a >= 2^63, else 0).  The compat transform uses these
// values for psi^-1 and N^-1 (:179-182), so its inverse matches the
// reference bit for bit at every q -- at q >= 2^63 that is the reference's
// all-zero inverse.  Wrapping arithmetic; x / 0 = 0 and x % 0 = x (the
// AArch64 semantics of the platform the reference targets).
u64 ref_mod_inverse(u64 a, u64 m) {
    if (m <= 1) return 0;
    const int64_t m0 = (int64_t)m;
    int64_t x0 = 0, x1 = 1, as = (int64_t)(a % m), ms = (int64_t)m;
    while (as > 1) {
        const int64_t qt = ms == 0 ? 0 : (ms == -1 ? -as : as / ms);
        int64_t t = ms;
        ms = ms == 0 ? as : (ms == -1 ? 0 : as % ms);
        as = t;
        t = x0;
        x0 = (int64_t)((u64)x1 - (u64)qt * (u64)x0);
        x1 = t;
    }
    if (x1 < 0) x1 = (int64_t)((u64)x1 + (u64)m0);
    return (u64)x1;
}

template <typename W>
W neg_inv_pow2(W q) {  // -q^-1 mod 2^W (q odd), Newton
    W x = q;
    for (int i = 0; i < 6; ++i) x *= W(2) - q * x;
    return W(0) - x;
}
template <typename W>
FHE_NS::Tw<W> make_tw(u64 w, u64 q) {
    constexpr int BITS = sizeof(W) * 8;
    FHE_NS::Tw<W> t;
    t.w = (W)w;
    t.wp = (W)(((u128)w << BITS) / q);
    return t;
}

// ---------------------------------------------------------------- context
struct Tables {
    void *twf = nullptr, *twi = nullptr;
    void *wtf = nullptr, *wti = nullptr;  // q >= 2^62: Montgomery-form stage tables (ntt_wide.hip)
};

}  // namespace

struct fhe_ctx {
    u32 n = 0, logn = 0;
    u64 q = 0, psi = 0, psi_inv = 0, inv_n = 0;
    int mode = 0, device = 0, word = 64;
    bool wide = false;  // q >= 2^62: transforms in ntt_wide.hip, fused ciphertext kernels unavailable
    hipStream_t own_stream = nullptr, stream = nullptr;
    Tables tab;
    FHE_NS::Plan plan{};
    FHE_NS::BigSync big_sync;  // plan.big_sync
    std::vector<u64> fwd_tw, inv_tw;  // reference twiddle vectors (host copy)
    // host staging pipeline of the FHE_HOST batch calls (staged()): kSlots
    // slots, each a stream, pinned host buffers and device buffers for two
    // inputs and one output, so that the host copy of chunk k+1, the H2D of
    // k+1, the kernel of k and the D2H of k-1 overlap
    struct Pipe {
        static constexpr int kSlots = 3;
        hipStream_t st[kSlots] = {};
        hipEvent_t done[kSlots] = {};
        void *pin[kSlots][3] = {};
        void *dev[kSlots][3] = {};
        size_t bytes = 0;  // per buffer
    } pipe;
    std::mutex scratch_mu;
    // blind rotation: ping-pong accumulator buffer and the captured launch
    // sequence (1 rotation + lwe_dim CMux steps + copy) as a hipGraph, reused
    // while the call's buffers and shape are unchanged
    struct BrGraph {
        const void *acc = nullptr, *lwe_a = nullptr, *lwe_b = nullptr, *bsk = nullptr;
        size_t batch = 0;
        uint32_t k = 0, base_log = 0, level = 0, dim = 0;
        uint64_t lwe_q = 0;
        hipStream_t stream = nullptr;
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
    } br;
    std::mutex br_mu;
    void *br_tmp = nullptr;
    size_t br_tmp_bytes = 0;
    // completion of the last enqueued use of br_tmp: a call on another
    // stream waits for it before reusing the buffer
    hipEvent_t br_done = nullptr;
    hipStream_t br_done_stream = nullptr;
    // multi-device context (fhe_ctx_create_multi): one full context per
    // listed device; this object then only holds the parameters and routes
    // every call to them
    std::vector<fhe_ctx *> subs;
    bool multi() const { return !subs.empty(); }
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// NTTProcessor::find_primitive_root (ntt_processor.cpp:92-128): smallest
// g >= 2 with psi = g^((q-1)/2N), psi^2N == 1, psi^N == q-1.  The search is
// capped (the reference loops to q; a prime q finds g within a few tries).
int find_psi(u32 n, u64 q, u64 &psi) {
    const u64 two_n = (u64)n * 2;
    if ((q - 1) % two_n != 0)
        return fail(FHE_ERR_NOT_NTT_FRIENDLY, "Modulus is not NTT-friendly: q \xe2\x89\xa2 1 (mod 2N)");
    const u64 e = (q - 1) / two_n;
    const u64 cap = std::min<u64>(q, (u64)1 << 22);
    for (u64 g = 2; g < cap; ++g) {
        const u64 w = powmod(g, e, q);
        if (powmod(w, two_n, q) == 1 && powmod(w, n, q) == q - 1) {
            psi = w;
            return FHE_OK;
        }
    }
    return fail(FHE_ERR_NO_ROOT, "Could not find primitive root for given parameters");
}

template <typename W>
int build_tables(fhe_ctx *c, FHE_NS::NttArgs<W> &A) {
    const u32 n = c->n, L = c->logn;
    const u64 q = c->q;
    constexpr int BITS = sizeof(W) * 8;
    std::vector<FHE_NS::Tw<W>> twf(n), twi(n);
    // stage-major: entry 2^s + j holds the twiddle of butterfly j in stage s.
    // compat: psi^(j*N/2^(s+1)) (ntt_processor.cpp:283-286).  negacyclic:
    // psi^((2j+1)*N/2^(s+1)) -- the cyclic transform of the psi^i-twisted
    // input, X_k = sum_i a_i psi^(i(2k+1)), with the twist merged into the
    // stages (stage s of size 2m = 2^(s+1) is a negacyclic transform with
    // root psi^(N/2m), so its butterfly j takes that root to the 2j+1).  The
    // inverse table holds the inverse of every entry, so the same kernels
    // (and the N^-1 fold) serve both modes, with no twist or untwist pass.
    for (u32 s = 0; s < L; ++s) {
        for (u32 j = 0; j < (1u << s); ++j) {
            const u64 ex = c->mode == FHE_MODE_COMPAT ? (u64)j * (n >> (s + 1)) : (u64)(2 * j + 1) * (n >> (s + 1));
            twf[(1u << s) + j] = make_tw<W>(c->fwd_tw[ex], q);
            twi[(1u << s) + j] = make_tw<W>(c->inv_tw[ex], q);
        }
    }
    twf[0] = make_tw<W>(1, q);
    twi[0] = make_tw<W>(1, q);
    if constexpr (sizeof(W) == 4 && FHE_NS::kNegFwdTw)
        for (auto &t : twf) t.w = (W)(0u - t.w);  // Arith::ct's negated-twiddle butterfly
    const u64 R = (u64)((((u128)1) << BITS) % q);
    const u64 ninv_r = mulmod(c->inv_n, R, q);
    const size_t bytes = sizeof(FHE_NS::Tw<W>) * n;
    void **dst[2] = {&c->tab.twf, &c->tab.twi};
    const void *srcs[2] = {twf.data(), twi.data()};
    for (int i = 0; i < 2; ++i) {
        HIP_TRY(hipMalloc(dst[i], bytes), "hipMalloc(twiddles)");
        HIP_TRY(hipMemcpy(*dst[i], srcs[i], bytes, hipMemcpyHostToDevice), "hipMemcpy(twiddles)");
    }
    A.twf = (const FHE_NS::Tw<W> *)c->tab.twf;
    A.twi = (const FHE_NS::Tw<W> *)c->tab.twi;
    A.ar.q = (W)q;
    A.ar.q2 = (W)(2 * q);
    A.ar.qinv = neg_inv_pow2<W>((W)q);
    A.ar.r2 = (W)mulmod(R, R, q);
    A.q64 = q;
    A.mu64 = (u64)((((u128)1) << 64) / q);
    // stage-0 twiddle w0 (1 in compat mode, psi^(N/2) in negacyclic mode)
    // and its inverse, folded into the scaled stage-0 butterflies
    const u64 w0 = L ? c->fwd_tw[c->mode == FHE_MODE_COMPAT ? 0 : n / 2] : 1;
    const u64 w0i = L ? c->inv_tw[c->mode == FHE_MODE_COMPAT ? 0 : n / 2] : 1;
    A.ninv = {make_tw<W>(c->inv_n, q), make_tw<W>(mulmod(c->inv_n, w0i, q), q)};
    A.ninv_r = {make_tw<W>(ninv_r, q), make_tw<W>(mulmod(ninv_r, w0i, q), q)};
    A.rs = {make_tw<W>(R, q), make_tw<W>(mulmod(R, w0, q), q)};
    A.rmod = make_tw<W>(R, q);
    A.one = make_tw<W>(1, q);
    return FHE_OK;
}

// q >= 2^62 (ntt_wide.hip): the same stage-major twiddles in Montgomery form
// (w 2^64 mod q) plus the Montgomery constants of WideArgs.
int build_wide_tables(fhe_ctx *c) {
    const u32 n = c->n, L = c->logn;
    const u64 q = c->q;
    const u64 R = (u64)((((u128)1) << 64) % q);
    std::vector<u64> twf(n), twi(n);
    twf[0] = twi[0] = R;
    for (u32 s = 0; s < L; ++s)
        for (u32 j = 0; j < (1u << s); ++j) {
            const u64 ex = c->mode == FHE_MODE_COMPAT ? (u64)j * (n >> (s + 1)) : (u64)(2 * j + 1) * (n >> (s + 1));
            twf[(1u << s) + j] = mulmod(c->fwd_tw[ex], R, q);
            twi[(1u << s) + j] = mulmod(c->inv_tw[ex], R, q);
        }
    const size_t bytes = sizeof(u64) * n;
    HIP_TRY(hipMalloc(&c->tab.wtf, bytes), "hipMalloc(twiddles)");
    HIP_TRY(hipMalloc(&c->tab.wti, bytes), "hipMalloc(twiddles)");
    HIP_TRY(hipMemcpy(c->tab.wtf, twf.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy(twiddles)");
    HIP_TRY(hipMemcpy(c->tab.wti, twi.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy(twiddles)");
    FHE_NS::WideArgs &W = c->plan.wa;
    W.twf = (const u64 *)c->tab.wtf;
    W.twi = (const u64 *)c->tab.wti;
    W.q = q;
    W.qinv = neg_inv_pow2<u64>(q);
    W.mu = (u64)((((u128)1) << 64) / q);
    W.r2 = mulmod(R, R, q);
    W.ninv_m = mulmod(c->inv_n, R, q);
    W.ninv_r2 = mulmod(W.ninv_m, R, q);
    return FHE_OK;
}

void free_pipe(fhe_ctx *c) {
    auto &P = c->pipe;
    for (int i = 0; i < fhe_ctx::Pipe::kSlots; ++i) {
        if (P.st[i]) (void)hipStreamSynchronize(P.st[i]);
        for (int j = 0; j < 3; ++j) {
            if (P.pin[i][j]) (void)hipHostFree(P.pin[i][j]);
            if (P.dev[i][j]) (void)hipFree(P.dev[i][j]);
            P.pin[i][j] = P.dev[i][j] = nullptr;
        }
        if (P.done[i]) (void)hipEventDestroy(P.done[i]);
        if (P.st[i]) (void)hipStreamDestroy(P.st[i]);
        P.done[i] = nullptr;
        P.st[i] = nullptr;
    }
    P.bytes = 0;
}

void free_tables(fhe_ctx *c) {
    void *p[4] = {c->tab.twf, c->tab.twi, c->tab.wtf, c->tab.wti};
    for (void *x : p)
        if (x) (void)hipFree(x);
    c->tab = Tables{};
    free_pipe(c);
    for (auto &s : c->plan.big_scratch)
        if (s) { (void)hipFree(s); s = nullptr; }
    if (c->big_sync.done) { (void)hipEventDestroy(c->big_sync.done); c->big_sync.done = nullptr; }
    if (c->br.exec) (void)hipGraphExecDestroy(c->br.exec);
    if (c->br.graph) (void)hipGraphDestroy(c->br.graph);
    c->br = fhe_ctx::BrGraph{};
    if (c->br_tmp) { (void)hipFree(c->br_tmp); c->br_tmp = nullptr; }
    c->br_tmp_bytes = 0;
    if (c->br_done) { (void)hipEventDestroy(c->br_done); c->br_done = nullptr; }
}

FHE_NS::ModConsts mod_consts(u64 q) {
    FHE_NS::ModConsts m{};
    m.q = q;
    m.mu = q > 1 ? (u64)((((u128)1) << 64) / q) : 0;
    m.fast = (q & 1) && q > 1 && !(q >> 63);
    if ((q & 1) && q > 1) {  // Montgomery constants for any odd q (the key MAC at q >= 2^62 uses them)
        m.qinv = neg_inv_pow2<u64>(q);
        const u64 R = (u64)((((u128)1) << 64) % q);
        m.r2 = mulmod(R, R, q);
    }
    return m;
}

int check_ctx(const fhe_ctx *c) {
    if (!c) return fail(FHE_ERR_INVALID_ARG, "null context");
    return FHE_OK;
}

// ---------------------------------------------------------------- multi-device routing
// The sub-context that owns device buffer p (FHE_DEVICE calls run where
// their data lives).
fhe_ctx *sub_for_pointer(const fhe_ctx *m, const void *p) {
    hipPointerAttribute_t at{};
    if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    for (fhe_ctx *s : m->subs)
        if (s->device == at.device) return s;
    return nullptr;
}

// Run fn(sub, lo, count) over a multi-device context.  FHE_HOST: the batch
// is cut into ndev contiguous balanced ranges (fhe_gpu/shard.py's
// shard_range), one host thread per device (the last range on the calling
// thread), as the reference's batch_encrypt chunks a batch over threads that
// share one read-only NTTProcessor (encryption.cpp:472, 520-533).
// FHE_DEVICE: the whole batch on the sub-context of the device that holds
// `probe`.
template <typename F>
int multi_run(fhe_ctx *m, size_t batch, int where, const void *probe, F &&fn) {
    if (where != FHE_HOST && where != FHE_DEVICE) return fail(FHE_ERR_INVALID_ARG, "where must be FHE_HOST or FHE_DEVICE");
    if (batch == 0) return FHE_OK;
    if (where == FHE_DEVICE) {
        fhe_ctx *s = sub_for_pointer(m, probe);
        if (!s) return fail(FHE_ERR_INVALID_ARG, "device buffer is not memory of any device of this context");
        return fn(s, (size_t)0, batch);
    }
    const size_t nd = m->subs.size(), base = batch / nd, extra = batch % nd;
    std::vector<int> rc(nd, FHE_OK);
    std::vector<std::string> msg(nd);
    std::vector<std::thread> th;
    size_t lo = 0;
    for (size_t i = 0; i < nd; ++i) {
        const size_t cnt = base + (i < extra ? 1 : 0);
        if (cnt) {
            auto job = [&, i, lo, cnt] {
                rc[i] = fn(m->subs[i], lo, cnt);
                if (rc[i] != FHE_OK) msg[i] = g_err;
            };
            if (i + 1 == nd) job();
            else th.emplace_back(job);
        }
        lo += cnt;
    }
    for (auto &t : th) t.join();
    for (size_t i = 0; i < nd; ++i)
        if (rc[i] != FHE_OK) return fail(rc[i], msg[i]);
    return FHE_OK;
}
// Whole-call routing for the single-buffer entry points (key preparation):
// the device of `probe` (FHE_DEVICE) or the first device (FHE_HOST).
template <typename F>
int multi_one(fhe_ctx *m, int where, const void *probe, F &&fn) {
    if (where == FHE_DEVICE) {
        fhe_ctx *s = sub_for_pointer(m, probe);
        if (!s) return fail(FHE_ERR_INVALID_ARG, "device buffer is not memory of any device of this context");
        return fn(s);
    }
    return fn(m->subs[0]);
}
// Route a batch entry point of a multi-device context: CALL runs with `c`
// bound to the sub-context and [lo, lo + nb) its range of the batch.
#define FHE_MULTI(BATCH, WHERE, PROBE, CALL)                                                           \
    if (c && c->multi())                                                                               \
    return multi_run(c, (BATCH), (WHERE), (PROBE),                                                     \
                     [&](fhe_ctx *sub, size_t lo, size_t nb) { return [&](fhe_ctx *c) { return CALL; }(sub); })
#define FHE_MULTI_ONE(WHERE, PROBE, CALL) \
    if (c && c->multi()) return multi_one(c, (WHERE), (PROBE), [&](fhe_ctx *sub) { return [&](fhe_ctx *c) { return CALL; }(sub); })

// The context's plan with its launches redirected to stream s (the host
// staging pipeline runs chunks on its own streams).
static FHE_NS::Plan on(const fhe_ctx *c, hipStream_t s) {
    FHE_NS::Plan p = c->plan;
    p.stream = s;
    return p;
}

#define FHE_TRY_STAGE(expr)                   \
    do {                                      \
        if (int _rc = (expr)) return _rc;     \
    } while (0)

// Host <-> pinned copy on several threads (a single thread moves ~10 GB/s
// from pageable memory, well under what PCIe takes).
static void par_copy(void *dst, const void *src, size_t bytes) {
    static const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    const size_t min_piece = (size_t)4 << 20;
    const unsigned nt = (unsigned)std::max<size_t>(1, std::min<size_t>(hw, bytes / min_piece));
    if (nt <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const size_t piece = (bytes / nt + 63) & ~(size_t)63;
    std::vector<std::thread> th;
    for (unsigned i = 1; i < nt; ++i) {
        const size_t lo = i * piece;
        if (lo >= bytes) break;
        const size_t len = std::min(piece, bytes - lo);
        th.emplace_back([=] { std::memcpy((char *)dst + lo, (const char *)src + lo, len); });
    }
    std::memcpy(dst, src, std::min(piece, bytes));
    for (auto &t : th) t.join();
}

// Host staging: run fn(device pointers, n units, stream) over chunks of at
// most FHE_STAGE_MB MiB per buffer (default 64), pipelined over the
// context's kSlots slots (fhe_ctx::Pipe).  nin inputs, one output; all of
// `*_elems_per_unit` u64 per unit.  Synchronous: returns once every output
// chunk is back in `out`.
template <typename F>
int staged(fhe_ctx *c, const u64 *const *ins, int nin, size_t in_elems_per_unit, u64 *out,
           size_t out_elems_per_unit, size_t units, F &&fn) {
    std::lock_guard<std::mutex> lk(c->scratch_mu);
    auto &P = c->pipe;
    constexpr int S = fhe_ctx::Pipe::kSlots;
    static const size_t stage_bytes = [] {
        const char *v = std::getenv("FHE_STAGE_MB");
        const size_t mb = v ? (size_t)std::strtoull(v, nullptr, 10) : 64;
        return std::max<size_t>(1, mb) << 20;
    }();
    const size_t max_unit_bytes = std::max(in_elems_per_unit, out_elems_per_unit) * sizeof(u64);
    size_t chunk = std::max<size_t>(1, stage_bytes / max_unit_bytes);
    chunk = std::min(chunk, units);
    const size_t need = chunk * max_unit_bytes;
    if (P.bytes < need) {
        free_pipe(c);
        for (int i = 0; i < S; ++i) {
            HIP_TRY(hipStreamCreateWithFlags(&P.st[i], hipStreamNonBlocking), "hipStreamCreate(stage)");
            HIP_TRY(hipEventCreateWithFlags(&P.done[i], hipEventDisableTiming), "hipEventCreate(stage)");
            for (int j = 0; j < 3; ++j) {
                hipError_t e = hipMalloc(&P.dev[i][j], need);
                if (e == hipErrorOutOfMemory) return fail(FHE_ERR_OOM, "hipMalloc(stage): out of memory");
                HIP_TRY(e, "hipMalloc(stage)");
                HIP_TRY(hipHostMalloc(&P.pin[i][j], need, hipHostMallocDefault), "hipHostMalloc(stage)");
            }
        }
        P.bytes = need;
    }
    // order after work already queued on the context stream
    hipEvent_t entry = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&entry, hipEventDisableTiming), "hipEventCreate");
    HIP_TRY(hipEventRecord(entry, c->stream), "hipEventRecord");
    for (int i = 0; i < S; ++i) HIP_TRY(hipStreamWaitEvent(P.st[i], entry, 0), "hipStreamWaitEvent");
    (void)hipEventDestroy(entry);
    const size_t nchunks = (units + chunk - 1) / chunk;
    auto drain = [&](size_t k) -> int {  // chunk k's output back to `out`
        const int sl = (int)(k % S);
        HIP_TRY(hipEventSynchronize(P.done[sl]), "hipEventSynchronize(stage)");
        const size_t u0 = k * chunk, nu = std::min(chunk, units - u0);
        par_copy(out + u0 * out_elems_per_unit, P.pin[sl][2], nu * out_elems_per_unit * 8);
        return FHE_OK;
    };
    int rc = FHE_OK;
    for (size_t k = 0; k < nchunks && rc == FHE_OK; ++k) {
        const int sl = (int)(k % S);
        if (k >= (size_t)S && (rc = drain(k - S)) != FHE_OK) break;
        const size_t u0 = k * chunk, nu = std::min(chunk, units - u0);
        const u64 *dins[3] = {nullptr, nullptr, nullptr};
        for (int i = 0; i < nin; ++i) {
            const size_t b = nu * in_elems_per_unit * 8;
            par_copy(P.pin[sl][i], ins[i] + u0 * in_elems_per_unit, b);
            hipError_t e = hipMemcpyAsync(P.dev[sl][i], P.pin[sl][i], b, hipMemcpyHostToDevice, P.st[sl]);
            if (e != hipSuccess) { rc = hip_fail(e, "hipMemcpyAsync(H2D)"); break; }
            dins[i] = (const u64 *)P.dev[sl][i];
        }
        if (rc != FHE_OK) break;
        hipError_t e = fn(dins, (u64 *)P.dev[sl][2], nu, P.st[sl]);
        if (e == hipSuccess)
            e = hipMemcpyAsync(P.pin[sl][2], P.dev[sl][2], nu * out_elems_per_unit * 8, hipMemcpyDeviceToHost, P.st[sl]);
        if (e == hipSuccess) e = hipEventRecord(P.done[sl], P.st[sl]);
        if (e != hipSuccess) rc = hip_fail(e, "kernel launch");
    }
    if (rc != FHE_OK) {
        for (int i = 0; i < S; ++i) (void)hipStreamSynchronize(P.st[i]);
        return rc;
    }
    for (size_t k = nchunks > (size_t)S ? nchunks - S : 0; k < nchunks; ++k) FHE_TRY_STAGE(drain(k));
    return FHE_OK;
}

// Common driver for ops over [batch][n] buffers.
template <typename F>
int run_poly_op(fhe_ctx *c, const u64 *a, const u64 *b, u64 *out, size_t batch, int where, size_t in_per,
                size_t out_per, F &&fn) {
    if (int rc = check_ctx(c)) return rc;
    if ((!a && batch) || (!out && batch)) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    if (where != FHE_HOST && where != FHE_DEVICE) return fail(FHE_ERR_INVALID_ARG, "where must be FHE_HOST or FHE_DEVICE");
    if (batch == 0) return FHE_OK;
    DeviceGuard g(c->device);
    if (where == FHE_DEVICE) {
        const u64 *ins[3] = {a, b, nullptr};
        HIP_TRY(fn(ins, out, batch, c->stream), "kernel launch");
        return FHE_OK;
    }
    const u64 *ins[2] = {a, b};
    return staged(c, ins, b ? 2 : 1, in_per, out, out_per, batch, fn);
}

// ---------------------------------------------------------------- ciphertext ops
#define FHE_TRY(expr)                 \
    do {                              \
        if (int _rc = (expr)) return _rc; \
    } while (0)

// Device temporaries of one call, stream-ordered (no device-wide sync).
class StreamTemp {
    std::vector<void *> p_;
    hipStream_t s_;

  public:
    explicit StreamTemp(hipStream_t s) : s_(s) {}
    ~StreamTemp() {
        for (void *x : p_) (void)hipFreeAsync(x, s_);
    }
    int alloc(size_t bytes, u64 *&out) {
        void *d = nullptr;
        hipError_t e = hipMallocAsync(&d, bytes ? bytes : 8, s_);
        if (e == hipErrorOutOfMemory) return fail(FHE_ERR_OOM, "hipMallocAsync: out of memory");
        if (e != hipSuccess) return hip_fail(e, "hipMallocAsync");
        p_.push_back(d);
        out = (u64 *)d;
        return FHE_OK;
    }
};

// Host-resident calls of the multi-buffer entry points: every host buffer is
// copied to a device temporary (inputs) or allocated (outputs), the device
// path runs, outputs are copied back.  No chunking: these ops are used at
// ciphertext-batch sizes far below HBM capacity.
class HostStage {
    std::vector<void *> allocs_;
    struct Back { void *host; const void *dev; size_t bytes; };
    std::vector<Back> back_;
    hipStream_t s_;

  public:
    explicit HostStage(hipStream_t s) : s_(s) {}
    ~HostStage() {
        for (void *p : allocs_) (void)hipFreeAsync(p, s_);
    }
    // where == FHE_DEVICE: pass through; else stage.  dir: 1 in, 2 out, 3 in/out.
    // Temporaries come from the device's stream-ordered pool (kept warm by
    // the release threshold set at context creation): no hipMalloc/hipFree
    // device synchronisation per call.
    template <typename T>
    int map(int where, T *&ptr, size_t bytes, int dir) {
        if (where == FHE_DEVICE || ptr == nullptr || bytes == 0) return FHE_OK;
        void *d = nullptr;
        hipError_t e = hipMallocAsync(&d, bytes, s_);
        if (e == hipErrorOutOfMemory) return fail(FHE_ERR_OOM, "hipMallocAsync: out of memory");
        if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(stage)");
        allocs_.push_back(d);
        if (dir & 1) HIP_TRY(hipMemcpyAsync(d, (const void *)ptr, bytes, hipMemcpyHostToDevice, s_), "hipMemcpy(H2D)");
        if (dir & 2) back_.push_back({(void *)ptr, d, bytes});
        ptr = (T *)d;
        return FHE_OK;
    }
    int finish() {
        for (auto &b : back_) HIP_TRY(hipMemcpyAsync(b.host, b.dev, b.bytes, hipMemcpyDeviceToHost, s_), "hipMemcpy(D2H)");
        HIP_TRY(hipStreamSynchronize(s_), "hipStreamSynchronize");
        return FHE_OK;
    }
};

static bool overlaps(const void *a, size_t an, const void *b, size_t bn) {
    const char *x = (const char *)a, *y = (const char *)b;
    return a && b && an && bn && x < y + bn && y < x + an;
}

static int check_common(const fhe_ctx *c, int where, size_t batch) {
    if (int rc = check_ctx(c)) return rc;
    if (where != FHE_HOST && where != FHE_DEVICE) return fail(FHE_ERR_INVALID_ARG, "where must be FHE_HOST or FHE_DEVICE");
    (void)batch;
    return FHE_OK;
}
static int check_fused(const fhe_ctx *c, const char *what) {
    if ((int)c->logn > FHE_NS::kMaxFusedLogN)
        return fail(FHE_ERR_UNSUPPORTED, std::string(what) + " implemented for degrees up to 16384");
    if (c->wide) return fail(FHE_ERR_UNSUPPORTED, std::string(what) + " implemented for moduli below 2^62");
    return FHE_OK;
}
static int check_relin_decomp(uint32_t base_log, uint32_t level) {
    if (base_log == 0 || base_log > 63 || (level > 0 && (u64)(level - 1) * base_log >= 64))
        return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    return FHE_OK;
}

// Montgomery word of the prepared keys for launch_mac_keys: 32 / 64, or 65
// for q >= 2^62 (canonical Montgomery products with the carry bit).
static int mac_word(const fhe_ctx *c) { return c->wide ? 65 : c->word; }

// Composed (unfused) ciphertext multiply for n > 16384: 4 forward
// transforms, tensor, 3 inverse transforms through a temporary.
static int ct_mul_composed(fhe_ctx *c, const u64 *x, const u64 *y, u64 *out, size_t batch) {
    const size_t n = c->n;
    StreamTemp tmp(c->stream);
    u64 *tx = nullptr;
    FHE_TRY(tmp.alloc(batch * 4 * n * 8, tx));
    u64 *ty = tx + batch * 2 * n;
    hipError_t e = FHE_NS::launch_fwd(c->plan, x, tx, batch * 2, 0);
    if (e == hipSuccess) e = FHE_NS::launch_fwd(c->plan, y, ty, batch * 2, 0);
    if (e == hipSuccess) e = FHE_NS::launch_tensor_ntt(mod_consts(c->q), tx, ty, out, c->n, batch, c->stream);
    if (e == hipSuccess) e = FHE_NS::launch_inv(c->plan, out, out, batch * 3);
    if (e != hipSuccess) return hip_fail(e, "ct_multiply");
    return FHE_OK;
}

static int ct_mul_device(fhe_ctx *c, const u64 *x, const u64 *y, u64 *out, size_t batch, int is_ntt) {
    const size_t in_b = batch * 2 * c->n * 8, out_b = batch * 3 * c->n * 8;
    if (overlaps(out, out_b, x, in_b) || overlaps(out, out_b, y, in_b))
        return fail(FHE_ERR_INVALID_ARG, "output must not overlap the input ciphertexts");
    if (is_ntt) {
        HIP_TRY(FHE_NS::launch_tensor_ntt(mod_consts(c->q), x, y, out, c->n, batch, c->stream), "tensor kernel");
        return FHE_OK;
    }
    if ((int)c->logn > FHE_NS::kMaxFusedLogN || c->wide) return ct_mul_composed(c, x, y, out, batch);
    HIP_TRY(FHE_NS::launch_ct_mul(c->plan, x, y, out, batch), "ct_mul kernel");
    return FHE_OK;
}

// Composed TFHE external product for shapes the fused kernel does not take
// (GLWE dimension k > 1, N > 16384): decompose every GLWE row
// (decompose_polynomial), forward-transform all digit polynomials, the
// NTT-domain key MAC per output component, inverse.  Bit-identical to the
// fused kernel and to the reference's per-row inverse-and-add, since every
// step is exact over Z_q and the inverse is linear.  Device pointers; the
// digits are staged in chunks of at most ~1 GiB, in `dig` when the caller
// owns a buffer of extprod_digit_words() (the blind-rotation loop: one
// buffer for every step), else in a stream-ordered temporary.  Asynchronous
// on the context stream.
static size_t extprod_digit_words(const fhe_ctx *c, uint32_t k1, uint32_t level, size_t batch) {
    const size_t per = (size_t)k1 * level * c->n;
    return std::max<size_t>(1, std::min(batch, ((size_t)1 << 27) / per)) * per;
}
static int extprod_composed(fhe_ctx *c, uint32_t k1, uint32_t level, uint32_t base_log, const u64 *glwe,
                            const u64 *ggsw, u64 *out, size_t batch, u64 *dig = nullptr) {
    const size_t n = c->n, rows = (size_t)k1 * level;
    const size_t chunk = extprod_digit_words(c, k1, level, batch) / (rows * n);
    const FHE_NS::ModConsts m = mod_consts(c->q);
    StreamTemp tmp(c->stream);
    if (!dig) FHE_TRY(tmp.alloc(chunk * rows * n * 8, dig));
    for (size_t b0 = 0; b0 < batch; b0 += chunk) {
        const size_t nb = std::min(chunk, batch - b0);
        const u64 *g = glwe + b0 * k1 * n;
        u64 *o = out + b0 * k1 * n;
        hipError_t e = FHE_NS::launch_decompose(m, g, dig, (u32)n, nb * k1, base_log, level, c->stream);
        if (e == hipSuccess) e = FHE_NS::launch_fwd(c->plan, dig, dig, nb * rows, 0);
        if (e == hipSuccess)
            e = FHE_NS::launch_mac_keys(m, mac_word(c), dig, ggsw, o, (u32)n, nb, (u32)rows, k1, 0, c->stream);
        if (e == hipSuccess) e = FHE_NS::launch_inv(c->plan, o, o, nb * k1);
        if (e != hipSuccess) return hip_fail(e, "composed external product");
    }
    return FHE_OK;
}

// Composed relinearisation for N > 16384: unsigned LSB-first digits of c2,
// forward transforms, MAC with the (a_l, b_l) pairs swapped per component,
// inverse, + c_j.
static int relin_composed(fhe_ctx *c, uint32_t base_log, uint32_t level, const u64 *ct3, const u64 *rlk, u64 *out,
                          size_t batch) {
    const size_t n = c->n, per = (size_t)level * n * 8;
    const size_t chunk = std::max<size_t>(1, std::min(batch, ((size_t)1 << 30) / per));
    const FHE_NS::ModConsts m = mod_consts(c->q);
    StreamTemp tmp(c->stream);
    u64 *dig = nullptr;
    FHE_TRY(tmp.alloc(chunk * per, dig));
    for (size_t b0 = 0; b0 < batch; b0 += chunk) {
        const size_t nb = std::min(chunk, batch - b0);
        const u64 *x = ct3 + b0 * 3 * n;
        u64 *o = out + b0 * 2 * n;
        hipError_t e = FHE_NS::launch_relin_digits(x, dig, (u32)n, nb, base_log, level, c->stream);
        if (e == hipSuccess) e = FHE_NS::launch_fwd(c->plan, dig, dig, nb * level, 0);
        if (e == hipSuccess) e = FHE_NS::launch_mac_keys(m, mac_word(c), dig, rlk, o, (u32)n, nb, level, 2, 1, c->stream);
        if (e == hipSuccess) e = FHE_NS::launch_inv(c->plan, o, o, nb * 2);
        if (e == hipSuccess) e = FHE_NS::launch_add_rows(m, o, x, (u32)n, nb, 2, 3, c->stream);
        if (e != hipSuccess) return hip_fail(e, "composed relinearisation");
    }
    return FHE_OK;
}

static int relin_device(fhe_ctx *c, uint32_t base_log, uint32_t level, const u64 *ct3, const u64 *rlk, u64 *out,
                        size_t batch) {
    const size_t n = c->n;
    if (overlaps(out, batch * 2 * n * 8, ct3, batch * 3 * n * 8))
        return fail(FHE_ERR_INVALID_ARG, "output must not overlap the input ciphertexts");
    if (level == 0) {  // no key pairs: c0, c1 copied (encryption.cpp:966-972)
        HIP_TRY(hipMemcpy2DAsync(out, 2 * n * 8, ct3, 3 * n * 8, 2 * n * 8, batch, hipMemcpyDeviceToDevice, c->stream),
                "hipMemcpy2D");
        return FHE_OK;
    }
    if ((int)c->logn > FHE_NS::kMaxFusedLogN || c->wide) return relin_composed(c, base_log, level, ct3, rlk, out, batch);
    HIP_TRY(FHE_NS::launch_relin(c->plan, (int)level, (int)base_log, ct3, rlk, out, batch), "relin kernel");
    return FHE_OK;
}

}  // namespace

// =====================================================================
extern "C" {

const char *fhe_last_error(void) { return g_err.c_str(); }
const char *fhe_version(void) { return "fhe-mi355x 0.1.0 (gfx950)"; }

int fhe_detect(fhe_hw_caps *caps) {
    if (!caps) return fail(FHE_ERR_INVALID_ARG, "null caps");
    std::memset(caps, 0, sizeof(*caps));
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    caps->device_count = count;
    if (count > 0) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, 0) == hipSuccess) {
            caps->compute_units = p.multiProcessorCount;
            caps->wavefront_size = p.warpSize;
            caps->hbm_bytes = p.totalGlobalMem;
            caps->lds_bytes_per_cu = p.maxSharedMemoryPerMultiProcessor;
            std::snprintf(caps->arch, sizeof(caps->arch), "%s", p.gcnArchName);
            std::snprintf(caps->name, sizeof(caps->name), "%s", p.name);
            caps->xcds = std::strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 8 : 1;
        }
    }
    return FHE_OK;
}

int fhe_ctx_create(uint32_t n, uint64_t q, int mode, int device, fhe_ctx **out) {
    if (!out) return fail(FHE_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    // NTTProcessor constructor validation order (ntt_processor.cpp:140-153)
    if (n == 0 || (n & (n - 1)) != 0) return fail(FHE_ERR_DEGREE_POW2, "Polynomial degree must be a power of 2");
    if (n < 4 || n > 65536) return fail(FHE_ERR_DEGREE_RANGE, "Polynomial degree must be between 4 and 65536");
    if ((q & 1) == 0) return fail(FHE_ERR_MODULUS_EVEN, "Modulus must be odd");
    if (mode != FHE_MODE_COMPAT && mode != FHE_MODE_NEGACYCLIC) return fail(FHE_ERR_INVALID_ARG, "unknown mode");
    u64 psi = 0;
    if (int rc = find_psi(n, q, psi)) return rc;
    u32 logn = 0;
    while ((1u << logn) < n) ++logn;
    if ((int)logn > FHE_NS::kMaxLogN)
        return fail(FHE_ERR_UNSUPPORTED, "GPU kernels implement degrees up to 16384 (got " + std::to_string(n) + ")");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(FHE_ERR_DEVICE, "no HIP device available (the backend has no CPU fallback)");
    if (device < 0 || device >= count) return fail(FHE_ERR_INVALID_ARG, "device ordinal out of range");

    fhe_ctx *c = new fhe_ctx();
    c->n = n; c->logn = logn; c->q = q; c->psi = psi; c->mode = mode; c->device = device;
    c->word = q < (1ull << 30) ? 32 : 64;
    c->wide = (q >> 62) != 0;
    if (!invmod(psi, q, c->psi_inv) || !invmod(n, q, c->inv_n)) {
        delete c;
        return fail(FHE_ERR_NO_ROOT, "Could not find primitive root for given parameters");
    }
    if (mode == FHE_MODE_COMPAT) {  // the reference's own constants (equal to the true inverses below 2^63)
        c->psi_inv = ref_mod_inverse(psi, q);
        c->inv_n = ref_mod_inverse(n, q);
    }
    c->fwd_tw.resize(n);
    c->inv_tw.resize(n);
    c->fwd_tw[0] = c->inv_tw[0] = 1;
    for (u32 i = 1; i < n; ++i) {
        c->fwd_tw[i] = mulmod(c->fwd_tw[i - 1], psi, q);
        c->inv_tw[i] = mulmod(c->inv_tw[i - 1], c->psi_inv, q);
    }
    DeviceGuard g(device);
    int rc = c->word == 32 ? build_tables<u32>(c, c->plan.a32) : build_tables<u64>(c, c->plan.a64);
    if (rc == FHE_OK && c->wide) rc = build_wide_tables(c);
    if (rc == FHE_OK && (int)logn > FHE_NS::kMaxFusedLogN) {
        // two-pass transforms (ntt_big.hip): 2 x 256 MiB of chunk scratch
        c->plan.big_chunk = ((size_t)1 << 25) >> logn;
        for (auto &sp : c->plan.big_scratch) {
            hipError_t e = hipMalloc((void **)&sp, c->plan.big_chunk * n * sizeof(u64));
            if (e != hipSuccess) { rc = hip_fail(e, "hipMalloc(big-N scratch)"); break; }
        }
    }
    if (rc == FHE_OK) {
        hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
        if (e != hipSuccess) rc = hip_fail(e, "hipStreamCreate");
    }
    if (rc == FHE_OK) {
        // call temporaries (HostStage, StreamTemp) come from the device's
        // stream-ordered pool; keep up to 8 GiB of it cached across
        // synchronisations instead of returning it to the driver each time
        hipMemPool_t pool = nullptr;
        if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess && pool) {
            uint64_t keep = (uint64_t)8 << 30;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        }
        (void)hipGetLastError();
    }
    if (rc != FHE_OK) {
        free_tables(c);
        delete c;
        return rc;
    }
    c->stream = c->own_stream;
    c->plan.logn = logn;
    c->plan.word = c->word;
    c->plan.wide = c->wide;
    c->plan.lazy = c->word == 32 && (u128)(4 + 2 * logn) * q <= ((u128)1 << 32);
    c->plan.stream = c->stream;
    c->plan.big_sync = &c->big_sync;
    *out = c;
    return FHE_OK;
}

int fhe_ctx_create_multi(uint32_t n, uint64_t q, int mode, const int *devices, int ndev, fhe_ctx **out) {
    if (!out) return fail(FHE_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    if (!devices || ndev < 1) return fail(FHE_ERR_INVALID_ARG, "at least one device required");
    fhe_ctx *m = new fhe_ctx();
    for (int i = 0; i < ndev; ++i) {
        fhe_ctx *s = nullptr;
        const int rc = fhe_ctx_create(n, q, mode, devices[i], &s);
        if (rc != FHE_OK) {
            const std::string msg = g_err;
            fhe_ctx_destroy(m);
            return fail(rc, msg);
        }
        m->subs.push_back(s);
    }
    const fhe_ctx *s0 = m->subs[0];
    m->n = s0->n; m->logn = s0->logn; m->q = s0->q; m->psi = s0->psi; m->psi_inv = s0->psi_inv;
    m->inv_n = s0->inv_n; m->mode = s0->mode; m->device = s0->device; m->word = s0->word;
    m->fwd_tw = s0->fwd_tw; m->inv_tw = s0->inv_tw;
    m->stream = s0->stream;
    *out = m;
    return FHE_OK;
}

int fhe_ctx_device_count(const fhe_ctx *c, int *ndev) {
    if (int rc = check_ctx(c)) return rc;
    if (!ndev) return fail(FHE_ERR_INVALID_ARG, "null out");
    *ndev = c->multi() ? (int)c->subs.size() : 1;
    return FHE_OK;
}

int fhe_ctx_sub(const fhe_ctx *c, int i, fhe_ctx **out) {
    if (int rc = check_ctx(c)) return rc;
    if (!out) return fail(FHE_ERR_INVALID_ARG, "null out");
    const int nd = c->multi() ? (int)c->subs.size() : 1;
    if (i < 0 || i >= nd) return fail(FHE_ERR_INVALID_ARG, "device index out of range");
    *out = c->multi() ? c->subs[i] : const_cast<fhe_ctx *>(c);
    return FHE_OK;
}

void fhe_ctx_destroy(fhe_ctx *c) {
    if (!c) return;
    if (c->multi()) {
        for (auto it = c->subs.rbegin(); it != c->subs.rend(); ++it) fhe_ctx_destroy(*it);
        delete c;
        return;
    }
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_tables(c);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int fhe_ctx_set_stream(fhe_ctx *c, void *s) {
    if (int rc = check_ctx(c)) return rc;
    if (c->multi()) {  // the sub-context(s) of the stream's device
        int dev = -1;
        HIP_TRY(s ? hipStreamGetDevice((hipStream_t)s, &dev) : hipGetDevice(&dev), "hipStreamGetDevice");
        bool hit = false;
        for (fhe_ctx *sub : c->subs)
            if (sub->device == dev) {
                if (int rc = fhe_ctx_set_stream(sub, s)) return rc;
                hit = true;
            }
        if (!hit) return fail(FHE_ERR_INVALID_ARG, "stream is not on any device of this context");
        return FHE_OK;
    }
    c->stream = (hipStream_t)s;  // NULL is the device's null (legacy default) stream
    c->plan.stream = c->stream;
    return FHE_OK;
}
void *fhe_ctx_stream(const fhe_ctx *c) { return c ? (void *)c->stream : nullptr; }
int fhe_ctx_synchronize(fhe_ctx *c) {
    if (int rc = check_ctx(c)) return rc;
    if (c->multi()) {
        for (fhe_ctx *sub : c->subs)
            if (int rc = fhe_ctx_synchronize(sub)) return rc;
        return FHE_OK;
    }
    DeviceGuard g(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    return FHE_OK;
}

int fhe_ctx_get_info(const fhe_ctx *c, fhe_ctx_info *info) {
    if (int rc = check_ctx(c)) return rc;
    if (!info) return fail(FHE_ERR_INVALID_ARG, "null info");
    info->n = c->n; info->log_n = c->logn; info->q = c->q; info->psi = c->psi; info->psi_inv = c->psi_inv;
    info->inv_n = c->inv_n; info->mode = c->mode; info->word_bits = c->word; info->device = c->device;
    const int loge = c->logn < 4 ? (int)c->logn : 4;
    const int t = 1 << ((c->logn > (u32)FHE_NS::kMaxFusedLogN ? (u32)FHE_NS::kMaxFusedLogN : c->logn) - loge);
    info->polys_per_block = t >= 256 ? 1 : 256 / t;
    info->threads_per_block = t * info->polys_per_block;
    return FHE_OK;
}

int fhe_ctx_get_twiddles(const fhe_ctx *c, uint64_t *fwd, uint64_t *inv) {
    if (int rc = check_ctx(c)) return rc;
    if (fwd) std::memcpy(fwd, c->fwd_tw.data(), 8 * c->n);
    if (inv) std::memcpy(inv, c->inv_tw.data(), 8 * c->n);
    return FHE_OK;
}

int fhe_ntt_fwd_batch(fhe_ctx *c, const uint64_t *in, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, in, fhe_ntt_fwd_batch(c, in + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    return run_poly_op(c, in, nullptr, out, batch, where, c->n, c->n,
                       [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) { return FHE_NS::launch_fwd(on(c, st), d[0], o, nb, 0); });
}
int fhe_ntt_inv_batch(fhe_ctx *c, const uint64_t *in, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, in, fhe_ntt_inv_batch(c, in + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    return run_poly_op(c, in, nullptr, out, batch, where, c->n, c->n,
                       [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) { return FHE_NS::launch_inv(on(c, st), d[0], o, nb); });
}
int fhe_ntt_fwd_mul_batch(fhe_ctx *c, const uint64_t *a, const uint64_t *w, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, a, fhe_ntt_fwd_mul_batch(c, a + lo * c->n, w + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    if (!w && batch) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    return run_poly_op(c, a, w, out, batch, where, c->n, c->n, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_fwd_mul(on(c, st), d[0], d[1], o, nb);
    });
}
int fhe_polymul_batch(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, a, fhe_polymul_batch(c, a + lo * c->n, b + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    if (!b && batch) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    return run_poly_op(c, a, b, out, batch, where, c->n, c->n, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_polymul(on(c, st), d[0], d[1], o, nb);
    });
}
int fhe_pointwise_batch(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, a, fhe_pointwise_batch(c, a + lo * c->n, b + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    if (!b && batch) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const FHE_NS::ModConsts m = mod_consts(c->q);
    return run_poly_op(c, a, b, out, batch, where, c->n, c->n, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_modmul(m, d[0], d[1], o, nb * c->n, st);
    });
}
int fhe_poly_add_batch(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, a, fhe_poly_add_batch(c, a + lo * c->n, b + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    if (!b && batch) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const FHE_NS::ModConsts m = mod_consts(c->q);
    return run_poly_op(c, a, b, out, batch, where, c->n, c->n, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_addsub(m, d[0], d[1], o, nb * c->n, 0, st);
    });
}
int fhe_poly_sub_batch(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, a, fhe_poly_sub_batch(c, a + lo * c->n, b + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    if (!b && batch) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const FHE_NS::ModConsts m = mod_consts(c->q);
    return run_poly_op(c, a, b, out, batch, where, c->n, c->n, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_addsub(m, d[0], d[1], o, nb * c->n, 1, st);
    });
}
int fhe_poly_neg_batch(fhe_ctx *c, const uint64_t *a, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, a, fhe_poly_neg_batch(c, a + lo * c->n, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    return run_poly_op(c, a, nullptr, out, batch, where, c->n, c->n, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_neg(c->q, d[0], o, nb * c->n, st);
    });
}
int fhe_poly_mul_scalar_batch(fhe_ctx *c, const uint64_t *a, uint64_t scalar, uint64_t *out, size_t batch,
                              int where) {
    FHE_MULTI(batch, where, a, fhe_poly_mul_scalar_batch(c, a + lo * c->n, scalar, out + lo * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    const FHE_NS::ModConsts m = mod_consts(c->q);
    const u64 s = scalar % c->q;
    const u64 sp = (u64)(((u128)s << 64) / c->q);
    return run_poly_op(c, a, nullptr, out, batch, where, c->n, c->n, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_mul_scalar(m, d[0], s, sp, o, nb * c->n, st);
    });
}

// GLWE dimension: the fused kernels take k = 1 (and N <= 16384); other
// shapes run composed (extprod_composed).
constexpr uint32_t kMaxGlweDim = 16;
static bool fused_tfhe(const fhe_ctx *c, uint32_t k) {
    return k == 1 && (int)c->logn <= FHE_NS::kMaxFusedLogN && !c->wide;
}
static int check_decomp(const fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level) {
    (void)c;
    if (k == 0 || k > kMaxGlweDim) return fail(FHE_ERR_UNSUPPORTED, "GLWE dimension k must be between 1 and 16");
    if (level == 0 || base_log == 0 || base_log > 63 || (u64)base_log * level > 64)
        return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    return FHE_OK;
}

int fhe_ggsw_prepare(fhe_ctx *c, uint32_t k, uint32_t level, const uint64_t *ggsw, uint64_t *ggsw_ntt, int where) {
    FHE_MULTI_ONE(where, ggsw, fhe_ggsw_prepare(c, k, level, ggsw, ggsw_ntt, where));
    if (int rc = check_ctx(c)) return rc;
    if (k == 0 || k > kMaxGlweDim) return fail(FHE_ERR_UNSUPPORTED, "GLWE dimension k must be between 1 and 16");
    if (level == 0) return fail(FHE_ERR_INVALID_ARG, "level must be >= 1");
    const size_t polys = (size_t)(k + 1) * level * (k + 1);
    return run_poly_op(c, ggsw, nullptr, ggsw_ntt, polys, where, c->n, c->n,
                       [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) { return FHE_NS::launch_fwd(on(c, st), d[0], o, nb, 1); });
}

int fhe_external_product_batch(fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level, const uint64_t *glwe,
                               const uint64_t *ggsw_ntt, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, glwe, fhe_external_product_batch(c, k, base_log, level, glwe + lo * (k + 1) * c->n, ggsw_ntt, out + lo * (k + 1) * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    if (int rc = check_decomp(c, k, base_log, level)) return rc;
    if (!ggsw_ntt && batch) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const size_t per = (size_t)(k + 1) * c->n;
    if (!fused_tfhe(c, k)) {
        if (batch == 0) return FHE_OK;
        if (!glwe || !out) return fail(FHE_ERR_INVALID_ARG, "null buffer");
        DeviceGuard g(c->device);
        HostStage hs(c->stream);
        const size_t bytes = batch * per * 8;
        FHE_TRY(hs.map(where, glwe, bytes, 1));
        FHE_TRY(hs.map(where, ggsw_ntt, (size_t)(k + 1) * level * per * 8, 1));
        FHE_TRY(hs.map(where, out, bytes, 2));
        if (overlaps(out, bytes, glwe, bytes)) return fail(FHE_ERR_INVALID_ARG, "output must not overlap the input");
        FHE_TRY(extprod_composed(c, k + 1, level, base_log, glwe, ggsw_ntt, out, batch));
        return where == FHE_HOST ? hs.finish() : FHE_OK;
    }
    if (where == FHE_HOST && batch) {
        // the key is shared by every ciphertext: upload it once
        DeviceGuard g(c->device);
        const size_t kbytes = (size_t)(k + 1) * level * (k + 1) * c->n * 8;
        void *dk = nullptr;
        HIP_TRY(hipMalloc(&dk, kbytes), "hipMalloc(ggsw)");
        hipError_t e = hipMemcpy(dk, ggsw_ntt, kbytes, hipMemcpyHostToDevice);
        int rc = e != hipSuccess ? hip_fail(e, "hipMemcpy(ggsw)") : FHE_OK;
        if (rc == FHE_OK)
            rc = run_poly_op(c, glwe, nullptr, out, batch, where, per, per, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
                return FHE_NS::launch_extprod(on(c, st), (int)k + 1, (int)level, (int)base_log, d[0], (const u64 *)dk, o, nb);
            });
        (void)hipFree(dk);
        return rc;
    }
    return run_poly_op(c, glwe, nullptr, out, batch, where, per, per, [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
        return FHE_NS::launch_extprod(on(c, st), (int)k + 1, (int)level, (int)base_log, d[0], ggsw_ntt, o, nb);
    });
}

int fhe_decompose_batch(fhe_ctx *c, uint32_t base_log, uint32_t level, const uint64_t *poly, uint64_t *out,
                        size_t npoly, int where) {
    FHE_MULTI(npoly, where, poly, fhe_decompose_batch(c, base_log, level, poly + lo * c->n, out + lo * (size_t)level * c->n, nb, where));
    if (int rc = check_ctx(c)) return rc;
    if (level == 0 || base_log == 0 || base_log > 63 || (u64)base_log * level > 64)
        return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    const FHE_NS::ModConsts m = mod_consts(c->q);
    return run_poly_op(c, poly, nullptr, out, npoly, where, c->n, (size_t)c->n * level,
                       [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) {
                           return FHE_NS::launch_decompose(m, d[0], o, c->n, nb, base_log, level, st);
                       });
}


int fhe_ct_multiply_batch(fhe_ctx *c, const uint64_t *ct1, const uint64_t *ct2, uint64_t *out, size_t batch,
                          int is_ntt, int where) {
    FHE_MULTI(batch, where, ct1, fhe_ct_multiply_batch(c, ct1 + lo * 2 * c->n, ct2 + lo * 2 * c->n, out + lo * 3 * c->n, nb, is_ntt, where));
    FHE_TRY(check_common(c, where, batch));
    if (batch == 0) return FHE_OK;
    if (!ct1 || !ct2 || !out) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, ct1, batch * 2 * n * 8, 1));
    FHE_TRY(hs.map(where, ct2, batch * 2 * n * 8, 1));
    FHE_TRY(hs.map(where, out, batch * 3 * n * 8, 2));
    FHE_TRY(ct_mul_device(c, ct1, ct2, out, batch, is_ntt));
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_relin_key_prepare(fhe_ctx *c, uint32_t level, const uint64_t *rlk, uint64_t *rlk_ntt, int where) {
    FHE_MULTI_ONE(where, rlk, fhe_relin_key_prepare(c, level, rlk, rlk_ntt, where));
    if (int rc = check_ctx(c)) return rc;
    return run_poly_op(c, rlk, nullptr, rlk_ntt, (size_t)2 * level, where, c->n, c->n,
                       [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) { return FHE_NS::launch_fwd(on(c, st), d[0], o, nb, 1); });
}

int fhe_relinearize_batch(fhe_ctx *c, uint32_t base_log, uint32_t level, const uint64_t *ct3,
                          const uint64_t *rlk_ntt, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, ct3, fhe_relinearize_batch(c, base_log, level, ct3 + lo * 3 * c->n, rlk_ntt, out + lo * 2 * c->n, nb, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_relin_decomp(base_log, level));
    if (batch == 0) return FHE_OK;
    if (!ct3 || !out || (level && !rlk_ntt)) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, ct3, batch * 3 * n * 8, 1));
    FHE_TRY(hs.map(where, rlk_ntt, (size_t)level * 2 * n * 8, 1));
    FHE_TRY(hs.map(where, out, batch * 2 * n * 8, 2));
    FHE_TRY(relin_device(c, base_log, level, ct3, rlk_ntt, out, batch));
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_ct_multiply_relin_batch(fhe_ctx *c, uint32_t base_log, uint32_t level, const uint64_t *ct1,
                                const uint64_t *ct2, const uint64_t *rlk_ntt, uint64_t *out, size_t batch,
                                int where) {
    FHE_MULTI(batch, where, ct1, fhe_ct_multiply_relin_batch(c, base_log, level, ct1 + lo * 2 * c->n, ct2 + lo * 2 * c->n, rlk_ntt, out + lo * 2 * c->n, nb, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_relin_decomp(base_log, level));
    if (batch == 0) return FHE_OK;
    if (!ct1 || !ct2 || !out || (level && !rlk_ntt)) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, ct1, batch * 2 * n * 8, 1));
    FHE_TRY(hs.map(where, ct2, batch * 2 * n * 8, 1));
    FHE_TRY(hs.map(where, rlk_ntt, (size_t)level * 2 * n * 8, 1));
    FHE_TRY(hs.map(where, out, batch * 2 * n * 8, 2));
    {
        StreamTemp tmp(c->stream);
        u64 *ct3 = nullptr;
        FHE_TRY(tmp.alloc(batch * 3 * n * 8, ct3));
        FHE_TRY(ct_mul_device(c, ct1, ct2, ct3, batch, 0));
        FHE_TRY(relin_device(c, base_log, level, ct3, rlk_ntt, out, batch));
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

// ---------------------------------------------------------------- EncryptionEngine encrypt / decrypt
int fhe_secret_key_prepare(fhe_ctx *c, const uint64_t *sk, uint64_t *sk_prep, int where) {
    FHE_MULTI_ONE(where, sk, fhe_secret_key_prepare(c, sk, sk_prep, where));
    FHE_TRY(check_common(c, where, 1));
    FHE_TRY(check_fused(c, "encryption"));
    if (!sk || !sk_prep) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, sk, n * 8, 1));
    FHE_TRY(hs.map(where, sk_prep, 2 * n * 8, 2));
    {
        StreamTemp tmp(c->stream);
        u64 *f = nullptr;
        FHE_TRY(tmp.alloc(n * 8, f));
        // row 0: fwd(s) R; row 1: fwd(s) * fwd(s) R (decrypt's sk^2, encryption.cpp:271)
        HIP_TRY(FHE_NS::launch_fwd(c->plan, sk, f, 1, 0), "fwd kernel");
        HIP_TRY(FHE_NS::launch_fwd(c->plan, sk, sk_prep, 1, 1), "fwd kernel");
        HIP_TRY(FHE_NS::launch_modmul(mod_consts(c->q), f, sk_prep, sk_prep + n, n, c->stream), "modmul kernel");
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_public_key_prepare(fhe_ctx *c, const uint64_t *pk, uint64_t *pk_prep, int where) {
    FHE_MULTI_ONE(where, pk, fhe_public_key_prepare(c, pk, pk_prep, where));
    if (int rc = check_ctx(c)) return rc;
    FHE_TRY(check_fused(c, "encryption"));
    return run_poly_op(c, pk, nullptr, pk_prep, 2, where, c->n, c->n,
                       [&](const u64 *const *d, u64 *o, size_t nb, hipStream_t st) { return FHE_NS::launch_fwd(on(c, st), d[0], o, nb, 1); });
}

int fhe_encrypt_batch(fhe_ctx *c, uint64_t t, const uint64_t *pk_prep, const uint64_t *values, const uint64_t *u,
                      const uint64_t *e1, const uint64_t *e2, uint64_t *ct, size_t batch, int where) {
    FHE_MULTI(batch, where, ct, fhe_encrypt_batch(c, t, pk_prep, values + lo * c->n, u + lo * c->n, e1 + lo * c->n,
                                                  e2 + lo * c->n, ct + lo * 2 * c->n, nb, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_fused(c, "encryption"));
    if (batch == 0) return FHE_OK;
    if (!pk_prep || !values || !u || !e1 || !e2 || !ct) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, pk_prep, 2 * n * 8, 1));
    FHE_TRY(hs.map(where, values, batch * n * 8, 1));
    FHE_TRY(hs.map(where, u, batch * n * 8, 1));
    FHE_TRY(hs.map(where, e1, batch * n * 8, 1));
    FHE_TRY(hs.map(where, e2, batch * n * 8, 1));
    FHE_TRY(hs.map(where, ct, batch * 2 * n * 8, 2));
    const u64 *ins[5] = {values, u, e1, e2, pk_prep};
    for (const u64 *x : ins)
        if (overlaps(ct, batch * 2 * n * 8, x, (x == pk_prep ? 2 : batch) * n * 8))
            return fail(FHE_ERR_INVALID_ARG, "output must not overlap the inputs");
    HIP_TRY(FHE_NS::launch_encrypt(c->plan, t, pk_prep, values, u, e1, e2, ct, batch), "encrypt kernel");
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_decrypt_batch(fhe_ctx *c, uint64_t t, const uint64_t *sk_prep, const uint64_t *ct, uint32_t components,
                      int is_ntt, uint64_t *values, uint64_t *phase, uint64_t *max_noise, size_t batch, int where) {
    FHE_MULTI(batch, where, ct, fhe_decrypt_batch(c, t, sk_prep, ct + lo * components * c->n, components, is_ntt,
                                                  values ? values + lo * c->n : nullptr,
                                                  phase ? phase + lo * c->n : nullptr,
                                                  max_noise ? max_noise + lo : nullptr, nb, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_fused(c, "decryption"));
    if (components != 2 && components != 3) return fail(FHE_ERR_INVALID_ARG, "components must be 2 or 3");
    if (batch == 0) return FHE_OK;
    if (!sk_prep || !ct) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, sk_prep, 2 * n * 8, 1));
    FHE_TRY(hs.map(where, ct, batch * components * n * 8, 1));
    FHE_TRY(hs.map(where, values, batch * n * 8, 2));
    FHE_TRY(hs.map(where, phase, batch * n * 8, 2));
    FHE_TRY(hs.map(where, max_noise, batch * 8, 2));
    const size_t ctb = batch * components * n * 8;
    if (overlaps(values, batch * n * 8, ct, ctb) || overlaps(phase, batch * n * 8, ct, ctb))
        return fail(FHE_ERR_INVALID_ARG, "output must not overlap the ciphertexts");
    int rc = FHE_OK;
    {
        StreamTemp tmp(c->stream);
        u64 *ph = phase;
        // degree-2 coefficient-form decryption keeps its partial phase in the phase row
        if (!ph && components == 3 && !is_ntt) rc = tmp.alloc(batch * n * 8, ph);
        if (rc == FHE_OK) {
            hipError_t e = FHE_NS::launch_decrypt(c->plan, t, sk_prep, ct, (int)components, is_ntt, ph,
                                                  phase != nullptr, values, max_noise, batch);
            if (e != hipSuccess) rc = hip_fail(e, "decrypt kernel");
        }
    }
    if (rc != FHE_OK) return rc;
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_add_plain_batch(fhe_ctx *c, uint64_t t, const uint64_t *ct, const uint64_t *values, int is_ntt, uint64_t *out,
                        size_t batch, int where) {
    FHE_MULTI(batch, where, ct, fhe_add_plain_batch(c, t, ct + lo * 2 * c->n, values + lo * c->n, is_ntt,
                                                    out + lo * 2 * c->n, nb, where));
    FHE_TRY(check_common(c, where, batch));
    if (is_ntt) FHE_TRY(check_fused(c, "add_plain on NTT-domain ciphertexts"));
    if (batch == 0) return FHE_OK;
    if (!ct || !values || !out) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, ct, batch * 2 * n * 8, 1));
    FHE_TRY(hs.map(where, values, batch * n * 8, 1));
    FHE_TRY(hs.map(where, out, batch * 2 * n * 8, 2));
    if (is_ntt && overlaps(out, batch * 2 * n * 8, values, batch * n * 8))
        return fail(FHE_ERR_INVALID_ARG, "output must not overlap the plaintext");
    HIP_TRY(FHE_NS::launch_add_plain(c->plan, t, ct, values, is_ntt, out, batch), "add_plain kernel");
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

// ---------------------------------------------------------------- randomness and key material
// (keygen.hip): SecureRandom's draws from a seeded ChaCha20 stream, keys and
// encryptions composed from them and the ring kernels, on the device.
static FHE_NS::ChaChaKey chacha_key(const uint64_t seed[4]) {
    FHE_NS::ChaChaKey k;
    for (int i = 0; i < 4; ++i) {
        k.k[2 * i] = (uint32_t)seed[i];
        k.k[2 * i + 1] = (uint32_t)(seed[i] >> 32);
    }
    return k;
}
static int check_sample(int kind, const uint64_t *seed) {
    if (!seed) return fail(FHE_ERR_INVALID_ARG, "null seed");
    if (kind < FHE_SAMPLE_UNIFORM || kind > FHE_SAMPLE_RAW) return fail(FHE_ERR_INVALID_ARG, "unknown sample kind");
    return FHE_OK;
}

int fhe_sample_batch(fhe_ctx *c, int kind, const uint64_t seed[4], uint64_t stream, double std_dev, uint64_t *out,
                     size_t count, int where) {
    FHE_MULTI_ONE(where, out, fhe_sample_batch(c, kind, seed, stream, std_dev, out, count, where));
    FHE_TRY(check_common(c, where, count));
    FHE_TRY(check_sample(kind, seed));
    if (count == 0) return FHE_OK;
    if (!out) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, out, count * 8, 2));
    HIP_TRY(FHE_NS::launch_sample(kind, chacha_key(seed), stream, c->q, std_dev, out, count, c->stream), "sample kernel");
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_encrypt_sampled_batch(fhe_ctx *c, uint64_t t, const uint64_t *pk_prep, const uint64_t *values,
                              const uint64_t seed[4], uint64_t stream, double std_dev, uint64_t *ct, size_t batch,
                              int where) {
    FHE_MULTI_ONE(where, ct, fhe_encrypt_sampled_batch(c, t, pk_prep, values, seed, stream, std_dev, ct, batch, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_fused(c, "encryption"));
    FHE_TRY(check_sample(FHE_SAMPLE_UNIFORM, seed));
    if (batch == 0) return FHE_OK;
    if (!pk_prep || !values || !ct) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n, cnt = batch * n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, pk_prep, 2 * n * 8, 1));
    FHE_TRY(hs.map(where, values, cnt * 8, 1));
    FHE_TRY(hs.map(where, ct, 2 * cnt * 8, 2));
    if (overlaps(ct, 2 * cnt * 8, values, cnt * 8) || overlaps(ct, 2 * cnt * 8, pk_prep, 2 * n * 8))
        return fail(FHE_ERR_INVALID_ARG, "output must not overlap the inputs");
    {
        // encrypt_internal (encryption.cpp:174-180): u ternary, e1 and e2
        // error polynomials -- streams stream, stream + 1, stream + 2
        StreamTemp tmp(c->stream);
        u64 *u = nullptr;
        FHE_TRY(tmp.alloc(3 * cnt * 8, u));
        const FHE_NS::ChaChaKey key = chacha_key(seed);
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kTernary, key, stream, c->q, 0, u, cnt, c->stream), "sample kernel");
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kGaussian, key, stream + 1, c->q, std_dev, u + cnt, cnt, c->stream),
                "sample kernel");
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kGaussian, key, stream + 2, c->q, std_dev, u + 2 * cnt, cnt, c->stream),
                "sample kernel");
        HIP_TRY(FHE_NS::launch_encrypt(c->plan, t, pk_prep, values, u, u + cnt, u + 2 * cnt, ct, batch),
                "encrypt kernel");
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

// r = a (*) b in the context's transform product, one launch pair
static hipError_t ring_mul(fhe_ctx *c, const u64 *a, const u64 *b, u64 *r, size_t batch) {
    return FHE_NS::launch_polymul(c->plan, a, b, r, batch);
}

int fhe_public_key_generate(fhe_ctx *c, const uint64_t *sk, const uint64_t seed[4], uint64_t stream, double std_dev,
                            uint64_t *pk, int where) {
    FHE_MULTI_ONE(where, pk, fhe_public_key_generate(c, sk, seed, stream, std_dev, pk, where));
    FHE_TRY(check_common(c, where, 1));
    FHE_TRY(check_sample(FHE_SAMPLE_UNIFORM, seed));
    if (!sk || !pk) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    if (overlaps(sk, c->n * 8, pk, 2 * c->n * 8)) return fail(FHE_ERR_INVALID_ARG, "output must not overlap the key");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, sk, n * 8, 1));
    FHE_TRY(hs.map(where, pk, 2 * n * 8, 2));
    {
        // generate_public_key (key_manager.cpp:218-246): a uniform, e error,
        // b = from_ntt(to_ntt(a) (.) to_ntt(s)) + e
        StreamTemp tmp(c->stream);
        u64 *e = nullptr;
        FHE_TRY(tmp.alloc(n * 8, e));
        const FHE_NS::ChaChaKey key = chacha_key(seed);
        const FHE_NS::ModConsts m = mod_consts(c->q);
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kUniform, key, stream, c->q, 0, pk, n, c->stream), "sample kernel");
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kGaussian, key, stream + 1, c->q, std_dev, e, n, c->stream),
                "sample kernel");
        HIP_TRY(ring_mul(c, pk, sk, pk + n, 1), "polymul kernel");
        HIP_TRY(FHE_NS::launch_addsub(m, pk + n, e, pk + n, n, 0, c->stream), "add kernel");
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_eval_key_generate(fhe_ctx *c, const uint64_t *sk, uint32_t base_log, uint32_t level, const uint64_t seed[4],
                          uint64_t stream, double std_dev, uint64_t *rlk, int where) {
    FHE_MULTI_ONE(where, rlk, fhe_eval_key_generate(c, sk, base_log, level, seed, stream, std_dev, rlk, where));
    FHE_TRY(check_common(c, where, 1));
    FHE_TRY(check_sample(FHE_SAMPLE_UNIFORM, seed));
    if (base_log == 0 || base_log > 63) return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    if (level == 0) return FHE_OK;
    if (!sk || !rlk) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, sk, n * 8, 1));
    FHE_TRY(hs.map(where, rlk, (size_t)level * 2 * n * 8, 2));
    {
        // generate_eval_key (key_manager.cpp:252-333): s^2 = s (*) s; level l:
        // a_l uniform (stream + 2l), e_l error (stream + 2l + 1),
        // b_l = a_l (*) s + e_l + s^2 * base^l, with the reference's u64
        // power update power = (power * base) % q
        StreamTemp tmp(c->stream);
        u64 *s2 = nullptr, *e = nullptr, *sc = nullptr;
        FHE_TRY(tmp.alloc(n * 8, s2));
        FHE_TRY(tmp.alloc(n * 8, e));
        FHE_TRY(tmp.alloc(n * 8, sc));
        const FHE_NS::ChaChaKey key = chacha_key(seed);
        const FHE_NS::ModConsts m = mod_consts(c->q);
        HIP_TRY(ring_mul(c, sk, sk, s2, 1), "polymul kernel");
        const u64 base = 1ull << base_log;
        u64 power = 1;
        for (uint32_t l = 0; l < level; ++l) {
            u64 *a = rlk + (size_t)2 * l * n, *b = a + n;
            HIP_TRY(FHE_NS::launch_sample(FHE_NS::kUniform, key, stream + 2 * l, c->q, 0, a, n, c->stream),
                    "sample kernel");
            HIP_TRY(FHE_NS::launch_sample(FHE_NS::kGaussian, key, stream + 2 * l + 1, c->q, std_dev, e, n, c->stream),
                    "sample kernel");
            HIP_TRY(ring_mul(c, a, sk, b, 1), "polymul kernel");
            HIP_TRY(FHE_NS::launch_addsub(m, b, e, b, n, 0, c->stream), "add kernel");
            const u64 sp = power % c->q;  // multiply_scalar's (a * (s % q)) % q
            HIP_TRY(FHE_NS::launch_mul_scalar(m, s2, sp, (u64)(((u128)sp << 64) / c->q), sc, n, c->stream),
                    "scalar kernel");
            HIP_TRY(FHE_NS::launch_addsub(m, b, sc, b, n, 0, c->stream), "add kernel");
            power = (power * base) % c->q;  // u64 product, as the reference
        }
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_ggsw_encrypt_batch(fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level, const int64_t *values,
                           size_t count, const uint64_t *sk, const uint64_t seed[4], uint64_t stream, double std_dev,
                           uint64_t *out, int where) {
    FHE_MULTI_ONE(where, out, fhe_ggsw_encrypt_batch(c, k, base_log, level, values, count, sk, seed, stream, std_dev,
                                                     out, where));
    FHE_TRY(check_common(c, where, count));
    FHE_TRY(check_sample(FHE_SAMPLE_UNIFORM, seed));
    if (k == 0 || k > kMaxGlweDim) return fail(FHE_ERR_UNSUPPORTED, "GLWE dimension k must be between 1 and 16");
    if (level == 0 || base_log == 0 || base_log > 63) return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    if (count == 0) return FHE_OK;
    if (!values || !sk || !out) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t n = c->n, rows = count * (k + 1) * level;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, values, count * 8, 1));
    FHE_TRY(hs.map(where, sk, n * 8, 1));
    FHE_TRY(hs.map(where, out, rows * (k + 1) * n * 8, 2));
    {
        // encrypt_ggsw (bootstrap_engine.cpp:268-306): per row an
        // encrypt_glwe_zero (:190-227) -- masks uniform (stream), error
        // (stream + 1), body = sum_i mask_i (*) s + e -- plus the gadget term
        StreamTemp tmp(c->stream);
        u64 *masks = nullptr, *prod = nullptr, *err = nullptr, *fs = nullptr;
        FHE_TRY(tmp.alloc(rows * k * n * 8, masks));
        FHE_TRY(tmp.alloc(rows * k * n * 8, prod));
        FHE_TRY(tmp.alloc(rows * n * 8, err));
        FHE_TRY(tmp.alloc(n * 8, fs));
        const FHE_NS::ChaChaKey key = chacha_key(seed);
        const FHE_NS::ModConsts m = mod_consts(c->q);
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kUniform, key, stream, c->q, 0, masks, rows * k * n, c->stream),
                "sample kernel");
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kGaussian, key, stream + 1, c->q, std_dev, err, rows * n, c->stream),
                "sample kernel");
        HIP_TRY(FHE_NS::launch_fwd(c->plan, sk, fs, 1, 0), "fwd kernel");
        HIP_TRY(FHE_NS::launch_fwd(c->plan, masks, prod, rows * k, 0), "fwd kernel");
        HIP_TRY(FHE_NS::launch_modmul_bcast(m, prod, fs, prod, (uint32_t)n, rows * k, c->stream), "modmul kernel");
        HIP_TRY(FHE_NS::launch_inv(c->plan, prod, prod, rows * k), "inv kernel");
        HIP_TRY(FHE_NS::launch_ggsw_finish(m, prod, masks, err, values, out, (uint32_t)n, k, level, base_log, count,
                                           c->stream),
                "ggsw kernel");
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_ksk_generate(fhe_ctx *c, uint32_t base_log, uint32_t level, const uint64_t *glwe_sk, uint32_t n_in,
                     const int64_t *lwe_sk, uint32_t lwe_dim, const uint64_t seed[4], uint64_t stream, double std_dev,
                     uint64_t *ksk_a, uint64_t *ksk_b, int where) {
    FHE_MULTI_ONE(where, ksk_b, fhe_ksk_generate(c, base_log, level, glwe_sk, n_in, lwe_sk, lwe_dim, seed, stream,
                                                 std_dev, ksk_a, ksk_b, where));
    FHE_TRY(check_common(c, where, 1));
    FHE_TRY(check_sample(FHE_SAMPLE_UNIFORM, seed));
    if (base_log == 0 || base_log > 63) return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    const size_t entries = (size_t)n_in * level;
    if (entries == 0) return FHE_OK;
    if (!glwe_sk || !ksk_b || (lwe_dim && (!lwe_sk || !ksk_a))) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, glwe_sk, (size_t)n_in * 8, 1));
    FHE_TRY(hs.map(where, lwe_sk, (size_t)lwe_dim * 8, 1));
    FHE_TRY(hs.map(where, ksk_a, entries * lwe_dim * 8, 2));
    FHE_TRY(hs.map(where, ksk_b, entries * 8, 2));
    {
        // generate_key_switch_key (bootstrap_engine.cpp:367-420): entry
        // e = i L + l: a_e uniform (stream), error (stream + 1)
        StreamTemp tmp(c->stream);
        u64 *err = nullptr;
        FHE_TRY(tmp.alloc(entries * 8, err));
        const FHE_NS::ChaChaKey key = chacha_key(seed);
        const FHE_NS::ModConsts m = mod_consts(c->q);
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kUniform, key, stream, c->q, 0, ksk_a, entries * lwe_dim, c->stream),
                "sample kernel");
        HIP_TRY(FHE_NS::launch_sample(FHE_NS::kGaussian, key, stream + 1, c->q, std_dev > 0 ? std_dev : 3.2, err,
                                      entries, c->stream),
                "sample kernel");
        HIP_TRY(FHE_NS::launch_ksk_body(m, glwe_sk, lwe_sk, ksk_a, err, ksk_b, n_in, level, base_log, lwe_dim,
                                        c->stream),
                "ksk kernel");
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_lwe_decrypt_batch(uint64_t q, uint64_t t, const int64_t *sk, uint32_t dim, const uint64_t *lwe_a,
                          const uint64_t *lwe_b, uint64_t *values, uint64_t *phase, size_t batch, int where, int device,
                          void *stream) {
    if (q < 2) return fail(FHE_ERR_ZERO_MODULUS, "LWE modulus must be >= 2");
    if (where != FHE_HOST && where != FHE_DEVICE) return fail(FHE_ERR_INVALID_ARG, "where must be FHE_HOST or FHE_DEVICE");
    if (batch == 0) return FHE_OK;
    if (!lwe_b || (dim && (!sk || !lwe_a))) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(FHE_ERR_DEVICE, "no HIP device available (the backend has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(FHE_ERR_INVALID_ARG, "device ordinal out of range");
    DeviceGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    HostStage hs(s);
    FHE_TRY(hs.map(where, sk, (size_t)dim * 8, 1));
    FHE_TRY(hs.map(where, lwe_a, batch * dim * 8, 1));
    FHE_TRY(hs.map(where, lwe_b, batch * 8, 1));
    FHE_TRY(hs.map(where, values, batch * 8, 2));
    FHE_TRY(hs.map(where, phase, batch * 8, 2));
    HIP_TRY(FHE_NS::launch_lwe_decrypt(q, t, sk, dim, lwe_a, lwe_b, values, phase, batch, s), "lwe decrypt kernel");
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

// ---------------------------------------------------------------- RNS ring
struct fhe_rns_ctx {
    std::vector<fhe_ctx *> limbs;
};

int fhe_rns_ctx_create(uint32_t n, const uint64_t *moduli, uint32_t count, int mode, int device, fhe_rns_ctx **out) {
    if (!out) return fail(FHE_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    // PolynomialRing(degree, moduli) (polynomial_ring.cpp:228-230)
    if (count == 0 || !moduli) return fail(FHE_ERR_INVALID_ARG, "At least one modulus required");
    fhe_rns_ctx *r = new fhe_rns_ctx();
    for (uint32_t i = 0; i < count; ++i) {
        fhe_ctx *c = nullptr;
        const int rc = fhe_ctx_create(n, moduli[i], mode, device, &c);
        if (rc != FHE_OK) {
            const std::string msg = g_err;
            fhe_rns_ctx_destroy(r);
            return fail(rc, msg);
        }
        if (!r->limbs.empty()) fhe_ctx_set_stream(c, r->limbs[0]->stream);  // one stream: limbs run in order
        r->limbs.push_back(c);
    }
    *out = r;
    return FHE_OK;
}

void fhe_rns_ctx_destroy(fhe_rns_ctx *r) {
    if (!r) return;
    for (auto it = r->limbs.rbegin(); it != r->limbs.rend(); ++it) fhe_ctx_destroy(*it);
    delete r;
}

int fhe_rns_ctx_limb(const fhe_rns_ctx *r, uint32_t i, fhe_ctx **out) {
    if (!r || !out) return fail(FHE_ERR_INVALID_ARG, "null argument");
    if (i >= r->limbs.size()) return fail(FHE_ERR_INVALID_ARG, "limb index out of range");
    *out = r->limbs[i];
    return FHE_OK;
}

extern "C++" {
template <typename F>
static int rns_each(fhe_rns_ctx *r, size_t batch, F &&fn) {
    if (!r) return fail(FHE_ERR_INVALID_ARG, "null context");
    for (size_t i = 0; i < r->limbs.size(); ++i)
        if (int rc = fn(r->limbs[i], i * batch * r->limbs[i]->n)) return rc;
    return FHE_OK;
}
}
#define RNS_UNARY(NAME, FN)                                                                              \
    int NAME(fhe_rns_ctx *r, const uint64_t *in, uint64_t *out, size_t batch, int where) {              \
        if (batch && (!in || !out)) return fail(FHE_ERR_INVALID_ARG, "null buffer");                     \
        return rns_each(r, batch, [&](fhe_ctx *c, size_t off) { return FN(c, in + off, out + off, batch, where); }); \
    }
#define RNS_BINARY(NAME, FN)                                                                             \
    int NAME(fhe_rns_ctx *r, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t batch, int where) { \
        if (batch && (!a || !b || !out)) return fail(FHE_ERR_INVALID_ARG, "null buffer");                \
        return rns_each(r, batch,                                                                        \
                        [&](fhe_ctx *c, size_t off) { return FN(c, a + off, b + off, out + off, batch, where); }); \
    }
RNS_UNARY(fhe_rns_ntt_fwd_batch, fhe_ntt_fwd_batch)
RNS_UNARY(fhe_rns_ntt_inv_batch, fhe_ntt_inv_batch)
RNS_BINARY(fhe_rns_polymul_batch, fhe_polymul_batch)
RNS_BINARY(fhe_rns_pointwise_batch, fhe_pointwise_batch)
RNS_BINARY(fhe_rns_add_batch, fhe_poly_add_batch)
RNS_BINARY(fhe_rns_sub_batch, fhe_poly_sub_batch)
#undef RNS_UNARY
#undef RNS_BINARY

static int check_tfhe(const fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level) {
    FHE_TRY(check_fused(c, "external product"));
    if (k != 1) return fail(FHE_ERR_UNSUPPORTED, "external product implemented for GLWE dimension k = 1");
    if (level == 0 || base_log == 0 || base_log > 63 || (u64)base_log * level > 64)
        return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    return FHE_OK;
}

// Blind rotation / bootstrap: the fused kernels take k = 1 and N <= 16384;
// other shapes (k = 2..16, N = 32768 / 65536) run composed step by step.
static int check_br(const fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level) {
    return fused_tfhe(c, k) ? check_tfhe(c, k, base_log, level) : check_decomp(c, k, base_log, level);
}

// blind_rotate (bootstrap_engine.cpp:547-577) for the shapes without a fused
// CMux: X^-round(b 2N/q) acc, then per LWE coefficient d = X^r cur - cur,
// ExtProd(bsk_i, d) composed (decompose, batched transforms, key MAC,
// inverse), cur + product -- ping-ponging two device buffers; skipped steps
// (r == 0) copy cur through.  Every temporary (one digit buffer for all
// steps) is allocated once, stream-ordered -- or carved from `scratch` (the
// context's persistent buffer of blind_rotate_scratch_bytes, when the call
// is captured into a hipGraph); nothing synchronises the host.
static size_t blind_rotate_scratch_bytes(const fhe_ctx *c, uint32_t k, uint32_t level, size_t batch) {
    return 3 * batch * (k + 1) * c->n * 8 + extprod_digit_words(c, k + 1, level, batch) * 8;
}
static int blind_rotate_composed(fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level, uint32_t lwe_dim,
                                 const u64 *lwe_a, const u64 *lwe_b, uint64_t lwe_q, const u64 *bsk_ntt, u64 *acc,
                                 size_t batch, u64 *scratch = nullptr) {
    const size_t n = c->n, k1 = k + 1, bytes = batch * k1 * n * 8;
    const size_t ggsw_words = k1 * level * k1 * n;
    const FHE_NS::ModConsts m = mod_consts(c->q);
    StreamTemp tmp(c->stream);
    u64 *cur = nullptr, *d = nullptr, *ep = nullptr, *dig = nullptr;
    if (scratch) {
        cur = scratch;
        d = cur + bytes / 8;
        ep = d + bytes / 8;
        dig = ep + bytes / 8;
    } else {
        FHE_TRY(tmp.alloc(bytes, cur));
        FHE_TRY(tmp.alloc(bytes, d));
        FHE_TRY(tmp.alloc(bytes, ep));
        FHE_TRY(tmp.alloc(extprod_digit_words(c, (uint32_t)k1, level, batch) * 8, dig));
    }
    HIP_TRY(FHE_NS::launch_rotate(m, acc, cur, (uint32_t)n, (uint32_t)k1, batch, nullptr, lwe_b, lwe_q, c->stream),
            "rotate kernel");
    for (uint32_t i = 0; i < lwe_dim; ++i) {
        HIP_TRY(FHE_NS::launch_br_diff(m, cur, d, (uint32_t)n, (uint32_t)k1, batch, lwe_a, lwe_dim, i, lwe_q, c->stream),
                "blind rotate step kernel");
        FHE_TRY(extprod_composed(c, (uint32_t)k1, level, base_log, d, bsk_ntt + ggsw_words * i, ep, batch, dig));
        HIP_TRY(FHE_NS::launch_br_add(m, cur, ep, d, (uint32_t)n, (uint32_t)k1, batch, lwe_a, lwe_dim, i, lwe_q,
                                      c->stream),
                "blind rotate step kernel");
        std::swap(cur, d);
    }
    HIP_TRY(hipMemcpyAsync(acc, cur, bytes, hipMemcpyDeviceToDevice, c->stream), "hipMemcpyAsync");
    return FHE_OK;
}

int fhe_glwe_rotate_batch(fhe_ctx *c, uint32_t k, const int32_t *rot, const uint64_t *glwe, uint64_t *out,
                          size_t batch, int where) {
    FHE_MULTI(batch, where, glwe, fhe_glwe_rotate_batch(c, k, rot + lo, glwe + lo * (k + 1) * c->n, out + lo * (k + 1) * c->n, nb, where));
    FHE_TRY(check_common(c, where, batch));
    if (batch == 0) return FHE_OK;
    if (!rot || !glwe || !out) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const size_t bytes = batch * (k + 1) * c->n * 8;
    DeviceGuard g(c->device);
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, rot, batch * sizeof(int32_t), 1));
    FHE_TRY(hs.map(where, glwe, bytes, 1));
    FHE_TRY(hs.map(where, out, bytes, 2));
    if (overlaps(glwe, bytes, out, bytes)) return fail(FHE_ERR_INVALID_ARG, "output must not overlap the input");
    HIP_TRY(FHE_NS::launch_rotate(mod_consts(c->q), glwe, out, c->n, k + 1, batch, rot, nullptr, 0, c->stream),
            "rotate kernel");
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_cmux_batch(fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level, const uint64_t *ggsw_ntt,
                   const uint64_t *ct0, const uint64_t *ct1, uint64_t *out, size_t batch, int where) {
    FHE_MULTI(batch, where, ct0, fhe_cmux_batch(c, k, base_log, level, ggsw_ntt, ct0 + lo * (k + 1) * c->n, ct1 + lo * (k + 1) * c->n, out + lo * (k + 1) * c->n, nb, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_decomp(c, k, base_log, level));
    if (batch == 0) return FHE_OK;
    if (!ggsw_ntt || !ct0 || !ct1 || !out) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const size_t n = c->n, bytes = batch * (k + 1) * n * 8;
    DeviceGuard g(c->device);
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, ggsw_ntt, (size_t)(k + 1) * level * (k + 1) * n * 8, 1));
    FHE_TRY(hs.map(where, ct0, bytes, 1));
    FHE_TRY(hs.map(where, ct1, bytes, 1));
    FHE_TRY(hs.map(where, out, bytes, 2));
    if (overlaps(out, bytes, ct0, bytes) || overlaps(out, bytes, ct1, bytes))
        return fail(FHE_ERR_INVALID_ARG, "output must not overlap the inputs");
    if (fused_tfhe(c, k)) {
        HIP_TRY(FHE_NS::launch_cmux(c->plan, (int)k + 1, (int)level, (int)base_log, ggsw_ntt, ct0, ct1, out, batch),
                "cmux kernel");
    } else {  // ct0 + ExtProd(ct1 - ct0) composed (cmux :520-540)
        const FHE_NS::ModConsts m = mod_consts(c->q);
        const size_t cnt = batch * (k + 1) * n;
        HIP_TRY(FHE_NS::launch_addsub(m, ct1, ct0, out, cnt, 1, c->stream), "sub kernel");
        StreamTemp st(c->stream);
        u64 *tmp = nullptr;
        FHE_TRY(st.alloc(bytes, tmp));
        FHE_TRY(extprod_composed(c, k + 1, level, base_log, out, ggsw_ntt, tmp, batch));
        HIP_TRY(FHE_NS::launch_addsub(m, tmp, ct0, out, cnt, 0, c->stream), "add kernel");
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

// Largest batch the single-launch blind rotation takes.  Measured on MI355X
// (tfhe-128-fast shape, q = 62-bit prime): batch 64 6.8 ms vs 39.2 ms per-step
// launches, batch 8192 103 ms vs 184 ms -- it wins at every size, so the
// per-step path only serves unsupported shapes and
// FHE_BR_PERSIST_MAX=0.
constexpr size_t kBrPersistMax = ~(size_t)0;

int fhe_blind_rotate_batch(fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level, uint32_t lwe_dim,
                           const uint64_t *lwe_a, const uint64_t *lwe_b, uint64_t lwe_q, const uint64_t *bsk_ntt,
                           uint64_t *acc, size_t batch, int where) {
    FHE_MULTI(batch, where, acc, fhe_blind_rotate_batch(c, k, base_log, level, lwe_dim, lwe_a + lo * lwe_dim, lwe_b + lo, lwe_q, bsk_ntt, acc + lo * (k + 1) * c->n, nb, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_br(c, k, base_log, level));
    if (lwe_q == 0) return fail(FHE_ERR_ZERO_MODULUS, "LWE modulus must be non-zero");
    if (batch == 0) return FHE_OK;
    if (!lwe_b || !acc || (lwe_dim && (!lwe_a || !bsk_ntt))) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const size_t n = c->n, bytes = batch * (k + 1) * n * 8;
    const size_t ggsw_words = (size_t)(k + 1) * level * (k + 1) * n;
    DeviceGuard g(c->device);
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, lwe_a, batch * lwe_dim * 8, 1));
    FHE_TRY(hs.map(where, lwe_b, batch * 8, 1));
    FHE_TRY(hs.map(where, bsk_ntt, ggsw_words * lwe_dim * 8, 1));
    FHE_TRY(hs.map(where, acc, bytes, 3));
    static const bool no_graph = std::getenv("FHE_NO_GRAPH") && std::getenv("FHE_NO_GRAPH")[0] == '1';
    // The whole loop as one launch with the accumulators in LDS
    // (ntt_br.hip; k = 1 and k = 2 at small N); FHE_BR_PERSIST_MAX caps the
    // batch it takes (0 = never).
    const char *pm = std::getenv("FHE_BR_PERSIST_MAX");
    const size_t persist_max = pm ? (size_t)std::strtoull(pm, nullptr, 10) : kBrPersistMax;
    if (lwe_dim > 0 && batch <= persist_max && (int)c->logn <= FHE_NS::kMaxFusedLogN &&
        FHE_NS::br_persist_supported(c->plan, (int)k + 1)) {
        HIP_TRY(FHE_NS::launch_br_persist(c->plan, (int)k + 1, (int)level, (int)base_log, acc, bsk_ntt, lwe_a, lwe_b,
                                          lwe_dim, lwe_q, batch),
                "blind rotate kernel");
        return where == FHE_HOST ? hs.finish() : FHE_OK;
    }
    const bool composed = !fused_tfhe(c, k);
    // composed steps (k > 1, N > 16384, q >= 2^62): six launches per CMux;
    // device-resident calls with fused transforms are captured into the
    // context's hipGraph below (persistent scratch, no stream allocations)
    const bool composed_graph = composed && !no_graph && where == FHE_DEVICE && c->stream != nullptr && lwe_dim > 0 &&
                                (int)c->logn <= FHE_NS::kMaxFusedLogN;
    if (composed && !composed_graph) {
        FHE_TRY(blind_rotate_composed(c, k, base_log, level, lwe_dim, lwe_a, lwe_b, lwe_q, bsk_ntt, acc, batch));
        return where == FHE_HOST ? hs.finish() : FHE_OK;
    }
    std::lock_guard<std::mutex> lk(c->br_mu);
    const size_t need = composed ? blind_rotate_scratch_bytes(c, k, level, batch) : bytes;
    if (c->br_tmp_bytes < need) {
        if (c->br.exec) { (void)hipGraphExecDestroy(c->br.exec); c->br.exec = nullptr; }
        if (c->br.graph) { (void)hipGraphDestroy(c->br.graph); c->br.graph = nullptr; }
        if (c->br_tmp) (void)hipFree(c->br_tmp);
        c->br_tmp = nullptr;
        c->br_tmp_bytes = 0;
        HIP_TRY(hipMalloc(&c->br_tmp, need), "hipMalloc(blind rotate)");
        c->br_tmp_bytes = need;
    }
    u64 *tmp = (u64 *)c->br_tmp;
    // br_tmp may still be in use by a call enqueued on another stream
    if (c->br_done && c->br_done_stream != c->stream)
        HIP_TRY(hipStreamWaitEvent(c->stream, c->br_done, 0), "hipStreamWaitEvent");
    // acc <- X^-round(b 2N / q) acc, into tmp; then lwe_dim CMux steps
    // ping-ponging tmp <-> acc; the result is copied back into acc if it
    // ended in tmp.
    auto enqueue = [&]() -> hipError_t {
        if (composed)
            return blind_rotate_composed(c, k, base_log, level, lwe_dim, lwe_a, lwe_b, lwe_q, bsk_ntt, acc, batch, tmp)
                           == FHE_OK ? hipSuccess : hipErrorLaunchFailure;
        hipError_t e = FHE_NS::launch_rotate(mod_consts(c->q), acc, tmp, c->n, k + 1, batch, nullptr, lwe_b, lwe_q,
                                             c->stream);
        u64 *cur = tmp, *nxt = acc;
        for (uint32_t i = 0; e == hipSuccess && i < lwe_dim; ++i) {
            e = FHE_NS::launch_cmux_rotate(c->plan, (int)k + 1, (int)level, (int)base_log, cur,
                                           bsk_ntt + ggsw_words * i, nxt, batch, lwe_a, lwe_dim, i, lwe_q);
            std::swap(cur, nxt);
        }
        if (e == hipSuccess && cur != acc) e = hipMemcpyAsync(acc, cur, bytes, hipMemcpyDeviceToDevice, c->stream);
        return e;
    };
    // Device-resident calls: the lwe_dim + 2 launches are captured once into
    // a hipGraph and replayed while (buffers, shape, stream) are unchanged.
    // The legacy null stream cannot be captured; FHE_NO_GRAPH=1 disables
    // graphs.
    fhe_ctx::BrGraph &G = c->br;
    const bool same = G.exec && G.acc == acc && G.lwe_a == lwe_a && G.lwe_b == lwe_b && G.bsk == bsk_ntt &&
                      G.batch == batch && G.k == k && G.base_log == base_log && G.level == level &&
                      G.dim == lwe_dim && G.lwe_q == lwe_q && G.stream == c->stream;
    hipError_t e = hipSuccess;
    if (!no_graph && where == FHE_DEVICE && c->stream != nullptr && lwe_dim > 0) {
        if (!same) {
            if (G.exec) (void)hipGraphExecDestroy(G.exec);
            if (G.graph) (void)hipGraphDestroy(G.graph);
            G = fhe_ctx::BrGraph{};
            hipGraph_t graph = nullptr;
            hipGraphExec_t exec = nullptr;
            e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed);
            if (e == hipSuccess) {
                hipError_t e1 = enqueue();
                hipError_t e2 = hipStreamEndCapture(c->stream, &graph);
                e = e1 != hipSuccess ? e1 : e2;
            }
            if (e == hipSuccess) e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
            if (e == hipSuccess) {
                G.acc = acc; G.lwe_a = lwe_a; G.lwe_b = lwe_b; G.bsk = bsk_ntt; G.batch = batch; G.k = k;
                G.base_log = base_log; G.level = level; G.dim = lwe_dim; G.lwe_q = lwe_q; G.stream = c->stream;
                G.graph = graph; G.exec = exec;
            } else {
                if (graph) (void)hipGraphDestroy(graph);
                (void)hipGetLastError();
            }
        }
        e = G.exec ? hipGraphLaunch(G.exec, c->stream) : enqueue();
    } else {
        e = enqueue();
    }
    if (e != hipSuccess) return hip_fail(e, "blind rotate");
    if (!c->br_done) HIP_TRY(hipEventCreateWithFlags(&c->br_done, hipEventDisableTiming), "hipEventCreate");
    HIP_TRY(hipEventRecord(c->br_done, c->stream), "hipEventRecord");
    c->br_done_stream = c->stream;
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_sample_extract_batch(fhe_ctx *c, uint32_t k, const uint64_t *glwe, uint64_t *lwe_a, uint64_t *lwe_b,
                             size_t batch, int where) {
    FHE_MULTI(batch, where, glwe, fhe_sample_extract_batch(c, k, glwe + lo * (k + 1) * c->n, lwe_a + lo * k * c->n, lwe_b + lo, nb, where));
    FHE_TRY(check_common(c, where, batch));
    if (batch == 0) return FHE_OK;
    if (!glwe || !lwe_b || (k && !lwe_a)) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    const size_t n = c->n;
    DeviceGuard g(c->device);
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, glwe, batch * (k + 1) * n * 8, 1));
    FHE_TRY(hs.map(where, lwe_a, batch * k * n * 8, 2));
    FHE_TRY(hs.map(where, lwe_b, batch * 8, 2));
    if (k == 0) {  // body only
        HIP_TRY(hipMemcpy2DAsync(lwe_b, 8, glwe, n * 8, 8, batch, hipMemcpyDeviceToDevice, c->stream), "hipMemcpy2D");
    } else {
        HIP_TRY(FHE_NS::launch_sample_extract(mod_consts(c->q), glwe, lwe_a, lwe_b, c->n, k, batch, c->stream),
                "sample extract kernel");
    }
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_key_switch_batch(uint64_t q, uint32_t base_log, uint32_t level, uint32_t in_dim, uint32_t out_dim,
                         const uint64_t *ksk_a, const uint64_t *ksk_b, const uint64_t *lwe_a, const uint64_t *lwe_b,
                         uint64_t *out_a, uint64_t *out_b, size_t batch, int where, int device, void *stream) {
    if (q < 2) return fail(FHE_ERR_ZERO_MODULUS, "key switch modulus must be >= 2");
    if (where != FHE_HOST && where != FHE_DEVICE) return fail(FHE_ERR_INVALID_ARG, "where must be FHE_HOST or FHE_DEVICE");
    if (base_log == 0 || base_log > 63 || (level > 0 && (u64)(level - 1) * base_log >= 64))
        return fail(FHE_ERR_INVALID_ARG, "invalid decomposition (base_log, level)");
    if (batch == 0) return FHE_OK;
    const size_t entries = (size_t)in_dim * level;
    if (!lwe_b || !out_b || (entries && (!lwe_a || !ksk_b)) || (entries && out_dim && !ksk_a) || (out_dim && !out_a))
        return fail(FHE_ERR_INVALID_ARG, "null buffer");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(FHE_ERR_DEVICE, "no HIP device available (the backend has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(FHE_ERR_INVALID_ARG, "device ordinal out of range");
    DeviceGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    HostStage hs(s);
    FHE_TRY(hs.map(where, ksk_a, entries * out_dim * 8, 1));
    FHE_TRY(hs.map(where, ksk_b, entries * 8, 1));
    FHE_TRY(hs.map(where, lwe_a, batch * in_dim * 8, 1));
    FHE_TRY(hs.map(where, lwe_b, batch * 8, 1));
    FHE_TRY(hs.map(where, out_a, batch * out_dim * 8, 2));
    FHE_TRY(hs.map(where, out_b, batch * 8, 2));
    HIP_TRY(FHE_NS::launch_key_switch(mod_consts(q), base_log, level, in_dim, out_dim, ksk_a, ksk_b, lwe_a, lwe_b, out_a,
                                      out_b, batch, s),
            "key switch kernel");
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

int fhe_bootstrap_batch(fhe_ctx *c, uint32_t k, uint32_t base_log, uint32_t level, uint32_t lwe_dim,
                        const uint64_t *lwe_a, const uint64_t *lwe_b, uint64_t lwe_q, const uint64_t *bsk_ntt,
                        const uint64_t *test_poly, uint32_t ks_base_log, uint32_t ks_level, uint32_t out_dim,
                        const uint64_t *ksk_a, const uint64_t *ksk_b, uint64_t *out_a, uint64_t *out_b, size_t batch,
                        int where) {
    FHE_MULTI(batch, where, lwe_b, fhe_bootstrap_batch(c, k, base_log, level, lwe_dim, lwe_a + lo * lwe_dim, lwe_b + lo,
                                                       lwe_q, bsk_ntt, test_poly, ks_base_log, ks_level, out_dim,
                                                       ksk_a, ksk_b, out_a + lo * out_dim, out_b + lo, nb, where));
    FHE_TRY(check_common(c, where, batch));
    FHE_TRY(check_br(c, k, base_log, level));
    if (lwe_q == 0) return fail(FHE_ERR_ZERO_MODULUS, "LWE modulus must be non-zero");
    if (ks_base_log == 0 || ks_base_log > 63 || (ks_level > 0 && (u64)(ks_level - 1) * ks_base_log >= 64))
        return fail(FHE_ERR_INVALID_ARG, "invalid key-switch decomposition (base_log, level)");
    if (batch == 0) return FHE_OK;
    const size_t n = c->n, in_dim = (size_t)k * n, entries = in_dim * ks_level;
    if (!lwe_b || !test_poly || !out_b || (lwe_dim && (!lwe_a || !bsk_ntt)) || (entries && !ksk_b) ||
        (entries && out_dim && !ksk_a) || (out_dim && !out_a))
        return fail(FHE_ERR_INVALID_ARG, "null buffer");
    DeviceGuard g(c->device);
    const size_t ggsw_words = (size_t)(k + 1) * level * (k + 1) * n;
    HostStage hs(c->stream);
    FHE_TRY(hs.map(where, lwe_a, batch * lwe_dim * 8, 1));
    FHE_TRY(hs.map(where, lwe_b, batch * 8, 1));
    FHE_TRY(hs.map(where, bsk_ntt, ggsw_words * lwe_dim * 8, 1));
    FHE_TRY(hs.map(where, test_poly, n * 8, 1));
    FHE_TRY(hs.map(where, ksk_a, entries * out_dim * 8, 1));
    FHE_TRY(hs.map(where, ksk_b, entries * 8, 1));
    FHE_TRY(hs.map(where, out_a, batch * out_dim * 8, 2));
    FHE_TRY(hs.map(where, out_b, batch * 8, 2));
    int rc = FHE_OK;
    {
        // bootstrap_with_test_poly (bootstrap_engine.cpp:684-708): acc =
        // (0, .., 0, test_poly) -> blind_rotate -> sample_extract ->
        // key_switch (GLWE modulus), all on the context stream
        StreamTemp tmp(c->stream);
        u64 *acc = nullptr, *ea = nullptr, *eb = nullptr;
        FHE_TRY(tmp.alloc(batch * (k + 1) * n * 8, acc));
        FHE_TRY(tmp.alloc(batch * in_dim * 8, ea));
        FHE_TRY(tmp.alloc(batch * 8, eb));
        HIP_TRY(FHE_NS::launch_glwe_init(test_poly, acc, (uint32_t)n, k + 1, batch, c->stream), "glwe init kernel");
        rc = fhe_blind_rotate_batch(c, k, base_log, level, lwe_dim, lwe_a, lwe_b, lwe_q, bsk_ntt, acc, batch,
                                    FHE_DEVICE);
        if (rc == FHE_OK) {
            hipError_t e = FHE_NS::launch_sample_extract(mod_consts(c->q), acc, ea, eb, (uint32_t)n, k, batch, c->stream);
            if (e == hipSuccess)
                e = FHE_NS::launch_key_switch(mod_consts(c->q), ks_base_log, ks_level, (uint32_t)in_dim, out_dim, ksk_a,
                                              ksk_b, ea, eb, out_a, out_b, batch, c->stream);
            if (e != hipSuccess) rc = hip_fail(e, "bootstrap");
        }
    }
    if (rc != FHE_OK) return rc;
    return where == FHE_HOST ? hs.finish() : FHE_OK;
}

// ---------------------------------------------------------------- context-free kernels
static int run_flat(int device, void *stream, int where, const u64 *a, const u64 *b, u64 *c, size_t count,
                    size_t width, hipError_t (*fn)(const void *, const u64 *, const u64 *, u64 *, size_t, hipStream_t),
                    const void *arg) {
    if (where != FHE_HOST && where != FHE_DEVICE) return fail(FHE_ERR_INVALID_ARG, "where must be FHE_HOST or FHE_DEVICE");
    if (count == 0) return FHE_OK;
    if (!a || !b || !c) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(FHE_ERR_DEVICE, "no HIP device available (the backend has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(FHE_ERR_INVALID_ARG, "device ordinal out of range");
    DeviceGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    if (where == FHE_DEVICE) {
        HIP_TRY(fn(arg, a, b, c, count, s), "kernel launch");
        return FHE_OK;
    }
    const size_t bytes = count * width * 8;
    void *da = nullptr, *db = nullptr, *dc = nullptr;
    hipError_t e = hipMalloc(&da, bytes);
    if (e == hipSuccess) e = hipMalloc(&db, bytes);
    if (e == hipSuccess) e = hipMalloc(&dc, bytes);
    if (e == hipSuccess) e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = fn(arg, (const u64 *)da, (const u64 *)db, (u64 *)dc, count, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipMemcpy(c, dc, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(dc);
    if (e != hipSuccess) return hip_fail(e, "modular kernel");
    return FHE_OK;
}

static hipError_t modmul_thunk(const void *arg, const u64 *a, const u64 *b, u64 *c, size_t n, hipStream_t s) {
    return FHE_NS::launch_modmul(*(const FHE_NS::ModConsts *)arg, a, b, c, n, s);
}
int fhe_modmul_batch(uint64_t q, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t count, int where,
                     int device, void *stream) {
    if (q == 0) return fail(FHE_ERR_ZERO_MODULUS, "Modulus must be non-zero for Barrett reduction");
    const FHE_NS::ModConsts m = mod_consts(q);
    return run_flat(device, stream, where, a, b, c, count, 1, modmul_thunk, &m);
}

// MultiLimbMontgomeryConstants (modular_arithmetic.cpp:471-486) with 2 limbs,
// including multi_limb_mod_proper's truncated shifted modulus and strict
// comparison (:361-429), so the constants match the reference bit for bit.
static void ml_reduce(const u64 *a, size_t asz, const u64 *mod, u64 *out) {
    const size_t nl = 2, rs = std::max(asz, nl);
    u64 rem[4] = {0, 0, 0, 0};
    std::memcpy(rem, a, asz * 8);
    if (asz <= nl) {
        const u64 hi = asz > 1 ? a[1] : 0;
        if (hi < mod[1] || (hi == mod[1] && a[0] < mod[0])) {
            out[0] = a[0];
            out[1] = hi;
            return;
        }
    }
    for (int bp = (int)(rs * 64) - 1; bp >= 0; --bp) {
        const size_t ls = (size_t)bp / 64, bs = (size_t)bp % 64;
        u64 sh[4] = {0, 0, 0, 0};
        for (size_t i = 0; i < nl && i + ls < rs; ++i) {
            if (bs == 0) sh[i + ls] = mod[i];
            else {
                sh[i + ls] |= mod[i] << bs;
                if (i + ls + 1 < rs) sh[i + ls + 1] = mod[i] >> (64 - bs);
            }
        }
        bool can = false;
        for (int i = (int)rs - 1; i >= 0; --i) {
            if (rem[i] > sh[i]) { can = true; break; }
            if (rem[i] < sh[i]) break;
        }
        if (can) {
            u64 borrow = 0;
            for (size_t i = 0; i < rs; ++i) {
                const u64 r = rem[i], s = sh[i];
                rem[i] = r - s - borrow;
                borrow = (r < s + borrow) ? 1 : 0;
            }
        }
    }
    out[0] = rem[0];
    out[1] = rem[1];
}

int fhe_ml_constants(const uint64_t q[2], uint64_t out[7]) {
    if (!q || !out) return fail(FHE_ERR_INVALID_ARG, "null argument");
    if ((q[0] == 0 && q[1] == 0) || (q[0] & 1) == 0)
        return fail(FHE_ERR_MONT_MODULUS, "Modulus must be odd and non-zero for Montgomery arithmetic");
    const u64 rl[3] = {0, 0, 1};
    u64 r[2], r2[2];
    ml_reduce(rl, 3, q, r);
    u64 prod[4] = {0, 0, 0, 0};
    for (int i = 0; i < 2; ++i) {
        u64 carry = 0;
        for (int j = 0; j < 2; ++j) {
            u128 p = (u128)r[i] * r[j] + prod[i + j] + carry;
            prod[i + j] = (u64)p;
            carry = (u64)(p >> 64);
        }
        prod[i + 2] = carry;
    }
    ml_reduce(prod, 4, q, r2);
    u64 x = q[0];
    for (int i = 0; i < 5; ++i) x = x * (2 - q[0] * x);
    out[0] = q[0]; out[1] = q[1]; out[2] = r[0]; out[3] = r[1]; out[4] = r2[0]; out[5] = r2[1];
    out[6] = (~x) + 1;
    return FHE_OK;
}

static hipError_t ml_thunk(const void *arg, const u64 *a, const u64 *b, u64 *c, size_t n, hipStream_t s) {
    return FHE_NS::launch_ml_montmul((const u64 *)arg, a, b, c, n, s);
}
int fhe_ml_montmul_batch(const uint64_t q[2], const uint64_t *a, const uint64_t *b, uint64_t *c, size_t count,
                         int where, int device, void *stream) {
    u64 consts[7];
    if (int rc = fhe_ml_constants(q, consts)) return rc;
    return run_flat(device, stream, where, a, b, c, count, 2, ml_thunk, consts);
}

// ---------------------------------------------------------------- N-API ModularArithmetic (scalar)
// modular_arithmetic.cpp:8-31 extended Euclid with unsigned a, m and signed
// x0/x1 (m0 = (int64)m).  A zero divisor (gcd(q, 2^64-1) > 1) traps on x86
// in the reference; here it takes the AArch64 result (x/0 = 0, x%0 = x), the
// platform the reference ships for.
static u64 compat_mod_inverse(u64 a, u64 m) {
    if (m == 0) return 0;
    const int64_t m0 = (int64_t)m;
    int64_t x0 = 0, x1 = 1;
    if (m == 1) return 0;
    while (a > 1) {
        const int64_t qq = (int64_t)(m == 0 ? 0 : a / m);
        int64_t t = (int64_t)m;
        m = m == 0 ? a : a % m;
        a = (u64)t;
        t = x0;
        x0 = (int64_t)((u64)x1 - (u64)qq * (u64)x0);
        x1 = t;
    }
    if (x1 < 0) x1 = (int64_t)((u64)x1 + (u64)m0);
    return (u64)x1;
}

int fhe_mont_constants_compat(uint64_t q, uint64_t k[4]) {
    if (!k) return fail(FHE_ERR_INVALID_ARG, "null argument");
    if (q == 0 || (q & 1) == 0)
        return fail(FHE_ERR_MONT_MODULUS, "Modulus must be odd and non-zero for Montgomery arithmetic");
    const u64 rq = (u64)((((u128)1) << 64) % q);
    k[0] = q;
    k[1] = rq;
    k[2] = (u64)((u128)rq * rq % q);
    k[3] = (~compat_mod_inverse(q, UINT64_MAX)) + 1;
    return FHE_OK;
}
static u64 compat_reduce(const u64 k[4], u64 hi, u64 lo) {  // :84-111
    const u64 m = lo * k[3];
    const u128 mq = (u128)m * k[0];
    const u128 sum = ((u128)hi << 64) + lo + mq;
    u64 t = (u64)(sum >> 64);
    if (t >= k[0]) t -= k[0];
    return t;
}
uint64_t fhe_compat_montgomery_mul(const uint64_t k[4], uint64_t a, uint64_t b) {
    const u128 p = (u128)a * b;
    return compat_reduce(k, (u64)(p >> 64), (u64)p);
}
uint64_t fhe_compat_to_montgomery(const uint64_t k[4], uint64_t a) { return fhe_compat_montgomery_mul(k, a, k[2]); }
uint64_t fhe_compat_from_montgomery(const uint64_t k[4], uint64_t a) { return compat_reduce(k, 0, a); }
uint64_t fhe_compat_mod_add(uint64_t q, uint64_t a, uint64_t b) {
    a %= q; b %= q;
    u64 s = a + b;
    if (s < a || s >= q) s -= q;
    return s;
}
uint64_t fhe_compat_mod_sub(uint64_t q, uint64_t a, uint64_t b) {
    a %= q; b %= q;
    return a >= b ? a - b : q - (b - a);
}

// ---------------------------------------------------------------- context-owned device memory
// Stream-ordered allocations on a context's (first) device for callers that
// keep ciphertexts and keys resident (the N-API DeviceBuffer handles): the
// pool keeps freed blocks warm, and a free is ordered after all work already
// enqueued on the context stream, so no device-wide synchronisation.
int fhe_ctx_alloc(fhe_ctx *c, size_t bytes, void **out) {
    if (int rc = check_ctx(c)) return rc;
    if (!out) return fail(FHE_ERR_INVALID_ARG, "null out");
    fhe_ctx *s = c->multi() ? c->subs[0] : c;
    DeviceGuard g(s->device);
    hipError_t e = hipMallocAsync(out, bytes ? bytes : 8, s->stream);
    if (e == hipErrorOutOfMemory) return fail(FHE_ERR_OOM, "hipMallocAsync: out of memory");
    HIP_TRY(e, "hipMallocAsync");
    return FHE_OK;
}
int fhe_ctx_free(fhe_ctx *c, void *p) {
    if (int rc = check_ctx(c)) return rc;
    if (!p) return FHE_OK;
    fhe_ctx *s = c->multi() ? c->subs[0] : c;
    DeviceGuard g(s->device);
    HIP_TRY(hipFreeAsync(p, s->stream), "hipFreeAsync");
    return FHE_OK;
}
int fhe_ctx_memcpy(fhe_ctx *c, void *dst, const void *src, size_t bytes, int kind) {
    if (int rc = check_ctx(c)) return rc;
    if (bytes == 0) return FHE_OK;
    if (!dst || !src) return fail(FHE_ERR_INVALID_ARG, "null buffer");
    fhe_ctx *s = c->multi() ? c->subs[0] : c;
    DeviceGuard g(s->device);
    const hipMemcpyKind k = kind == FHE_COPY_H2D ? hipMemcpyHostToDevice
                          : kind == FHE_COPY_D2H ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    if (kind != FHE_COPY_H2D && kind != FHE_COPY_D2H && kind != FHE_COPY_D2D)
        return fail(FHE_ERR_INVALID_ARG, "unknown copy kind");
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, k, s->stream), "hipMemcpyAsync");
    if (kind != FHE_COPY_D2D) HIP_TRY(hipStreamSynchronize(s->stream), "hipStreamSynchronize");
    return FHE_OK;
}

// ---------------------------------------------------------------- memory / events
int fhe_dev_alloc(int device, size_t bytes, void **out) {
    if (!out) return fail(FHE_ERR_INVALID_ARG, "null out");
    DeviceGuard g(device);
    hipError_t e = hipMalloc(out, bytes);
    if (e == hipErrorOutOfMemory) return fail(FHE_ERR_OOM, "hipMalloc: out of memory");
    HIP_TRY(e, "hipMalloc");
    return FHE_OK;
}
int fhe_dev_free(void *p) {
    if (p) HIP_TRY(hipFree(p), "hipFree");
    return FHE_OK;
}
int fhe_memcpy_h2d(void *d, const void *s, size_t b) {
    HIP_TRY(hipMemcpy(d, s, b, hipMemcpyHostToDevice), "hipMemcpy(H2D)");
    return FHE_OK;
}
int fhe_memcpy_d2h(void *d, const void *s, size_t b) {
    HIP_TRY(hipMemcpy(d, s, b, hipMemcpyDeviceToHost), "hipMemcpy(D2H)");
    return FHE_OK;
}
int fhe_device_synchronize(int device) {
    DeviceGuard g(device);
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return FHE_OK;
}
int fhe_event_create(void **ev) {
    if (!ev) return fail(FHE_ERR_INVALID_ARG, "null out");
    HIP_TRY(hipEventCreate((hipEvent_t *)ev), "hipEventCreate");
    return FHE_OK;
}
int fhe_event_destroy(void *ev) {
    if (ev) HIP_TRY(hipEventDestroy((hipEvent_t)ev), "hipEventDestroy");
    return FHE_OK;
}
int fhe_event_record(void *ev, void *s) {
    HIP_TRY(hipEventRecord((hipEvent_t)ev, (hipStream_t)s), "hipEventRecord");
    return FHE_OK;
}
int fhe_event_elapsed_ms(void *a, void *b, float *ms) {
    HIP_TRY(hipEventSynchronize((hipEvent_t)b), "hipEventSynchronize");
    HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b), "hipEventElapsedTime");
    return FHE_OK;
}

}  // extern "C"
