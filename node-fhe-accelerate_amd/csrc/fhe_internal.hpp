// fhe_internal.hpp -- interface between the host C-ABI (fhe_gpu.cpp) and the
// kernel translation units.  Not installed; no torch types anywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>

#include "ntt_core.hpp"

namespace FHE_NS {

// Orders every use of a context's big-N scratch (Plan::big_scratch): the
// launch sequence of one two-pass transform is enqueued under `mu`, and a
// sequence on another stream first waits for `done`, the completion of the
// previous one.  Host threads and streams (the staging slots, async N-API
// jobs, a caller's own stream) may then share one context.
struct BigSync {
    std::mutex mu;
    hipEvent_t done = nullptr;
    hipStream_t last = nullptr;
};

// Moduli 2^62 <= q < 2^64 (ntt_wide.hip): canonical arithmetic, twiddles in
// Montgomery form (w 2^64 mod q), stage-major like NttArgs' tables.
struct WideArgs {
    const uint64_t *twf, *twi;
    uint64_t q, qinv, mu;   // qinv = -q^-1 mod 2^64, mu = floor(2^64 / q)
    uint64_t r2;            // 2^128 mod q
    uint64_t ninv_m;        // N^-1 2^64 mod q
    uint64_t ninv_r2;       // N^-1 2^128 mod q (after a Montgomery pointwise product)
};

struct Plan {
    uint32_t logn;
    int word;   // 32 or 64
    int wide;   // q >= 2^62: every transform takes ntt_wide.hip
    int lazy;   // 32-bit path with (4 + 2L) q <= 2^32: forward stages skip reductions
    int compat; // compat-mode tables (unit twiddle in pass 0): hot kernels take gk_compat keys
    int cus;    // compute units of the context's device (persistent grids)
    hipStream_t stream;
    // N > 2^kMaxFusedLogN (ntt_big.hip): two chunk-sized scratch buffers
    uint64_t *big_scratch[2];
    size_t big_chunk;  // polynomials per scratch chunk
    BigSync *big_sync; // owned by the context
    NttArgs<uint32_t> a32;
    NttArgs<uint64_t> a64;
    WideArgs wa;  // wide != 0
};

constexpr int kMinLogN = 2;
constexpr int kMaxFusedLogN = 14;  // one workgroup per polynomial up to here
constexpr int kMaxLogN = 16;       // NTTProcessor's limit (ntt_processor.cpp:146)

// Forward NTT; epi 0: canonical output, 1: output * R mod q (Montgomery
// form, used to prepare GGSW keys).
hipError_t launch_fwd(const Plan &p, const uint64_t *in, uint64_t *out, size_t batch, int epi);
hipError_t launch_inv(const Plan &p, const uint64_t *in, uint64_t *out, size_t batch);
// out = fwd(a) (.) w  (config C3: NTT + modmul)
hipError_t launch_fwd_mul(const Plan &p, const uint64_t *a, const uint64_t *w, uint64_t *out, size_t batch);
// c = inv(fwd(a) (.) fwd(b))  (PolynomialRing::multiply)
hipError_t launch_polymul(const Plan &p, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch);
// RNS ring in one launch (grid.y = limb): `limbs` contiguous [batch][N]
// blocks, limb l with the transform constants tab[l] (a device array of
// NttArgs<uint32_t> or NttArgs<uint64_t> per p.word); every limb shares p's
// degree, word and laziness.  inv_limbs: inverse (b == nullptr) or polymul.
hipError_t launch_fwd_limbs(const Plan &p, const void *tab, int limbs, const uint64_t *in, uint64_t *out,
                            size_t batch);
hipError_t launch_inv_limbs(const Plan &p, const void *tab, int limbs, const uint64_t *a, const uint64_t *b,
                            uint64_t *c, size_t batch);
// q >= 2^62 (Plan::wide), any N: op as launch_big
hipError_t launch_wide(const Plan &p, int op, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch);
// N > 2^kMaxFusedLogN: op 0 fwd, 1 fwd*R, 2 fwd (.) b, 3 inv, 4 polymul
hipError_t launch_big(const Plan &p, int op, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t batch);
// TFHE external product, GGSW already in NTT-Montgomery form.
hipError_t launch_extprod(const Plan &p, int k1, int level, int base_log, const uint64_t *glwe,
                          const uint64_t *ggsw, uint64_t *out, size_t batch);
// Several decomposition levels at N = 16384, 64-bit words, k1 == 2,
// base_log <= 31 (ntt_ext2.hip): accumulators in VGPRs, one HBM pass.
bool extprod_acc_supported(const Plan &p, int k1, int level, int base_log);
hipError_t launch_extprod_acc(const Plan &p, int level, int base_log, const uint64_t *glwe, const uint64_t *ggsw,
                              uint64_t *out, size_t batch);

// Relinearisation (EncryptionEngine::relinearize): ct3 [batch][3][n],
// rlk [level][2][n] (a_l, b_l) in NTT-Montgomery form -> out [batch][2][n].
hipError_t launch_relin(const Plan &p, int level, int base_log, const uint64_t *ct3, const uint64_t *rlk,
                        uint64_t *out, size_t batch);
// One blind-rotation CMux step over a batch of GLWE accumulators (ping-pong
// buffers acc_in -> acc_out); step = LWE mask index i, bsk[i] = ggsw.
hipError_t launch_cmux_rotate(const Plan &p, int k1, int level, int base_log, const uint64_t *acc_in,
                              const uint64_t *ggsw, uint64_t *acc_out, size_t batch, const uint64_t *lwe_a,
                              uint32_t lwe_dim, uint32_t step, uint64_t lwe_q);
// The whole blind rotation (initial X^-round(b 2N/q) rotation + lwe_dim
// CMux steps) of a small batch in ONE launch (ntt_br.hip): one workgroup per
// ciphertext, accumulators resident in LDS across all steps.  k1 == 2 and
// 512 <= N <= 2048 only (br_persist_supported); acc is updated in place.
bool br_persist_supported(const Plan &p, int k1);
// k = 1 on two CUs per ciphertext (N = 1024..4096, grid 16 ceil(batch / 8)
// <= CUs); scratch: br_pair_scratch_bytes (flags zeroed by the launch).  A
// workgroup whose partner does not answer within timeout_ticks (100 MHz)
// gives up on its ciphertext; the launch is followed by a repair pass
// (k_br_persist) over the given-up ciphertexts, each counted in *repairs.
// With multi set, levels 2 / 3 at small batches take 2 level CUs per
// ciphertext instead (k_br_multi; br_multi_members), same protocol and repair.
struct BrPairOpts {
    uint64_t timeout_ticks;
    bool coop;                     // hipLaunchCooperativeKernel (grid checked against occupancy)
    unsigned long long *repairs;   // device counter
    bool multi;                    // k_br_multi where br_multi_members > 0
};
bool br_pair_supported(const Plan &p, int k1, size_t batch);
int br_multi_members(const Plan &p, int level, size_t batch);
size_t br_pair_scratch_bytes(const Plan &p, size_t batch, int level, bool multi);
hipError_t launch_br_pair(const Plan &p, int level, int base_log, uint64_t *acc, const uint64_t *bsk,
                          const uint64_t *lwe_a, const uint64_t *lwe_b, uint32_t lwe_dim, uint64_t lwe_q, size_t batch,
                          void *scratch, const BrPairOpts &o);
hipError_t launch_br_persist(const Plan &p, int k1, int level, int base_log, uint64_t *acc, const uint64_t *bsk,
                             const uint64_t *lwe_a, const uint64_t *lwe_b, uint32_t lwe_dim, uint64_t lwe_q,
                             size_t batch);
// CMux(ggsw, ct0, ct1) = ct0 + ggsw (x) (ct1 - ct0)
hipError_t launch_cmux(const Plan &p, int k1, int level, int base_log, const uint64_t *ggsw, const uint64_t *ct0,
                       const uint64_t *ct1, uint64_t *out, size_t batch);
// Ciphertext multiply (coefficient form): x, y [batch][2][n] -> out [batch][3][n]
hipError_t launch_ct_mul(const Plan &p, const uint64_t *x, const uint64_t *y, uint64_t *out, size_t batch);

// EncryptionEngine encrypt / decrypt / add_plain (ntt_engine.hip); keys
// prepared NTT x R (Montgomery form): pk_prep (pk.a, pk.b), sk_prep (s, s^2).
// t = plaintext modulus (0 -> 4).  decrypt: phase [batch][n] is required for
// comps == 3 on coefficient-form ciphertexts (the partial phase lives there);
// store_phase selects whether the final phase is written.
hipError_t launch_encrypt(const Plan &p, uint64_t t, const uint64_t *pk_prep, const uint64_t *vals,
                          const uint64_t *u, const uint64_t *e1, const uint64_t *e2, uint64_t *ct, size_t batch);
hipError_t launch_decrypt(const Plan &p, uint64_t t, const uint64_t *sk_prep, const uint64_t *ct, int comps,
                          int is_ntt, uint64_t *phase, int store_phase, uint64_t *dec, uint64_t *noise, size_t batch);
hipError_t launch_add_plain(const Plan &p, uint64_t t, const uint64_t *ct, const uint64_t *vals, int is_ntt,
                            uint64_t *out, size_t batch);
// Composed encrypt / decrypt / add_plain (engine_composed.hip) for q >= 2^62
// and N > 16384: elementwise finishing passes around batched transforms.
hipError_t launch_enc_finish(uint64_t q, uint64_t t, const uint64_t *t0, const uint64_t *t1, const uint64_t *e1,
                             const uint64_t *e2, const uint64_t *vals, uint64_t *ct, uint32_t n, size_t batch,
                             hipStream_t s);
hipError_t launch_sub_row(uint64_t q, const uint64_t *src, uint32_t comps, const uint64_t *x, uint64_t *out, uint32_t n,
                          size_t batch, hipStream_t s);
hipError_t launch_decode(uint64_t q, uint64_t t, const uint64_t *phase, uint64_t *dec, uint64_t *noise, uint32_t n,
                         size_t batch, hipStream_t s);
hipError_t launch_add_plain_fin(uint64_t q, const uint64_t *ct, const uint64_t *f, uint64_t *out, uint32_t n, size_t batch,
                                hipStream_t s);
hipError_t launch_encode(uint64_t q, uint64_t t, const uint64_t *vals, uint64_t *out, size_t count, hipStream_t s);
// acc [batch][k1][n] = (0, .., 0, test_poly): bootstrap's accumulator
hipError_t launch_glwe_init(const uint64_t *test_poly, uint64_t *acc, uint32_t n, uint32_t k1, size_t batch,
                            hipStream_t s);

// Elementwise kernels (elementwise.hip).
struct ModConsts {
    uint64_t q, mu, qinv, r2;  // mu = floor(2^64/q); Montgomery R = 2^64
    int fast;                  // q odd and q < 2^63
};
// Composed TFHE / BFV paths (k > 1, N > 16384): key MAC of NTT-domain
// digits, relinearisation digits, row-wise mod_add.
hipError_t launch_mac_keys(const ModConsts &m, int word, const uint64_t *x, const uint64_t *g, uint64_t *out,
                           uint32_t n, size_t batch, uint32_t rows, uint32_t k1, int swap, hipStream_t s);
hipError_t launch_relin_digits(const uint64_t *ct3, uint64_t *out, uint32_t n, size_t batch, uint32_t base_log,
                               uint32_t level, hipStream_t s);
hipError_t launch_add_rows(const ModConsts &m, uint64_t *out, const uint64_t *src, uint32_t n, size_t batch,
                           uint32_t rows, uint32_t src_rows, hipStream_t s);
hipError_t launch_modmul(const ModConsts &m, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t n,
                         hipStream_t s);
hipError_t launch_addsub(const ModConsts &m, const uint64_t *a, const uint64_t *b, uint64_t *c, size_t n, int sub,
                         hipStream_t s);
hipError_t launch_neg(uint64_t q, const uint64_t *a, uint64_t *c, size_t n, hipStream_t s);
// RNS ring: pointwise product (op 0), add (1), sub (2) over [limbs][per] with
// per-limb constants tab[limb] (device array), one launch.
hipError_t launch_ew_limbs(const ModConsts *tab, int limbs, const uint64_t *a, const uint64_t *b, uint64_t *c,
                           size_t per, int op, hipStream_t s);
hipError_t launch_mul_scalar(const ModConsts &m, const uint64_t *a, uint64_t sc, uint64_t sc_shoup, uint64_t *c,
                             size_t n, hipStream_t s);
hipError_t launch_ml_montmul(const uint64_t consts[7], const uint64_t *a, const uint64_t *b, uint64_t *c, size_t n,
                             hipStream_t s);
// Tensor product of NTT-form ciphertexts: x, y [batch][2][n] -> [batch][3][n]
hipError_t launch_tensor_ntt(const ModConsts &m, const uint64_t *x, const uint64_t *y, uint64_t *out, uint32_t n,
                             size_t batch, hipStream_t s);
// GLWE rotation by X^r (multiply_glwe_by_monomial): polys per ciphertext =
// k1; r = rot[c], or when rot == nullptr r = -(int32)((b[c]*2N + q/2)/q)
// (blind_rotate's initial rotation by the LWE body).
hipError_t launch_rotate(const ModConsts &m, const uint64_t *in, uint64_t *out, uint32_t n, uint32_t k1, size_t batch,
                         const int32_t *rot, const uint64_t *lwe_b, uint64_t lwe_q, hipStream_t s);
// Composed blind-rotation step (lwe.hip k_br_diff / k_br_add)
hipError_t launch_br_diff(const ModConsts &m, const uint64_t *cur, uint64_t *d, uint32_t n, uint32_t k1, size_t batch,
                          const uint64_t *lwe_a, uint32_t dim, uint32_t step, uint64_t lwe_q, hipStream_t s);
hipError_t launch_br_add(const ModConsts &m, const uint64_t *cur, const uint64_t *ep, uint64_t *nxt, uint32_t n,
                         uint32_t k1, size_t batch, const uint64_t *lwe_a, uint32_t dim, uint32_t step, uint64_t lwe_q,
                         hipStream_t s);
// sample_extract: glwe [batch][k+1][n] -> lwe_a [batch][k*n], lwe_b [batch]
hipError_t launch_sample_extract(const ModConsts &m, const uint64_t *glwe, uint64_t *lwe_a, uint64_t *lwe_b,
                                 uint32_t n, uint32_t k, size_t batch, hipStream_t s);
// LWE key switch (BootstrapEngine::key_switch); scratch of
// key_switch_scratch_bytes (0: none needed) for the split partial sums.
size_t key_switch_scratch_bytes(const ModConsts &m, uint32_t base_log, uint32_t level, uint32_t in_dim,
                                uint32_t out_dim, size_t batch);
hipError_t launch_key_switch(const ModConsts &m, uint32_t base_log, uint32_t level, uint32_t in_dim, uint32_t out_dim,
                             const uint64_t *ksk_a, const uint64_t *ksk_b, const uint64_t *lwe_a,
                             const uint64_t *lwe_b, uint64_t *out_a, uint64_t *out_b, size_t batch, void *scratch,
                             hipStream_t s);
hipError_t launch_decompose(const ModConsts &m, const uint64_t *poly, uint64_t *out, uint32_t n, size_t npoly,
                            uint32_t base_log, uint32_t level, hipStream_t s);

}  // namespace FHE_NS
