// keygen.hpp -- launchers of keygen.hip (device randomness, key material,
// LWE decryption).  Kept out of fhe_internal.hpp so that the transform
// kernels do not rebuild when these change.
#pragma once
#include "fhe_internal.hpp"

namespace FHE_NS {

// Sample kinds (include/fhe_gpu.h FHE_SAMPLE_*): SecureRandom's draws
// (key_manager.cpp:53-115) from a ChaCha20 stream instead of the OS device.
enum SampleKind { kUniform = 0, kTernary = 1, kGaussian = 2, kBinary = 3, kRaw = 4 };

struct ChaChaKey {
    uint32_t k[8];
};

// out[i], i < count: one draw of `kind` for element i of stream (key, nonce)
hipError_t launch_sample(int kind, const ChaChaKey &key, uint64_t nonce, uint64_t q, double std_dev, uint64_t *out,
                         size_t count, hipStream_t s);
// out[b][j] = x[b][j] * y[j] mod q (any u64 inputs), b < batch
hipError_t launch_modmul_bcast(const ModConsts &m, const uint64_t *x, const uint64_t *y, uint64_t *out, uint32_t n,
                               size_t batch, hipStream_t s);
// encrypt_ggsw's rows (bootstrap_engine.cpp:268-306): from the canonical
// mask * sk products prod [rows][k][n], the masks [rows][k][n] and errors
// [rows][n] (rows = count (k+1) L), out [rows][k+1][n] with the gadget term
// of values[c] added to coefficient 0 of component row / L of row
// (row, l) = (r / L, r % L) within ciphertext c.
hipError_t launch_ggsw_finish(const ModConsts &m, const uint64_t *prod, const uint64_t *masks, const uint64_t *err,
                              const int64_t *values, uint64_t *out, uint32_t n, uint32_t k, uint32_t level,
                              uint32_t base_log, size_t count, hipStream_t s);
// generate_key_switch_key's bodies (bootstrap_engine.cpp:388-415): entry
// e = i L + l, b[e] = ((u64)((<a_e, s> + err_e) % (int64)q) + gadget) % q
hipError_t launch_ksk_body(const ModConsts &m, const uint64_t *glwe_sk, const int64_t *lwe_sk, const uint64_t *a,
                           const uint64_t *err, uint64_t *b, uint32_t n_in, uint32_t level, uint32_t base_log,
                           uint32_t lwe_dim, hipStream_t s);
// LWE decryption: phase = b - sum_j a_j s_j (mod q), m = decode(phase)
hipError_t launch_lwe_decrypt(uint64_t q, uint64_t t, const int64_t *sk, uint32_t dim, const uint64_t *a,
                              const uint64_t *b, uint64_t *m, uint64_t *phase, size_t batch, hipStream_t s);

}  // namespace FHE_NS
