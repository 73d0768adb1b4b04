// ntt_engine_dec.hip -- EncryptionEngine::decrypt / decrypt_packed with the
// noise measure (encryption.cpp:234-400), batched: k_decrypt
// (engine_kernels.hpp).
#include "engine_kernels.hpp"

namespace FHE_NS {

hipError_t launch_decrypt(const Plan &p, uint64_t t, const uint64_t *sk_prep, const uint64_t *ct, int comps,
                          int is_ntt, uint64_t *phase, int store_phase, uint64_t *dec, uint64_t *noise, size_t batch) {
    if (p.logn > kMaxFusedLogN) return hipErrorInvalidValue;
    EngArgs E{};
    E.ct = ct; E.key = sk_prep; E.out = phase; E.dec = dec; E.noise = noise; E.batch = batch;
    E.comps = comps; E.is_ntt = is_ntt; E.store_phase = store_phase;
    E.D = make_decoder(plan_q(p), t);
    return eng_any<1>(p, E);
}

}  // namespace FHE_NS
