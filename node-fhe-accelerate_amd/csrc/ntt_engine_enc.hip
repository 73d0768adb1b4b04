// ntt_engine_enc.hip -- EncryptionEngine::encrypt_internal
// (encryption.cpp:171-205), batched: k_encrypt (engine_kernels.hpp).
#include "engine_kernels.hpp"

namespace FHE_NS {

hipError_t launch_encrypt(const Plan &p, uint64_t t, const uint64_t *pk_prep, const uint64_t *vals,
                          const uint64_t *u, const uint64_t *e1, const uint64_t *e2, uint64_t *ct, size_t batch) {
    if (p.logn > kMaxFusedLogN) return hipErrorInvalidValue;
    EngArgs E{};
    E.key = pk_prep; E.vals = vals; E.u = u; E.e1 = e1; E.e2 = e2; E.out = ct; E.batch = batch;
    E.D = make_decoder(plan_q(p), t);
    return eng_any<0>(p, E);
}

}  // namespace FHE_NS
