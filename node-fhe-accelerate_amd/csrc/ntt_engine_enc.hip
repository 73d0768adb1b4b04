// ntt_engine_enc.hip -- EncryptionEngine::encrypt_internal
// (encryption.cpp:171-205), batched: k_encrypt (engine_kernels.hpp).
// Flag-free 64-bit arithmetic with the carry-free mulhi in this unit (as in
// ntt_inv.hip; fhe_arith.hpp FHE_U64_NOVCC, FHE_MULHI64=4): fewer static VALU
// issue cycles in its 64-bit kernels and fewer of them with scratch (round 6,
// DESIGN.md section 5).
#ifndef FHE_U64_NOVCC
#define FHE_U64_NOVCC 1
#endif
#ifndef FHE_MULHI64
#define FHE_MULHI64 4
#endif
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
