// VALU issue-rate microbenchmark for the instructions a modular butterfly can
// be built from (lab tool, not product code).  Each thread runs 8 independent
// dependency chains of one instruction so latency is hidden; the grid fills
// every SIMD.  Prints wave-instructions per CU per clock-equivalent as
// lane-ops/s for the whole chip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 2048;
constexpr int CH = 8;

#define KERNEL(NAME, T, INIT, BODY)                                                    \
    __global__ void __launch_bounds__(256) NAME(T *out, uint32_t seed) {               \
        T v[CH];                                                                       \
        _Pragma("unroll") for (int c = 0; c < CH; ++c) v[c] = INIT;                    \
        for (int it = 0; it < ITERS; ++it) {                                           \
            _Pragma("unroll") for (int c = 0; c < CH; ++c) { BODY; }                   \
        }                                                                              \
        T s = v[0];                                                                    \
        _Pragma("unroll") for (int c = 1; c < CH; ++c) s += v[c];                      \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                       \
    }

#define SEED32 (uint32_t)(seed + threadIdx.x * 7u + c)
KERNEL(k_mul_lo, uint32_t, SEED32, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_mul_hi, uint32_t, SEED32, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_mul_u24, uint32_t, SEED32, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_mulhi_u24, uint32_t, SEED32, asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_mad_u24, uint32_t, SEED32, asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_add, uint32_t, SEED32, asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_add3, uint32_t, SEED32, asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_min, uint32_t, SEED32, asm volatile("v_min_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_mad64, uint64_t, (uint64_t)SEED32, asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(v[c]) : "v"(seed) : "vcc"))
KERNEL(k_lshl_add64, uint64_t, (uint64_t)SEED32, asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(v[c])))
KERNEL(k_fma64, double, (double)SEED32, asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(v[c]) : "v"((double)seed)))
KERNEL(k_mul64, double, (double)SEED32, asm volatile("v_mul_f64 %0, %0, %1" : "+v"(v[c]) : "v"((double)seed)))
KERNEL(k_fma32, float, (float)SEED32, asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(v[c]) : "v"((float)seed)))
KERNEL(k_cvt_f64_u32, double, (double)SEED32, { uint32_t t; asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(t) : "v"(v[c])); asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(v[c]) : "v"(t)); })
KERNEL(k_cvt_f32_u32, float, (float)SEED32, { uint32_t t; asm volatile("v_cvt_u32_f32 %0, %1" : "=v"(t) : "v"(v[c])); asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(v[c]) : "v"(t)); })
KERNEL(k_sub, uint32_t, SEED32, asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_mov, uint32_t, SEED32, asm volatile("v_mov_b32 %0, %1" : "=v"(v[c]) : "v"(v[(c + 1) % CH])))
KERNEL(k_and, uint32_t, SEED32, asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_lshr, uint32_t, SEED32, asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_bfi, uint32_t, SEED32, asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_lshr64, uint64_t, (uint64_t)SEED32, asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(v[c])))
KERNEL(k_addco, uint32_t, SEED32, asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(v[c]) : "v"(seed) : "vcc"))
KERNEL(k_addc, uint32_t, SEED32, asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(v[c]) : "v"(seed) : "vcc"))
KERNEL(k_cndmask, uint32_t, SEED32, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[c]) : "v"(seed) : "vcc"))
KERNEL(k_cmp64, uint64_t, (uint64_t)SEED32, { uint64_t m; asm volatile("v_cmp_lt_u64_e64 %0, %1, %2" : "=s"(m) : "v"(v[c]), "v"((uint64_t)seed)); asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(*(uint32_t *)&v[c]) : "v"(seed), "s"(m)); })
KERNEL(k_cmp32, uint32_t, SEED32, { uint64_t m; asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(v[c]), "v"(seed)); asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(seed), "s"(m)); })
KERNEL(k_not, uint32_t, SEED32, asm volatile("v_not_b32 %0, %0" : "+v"(v[c])))
KERNEL(k_ashr, uint32_t, SEED32, asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_subrev, uint32_t, SEED32, asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_subco, uint32_t, SEED32, asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(v[c]) : "v"(seed) : "vcc"))
KERNEL(k_subb, uint32_t, SEED32, asm volatile("v_subb_co_u32 %0, vcc, %0, %1, vcc" : "+v"(v[c]) : "v"(seed) : "vcc"))
KERNEL(k_lshl32, uint32_t, SEED32, asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_or, uint32_t, SEED32, asm volatile("v_or_b32 %0, %0, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_or3, uint32_t, SEED32, asm volatile("v_or3_b32 %0, %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_lshladd32, uint32_t, SEED32, asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_andor, uint32_t, SEED32, asm volatile("v_and_or_b32 %0, %0, %1, %0" : "+v"(v[c]) : "v"(seed)))
KERNEL(k_lshl64, uint64_t, (uint64_t)SEED32, asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(v[c])))
KERNEL(k_mov64, uint64_t, (uint64_t)SEED32, asm volatile("v_mov_b64 %0, %1" : "=v"(v[c]) : "v"(v[(c + 1) % CH])))
KERNEL(k_cmpu64, uint64_t, (uint64_t)SEED32, { uint64_t m; asm volatile("v_cmp_le_u64_e64 %0, %1, %2" : "=s"(m) : "v"(v[c]), "v"((uint64_t)seed)); })
KERNEL(k_cmpu32, uint32_t, SEED32, { uint64_t m; asm volatile("v_cmp_ne_u32_e64 %0, %1, %2" : "=s"(m) : "v"(v[c]), "v"(seed)); })
KERNEL(k_cndsg, uint32_t, SEED32, asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[c]) : "v"(seed), "s"((uint64_t)seed * 0x9E3779B97F4A7C15ull)))
KERNEL(k_bitop3, uint32_t, SEED32, asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(v[c]) : "v"(seed)))
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ inline f2 mkf2(float a, float b) { f2 r; r.x = a; r.y = b; return r; }
KERNEL(k_pk_fma32, f2, mkf2((float)SEED32, 1.f), asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(v[c]) : "v"(mkf2((float)seed, 2.f))))

struct Case { const char *name; void (*launch)(void *, uint32_t, int); double ops_per_iter; size_t elt; };

template <typename T, void (*K)(T *, uint32_t)>
void launch(void *out, uint32_t seed, int blocks) { K<<<blocks, 256>>>((T *)out, seed); }

int main() {
    int dev;
    hipDeviceProp_t p;
    CK(hipGetDevice(&dev));
    CK(hipGetDeviceProperties(&p, dev));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 32;  // 32 x 4 waves per CU = 32 waves per SIMD
    void *out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 16));
    Case cases[] = {
        {"v_mul_lo_u32", launch<uint32_t, k_mul_lo>, 1, 4},
        {"v_mul_hi_u32", launch<uint32_t, k_mul_hi>, 1, 4},
        {"v_mul_u32_u24", launch<uint32_t, k_mul_u24>, 1, 4},
        {"v_mul_hi_u32_u24", launch<uint32_t, k_mulhi_u24>, 1, 4},
        {"v_mad_u32_u24", launch<uint32_t, k_mad_u24>, 1, 4},
        {"v_add_u32", launch<uint32_t, k_add>, 1, 4},
        {"v_add3_u32", launch<uint32_t, k_add3>, 1, 4},
        {"v_min_u32", launch<uint32_t, k_min>, 1, 4},
        {"v_mad_u64_u32", launch<uint64_t, k_mad64>, 1, 8},
        {"v_lshl_add_u64", launch<uint64_t, k_lshl_add64>, 1, 8},
        {"v_sub_u32", launch<uint32_t, k_sub>, 1, 4},
        {"v_mov_b32", launch<uint32_t, k_mov>, 1, 4},
        {"v_and_b32", launch<uint32_t, k_and>, 1, 4},
        {"v_lshrrev_b32", launch<uint32_t, k_lshr>, 1, 4},
        {"v_bfi_b32", launch<uint32_t, k_bfi>, 1, 4},
        {"v_lshrrev_b64", launch<uint64_t, k_lshr64>, 1, 8},
        {"v_add_co_u32", launch<uint32_t, k_addco>, 1, 4},
        {"v_addc_co_u32", launch<uint32_t, k_addc>, 1, 4},
        {"v_cndmask_b32", launch<uint32_t, k_cndmask>, 1, 4},
        {"v_cmp_lt_u64+v_cndmask", launch<uint64_t, k_cmp64>, 2, 8},
        {"v_cmp_lt_u32+v_cndmask", launch<uint32_t, k_cmp32>, 2, 4},
        {"v_not_b32", launch<uint32_t, k_not>, 1, 4},
        {"v_ashrrev_i32", launch<uint32_t, k_ashr>, 1, 4},
        {"v_subrev_u32", launch<uint32_t, k_subrev>, 1, 4},
        {"v_sub_co_u32", launch<uint32_t, k_subco>, 1, 4},
        {"v_subb_co_u32", launch<uint32_t, k_subb>, 1, 4},
        {"v_lshlrev_b32", launch<uint32_t, k_lshl32>, 1, 4},
        {"v_or_b32", launch<uint32_t, k_or>, 1, 4},
        {"v_or3_b32", launch<uint32_t, k_or3>, 1, 4},
        {"v_lshl_add_u32", launch<uint32_t, k_lshladd32>, 1, 4},
        {"v_and_or_b32", launch<uint32_t, k_andor>, 1, 4},
        {"v_lshlrev_b64", launch<uint64_t, k_lshl64>, 1, 8},
        {"v_mov_b64", launch<uint64_t, k_mov64>, 1, 8},
        {"v_cmp_le_u64", launch<uint64_t, k_cmpu64>, 1, 8},
        {"v_cmp_ne_u32", launch<uint32_t, k_cmpu32>, 1, 4},
        {"v_cndmask_b32(sgpr)", launch<uint32_t, k_cndsg>, 1, 4},
        {"v_bitop3_b32", launch<uint32_t, k_bitop3>, 1, 4},
        {"v_fma_f64", launch<double, k_fma64>, 1, 8},
        {"v_mul_f64", launch<double, k_mul64>, 1, 8},
        {"v_fma_f32", launch<float, k_fma32>, 1, 4},
        {"v_pk_fma_f32(2 lanes)", launch<f2, k_pk_fma32>, 1, 8},
        {"cvt_u32_f64+cvt_f64_u32", launch<double, k_cvt_f64_u32>, 2, 8},
        {"cvt_u32_f32+cvt_f32_u32", launch<float, k_cvt_f32_u32>, 2, 4},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("device %s, %d CUs, clock %d kHz\n", p.name, cus, p.clockRate);
    for (auto &c : cases) {
        c.launch(out, 3, blocks);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) c.launch(out, 3 + r, blocks);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double insts = 5.0 * blocks * 256.0 * ITERS * CH * c.ops_per_iter;  // lane-instructions
        const double rate = insts / (ms * 1e-3);
        // lane-ops per CU per clock (64 = one wave64 instruction per clock per CU... 4 SIMDs x 16 lanes)
        const double per_cu_clk = rate / cus / (p.clockRate * 1e3);
        printf("%-26s %8.3f ms  %8.2f Tlane-ops/s  %6.1f lane-ops/CU/clk\n", c.name, ms, rate / 1e12, per_cu_clk);
    }
    return 0;
}
