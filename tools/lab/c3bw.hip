// Streaming ceiling of the C3 access shape (lab tool): two 8 GiB inputs read,
// one 8 GiB output written, one 16384-word "polynomial" per workgroup, as
// k_ntt_fwd_mul does -- without the transform.  Variants: 8 or 16 B per lane,
// nt or default cache policy, workgroup size.  hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e) {                                                                  \
            printf("err %s line %d\n", hipGetErrorString(e), __LINE__);           \
            return 1;                                                             \
        }                                                                         \
    } while (0)
constexpr int N = 16384;

template <int T, bool NT>
__global__ void __launch_bounds__(T) rw8(const uint64_t *__restrict__ a, const uint64_t *__restrict__ w,
                                         uint64_t *__restrict__ o) {
    constexpr int E = N / T;
    const size_t base = (size_t)blockIdx.x * N;
    uint64_t v[E], x[E];
#pragma unroll
    for (int t = 0; t < E; ++t) {
        v[t] = NT ? __builtin_nontemporal_load(a + base + threadIdx.x + t * T) : a[base + threadIdx.x + t * T];
        x[t] = NT ? __builtin_nontemporal_load(w + base + threadIdx.x + t * T) : w[base + threadIdx.x + t * T];
    }
#pragma unroll
    for (int t = 0; t < E; ++t) {
        if (NT) __builtin_nontemporal_store(v[t] ^ x[t], o + base + threadIdx.x + t * T);
        else o[base + threadIdx.x + t * T] = v[t] ^ x[t];
    }
}
template <int T, bool NT>
__global__ void __launch_bounds__(T) rw16(const u64x2 *__restrict__ a, const u64x2 *__restrict__ w,
                                          u64x2 *__restrict__ o) {
    constexpr int E = N / 2 / T;
    const size_t base = (size_t)blockIdx.x * (N / 2);
    u64x2 v[E], x[E];
#pragma unroll
    for (int t = 0; t < E; ++t) {
        v[t] = NT ? __builtin_nontemporal_load(a + base + threadIdx.x + t * T) : a[base + threadIdx.x + t * T];
        x[t] = NT ? __builtin_nontemporal_load(w + base + threadIdx.x + t * T) : w[base + threadIdx.x + t * T];
    }
#pragma unroll
    for (int t = 0; t < E; ++t) {
        if (NT) __builtin_nontemporal_store(v[t] ^ x[t], o + base + threadIdx.x + t * T);
        else o[base + threadIdx.x + t * T] = v[t] ^ x[t];
    }
}

int main() {
    const size_t polys = 65536, n = polys * N;  // 8 GiB per buffer
    uint64_t *a, *w, *o;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&w, n * 8));
    CK(hipMalloc(&o, n * 8));
    CK(hipMemset(a, 1, n * 8));
    CK(hipMemset(w, 2, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 2; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-24s %7.3f ms  %7.1f GB/s\n", name, ms, 3.0 * n * 8 / ms / 1e6);
        return 0;
    };
    const dim3 g(polys);
    run("8B T=1024 nt", [&] { rw8<1024, true><<<g, 1024>>>(a, w, o); });
    run("8B T=1024", [&] { rw8<1024, false><<<g, 1024>>>(a, w, o); });
    run("8B T=512 nt", [&] { rw8<512, true><<<g, 512>>>(a, w, o); });
    run("16B T=512 nt", [&] { rw16<512, true><<<g, 512>>>((const u64x2 *)a, (const u64x2 *)w, (u64x2 *)o); });
    run("16B T=512", [&] { rw16<512, false><<<g, 512>>>((const u64x2 *)a, (const u64x2 *)w, (u64x2 *)o); });
    run("16B T=1024 nt", [&] { rw16<1024, true><<<g, 1024>>>((const u64x2 *)a, (const u64x2 *)w, (u64x2 *)o); });
    run("16B T=256 nt", [&] { rw16<256, true><<<g, 256>>>((const u64x2 *)a, (const u64x2 *)w, (u64x2 *)o); });
    return 0;
}
