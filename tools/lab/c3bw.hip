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

// read-only (the two input streams) and write-only shapes of the same access
template <int T>
__global__ void __launch_bounds__(T) rd16(const u64x2 *__restrict__ a, const u64x2 *__restrict__ w, u64x2 *__restrict__ o) {
    constexpr int E = N / 2 / T;
    const size_t base = (size_t)blockIdx.x * (N / 2);
    u64x2 v[E], x[E];
#pragma unroll
    for (int t = 0; t < E; ++t) {
        v[t] = __builtin_nontemporal_load(a + base + threadIdx.x + t * T);
        x[t] = __builtin_nontemporal_load(w + base + threadIdx.x + t * T);
    }
    u64x2 r = v[0] ^ x[0];
#pragma unroll
    for (int t = 1; t < E; ++t) r ^= v[t] ^ x[t];
    if (r.x == 0x123456789ull) o[blockIdx.x * T + threadIdx.x] = r;
}
template <int T>
__global__ void __launch_bounds__(T) wr16(u64x2 *__restrict__ o) {
    constexpr int E = N / 2 / T;
    const size_t base = (size_t)blockIdx.x * (N / 2);
#pragma unroll
    for (int t = 0; t < E; ++t) {
        u64x2 v;
        v.x = base + t;
        v.y = threadIdx.x;
        __builtin_nontemporal_store(v, o + base + threadIdx.x + t * T);
    }
}
// LDS-DMA (global_load_lds_dwordx4) reads of both inputs, 16 KiB per input per
// chunk, then LDS -> VGPR, XOR, 16-byte nt stores
template <int T>
__global__ void __launch_bounds__(T) glds16(const u64x2 *__restrict__ a, const u64x2 *__restrict__ w,
                                            u64x2 *__restrict__ o) {
    constexpr int CH = 1024;  // u64x2 per input per chunk (16 KiB)
    __shared__ u64x2 la[2][CH], lw[2][CH];
    const size_t base = (size_t)blockIdx.x * (N / 2);
    auto issue = [&](int c, int buf) {
        for (int i = threadIdx.x; i < CH; i += T) {
            __builtin_amdgcn_global_load_lds((const void *)(a + base + c * CH + i), (__attribute__((address_space(3))) void *)&la[buf][i - threadIdx.x % 64 + 0], 16, 0, 2);
            __builtin_amdgcn_global_load_lds((const void *)(w + base + c * CH + i), (__attribute__((address_space(3))) void *)&lw[buf][i - threadIdx.x % 64 + 0], 16, 0, 2);
        }
    };
    constexpr int NC = N / 2 / CH;
    issue(0, 0);
    for (int c = 0; c < NC; ++c) {
        if (c + 1 < NC) {
            issue(c + 1, (c + 1) & 1);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * CH / T) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        for (int i = threadIdx.x; i < CH; i += T)
            __builtin_nontemporal_store(la[c & 1][i] ^ lw[c & 1][i], o + base + c * CH + i);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
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
    run("read-only 16B T=512 nt", [&] { rd16<512><<<g, 512>>>((const u64x2 *)a, (const u64x2 *)w, (u64x2 *)o); });
    run("write-only 16B T=512 nt", [&] { wr16<512><<<g, 512>>>((u64x2 *)o); });
    run("glds 16B T=512", [&] { glds16<512><<<g, 512>>>((const u64x2 *)a, (const u64x2 *)w, (u64x2 *)o); });
    run("glds 16B T=256", [&] { glds16<256><<<g, 256>>>((const u64x2 *)a, (const u64x2 *)w, (u64x2 *)o); });
    return 0;
}
