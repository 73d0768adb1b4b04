// Streaming bandwidth microbenchmark: 8 B vs 16 B per lane, and the NTT
// pass-0 access shape (16 loads per thread at stride T).  Lab tool only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
#define CK(x) do{hipError_t e=(x); if(e){printf("err %s line %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

__global__ void copy8(const uint64_t* __restrict__ a, uint64_t* __restrict__ b, size_t n) {
  size_t s = (size_t)gridDim.x*blockDim.x;
  for (size_t i = blockIdx.x*(size_t)blockDim.x+threadIdx.x; i < n; i += s) b[i] = a[i] + 1;
}
__global__ void copy16(const u64x2* __restrict__ a, u64x2* __restrict__ b, size_t n2) {
  size_t s = (size_t)gridDim.x*blockDim.x;
  for (size_t i = blockIdx.x*(size_t)blockDim.x+threadIdx.x; i < n2; i += s) { u64x2 v = a[i]; v.x += 1; v.y += 1; b[i] = v; }
}
// one block per "polynomial" of 16384 u64, 1024 threads, 16 loads at stride 1024, store same
template<int NT>
__global__ void __launch_bounds__(1024) poly_rw(const uint64_t* __restrict__ a, uint64_t* __restrict__ b) {
  const uint64_t* src = a + (size_t)blockIdx.x * 16384;
  uint64_t* dst = b + (size_t)blockIdx.x * 16384;
  uint64_t v[16];
  #pragma unroll
  for (int t = 0; t < 16; ++t) v[t] = NT ? __builtin_nontemporal_load(src + threadIdx.x + t*1024) : src[threadIdx.x + t*1024];
  #pragma unroll
  for (int t = 0; t < 16; ++t) { if (NT) __builtin_nontemporal_store(v[t] + 1, dst + threadIdx.x + t*1024); else dst[threadIdx.x + t*1024] = v[t] + 1; }
}
// same but 16 B per lane: 8 loads of u64x2 at stride 2048 (elements)
__global__ void __launch_bounds__(1024) poly_rw16(const u64x2* __restrict__ a, u64x2* __restrict__ b) {
  const u64x2* src = a + (size_t)blockIdx.x * 8192;
  u64x2* dst = b + (size_t)blockIdx.x * 8192;
  u64x2 v[8];
  #pragma unroll
  for (int t = 0; t < 8; ++t) v[t] = src[threadIdx.x + t*1024];
  #pragma unroll
  for (int t = 0; t < 8; ++t) { v[t].x += 1; v[t].y += 1; dst[threadIdx.x + t*1024] = v[t]; }
}

int main() {
  const size_t n = (size_t)1 << 30;  // 8 GiB per buffer
  uint64_t *a, *b;
  CK(hipMalloc(&a, n*8)); CK(hipMalloc(&b, n*8));
  CK(hipMemset(a, 1, n*8)); CK(hipMemset(b, 0, n*8));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    hipDeviceSynchronize();
    hipEventRecord(e0); for (int r = 0; r < 5; ++r) launch(); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, 2.0*n*8/ms/1e6);
  };
  for (int g : {1024, 2048, 4096, 8192, 16384}) {
    char nm[64];
    snprintf(nm, 64, "copy8 grid=%d", g);  run(nm, [&]{ copy8<<<g,256>>>(a,b,n); });
    snprintf(nm, 64, "copy16 grid=%d", g); run(nm, [&]{ copy16<<<g,256>>>((const u64x2*)a,(u64x2*)b,n/2); });
  }
  run("poly_rw 8B", [&]{ poly_rw<0><<<n/16384,1024>>>(a,b); });
  run("poly_rw 8B nt", [&]{ poly_rw<1><<<n/16384,1024>>>(a,b); });
  run("poly_rw 16B", [&]{ poly_rw16<<<n/16384,1024>>>((const u64x2*)a,(u64x2*)b); });
  return 0;
}
