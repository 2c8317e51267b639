// Microbenchmark: integer-multiply instruction rates and 256-bit Montgomery
// multiplication variants on gfx950. Standalone: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

struct F { uint32_t v[8]; };
__constant__ uint32_t Q[8] = {0xd87cfd47u,0x3c208c16u,0x6871ca8du,0x97816a91u,0x8181585du,0xb85045b6u,0xe131a029u,0x30644e72u};
#define QINV 0xe4866389u

__device__ __forceinline__ F final_sub(const uint32_t* t) {
  uint32_t r[8]; uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) { uint64_t d = (uint64_t)t[j] - Q[j] - br; r[j] = (uint32_t)d; br = (uint32_t)(d >> 63); }
  F o; bool ge = (br == 0);
#pragma unroll
  for (int j = 0; j < 8; j++) o.v[j] = ge ? r[j] : t[j];
  return o;
}

// V0: CIOS, compiler-generated
__device__ __forceinline__ F mm_cios(const F& a, const F& b) {
  uint32_t t[9];
#pragma unroll
  for (int j = 0; j < 9; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) { uint64_t x = (uint64_t)a.v[j] * b.v[i] + t[j] + c; t[j] = (uint32_t)x; c = x >> 32; }
    uint64_t s = (uint64_t)t[8] + c; t[8] = (uint32_t)s;
    uint32_t m = t[0] * QINV;
    uint64_t x = (uint64_t)m * Q[0] + t[0]; c = x >> 32;
#pragma unroll
    for (int j = 1; j < 8; j++) { x = (uint64_t)m * Q[j] + t[j] + c; t[j-1] = (uint32_t)x; c = x >> 32; }
    s = (uint64_t)t[8] + c; t[7] = (uint32_t)s; t[8] = (uint32_t)(s>>32);
  }
  return final_sub(t);
}

// V1: FIPS product scanning with asm mad+carry
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, %2, %1" : "+v"(acc), "=&s"(cy), "+v"(c2) : "v"(a), "v"(b));
}
__device__ __forceinline__ F mm_fips(const F& a, const F& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0; uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) { mac(acc, c2, a.v[j], b.v[k-j]); mac(acc, c2, m[j], Q[k-j]); }
    mac(acc, c2, a.v[k], b.v[0]);
    m[k] = (uint32_t)acc * QINV;
    mac(acc, c2, m[k], Q[0]);
    acc = (acc >> 32) | ((uint64_t)c2 << 32); c2 = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int j = k - 7; j < 8; j++) { mac(acc, c2, a.v[j], b.v[k-j]); mac(acc, c2, m[j], Q[k-j]); }
    t[k-8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32); c2 = 0;
  }
  t[7] = (uint32_t)acc;
  return final_sub(t);
}

template <int V>
__global__ void __launch_bounds__(256) k_mm(F* out, const F* in, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  F a = in[i & 1023], b = in[(i + 1) & 1023];
  for (int it = 0; it < iters; it++) { a = (V == 0) ? mm_cios(a, b) : mm_fips(a, b); }
  out[i] = a;
}

template <int K>
__global__ void __launch_bounds__(256) k_mad64(uint32_t* out, uint32_t a, int iters) {
  uint64_t acc[K];
#pragma unroll
  for (int i = 0; i < K; i++) acc[i] = threadIdx.x + i;
  uint32_t x = a + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < K; i++) acc[i] = (uint64_t)x * (uint32_t)(acc[i] >> 32) + acc[i];
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < K; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}
template <int K>
__global__ void __launch_bounds__(256) k_mullo(uint32_t* out, uint32_t a, int iters) {
  uint32_t acc[K];
#pragma unroll
  for (int i = 0; i < K; i++) acc[i] = threadIdx.x + i;
  uint32_t x = a + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < K; i++) acc[i] = acc[i] * x;
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < K; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int K>
__global__ void __launch_bounds__(256) k_fma64(double* out, double a, double b, int iters) {
  double acc[K];
#pragma unroll
  for (int i = 0; i < K; i++) acc[i] = threadIdx.x + i;
  double x = a + threadIdx.x * 1e-9;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < K; i++) acc[i] = __builtin_fma(acc[i], x, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < K; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int K>
__global__ void __launch_bounds__(256) k_add(uint32_t* out, uint32_t a, uint32_t b, int iters) {
  uint32_t acc[K];
#pragma unroll
  for (int i = 0; i < K; i++) acc[i] = threadIdx.x + i;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < K; i++) acc[i] = (acc[i] ^ a) + b;
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < K; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 16, threads = 256;
  const long nthreads = (long)blocks * threads;
  void* out; CHECK(hipMalloc(&out, nthreads * sizeof(F)));
  F* in; CHECK(hipMalloc(&in, 1024 * sizeof(F)));
  F h[1024]; for (int i = 0; i < 1024; i++) for (int j = 0; j < 8; j++) h[i].v[j] = (uint32_t)(rand() * 2654435761u) & (j == 7 ? 0x0fffffffu : 0xffffffffu);
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
#define TIME(name, ops_per_thread, launch) do { launch; CHECK(hipDeviceSynchronize()); hipEventRecord(e0); launch; hipEventRecord(e1); CHECK(hipEventSynchronize(e1)); hipEventElapsedTime(&ms, e0, e1); \
    double ops = (double)nthreads * (ops_per_thread); printf("%-28s %8.3f ms  %10.2f G/s\n", name, ms, ops / ms / 1e6); } while (0)
  const int it = 2000;
  TIME("v_mad_u64_u32 (dep chains 8)", 8.0 * it, (k_mad64<8><<<blocks, threads>>>((uint32_t*)out, 7, it)));
  TIME("v_mul_lo_u32 (chains 8)", 8.0 * it, (k_mullo<8><<<blocks, threads>>>((uint32_t*)out, 7, it)));
  TIME("v_fma_f64 (chains 8)", 8.0 * it, (k_fma64<8><<<blocks, threads>>>((double*)out, 1.0000001, 1e-7, it)));
  TIME("v_add/xor u32 (chains 8)", 16.0 * it, (k_add<8><<<blocks, threads>>>((uint32_t*)out, 7, 9, it)));
  const int it2 = 200;
  TIME("montmul CIOS (compiler)", 1.0 * it2, (k_mm<0><<<blocks, threads>>>((F*)out, in, it2)));
  TIME("montmul FIPS (asm mac)", 1.0 * it2, (k_mm<1><<<blocks, threads>>>((F*)out, in, it2)));
  return 0;
}
