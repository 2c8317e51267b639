// Microbenchmark 2: v_mad_u64_u32 dependent latency and 29-bit Montgomery mul
// throughput / single-wave latency (tools/, dev only).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../zelana_amd/csrc/ec.h"
using namespace zk;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_mad_lat(uint64_t* out, uint32_t a, int iters) {
  uint64_t acc = threadIdx.x;
  uint32_t x = a + threadIdx.x;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) acc = (uint64_t)x * (uint32_t)(acc >> 7) + acc;
  }
  out[threadIdx.x] = acc;
}
template <bool SQR>
__global__ void __launch_bounds__(256) k_mul29(Fe* out, const Fe* in, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fe a = in[i & 1023], b = in[(i + 1) & 1023];
  for (int it = 0; it < iters; it++) a = SQR ? sqr<FqP>(a) : mul<FqP>(a, b);
  out[i] = a;
}
__global__ void __launch_bounds__(256) k_madd(Fe* out, const Fe* in, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  Xyzz<FqOps> acc;
  acc.x = in[i & 1023]; acc.y = in[(i + 3) & 1023]; acc.zz = in[(i + 5) & 1023]; acc.zzz = in[(i + 7) & 1023];
  Aff<FqOps> p; p.x = in[(i + 1) & 1023]; p.y = in[(i + 2) & 1023];
  for (int it = 0; it < iters; it++) acc = xyzz_madd(acc, p);
  out[i] = acc.x;
}

int main() {
  Fe h[1024];
  for (int i = 0; i < 1024; i++) for (int j = 0; j < 9; j++) h[i].v[j] = (uint32_t)(rand()) & (j == 8 ? 0x3fffffu : LMASK);
  Fe *in, *out; uint64_t* o64;
  CHECK(hipMalloc(&in, sizeof(h))); CHECK(hipMalloc(&out, 256 * 16 * 256 * sizeof(Fe))); CHECK(hipMalloc(&o64, 1 << 16));
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms;
  // latency: one wave
  int it = 20000;
  k_mad_lat<<<1, 64>>>(o64, 3, it); CHECK(hipDeviceSynchronize());
  hipEventRecord(e0); k_mad_lat<<<1, 64>>>(o64, 3, it); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("mad_u64 dependent chain: %.2f ns/op (1 wave)\n", ms * 1e6 / (it * 16.0));
  int it2 = 2000;
  k_mul29<false><<<1, 64>>>(out, in, it2); CHECK(hipDeviceSynchronize());
  hipEventRecord(e0); k_mul29<false><<<1, 64>>>(out, in, it2); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("mul29 latency (1 wave): %.1f ns\n", ms * 1e6 / it2);
  hipEventRecord(e0); k_madd<<<1, 64>>>(out, in, it2 / 10); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("madd latency (1 wave): %.1f ns\n", ms * 1e6 / (it2 / 10));
  const int blocks = 256 * 16; it2 = 200;
  for (int sq = 0; sq < 2; sq++) {
    auto k = sq ? k_mul29<true> : k_mul29<false>;
    k<<<blocks, 256>>>(out, in, it2); CHECK(hipDeviceSynchronize());
    hipEventRecord(e0); k<<<blocks, 256>>>(out, in, it2); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("%s29 throughput: %.1f G/s\n", sq ? "sqr" : "mul", (double)blocks * 256 * it2 / ms / 1e6);
  }
  k_madd<<<blocks, 256>>>(out, in, 20); CHECK(hipDeviceSynchronize());
  hipEventRecord(e0); k_madd<<<blocks, 256>>>(out, in, 20); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("madd throughput: %.2f G/s\n", (double)blocks * 256 * 20 / ms / 1e6);
  return 0;
}
