// Microbenchmark: does a low-VGPR, memory-bound kernel on a second stream run
// beside a VALU-bound high-VGPR kernel (G1 mixed additions, ~3 waves/SIMD)?
// Prints A alone, B alone and A || B wall times.
// Standalone: hipcc -O3 --offload-arch=gfx950 tools/mb_corun.hip -o mb_corun
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../zelana_amd/csrc/ec.h"

using namespace zk;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ Fe fe_of(uint32_t s) {
  Fe r;
  for (int i = 0; i < NL; i++) { s = s * 1664525u + 1013904223u; r.v[i] = s & LMASK; }
  r.v[NL - 1] &= 0x1fffff;
  return r;
}
template <bool W2>
__global__ void __launch_bounds__(256) k_valu(uint32_t* out, int iters) {
  if constexpr (W2) asm volatile("" ::: "v183");  // 184 VGPRs: 2 waves per SIMD
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  Xyzz<FqOps> v{fe_of(t), fe_of(t + 7), fe_of(t + 11), fe_of(t + 13)};
  Fe ax = fe_of(t + 31), ay = fe_of(t + 37);
  for (int i = 0; i < iters; i++) {
    bool inf;
    v = xyzz_madd_g1f(v, ax, ay, &inf);
    ax.v[0] ^= i;
  }
  uint32_t o = 0;
  for (int i = 0; i < NL; i++) o ^= v.x.v[i] ^ v.y.v[i] ^ v.zz.v[i] ^ v.zzz.v[i];
  out[t] = o;
}
// streaming copy with a light LDS stage (like a sort scatter's traffic);
// dynamic LDS (lds_bytes) only reserves space, as the sort's sub-tiles would
__global__ void __launch_bounds__(256) k_mem(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  extern __shared__ uint4 sh[];
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    sh[threadIdx.x] = a[i];
    __syncthreads();
    b[i] = sh[255 - threadIdx.x];
    __syncthreads();
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const size_t n = (size_t)1 << 26;  // 1 GB per buffer
  uint32_t* d;
  uint4 *a, *b;
  CHECK(hipMalloc(&d, 256 * 64 * 256 * 4));
  CHECK(hipMalloc(&a, n * 16));
  CHECK(hipMalloc(&b, n * 16));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1)); CHECK(hipEventCreate(&e2));
  const int ga = 256 * 12, gb = 256 * 4;  // A: 12 workgroups per CU queued (3 waves/SIMD resident)
  bool w2 = false;
  size_t lds = 4096;
  auto run = [&](bool A, bool B) {
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, s1));
    CHECK(hipStreamWaitEvent(s2, e0, 0));
    if (A) {
      if (w2) k_valu<true><<<ga, 256, 0, s1>>>(d, iters);
      else k_valu<false><<<ga, 256, 0, s1>>>(d, iters);
    }
    if (B) for (int r = 0; r < 4; r++) k_mem<<<gb, 256, lds, s2>>>(a, b, n);
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventRecord(e2, s2));
    CHECK(hipDeviceSynchronize());
    float m1, m2;
    CHECK(hipEventElapsedTime(&m1, e0, e1));
    CHECK(hipEventElapsedTime(&m2, e0, e2));
    return m1 > m2 ? m1 : m2;
  };
  CHECK(hipFuncSetAttribute((const void*)k_mem, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  run(true, true);
  for (int cfg = 0; cfg < 4; cfg++) {
    w2 = cfg & 1;
    lds = cfg & 2 ? 105 * 1024 : 4096;
    float ta = run(true, false), tb = run(false, true), tab = run(true, true);
    printf("A %s, B lds %zu KB: A alone %.3f ms, B alone %.3f ms, A||B %.3f ms (sum %.3f)\n", w2 ? "2 waves" : "3 waves",
           lds / 1024, ta, tb, tab, ta + tb);
  }
  return 0;
}
