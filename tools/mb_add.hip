// Microbenchmark: latency and throughput of one G1 XYZZ addition (ec.h) in
// registers, at k waves per SIMD (grid = 256 CUs x k workgroups of 4 waves).
// Standalone: hipcc -O3 --offload-arch=gfx950 tools/mb_add.hip -o mb_add
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

template <int MODE>
__global__ void __launch_bounds__(256) k_add(uint32_t* out, int iters) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  Xyzz<FqOps> v{fe_of(t), fe_of(t + 7), fe_of(t + 11), fe_of(t + 13)};
  Xyzz<FqOps> q{fe_of(t + 17), fe_of(t + 19), fe_of(t + 23), fe_of(t + 29)};
  Aff<FqOps> a{fe_of(t + 31), fe_of(t + 37)};
  for (int i = 0; i < iters; i++) {
    if constexpr (MODE == 0) v = xyzz_add_g1(v, q);
    else v = xyzz_madd_g1(v, a);
    q.x.v[0] ^= i;  // keep q live and changing
    a.x.v[0] ^= i;
  }
  uint32_t o = 0;
  for (int i = 0; i < NL; i++) o ^= v.x.v[i] ^ v.y.v[i] ^ v.zz.v[i] ^ v.zzz.v[i];
  out[t] = o;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  uint32_t* d;
  CHECK(hipMalloc(&d, 256 * 8 * 256 * 4));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int mode = 0; mode < 2; mode++) {
    for (int k : {1, 2, 3, 4, 8}) {
      auto kern = mode == 0 ? k_add<0> : k_add<1>;
      kern<<<256 * k, 256>>>(d, iters);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(a));
      kern<<<256 * k, 256>>>(d, iters);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      const double adds = 256.0 * k * 256 * iters;
      printf("%s  waves/SIMD %d: %.3f ms, latency per add %.2f us, %.2f G adds/s\n", mode ? "madd_g1" : "add_g1 ", k,
             ms, ms * 1e3 / iters, adds / ms / 1e6);
    }
  }
  return 0;
}
