// Microbenchmark: the G2 bucket accumulation's mixed
// addition (ec.h xyzz_madd_g2) in one lane per bucket against a two-lane Fq2
// split -- lane 2k holds the c0 components of a bucket's coordinates, lane
// 2k+1 the c1 components, and every Fq2 product is one two-product Montgomery
// pass per lane (f2_mul_n already forms c0 and c1 as separate passes), with
// the partner's operands exchanged by DPP quad permutes.  Both run the same
// chain of additions in registers over the same inputs; the split's results
// are checked against the one-lane form (bit-exact: same passes, same bounds).
// Standalone: hipcc -O3 --offload-arch=gfx950 tools/mb_g2split.hip -o mb_g2split
//   ./mb_g2split [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../zelana_amd/csrc/ec.h"

using namespace zk;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ Fe fe_of(uint32_t s) {
  Fe r;
  for (int i = 0; i < NL; i++) { s = s * 1664525u + 1013904223u; r.v[i] = s & LMASK; }
  r.v[NL - 1] &= 0x1fffff;  // < 2^253 < p
  return r;
}
// inputs of bucket b: point (x, y, zz, zzz) and base (qx, qy), component c
__device__ Fe in_of(uint32_t b, int k, int c) { return fe_of(b * 97u + (uint32_t)(2 * k + c) * 13u + 1u); }

// ---- one lane per bucket (the kernel's form), with the MSM's launch bounds
__global__ void __launch_bounds__(256, 2) k_one(uint32_t* out, int iters) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  Xyzz<Fq2Ops> v;
  v.x = {in_of(b, 0, 0), in_of(b, 0, 1)};
  v.y = {in_of(b, 1, 0), in_of(b, 1, 1)};
  v.zz = {in_of(b, 2, 0), in_of(b, 2, 1)};
  v.zzz = {in_of(b, 3, 0), in_of(b, 3, 1)};
  Aff<Fq2Ops> q;
  q.x = {in_of(b, 4, 0), in_of(b, 4, 1)};
  q.y = {in_of(b, 5, 0), in_of(b, 5, 1)};
  for (int i = 0; i < iters; i++) {
    v = xyzz_madd_g2(v, q);
    q.x.c0.v[0] ^= (uint32_t)i & 7u;  // a new base each step (stays < 2p)
  }
  uint32_t* o = out + (size_t)b * 72;
  const Fe* f[8] = {&v.x.c0, &v.x.c1, &v.y.c0, &v.y.c1, &v.zz.c0, &v.zz.c1, &v.zzz.c0, &v.zzz.c1};
  for (int k = 0; k < 8; k++)
    for (int i = 0; i < NL; i++) o[k * 9 + i] = f[k]->v[i];
}

// ---- two lanes per bucket
__device__ __forceinline__ uint32_t swp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ Fe px(const Fe& a) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = swp(a.v[i]);
  return r;
}
__device__ __forceinline__ Fe sel(bool c, const Fe& a, const Fe& b) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}
// this lane's component of a*b (f2_mul_n): c0 = a0 b0 - a1 b1, c1 = a0 b1 + a1 b0
__device__ __forceinline__ Fe s_mul(bool c1, const Fe& a, const Fe& ap, const Fe& b, const Fe& bp) {
  return mul2<FqPn>(sel(c1, ap, a), b, sel(c1, a, ap), sel(c1, bp, subk<FqPn, 4>(fe_zero(), bp)));
}
// f2_sqr_n: c0 = (a0 + a1)(a0 - a1), c1 = 2 a0 a1
__device__ __forceinline__ Fe s_sqr(bool c1, const Fe& a, const Fe& ap) {
  return mul<FqPn>(add_lazy(sel(c1, ap, a), ap), sel(c1, a, subk<FqPn, 4>(a, ap)));
}
struct Half {
  Fe x, y, zz, zzz;
};
__device__ __forceinline__ Half s_madd(bool c1, const Half& p, const Fe& qx, const Fe& qy) {
  const Fe qxp = px(qx), qyp = px(qy), zzp = px(p.zz), zzzp = px(p.zzz);
  const Fe u2 = s_mul(c1, qx, qxp, p.zz, zzp), s2 = s_mul(c1, qy, qyp, p.zzz, zzzp);
  const Fe pp_ = subk<FqPn, 2>(u2, p.x);
  const Fe rr = subk<FqPn, 2>(s2, p.y);
  const Fe pp_p = px(pp_), rrp = px(rr);
  const Fe pp = s_sqr(c1, pp_, pp_p);
  // the equal-x test of xyzz_madd_g2, on both components (never true here;
  // the branch body is a stand-in so the test is not optimised away)
  {
    const uint32_t z = is_zero<FqPn>(pp) ? 1u : 0u;
    if (z & swp(z)) return Half{qx, qy, pp, pp};
  }
  const Fe r2 = s_sqr(c1, rr, rrp);
  const Fe ppp_in = px(pp);
  const Fe ppp = s_mul(c1, pp_, pp_p, pp, ppp_in), qq = s_mul(c1, p.x, px(p.x), pp, ppp_in);
  Half r;
  r.x = reduce8<FqPn>(subk<FqPn, 6>(r2, add_lazy(add_lazy(ppp, qq), qq)));
  const Fe qx2 = subk<FqPn, 2>(qq, r.x);
  const Fe ny = subk<FqPn, 2>(fe_zero(), p.y);
  const Fe qx2p = px(qx2), nyp = px(ny), pppp = px(ppp);
  // c0 = rr0 qx0 + rr1 (-qx1) + ny0 ppp0 + ny1 (-ppp1); c1 = rr0 qx1 + rr1 qx0 + ny0 ppp1 + ny1 ppp0
  r.y = mul4<FqPn>(sel(c1, rrp, rr), qx2, sel(c1, rr, rrp), sel(c1, qx2p, subk<FqPn, 4>(fe_zero(), qx2p)),
                   sel(c1, nyp, ny), ppp, sel(c1, ny, nyp), sel(c1, pppp, subk<FqPn, 2>(fe_zero(), pppp)));
  r.zz = s_mul(c1, p.zz, zzp, pp, ppp_in);
  r.zzz = s_mul(c1, p.zzz, zzzp, ppp, pppp);
  return r;
}
template <int MINW>
__global__ void __launch_bounds__(256, MINW) k_split(uint32_t* out, int iters) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x, b = t >> 1;
  const int c = (int)(t & 1);
  const bool c1 = c == 1;
  Half v{in_of(b, 0, c), in_of(b, 1, c), in_of(b, 2, c), in_of(b, 3, c)};
  Fe qx = in_of(b, 4, c), qy = in_of(b, 5, c);
  for (int i = 0; i < iters; i++) {
    v = s_madd(c1, v, qx, qy);
    if (!c1) qx.v[0] ^= (uint32_t)i & 7u;
  }
  uint32_t* o = out + (size_t)b * 72;
  const Fe* f[4] = {&v.x, &v.y, &v.zz, &v.zzz};
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < NL; i++) o[(2 * k + c) * 9 + i] = f[k]->v[i];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  const int blocks1 = 256 * 8;  // one-lane: 2048 x 256 buckets
  const size_t nb = (size_t)blocks1 * 256;
  uint32_t *d1, *d2;
  CHECK(hipMalloc(&d1, nb * 72 * 4));
  CHECK(hipMalloc(&d2, nb * 72 * 4));
  hipEvent_t ev0, ev1;
  CHECK(hipEventCreate(&ev0));
  CHECK(hipEventCreate(&ev1));
  auto run = [&](auto kern, int blocks, uint32_t* d, const char* name) {
    kern<<<blocks, 256>>>(d, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
      CHECK(hipEventRecord(ev0));
      kern<<<blocks, 256>>>(d, iters);
      CHECK(hipEventRecord(ev1));
      CHECK(hipEventSynchronize(ev1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, ev0, ev1));
      if (ms < best) best = ms;
    }
    printf("%-28s %8.3f ms  %7.3f G madd/s\n", name, best, (double)nb * iters / best / 1e6);
  };
  run(k_one, blocks1, d1, "one lane per bucket");
  run(k_split<2>, 2 * blocks1, d2, "two-lane split (minw 2)");
  uint32_t* h1 = (uint32_t*)malloc(nb * 72 * 4);
  uint32_t* h2 = (uint32_t*)malloc(nb * 72 * 4);
  CHECK(hipMemcpy(h1, d1, nb * 72 * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h2, d2, nb * 72 * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < nb * 72; i++) bad += h1[i] != h2[i];
  printf("split vs one lane: %zu of %zu words differ\n", bad, nb * 72);
  run(k_split<3>, 2 * blocks1, d2, "two-lane split (minw 3)");
  run(k_split<4>, 2 * blocks1, d2, "two-lane split (minw 4)");
  return bad ? 1 : 0;
}
