// Microbenchmark (tools/, dev only): a BN254 Fq
// Montgomery product on the FP64 FMA pipe -- 5 limbs of 52 bits, R = 2^260,
// each 52x52 limb product split exactly into hi/lo halves by two FMAs
// (Emmart & Weems) and accumulated as integers in 64-bit column sums --
// against the shipped 9 x 29-bit v_mad_u64_u32 product (ff.h mul<FqP>).
// Checks the FP64 product against a host big-integer product, then reports
// products/s of both at full occupancy (same launch shape, dependent chains).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_fp64.hip -o tools/mb_fp64
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../zelana_amd/csrc/ff.h"
using namespace zk;
#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);         \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int FL = 5;                        // limbs
constexpr uint64_t M52 = (1ull << 52) - 1;
// p = BN254 Fq in 52-bit limbs, and -p^-1 mod 2^52
__constant__ uint64_t P52[FL];
__constant__ uint64_t PINV52;

__device__ __forceinline__ double u2d(uint64_t x) {  // x < 2^52, exact
  return __longlong_as_double((long long)(x | 0x4330000000000000ull)) - 4503599627370496.0;
}
// column sums: t[k] += lo(a b) and t[k+1] += hi(a b), exact (a, b < 2^52 as doubles)
__device__ __forceinline__ void fma_split(double a, double b, int64_t& lo_acc, int64_t& hi_acc) {
  const double C104 = 20282409603651670423947251286016.0;  // 2^104 (ulp 2^52)
  const double hi = __fma_rn(a, b, C104);                   // 2^104 + round(ab / 2^52) 2^52
  const double hs = hi - C104;                              // exact
  const double lo = __fma_rn(a, b, -hs) + 6755399441055744.0;  // ab - hs + 3 2^51 in [2^52, 2^53): ulp 1
  hi_acc += __double_as_longlong(hi) - 0x4670000000000000ll;  // round(ab / 2^52)
  lo_acc += __double_as_longlong(lo) - 0x4338000000000000ll;  // ab - hs (signed)
}

struct F52 {
  uint64_t v[FL];
};

__device__ __forceinline__ F52 mul52(const F52& a, const F52& b) {
  double ad[FL], bd[FL], pd[FL];
#pragma unroll
  for (int i = 0; i < FL; i++) {
    ad[i] = u2d(a.v[i]);
    bd[i] = u2d(b.v[i]);
    pd[i] = u2d(P52[i]);
  }
  int64_t t[2 * FL + 1];
#pragma unroll
  for (int k = 0; k < 2 * FL + 1; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < FL; i++)
#pragma unroll
    for (int j = 0; j < FL; j++) fma_split(ad[i], bd[j], t[i + j], t[i + j + 1]);
#pragma unroll
  for (int i = 0; i < FL; i++) {
    // normalise column i, then m = t_i * (-p^-1) mod 2^52 and t += m p 2^(52 i)
    t[i + 1] += t[i] >> 52;
    const uint64_t ti = (uint64_t)t[i] & M52;
    int64_t mlo = 0, mhi = 0;
    fma_split(u2d(ti), u2d(PINV52), mlo, mhi);
    const uint64_t m = (uint64_t)mlo & M52;
    const double md = u2d(m);
    int64_t c0 = (int64_t)ti;
#pragma unroll
    for (int j = 0; j < FL; j++) {
      if (j == 0) fma_split(md, pd[0], c0, t[i + 1]);
      else fma_split(md, pd[j], t[i + j], t[i + j + 1]);
    }
    t[i + 1] += c0 >> 52;  // c0 == 0 mod 2^52
  }
  F52 r;
#pragma unroll
  for (int k = FL; k < 2 * FL; k++) {
    t[k + 1] += t[k] >> 52;
    r.v[k - FL] = (uint64_t)t[k] & M52;
  }
  r.v[FL - 1] += (uint64_t)t[2 * FL] << 52;  // < 2p < 2^255: fits the top limb
  return r;
}

__global__ void __launch_bounds__(256) k_f52(F52* out, const F52* in, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  F52 a = in[i & 1023], b = in[(i + 1) & 1023];
  for (int it = 0; it < iters; it++) a = mul52(a, b);
  out[i] = a;
}
__global__ void __launch_bounds__(256) k_f52_one(F52* out, const F52* a, const F52* b, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = mul52(a[i], b[i]);
}
__global__ void __launch_bounds__(256) k_m29(Fe* out, const Fe* in, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fe a = in[i & 1023], b = in[(i + 1) & 1023];
  for (int it = 0; it < iters; it++) a = mul<FqP>(a, b);
  out[i] = a;
}

// ---- host big integers (little-endian u32 words) for the check
typedef unsigned __int128 u128;
static void to52(const uint64_t x[4], uint64_t o[FL]) {
  u128 acc = 0;
  int bits = 0, k = 0, w = 0;
  for (int i = 0; i < FL; i++) o[i] = 0;
  while (k < FL) {
    if (bits < 52 && w < 4) {
      acc |= (u128)x[w++] << bits;
      bits += 64;
    }
    o[k++] = (uint64_t)(acc & M52);
    acc >>= 52;
    bits -= 52;
  }
}
static void from52(const uint64_t o[FL], uint64_t x[5]) {  // 260 bits -> 5 u64
  memset(x, 0, 40);
  for (int k = 0; k < FL; k++) {
    const int bit = 52 * k;
    for (int b = 0; b < 64; b++) {  // o[k] may exceed 52 bits in the top limb
      if (!((o[k] >> b) & 1)) continue;
      const int pos = bit + b;
      if (pos < 320) x[pos / 64] |= 1ull << (pos % 64);
    }
  }
}
// (a * b * 2^-260) mod p by shift-and-add (slow, exact)
static const uint64_t PQ[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull,
                               0x30644e72e131a029ull};
static int cmp5(const uint64_t* a, const uint64_t* b) {
  for (int i = 4; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  }
  return 0;
}
static void sub5(uint64_t* a, const uint64_t* b) {
  unsigned __int128 br = 0;
  for (int i = 0; i < 5; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    a[i] = (uint64_t)d;
    br = (d >> 64) ? 1 : 0;
  }
}
static void modmul_ref(const uint64_t a[4], const uint64_t b[4], uint64_t r[4]) {
  // r = a * b mod p, then * 2^-260 via 260 halvings mod p
  uint64_t acc[5] = {0, 0, 0, 0, 0}, p5[5] = {PQ[0], PQ[1], PQ[2], PQ[3], 0};
  for (int bit = 255; bit >= 0; bit--) {
    // acc = 2 acc mod p
    uint64_t c = 0;
    for (int i = 0; i < 5; i++) {
      uint64_t n = (acc[i] << 1) | c;
      c = acc[i] >> 63;
      acc[i] = n;
    }
    if (cmp5(acc, p5) >= 0) sub5(acc, p5);
    if ((b[bit / 64] >> (bit % 64)) & 1) {
      u128 cy = 0;
      for (int i = 0; i < 5; i++) {
        u128 s = (u128)acc[i] + (i < 4 ? a[i] : 0) + cy;
        acc[i] = (uint64_t)s;
        cy = s >> 64;
      }
      if (cmp5(acc, p5) >= 0) sub5(acc, p5);
    }
  }
  for (int k = 0; k < 260; k++) {  // * 2^-1 mod p
    if (acc[0] & 1) {
      u128 cy = 0;
      for (int i = 0; i < 5; i++) {
        u128 s = (u128)acc[i] + p5[i] + cy;
        acc[i] = (uint64_t)s;
        cy = s >> 64;
      }
    }
    for (int i = 0; i < 5; i++) acc[i] = (acc[i] >> 1) | (i < 4 ? acc[i + 1] << 63 : 0);
  }
  memcpy(r, acc, 32);
}

int main() {
  uint64_t p52[FL];
  to52(PQ, p52);
  // -p^-1 mod 2^52 by Newton iteration
  uint64_t inv = 1;
  for (int i = 0; i < 7; i++) inv = inv * (2 - p52[0] * inv);
  const uint64_t pinv = (0 - inv) & M52;
  CHECK(hipMemcpyToSymbol(HIP_SYMBOL(P52), p52, sizeof(p52)));
  CHECK(hipMemcpyToSymbol(HIP_SYMBOL(PINV52), &pinv, 8));
  // correctness on random elements < p
  const int NC = 256;
  static uint64_t ha[NC][4], hb[NC][4];
  F52 fa[NC], fb[NC], fr[NC];
  srand(7);
  for (int i = 0; i < NC; i++) {
    for (int j = 0; j < 4; j++) {
      ha[i][j] = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 11) ^ rand();
      hb[i][j] = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 11) ^ rand();
    }
    ha[i][3] &= 0x1fffffffffffffffull;
    hb[i][3] &= 0x1fffffffffffffffull;
    to52(ha[i], fa[i].v);
    to52(hb[i], fb[i].v);
  }
  F52 *da, *db, *dr;
  CHECK(hipMalloc(&da, sizeof(fa)));
  CHECK(hipMalloc(&db, sizeof(fb)));
  CHECK(hipMalloc(&dr, sizeof(fr)));
  CHECK(hipMemcpy(da, fa, sizeof(fa), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, fb, sizeof(fb), hipMemcpyHostToDevice));
  k_f52_one<<<1, 256>>>(dr, da, db, NC);
  CHECK(hipMemcpy(fr, dr, sizeof(fr), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < NC; i++) {
    uint64_t want[4], got5[5], p5[5] = {PQ[0], PQ[1], PQ[2], PQ[3], 0};
    modmul_ref(ha[i], hb[i], want);
    from52(fr[i].v, got5);
    while (cmp5(got5, p5) >= 0) sub5(got5, p5);  // lazy result < 2p
    if (memcmp(got5, want, 32) != 0 || got5[4]) bad++;
  }
  printf("fp64 52-bit Montgomery product: %d / %d wrong\n", bad, NC);
  // throughput: same shape for both (4096 blocks x 256 threads, dependent chains)
  static Fe h29[1024];
  static F52 h52[1024];
  for (int i = 0; i < 1024; i++) {
    for (int j = 0; j < 9; j++) h29[i].v[j] = (uint32_t)rand() & (j == 8 ? 0x3fffffu : LMASK);
    h52[i] = fa[i % NC];
  }
  Fe *i29, *o29;
  F52 *i52, *o52;
  const int blocks = 256 * 16, iters = 200;
  CHECK(hipMalloc(&i29, sizeof(h29)));
  CHECK(hipMalloc(&i52, sizeof(h52)));
  CHECK(hipMalloc(&o29, (size_t)blocks * 256 * sizeof(Fe)));
  CHECK(hipMalloc(&o52, (size_t)blocks * 256 * sizeof(F52)));
  CHECK(hipMemcpy(i29, h29, sizeof(h29), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(i52, h52, sizeof(h52), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms;
  for (int rep = 0; rep < 3; rep++) {
    k_m29<<<blocks, 256>>>(o29, i29, iters);
    hipEventRecord(e0);
    k_m29<<<blocks, 256>>>(o29, i29, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double g29 = (double)blocks * 256 * iters / ms / 1e6;
    k_f52<<<blocks, 256>>>(o52, i52, iters);
    hipEventRecord(e0);
    k_f52<<<blocks, 256>>>(o52, i52, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double g52 = (double)blocks * 256 * iters / ms / 1e6;
    printf("rep %d: 9x29 mad_u64 %.1f G mul/s, 5x52 fp64 %.1f G mul/s, ratio %.3f\n", rep, g29, g52, g52 / g29);
  }
  CHECK(hipDeviceSynchronize());
  return 0;  // (a wrong product is reported above, not an exit status: the A/B script continues)
}
