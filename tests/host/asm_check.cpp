// Host check of the staged Groth16 assembly (msm_host.cpp groth16_asm_*):
// A, B, C must equal ark-groth16's formula evaluated step by step --
//   A = r d1 + a0 + a + alpha,  B = s d2 + b2_0 + b2 + beta2,
//   B1 = s d1 + b1_0 + b1 + beta1 (0 when r = 0),  C = s A + r B1 - r (s d1) + l + h
// -- with plain double-and-add products, for random keys / MSM results,
// r = 0, s = 0, r = 1 and MSM results at infinity, through both the one-call
// wrapper and the per-key table path.  Prints "ok <n>".
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../zelana_amd/csrc/host_field.h"
#include "../../zelana_amd/csrc/zkmi_internal_host.h"

using namespace zkh;
using zk::Xyzz;

static uint64_t rng = 0x243F6A8885A308D3ull;
static uint64_t next() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}
template <class F>
static Xyzz<F> mul(Xyzz<F> p, const uint64_t k[4]) {
  Xyzz<F> acc = zk::xyzz_inf<F>();
  for (int b = 255; b >= 0; b--) {
    acc = zk::xyzz_dbl(acc);
    if ((k[b / 64] >> (b % 64)) & 1) acc = zk::xyzz_add(acc, p);
  }
  return acc;
}
static void aff1(const Xyzz<HFq>& p, uint64_t o[8]) {
  if (zk::xyzz_is_inf(p)) {
    memset(o, 0, 64);
    return;
  }
  to_canon(o, fmul(p.x, finv(p.zz)));
  to_canon(o + 4, fmul(p.y, finv(p.zzz)));
}
static void aff2(const Xyzz<HFq2>& p, uint64_t o[16]) {
  if (zk::xyzz_is_inf(p)) {
    memset(o, 0, 128);
    return;
  }
  F42 x = HFq2::mul(p.x, HFq2::inv(p.zz)), y = HFq2::mul(p.y, HFq2::inv(p.zzz));
  to_canon(o, x.c0);
  to_canon(o + 4, x.c1);
  to_canon(o + 8, y.c0);
  to_canon(o + 12, y.c1);
}
static Xyzz<HFq> pt1(const uint64_t a[8]) {
  bool z = true;
  for (int i = 0; i < 8; i++) z &= a[i] == 0;
  if (z) return zk::xyzz_inf<HFq>();
  return zk::xyzz_from_aff(zk::Aff<HFq>{from_canon(a), from_canon(a + 4)});
}
static Xyzz<HFq2> pt2(const uint64_t a[16]) {
  bool z = true;
  for (int i = 0; i < 16; i++) z &= a[i] == 0;
  if (z) return zk::xyzz_inf<HFq2>();
  return zk::xyzz_from_aff(
      zk::Aff<HFq2>{{from_canon(a), from_canon(a + 4)}, {from_canon(a + 8), from_canon(a + 12)}});
}
static void scalar(uint64_t k[4]) {
  for (int i = 0; i < 4; i++) k[i] = next();
  k[3] &= 0x0fffffffffffffffull;  // < 2^252 < r
}

int main() {
  const uint64_t g1[8] = {1, 0, 0, 0, 2, 0, 0, 0};
  const uint64_t g2[16] = {0x46debd5cd992f6edULL, 0x674322d4f75edaddULL, 0x426a00665e5c4479ULL, 0x1800deef121f1e76ULL,
                           0x97e485b7aef312c2ULL, 0xf1aa493335a9e712ULL, 0x7260bfb731fb5d25ULL, 0x198e9393920d483aULL,
                           0x4ce6cc0166fa7daaULL, 0xe3d1e7690c43d37bULL, 0x4aab71808dcb408fULL, 0x12c85ea5db8c6debULL,
                           0x55acdadcd122975bULL, 0xbc4b313370b38ef3ULL, 0xec9e99ad690c3395ULL, 0x090689d0585ff075ULL};
  const Xyzz<HFq> G1 = pt1(g1);
  const Xyzz<HFq2> G2 = pt2(g2);
  int n = 0, bad = 0;
  for (int t = 0; t < 6; t++) {
    // key and MSM results: random multiples of the generators (t = 5: MSMs at infinity)
    uint64_t P1[9][8], P2[4][16], k[4];
    for (int i = 0; i < 9; i++) {
      scalar(k);
      aff1(t == 5 && i >= 4 ? zk::xyzz_inf<HFq>() : mul(G1, k), P1[i]);
    }
    for (int i = 0; i < 4; i++) {
      scalar(k);
      aff2(t == 5 && i >= 3 ? zk::xyzz_inf<HFq2>() : mul(G2, k), P2[i]);
    }
    const uint64_t *alpha = P1[0], *beta1 = P1[1], *d1 = P1[2], *a0 = P1[3], *b10 = P1[4], *h = P1[5], *l = P1[6],
                   *a = P1[7], *b1 = P1[8];
    const uint64_t *beta2 = P2[0], *d2 = P2[1], *b20 = P2[2], *b2 = P2[3];
    std::vector<uint64_t> tab1(zk::groth16_asm_table_words(0)), tab2(zk::groth16_asm_table_words(1));
    zk::groth16_asm_tables(d1, d2, tab1.data(), tab2.data());
    uint64_t r[4], s[4];
    for (int c = 0; c < 5; c++) {
      scalar(r);
      scalar(s);
      if (c == 1) memset(r, 0, 32);
      if (c == 2) memset(s, 0, 32);
      if (c == 3) r[0] = 1, r[1] = r[2] = r[3] = 0;
      // ark-groth16, step by step
      Xyzz<HFq> A = zk::xyzz_add(zk::xyzz_add(zk::xyzz_add(mul(pt1(d1), r), pt1(a0)), pt1(a)), pt1(alpha));
      Xyzz<HFq2> B = zk::xyzz_add(zk::xyzz_add(zk::xyzz_add(mul(pt2(d2), s), pt2(b20)), pt2(b2)), pt2(beta2));
      Xyzz<HFq> B1 = zk::xyzz_inf<HFq>();
      if (r[0] | r[1] | r[2] | r[3])
        B1 = zk::xyzz_add(zk::xyzz_add(zk::xyzz_add(mul(pt1(d1), s), pt1(b10)), pt1(b1)), pt1(beta1));
      uint64_t eA[8], eB[16], eC[8], sd[8], B1a[8];
      aff1(A, eA);
      aff2(B, eB);
      aff1(B1, B1a);
      aff1(mul(pt1(d1), s), sd);
      Xyzz<HFq> rsd = mul(pt1(sd), r);
      rsd.y = HFq::neg(rsd.y);
      Xyzz<HFq> C = zk::xyzz_add(mul(pt1(eA), s), mul(pt1(B1a), r));
      C = zk::xyzz_add(zk::xyzz_add(zk::xyzz_add(C, rsd), pt1(l)), pt1(h));
      aff1(C, eC);
      // the product's two paths
      uint64_t oA[8], oB[16], oC[8];
      zk::groth16_assemble(alpha, beta1, d1, beta2, d2, a0, b10, b20, h, l, a, b1, b2, r, s, oA, oB, oC);
      bad += memcmp(oA, eA, 64) || memcmp(oB, eB, 128) || memcmp(oC, eC, 64);
      zk::G16Asm st;
      zk::groth16_asm_fixed_tab(tab1.data(), tab2.data(), r, s, &st);
      zk::groth16_asm_ab(alpha, beta1, a0, b10, a, b1, r, s, &st);
      zk::groth16_asm_b(beta2, b20, b2, &st, oB);
      zk::groth16_asm_c(l, h, &st, oA, oC);
      bad += memcmp(oA, eA, 64) || memcmp(oB, eB, 128) || memcmp(oC, eC, 64);
      n += 2;
    }
  }
  if (bad) {
    printf("FAIL %d of %d\n", bad, n);
    return 1;
  }
  printf("ok %d\n", n);
  return 0;
}
