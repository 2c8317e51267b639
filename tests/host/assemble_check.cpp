// Host check of the sharded-MSM epilogue (msm_host.cpp
// msm_host_assemble_combine, what msm_wait runs on every rank's exchanged
// payload): window shards placed at their global windows and point shards
// summed term by term must give the one-rank result -- G1 and G2, uneven
// window splits, several segments per term, a rank whose terms are all at
// infinity.  The multi-rank hardware path is the driver's; this pins the
// host side of it on the CPU.  Prints "ok <n>".
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../zelana_amd/csrc/host_field.h"
#include "../../zelana_amd/csrc/zkmi_internal_host.h"

using namespace zkh;
using zk::Xyzz;

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}
template <class F>
static Xyzz<F> mul(Xyzz<F> p, uint64_t k) {
  Xyzz<F> acc = zk::xyzz_inf<F>();
  for (int b = 63; b >= 0; b--) {
    acc = zk::xyzz_dbl(acc);
    if ((k >> b) & 1) acc = zk::xyzz_add(acc, p);
  }
  return acc;
}
static void put_f(uint32_t* w, const F4& a) {
  uint64_t c[4];
  to_canon(c, a);
  for (int i = 0; i < 4; i++) w[2 * i] = (uint32_t)c[i], w[2 * i + 1] = (uint32_t)(c[i] >> 32);
}
static void put_f(uint32_t* w, const F42& a) {
  put_f(w, a.c0);
  put_f(w + 8, a.c1);
}
template <class F, int CW>
static void put_term(uint32_t* w, const Xyzz<F>& p) {  // canonical packed XYZZ (all-zero = infinity)
  if (zk::xyzz_is_inf(p)) {
    memset(w, 0, 4 * CW * 4);
    return;
  }
  put_f(w, p.x);
  put_f(w + CW, p.y);
  put_f(w + 2 * CW, p.zz);
  put_f(w + 3 * CW, p.zzz);
}

template <class F, int CW>
static int run(const Xyzz<F>& G, int g2, int c, int W, int sb) {
  const int bb = c - 1, XW = 4 * CW, nt = W * (bb + 1);  // terms per rank
  const size_t TW = (size_t)XW * sb, skip = 4;
  int bad = 0;
  // every term segment a random multiple of G (some at infinity)
  std::vector<Xyzz<F>> A(nt * sb), B(nt * sb);
  for (auto& p : A) p = next() % 7 == 0 ? zk::xyzz_inf<F>() : mul(G, next() >> 8);
  for (auto& p : B) p = next() % 7 == 0 ? zk::xyzz_inf<F>() : mul(G, next() >> 8);
  auto payload = [&](std::vector<uint32_t>& buf, size_t stride, int r, int w0, int wn,
                     const std::vector<Xyzz<F>>& t) {
    uint32_t* s = buf.data() + (size_t)r * stride;
    s[3] = ((uint32_t)w0 << 16) | (uint32_t)wn;
    for (int w = 0; w < wn; w++)
      for (int j = 0; j <= bb; j++)
        for (int g = 0; g < sb; g++)
          put_term<F, CW>(s + skip + ((size_t)w * (bb + 1) + j) * TW + (size_t)g * XW,
                          t[((size_t)(w0 + w) * (bb + 1) + j) * sb + g]);
  };
  const size_t stride = skip + (size_t)nt * TW;
  const int one[1] = {0};
  // reference: one rank, terms A
  std::vector<uint32_t> ref(stride, 0);
  payload(ref, stride, 0, 0, W, A);
  uint64_t want[16], got[16];
  zk::msm_host_assemble_combine(ref.data(), stride, skip, one, 1, false, g2, c, W, bb, sb, want);
  // window shards: uneven splits over 3 ranks (and 4 ranks with one empty)
  for (int split = 0; split < 2; split++) {
    const int nr = split ? 4 : 3;
    std::vector<uint32_t> buf((size_t)nr * stride, 0);
    std::vector<int> live;
    for (int r = 0; r < nr; r++) {
      int w0 = split ? (r == 0 ? 0 : (r - 1) * W / 3) : r * W / nr;
      int w1 = split ? (r == 0 ? 0 : r * W / 3) : (r + 1) * W / nr;
      if (w1 > w0) live.push_back(r);
      payload(buf, stride, r, w0, w1 - w0, A);
    }
    zk::msm_host_assemble_combine(buf.data(), stride, skip, live.data(), (int)live.size(), true, g2, c, W, bb, sb,
                                  got);
    bad += memcmp(got, want, (g2 ? 16 : 8) * 8) != 0;
  }
  // point shards: ranks with terms A and B against one rank with A + B
  {
    std::vector<Xyzz<F>> S(nt * sb);
    for (size_t i = 0; i < S.size(); i++) S[i] = zk::xyzz_add(A[i], B[i]);
    std::vector<uint32_t> one_rank(stride, 0), two((size_t)2 * stride, 0);
    payload(one_rank, stride, 0, 0, W, S);
    payload(two, stride, 0, 0, W, A);
    payload(two, stride, 1, 0, W, B);
    const int both[2] = {0, 1};
    zk::msm_host_assemble_combine(one_rank.data(), stride, skip, one, 1, false, g2, c, W, bb, sb, want);
    zk::msm_host_assemble_combine(two.data(), stride, skip, both, 2, false, g2, c, W, bb, sb, got);
    bad += memcmp(got, want, (g2 ? 16 : 8) * 8) != 0;
  }
  return bad;
}

int main() {
  const uint64_t g1[8] = {1, 0, 0, 0, 2, 0, 0, 0};
  const uint64_t g2[16] = {0x46debd5cd992f6edULL, 0x674322d4f75edaddULL, 0x426a00665e5c4479ULL, 0x1800deef121f1e76ULL,
                           0x97e485b7aef312c2ULL, 0xf1aa493335a9e712ULL, 0x7260bfb731fb5d25ULL, 0x198e9393920d483aULL,
                           0x4ce6cc0166fa7daaULL, 0xe3d1e7690c43d37bULL, 0x4aab71808dcb408fULL, 0x12c85ea5db8c6debULL,
                           0x55acdadcd122975bULL, 0xbc4b313370b38ef3ULL, 0xec9e99ad690c3395ULL, 0x090689d0585ff075ULL};
  const Xyzz<HFq> G1 = zk::xyzz_from_aff(zk::Aff<HFq>{from_canon(g1), from_canon(g1 + 4)});
  const Xyzz<HFq2> G2 =
      zk::xyzz_from_aff(zk::Aff<HFq2>{{from_canon(g2), from_canon(g2 + 4)}, {from_canon(g2 + 8), from_canon(g2 + 12)}});
  int bad = 0, n = 0;
  bad += run<HFq, 8>(G1, 0, 4, 5, 2), n += 3;
  bad += run<HFq, 8>(G1, 0, 3, 7, 1), n += 3;
  bad += run<HFq2, 16>(G2, 1, 4, 4, 2), n += 3;
  if (bad) {
    printf("FAIL %d of %d\n", bad, n);
    return 1;
  }
  printf("ok %d\n", n);
  return 0;
}
