// Host build of the device field/curve code (ff.h / ec.h are host+device):
// the lazy G1 mixed addition xyzz_madd_g1 must give the same group element
// as the reference-form xyzz_madd over long accumulation chains (and so must
// the msm.hip acc_step rule: second point by the affine + affine xyzz_mmadd_*), including
// P == Q, P == -Q, lazy X inputs and negated bases.  Prints "ok <n>".
#include <stdio.h>
#include <stdlib.h>

#include "../../zelana_amd/csrc/ec.h"

using namespace zk;
using F = FqOps;

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}
static Fe inv(const Fe& a) {
  const uint64_t e[4] = {0x3c208c16d87cfd45ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull};
  return pow<FqP>(a, e);
}
static Aff<F> to_aff(const Xyzz<F>& p) {
  Fe t = inv(mul<FqP>(p.zz, p.zzz));
  Aff<F> a;
  a.x = reduce<FqP>(reduce8<FqP>(mul<FqP>(p.x, mul<FqP>(t, p.zzz))));
  a.y = reduce<FqP>(mul<FqP>(p.y, mul<FqP>(t, p.zz)));
  return a;
}
static bool same(const Xyzz<F>& a, const Xyzz<F>& b) {
  bool ia = xyzz_is_inf(a), ib = xyzz_is_inf(b);
  if (ia || ib) return ia == ib;
  Aff<F> x = to_aff(a), y = to_aff(b);
  for (int i = 0; i < NL; i++)
    if (x.x.v[i] != y.x.v[i] || x.y.v[i] != y.y.v[i]) return false;
  return true;
}

// G2 (Fq2) chains: xyzz_madd_g2 vs the generic formula over Fq2Ops
static const uint32_t G2GEN[32] = {
    0xd992f6edu, 0x46debd5cu, 0xf75edaddu, 0x674322d4u, 0x5e5c4479u, 0x426a0066u, 0x121f1e76u, 0x1800deefu,
    0xaef312c2u, 0x97e485b7u, 0x35a9e712u, 0xf1aa4933u, 0x31fb5d25u, 0x7260bfb7u, 0x920d483au, 0x198e9393u,
    0x66fa7daau, 0x4ce6cc01u, 0x0c43d37bu, 0xe3d1e769u, 0x8dcb408fu, 0x4aab7180u, 0xdb8c6debu, 0x12c85ea5u,
    0xd122975bu, 0x55acdadcu, 0x70b38ef3u, 0xbc4b3133u, 0x690c3395u, 0xec9e99adu, 0x585ff075u, 0x090689d0u};
using F2 = Fq2Ops;
static Fe2 inv2(const Fe2& a) {
  Fe nrm = add<FqP>(sqr<FqP>(a.c0), sqr<FqP>(a.c1));
  Fe ni = inv(nrm);
  return Fe2{mul<FqP>(a.c0, ni), neg<FqP>(mul<FqP>(a.c1, ni))};
}
static Aff<F2> to_aff2(const Xyzz<F2>& p) {
  Fe2 t = inv2(f2_mul(p.zz, p.zzz));
  Fe2 x = f2_mul(p.x, f2_mul(t, p.zzz)), y = f2_mul(p.y, f2_mul(t, p.zz));
  Aff<F2> a;
  a.x = {reduce<FqP>(x.c0), reduce<FqP>(x.c1)};
  a.y = {reduce<FqP>(y.c0), reduce<FqP>(y.c1)};
  return a;
}
static bool same2(const Xyzz<F2>& a, const Xyzz<F2>& b) {
  bool ia = xyzz_is_inf(a), ib = xyzz_is_inf(b);
  if (ia || ib) return ia == ib;
  Aff<F2> x = to_aff2(a), y = to_aff2(b);
  for (int i = 0; i < NL; i++)
    if (x.x.c0.v[i] != y.x.c0.v[i] || x.x.c1.v[i] != y.x.c1.v[i] || x.y.c0.v[i] != y.y.c0.v[i] ||
        x.y.c1.v[i] != y.y.c1.v[i])
      return false;
  return true;
}
static int check_g2() {
  Aff<F2> g;
  g.x = {to_mont<FqP>(unpack(G2GEN)), to_mont<FqP>(unpack(G2GEN + 8))};
  g.y = {to_mont<FqP>(unpack(G2GEN + 16)), to_mont<FqP>(unpack(G2GEN + 24))};
  const int NP = 12;
  Aff<F2> pts[NP];
  for (int i = 0; i < NP; i++) {
    Xyzz<F2> acc = xyzz_inf<F2>();
    uint64_t k = next() | 1;
    for (int b = 63; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      if ((k >> b) & 1) acc = xyzz_madd(acc, g);
    }
    pts[i] = to_aff2(acc);
  }
  int checks = 0;
  for (int trial = 0; trial < 60; trial++) {
    Xyzz<F2> a = xyzz_inf<F2>(), b = xyzz_inf<F2>(), c = xyzz_inf<F2>();
    bool naff = false;
    auto step = [&](const Aff<F2>& q) {
      if (xyzz_is_inf(c)) {
        c = xyzz_from_aff(q);
        naff = true;
      } else if (naff) {
        c = xyzz_mmadd_g2({c.x, c.y}, q);
        naff = false;
      } else {
        c = xyzz_madd_g2(c, q);
      }
    };
    int len = 1 + (int)(next() % 24), prev = -1;
    for (int s = 0; s < len; s++) {
      int j = (int)(next() % NP);
      bool neg_ = next() & 1;
      uint64_t mode = next() % 6;
      if (mode == 0 && prev >= 0) j = prev;
      Aff<F2> qa = pts[j], qb = pts[j];
      if (neg_) qa.y = f2_neg(qa.y);
      qb.y = {fq_cneg(qb.y.c0, neg_), fq_cneg(qb.y.c1, neg_)};
      a = xyzz_madd(a, qa);
      b = xyzz_madd_g2(b, qb);
      step(qb);
      if (mode == 1) {
        Aff<F2> na = qa, nb = pts[j];
        na.y = f2_neg(qa.y);
        nb.y = {fq_cneg(nb.y.c0, !neg_), fq_cneg(nb.y.c1, !neg_)};
        a = xyzz_madd(a, na);
        b = xyzz_madd_g2(b, nb);
        step(nb);
      }
      prev = j;
      if (!same2(a, b) || !same2(a, c)) {
        printf("G2 mismatch trial %d step %d\n", trial, s);
        return -1;
      }
      checks++;
    }
    Aff<F2> q = pts[trial % NP];
    if (!same2(xyzz_madd_g2(xyzz_from_aff(q), q), xyzz_mdbl(q)) || !same2(xyzz_mmadd_g2(q, q), xyzz_mdbl(q))) {
      printf("G2 doubling mismatch\n");
      return -1;
    }
    {
      Xyzz<F2> other = xyzz_madd(xyzz_madd(xyzz_inf<F2>(), pts[(trial + 3) % NP]), pts[(trial + 5) % NP]);
      Xyzz<F2> neg_a = a;
      neg_a.y = f2_neg(a.y);
      if (!same2(xyzz_add_g2(a, other), xyzz_add(a, other)) || !same2(xyzz_add_g2(a, a), xyzz_add(a, a)) ||
          !xyzz_is_inf(xyzz_add_g2(a, neg_a)) != !xyzz_is_inf(xyzz_add(a, neg_a)) ||
          !same2(xyzz_add_g2(xyzz_inf<F2>(), other), other)) {
        printf("G2 full add mismatch trial %d\n", trial);
        return -1;
      }
    }
    Aff<F2> nq = q, w = pts[(trial + 1) % NP];
    nq.y = {fq_cneg(q.y.c0, true), fq_cneg(q.y.c1, true)};
    if (!xyzz_is_inf(xyzz_mmadd_g2(q, nq)) || !same2(xyzz_mmadd_g2(q, w), xyzz_madd(xyzz_from_aff(q), w))) {
      printf("G2 mmadd mismatch\n");
      return -1;
    }
  }
  return checks;
}

// reduce_q32 (one-pass [0, 32p) -> [0, 2p)) on x = k p + e for every k < 32,
// e in {0, 1, p - 1, random}: the result is < 2p and congruent to e.
template <class P>
static bool check_reduce_q32() {
  for (uint32_t k = 0; k < 32; k++) {
    for (int kind = 0; kind < 8; kind++) {
      Fe e = fe_zero();
      if (kind == 1) e.v[0] = 1;
      if (kind == 2) {  // p - 1
        e = fe_const<P>(P::P);
        e.v[0] -= 1;
      }
      if (kind >= 3) {  // random < p: random limbs, top limb below p's
        for (int i = 0; i < NL; i++) e.v[i] = (uint32_t)next() & LMASK;
        e.v[NL - 1] %= P::P[NL - 1];
      }
      Fe x;
      uint64_t c = 0;
      for (int i = 0; i < NL; i++) {
        uint64_t t = (uint64_t)k * P::P[i] + e.v[i] + c;
        x.v[i] = (uint32_t)t & LMASK;
        c = t >> 29;
      }
      x.v[NL - 1] += (uint32_t)(c << 29);
      if (kind >= 6) {  // same value, unnormalised limbs (< 2^31) as limb-wise sums leave them
        for (int i = 0; i < NL - 1; i++) {
          const uint32_t mv = (x.v[i + 1] > 3) ? 3 : x.v[i + 1];
          x.v[i] += mv << 29;
          x.v[i + 1] -= mv;
        }
      }
      Fe r = reduce_q32<P>(x);
      Fe two = fe_const<P>(P::P2);
      // r < 2p: compare from the top limb
      int cmp = 0;
      for (int i = NL - 1; i >= 0 && !cmp; i--) cmp = r.v[i] < two.v[i] ? -1 : r.v[i] > two.v[i] ? 1 : 0;
      Fe a = reduce<P>(r), b = reduce<P>(e);
      bool same_ = true;
      for (int i = 0; i < NL; i++) same_ = same_ && a.v[i] == b.v[i] && r.v[i] <= LMASK;
      if (cmp >= 0 || !same_) {
        printf("reduce_q32 mismatch k=%u kind=%d\n", k, kind);
        return false;
      }
    }
  }
  return true;
}

int main() {
  if (!check_reduce_q32<FqP>() || !check_reduce_q32<FrP>()) return 1;
  Aff<F> g;
  g.x = to_mont<FqP>(Fe{{1, 0, 0, 0, 0, 0, 0, 0, 0}});
  g.y = to_mont<FqP>(Fe{{2, 0, 0, 0, 0, 0, 0, 0, 0}});
  // table of random affine points k*G
  const int NP = 24;
  Aff<F> pts[NP];
  for (int i = 0; i < NP; i++) {
    Xyzz<F> acc = xyzz_inf<F>();
    uint64_t k = next() | 1;
    for (int b = 63; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      if ((k >> b) & 1) acc = xyzz_madd(acc, g);
    }
    pts[i] = to_aff(acc);
  }
  int checks = 0;
  for (int trial = 0; trial < 200; trial++) {
    Xyzz<F> a = xyzz_inf<F>(), b = xyzz_inf<F>(), c = xyzz_inf<F>(), df = xyzz_inf<F>();
    int dphase = 0;  // acc_items_g1 rule: 0 empty, 1 one affine point, 2 xyzz_madd_g1f
    // y of a base as the one-lane-per-bucket G1 kernel feeds it: borrow-form 2p - y
    // (limb-wise, unnormalised) for a negative digit
    auto dstep = [&](const Aff<F>& q, bool ng) {
      const Fe y = ng ? bsub(FqP::B2_1, q.y) : q.y;
      if (dphase == 0) {
        df = xyzz_from_aff(Aff<F>{q.x, reduce_q32<FqP>(y)});
        dphase = 1;
      } else if (dphase == 1) {
        df = xyzz_mmadd_g1({df.x, df.y}, Aff<F>{q.x, reduce_q32<FqP>(y)});
        dphase = xyzz_is_inf(df) ? 0 : 2;
      } else {
        bool inf = false;
        df = xyzz_madd_g1f(df, q.x, y, &inf);
        if (inf) dphase = 0;
      }
    };
    bool naff = false;  // msm.hip acc_step: first point as is, second by xyzz_mmadd_g1
    auto step = [&](const Aff<F>& q) {
      if (xyzz_is_inf(c)) {
        c = xyzz_from_aff(q);
        naff = true;
      } else if (naff) {
        c = xyzz_mmadd_g1({c.x, c.y}, q);
        naff = false;
      } else {
        c = xyzz_madd_g1(c, q);
      }
    };
    int len = 1 + (int)(next() % 40);
    int prev = -1;
    for (int s = 0; s < len; s++) {
      int j = (int)(next() % NP);
      bool neg_ = next() & 1;
      uint64_t mode = next() % 8;
      if (mode == 0 && prev >= 0) j = prev;  // repeated base
      Aff<F> q = pts[j];
      Aff<F> qa = q;
      if (neg_) qa.y = neg<FqP>(q.y);
      Aff<F> qb = q;
      qb.y = fq_cneg(q.y, neg_);
      a = xyzz_madd(a, qa);
      b = xyzz_madd_g1(b, qb);
      step(qb);
      dstep(q, neg_);
      if (mode == 1) {  // cancel: add -Q right after Q
        Aff<F> na = qa, nb = q;
        na.y = neg<FqP>(qa.y);
        nb.y = fq_cneg(q.y, !neg_);
        a = xyzz_madd(a, na);
        b = xyzz_madd_g1(b, nb);
        step(nb);
        dstep(q, !neg_);
      }
      prev = j;
      if (!same(a, b) || !same(a, c) || !same(a, df)) {
        printf("mismatch trial %d step %d\n", trial, s);
        return 1;
      }
      checks++;
    }
    // a run that is exactly Q + Q (doubling) and Q + (-Q) (infinity)
    Xyzz<F> d = xyzz_madd_g1(xyzz_from_aff(pts[trial % NP]), pts[trial % NP]);
    if (!same(d, xyzz_mdbl(pts[trial % NP]))) {
      printf("doubling mismatch\n");
      return 1;
    }
    Aff<F> n = pts[trial % NP];
    n.y = fq_cneg(n.y, true);
    if (!xyzz_is_inf(xyzz_madd_g1(xyzz_from_aff(pts[trial % NP]), n))) {
      printf("cancel mismatch\n");
      return 1;
    }
    // full additions (bucket reductions): lazy form vs the generic formula,
    // on chain values with non-trivial ZZ, including P + P and P + (-P)
    {
      Xyzz<F> other = xyzz_madd(xyzz_madd(xyzz_inf<F>(), pts[(trial + 3) % NP]), pts[(trial + 5) % NP]);
      Xyzz<F> neg_a = a;
      neg_a.y = neg<FqP>(a.y);
      if (!same(xyzz_add_g1(a, other), xyzz_add(a, other)) || !same(xyzz_add_g1(a, a), xyzz_add(a, a)) ||
          !xyzz_is_inf(xyzz_add_g1(a, neg_a)) != !xyzz_is_inf(xyzz_add(a, neg_a)) ||
          !same(xyzz_add_g1(xyzz_inf<F>(), other), other) || !same(xyzz_add_g1(other, xyzz_inf<F>()), other)) {
        printf("full add mismatch trial %d\n", trial);
        return 1;
      }
    }
    // xyzz_madd_g1f on a multi-point accumulator: + itself (doubling), + its
    // negation (borrow-form y: infinity), and the output bounds
    if (dphase == 2) {
      Aff<F> s = to_aff(df);
      bool inf = true;
      Xyzz<F> dd = xyzz_madd_g1f(df, s.x, s.y, &inf);
      if (inf || !same(dd, xyzz_mdbl(s))) {
        printf("madd_g1f doubling mismatch trial %d\n", trial);
        return 1;
      }
      xyzz_madd_g1f(df, s.x, bsub(FqP::B2_1, s.y), &inf);
      const Fe p8 = fe_const<FqP>(FqP::P8), p2 = fe_const<FqP>(FqP::P2);
      auto lt = [](const Fe& a, const Fe& b) {
        for (int i = NL - 1; i >= 0; i--)
          if (a.v[i] != b.v[i]) return a.v[i] < b.v[i];
        return false;
      };
      bool norm = true;
      for (int i = 0; i < NL - 1; i++)
        norm = norm && df.x.v[i] <= LMASK && df.y.v[i] <= LMASK && df.zz.v[i] <= LMASK && df.zzz.v[i] <= LMASK;
      if (!inf || !norm || !lt(df.x, p8) || !lt(df.y, p2) || !lt(df.zz, p2) || !lt(df.zzz, p2)) {
        printf("madd_g1f cancellation / bounds mismatch trial %d\n", trial);
        return 1;
      }
    }
    // affine + affine: doubling, cancellation, and the generic case
    const Aff<F>& u = pts[trial % NP];
    const Aff<F>& w = pts[(trial + 1) % NP];
    if (!same(xyzz_mmadd_g1(u, u), xyzz_mdbl(u)) || !xyzz_is_inf(xyzz_mmadd_g1(u, n)) ||
        !same(xyzz_mmadd_g1(u, w), xyzz_madd(xyzz_from_aff(u), w))) {
      printf("mmadd mismatch\n");
      return 1;
    }
  }
  int c2 = check_g2();
  if (c2 < 0) return 1;
  printf("ok %d %d\n", checks, c2);
  return 0;
}
