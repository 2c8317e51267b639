// ec.h — BN254 G1 / G2 point arithmetic in XYZZ coordinates (x = X/ZZ,
// y = Y/ZZZ, ZZ^3 = ZZZ^2), host+device, templated over the coordinate field
// (FqOps for G1, Fq2Ops for G2).  XYZZ mixed addition is 8M+2S with no
// inversion, the cheapest formula for Pippenger bucket accumulation; the point
// at infinity is ZZ = ZZZ = 0.  Formulas: EFD "xyzz" a=0 (madd-2008-s,
// add-2008-s, dbl-2008-s-1, mdbl-2008-s-1).  All exceptional cases (P == Q,
// P == -Q, infinity) are handled, so the result equals arkworks' group law
// exactly (parity is point equality: SURVEY.md §8a a7/a8).
#pragma once
#include "ff.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define ZK_HD_NOINLINE __host__ __device__ __noinline__
#else
#define ZK_HD_NOINLINE inline
#endif

namespace zk {


template <class F>
struct Aff {
  typename F::T x, y;
};
template <class F>
struct Xyzz {
  typename F::T x, y, zz, zzz;
};

template <class F>
ZK_HD Xyzz<F> xyzz_inf() {
  Xyzz<F> r;
  r.x = F::zero();
  r.y = F::zero();
  r.zz = F::zero();
  r.zzz = F::zero();
  return r;
}
// Infinity is always materialised as exact zeros (xyzz_inf, zero-filled
// buckets), and a finite point's ZZ is a product of non-zero field elements, so
// a raw all-limbs-zero test is exact and ~3x cheaper than a reduced compare.
template <class F>
ZK_HD bool xyzz_is_inf(const Xyzz<F>& p) {
  return F::is_zero_raw(p.zz);
}
template <class F>
ZK_HD Xyzz<F> xyzz_from_aff(const Aff<F>& a) {
  Xyzz<F> r;
  r.x = a.x;
  r.y = a.y;
  r.zz = F::one();
  r.zzz = F::one();
  return r;
}

// 2 * (affine point) -> XYZZ   (mdbl-2008-s-1)
template <class F>
ZK_HD Xyzz<F> xyzz_mdbl(const Aff<F>& a) {
  using T = typename F::T;
  T u = F::dbl(a.y);
  T v = F::sqr(u);
  T w = F::mul(u, v);
  T s = F::mul(a.x, v);
  T x2 = F::sqr(a.x);
  T m = F::add(F::dbl(x2), x2);
  Xyzz<F> r;
  r.x = F::sub(F::sqr(m), F::dbl(s));
  r.y = F::sub(F::mul(m, F::sub(s, r.x)), F::mul(w, a.y));
  r.zz = v;
  r.zzz = w;
  return r;
}

// 2 * P   (dbl-2008-s-1, a = 0)
template <class F>
ZK_HD Xyzz<F> xyzz_dbl(const Xyzz<F>& p) {
  using T = typename F::T;
  if (xyzz_is_inf(p)) return p;
  T u = F::dbl(p.y);
  T v = F::sqr(u);
  T w = F::mul(u, v);
  T s = F::mul(p.x, v);
  T x2 = F::sqr(p.x);
  T m = F::add(F::dbl(x2), x2);
  Xyzz<F> r;
  r.x = F::sub(F::sqr(m), F::dbl(s));
  r.y = F::sub(F::mul(m, F::sub(s, r.x)), F::mul(w, p.y));
  r.zz = F::mul(v, p.zz);
  r.zzz = F::mul(w, p.zzz);
  return r;
}

// P + Q, Q affine   (madd-2008-s)
template <class F>
ZK_HD Xyzz<F> xyzz_madd(const Xyzz<F>& p, const Aff<F>& q) {
  using T = typename F::T;
  if (xyzz_is_inf(p)) return xyzz_from_aff(q);
  T pp_ = F::sub(F::mul(q.x, p.zz), p.x);   // P
  T rr = F::sub(F::mul(q.y, p.zzz), p.y);   // R
  if (F::is_zero(pp_)) {
    if (F::is_zero(rr)) return xyzz_mdbl(q);
    return xyzz_inf<F>();
  }
  T pp = F::sqr(pp_);
  T ppp = F::mul(pp_, pp);
  T qq = F::mul(p.x, pp);
  Xyzz<F> r;
  r.x = F::sub(F::sub(F::sqr(rr), ppp), F::dbl(qq));
  r.y = F::sub(F::mul(rr, F::sub(qq, r.x)), F::mul(p.y, ppp));
  r.zz = F::mul(p.zz, pp);
  r.zzz = F::mul(p.zzz, ppp);
  return r;
}

// G1 bucket-accumulation form of madd-2008-s with lazy reduction: the same
// group law as xyzz_madd, ~15% fewer VALU instructions.
//   * subtractions are single-pass biased forms (subk), R is a lazy sum,
//   * Y3 = R (Q - X3) - Y1 PPP is one two-product Montgomery pass (mul2),
//   * X is kept in [0, 8p) across the loop (reduce8 before it is stored).
// Every multiplication input stays inside the bounds stated in ff.h.
// In: p.x < 8p, p.y/p.zz/p.zzz < 2p, q < 2p.  Out: x < 8p, y/zz/zzz < 2p.
ZK_HD Xyzz<FqOps> xyzz_madd_g1(const Xyzz<FqOps>& p, const Aff<FqOps>& q) {
  if (xyzz_is_inf(p)) return xyzz_from_aff(q);
  Fe u2 = mul<FqP>(q.x, p.zz);
  Fe s2 = mul<FqP>(q.y, p.zzz);
  Fe pp_ = subk<FqP, 8>(u2, p.x);         // U2 - X1 + 8p   in (0, 10p)
  Fe ny1 = subk<FqP, 2>(fe_zero(), p.y);  // 2p - Y1        in (0, 2p]
  Fe rr = add_lazy(s2, ny1);              // S2 - Y1 + 2p   < 4p, limbs < 2^30
  Fe pp = sqr<FqP>(pp_);                  // < 2p
  if (is_zero<FqP>(pp)) {                 // U2 == X1
    Fe rn = reduce8<FqP>(subk<FqP, 2>(s2, p.y));
    if (is_zero<FqP>(rn)) return xyzz_mdbl(q);
    return xyzz_inf<FqOps>();
  }
  Fe ppp = mul<FqP>(pp_, pp);
  Fe qq = mul<FqP>(p.x, pp);
  Fe t = add_lazy(add_lazy(ppp, qq), qq);  // PPP + 2Q < 6p, limbs < 3*2^29
  Xyzz<FqOps> r;
  r.x = subk<FqP, 6>(sqr<FqP>(rr), t);     // R^2 - PPP - 2Q + 6p in (0, 8p)
  Fe qx = subk<FqP, 8>(qq, r.x);           // Q - X3 + 8p in (0, 10p)
  r.y = mul2<FqP>(rr, qx, ny1, ppp);       // R (Q - X3) - Y1 PPP
  r.zz = mul<FqP>(p.zz, pp);
  r.zzz = mul<FqP>(p.zzz, ppp);
  return r;
}
// xyzz_madd_g1 with every subtraction folded into a Montgomery product: the
// mixed addition of the one-lane-per-bucket accumulation (msm.hip).
//   P  = U2 - X1 + 8p        = mul_add(x2, ZZ1, 8p - X1)      (0, 9.01p)
//   R  = S2 - Y1 + 4p        = mul_add(y2, ZZZ1, 4p - Y1)     (2p, 5.03p)
//   X3 = R^2 - PPP - 2Q + 6p = sqr_add(R, 6p - PPP - 2Q)      (2.7p, 7.2p)
//   Y3 = R (Q - X3 + 10p) + (4p - Y1) PPP                     (0, 1.36p)
// The borrow-form differences (FqP::BK_m, ff.h bsub*) need no carry pass, and
// mul_add/sqr_add normalise the sums in their own carry chain: ~110 fewer
// VALU instructions per entry than xyzz_madd_g1 for the same group law.
// Bounds: every product stays below 169 p^2 (squares: P^2 < 81.2 p^2); mul2's
// columns stay below 2^64 with R normalised and Q - X3 + 10p's limbs
// < 1.5 2^30 (3 2^59 per term, 9 terms).
// In: p finite, p.x < 8p, p.y/zz/zzz < 2p, all normalised; qx < 2p normalised;
// qy value < 2p, limbs < 2^30 (e.g. a borrow-form 2p - y).  Out: x < 8p,
// y/zz/zzz < 2p, normalised; *inf set when the sum is the point at infinity
// (Q == -P); Q == P returns 2Q (xyzz_mdbl).
ZK_HD Xyzz<FqOps> xyzz_madd_g1f(const Xyzz<FqOps>& p, const Fe& qx, const Fe& qy, bool* inf) {
  const Fe ny1 = bsub(FqP::B4_1, p.y);                            // 4p - Y1, limbs < 2^30
  const Fe pp_ = mul_add<FqP>(qx, p.zz, bsub(FqP::B8_1, p.x));  // U2 - X1 + 8p
  const Fe rr = mul_add<FqP>(qy, p.zzz, ny1);                    // S2 - Y1 + 4p
  const Fe pp = sqr<FqP>(pp_);                                   // < 1.48p: == 0 mod p iff in {0, p}
  // (Round 6: a 4-instruction filter on limbs 0 and 8 in front of this 9-limb
  // test, -18 VALU per entry, measured 0.5% slower on the 2^20 loop: the
  // extra branch level costs more than the instructions it removes.)
  uint32_t z = 0, e = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    z |= pp.v[i];
    e |= pp.v[i] ^ FqP::P[i];
  }
  *inf = false;
  if (z == 0 || e == 0) {  // U2 == X1: Q = +-P
    if (is_zero<FqP>(reduce_q32<FqP>(rr))) return xyzz_mdbl(Aff<FqOps>{qx, reduce_q32<FqP>(qy)});
    *inf = true;
    return xyzz_inf<FqOps>();
  }
  const Fe ppp = mul<FqP>(pp_, pp);
  const Fe qq = mul<FqP>(p.x, pp);
  Xyzz<FqOps> r;
  r.x = sqr_add<FqP>(rr, bsub2(FqP::B6_3, ppp, qq));
  r.y = mul2<FqP>(rr, bsubadd(FqP::B10_1, r.x, qq), ny1, ppp);
  r.zz = mul<FqP>(p.zz, pp);
  r.zzz = mul<FqP>(p.zzz, ppp);
  return r;
}

// P + Q with both affine (mmadd-2008-s): xyzz_madd_g1 with ZZ1 = ZZZ1 = 1, so
// U2 = x2, S2 = y2, ZZ3 = PP, ZZZ3 = PPP -- four products fewer (the second
// entry of every bucket; the first is xyzz_from_aff).  Same field values as
// xyzz_madd_g1(xyzz_from_aff(p), q).  In: p, q < 2p.  Out: as xyzz_madd_g1.
ZK_HD Xyzz<FqOps> xyzz_mmadd_g1(const Aff<FqOps>& p, const Aff<FqOps>& q) {
  Fe pp_ = subk<FqP, 2>(q.x, p.x);        // x2 - x1 + 2p   in (0, 4p)
  Fe ny1 = subk<FqP, 2>(fe_zero(), p.y);  // 2p - y1        in (0, 2p]
  Fe rr = add_lazy(q.y, ny1);             // y2 - y1 + 2p   < 4p, limbs < 2^30
  Fe pp = sqr<FqP>(pp_);
  if (is_zero<FqP>(pp)) {
    Fe rn = reduce8<FqP>(subk<FqP, 2>(q.y, p.y));
    if (is_zero<FqP>(rn)) return xyzz_mdbl(q);
    return xyzz_inf<FqOps>();
  }
  Fe ppp = mul<FqP>(pp_, pp);
  Fe qq = mul<FqP>(p.x, pp);
  Fe t = add_lazy(add_lazy(ppp, qq), qq);
  Xyzz<FqOps> r;
  r.x = subk<FqP, 6>(sqr<FqP>(rr), t);
  Fe qx = subk<FqP, 8>(qq, r.x);
  r.y = mul2<FqP>(rr, qx, ny1, ppp);
  r.zz = pp;
  r.zzz = ppp;
  return r;
}
// Fq2 counterpart of xyzz_mmadd_g1 (four Fq2 products fewer than
// xyzz_madd_g2).  In: p, q < 2p.  Out: as xyzz_madd_g2.
ZK_HD Xyzz<Fq2Ops> xyzz_mmadd_g2(const Aff<Fq2Ops>& p, const Aff<Fq2Ops>& q) {
  Fe2 pp_ = {subk<FqPn, 2>(q.x.c0, p.x.c0), subk<FqPn, 2>(q.x.c1, p.x.c1)};  // (0, 4p)
  Fe2 rr = {subk<FqPn, 2>(q.y.c0, p.y.c0), subk<FqPn, 2>(q.y.c1, p.y.c1)};   // (0, 4p)
  Fe2 pp = f2_sqr_n(pp_);
  if (f2_is_zero(pp)) {
    if (is_zero<FqPn>(reduce8<FqPn>(rr.c0)) && is_zero<FqPn>(reduce8<FqPn>(rr.c1))) return xyzz_mdbl(q);
    return xyzz_inf<Fq2Ops>();
  }
  Fe2 r2 = f2_sqr_n(rr);
  Fe2 ppp = f2_mul_n(pp_, pp), qq = f2_mul_n(p.x, pp);
  Xyzz<Fq2Ops> r;
  r.x.c0 = reduce8<FqPn>(subk<FqPn, 6>(r2.c0, add_lazy(add_lazy(ppp.c0, qq.c0), qq.c0)));
  r.x.c1 = reduce8<FqPn>(subk<FqPn, 6>(r2.c1, add_lazy(add_lazy(ppp.c1, qq.c1), qq.c1)));
  Fe2 qx = {subk<FqPn, 2>(qq.c0, r.x.c0), subk<FqPn, 2>(qq.c1, r.x.c1)};  // (0, 4p)
  Fe ny0 = subk<FqPn, 2>(fe_zero(), p.y.c0), ny1 = subk<FqPn, 2>(fe_zero(), p.y.c1);
  Fe nqx1 = subk<FqPn, 4>(fe_zero(), qx.c1), nppp1 = subk<FqPn, 2>(fe_zero(), ppp.c1);
  r.y.c0 = mul4<FqPn>(rr.c0, qx.c0, rr.c1, nqx1, ny0, ppp.c0, ny1, nppp1);
  r.y.c1 = mul4<FqPn>(rr.c0, qx.c1, rr.c1, qx.c0, ny0, ppp.c1, ny1, ppp.c0);
  r.zz = pp;
  r.zzz = ppp;
  return r;
}
// G2 (Fq2) counterpart: lazy single-pass subtractions, Fq2 products with one
// reduction per component, Y3 as two four-product passes.  X stays < 2p here
// (Fq2 squares of lazy sums would leave the 169 p^2 product bound).
// In/out: all coordinates < 2p, normalised.
ZK_HD Xyzz<Fq2Ops> xyzz_madd_g2(const Xyzz<Fq2Ops>& p, const Aff<Fq2Ops>& q) {
  if (xyzz_is_inf(p)) return xyzz_from_aff(q);
  Fe2 u2 = f2_mul_n(q.x, p.zz), s2 = f2_mul_n(q.y, p.zzz);
  Fe2 pp_ = {subk<FqPn, 2>(u2.c0, p.x.c0), subk<FqPn, 2>(u2.c1, p.x.c1)};  // (0, 4p)
  Fe2 rr = {subk<FqPn, 2>(s2.c0, p.y.c0), subk<FqPn, 2>(s2.c1, p.y.c1)};   // (0, 4p)
  Fe2 pp = f2_sqr_n(pp_);
  if (f2_is_zero(pp)) {
    if (is_zero<FqPn>(reduce8<FqPn>(rr.c0)) && is_zero<FqPn>(reduce8<FqPn>(rr.c1))) return xyzz_mdbl(q);
    return xyzz_inf<Fq2Ops>();
  }
  Fe2 r2 = f2_sqr_n(rr);
  Fe2 ppp = f2_mul_n(pp_, pp), qq = f2_mul_n(p.x, pp);
  Xyzz<Fq2Ops> r;
  r.x.c0 = reduce8<FqPn>(subk<FqPn, 6>(r2.c0, add_lazy(add_lazy(ppp.c0, qq.c0), qq.c0)));
  r.x.c1 = reduce8<FqPn>(subk<FqPn, 6>(r2.c1, add_lazy(add_lazy(ppp.c1, qq.c1), qq.c1)));
  Fe2 qx = {subk<FqPn, 2>(qq.c0, r.x.c0), subk<FqPn, 2>(qq.c1, r.x.c1)};  // (0, 4p)
  Fe ny0 = subk<FqPn, 2>(fe_zero(), p.y.c0), ny1 = subk<FqPn, 2>(fe_zero(), p.y.c1);
  Fe nqx1 = subk<FqPn, 4>(fe_zero(), qx.c1), nppp1 = subk<FqPn, 2>(fe_zero(), ppp.c1);
  r.y.c0 = mul4<FqPn>(rr.c0, qx.c0, rr.c1, nqx1, ny0, ppp.c0, ny1, nppp1);
  r.y.c1 = mul4<FqPn>(rr.c0, qx.c1, rr.c1, qx.c0, ny0, ppp.c1, ny1, ppp.c0);
  r.zz = f2_mul_n(p.zz, pp);
  r.zzz = f2_mul_n(p.zzz, ppp);
  return r;
}

// P + Q with both in XYZZ (add-2008-s) in the lazy forms of xyzz_madd_g1:
// U1/S1 take the place of X1/Y1, Y3 is one two-product pass, and X3 is
// brought back to [0, 2p) so the contract is xyzz_add's (the bucket
// reductions store and exchange these points).  In/out: coordinates < 2p,
// normalised.
template <class P = FqP>
ZK_HD Xyzz<FqOps> xyzz_add_g1(const Xyzz<FqOps>& p, const Xyzz<FqOps>& q) {
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  Fe u1 = mul<P>(p.x, q.zz);
  Fe u2 = mul<P>(q.x, p.zz);
  Fe s1 = mul<P>(p.y, q.zzz);
  Fe s2 = mul<P>(q.y, p.zzz);
  Fe pp_ = subk<P, 2>(u2, u1);          // U2 - U1 + 2p   in (0, 4p)
  Fe ny1 = subk<P, 2>(fe_zero(), s1);   // 2p - S1        in (0, 2p]
  Fe rr = add_lazy(s2, ny1);              // S2 - S1 + 2p   < 4p, limbs < 2^30
  Fe pp = sqr<P>(pp_);
  if (is_zero<P>(pp)) {
    Fe rn = reduce8<P>(subk<P, 2>(s2, s1));
    if (is_zero<P>(rn)) return xyzz_dbl(p);
    return xyzz_inf<FqOps>();
  }
  Fe ppp = mul<P>(pp_, pp);
  Fe qq = mul<P>(u1, pp);
  Fe t = add_lazy(add_lazy(ppp, qq), qq);  // PPP + 2Q < 6p, limbs < 3*2^29
  Xyzz<FqOps> r;
  Fe x = subk<P, 6>(sqr<P>(rr), t);    // in (0, 8p)
  Fe qx = subk<P, 8>(qq, x);             // Q - X3 + 8p in (0, 10p)
  r.y = mul2<P>(rr, qx, ny1, ppp);       // R (Q - X3) - S1 PPP
  r.x = reduce8<P>(x);
  r.zz = mul<P>(mul<P>(p.zz, q.zz), pp);
  r.zzz = mul<P>(mul<P>(p.zzz, q.zzz), ppp);
  return r;
}
// Fq2 counterpart (the products of xyzz_madd_g2: one reduction per component).
// In/out: coordinates < 2p, normalised.
ZK_HD Xyzz<Fq2Ops> xyzz_add_g2(const Xyzz<Fq2Ops>& p, const Xyzz<Fq2Ops>& q) {
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  Fe2 u1 = f2_mul_n(p.x, q.zz), u2 = f2_mul_n(q.x, p.zz);
  Fe2 s1 = f2_mul_n(p.y, q.zzz), s2 = f2_mul_n(q.y, p.zzz);
  Fe2 pp_ = {subk<FqPn, 2>(u2.c0, u1.c0), subk<FqPn, 2>(u2.c1, u1.c1)};  // (0, 4p)
  Fe2 rr = {subk<FqPn, 2>(s2.c0, s1.c0), subk<FqPn, 2>(s2.c1, s1.c1)};   // (0, 4p)
  Fe2 pp = f2_sqr_n(pp_);
  if (f2_is_zero(pp)) {
    if (is_zero<FqPn>(reduce8<FqPn>(rr.c0)) && is_zero<FqPn>(reduce8<FqPn>(rr.c1))) return xyzz_dbl(p);
    return xyzz_inf<Fq2Ops>();
  }
  Fe2 r2 = f2_sqr_n(rr);
  Fe2 ppp = f2_mul_n(pp_, pp), qq = f2_mul_n(u1, pp);
  Xyzz<Fq2Ops> r;
  r.x.c0 = reduce8<FqPn>(subk<FqPn, 6>(r2.c0, add_lazy(add_lazy(ppp.c0, qq.c0), qq.c0)));
  r.x.c1 = reduce8<FqPn>(subk<FqPn, 6>(r2.c1, add_lazy(add_lazy(ppp.c1, qq.c1), qq.c1)));
  Fe2 qx = {subk<FqPn, 2>(qq.c0, r.x.c0), subk<FqPn, 2>(qq.c1, r.x.c1)};  // (0, 4p)
  Fe ny0 = subk<FqPn, 2>(fe_zero(), s1.c0), ny1 = subk<FqPn, 2>(fe_zero(), s1.c1);
  Fe nqx1 = subk<FqPn, 4>(fe_zero(), qx.c1), nppp1 = subk<FqPn, 2>(fe_zero(), ppp.c1);
  r.y.c0 = mul4<FqPn>(rr.c0, qx.c0, rr.c1, nqx1, ny0, ppp.c0, ny1, nppp1);
  r.y.c1 = mul4<FqPn>(rr.c0, qx.c1, rr.c1, qx.c0, ny0, ppp.c1, ny1, ppp.c0);
  r.zz = f2_mul_n(f2_mul_n(p.zz, q.zz), pp);
  r.zzz = f2_mul_n(f2_mul_n(p.zzz, q.zzz), ppp);
  return r;
}

// conditional negation of an affine y (< 2p) without a borrow/fix-up pass
ZK_HD Fe fq_cneg(const Fe& y, bool neg_) {
  Fe n = subk<FqP, 2>(fe_zero(), y);
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = neg_ ? n.v[i] : y.v[i];
  return r;
}

// P + Q   (add-2008-s)
template <class F>
ZK_HD Xyzz<F> xyzz_add(const Xyzz<F>& p, const Xyzz<F>& q) {
  using T = typename F::T;
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  T u1 = F::mul(p.x, q.zz);
  T u2 = F::mul(q.x, p.zz);
  T s1 = F::mul(p.y, q.zzz);
  T s2 = F::mul(q.y, p.zzz);
  T pp_ = F::sub(u2, u1);
  T rr = F::sub(s2, s1);
  if (F::is_zero(pp_)) {
    if (F::is_zero(rr)) return xyzz_dbl(p);
    return xyzz_inf<F>();
  }
  T pp = F::sqr(pp_);
  T ppp = F::mul(pp_, pp);
  T qq = F::mul(u1, pp);
  Xyzz<F> r;
  r.x = F::sub(F::sub(F::sqr(rr), ppp), F::dbl(qq));
  r.y = F::sub(F::mul(rr, F::sub(qq, r.x)), F::mul(s1, ppp));
  r.zz = F::mul(F::mul(p.zz, q.zz), pp);
  r.zzz = F::mul(F::mul(p.zzz, q.zzz), ppp);
  return r;
}

template <class F>
ZK_HD Aff<F> aff_neg(const Aff<F>& a) {
  Aff<F> r = a;
  r.y = F::neg(a.y);
  return r;
}

}  // namespace zk

