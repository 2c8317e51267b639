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

