// host_field.h — x86 host BN254 Fq / Fq2 (4 x 64, Montgomery R = 2^256) used
// only for the O(windows) epilogue of a GPU MSM (Horner over ~256 window/bit
// sums, ~255 doublings: a strictly sequential chain that a single CPU core
// runs ~20x faster than a single GPU lane) and for final affine conversion /
// serialisation.  Plugs into the same ec.h XYZZ templates as the device code.
#pragma once
#include <stdint.h>
#include <string.h>

#include "ec.h"

namespace zkh {

typedef unsigned __int128 u128;

struct F4 {
  uint64_t l[4];
};

static const uint64_t QP[4] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL,
                               0x30644e72e131a029ULL};
static const uint64_t QINV = 0x87d20782e4866389ULL;  // -q^-1 mod 2^64
static const uint64_t QR2[4] = {0xf32cfc5b538afa89ULL, 0xb5e71911d44501fbULL, 0x47ab1eff0a417ff6ULL,
                                0x06d89f71cab8351fULL};  // 2^512 mod q
static const uint64_t QONE[4] = {0xd35d438dc58f0d9dULL, 0x0a78eb28f5c70b3dULL, 0x666ea36f7879462cULL,
                                 0x0e0a77c19a07df2fULL};  // 2^256 mod q

inline bool geq(const uint64_t a[4], const uint64_t b[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return true;
}
inline uint64_t sub4(uint64_t o[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    o[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
inline uint64_t add4(uint64_t o[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a[i] + b[i] + c;
    o[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  return c;
}
// Fully unrolled CIOS; q < 2^254 leaves the top word's 2 high bits free, so
// the running value never exceeds 5 words ("no-carry" Montgomery).
#define ZKH_MAC(t, a, b, c)                 \
  do {                                      \
    u128 x_ = (u128)(a) * (b) + (t) + (c);  \
    (t) = (uint64_t)x_;                     \
    (c) = (uint64_t)(x_ >> 64);             \
  } while (0)
inline F4 fmul(const F4& a, const F4& b) {
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, c, m, hi;
#define ZKH_ROUND(bi)                                                     \
  c = 0;                                                                  \
  ZKH_MAC(t0, a.l[0], bi, c);                                             \
  ZKH_MAC(t1, a.l[1], bi, c);                                             \
  ZKH_MAC(t2, a.l[2], bi, c);                                             \
  ZKH_MAC(t3, a.l[3], bi, c);                                             \
  hi = c;                                                                 \
  m = t0 * QINV;                                                          \
  c = (uint64_t)(((u128)m * QP[0] + t0) >> 64);                           \
  {                                                                       \
    u128 x_ = (u128)m * QP[1] + t1 + c; t0 = (uint64_t)x_; c = (uint64_t)(x_ >> 64); \
    x_ = (u128)m * QP[2] + t2 + c; t1 = (uint64_t)x_; c = (uint64_t)(x_ >> 64);      \
    x_ = (u128)m * QP[3] + t3 + c; t2 = (uint64_t)x_; c = (uint64_t)(x_ >> 64);      \
    t3 = hi + c;                                                          \
  }
  ZKH_ROUND(b.l[0]) ZKH_ROUND(b.l[1]) ZKH_ROUND(b.l[2]) ZKH_ROUND(b.l[3])
#undef ZKH_ROUND
  F4 r = {{t0, t1, t2, t3}};
  if (geq(r.l, QP)) sub4(r.l, r.l, QP);
  return r;
}
inline F4 fadd(const F4& a, const F4& b) {
  F4 r;
  uint64_t c = add4(r.l, a.l, b.l);
  if (c || geq(r.l, QP)) sub4(r.l, r.l, QP);
  return r;
}
inline F4 fsub(const F4& a, const F4& b) {
  F4 r;
  if (sub4(r.l, a.l, b.l)) add4(r.l, r.l, QP);
  return r;
}
inline bool fzero(const F4& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }
inline F4 fconst(const uint64_t c[4]) {
  F4 r;
  memcpy(r.l, c, 32);
  return r;
}
inline F4 from_canon(const uint64_t c[4]) { return fmul(fconst(c), fconst(QR2)); }
inline void to_canon(uint64_t c[4], const F4& a) {
  F4 one = {{1, 0, 0, 0}};
  F4 t = fmul(a, one);
  memcpy(c, t.l, 32);
}
inline F4 fpow(const F4& a, const uint64_t e[4]) {
  F4 r = fconst(QONE), b = a;
  for (int i = 255; i >= 0; i--) {
    r = fmul(r, r);
    if ((e[i / 64] >> (i % 64)) & 1) r = fmul(r, b);
  }
  return r;
}
inline F4 finv(const F4& a) {
  uint64_t e[4];
  uint64_t two[4] = {2, 0, 0, 0};
  sub4(e, QP, two);
  return fpow(a, e);
}

struct HFq {
  using T = F4;
  static T mul(const T& a, const T& b) { return fmul(a, b); }
  static T sqr(const T& a) { return fmul(a, a); }
  static T add(const T& a, const T& b) { return fadd(a, b); }
  static T sub(const T& a, const T& b) { return fsub(a, b); }
  static T dbl(const T& a) { return fadd(a, a); }
  static T neg(const T& a) { return fsub(F4{{0, 0, 0, 0}}, a); }
  static bool is_zero(const T& a) { return fzero(a); }
  static bool is_zero_raw(const T& a) { return fzero(a); }
  static T zero() { return F4{{0, 0, 0, 0}}; }
  static T one() { return fconst(QONE); }
};

struct F42 {
  F4 c0, c1;
};
struct HFq2 {
  using T = F42;
  static T mul(const T& a, const T& b) {
    F4 t0 = fmul(a.c0, b.c0), t1 = fmul(a.c1, b.c1);
    F4 t2 = fmul(fadd(a.c0, a.c1), fadd(b.c0, b.c1));
    return {fsub(t0, t1), fsub(fsub(t2, t0), t1)};
  }
  static T sqr(const T& a) { return mul(a, a); }
  static T add(const T& a, const T& b) { return {fadd(a.c0, b.c0), fadd(a.c1, b.c1)}; }
  static T sub(const T& a, const T& b) { return {fsub(a.c0, b.c0), fsub(a.c1, b.c1)}; }
  static T dbl(const T& a) { return add(a, a); }
  static T neg(const T& a) { return sub(zero(), a); }
  static bool is_zero(const T& a) { return fzero(a.c0) && fzero(a.c1); }
  static bool is_zero_raw(const T& a) { return fzero(a.c0) && fzero(a.c1); }
  static T zero() { return {F4{{0, 0, 0, 0}}, F4{{0, 0, 0, 0}}}; }
  static T one() { return {fconst(QONE), F4{{0, 0, 0, 0}}}; }
  static T inv(const T& a) {
    F4 n = fadd(fmul(a.c0, a.c0), fmul(a.c1, a.c1));
    F4 ni = finv(n);
    return {fmul(a.c0, ni), fsub(F4{{0, 0, 0, 0}}, fmul(a.c1, ni))};
  }
};

}  // namespace zkh
