/*
 * ec.c — BN254 G1 (y^2 = x^3 + 3 over Fq) and G2 (y^2 = x^3 + 3/(9+u) over Fq2)
 * in Jacobian coordinates, restating ark-ec 0.5.0 short_weierstrass::Projective
 * (Cargo.lock:290) and ark-bn254 0.5.0 curve configs.  Test infrastructure only.
 *
 * Formulas: dbl-2009-l, add-2007-bl, madd-2007-bl (a = 0).  Any correct
 * formula gives the same affine result, which is all parity depends on.
 */
#include <string.h>
#include <stdlib.h>
#include "oracle.h"

/* ---- generic template over (T, ops) ---- */
#define DEFINE_CURVE(P, J, A, T, ADD, SUB, MUL, SQR, DBL, NEG, ISZ, EQ, INV, ONE, ZERO)      \
  void P##_set_inf(J* p) { memset(p, 0, sizeof(*p)); }                                     \
  static int P##_is_inf(const J* p) { return ISZ(&p->z); }                                 \
  void P##_from_affine(J* o, const A* a) {                                                 \
    if (a->inf) { P##_set_inf(o); return; }                                               \
    o->x = a->x; o->y = a->y; ONE(&o->z);                                                  \
  }                                                                                        \
  void P##_to_affine(A* o, const J* p) {                                                   \
    if (P##_is_inf(p)) { memset(o, 0, sizeof(*o)); o->inf = 1; return; }                   \
    T zi, zi2, zi3;                                                                        \
    INV(&zi, &p->z); SQR(&zi2, &zi); MUL(&zi3, &zi2, &zi);                                 \
    MUL(&o->x, &p->x, &zi2); MUL(&o->y, &p->y, &zi3); o->inf = 0;                          \
  }                                                                                        \
  void P##_dbl(J* o, const J* p) {                                                         \
    if (P##_is_inf(p)) { *o = *p; return; }                                                \
    T a, b, c, d, e, f, t;                                                                 \
    SQR(&a, &p->x); SQR(&b, &p->y); SQR(&c, &b);                                           \
    ADD(&t, &p->x, &b); SQR(&t, &t); SUB(&t, &t, &a); SUB(&t, &t, &c); DBL(&d, &t);        \
    DBL(&e, &a); ADD(&e, &e, &a); SQR(&f, &e);                                             \
    T z3; MUL(&z3, &p->y, &p->z); DBL(&z3, &z3);                                           \
    T x3; DBL(&t, &d); SUB(&x3, &f, &t);                                                   \
    T y3; SUB(&t, &d, &x3); MUL(&y3, &e, &t);                                              \
    DBL(&c, &c); DBL(&c, &c); DBL(&c, &c); SUB(&y3, &y3, &c);                              \
    o->x = x3; o->y = y3; o->z = z3;                                                       \
  }                                                                                        \
  void P##_add(J* o, const J* p, const J* q) {                                             \
    if (P##_is_inf(p)) { *o = *q; return; }                                                \
    if (P##_is_inf(q)) { *o = *p; return; }                                                \
    T z1z1, z2z2, u1, u2, s1, s2, h, i, j, r, v, t;                                        \
    SQR(&z1z1, &p->z); SQR(&z2z2, &q->z);                                                  \
    MUL(&u1, &p->x, &z2z2); MUL(&u2, &q->x, &z1z1);                                        \
    MUL(&s1, &p->y, &q->z); MUL(&s1, &s1, &z2z2);                                          \
    MUL(&s2, &q->y, &p->z); MUL(&s2, &s2, &z1z1);                                          \
    SUB(&h, &u2, &u1); SUB(&r, &s2, &s1);                                                  \
    if (ISZ(&h)) {                                                                         \
      if (ISZ(&r)) { P##_dbl(o, p); return; }                                              \
      P##_set_inf(o); return;                                                              \
    }                                                                                      \
    DBL(&i, &h); SQR(&i, &i); MUL(&j, &h, &i); DBL(&r, &r); MUL(&v, &u1, &i);              \
    T x3, y3, z3;                                                                          \
    SQR(&x3, &r); SUB(&x3, &x3, &j); DBL(&t, &v); SUB(&x3, &x3, &t);                       \
    SUB(&t, &v, &x3); MUL(&y3, &r, &t); MUL(&t, &s1, &j); DBL(&t, &t); SUB(&y3, &y3, &t);  \
    ADD(&t, &p->z, &q->z); SQR(&t, &t); SUB(&t, &t, &z1z1); SUB(&t, &t, &z2z2);            \
    MUL(&z3, &t, &h);                                                                      \
    o->x = x3; o->y = y3; o->z = z3;                                                       \
  }                                                                                        \
  void P##_add_mixed(J* o, const J* p, const A* q) {                                       \
    if (q->inf) { *o = *p; return; }                                                       \
    if (P##_is_inf(p)) { P##_from_affine(o, q); return; }                                  \
    T z1z1, u2, s2, h, hh, i, j, r, v, t;                                                  \
    SQR(&z1z1, &p->z); MUL(&u2, &q->x, &z1z1);                                             \
    MUL(&s2, &q->y, &p->z); MUL(&s2, &s2, &z1z1);                                          \
    SUB(&h, &u2, &p->x); SUB(&r, &s2, &p->y);                                              \
    if (ISZ(&h)) {                                                                         \
      if (ISZ(&r)) { P##_dbl(o, p); return; }                                              \
      P##_set_inf(o); return;                                                              \
    }                                                                                      \
    SQR(&hh, &h); DBL(&i, &hh); DBL(&i, &i); MUL(&j, &h, &i); DBL(&r, &r);                 \
    MUL(&v, &p->x, &i);                                                                    \
    T x3, y3, z3;                                                                          \
    SQR(&x3, &r); SUB(&x3, &x3, &j); DBL(&t, &v); SUB(&x3, &x3, &t);                       \
    SUB(&t, &v, &x3); MUL(&y3, &r, &t); MUL(&t, &p->y, &j); DBL(&t, &t);                   \
    SUB(&y3, &y3, &t);                                                                     \
    ADD(&t, &p->z, &h); SQR(&t, &t); SUB(&t, &t, &z1z1); SUB(&z3, &t, &hh);                \
    o->x = x3; o->y = y3; o->z = z3;                                                       \
  }

/* Fq wrappers */
static void q_add(fe* o, const fe* a, const fe* b) { fe_add(&FQ, o, a, b); }
static void q_sub(fe* o, const fe* a, const fe* b) { fe_sub(&FQ, o, a, b); }
static void q_mul(fe* o, const fe* a, const fe* b) { fe_mul(&FQ, o, a, b); }
static void q_sqr(fe* o, const fe* a) { fe_mul(&FQ, o, a, a); }
static void q_dbl(fe* o, const fe* a) { fe_add(&FQ, o, a, a); }
static void q_neg(fe* o, const fe* a) { fe_neg(&FQ, o, a); }
static int q_isz(const fe* a) { return fe_is_zero(a); }
static int q_eq(const fe* a, const fe* b) { return fe_eq(a, b); }
static void q_inv(fe* o, const fe* a) { fe_inv(&FQ, o, a); }
static void q_one(fe* o) { *o = FQ.one; }
static void q_zero(fe* o) { memset(o, 0, sizeof(*o)); }
static void q2_one(fe2* o) { o->c0 = FQ.one; memset(&o->c1, 0, sizeof(fe)); }
static void q2_zero(fe2* o) { memset(o, 0, sizeof(*o)); }

DEFINE_CURVE(g1, g1j, g1a, fe, q_add, q_sub, q_mul, q_sqr, q_dbl, q_neg, q_isz, q_eq, q_inv, q_one, q_zero)
DEFINE_CURVE(g2, g2j, g2a, fe2, fe2_add, fe2_sub, fe2_mul, fe2_sqr, fe2_dbl, fe2_neg, fe2_is_zero, fe2_eq, fe2_inv, q2_one, q2_zero)

void g1_neg(g1j* o, const g1j* p) { *o = *p; fe_neg(&FQ, &o->y, &p->y); }

int g1j_eq(const g1j* a, const g1j* b) {
  g1a x, y;
  g1_to_affine(&x, a);
  g1_to_affine(&y, b);
  if (x.inf || y.inf) return x.inf == y.inf;
  return fe_eq(&x.x, &y.x) && fe_eq(&x.y, &y.y);
}

void g1_mul(g1j* o, const g1j* p, const uint64_t k[4]) {
  g1j r;
  g1_set_inf(&r);
  for (int i = 255; i >= 0; i--) {
    g1_dbl(&r, &r);
    if ((k[i / 64] >> (i % 64)) & 1) g1_add(&r, &r, p);
  }
  *o = r;
}
void g2_mul(g2j* o, const g2j* p, const uint64_t* k, int nlimbs) {
  g2j r;
  g2_set_inf(&r);
  for (int i = nlimbs * 64 - 1; i >= 0; i--) {
    g2_dbl(&r, &r);
    if ((k[i / 64] >> (i % 64)) & 1) g2_add(&r, &r, p);
  }
  *o = r;
}

int g1_is_on_curve(const g1a* a) {
  if (a->inf) return 1;
  fe l, r, three;
  fe_sqr(&FQ, &l, &a->y);
  fe_sqr(&FQ, &r, &a->x);
  fe_mul(&FQ, &r, &r, &a->x);
  fe_set_u64(&FQ, &three, 3);
  fe_add(&FQ, &r, &r, &three);
  return fe_eq(&l, &r);
}
int g2_is_on_curve(const g2a* a) {
  if (a->inf) return 1;
  fe2 l, r;
  fe2_sqr(&l, &a->y);
  fe2_sqr(&r, &a->x);
  fe2_mul(&r, &r, &a->x);
  fe2_add(&r, &r, &G2_B);
  return fe2_eq(&l, &r);
}

/* ------------------------------------------------------------ rand points */
/* ark-ec 0.5 short_weierstrass UniformRand: loop { x = F::rand; greatest =
 * bool; if get_point_from_x_unchecked(x, greatest) -> mul_by_cofactor }.
 * SURVEY.md Appendix A.3 / A.4. */
void g1_rand(g1j* o, chacha_rng* r) {
  for (;;) {
    fe x;
    fe_rand(&FQ, &x, r);
    int greatest = (rng_next_u32(r) >> 31) == 1;
    fe rhs, three, y;
    fe_sqr(&FQ, &rhs, &x);
    fe_mul(&FQ, &rhs, &rhs, &x);
    fe_set_u64(&FQ, &three, 3);
    fe_add(&FQ, &rhs, &rhs, &three);
    if (!fe_sqrt(&FQ, &y, &rhs)) continue;
    fe ny;
    fe_neg(&FQ, &ny, &y);
    /* (smaller, larger) by canonical order; greatest selects larger */
    fe smaller = y, larger = ny;
    if (fe_cmp_canon(&FQ, &y, &ny) >= 0) { smaller = ny; larger = y; }
    g1a a = {x, greatest ? larger : smaller, 0};
    g1_from_affine(o, &a); /* cofactor 1 */
    return;
  }
}

static const uint64_t G2_COFACTOR[4] = {0x345f2299c0f9fa8dULL, 0x06ceecda572a2489ULL,
                                        0xb85045b68181585eULL, 0x30644e72e131a029ULL};
void g2_rand(g2j* o, chacha_rng* r) {
  for (;;) {
    fe2 x;
    fe_rand(&FQ, &x.c0, r);
    fe_rand(&FQ, &x.c1, r);
    int greatest = (rng_next_u32(r) >> 31) == 1;
    fe2 rhs, y;
    fe2_sqr(&rhs, &x);
    fe2_mul(&rhs, &rhs, &x);
    fe2_add(&rhs, &rhs, &G2_B);
    if (!fe2_sqrt(&y, &rhs)) continue;
    fe2 ny;
    fe2_neg(&ny, &y);
    fe2 smaller = y, larger = ny;
    if (fe2_cmp(&y, &ny) >= 0) { smaller = ny; larger = y; }
    g2a a = {x, greatest ? larger : smaller, 0};
    g2j p;
    g2_from_affine(&p, &a);
    g2_mul(o, &p, G2_COFACTOR, 4);
    return;
  }
}
