/*
 * ff.c — BN254 Fq / Fr / Fq2 arithmetic, restating ark-ff 0.5.0 Fp<MontBackend,4>
 * (Cargo.lock:344) and ark-bn254 0.5.0 (Cargo.lock:226) field configs.
 * Test infrastructure only (see oracle.h).
 *
 * Representation follows arkworks exactly: 4 x u64 little-endian limbs in
 * Montgomery form with R = 2^256, so Fp::rand's raw limbs
 * are interpreted identically.
 */
#include <string.h>
#include "oracle.h"

typedef unsigned __int128 u128;

field FQ = {{0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL,
             0x30644e72e131a029ULL}, 0, {{0}}, {{0}}, 254};
field FR = {{0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
             0x30644e72e131a029ULL}, 0, {{0}}, {{0}}, 254};

static int geq_p(const uint64_t a[4], const uint64_t p[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > p[i]) return 1;
    if (a[i] < p[i]) return 0;
  }
  return 1;
}
static uint64_t sub4(uint64_t o[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    o[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
static uint64_t add4(uint64_t o[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a[i] + b[i] + c;
    o[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  return c;
}

void fe_add(const field* F, fe* o, const fe* a, const fe* b) {
  uint64_t t[4];
  uint64_t c = add4(t, a->l, b->l);
  if (c || geq_p(t, F->p)) sub4(t, t, F->p);
  memcpy(o->l, t, 32);
}
void fe_sub(const field* F, fe* o, const fe* a, const fe* b) {
  uint64_t t[4];
  if (sub4(t, a->l, b->l)) add4(t, t, F->p);
  memcpy(o->l, t, 32);
}
void fe_dbl(const field* F, fe* o, const fe* a) { fe_add(F, o, a, a); }
void fe_neg(const field* F, fe* o, const fe* a) {
  if (fe_is_zero(a)) { memset(o, 0, sizeof(fe)); return; }
  sub4(o->l, F->p, a->l);
}
int fe_is_zero(const fe* a) { return (a->l[0] | a->l[1] | a->l[2] | a->l[3]) == 0; }
int fe_eq(const fe* a, const fe* b) { return memcmp(a->l, b->l, 32) == 0; }

/* CIOS Montgomery multiplication, 4 x 64 */
void fe_mul(const field* F, fe* o, const fe* a, const fe* b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      u128 x = (u128)a->l[j] * b->l[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * F->inv;
    u128 x = (u128)m * F->p[0] + t[0];
    c = (uint64_t)(x >> 64);
    for (int j = 1; j < 4; j++) {
      x = (u128)m * F->p[j] + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  if (t[4] || geq_p(t, F->p)) sub4(t, t, F->p);
  memcpy(o->l, t, 32);
}
void fe_sqr(const field* F, fe* o, const fe* a) { fe_mul(F, o, a, a); }

void fe_from_canon(const field* F, fe* o, const uint64_t c[4]) {
  fe t;
  memcpy(t.l, c, 32);
  fe_mul(F, o, &t, &F->r2);
}
void fe_to_canon(const field* F, uint64_t c[4], const fe* a) {
  fe one = {{1, 0, 0, 0}}, t;
  fe_mul(F, &t, a, &one);
  memcpy(c, t.l, 32);
}
void fe_set_u64(const field* F, fe* o, uint64_t v) {
  uint64_t c[4] = {v, 0, 0, 0};
  fe_from_canon(F, o, c);
}
int fe_cmp_canon(const field* F, const fe* a, const fe* b) {
  uint64_t x[4], y[4];
  fe_to_canon(F, x, a);
  fe_to_canon(F, y, b);
  for (int i = 3; i >= 0; i--) {
    if (x[i] > y[i]) return 1;
    if (x[i] < y[i]) return -1;
  }
  return 0;
}
void fe_pow(const field* F, fe* o, const fe* a, const uint64_t* e, int nlimbs) {
  fe r = F->one, b = *a;
  for (int i = nlimbs * 64 - 1; i >= 0; i--) {
    fe_sqr(F, &r, &r);
    if ((e[i / 64] >> (i % 64)) & 1) fe_mul(F, &r, &r, &b);
  }
  *o = r;
}
void fe_inv(const field* F, fe* o, const fe* a) {
  uint64_t e[4];
  uint64_t two[4] = {2, 0, 0, 0};
  sub4(e, F->p, two);
  fe_pow(F, o, a, e, 4);
}
int fe_legendre_is_square(const field* F, const fe* a) {
  if (fe_is_zero(a)) return 1;
  uint64_t e[4], one[4] = {1, 0, 0, 0};
  sub4(e, F->p, one);
  /* (p-1)/2 */
  for (int i = 0; i < 4; i++) e[i] = (e[i] >> 1) | (i < 3 ? e[i + 1] << 63 : 0);
  fe t;
  fe_pow(F, &t, a, e, 4);
  return fe_eq(&t, &F->one);
}
/* p = 3 mod 4: sqrt = a^((p+1)/4) */
int fe_sqrt(const field* F, fe* o, const fe* a) {
  uint64_t e[4], one[4] = {1, 0, 0, 0};
  add4(e, F->p, one);
  for (int k = 0; k < 2; k++)
    for (int i = 0; i < 4; i++) e[i] = (e[i] >> 1) | (i < 3 ? e[i + 1] << 63 : 0);
  fe t, s;
  fe_pow(F, &t, a, e, 4);
  fe_sqr(F, &s, &t);
  if (!fe_eq(&s, a)) return 0;
  *o = t;
  return 1;
}

/* ------------------------------------------------------------------ Fq2 */
void fe2_add(fe2* o, const fe2* a, const fe2* b) { fe_add(&FQ, &o->c0, &a->c0, &b->c0); fe_add(&FQ, &o->c1, &a->c1, &b->c1); }
void fe2_sub(fe2* o, const fe2* a, const fe2* b) { fe_sub(&FQ, &o->c0, &a->c0, &b->c0); fe_sub(&FQ, &o->c1, &a->c1, &b->c1); }
void fe2_neg(fe2* o, const fe2* a) { fe_neg(&FQ, &o->c0, &a->c0); fe_neg(&FQ, &o->c1, &a->c1); }
void fe2_dbl(fe2* o, const fe2* a) { fe2_add(o, a, a); }
void fe2_mul(fe2* o, const fe2* a, const fe2* b) {
  fe t0, t1, t2, s0, s1;
  fe_mul(&FQ, &t0, &a->c0, &b->c0);
  fe_mul(&FQ, &t1, &a->c1, &b->c1);
  fe_add(&FQ, &s0, &a->c0, &a->c1);
  fe_add(&FQ, &s1, &b->c0, &b->c1);
  fe_mul(&FQ, &t2, &s0, &s1);
  fe_sub(&FQ, &o->c0, &t0, &t1);           /* u^2 = -1 */
  fe_sub(&FQ, &t2, &t2, &t0);
  fe_sub(&FQ, &o->c1, &t2, &t1);
}
void fe2_sqr(fe2* o, const fe2* a) { fe2_mul(o, a, a); }
void fe2_inv(fe2* o, const fe2* a) {
  fe n, t;
  fe_sqr(&FQ, &n, &a->c0);
  fe_sqr(&FQ, &t, &a->c1);
  fe_add(&FQ, &n, &n, &t);
  fe_inv(&FQ, &n, &n);
  fe_mul(&FQ, &o->c0, &a->c0, &n);
  fe_mul(&FQ, &t, &a->c1, &n);
  fe_neg(&FQ, &o->c1, &t);
}
int fe2_is_zero(const fe2* a) { return fe_is_zero(&a->c0) && fe_is_zero(&a->c1); }
int fe2_eq(const fe2* a, const fe2* b) { return fe_eq(&a->c0, &b->c0) && fe_eq(&a->c1, &b->c1); }
int fe2_cmp(const fe2* a, const fe2* b) {
  int c = fe_cmp_canon(&FQ, &a->c1, &b->c1);
  if (c) return c;
  return fe_cmp_canon(&FQ, &a->c0, &b->c0);
}
void fe2_pow(fe2* o, const fe2* a, const uint64_t* e, int nlimbs) {
  fe2 r, b = *a;
  r.c0 = FQ.one;
  memset(&r.c1, 0, sizeof(fe));
  for (int i = nlimbs * 64 - 1; i >= 0; i--) {
    fe2_sqr(&r, &r);
    if ((e[i / 64] >> (i % 64)) & 1) fe2_mul(&r, &r, &b);
  }
  *o = r;
}
/* sqrt in Fq2 for q = 3 mod 4 (Adj & Rodriguez-Henriquez, Alg. 9).  Which root
 * is returned does not matter to callers: they select between y and -y by
 * arkworks ordering. */
int fe2_sqrt(fe2* o, const fe2* a) {
  if (fe2_is_zero(a)) { memset(o, 0, sizeof(*o)); return 1; }
  uint64_t e[4], three[4] = {3, 0, 0, 0}, one[4] = {1, 0, 0, 0};
  sub4(e, FQ.p, three);
  for (int k = 0; k < 2; k++)
    for (int i = 0; i < 4; i++) e[i] = (e[i] >> 1) | (i < 3 ? e[i + 1] << 63 : 0);
  fe2 a1, alpha, a0, x0, t;
  fe2_pow(&a1, a, e, 4);                 /* a^((q-3)/4) */
  fe2_mul(&t, &a1, a);
  fe2_mul(&alpha, &a1, &t);              /* a^((q-1)/2) */
  /* a0 = alpha^q * alpha = conj(alpha) * alpha = norm */
  fe2 conj = alpha;
  fe_neg(&FQ, &conj.c1, &alpha.c1);
  fe2_mul(&a0, &conj, &alpha);
  fe2 minus_one;
  fe_neg(&FQ, &minus_one.c0, &FQ.one);
  memset(&minus_one.c1, 0, sizeof(fe));
  if (fe2_eq(&a0, &minus_one)) return 0;
  fe2_mul(&x0, &a1, a);
  if (fe2_eq(&alpha, &minus_one)) {
    /* x = u * x0 */
    fe2 r;
    fe_neg(&FQ, &r.c0, &x0.c1);
    r.c1 = x0.c0;
    *o = r;
  } else {
    fe2 b = alpha;
    fe_add(&FQ, &b.c0, &b.c0, &FQ.one);
    uint64_t e2[4];
    sub4(e2, FQ.p, one);
    for (int i = 0; i < 4; i++) e2[i] = (e2[i] >> 1) | (i < 3 ? e2[i + 1] << 63 : 0);
    fe2_pow(&b, &b, e2, 4);
    fe2_mul(o, &b, &x0);
  }
  fe2 chk;
  fe2_sqr(&chk, o);
  return fe2_eq(&chk, a);
}

fe2 G2_B;

static void init_field(field* F) {
  /* inv = -p^{-1} mod 2^64 by Newton iteration */
  uint64_t x = 1;
  for (int i = 0; i < 7; i++) x *= 2 - F->p[0] * x;
  F->inv = (uint64_t)0 - x;
  /* one = 2^256 mod p by doubling 1 256 times; r2 = 2^512 mod p */
  uint64_t t[4] = {1, 0, 0, 0};
  for (int i = 0; i < 512; i++) {
    uint64_t c = add4(t, t, t);
    if (c || geq_p(t, F->p)) sub4(t, t, F->p);
    if (i == 255) memcpy(F->one.l, t, 32);
  }
  memcpy(F->r2.l, t, 32);
}

static int inited = 0;
void oracle_init(void) {
  if (inited) return;
  init_field(&FQ);
  init_field(&FR);
  /* G2_B = 3 / (9 + u) */
  fe2 nine_u, three;
  fe_set_u64(&FQ, &nine_u.c0, 9);
  nine_u.c1 = FQ.one;
  fe_set_u64(&FQ, &three.c0, 3);
  memset(&three.c1, 0, sizeof(fe));
  fe2 inv;
  fe2_inv(&inv, &nine_u);
  fe2_mul(&G2_B, &three, &inv);
  inited = 1;
}

void oracle_fr_mul(const uint64_t a[4], const uint64_t b[4], uint64_t o[4]) {
  oracle_init();
  fe x, y, z;
  fe_from_canon(&FR, &x, a);
  fe_from_canon(&FR, &y, b);
  fe_mul(&FR, &z, &x, &y);
  fe_to_canon(&FR, o, &z);
}
void oracle_fq_mul(const uint64_t a[4], const uint64_t b[4], uint64_t o[4]) {
  oracle_init();
  fe x, y, z;
  fe_from_canon(&FQ, &x, a);
  fe_from_canon(&FQ, &y, b);
  fe_mul(&FQ, &z, &x, &y);
  fe_to_canon(&FQ, o, &z);
}
void oracle_fr_inv(const uint64_t a[4], uint64_t o[4]) {
  oracle_init();
  fe x, z;
  fe_from_canon(&FR, &x, a);
  fe_inv(&FR, &z, &x);
  fe_to_canon(&FR, o, &z);
}
