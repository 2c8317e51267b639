/*
 * api.c — canonical-bytes C API of the oracle, arkworks point serialization
 * (ark-serialize 0.5.0 / ark-ec 0.5.0 SWFlags) and
 * deterministic synthetic-input generators.
 * Test infrastructure only.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

/* ---- canonical <-> internal ---- */
static void g1a_from_canon(g1a* a, const uint64_t p[8]) {
  int z = 1;
  for (int i = 0; i < 8; i++) z &= p[i] == 0;
  memset(a, 0, sizeof(*a));
  if (z) { a->inf = 1; return; }
  fe_from_canon(&FQ, &a->x, p);
  fe_from_canon(&FQ, &a->y, p + 4);
}
static void g1a_to_canon(uint64_t p[8], const g1a* a) {
  if (a->inf) { memset(p, 0, 64); return; }
  fe_to_canon(&FQ, p, &a->x);
  fe_to_canon(&FQ, p + 4, &a->y);
}
static void g2a_from_canon(g2a* a, const uint64_t p[16]) {
  int z = 1;
  for (int i = 0; i < 16; i++) z &= p[i] == 0;
  memset(a, 0, sizeof(*a));
  if (z) { a->inf = 1; return; }
  fe_from_canon(&FQ, &a->x.c0, p);
  fe_from_canon(&FQ, &a->x.c1, p + 4);
  fe_from_canon(&FQ, &a->y.c0, p + 8);
  fe_from_canon(&FQ, &a->y.c1, p + 12);
}
static void g2a_to_canon(uint64_t p[16], const g2a* a) {
  if (a->inf) { memset(p, 0, 128); return; }
  fe_to_canon(&FQ, p, &a->x.c0);
  fe_to_canon(&FQ, p + 4, &a->x.c1);
  fe_to_canon(&FQ, p + 8, &a->y.c0);
  fe_to_canon(&FQ, p + 12, &a->y.c1);
}
void oracle_g1j_to_canon(uint64_t p[8], const g1j* j) {
  g1a a;
  g1_to_affine(&a, j);
  g1a_to_canon(p, &a);
}
void oracle_g2j_to_canon(uint64_t p[16], const g2j* j) {
  g2a a;
  g2_to_affine(&a, j);
  g2a_to_canon(p, &a);
}
void oracle_g1a_from_canon(g1a* a, const uint64_t p[8]) { g1a_from_canon(a, p); }
void oracle_g2a_from_canon(g2a* a, const uint64_t p[16]) { g2a_from_canon(a, p); }

void oracle_g1_rand(void* rng, uint64_t out[8]) {
  g1j p;
  g1_rand(&p, (chacha_rng*)rng);
  oracle_g1j_to_canon(out, &p);
}
void oracle_g2_rand(void* rng, uint64_t out[16]) {
  g2j p;
  g2_rand(&p, (chacha_rng*)rng);
  oracle_g2j_to_canon(out, &p);
}
void oracle_g1_add(const uint64_t a[8], const uint64_t b[8], uint64_t o[8]) {
  oracle_init();
  g1a x, y;
  g1j j;
  g1a_from_canon(&x, a);
  g1a_from_canon(&y, b);
  g1_from_affine(&j, &x);
  g1_add_mixed(&j, &j, &y);
  oracle_g1j_to_canon(o, &j);
}
void oracle_g1_mul(const uint64_t p[8], const uint64_t k[4], uint64_t o[8]) {
  oracle_init();
  g1a x;
  g1j j;
  g1a_from_canon(&x, p);
  g1_from_affine(&j, &x);
  g1_mul(&j, &j, k);
  oracle_g1j_to_canon(o, &j);
}
void oracle_g2_mul(const uint64_t p[16], const uint64_t k[4], uint64_t o[16]) {
  oracle_init();
  g2a x;
  g2j j;
  g2a_from_canon(&x, p);
  g2_from_affine(&j, &x);
  g2_mul(&j, &j, k, 4);
  oracle_g2j_to_canon(o, &j);
}
int oracle_g1_on_curve(const uint64_t p[8]) {
  oracle_init();
  g1a a;
  g1a_from_canon(&a, p);
  return g1_is_on_curve(&a);
}
int oracle_g2_on_curve(const uint64_t p[16]) {
  oracle_init();
  g2a a;
  g2a_from_canon(&a, p);
  return g2_is_on_curve(&a);
}

/* ------------------------------------------------------ serialization */
/* SWFlags (ark-ec 0.5 models/short_weierstrass/serialization_flags.rs):
 * YIsNegative = bit 7 ("y > -y"), PointAtInfinity = bit 6, both carried in the
 * top bits of the last byte of the last serialized field element. */
static void put_canon(uint8_t* out, const uint64_t c[4]) {
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(c[i / 8] >> (8 * (i % 8)));
}
static void get_canon(uint64_t c[4], const uint8_t* in) {
  memset(c, 0, 32);
  for (int i = 0; i < 32; i++) c[i / 8] |= (uint64_t)in[i] << (8 * (i % 8));
}
void oracle_g1_serialize(const uint64_t p[8], int compress, uint8_t* out) {
  oracle_init();
  g1a a;
  g1a_from_canon(&a, p);
  size_t len = compress ? 32 : 64;
  memset(out, 0, len);
  if (a.inf) { out[len - 1] |= 0x40; return; }
  fe ny;
  fe_neg(&FQ, &ny, &a.y);
  int neg = fe_cmp_canon(&FQ, &a.y, &ny) > 0;
  put_canon(out, p);
  if (!compress) put_canon(out + 32, p + 4);
  if (neg) out[len - 1] |= 0x80;
}
void oracle_g2_serialize(const uint64_t p[16], int compress, uint8_t* out) {
  oracle_init();
  g2a a;
  g2a_from_canon(&a, p);
  size_t len = compress ? 64 : 128;
  memset(out, 0, len);
  if (a.inf) { out[len - 1] |= 0x40; return; }
  fe2 ny;
  fe2_neg(&ny, &a.y);
  int neg = fe2_cmp(&a.y, &ny) > 0;
  put_canon(out, p);
  put_canon(out + 32, p + 4);
  if (!compress) { put_canon(out + 64, p + 8); put_canon(out + 96, p + 12); }
  if (neg) out[len - 1] |= 0x80;
}
static int canon_lt_q(const uint64_t c[4]) {
  for (int i = 3; i >= 0; i--) {
    if (c[i] < FQ.p[i]) return 1;
    if (c[i] > FQ.p[i]) return 0;
  }
  return 0;
}
/* returns 1 on success (point validated on-curve; G2 subgroup checked) */
int oracle_g1_deserialize(const uint8_t* in, int compress, uint64_t out[8]) {
  oracle_init();
  size_t len = compress ? 32 : 64;
  uint8_t buf[64];
  memcpy(buf, in, len);
  int neg = (buf[len - 1] >> 7) & 1, inf = (buf[len - 1] >> 6) & 1;
  buf[len - 1] &= 0x3f;
  if (inf) { memset(out, 0, 64); return 1; }
  uint64_t x[4], y[4];
  get_canon(x, buf);
  if (!canon_lt_q(x)) return 0;
  g1a a;
  fe_from_canon(&FQ, &a.x, x);
  a.inf = 0;
  if (compress) {
    fe rhs, three;
    fe_sqr(&FQ, &rhs, &a.x);
    fe_mul(&FQ, &rhs, &rhs, &a.x);
    fe_set_u64(&FQ, &three, 3);
    fe_add(&FQ, &rhs, &rhs, &three);
    fe yy, ny;
    if (!fe_sqrt(&FQ, &yy, &rhs)) return 0;
    fe_neg(&FQ, &ny, &yy);
    fe smaller = yy, larger = ny;
    if (fe_cmp_canon(&FQ, &yy, &ny) >= 0) { smaller = ny; larger = yy; }
    a.y = neg ? larger : smaller;
  } else {
    get_canon(y, buf + 32);
    if (!canon_lt_q(y)) return 0;
    fe_from_canon(&FQ, &a.y, y);
  }
  if (!g1_is_on_curve(&a)) return 0;
  g1a_to_canon(out, &a);
  return 1;
}
static const uint64_t FR_MOD[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL,
                                   0xb85045b68181585dULL, 0x30644e72e131a029ULL};
int oracle_g2_in_subgroup(const g2a* a) {
  g2j p, r;
  g2_from_affine(&p, a);
  g2_mul(&r, &p, FR_MOD, 4);
  return fe2_is_zero(&r.z);
}
int oracle_g2_deserialize(const uint8_t* in, int compress, uint64_t out[16]) {
  oracle_init();
  size_t len = compress ? 64 : 128;
  uint8_t buf[128];
  memcpy(buf, in, len);
  int neg = (buf[len - 1] >> 7) & 1, inf = (buf[len - 1] >> 6) & 1;
  buf[len - 1] &= 0x3f;
  if (inf) { memset(out, 0, 128); return 1; }
  uint64_t c[4];
  g2a a;
  a.inf = 0;
  get_canon(c, buf);
  if (!canon_lt_q(c)) return 0;
  fe_from_canon(&FQ, &a.x.c0, c);
  get_canon(c, buf + 32);
  if (!canon_lt_q(c)) return 0;
  fe_from_canon(&FQ, &a.x.c1, c);
  if (compress) {
    fe2 rhs, yy, ny;
    fe2_sqr(&rhs, &a.x);
    fe2_mul(&rhs, &rhs, &a.x);
    fe2_add(&rhs, &rhs, &G2_B);
    if (!fe2_sqrt(&yy, &rhs)) return 0;
    fe2_neg(&ny, &yy);
    fe2 smaller = yy, larger = ny;
    if (fe2_cmp(&yy, &ny) >= 0) { smaller = ny; larger = yy; }
    a.y = neg ? larger : smaller;
  } else {
    get_canon(c, buf + 64);
    if (!canon_lt_q(c)) return 0;
    fe_from_canon(&FQ, &a.y.c0, c);
    get_canon(c, buf + 96);
    if (!canon_lt_q(c)) return 0;
    fe_from_canon(&FQ, &a.y.c1, c);
  }
  if (!g2_is_on_curve(&a)) return 0;
  if (!oracle_g2_in_subgroup(&a)) return 0;
  g2a_to_canon(out, &a);
  return 1;
}

/* ------------------------------------------------------ synthetic inputs */
void oracle_gen_scalars(uint64_t seed, size_t n, uint64_t* out) {
  oracle_init();
  chacha_rng r;
  rng_seed_from_u64(&r, seed);
  for (size_t i = 0; i < n; i++) {
    fe x;
    fe_rand(&FR, &x, &r);
    fe_to_canon(&FR, out + 4 * i, &x);
  }
}

/* P_i = P0 + i*D computed in chunks: chunk start by scalar mul, then adds;
 * Jacobian results normalised with Montgomery batch inversion. */
typedef struct {
  int g2;
  g1j p0, d;
  g2j p0_2, d_2;
  size_t n, lo, hi;
  uint64_t* out;
} genpts_job;

static void* genpts_worker(void* arg) {
  genpts_job* jb = (genpts_job*)arg;
  size_t cnt = jb->hi - jb->lo;
  if (cnt == 0) return NULL;
  uint64_t k[4] = {jb->lo, 0, 0, 0};
  if (!jb->g2) {
    g1j* acc = (g1j*)malloc(cnt * sizeof(g1j));
    g1j cur, t;
    g1_mul(&t, &jb->d, k);
    g1_add(&cur, &jb->p0, &t);
    for (size_t i = 0; i < cnt; i++) {
      acc[i] = cur;
      g1_add(&cur, &cur, &jb->d);
    }
    /* batch inversion of z */
    fe* pre = (fe*)malloc(cnt * sizeof(fe));
    fe run = FQ.one;
    for (size_t i = 0; i < cnt; i++) {
      pre[i] = run;
      fe_mul(&FQ, &run, &run, &acc[i].z);
    }
    fe inv;
    fe_inv(&FQ, &inv, &run);
    for (size_t i = cnt; i-- > 0;) {
      fe zi, zi2, zi3, x, y;
      fe_mul(&FQ, &zi, &inv, &pre[i]);
      fe_mul(&FQ, &inv, &inv, &acc[i].z);
      fe_sqr(&FQ, &zi2, &zi);
      fe_mul(&FQ, &zi3, &zi2, &zi);
      fe_mul(&FQ, &x, &acc[i].x, &zi2);
      fe_mul(&FQ, &y, &acc[i].y, &zi3);
      uint64_t* o = jb->out + 8 * (jb->lo + i);
      fe_to_canon(&FQ, o, &x);
      fe_to_canon(&FQ, o + 4, &y);
    }
    free(pre);
    free(acc);
  } else {
    g2j cur, t;
    g2_mul(&t, &jb->d_2, k, 4);
    g2_add(&cur, &jb->p0_2, &t);
    for (size_t i = 0; i < cnt; i++) {
      oracle_g2j_to_canon(jb->out + 16 * (jb->lo + i), &cur);
      g2_add(&cur, &cur, &jb->d_2);
    }
  }
  return NULL;
}

static void gen_points(int g2, uint64_t seed, size_t n, uint64_t* out, int nthreads) {
  oracle_init();
  chacha_rng r;
  rng_seed_from_u64(&r, seed);
  genpts_job base;
  memset(&base, 0, sizeof(base));
  base.g2 = g2;
  if (!g2) { g1_rand(&base.p0, &r); g1_rand(&base.d, &r); }
  else { g2_rand(&base.p0_2, &r); g2_rand(&base.d_2, &r); }
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(nthreads * sizeof(pthread_t));
  genpts_job* jobs = (genpts_job*)malloc(nthreads * sizeof(genpts_job));
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = base;
    jobs[t].n = n;
    jobs[t].lo = n * t / nthreads;
    jobs[t].hi = n * (t + 1) / nthreads;
    jobs[t].out = out;
    pthread_create(&th[t], NULL, genpts_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}
void oracle_gen_points_g1(uint64_t seed, size_t n, uint64_t* out, int nthreads) {
  gen_points(0, seed, n, out, nthreads);
}
void oracle_gen_points_g2(uint64_t seed, size_t n, uint64_t* out, int nthreads) {
  gen_points(1, seed, n, out, nthreads);
}
