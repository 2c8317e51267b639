/*
 * groth16.c — restatement of ark-groth16 0.5.0 (Cargo.lock:411) over BN254 for
 * explicit R1CS matrices, as reached from Groth16Prover::prove
 * (core/src/sequencer/settlement/prover.rs:408) and keygen
 * (prover/src/bin/keygen.rs:87-91) / the seed-42 demo (prover/src/snarkjs.rs:153-159).
 *   setup: alpha, beta, gamma, delta, G1gen, G2gen, t,
 *          LibsnarkReduction::instance_map_with_evaluation (App. A.7)
 *   prove: r, s; witness_map_from_matrices (§8a a5); 5 MSMs; assembly (a4, A.8)
 * Test infrastructure + CPU baseline only.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

void oracle_ntt_internal(fe* a, uint32_t log_n, int dir, int coset, int nthreads);
void oracle_msm_g1_internal(g1j* out, const g1a* bases, const uint64_t* scalars, size_t n, int nthreads);
void oracle_msm_g2_internal(g2j* out, const g2a* bases, const uint64_t* scalars, size_t n, int nthreads);
void oracle_g1j_to_canon(uint64_t p[8], const g1j* j);
void oracle_g2j_to_canon(uint64_t p[16], const g2j* j);

typedef struct {
  size_t n, num_instance, num_witness;
  uint32_t log_n;
  g1a alpha_g1, beta_g1, delta_g1;
  g2a beta_g2, gamma_g2, delta_g2;
  g1a* gamma_abc;  /* num_instance */
  g1a* a_query;    /* num_instance + num_witness */
  g1a* b_g1_query; /* num_instance + num_witness */
  g2a* b_g2_query; /* num_instance + num_witness */
  g1a* h_query;    /* n - 1 */
  g1a* l_query;    /* num_witness */
} opk;

static uint32_t domain_log(size_t need) {
  uint32_t k = 0;
  while (((size_t)1 << k) < need) k++;
  return k;
}
static fe domain_omega(uint32_t log_n) {
  uint64_t c[4];
  extern void oracle_domain_omega(uint32_t, uint64_t*);
  oracle_domain_omega(log_n, c);
  fe w;
  fe_from_canon(&FR, &w, c);
  return w;
}

/* sum coeff * z[col] over one CSR row (ark-relations evaluate_constraint) */
static void eval_row(fe* o, const uint64_t* rowptr, const uint64_t* col, const uint64_t* val,
                     size_t row, const fe* z) {
  fe acc;
  memset(&acc, 0, sizeof(acc));
  for (uint64_t k = rowptr[row]; k < rowptr[row + 1]; k++) {
    fe c, t;
    fe_from_canon(&FR, &c, val + 4 * k);
    fe_mul(&FR, &t, &c, &z[col[k]]);
    fe_add(&FR, &acc, &acc, &t);
  }
  *o = acc;
}

/* ----------------------------------------------------------- witness map */
static fe* witness_map_internal(const oracle_r1cs* cs, const fe* z, uint32_t* log_n_out, int nthreads) {
  size_t m = cs->num_constraints, l = cs->num_instance;
  uint32_t log_n = domain_log(m + l);
  size_t n = (size_t)1 << log_n;
  fe* a = (fe*)calloc(n, sizeof(fe));
  fe* b = (fe*)calloc(n, sizeof(fe));
  fe* c = (fe*)calloc(n, sizeof(fe));
  for (size_t i = 0; i < m; i++) {
    eval_row(&a[i], cs->a_rowptr, cs->a_col, cs->a_val, i, z);
    eval_row(&b[i], cs->b_rowptr, cs->b_col, cs->b_val, i, z);
    eval_row(&c[i], cs->c_rowptr, cs->c_col, cs->c_val, i, z);
  }
  for (size_t j = 0; j < l; j++) a[m + j] = z[j];
  oracle_ntt_internal(a, log_n, 1, 0, nthreads);
  oracle_ntt_internal(b, log_n, 1, 0, nthreads);
  oracle_ntt_internal(a, log_n, 0, 1, nthreads);
  oracle_ntt_internal(b, log_n, 0, 1, nthreads);
  oracle_ntt_internal(c, log_n, 1, 0, nthreads);
  oracle_ntt_internal(c, log_n, 0, 1, nthreads);
  /* (g^n - 1)^-1 */
  fe g, gn, vinv;
  fe_set_u64(&FR, &g, 5);
  uint64_t e[4] = {n, 0, 0, 0};
  fe_pow(&FR, &gn, &g, e, 1);
  fe_sub(&FR, &vinv, &gn, &FR.one);
  fe_inv(&FR, &vinv, &vinv);
  for (size_t i = 0; i < n; i++) {
    fe t;
    fe_mul(&FR, &t, &a[i], &b[i]);
    fe_sub(&FR, &t, &t, &c[i]);
    fe_mul(&FR, &a[i], &t, &vinv);
  }
  oracle_ntt_internal(a, log_n, 1, 1, nthreads);
  free(b);
  free(c);
  *log_n_out = log_n;
  return a;
}

int oracle_witness_map(const oracle_r1cs* cs, const uint64_t* zc, uint64_t* h, int nthreads) {
  oracle_init();
  size_t nv = cs->num_instance + cs->num_witness;
  fe* z = (fe*)malloc(nv * sizeof(fe));
  for (size_t i = 0; i < nv; i++) fe_from_canon(&FR, &z[i], zc + 4 * i);
  uint32_t log_n;
  fe* hh = witness_map_internal(cs, z, &log_n, nthreads);
  for (size_t i = 0; i < ((size_t)1 << log_n); i++) fe_to_canon(&FR, h + 4 * i, &hh[i]);
  free(hh);
  free(z);
  return 0;
}

/* first constraint i with <A_i,z> * <B_i,z> != <C_i,z>, or -1 (test helper) */
long long oracle_r1cs_check(const oracle_r1cs* cs, const uint64_t* zc) {
  oracle_init();
  size_t nv = cs->num_instance + cs->num_witness;
  fe* z = (fe*)malloc(nv * sizeof(fe));
  for (size_t i = 0; i < nv; i++) fe_from_canon(&FR, &z[i], zc + 4 * i);
  long long bad = -1;
  for (size_t i = 0; i < cs->num_constraints && bad < 0; i++) {
    fe a, b, c, ab;
    eval_row(&a, cs->a_rowptr, cs->a_col, cs->a_val, i, z);
    eval_row(&b, cs->b_rowptr, cs->b_col, cs->b_val, i, z);
    eval_row(&c, cs->c_rowptr, cs->c_col, cs->c_val, i, z);
    fe_mul(&FR, &ab, &a, &b);
    if (!fe_eq(&ab, &c)) bad = (long long)i;
  }
  free(z);
  return bad;
}

/* ------------------------------------------------ fixed-base scalar mults */
/* table[i][j] = j * 2^(8i) * G (affine), 32 x 256 */
typedef struct { g1a* t1; g2a* t2; } fb_table;
static void fb_build_g1(g1a* tab, const g1j* gen) {
  g1j base = *gen;
  for (int i = 0; i < 32; i++) {
    g1j acc;
    g1_set_inf(&acc);
    for (int j = 0; j < 256; j++) {
      g1_to_affine(&tab[i * 256 + j], &acc);
      g1_add(&acc, &acc, &base);
    }
    for (int k = 0; k < 8; k++) g1_dbl(&base, &base);
  }
}
static void fb_build_g2(g2a* tab, const g2j* gen) {
  g2j base = *gen;
  for (int i = 0; i < 32; i++) {
    g2j acc;
    g2_set_inf(&acc);
    for (int j = 0; j < 256; j++) {
      g2_to_affine(&tab[i * 256 + j], &acc);
      g2_add(&acc, &acc, &base);
    }
    for (int k = 0; k < 8; k++) g2_dbl(&base, &base);
  }
}
typedef struct { int g2; const void* tab; const fe* sc; void* out; size_t lo, hi; } fb_job;
static void* fb_worker(void* arg) {
  fb_job* jb = (fb_job*)arg;
  for (size_t i = jb->lo; i < jb->hi; i++) {
    uint64_t k[4];
    fe_to_canon(&FR, k, &jb->sc[i]);
    if (!jb->g2) {
      const g1a* tab = (const g1a*)jb->tab;
      g1j acc;
      g1_set_inf(&acc);
      for (int w = 0; w < 32; w++) {
        int d = (int)((k[w / 8] >> (8 * (w % 8))) & 0xff);
        if (d) g1_add_mixed(&acc, &acc, &tab[w * 256 + d]);
      }
      g1_to_affine(&((g1a*)jb->out)[i], &acc);
    } else {
      const g2a* tab = (const g2a*)jb->tab;
      g2j acc;
      g2_set_inf(&acc);
      for (int w = 0; w < 32; w++) {
        int d = (int)((k[w / 8] >> (8 * (w % 8))) & 0xff);
        if (d) g2_add_mixed(&acc, &acc, &tab[w * 256 + d]);
      }
      g2_to_affine(&((g2a*)jb->out)[i], &acc);
    }
  }
  return NULL;
}
static void fb_msm(int g2, const void* tab, const fe* sc, size_t cnt, void* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(nthreads * sizeof(pthread_t));
  fb_job* jobs = (fb_job*)malloc(nthreads * sizeof(fb_job));
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (fb_job){g2, tab, sc, out, cnt * t / nthreads, cnt * (t + 1) / nthreads};
    pthread_create(&th[t], NULL, fb_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

/* ------------------------------------------------------------------ setup */
void* oracle_groth16_setup(const oracle_r1cs* cs, void* rngp, int nthreads) {
  oracle_init();
  chacha_rng* rng = (chacha_rng*)rngp;
  fe alpha, beta, gamma, delta;
  fe_rand(&FR, &alpha, rng);
  fe_rand(&FR, &beta, rng);
  fe_rand(&FR, &gamma, rng);
  fe_rand(&FR, &delta, rng);
  g1j g1gen;
  g2j g2gen;
  g1_rand(&g1gen, rng);
  g2_rand(&g2gen, rng);

  size_t m = cs->num_constraints, l = cs->num_instance, w = cs->num_witness, nv = l + w;
  uint32_t log_n = domain_log(m + l);
  size_t n = (size_t)1 << log_n;
  fe omega = domain_omega(log_n);
  /* t = Fr::rand while Z(t) == 0 (sample_element_outside_domain) */
  fe t, zt, tn;
  uint64_t en[4] = {n, 0, 0, 0};
  for (;;) {
    fe_rand(&FR, &t, rng);
    fe_pow(&FR, &tn, &t, en, 1);
    fe_sub(&FR, &zt, &tn, &FR.one);
    if (!fe_is_zero(&zt)) break;
  }
  /* Lagrange coefficients L_i(t) = Z(t) w^i / (n (t - w^i)) */
  fe* u = (fe*)malloc(n * sizeof(fe));
  {
    fe ninv, wi = FR.one, zn;
    fe_set_u64(&FR, &ninv, (uint64_t)n);
    fe_inv(&FR, &ninv, &ninv);
    fe_mul(&FR, &zn, &zt, &ninv);
    /* batch inversion of (t - w^i) */
    fe* d = (fe*)malloc(n * sizeof(fe));
    fe* pre = (fe*)malloc(n * sizeof(fe));
    fe* wp = (fe*)malloc(n * sizeof(fe));
    fe run = FR.one;
    for (size_t i = 0; i < n; i++) {
      wp[i] = wi;
      fe_sub(&FR, &d[i], &t, &wi);
      pre[i] = run;
      fe_mul(&FR, &run, &run, &d[i]);
      fe_mul(&FR, &wi, &wi, &omega);
    }
    fe inv;
    fe_inv(&FR, &inv, &run);
    for (size_t i = n; i-- > 0;) {
      fe di;
      fe_mul(&FR, &di, &inv, &pre[i]);
      fe_mul(&FR, &inv, &inv, &d[i]);
      fe_mul(&FR, &u[i], &zn, &wp[i]);
      fe_mul(&FR, &u[i], &u[i], &di);
    }
    free(d);
    free(pre);
    free(wp);
  }
  fe* A = (fe*)calloc(nv, sizeof(fe));
  fe* B = (fe*)calloc(nv, sizeof(fe));
  fe* C = (fe*)calloc(nv, sizeof(fe));
  for (size_t j = 0; j < l; j++) A[j] = u[m + j];
  for (size_t i = 0; i < m; i++) {
    const uint64_t* rp[3] = {cs->a_rowptr, cs->b_rowptr, cs->c_rowptr};
    const uint64_t* cl[3] = {cs->a_col, cs->b_col, cs->c_col};
    const uint64_t* vl[3] = {cs->a_val, cs->b_val, cs->c_val};
    fe* dst[3] = {A, B, C};
    for (int mtx = 0; mtx < 3; mtx++)
      for (uint64_t k = rp[mtx][i]; k < rp[mtx][i + 1]; k++) {
        fe cf, tt;
        fe_from_canon(&FR, &cf, vl[mtx] + 4 * k);
        fe_mul(&FR, &tt, &u[i], &cf);
        fe_add(&FR, &dst[mtx][cl[mtx][k]], &dst[mtx][cl[mtx][k]], &tt);
      }
  }
  free(u);
  fe gamma_inv, delta_inv;
  fe_inv(&FR, &gamma_inv, &gamma);
  fe_inv(&FR, &delta_inv, &delta);
  fe* gabc = (fe*)malloc(l * sizeof(fe));
  fe* L = (fe*)malloc((w + 1) * sizeof(fe));
  for (size_t j = 0; j < nv; j++) {
    fe x, y;
    fe_mul(&FR, &x, &beta, &A[j]);
    fe_mul(&FR, &y, &alpha, &B[j]);
    fe_add(&FR, &x, &x, &y);
    fe_add(&FR, &x, &x, &C[j]);
    if (j < l) fe_mul(&FR, &gabc[j], &x, &gamma_inv);
    else fe_mul(&FR, &L[j - l], &x, &delta_inv);
  }
  fe* H = (fe*)malloc(n * sizeof(fe));
  {
    fe base, tp = FR.one;
    fe_mul(&FR, &base, &zt, &delta_inv);
    for (size_t i = 0; i + 1 < n; i++) {
      fe_mul(&FR, &H[i], &base, &tp);
      fe_mul(&FR, &tp, &tp, &t);
    }
  }

  opk* pk = (opk*)calloc(1, sizeof(opk));
  pk->n = n;
  pk->log_n = log_n;
  pk->num_instance = l;
  pk->num_witness = w;
  g1a* t1 = (g1a*)malloc(32 * 256 * sizeof(g1a));
  g2a* t2 = (g2a*)malloc(32 * 256 * sizeof(g2a));
  fb_build_g1(t1, &g1gen);
  fb_build_g2(t2, &g2gen);
  pk->gamma_abc = (g1a*)malloc(l * sizeof(g1a));
  pk->a_query = (g1a*)malloc(nv * sizeof(g1a));
  pk->b_g1_query = (g1a*)malloc(nv * sizeof(g1a));
  pk->b_g2_query = (g2a*)malloc(nv * sizeof(g2a));
  pk->h_query = (g1a*)malloc((n - 1 + 1) * sizeof(g1a));
  pk->l_query = (g1a*)malloc((w + 1) * sizeof(g1a));
  fb_msm(1, t2, B, nv, pk->b_g2_query, nthreads);
  fb_msm(0, t1, A, nv, pk->a_query, nthreads);
  fb_msm(0, t1, B, nv, pk->b_g1_query, nthreads);
  fb_msm(0, t1, H, n - 1, pk->h_query, nthreads);
  fb_msm(0, t1, L, w, pk->l_query, nthreads);
  fb_msm(0, t1, gabc, l, pk->gamma_abc, nthreads);
  fe sc[3] = {alpha, beta, delta};
  g1a o1[3];
  fb_msm(0, t1, sc, 3, o1, 1);
  pk->alpha_g1 = o1[0];
  pk->beta_g1 = o1[1];
  pk->delta_g1 = o1[2];
  fe sc2[3] = {beta, gamma, delta};
  g2a o2[3];
  fb_msm(1, t2, sc2, 3, o2, 1);
  pk->beta_g2 = o2[0];
  pk->gamma_g2 = o2[1];
  pk->delta_g2 = o2[2];
  free(t1);
  free(t2);
  free(A);
  free(B);
  free(C);
  free(gabc);
  free(L);
  free(H);
  return pk;
}

void oracle_pk_free(void* p) {
  opk* pk = (opk*)p;
  if (!pk) return;
  free(pk->gamma_abc);
  free(pk->a_query);
  free(pk->b_g1_query);
  free(pk->b_g2_query);
  free(pk->h_query);
  free(pk->l_query);
  free(pk);
}
void oracle_pk_sizes(const void* p, uint64_t out[4]) {
  const opk* pk = (const opk*)p;
  out[0] = pk->n;
  out[1] = pk->num_instance;
  out[2] = pk->num_witness;
  out[3] = pk->n - 1;
}

/* ------------------------------------------------------------ serialization */
void oracle_g1_serialize(const uint64_t p[8], int compress, uint8_t* out);
void oracle_g2_serialize(const uint64_t p[16], int compress, uint8_t* out);
typedef struct { uint8_t* buf; size_t cap, len; } sink;
static void put(sink* s, const void* d, size_t n) {
  if (s->buf && s->len + n <= s->cap) memcpy(s->buf + s->len, d, n);
  s->len += n;
}
static void put_g1(sink* s, const g1a* a, int compress) {
  uint64_t c[8];
  uint8_t b[64];
  if (a->inf) memset(c, 0, 64);
  else { fe_to_canon(&FQ, c, &a->x); fe_to_canon(&FQ, c + 4, &a->y); }
  oracle_g1_serialize(c, compress, b);
  put(s, b, compress ? 32 : 64);
}
static void put_g2(sink* s, const g2a* a, int compress) {
  uint64_t c[16];
  uint8_t b[128];
  if (a->inf) memset(c, 0, 128);
  else {
    fe_to_canon(&FQ, c, &a->x.c0); fe_to_canon(&FQ, c + 4, &a->x.c1);
    fe_to_canon(&FQ, c + 8, &a->y.c0); fe_to_canon(&FQ, c + 12, &a->y.c1);
  }
  oracle_g2_serialize(c, compress, b);
  put(s, b, compress ? 64 : 128);
}
static void put_len(sink* s, uint64_t n) {
  uint8_t b[8];
  for (int i = 0; i < 8; i++) b[i] = (uint8_t)(n >> (8 * i));
  put(s, b, 8);
}
static void put_vk(sink* s, const opk* pk, int compress) {
  put_g1(s, &pk->alpha_g1, compress);
  put_g2(s, &pk->beta_g2, compress);
  put_g2(s, &pk->gamma_g2, compress);
  put_g2(s, &pk->delta_g2, compress);
  put_len(s, pk->num_instance);
  for (size_t i = 0; i < pk->num_instance; i++) put_g1(s, &pk->gamma_abc[i], compress);
}
size_t oracle_vk_serialize(const void* p, int compress, uint8_t* buf, size_t cap) {
  sink s = {buf, cap, 0};
  put_vk(&s, (const opk*)p, compress);
  return s.len;
}
size_t oracle_pk_serialize(const void* p, int compress, uint8_t* buf, size_t cap) {
  const opk* pk = (const opk*)p;
  sink s = {buf, cap, 0};
  size_t nv = pk->num_instance + pk->num_witness;
  put_vk(&s, pk, compress);
  put_g1(&s, &pk->beta_g1, compress);
  put_g1(&s, &pk->delta_g1, compress);
  put_len(&s, nv);
  for (size_t i = 0; i < nv; i++) put_g1(&s, &pk->a_query[i], compress);
  put_len(&s, nv);
  for (size_t i = 0; i < nv; i++) put_g1(&s, &pk->b_g1_query[i], compress);
  put_len(&s, nv);
  for (size_t i = 0; i < nv; i++) put_g2(&s, &pk->b_g2_query[i], compress);
  put_len(&s, pk->n - 1);
  for (size_t i = 0; i + 1 < pk->n; i++) put_g1(&s, &pk->h_query[i], compress);
  put_len(&s, pk->num_witness);
  for (size_t i = 0; i < pk->num_witness; i++) put_g1(&s, &pk->l_query[i], compress);
  return s.len;
}

/* ------------------------------------------------------------------ prove */
static void fe_vec_to_canon(uint64_t* out, const fe* v, size_t n) {
  for (size_t i = 0; i < n; i++) fe_to_canon(&FR, out + 4 * i, &v[i]);
}
int oracle_groth16_prove(const void* p, const oracle_r1cs* cs, const uint64_t* zc, void* rngp,
                         const uint64_t* rs, int nthreads, uint64_t out_a[8], uint64_t out_b[16],
                         uint64_t out_c[8], uint64_t* out_h) {
  oracle_init();
  const opk* pk = (const opk*)p;
  fe r, s;
  if (rs) {
    fe_from_canon(&FR, &r, rs);
    fe_from_canon(&FR, &s, rs + 4);
  } else {
    fe_rand(&FR, &r, (chacha_rng*)rngp);
    fe_rand(&FR, &s, (chacha_rng*)rngp);
  }
  size_t l = cs->num_instance, w = cs->num_witness, nv = l + w;
  fe* z = (fe*)malloc(nv * sizeof(fe));
  for (size_t i = 0; i < nv; i++) fe_from_canon(&FR, &z[i], zc + 4 * i);
  uint32_t log_n;
  fe* h = witness_map_internal(cs, z, &log_n, nthreads);
  size_t n = (size_t)1 << log_n;
  if (n != pk->n) { free(h); free(z); return -1; }
  uint64_t* hc = (uint64_t*)malloc(n * 32);
  fe_vec_to_canon(hc, h, n);
  if (out_h) memcpy(out_h, hc, n * 32);
  uint64_t* zcan = (uint64_t*)malloc(nv * 32);
  fe_vec_to_canon(zcan, z, nv);

  g1j h_acc, l_acc, a_acc, b1_acc;
  g2j b2_acc;
  oracle_msm_g1_internal(&h_acc, pk->h_query, hc, n - 1, nthreads);
  oracle_msm_g1_internal(&l_acc, pk->l_query, zcan + 4 * l, w, nthreads);
  /* assignment = instance[1..] ++ witness = z[1..] ; query[1..] */
  oracle_msm_g1_internal(&a_acc, pk->a_query + 1, zcan + 4, nv - 1, nthreads);
  oracle_msm_g1_internal(&b1_acc, pk->b_g1_query + 1, zcan + 4, nv - 1, nthreads);
  oracle_msm_g2_internal(&b2_acc, pk->b_g2_query + 1, zcan + 4, nv - 1, nthreads);

  uint64_t rc[4], sc[4], rsc[4];
  fe rsv;
  fe_mul(&FR, &rsv, &r, &s);
  fe_to_canon(&FR, rc, &r);
  fe_to_canon(&FR, sc, &s);
  fe_to_canon(&FR, rsc, &rsv);
  g1j delta1, t1;
  g1_from_affine(&delta1, &pk->delta_g1);
  /* A = r*delta + a_query[0] + msm + alpha */
  g1j g_a;
  g1_mul(&g_a, &delta1, rc);
  g1_add_mixed(&g_a, &g_a, &pk->a_query[0]);
  g1_add(&g_a, &g_a, &a_acc);
  g1_add_mixed(&g_a, &g_a, &pk->alpha_g1);
  /* B in G1 (r != 0) */
  g1j g1_b;
  g1_set_inf(&g1_b);
  if (!fe_is_zero(&r)) {
    g1_mul(&g1_b, &delta1, sc);
    g1_add_mixed(&g1_b, &g1_b, &pk->b_g1_query[0]);
    g1_add(&g1_b, &g1_b, &b1_acc);
    g1_add_mixed(&g1_b, &g1_b, &pk->beta_g1);
  }
  /* B in G2 */
  g2j delta2, g2_b;
  g2_from_affine(&delta2, &pk->delta_g2);
  g2_mul(&g2_b, &delta2, sc, 4);
  g2_add_mixed(&g2_b, &g2_b, &pk->b_g2_query[0]);
  g2_add(&g2_b, &g2_b, &b2_acc);
  g2_add_mixed(&g2_b, &g2_b, &pk->beta_g2);
  /* C = s*A + r*B1 - rs*delta + l + h */
  g1j g_c;
  g1_mul(&g_c, &g_a, sc);
  g1_mul(&t1, &g1_b, rc);
  g1_add(&g_c, &g_c, &t1);
  g1_mul(&t1, &delta1, rsc);
  g1_neg(&t1, &t1);
  g1_add(&g_c, &g_c, &t1);
  g1_add(&g_c, &g_c, &l_acc);
  g1_add(&g_c, &g_c, &h_acc);

  oracle_g1j_to_canon(out_a, &g_a);
  oracle_g2j_to_canon(out_b, &g2_b);
  oracle_g1j_to_canon(out_c, &g_c);
  free(h);
  free(hc);
  free(z);
  free(zcan);
  return 0;
}

/* raw pk export for tests: canonical affine arrays (caller sizes via pk_sizes) */
static void ex_g1(uint64_t* o, const g1a* a) {
  if (a->inf) { memset(o, 0, 64); return; }
  fe_to_canon(&FQ, o, &a->x);
  fe_to_canon(&FQ, o + 4, &a->y);
}
static void ex_g2(uint64_t* o, const g2a* a) {
  if (a->inf) { memset(o, 0, 128); return; }
  fe_to_canon(&FQ, o, &a->x.c0); fe_to_canon(&FQ, o + 4, &a->x.c1);
  fe_to_canon(&FQ, o + 8, &a->y.c0); fe_to_canon(&FQ, o + 12, &a->y.c1);
}
/* which: 0 alpha_g1,1 beta_g1,2 delta_g1 (G1, idx ignored); 3 beta_g2,4 gamma_g2,
 * 5 delta_g2 (G2); 6 gamma_abc[idx], 7 a_query, 8 b_g1_query, 9 b_g2_query (G2),
 * 10 h_query, 11 l_query */
void oracle_pk_get(const void* p, int which, size_t idx, uint64_t* out) {
  const opk* pk = (const opk*)p;
  switch (which) {
    case 0: ex_g1(out, &pk->alpha_g1); break;
    case 1: ex_g1(out, &pk->beta_g1); break;
    case 2: ex_g1(out, &pk->delta_g1); break;
    case 3: ex_g2(out, &pk->beta_g2); break;
    case 4: ex_g2(out, &pk->gamma_g2); break;
    case 5: ex_g2(out, &pk->delta_g2); break;
    case 6: ex_g1(out, &pk->gamma_abc[idx]); break;
    case 7: ex_g1(out, &pk->a_query[idx]); break;
    case 8: ex_g1(out, &pk->b_g1_query[idx]); break;
    case 9: ex_g2(out, &pk->b_g2_query[idx]); break;
    case 10: ex_g1(out, &pk->h_query[idx]); break;
    case 11: ex_g1(out, &pk->l_query[idx]); break;
  }
}
