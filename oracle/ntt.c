/*
 * ntt.c — ark-poly 0.5.0 Radix2EvaluationDomain (Cargo.lock:440) over BN254 Fr:
 * fft / ifft / coset variants in natural order, as used by ark-groth16's
 * LibsnarkReduction::witness_map_from_matrices.
 *   omega_n = g^((r-1)/2^28) ^ (2^28/n), g = Fr::GENERATOR = 5
 *   fft(a)[k]       = sum_i a_i omega^(ik)
 *   coset_fft(a)    = fft(a_i * g^i)
 *   ifft(A)[i]      = n^-1 sum_k A_k omega^(-ik)
 *   coset_ifft(A)   = ifft(A)_i * g^(-i)
 * Field results are exact, so any correct transform algorithm is bit-identical
 * to arkworks'.  This one is iterative radix-2 DIT after a bit-reversal, split
 * over pthreads stage by stage.  Test infrastructure + CPU baseline only.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static fe two_adic_root(void) {
  /* (r-1)/2^28 */
  uint64_t e[4];
  memcpy(e, FR.p, 32);
  e[0] -= 1;
  for (int k = 0; k < 28; k++)
    for (int i = 0; i < 4; i++) e[i] = (e[i] >> 1) | (i < 3 ? e[i + 1] << 63 : 0);
  fe g, w;
  fe_set_u64(&FR, &g, 5);
  fe_pow(&FR, &w, &g, e, 4);
  return w;
}

void oracle_domain_omega(uint32_t log_n, uint64_t out[4]) {
  oracle_init();
  fe w = two_adic_root();
  for (uint32_t i = log_n; i < 28; i++) fe_sqr(&FR, &w, &w);
  fe_to_canon(&FR, out, &w);
}

typedef struct {
  fe* a;
  const fe* tw; /* tw[j] = w^j, j < n/2 */
  uint32_t log_n;
  int tid, nthreads;
  pthread_barrier_t* bar;
} ntt_job;

static uint32_t bitrev(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

static void* ntt_worker(void* arg) {
  ntt_job* jb = (ntt_job*)arg;
  size_t n = (size_t)1 << jb->log_n;
  size_t lo = n * jb->tid / jb->nthreads, hi = n * (jb->tid + 1) / jb->nthreads;
  for (size_t i = lo; i < hi; i++) {
    size_t j = bitrev((uint32_t)i, jb->log_n);
    if (i < j) { fe t = jb->a[i]; jb->a[i] = jb->a[j]; jb->a[j] = t; }
  }
  pthread_barrier_wait(jb->bar);
  size_t half_total = n / 2;
  for (uint32_t s = 1; s <= jb->log_n; s++) {
    size_t m = (size_t)1 << s, h = m / 2, stride = n / m;
    /* butterfly index b in [0, n/2): block = b / h, j = b % h */
    size_t blo = half_total * jb->tid / jb->nthreads, bhi = half_total * (jb->tid + 1) / jb->nthreads;
    for (size_t b = blo; b < bhi; b++) {
      size_t blk = b / h, j = b % h;
      fe* u = &jb->a[blk * m + j];
      fe* v = u + h;
      fe t;
      fe_mul(&FR, &t, v, &jb->tw[j * stride]);
      fe_sub(&FR, v, u, &t);
      fe_add(&FR, u, u, &t);
    }
    pthread_barrier_wait(jb->bar);
  }
  return NULL;
}

/* in-place natural-order transform with root w (internal Montgomery data) */
static void ntt_core(fe* a, uint32_t log_n, const fe* w, int nthreads) {
  size_t n = (size_t)1 << log_n;
  if (n == 1) return;
  fe* tw = (fe*)malloc((n / 2) * sizeof(fe));
  tw[0] = FR.one;
  for (size_t j = 1; j < n / 2; j++) fe_mul(&FR, &tw[j], &tw[j - 1], w);
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n / 2) nthreads = (int)(n / 2);
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, nthreads);
  pthread_t* th = (pthread_t*)malloc(nthreads * sizeof(pthread_t));
  ntt_job* jobs = (ntt_job*)malloc(nthreads * sizeof(ntt_job));
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (ntt_job){a, tw, log_n, t, nthreads, &bar};
    pthread_create(&th[t], NULL, ntt_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  pthread_barrier_destroy(&bar);
  free(th);
  free(jobs);
  free(tw);
}

static void scale_powers(fe* a, size_t n, const fe* g) {
  fe p = FR.one;
  for (size_t i = 0; i < n; i++) {
    fe_mul(&FR, &a[i], &a[i], &p);
    fe_mul(&FR, &p, &p, g);
  }
}

/* internal (Montgomery) entry used by groth16.c */
void oracle_ntt_internal(fe* a, uint32_t log_n, int dir, int coset, int nthreads) {
  size_t n = (size_t)1 << log_n;
  fe w = two_adic_root();
  for (uint32_t i = log_n; i < 28; i++) fe_sqr(&FR, &w, &w);
  fe g;
  fe_set_u64(&FR, &g, 5);
  if (dir == 0) {
    if (coset) scale_powers(a, n, &g);
    ntt_core(a, log_n, &w, nthreads);
  } else {
    fe wi, ninv, gi;
    fe_inv(&FR, &wi, &w);
    ntt_core(a, log_n, &wi, nthreads);
    fe_set_u64(&FR, &ninv, (uint64_t)n);
    fe_inv(&FR, &ninv, &ninv);
    if (coset) {
      fe_inv(&FR, &gi, &g);
      fe p = ninv;
      for (size_t i = 0; i < n; i++) {
        fe_mul(&FR, &a[i], &a[i], &p);
        fe_mul(&FR, &p, &p, &gi);
      }
    } else {
      for (size_t i = 0; i < n; i++) fe_mul(&FR, &a[i], &a[i], &ninv);
    }
  }
}

void oracle_ntt(uint64_t* data, uint32_t log_n, int dir, int coset, int nthreads) {
  oracle_init();
  size_t n = (size_t)1 << log_n;
  fe* a = (fe*)malloc(n * sizeof(fe));
  for (size_t i = 0; i < n; i++) fe_from_canon(&FR, &a[i], data + 4 * i);
  oracle_ntt_internal(a, log_n, dir, coset, nthreads);
  for (size_t i = 0; i < n; i++) fe_to_canon(&FR, data + 4 * i, &a[i]);
  free(a);
}
