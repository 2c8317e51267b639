/*
 * msm.c — port of ark-ec 0.5.0 VariableBaseMSM::msm_bigint_wnaf (Cargo.lock:290)
 * as called 4x on G1 and 1x on G2 by ark-groth16's create_proof_with_assignment
 * (SURVEY.md §8a a7/a8).  Signed c-bit digits (make_digits), c = 3 for n < 32
 * else ln_without_floats(n) + 2 with ln_without_floats(n) = ceil_log2(n)*69/100,
 * 2^(c-1)... buckets per window, window sums in parallel (rayon over windows ->
 * pthreads over windows here), windows combined high-to-low by c doublings.
 * When the host has more threads than windows, each window is also cut into
 * point chunks (work item = window x chunk, chunk partials summed per window)
 * so every core works: the sum is the same group element, the CPU baseline
 * gets every core (bench.py), and no output changes.
 * Bases/scalars zip-truncate to the shorter input, as in arkworks.
 * Test infrastructure + timed CPU baseline ("port") only.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

void oracle_g1j_to_canon(uint64_t p[8], const g1j* j);
void oracle_g2j_to_canon(uint64_t p[16], const g2j* j);
void oracle_g1a_from_canon(g1a* a, const uint64_t p[8]);
void oracle_g2a_from_canon(g2a* a, const uint64_t p[16]);

static size_t ceil_log2(size_t n) {
  size_t k = 0;
  while (((size_t)1 << k) < n) k++;
  return k;
}
static int msm_window(size_t n) { return n < 32 ? 3 : (int)(ceil_log2(n) * 69 / 100) + 2; }

/* ark-ec make_digits: signed base-2^w digits, last digit absorbs the carry */
static void make_digits(const uint64_t s[4], int w, int num_bits, int32_t* out) {
  uint64_t radix = (uint64_t)1 << w, mask = radix - 1, carry = 0;
  int count = (num_bits + w - 1) / w;
  for (int i = 0; i < count; i++) {
    int bit_offset = i * w, u64_idx = bit_offset / 64, bit_idx = bit_offset % 64;
    uint64_t bit_buf;
    if (bit_idx < 64 - w || u64_idx == 3) bit_buf = s[u64_idx] >> bit_idx;
    else bit_buf = (s[u64_idx] >> bit_idx) | (s[u64_idx + 1] << (64 - bit_idx));
    uint64_t coef = carry + (bit_buf & mask);
    carry = (coef + radix / 2) >> w;
    int64_t digit = (int64_t)coef - (int64_t)(carry << w);
    if (i == count - 1) digit += (int64_t)(carry << w);
    out[i] = (int32_t)digit;
  }
}

/* chunks per window: minimises (rounds of work items) x (item time) with
 * item time ~ points per chunk + ~3 additions per bucket for its running sum */
static int msm_chunks(size_t n, int c, int count, int nthreads) {
  int best = 1;
  double best_t = 1e300;
  for (int k = 1; k <= 64; k++) {
    if ((size_t)k * 1024 > n && k > 1) break;
    double rounds = (double)(((size_t)count * k + nthreads - 1) / nthreads);
    double t = rounds * ((double)n / k + 3.0 * (double)((size_t)1 << c));
    if (t < best_t * 0.98) {
      best_t = t;
      best = k;
    }
  }
  return best;
}

#define DEFINE_MSM(P, J, A, T, NEG)                                                         \
  typedef struct {                                                                          \
    const A* bases; const int32_t* digits; size_t n; int c, count, next, nch;               \
    pthread_mutex_t* mu; J* sums;                                                           \
  } P##_msm_job;                                                                            \
  static void* P##_msm_worker(void* arg) {                                                  \
    P##_msm_job* jb = (P##_msm_job*)arg;                                                    \
    size_t nb = (size_t)1 << jb->c;                                                         \
    J* buckets = (J*)malloc(nb * sizeof(J));                                                \
    for (;;) {                                                                              \
      pthread_mutex_lock(jb->mu);                                                           \
      int item = jb->next++;                                                                \
      pthread_mutex_unlock(jb->mu);                                                         \
      if (item >= jb->count * jb->nch) break;                                               \
      int w = item / jb->nch, ch = item % jb->nch;                                          \
      size_t lo = jb->n * ch / jb->nch, hi = jb->n * (ch + 1) / jb->nch;                    \
      for (size_t b = 0; b < nb; b++) P##_set_inf(&buckets[b]);                             \
      for (size_t i = lo; i < hi; i++) {                                                    \
        int32_t d = jb->digits[i * jb->count + w];                                          \
        if (d > 0) P##_add_mixed(&buckets[d - 1], &buckets[d - 1], &jb->bases[i]);          \
        else if (d < 0) {                                                                   \
          A nb_ = jb->bases[i];                                                             \
          if (!nb_.inf) NEG(&nb_.y, &nb_.y);                                                \
          P##_add_mixed(&buckets[-d - 1], &buckets[-d - 1], &nb_);                          \
        }                                                                                   \
      }                                                                                     \
      J run, res;                                                                           \
      P##_set_inf(&run); P##_set_inf(&res);                                                 \
      for (size_t b = nb; b-- > 0;) { P##_add(&run, &run, &buckets[b]); P##_add(&res, &res, &run); } \
      jb->sums[item] = res;                                                                 \
    }                                                                                       \
    free(buckets);                                                                          \
    return NULL;                                                                            \
  }                                                                                         \
  typedef struct { const uint64_t* s; int32_t* d; size_t lo, hi; int c, count; } P##_dig_job; \
  static void* P##_dig_worker(void* arg) {                                                  \
    P##_dig_job* jb = (P##_dig_job*)arg;                                                    \
    for (size_t i = jb->lo; i < jb->hi; i++) make_digits(jb->s + 4 * i, jb->c, 254, jb->d + i * jb->count); \
    return NULL;                                                                            \
  }                                                                                         \
  static void P##_msm(J* out, const A* bases, const uint64_t* scalars, size_t n, int nthreads) { \
    if (nthreads < 1) nthreads = 1;                                                         \
    int c = msm_window(n), count = (254 + c - 1) / c;                                       \
    int32_t* digits = (int32_t*)malloc(n * count * sizeof(int32_t) + 8);                   \
    pthread_t* th = (pthread_t*)malloc(nthreads * sizeof(pthread_t));                       \
    P##_dig_job* dj = (P##_dig_job*)malloc(nthreads * sizeof(P##_dig_job));                 \
    for (int t = 0; t < nthreads; t++) {                                                    \
      dj[t].s = scalars; dj[t].d = digits; dj[t].c = c; dj[t].count = count;                \
      dj[t].lo = n * t / nthreads; dj[t].hi = n * (t + 1) / nthreads;                       \
      pthread_create(&th[t], NULL, P##_dig_worker, &dj[t]);                                 \
    }                                                                                       \
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);                           \
    int nch = msm_chunks(n, c, count, nthreads);                                            \
    J* sums = (J*)malloc((size_t)count * nch * sizeof(J));                                  \
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;                                         \
    P##_msm_job job = {bases, digits, n, c, count, 0, nch, &mu, sums};                      \
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, P##_msm_worker, &job);  \
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);                           \
    for (int w = 0; w < count; w++)                                                         \
      for (int k = 1; k < nch; k++) P##_add(&sums[w * nch], &sums[w * nch], &sums[w * nch + k]); \
    for (int w = 1; w < count; w++) sums[w] = sums[w * nch];                                \
    J total;                                                                                \
    P##_set_inf(&total);                                                                    \
    for (int w = count - 1; w >= 1; w--) {                                                  \
      P##_add(&total, &total, &sums[w]);                                                    \
      for (int k = 0; k < c; k++) P##_dbl(&total, &total);                                  \
    }                                                                                       \
    P##_add(out, &sums[0], &total);                                                         \
    free(sums); free(digits); free(th); free(dj);                                           \
  }

static void fq_neg_(fe* o, const fe* a) { fe_neg(&FQ, o, a); }
DEFINE_MSM(g1, g1j, g1a, fe, fq_neg_)
DEFINE_MSM(g2, g2j, g2a, fe2, fe2_neg)

void oracle_msm_g1_internal(g1j* out, const g1a* bases, const uint64_t* scalars, size_t n, int nthreads) {
  if (n == 0) { g1_set_inf(out); return; }
  g1_msm(out, bases, scalars, n, nthreads);
}
void oracle_msm_g2_internal(g2j* out, const g2a* bases, const uint64_t* scalars, size_t n, int nthreads) {
  if (n == 0) { g2_set_inf(out); return; }
  g2_msm(out, bases, scalars, n, nthreads);
}

void oracle_msm_g1(const uint64_t* points, const uint64_t* scalars, size_t n, int nthreads,
                   uint64_t out_affine[8]) {
  oracle_init();
  g1a* b = (g1a*)malloc((n + 1) * sizeof(g1a));
  for (size_t i = 0; i < n; i++) oracle_g1a_from_canon(&b[i], points + 8 * i);
  g1j r;
  oracle_msm_g1_internal(&r, b, scalars, n, nthreads);
  oracle_g1j_to_canon(out_affine, &r);
  free(b);
}
void oracle_msm_g2(const uint64_t* points, const uint64_t* scalars, size_t n, int nthreads,
                   uint64_t out_affine[16]) {
  oracle_init();
  g2a* b = (g2a*)malloc((n + 1) * sizeof(g2a));
  for (size_t i = 0; i < n; i++) oracle_g2a_from_canon(&b[i], points + 16 * i);
  g2j r;
  oracle_msm_g2_internal(&r, b, scalars, n, nthreads);
  oracle_g2j_to_canon(out_affine, &r);
  free(b);
}
