/*
 * rng.c — rand 0.8.5 StdRng = rand_chacha 0.3.1 ChaCha12Rng, seeded through
 * rand_core 0.6.4 SeedableRng::seed_from_u64 (PCG32 expansion), and ark-ff
 * 0.5.0 Fp::rand.  Reference call sites: prover.rs:354 (seed = batch_id),
 * keygen.rs:87 (seed 0), snarkjs.rs:153 (seed 42).  SURVEY.md Appendix A.1-A.2.
 * Test infrastructure only.
 *
 * KAT: seed_from_u64(42) first u64 = 0x86cc7763222724a2.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(a, b, c, d)                  \
  a += b; d ^= a; d = rotl(d, 16);      \
  c += d; b ^= c; b = rotl(b, 12);      \
  a += b; d ^= a; d = rotl(d, 8);       \
  c += d; b ^= c; b = rotl(b, 7);

static void chacha12_block(const uint32_t key[8], uint64_t ctr, uint32_t out[16]) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                     key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                     (uint32_t)ctr, (uint32_t)(ctr >> 32), 0, 0};
  uint32_t x[16];
  memcpy(x, in, sizeof(x));
  for (int i = 0; i < 6; i++) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}

void rng_seed_from_u64(chacha_rng* r, uint64_t state) {
  const uint64_t MUL = 6364136223846793005ULL, INC = 11634580027462260723ULL;
  for (int i = 0; i < 8; i++) {
    state = state * MUL + INC;
    uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    r->key[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
  }
  r->counter = 0;
  r->idx = 16;
}

uint32_t rng_next_u32(chacha_rng* r) {
  if (r->idx >= 16) {
    chacha12_block(r->key, r->counter++, r->buf);
    r->idx = 0;
  }
  return r->buf[r->idx++];
}
uint64_t rng_next_u64(chacha_rng* r) {
  uint64_t lo = rng_next_u32(r);
  uint64_t hi = rng_next_u32(r);
  return lo | (hi << 32);
}

/* ark-ff 0.5 Fp::rand: 4 u64 limbs, mask top limb with u64::MAX >> 2, reject
 * if >= p.  The limbs ARE the Montgomery representation. */
void fe_rand(const field* F, fe* o, chacha_rng* r) {
  for (;;) {
    for (int i = 0; i < 4; i++) o->l[i] = rng_next_u64(r);
    o->l[3] &= UINT64_MAX >> (256 - F->bits);
    int ge = 1;
    for (int i = 3; i >= 0; i--) {
      if (o->l[i] > F->p[i]) { ge = 1; break; }
      if (o->l[i] < F->p[i]) { ge = 0; break; }
    }
    if (!ge) return;
  }
}

void* oracle_rng_new(uint64_t seed) {
  oracle_init();
  chacha_rng* r = (chacha_rng*)malloc(sizeof(chacha_rng));
  rng_seed_from_u64(r, seed);
  return r;
}
void oracle_rng_free(void* rng) { free(rng); }
uint64_t oracle_rng_next_u64(void* rng) { return rng_next_u64((chacha_rng*)rng); }
void oracle_fr_rand(void* rng, uint64_t out[4]) {
  fe x;
  fe_rand(&FR, &x, (chacha_rng*)rng);
  fe_to_canon(&FR, out, &x);
}
void oracle_fq_rand(void* rng, uint64_t out[4]) {
  fe x;
  fe_rand(&FQ, &x, (chacha_rng*)rng);
  fe_to_canon(&FQ, out, &x);
}
