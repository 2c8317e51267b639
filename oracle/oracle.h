/*
 * oracle.h — CPU restatement of the arkworks 0.5.0 BN254 Groth16 algorithms
 * that Zelana's L2 batch prover calls (reference: core/src/sequencer/settlement/
 * prover.rs:350-425 -> ark_groth16::Groth16::<Bn254>::prove).
 *
 * THIS IS TEST INFRASTRUCTURE, NOT PRODUCT CODE.  Only tests/, the smoke() in
 * __graft_entry__.py and bench.py's cpu_baseline leg may load liboracle.so, and
 * only as the checker / the timed CPU baseline.  The product (libzkmi.so) never
 * links or calls it.
 *
 * Parity pins: the oracle regenerates the
 * reference's own fixtures byte-for-byte from SquareCircuit, seed 42
 * (prover/src/snarkjs.rs:15-31,141-160):
 *   onchain-programs/verifier/vk_snarkjs.json, proof_for_onchain.json,
 *   prover/l2_vk.json bytes 0..224.
 * See tests/test_oracle_fixtures.py.
 *
 * Conventions at this C boundary (same as include/zkmi.h):
 *   field elements   32 B, 4 x u64 little-endian, canonical (NOT Montgomery)
 *   G1 affine        x || y (64 B); the point at infinity is (0, 0)
 *   G2 affine        x.c0 || x.c1 || y.c0 || y.c1 (128 B); infinity is all-zero
 */
#ifndef ZKMI_ORACLE_H
#define ZKMI_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ fields */
typedef struct { uint64_t l[4]; } fe; /* Montgomery form, R = 2^256 */
typedef struct {
  uint64_t p[4];
  uint64_t inv;   /* -p^{-1} mod 2^64 */
  fe one;         /* R mod p */
  fe r2;          /* R^2 mod p */
  unsigned bits;  /* modulus bit size (254) */
} field;

extern field FQ; /* base field of BN254 */
extern field FR; /* scalar field of BN254 */
void oracle_init(void);

void fe_from_canon(const field* F, fe* o, const uint64_t c[4]);
void fe_to_canon(const field* F, uint64_t c[4], const fe* a);
void fe_mul(const field* F, fe* o, const fe* a, const fe* b);
void fe_sqr(const field* F, fe* o, const fe* a);
void fe_add(const field* F, fe* o, const fe* a, const fe* b);
void fe_sub(const field* F, fe* o, const fe* a, const fe* b);
void fe_neg(const field* F, fe* o, const fe* a);
void fe_dbl(const field* F, fe* o, const fe* a);
void fe_pow(const field* F, fe* o, const fe* a, const uint64_t* e, int nlimbs);
void fe_inv(const field* F, fe* o, const fe* a);
int fe_is_zero(const fe* a);
int fe_eq(const fe* a, const fe* b);
void fe_set_u64(const field* F, fe* o, uint64_t v);
int fe_cmp_canon(const field* F, const fe* a, const fe* b); /* compare canonical ints */
int fe_sqrt(const field* F, fe* o, const fe* a);            /* 1 if square (Fq only) */
int fe_legendre_is_square(const field* F, const fe* a);

typedef struct { fe c0, c1; } fe2; /* Fq2 = Fq[u]/(u^2+1) */
void fe2_add(fe2* o, const fe2* a, const fe2* b);
void fe2_sub(fe2* o, const fe2* a, const fe2* b);
void fe2_neg(fe2* o, const fe2* a);
void fe2_dbl(fe2* o, const fe2* a);
void fe2_mul(fe2* o, const fe2* a, const fe2* b);
void fe2_sqr(fe2* o, const fe2* a);
void fe2_inv(fe2* o, const fe2* a);
int fe2_is_zero(const fe2* a);
int fe2_eq(const fe2* a, const fe2* b);
int fe2_cmp(const fe2* a, const fe2* b); /* arkworks Ord: c1 first, then c0 */
int fe2_sqrt(fe2* o, const fe2* a);
void fe2_pow(fe2* o, const fe2* a, const uint64_t* e, int nlimbs);

/* ------------------------------------------------------------------ curves */
typedef struct { fe x, y, z; } g1j;   /* Jacobian; z == 0 is infinity */
typedef struct { fe x, y; int inf; } g1a;
typedef struct { fe2 x, y, z; } g2j;
typedef struct { fe2 x, y; int inf; } g2a;

extern fe2 G2_B; /* 3 / (9 + u) */

void g1_set_inf(g1j* p);
void g1_from_affine(g1j* o, const g1a* a);
void g1_to_affine(g1a* o, const g1j* p);
void g1_dbl(g1j* o, const g1j* p);
void g1_add(g1j* o, const g1j* p, const g1j* q);
void g1_add_mixed(g1j* o, const g1j* p, const g1a* q);
void g1_neg(g1j* o, const g1j* p);
void g1_mul(g1j* o, const g1j* p, const uint64_t k[4]); /* canonical scalar */
int g1_is_on_curve(const g1a* a);
int g1j_eq(const g1j* a, const g1j* b);

void g2_set_inf(g2j* p);
void g2_from_affine(g2j* o, const g2a* a);
void g2_to_affine(g2a* o, const g2j* p);
void g2_dbl(g2j* o, const g2j* p);
void g2_add(g2j* o, const g2j* p, const g2j* q);
void g2_add_mixed(g2j* o, const g2j* p, const g2a* q);
void g2_mul(g2j* o, const g2j* p, const uint64_t* k, int nlimbs);
int g2_is_on_curve(const g2a* a);

/* --------------------------------------------------------------------- rng */
/* rand_chacha 0.3.1 ChaCha12Rng (= rand 0.8 StdRng), rand_core 0.6.4
 * seed_from_u64.  SURVEY.md Appendix A.1 */
typedef struct {
  uint32_t key[8];
  uint64_t counter; /* next block index */
  uint32_t buf[16];
  int idx; /* next word in buf; 16 = empty */
} chacha_rng;
void rng_seed_from_u64(chacha_rng* r, uint64_t seed);
uint32_t rng_next_u32(chacha_rng* r);
uint64_t rng_next_u64(chacha_rng* r);
void fe_rand(const field* F, fe* o, chacha_rng* r);   /* ark-ff Fp::rand */
void g1_rand(g1j* o, chacha_rng* r);                  /* ark-ec Projective::rand */
void g2_rand(g2j* o, chacha_rng* r);

/* ------------------------------------------------------- exported C API */
/* everything below is ctypes-friendly: canonical little-endian bytes */
void* oracle_rng_new(uint64_t seed);
void oracle_rng_free(void* rng);
uint64_t oracle_rng_next_u64(void* rng);
void oracle_fr_rand(void* rng, uint64_t out[4]);
void oracle_fq_rand(void* rng, uint64_t out[4]);
void oracle_g1_rand(void* rng, uint64_t out_affine[8]);
void oracle_g2_rand(void* rng, uint64_t out_affine[16]);

/* field ops on canonical values (for tests) */
void oracle_fr_mul(const uint64_t a[4], const uint64_t b[4], uint64_t o[4]);
void oracle_fq_mul(const uint64_t a[4], const uint64_t b[4], uint64_t o[4]);
void oracle_fr_inv(const uint64_t a[4], uint64_t o[4]);

/* curve ops on canonical affine (tests) */
void oracle_g1_add(const uint64_t a[8], const uint64_t b[8], uint64_t o[8]);
void oracle_g1_mul(const uint64_t p[8], const uint64_t k[4], uint64_t o[8]);
void oracle_g2_mul(const uint64_t p[16], const uint64_t k[4], uint64_t o[16]);
int oracle_g1_on_curve(const uint64_t p[8]);
int oracle_g2_on_curve(const uint64_t p[16]);

/* generate deterministic synthetic MSM inputs:
 * scalars = Fr::rand from seed_from_u64(scalar_seed) (canonical);
 * points P0 = G1::rand, D = G1::rand from seed_from_u64(point_seed),
 * P_{i+1} = P_i + D, batch-normalised to affine. */
void oracle_gen_scalars(uint64_t seed, size_t n, uint64_t* out);
void oracle_gen_points_g1(uint64_t seed, size_t n, uint64_t* out, int nthreads);
void oracle_gen_points_g2(uint64_t seed, size_t n, uint64_t* out, int nthreads);

/* MSM: sum k_i P_i.  Port of ark-ec 0.5 VariableBaseMSM::msm_bigint_wnaf
 * (signed windows, c = ln(n)*69/100 + 2, parallel over windows). */
void oracle_msm_g1(const uint64_t* points, const uint64_t* scalars, size_t n,
                   int nthreads, uint64_t out_affine[8]);
void oracle_msm_g2(const uint64_t* points, const uint64_t* scalars, size_t n,
                   int nthreads, uint64_t out_affine[16]);

/* radix-2 domain over Fr, ark-poly Radix2EvaluationDomain (natural order).
 * dir: 0 = fft, 1 = ifft.  coset: 0 none, 1 = coset with offset GENERATOR (5).
 * data: n canonical Fr values, in place. */
void oracle_ntt(uint64_t* data, uint32_t log_n, int dir, int coset, int nthreads);

/* ---------------------------------------------------------------- groth16 */
/* R1CS in CSR form.  Variables: One = 0, instance i -> i (i < num_instance),
 * witness j -> num_instance + j.  Coefficients canonical Fr. */
typedef struct {
  size_t num_constraints, num_instance, num_witness;
  const uint64_t* a_rowptr; const uint64_t* a_col; const uint64_t* a_val;
  const uint64_t* b_rowptr; const uint64_t* b_col; const uint64_t* b_val;
  const uint64_t* c_rowptr; const uint64_t* c_col; const uint64_t* c_val;
} oracle_r1cs;

/* opaque proving key */
void* oracle_groth16_setup(const oracle_r1cs* cs, void* rng, int nthreads);
void oracle_pk_free(void* pk);
/* sizes: [n_domain, num_instance, num_witness, h_len] */
void oracle_pk_sizes(const void* pk, uint64_t out[4]);
/* serialized arkworks ProvingKey / VerifyingKey (compress = 1/0) */
size_t oracle_pk_serialize(const void* pk, int compress, uint8_t* buf, size_t cap);
size_t oracle_vk_serialize(const void* pk, int compress, uint8_t* buf, size_t cap);
/* z = full assignment (One, instance..., witness...) canonical.
 * r, s taken from rng in arkworks order (r then s) unless rs != NULL. */
int oracle_groth16_prove(const void* pk, const oracle_r1cs* cs, const uint64_t* z,
                         void* rng, const uint64_t* rs /* 8 u64 or NULL */,
                         int nthreads, uint64_t out_a[8], uint64_t out_b[16],
                         uint64_t out_c[8], uint64_t* out_h /* n canon or NULL */);
/* first unsatisfied constraint index, or -1 */
long long oracle_r1cs_check(const oracle_r1cs* cs, const uint64_t* z);
/* witness_map only: h (n canonical values) */
int oracle_witness_map(const oracle_r1cs* cs, const uint64_t* z, uint64_t* h,
                       int nthreads);

/* arkworks point serialization helpers (tests) */
void oracle_g1_serialize(const uint64_t p[8], int compress, uint8_t* out);
void oracle_g2_serialize(const uint64_t p[16], int compress, uint8_t* out);
int oracle_g1_deserialize(const uint8_t* in, int compress, uint64_t out[8]);
int oracle_g2_deserialize(const uint8_t* in, int compress, uint64_t out[16]);

#ifdef __cplusplus
}
#endif
#endif
