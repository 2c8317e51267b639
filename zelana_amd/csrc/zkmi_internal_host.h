// zkmi_internal_host.h — host-only helpers of libzkmi.so (no HIP dependency;
// compiled by g++ in msm_host.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace zk {
// MSM epilogue: terms[k] (k < nbits) = canonical packed XYZZ of weight 2^k;
// terms[nbits + w] (w < W) = window total T_w of weight 2^(c w).  Result is
// canonical affine (all-zero = infinity).
void msm_host_combine_g1(const uint32_t* terms, int nbits, int W, int c, int seg, uint64_t out[8]);
void msm_host_combine_g2(const uint32_t* terms, int nbits, int W, int c, int seg, uint64_t out[16]);
// sharded MSMs: every rank's payload (status block + bit sums) -> the
// combine's term layout (point shards summed, window shards placed) -> Horner
void msm_host_assemble_combine(const uint32_t* src, size_t stride, size_t skip, const int* live, int nl,
                               bool wmode, int g2, int c, int W, int bb, int sb, uint64_t* out);
void host_g1_add_affine(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]);
void host_g2_add_affine(const uint64_t a[16], const uint64_t b[16], uint64_t out[16]);
// arkworks compressed encodings and the Solana 256-byte proof layout
void g1_compress(const uint64_t p[8], uint8_t out[32]);
void g2_compress(const uint64_t p[16], uint8_t out[64]);
void proof_solana(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8], uint8_t out[256]);
// Groth16 proof assembly from the five MSM results (ark-groth16
// create_proof_with_assignment); all points canonical affine, r/s canonical.
// staged Groth16 assembly (msm_host.cpp): host XYZZ points in Montgomery words
struct G16Asm {
  uint64_t rd1[16];     // r delta_1
  uint64_t sd2[32];     // s delta_2
  uint64_t a_aff[8];    // A, affine canonical
  uint64_t c_part[16];  // s A + r B1'
};
void groth16_asm_fixed(const uint64_t delta_g1[8], const uint64_t delta_g2[16], const uint64_t r[4],
                       const uint64_t s[4], G16Asm* st);
size_t groth16_asm_table_words(int g2);
void groth16_asm_tables(const uint64_t delta_g1[8], const uint64_t delta_g2[16], uint64_t* tab1, uint64_t* tab2);
void groth16_asm_fixed_tab(const uint64_t* tab1, const uint64_t* tab2, const uint64_t r[4], const uint64_t s[4],
                           G16Asm* st);
void groth16_asm_ab(const uint64_t alpha_g1[8], const uint64_t beta_g1[8], const uint64_t a0[8],
                    const uint64_t b1_0[8], const uint64_t a_acc[8], const uint64_t b1_acc[8], const uint64_t r[4],
                    const uint64_t s[4], G16Asm* st);
void groth16_asm_b(const uint64_t beta_g2[16], const uint64_t b2_0[16], const uint64_t b2_acc[16], const G16Asm* st,
                   uint64_t b_out[16]);
void groth16_asm_c(const uint64_t l_acc[8], const uint64_t h_acc[8], const G16Asm* st, uint64_t a_out[8],
                   uint64_t c_out[8]);
void groth16_assemble(const uint64_t alpha_g1[8], const uint64_t beta_g1[8], const uint64_t delta_g1[8],
                      const uint64_t beta_g2[16], const uint64_t delta_g2[16], const uint64_t a0[8],
                      const uint64_t b1_0[8], const uint64_t b2_0[16], const uint64_t h_acc[8],
                      const uint64_t l_acc[8], const uint64_t a_acc[8], const uint64_t b1_acc[8],
                      const uint64_t b2_acc[16], const uint64_t r[4], const uint64_t s[4], uint64_t a_out[8],
                      uint64_t b_out[16], uint64_t c_out[8]);
}  // namespace zk
