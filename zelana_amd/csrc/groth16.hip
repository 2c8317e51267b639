// groth16.hip — Groth16 proving over BN254 on gfx950.  Replaces, behind the C
// ABI, what Zelana's Groth16Prover delegates to arkworks 0.5.0:
//   * ProvingKey::deserialize_compressed (core/src/sequencer/settlement/
//     prover.rs:263-267): point decompression + on-curve / subgroup validation
//     run as GPU kernels, queries stay resident in HBM (zkmi_pk_load);
//   * LibsnarkReduction::witness_map_from_matrices: sparse
//     mat-vec + 7 radix-2 transforms + pointwise QAP step, chained DIF/DIT so no
//     bit-reversal pass is ever needed (h comes out bit-reversed and h_query is
//     stored bit-reversed at load time);
//   * create_proof_with_assignment (§8a a4): 4 G1 + 1 G2 MSMs submitted back to
//     back (host epilogue of one overlaps the next's kernels), then the
//     O(1) assembly A = alpha + sum z a + r delta, B = beta + sum z b + s delta,
//     C = s A + r B1 - r s delta + sum_aux z l + sum h h_query on the host.
#include <string.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "dev_io.h"
#include "ec.h"
#include "zkmi_internal.h"

struct zkmi_pk {
  zkmi_ctx* ctx;
  uint64_t n = 0, num_instance = 0, num_witness = 0;
  uint32_t log_n = 0;
  uint64_t alpha_g1[8], beta_g1[8], delta_g1[8];
  uint64_t beta_g2[16], gamma_g2[16], delta_g2[16];
  std::vector<uint64_t> gamma_abc;  // num_instance x 8
  uint64_t a0[8], b1_0[8], b2_0[16];
  zkmi_bases *a_query = nullptr, *b_g1_query = nullptr, *b_g2_query = nullptr, *h_query_rev = nullptr,
             *l_query = nullptr;
  // B queries without their points at infinity (zkmi_pk_precompute): B_i(t) =
  // 0 for every variable no B row reads, half of them in a MiMC circuit.  The
  // prove MSMs run over b_idx's variables only (same sums: an infinity base
  // adds nothing).  The full sets stay for serialization.
  zkmi_bases *b_g1_c = nullptr, *b_g2_c = nullptr;
  uint32_t* d_bidx = nullptr;  // kept variable indices, ascending, in [1, V)
  size_t nb_c = 0;
  std::vector<uint8_t> vk_compressed;
  std::vector<uint64_t> asm_d1, asm_d2;  // host fixed-base tables of delta_1 / delta_2 (msm_host.cpp)
};

namespace zk {

// a key's delta tables for the staged assembly, once its delta_1 / delta_2 are set
static void pk_asm_tables(zkmi_pk* pk) {
  pk->asm_d1.resize(groth16_asm_table_words(0));
  pk->asm_d2.resize(groth16_asm_table_words(1));
  groth16_asm_tables(pk->delta_g1, pk->delta_g2, pk->asm_d1.data(), pk->asm_d2.data());
}

int ntt_raw(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int inv, bool dit);
int ntt_raw_epi(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int inv, bool dit, int epi, const uint32_t* lo,
                const uint32_t* hi);
int ntt_bitrev(zkmi_ctx* ctx, uint32_t* d, uint32_t logn);

// ------------------------------------------------------------ decoding
__constant__ uint32_t FQ_MOD32[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                     0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
__constant__ uint32_t G2B32_C0[8] = {0x24a138e5u, 0x3267e6dcu, 0x59dbefa3u, 0xb5b4c5e5u,
                                     0x1be06ac3u, 0x81be1899u, 0xceb8aaaeu, 0x2b149d40u};
__constant__ uint32_t G2B32_C1[8] = {0x85c315d2u, 0xe4a2bd06u, 0xe52d1852u, 0xa74fa084u,
                                     0xeed8fdf4u, 0xcd2cafadu, 0x3af0fed4u, 0x009713b0u};

__device__ __forceinline__ bool lt_q_words(const uint32_t* w) {
  for (int i = 7; i >= 0; i--) {
    if (w[i] != FQ_MOD32[i]) return w[i] < FQ_MOD32[i];
  }
  return false;
}
// compare two fully reduced values limb-wise: -1, 0, 1
__device__ __forceinline__ int fe_cmp(const Fe& a, const Fe& b) {
  for (int i = NL - 1; i >= 0; i--) {
    if (a.v[i] != b.v[i]) return a.v[i] > b.v[i] ? 1 : -1;
  }
  return 0;
}
__device__ Fe fq_pow64(const Fe& a, const uint64_t e[4]) { return pow<FqP>(a, e); }
__device__ Fe2 f2_pow(const Fe2& a, const uint64_t e[4]) {
  Fe2 r = f2_one();
  for (int i = 255; i >= 0; i--) {
    r = f2_sqr(r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = f2_mul(r, a);
  }
  return r;
}
__device__ bool f2_eq(const Fe2& a, const Fe2& b) { return eq<FqP>(a.c0, b.c0) && eq<FqP>(a.c1, b.c1); }
// canonical (reduced, non-Montgomery) value of a Montgomery element
__device__ Fe canon_q(const Fe& a) { return from_mont<FqP>(a); }

// sqrt in Fq2 for q = 3 mod 4 (Adj & Rodriguez-Henriquez, Alg. 9); which root
// is returned does not matter (the caller picks y or -y by the flag)
__device__ bool f2_sqrt(const Fe2& a, Fe2& out) {
  const uint64_t e34[4] = {0x4f082305b61f3f51ull, 0x65e05aa45a1c72a3ull, 0x6e14116da0605617ull,
                           0x0c19139cb84c680aull};  // (q-3)/4
  const uint64_t e12[4] = {0x9e10460b6c3e7ea3ull, 0xcbc0b548b438e546ull, 0xdc2822db40c0ac2eull,
                           0x183227397098d014ull};  // (q-1)/2
  Fe2 a1 = f2_pow(a, e34);
  Fe2 alpha = f2_mul(a1, f2_mul(a1, a));
  Fe2 conj = {alpha.c0, neg<FqP>(alpha.c1)};
  Fe2 a0 = f2_mul(conj, alpha);
  Fe2 m1 = {neg<FqP>(one<FqP>()), fe_zero()};
  if (f2_eq(a0, m1)) return false;
  Fe2 x0 = f2_mul(a1, a);
  if (f2_eq(alpha, m1)) {
    out = {neg<FqP>(x0.c1), x0.c0};
  } else {
    Fe2 b = {add<FqP>(alpha.c0, one<FqP>()), alpha.c1};
    out = f2_mul(f2_pow(b, e12), x0);
  }
  return f2_eq(f2_sqr(out), a);
}

// raw arkworks encodings (SWFlags in the top two bits of the last byte) ->
// canonical affine words; bad |= 1 on any invalid point
__global__ void __launch_bounds__(256) k_decode_g1(const uint32_t* __restrict__ raw, size_t n, int compressed,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ bad) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int words = compressed ? 8 : 16;
  uint32_t w[16];
  for (int k = 0; k < words; k++) w[k] = raw[i * words + k];
  uint32_t flags = w[words - 1] >> 30;
  w[words - 1] &= 0x3FFFFFFFu;
  uint32_t* o = out + i * 16;
  if (flags & 1) {  // PointAtInfinity (bit 6 of the last byte)
    for (int k = 0; k < 16; k++) o[k] = 0;
    return;
  }
  if (!lt_q_words(w) || (!compressed && !lt_q_words(w + 8))) {
    atomicOr(bad, 1u);
    return;
  }
  Fe x = to_mont<FqP>(unpack(w));
  Fe rhs = add<FqP>(mul<FqP>(sqr<FqP>(x), x), to_mont<FqP>(Fe{{3, 0, 0, 0, 0, 0, 0, 0, 0}}));
  Fe yc;
  if (compressed) {
    const uint64_t e14[4] = {0x4f082305b61f3f52ull, 0x65e05aa45a1c72a3ull, 0x6e14116da0605617ull,
                             0x0c19139cb84c680aull};  // (q+1)/4
    Fe y = fq_pow64(rhs, e14);
    if (!eq<FqP>(sqr<FqP>(y), rhs)) {
      atomicOr(bad, 1u);
      return;
    }
    Fe c = canon_q(y), nc = canon_q(neg<FqP>(y));
    bool larger_is_c = fe_cmp(c, nc) > 0;
    bool want_larger = (flags >> 1) & 1;  // YIsNegative <=> y > -y
    yc = (larger_is_c == want_larger) ? c : nc;
  } else {
    Fe y = to_mont<FqP>(unpack(w + 8));
    if (!eq<FqP>(sqr<FqP>(y), rhs)) {
      atomicOr(bad, 1u);
      return;
    }
    yc = canon_q(y);
  }
  st_fe(o, canon_q(x));
  st_fe(o + 8, yc);
}

__constant__ uint64_t FR_MOD64_G[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                                       0x30644e72e131a029ull};

__global__ void __launch_bounds__(256) k_decode_g2(const uint32_t* __restrict__ raw, size_t n, int compressed,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ bad) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int words = compressed ? 16 : 32;
  uint32_t w[32];
  for (int k = 0; k < words; k++) w[k] = raw[i * words + k];
  uint32_t flags = w[words - 1] >> 30;
  w[words - 1] &= 0x3FFFFFFFu;
  uint32_t* o = out + i * 32;
  if (flags & 1) {
    for (int k = 0; k < 32; k++) o[k] = 0;
    return;
  }
  for (int c = 0; c < words / 8; c++) {
    if (!lt_q_words(w + 8 * c)) {
      atomicOr(bad, 1u);
      return;
    }
  }
  Fe2 x = {to_mont<FqP>(unpack(w)), to_mont<FqP>(unpack(w + 8))};
  Fe2 b = {to_mont<FqP>(ldc_fe(G2B32_C0)), to_mont<FqP>(ldc_fe(G2B32_C1))};
  Fe2 rhs = f2_add(f2_mul(f2_sqr(x), x), b);
  Fe2 y;
  if (compressed) {
    if (!f2_sqrt(rhs, y)) {
      atomicOr(bad, 1u);
      return;
    }
    Fe2 ny = f2_neg(y);
    Fe yc0 = canon_q(y.c0), yc1 = canon_q(y.c1), nc0 = canon_q(ny.c0), nc1 = canon_q(ny.c1);
    int cmp = fe_cmp(yc1, nc1);
    if (cmp == 0) cmp = fe_cmp(yc0, nc0);  // arkworks Fq2 order: c1 first
    bool larger_is_y = cmp > 0;
    bool want_larger = (flags >> 1) & 1;
    if (larger_is_y != want_larger) y = ny;
  } else {
    y = {to_mont<FqP>(unpack(w + 16)), to_mont<FqP>(unpack(w + 24))};
    if (!f2_eq(f2_sqr(y), rhs)) {
      atomicOr(bad, 1u);
      return;
    }
  }
  // prime-order subgroup check: [r] P == O
  Aff<Fq2Ops> P = {x, y};
  Xyzz<Fq2Ops> acc = xyzz_inf<Fq2Ops>();
  for (int bit = 253; bit >= 0; bit--) {
    acc = xyzz_dbl(acc);
    if ((FR_MOD64_G[bit >> 6] >> (bit & 63)) & 1) acc = xyzz_madd(acc, P);
  }
  if (!xyzz_is_inf(acc)) {
    atomicOr(bad, 2u);
    return;
  }
  st_fe(o, canon_q(x.c0));
  st_fe(o + 8, canon_q(x.c1));
  st_fe(o + 16, canon_q(y.c0));
  st_fe(o + 24, canon_q(y.c1));
}

// out[p] = in[rev(p)]  (G1 canonical affine, 16 words), p < cnt
__global__ void __launch_bounds__(256) k_permute_rev(const uint32_t* __restrict__ in, uint32_t logn, size_t cnt,
                                                     uint32_t* __restrict__ out) {
  size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (p >= cnt) return;
  size_t src = logn ? (__brev((uint32_t)p) >> (32 - logn)) : 0;
  for (int k = 0; k < 16; k++) out[p * 16 + k] = in[src * 16 + k];
}

// ------------------------------------------------------------ witness map
// z (canonical) -> Montgomery copy for the mat-vec
__global__ void __launch_bounds__(256) k_to_mont_fr(const uint32_t* __restrict__ z, size_t n, uint32_t* __restrict__ zm) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_fe(zm + i * 8, to_mont<FrP>(ld_fe(z + i * 8)));
}
// rows i < m: out[i] = sum_k val_k * z[col_k]  (val canonical, z Montgomery ->
// canonical product); rows m <= i < m + l of A copy z (inputs appended to A
// only); the rest of the domain is zero.  (evaluate_constraint, §8a a5)
// Rows of at most MATVEC_SHORT terms are summed one lane per row (blocks
// below nsb).  The longer rows (Poseidon rounds' inlined linear combinations,
// 254-term bit recompositions) are listed at upload (upload_r1cs) and summed
// by lane groups in the blocks from nsb on: g lanes per row, g the power of
// two that leaves <= 4 terms per lane for the matrix's longest row, then a
// log2(g)-level shuffle tree; the group's first lane stores the row.  A long
// row then never serialises in one lane (config 1's C mat-vec took 262 us
// with one lane per row), and a matrix of many medium rows (config 1's B:
// 2,040 rows of 9-60 terms) spreads over many waves.
constexpr uint32_t MATVEC_SHORT = 8;
__device__ __forceinline__ Fe fe_shfl_xor(const Fe& a, int m) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = (uint32_t)__shfl_xor((int)a.v[i], m, 64);
  return r;
}
// [0, 16r) with limbs up to 2^32 (a limb-wise sum of <= 8 normalised values
// < 2r) -> [0, 2r), normalised: one carry pass, then the quotient-estimate
// reduction
__device__ __forceinline__ Fe fr_sum_reduce(Fe a) {
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    a.v[i + 1] += a.v[i] >> 29;
    a.v[i] &= LMASK;
  }
  return reduce_q32<FrP>(a);
}
// One term of a row.  DICT (the compact form, upload_r1cs): cv[k] = (column,
// coefficient id) into the matrix's coefficient dictionary (Montgomery form),
// id 0 = 1 (no product), z canonical: coef_M * z * R^-1 = coef * z.  Legacy:
// 32-B canonical coefficients times the Montgomery copy zm of z.
template <bool DICT>
__device__ __forceinline__ Fe mv_term(uint64_t k, const uint64_t* __restrict__ col, const uint32_t* __restrict__ val,
                                      const uint2* __restrict__ cv, const uint32_t* __restrict__ coef,
                                      const uint32_t* __restrict__ zm, const uint32_t* __restrict__ zc) {
  if constexpr (DICT) {
    const uint2 e = cv[k];
    Fe t = ld_fe(zc + (size_t)e.x * 8);
    if (e.y) t = mul<FrP>(ld_fe(coef + (size_t)e.y * 8), t);
    return t;
  } else {
    return mul<FrP>(ld_fe(val + k * 8), ld_fe(zm + col[k] * 8));
  }
}
template <bool DICT, class RP>
__global__ void __launch_bounds__(256) k_matvec(const RP* __restrict__ rowptr, const uint64_t* __restrict__ col,
                                                const uint32_t* __restrict__ val, const uint2* __restrict__ cv,
                                                const uint32_t* __restrict__ coef, const uint32_t* __restrict__ zm,
                                                const uint32_t* __restrict__ zc, size_t m, size_t l, size_t n,
                                                int is_a, const uint32_t* __restrict__ lrow, uint32_t nlong, int g,
                                                uint32_t nsb, uint32_t* __restrict__ out) {
  if (blockIdx.x < nsb) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fe acc = fe_zero();
    if (i < m) {
      const uint64_t k0 = rowptr[i], k1 = rowptr[i + 1];
      if (k1 - k0 > MATVEC_SHORT) return;  // a long row: the group blocks store it
      // limb-wise sum of <= MATVEC_SHORT products < 2r, one reduction (the
      // full modular add per term cost ~70 instructions)
      for (uint64_t k = k0; k < k1; k++) acc = add_lazy(acc, mv_term<DICT>(k, col, val, cv, coef, zm, zc));
      acc = fr_sum_reduce(acc);
    } else if (is_a && i < m + l) {
      acc = ld_fe(zc + (i - m) * 8);
    }
    st_fe(out + i * 8, acc);
    return;
  }
  const uint32_t t = (blockIdx.x - nsb) * blockDim.x + threadIdx.x;
  const uint32_t j = t / (uint32_t)g, gl = t % (uint32_t)g;
  Fe part = fe_zero();
  uint32_t row = 0;
  if (j < nlong) {
    row = lrow[j];
    const uint64_t k1 = rowptr[row + 1];
    for (uint64_t k = rowptr[row] + gl; k < k1; k += (uint32_t)g)
      part = add<FrP>(part, mv_term<DICT>(k, col, val, cv, coef, zm, zc));
  }
  for (int d = g >> 1; d >= 1; d >>= 1) part = add<FrP>(part, fe_shfl_xor(part, d));  // every lane shuffles
  if (j < nlong && gl == 0) st_fe(out + (size_t)row * 8, part);
}
// powers table: tab[x] = c * base^(x * step) for x < cnt (Montgomery), runs of 64
__global__ void __launch_bounds__(256) k_pow_table(uint32_t* __restrict__ tab, uint32_t cnt, const uint32_t* base_c,
                                                   uint64_t step, const uint32_t* mult_m) {
  uint32_t run = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x0 = run * 64;
  if (x0 >= cnt) return;
  Fe b = to_mont<FrP>(ld_fe(base_c));
  Fe bs = one<FrP>();
  {
    Fe bb = b;
    uint64_t e = step;
    while (e) {
      if (e & 1) bs = mul<FrP>(bs, bb);
      bb = sqr<FrP>(bb);
      e >>= 1;
    }
  }
  Fe cur = one<FrP>();
  {
    Fe bb = bs;
    uint64_t e = x0;
    while (e) {
      if (e & 1) cur = mul<FrP>(cur, bb);
      bb = sqr<FrP>(bb);
      e >>= 1;
    }
  }
  if (mult_m) cur = mul<FrP>(cur, ld_fe(mult_m));
  for (uint32_t k = 0; k < 64 && x0 + k < cnt; k++) {
    st_fe(tab + (size_t)(x0 + k) * 8, reduce<FrP>(cur));
    cur = mul<FrP>(cur, bs);
  }
}
// a = (a * b - c) * vinv  (natural order, coset evaluations).  a, b, c are in
// value form (the data never enter Montgomery form), so the Montgomery product
// a*b*R^-1 is brought back with one multiplication by R^2.
__global__ void __launch_bounds__(256) k_qap_combine(uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                     const uint32_t* __restrict__ c, size_t n,
                                                     const uint32_t* __restrict__ vinv_m) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fe ab = mul<FrP>(mul<FrP>(ld_fe(a + i * 8), ld_fe(b + i * 8)), fe_const<FrP>(FrP::R2));
  Fe t = sub<FrP>(ab, ld_fe(c + i * 8));
  st_fe(a + i * 8, mul<FrP>(t, ld_fe(vinv_m)));
}
// scalar constants for a domain: [n^-1 (canon), (g^n - 1)^-1 (Montgomery)]
__global__ void k_domain_consts(uint32_t logn, uint32_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const uint64_t rm2[4] = {0x43e1f593efffffffull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                           0x30644e72e131a029ull};  // r - 2
  Fe two = to_mont<FrP>(Fe{{2, 0, 0, 0, 0, 0, 0, 0, 0}});
  Fe nn = one<FrP>();
  for (uint32_t k = 0; k < logn; k++) nn = mul<FrP>(nn, two);
  Fe ninv = pow<FrP>(nn, rm2);
  st_fe(out, from_mont<FrP>(ninv));
  Fe g = to_mont<FrP>(Fe{{5, 0, 0, 0, 0, 0, 0, 0, 0}});
  Fe gn = g;
  for (uint32_t k = 0; k < logn; k++) gn = sqr<FrP>(gn);
  Fe v = sub<FrP>(gn, one<FrP>());
  st_fe(out + 8, pow<FrP>(v, rm2));
}

static const uint32_t G5[8] = {5, 0, 0, 0, 0, 0, 0, 0};
static const uint32_t GINV5[8] = {0xc6666667u, 0xe7f3fbd4u, 0xca4a2d06u, 0xa9ae5ce9u,
                                  0x33cd568bu, 0x49b9b57cu, 0x5a13d9aau, 0x135b5294u};
// per-log_n constants and coset power tables, cached in the context
int domain_cache(zkmi_ctx* ctx, uint32_t logn, DomainCache* dc) {
  char nm[64];
  snprintf(nm, sizeof(nm), "g16_consts_%u", logn);
  bool fresh = ctx->ws.bufs.find(nm) == ctx->ws.bufs.end();
  ZK_TRY(ctx->ws.get(nm, 96, (void**)&dc->consts));
  dc->ninv_m = dc->consts + 16;
  uint32_t nhi = std::max<uint32_t>(1, (uint32_t)(((1ull << logn) + (1u << COSET_KB) - 1) >> COSET_KB));
  uint32_t nlo = 1u << COSET_KB;
  const char* names[5] = {"lo_g", "hi_g", "lo_gi", "hi_gi", "hi_gf"};
  uint32_t** ptrs[5] = {&dc->lo_g, &dc->hi_g, &dc->lo_gi, &dc->hi_gi, &dc->hi_gf};
  for (int t = 0; t < 5; t++) {
    char tn[64];
    snprintf(tn, sizeof(tn), "g16_%s_%u", names[t], logn);
    ZK_TRY(ctx->ws.get(tn, (size_t)((t & 1) ? nhi : nlo) * 32, (void**)ptrs[t]));
  }
  if (fresh) {
    hipStream_t st = ctx->stream;
    k_domain_consts<<<1, 64, 0, st>>>(logn, dc->consts);
    uint32_t *cg, *cgi;
    ZK_TRY(ctx->ws.get("g16_gconst", 64, (void**)&cg));
    cgi = cg + 8;
    ZK_HIP(hipMemcpyAsync(cg, G5, 32, hipMemcpyHostToDevice, st));
    ZK_HIP(hipMemcpyAsync(cgi, GINV5, 32, hipMemcpyHostToDevice, st));
    // n^-1 as a Montgomery multiplier for the hi tables: convert via a tiny
    // table build with step 0 (tab[x] = n^-1 * base^0) is avoided: fold it in
    // through mult_m = Montgomery(n^-1) computed by k_to_mont_fr.
    uint32_t* ninv_m = dc->ninv_m;
    k_to_mont_fr<<<1, 64, 0, st>>>(dc->consts, 1, ninv_m);
    unsigned glo = (nlo / 64 + 255) / 256, ghi = ((nhi + 63) / 64 + 255) / 256;
    k_pow_table<<<glo, 256, 0, st>>>(dc->lo_g, nlo, cg, 1, nullptr);
    k_pow_table<<<ghi, 256, 0, st>>>(dc->hi_g, nhi, cg, 1ull << COSET_KB, ninv_m);
    k_pow_table<<<glo, 256, 0, st>>>(dc->lo_gi, nlo, cgi, 1, nullptr);
    k_pow_table<<<ghi, 256, 0, st>>>(dc->hi_gi, nhi, cgi, 1ull << COSET_KB, ninv_m);
    k_pow_table<<<ghi, 256, 0, st>>>(dc->hi_gf, nhi, cg, 1ull << COSET_KB, nullptr);
    ZK_HIP(hipGetLastError());
    ZK_HIP(hipStreamSynchronize(st));
  }
  return 0;
}

}  // namespace zk

// R1CS matrices resident in HBM (the circuit shape is fixed per proving key,
// Appendix B.1, so only the witness changes between proofs).
// Compact form (per matrix, when it has few distinct coefficients -- a real
// circuit's are +-1, powers of two and a few constants; zelana_batch has 9):
// u32 row pointers, one (u32 column, u32 coefficient id) pair per non-zero and
// a dictionary of the distinct coefficients in Montgomery form (id 0 = 1):
// 8 B per non-zero instead of 40 (u64 column + 32-B coefficient), and no
// Montgomery copy of z.  Otherwise the legacy CSR (u64 row pointers / columns,
// canonical coefficients).
struct zkmi_r1cs_dev {
  size_t m = 0, l = 0, w = 0;
  uint64_t* rp[3] = {nullptr, nullptr, nullptr};
  uint64_t* col[3] = {nullptr, nullptr, nullptr};
  uint32_t* val[3] = {nullptr, nullptr, nullptr};
  bool dict[3] = {false, false, false};
  uint32_t* rp32[3] = {nullptr, nullptr, nullptr};
  uint2* cv[3] = {nullptr, nullptr, nullptr};
  uint32_t* coef[3] = {nullptr, nullptr, nullptr};  // Montgomery, 8 words per id
  uint32_t ncoef[3] = {0, 0, 0};
  // rows longer than MATVEC_SHORT terms (k_matvec's lane-group blocks)
  uint32_t* lrow[3] = {nullptr, nullptr, nullptr};
  uint32_t nlong[3] = {0, 0, 0};
  int glong[3] = {2, 2, 2};  // lanes per long row
  bool owned = false;
  ~zkmi_r1cs_dev() {
    if (!owned) return;
    for (int t = 0; t < 3; t++) {
      hipFree(rp[t]);
      hipFree(col[t]);
      hipFree(val[t]);
      hipFree(rp32[t]);
      hipFree(cv[t]);
      hipFree(coef[t]);
      if (lrow[t]) hipFree(lrow[t]);
    }
  }
};

namespace zk {
using DevR1CS = zkmi_r1cs_dev;

// a matrix's coefficient dictionary: ids per non-zero (0 = the value 1) and
// the distinct values (canonical 4 x u64); false when there are too many
// distinct values for the compact form to pay (more than 1/4 of the non-zeros
// and more than 2^16), or the matrix is too large for u32 indices
struct CoefKey {
  uint64_t v[4];
  bool operator==(const CoefKey& o) const {
    return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2] && v[3] == o.v[3];
  }
};
struct CoefHash {
  size_t operator()(const CoefKey& k) const {
    uint64_t h = k.v[0] * 0x9E3779B97F4A7C15ull ^ (k.v[1] + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
    h ^= (k.v[2] * 0x165667B19E3779F9ull) ^ (k.v[3] * 0x27D4EB2F165667C5ull);
    return (size_t)(h ^ (h >> 29));
  }
};
static bool build_coef_dict(const uint64_t* vals, uint64_t nnz, size_t nv, std::vector<uint32_t>& ids,
                            std::vector<uint64_t>& dict) {
  if (nnz >= (1ull << 32) || nv >= (1ull << 32)) return false;
  const uint64_t cap = std::max<uint64_t>(1u << 16, nnz / 4);
  std::unordered_map<CoefKey, uint32_t, CoefHash> idx;
  dict.assign({1, 0, 0, 0});
  idx.emplace(CoefKey{{1, 0, 0, 0}}, 0u);
  ids.resize(nnz);
  CoefKey prev{{1, 0, 0, 0}};
  uint32_t prev_id = 0;
  for (uint64_t k = 0; k < nnz; k++) {
    const CoefKey key{{vals[4 * k], vals[4 * k + 1], vals[4 * k + 2], vals[4 * k + 3]}};
    if (key == prev) {  // runs of equal coefficients are common
      ids[k] = prev_id;
      continue;
    }
    auto it = idx.find(key);
    uint32_t id;
    if (it == idx.end()) {
      if (idx.size() >= cap) return false;
      id = (uint32_t)idx.size();
      idx.emplace(key, id);
      dict.insert(dict.end(), key.v, key.v + 4);
    } else {
      id = it->second;
    }
    ids[k] = prev_id = id;
    prev = key;
  }
  return true;
}

// validate + copy a host CSR R1CS to device; owned=true allocates dedicated
// buffers (zkmi_r1cs_create), otherwise context workspace is used
static int upload_r1cs(zkmi_ctx* ctx, const zkmi_r1cs* cs, DevR1CS* d, bool owned = false) {
  d->m = cs->num_constraints;
  d->l = cs->num_instance;
  d->w = cs->num_witness;
  d->owned = owned;
  const uint64_t* rps[3] = {cs->a_rowptr, cs->b_rowptr, cs->c_rowptr};
  const uint64_t* cols[3] = {cs->a_col, cs->b_col, cs->c_col};
  const uint64_t* vals[3] = {cs->a_val, cs->b_val, cs->c_val};
  const char* nm[3] = {"a", "b", "c"};
  size_t m = cs->num_constraints, nv = cs->num_instance + cs->num_witness;
  auto dev_buf = [&](const char* what, int t, size_t bytes, void** out) -> int {
    bytes = std::max<size_t>(bytes, 32);
    if (owned) {
      if (hipMalloc(out, bytes) != hipSuccess) {
        (void)hipGetLastError();
        set_error("r1cs: device allocation failed (matrix %s, %s, %zu bytes)", nm[t], what, bytes);
        return ZKMI_ENOMEM;
      }
      return 0;
    }
    char b[48];
    snprintf(b, sizeof(b), "r1cs_%s_%s", what, nm[t]);
    return ctx->ws.get(b, bytes, out);
  };
  for (int t = 0; t < 3; t++) {
    if (!rps[t] || (m && (!cols[t] || !vals[t]))) {
      set_error("r1cs: matrix %s missing", nm[t]);
      return ZKMI_EINVAL;
    }
    uint64_t nnz = rps[t][m];
    for (size_t i = 0; i < m; i++) {
      if (rps[t][i] > rps[t][i + 1]) {
        set_error("r1cs: matrix %s rowptr not monotone at %zu", nm[t], i);
        return ZKMI_EINVAL;
      }
    }
    for (uint64_t k = 0; k < nnz; k++) {
      if (cols[t][k] >= nv) {
        set_error("r1cs: matrix %s column %llu >= num_variables %zu", nm[t], (unsigned long long)cols[t][k], nv);
        return ZKMI_EINVAL;
      }
    }
    // long-row list for k_matvec (synchronous copy: the list is a temporary)
    std::vector<uint32_t> lr;
    uint64_t lmax = 0;
    for (size_t i = 0; i < m; i++) {
      const uint64_t len = rps[t][i + 1] - rps[t][i];
      if (len > MATVEC_SHORT) {
        lr.push_back((uint32_t)i);
        lmax = std::max(lmax, len);
      }
    }
    d->nlong[t] = (uint32_t)lr.size();
    d->glong[t] = 2;
    while (d->glong[t] < 64 && (uint64_t)d->glong[t] * 4 < lmax) d->glong[t] <<= 1;
    if (!lr.empty()) {
      ZK_TRY(dev_buf("long", t, lr.size() * 4, (void**)&d->lrow[t]));
      ZK_HIP(hipMemcpyAsync(d->lrow[t], lr.data(), lr.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    std::vector<uint32_t> ids;
    std::vector<uint64_t> dict;
    d->dict[t] = build_coef_dict(vals[t], nnz, nv, ids, dict);
    if (d->dict[t]) {
      d->ncoef[t] = (uint32_t)(dict.size() / 4);
      std::vector<uint32_t> rp32(m + 1);
      for (size_t i = 0; i <= m; i++) rp32[i] = (uint32_t)rps[t][i];
      std::vector<uint2> cv(nnz);
      for (uint64_t k = 0; k < nnz; k++) cv[k] = make_uint2((uint32_t)cols[t][k], ids[k]);
      uint32_t* canon = nullptr;
      ZK_TRY(dev_buf("rp32", t, (m + 1) * 4, (void**)&d->rp32[t]));
      ZK_TRY(dev_buf("cv", t, nnz * 8, (void**)&d->cv[t]));
      ZK_TRY(dev_buf("coef", t, dict.size() * 8, (void**)&d->coef[t]));
      ZK_TRY(ctx->ws.get("r1cs_coef_canon", dict.size() * 8, (void**)&canon));
      ZK_HIP(hipMemcpyAsync(d->rp32[t], rp32.data(), (m + 1) * 4, hipMemcpyHostToDevice, ctx->stream));
      if (nnz) ZK_HIP(hipMemcpyAsync(d->cv[t], cv.data(), nnz * 8, hipMemcpyHostToDevice, ctx->stream));
      ZK_HIP(hipMemcpyAsync(canon, dict.data(), dict.size() * 8, hipMemcpyHostToDevice, ctx->stream));
      k_to_mont_fr<<<(d->ncoef[t] + 255) / 256, 256, 0, ctx->stream>>>(canon, d->ncoef[t], d->coef[t]);
      ZK_HIP(hipGetLastError());
      ZK_HIP(hipStreamSynchronize(ctx->stream));  // the host staging vectors go out of scope
    } else {
      ZK_TRY(dev_buf("rp", t, (m + 1) * 8, (void**)&d->rp[t]));
      ZK_TRY(dev_buf("col", t, nnz * 8, (void**)&d->col[t]));
      ZK_TRY(dev_buf("val", t, nnz * 32, (void**)&d->val[t]));
      ZK_HIP(hipMemcpyAsync(d->rp[t], rps[t], (m + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
      if (nnz) {
        ZK_HIP(hipMemcpyAsync(d->col[t], cols[t], nnz * 8, hipMemcpyHostToDevice, ctx->stream));
        ZK_HIP(hipMemcpyAsync(d->val[t], vals[t], nnz * 32, hipMemcpyHostToDevice, ctx->stream));
      }
      ZK_HIP(hipStreamSynchronize(ctx->stream));  // (the long-row list is a temporary)
    }
  }
  return 0;
}

static uint32_t domain_log(size_t need) {
  uint32_t k = 0;
  while (((size_t)1 << k) < need) k++;
  return k;
}

// h (bit-reversed layout, canonical, n elements) into d_h from device z
static int witness_map_dev(zkmi_ctx* ctx, const DevR1CS& dr, const uint32_t* d_z, uint32_t logn, uint32_t* d_h) {
  hipStream_t st = ctx->stream;
  size_t m = dr.m, l = dr.l, nv = l + dr.w;
  size_t n = (size_t)1 << logn;
  DomainCache dc;
  ZK_TRY(domain_cache(ctx, logn, &dc));
  uint32_t *zm, *b, *c;
  zm = nullptr;  // Montgomery copy of z: the legacy CSR form only
  if (!dr.dict[0] || !dr.dict[1] || !dr.dict[2]) ZK_TRY(ctx->ws.get("wm_zm", nv * 32, (void**)&zm));
  ZK_TRY(ctx->ws.get("wm_b", n * 32, (void**)&b));
  ZK_TRY(ctx->ws.get("wm_c", n * 32, (void**)&c));
  uint32_t* a = d_h;
  unsigned gn = (unsigned)((n + 255) / 256);
  {
    ScopedKernelTimer tm(ctx, "g16_matvec");
    // (the legacy form multiplies canonical coefficients by a Montgomery copy
    // of z; the compact form needs none)
    if (!dr.dict[0] || !dr.dict[1] || !dr.dict[2])
      k_to_mont_fr<<<(unsigned)((nv + 255) / 256), 256, 0, st>>>(d_z, nv, zm);
    uint32_t* outs[3] = {a, b, c};
    for (int t = 0; t < 3; t++) {
      const unsigned gl = (unsigned)(((size_t)dr.nlong[t] * dr.glong[t] + 255) / 256);
      if (dr.dict[t])
        k_matvec<true, uint32_t><<<gn + gl, 256, 0, st>>>(dr.rp32[t], nullptr, nullptr, dr.cv[t], dr.coef[t], zm,
                                                          d_z, m, l, n, t == 0, dr.lrow[t], dr.nlong[t],
                                                          dr.glong[t], gn, outs[t]);
      else
        k_matvec<false, uint64_t><<<gn + gl, 256, 0, st>>>(dr.rp[t], dr.col[t], dr.val[t], nullptr, nullptr, zm,
                                                           d_z, m, l, n, t == 0, dr.lrow[t], dr.nlong[t],
                                                           dr.glong[t], gn, outs[t]);
    }
    ZK_HIP(hipGetLastError());
  }
  // evaluations -> coefficients (DIF, bit-reversed) -> * n^-1 g^i -> coset
  // evaluations (DIT, natural)
  uint32_t* vecs[3] = {a, b, c};
  // (the * n^-1 g^i scaling rides on the DIF's innermost pass)
  for (int t = 0; t < 3; t++) {
    ZK_TRY(ntt_raw_epi(ctx, vecs[t], logn, 1, false, 2, dc.lo_g, dc.hi_g));
    ZK_TRY(ntt_raw(ctx, vecs[t], logn, 0, true));
  }
  {
    ScopedKernelTimer tm(ctx, "g16_qap");
    k_qap_combine<<<gn, 256, 0, st>>>(a, b, c, n, dc.consts + 8);
  }
  // coset evaluations -> coefficients: DIF inverse, * n^-1 g^-i, reduce
  ZK_TRY(ntt_raw_epi(ctx, a, logn, 1, false, 2, dc.lo_gi, dc.hi_gi));
  ZK_HIP(hipGetLastError());
  return 0;
}

static int check_cs(const zkmi_r1cs* cs) {
  if (!cs || cs->num_instance < 1) {
    set_error("r1cs: need at least the One variable (num_instance >= 1)");
    return ZKMI_EINVAL;
  }
  return 0;
}

int witness_map_host(zkmi_ctx* ctx, const zkmi_r1cs* cs, const uint64_t* z, uint64_t* h_out) {
  ZK_TRY(check_cs(cs));
  size_t nv = cs->num_instance + cs->num_witness;
  uint32_t logn = domain_log(cs->num_constraints + cs->num_instance);
  if (logn > 28) {
    set_error("witness map: domain 2^%u exceeds Fr two-adicity", logn);
    return ZKMI_EINVAL;
  }
  size_t n = (size_t)1 << logn;
  uint32_t *dz, *dh;
  ZK_TRY(ctx->ws.get("g16_z", nv * 32, (void**)&dz));
  ZK_TRY(ctx->ws.get("g16_h", n * 32, (void**)&dh));
  ZK_HIP(hipMemcpyAsync(dz, z, nv * 32, hipMemcpyHostToDevice, ctx->stream));
  DevR1CS dr;
  ZK_TRY(upload_r1cs(ctx, cs, &dr));
  ZK_TRY(witness_map_dev(ctx, dr, dz, logn, dh));
  ZK_TRY(ntt_bitrev(ctx, dh, logn));  // natural order for the caller
  ZK_HIP(hipMemcpyAsync(h_out, dh, n * 32, hipMemcpyDeviceToHost, ctx->stream));
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  return timer_flush(ctx);
}

// ------------------------------------------------------------ pk load
struct Rd {
  const uint8_t* p;
  size_t len, off = 0;
  bool ok = true;
  const uint8_t* take(size_t k) {
    if (!ok || off + k > len) {
      ok = false;
      return nullptr;
    }
    const uint8_t* r = p + off;
    off += k;
    return r;
  }
  uint64_t u64() {
    const uint8_t* b = take(8);
    if (!b) return 0;
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)b[i] << (8 * i);
    return v;
  }
};

// decode `cnt` raw points (contiguous bytes) on the GPU -> canonical affine in d_out
static int decode_points(zkmi_ctx* ctx, int g2, const uint8_t* raw, size_t cnt, int compressed, uint32_t* d_out) {
  if (!cnt) return 0;
  size_t psz = (g2 ? 64 : 32) * (compressed ? 1 : 2);
  uint32_t *d_raw, *d_bad;
  ZK_TRY(ctx->ws.get("pk_raw", cnt * psz, (void**)&d_raw));
  ZK_TRY(ctx->ws.get("pk_bad", 4, (void**)&d_bad));
  ZK_HIP(hipMemsetAsync(d_bad, 0, 4, ctx->stream));
  ZK_HIP(hipMemcpyAsync(d_raw, raw, cnt * psz, hipMemcpyHostToDevice, ctx->stream));
  unsigned grid = (unsigned)((cnt + 255) / 256);
  {
    ScopedKernelTimer tm(ctx, g2 ? "pk_decode_g2" : "pk_decode_g1");
    if (g2) k_decode_g2<<<grid, 256, 0, ctx->stream>>>(d_raw, cnt, compressed, d_out, d_bad);
    else k_decode_g1<<<grid, 256, 0, ctx->stream>>>(d_raw, cnt, compressed, d_out, d_bad);
    ZK_HIP(hipGetLastError());
  }
  uint32_t bad = 0;
  ZK_HIP(hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, ctx->stream));
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  if (bad) {
    set_error("pk: invalid %s point encoding (%s)", g2 ? "G2" : "G1",
              (bad & 2) ? "not in the prime-order subgroup" : "not on curve / non-canonical");
    return ZKMI_EPOINT;
  }
  return 0;
}
static int decode_to_host(zkmi_ctx* ctx, int g2, const uint8_t* raw, size_t cnt, int compressed, uint64_t* host) {
  if (!cnt) return 0;
  uint32_t* d;
  ZK_TRY(ctx->ws.get("pk_small", cnt * (g2 ? 128 : 64), (void**)&d));
  ZK_TRY(decode_points(ctx, g2, raw, cnt, compressed, d));
  ZK_HIP(hipMemcpy(host, d, cnt * (g2 ? 128 : 64), hipMemcpyDeviceToHost));
  return 0;
}
static int decode_to_bases(zkmi_ctx* ctx, int g2, const uint8_t* raw, size_t cnt, int compressed, zkmi_bases** out,
                           uint32_t permute_logn = 0, size_t keep = (size_t)-1) {
  uint32_t* d;
  size_t pw = g2 ? 32 : 16;
  ZK_TRY(ctx->ws.get("pk_canon", std::max<size_t>(1, cnt) * pw * 4, (void**)&d));
  ZK_TRY(decode_points(ctx, g2, raw, cnt, compressed, d));
  if (permute_logn) {
    uint32_t* d2;
    ZK_TRY(ctx->ws.get("pk_perm", std::max<size_t>(1, keep) * pw * 4, (void**)&d2));
    // positions p < keep take h_query[rev(p)] (rev(p) < cnt for p < keep)
    k_permute_rev<<<(unsigned)((keep + 255) / 256), 256, 0, ctx->stream>>>(d, permute_logn, keep, d2);
    ZK_HIP(hipGetLastError());
    return bases_from_device_canon(ctx, g2, d2, keep, out);
  }
  return bases_from_device_canon(ctx, g2, d, cnt, out);
}

int pk_load(zkmi_ctx* ctx, const uint8_t* bytes, size_t len, int compressed, zkmi_pk** out) {
  *out = nullptr;
  const size_t s1 = compressed ? 32 : 64, s2 = compressed ? 64 : 128;
  Rd r{bytes, len};
  const uint8_t* alpha = r.take(s1);
  const uint8_t* g2s = r.take(3 * s2);  // beta, gamma, delta (G2)
  uint64_t nabc = r.u64();
  if (!r.ok || nabc == 0 || nabc > (1ull << 32)) {
    set_error("pk: truncated verifying key");
    return ZKMI_EINVAL;
  }
  const uint8_t* abc = r.take(nabc * s1);
  size_t vk_end = r.off;
  const uint8_t* bd1 = r.take(2 * s1);  // beta_g1, delta_g1
  uint64_t na = r.u64();
  const uint8_t* aq = r.ok ? r.take(na * s1) : nullptr;
  uint64_t nb1 = r.u64();
  const uint8_t* b1q = r.ok ? r.take(nb1 * s1) : nullptr;
  uint64_t nb2 = r.u64();
  const uint8_t* b2q = r.ok ? r.take(nb2 * s2) : nullptr;
  uint64_t nh = r.u64();
  const uint8_t* hq = r.ok ? r.take(nh * s1) : nullptr;
  uint64_t nl = r.u64();
  const uint8_t* lq = r.ok ? r.take(nl * s1) : nullptr;
  if (!r.ok || r.off != len) {
    set_error("pk: malformed ProvingKey encoding (parsed %zu of %zu bytes)", r.off, len);
    return ZKMI_EINVAL;
  }
  uint64_t n = nh + 1;
  if (na != nb1 || na != nb2 || na < nabc || nl != na - nabc || (n & (n - 1)) != 0) {
    set_error("pk: inconsistent query lengths (a %llu b1 %llu b2 %llu h %llu l %llu ic %llu)",
              (unsigned long long)na, (unsigned long long)nb1, (unsigned long long)nb2, (unsigned long long)nh,
              (unsigned long long)nl, (unsigned long long)nabc);
    return ZKMI_EINVAL;
  }
  zkmi_pk* pk = new zkmi_pk;
  pk->ctx = ctx;
  pk->n = n;
  pk->log_n = domain_log(n);
  pk->num_instance = nabc;
  pk->num_witness = nl;
  int rc = 0;
  auto fail = [&](int code) {
    zkmi_pk_destroy(pk);
    return code;
  };
  uint64_t small1[3 * 8];
  std::vector<uint8_t> s1buf(3 * s1);
  memcpy(s1buf.data(), alpha, s1);
  memcpy(s1buf.data() + s1, bd1, 2 * s1);
  if ((rc = decode_to_host(ctx, 0, s1buf.data(), 3, compressed, small1))) return fail(rc);
  memcpy(pk->alpha_g1, small1, 64);
  memcpy(pk->beta_g1, small1 + 8, 64);
  memcpy(pk->delta_g1, small1 + 16, 64);
  uint64_t small2[3 * 16];
  if ((rc = decode_to_host(ctx, 1, g2s, 3, compressed, small2))) return fail(rc);
  memcpy(pk->beta_g2, small2, 128);
  memcpy(pk->gamma_g2, small2 + 16, 128);
  memcpy(pk->delta_g2, small2 + 32, 128);
  pk->gamma_abc.resize(nabc * 8);
  if ((rc = decode_to_host(ctx, 0, abc, nabc, compressed, pk->gamma_abc.data()))) return fail(rc);
  if ((rc = decode_to_bases(ctx, 0, aq, na, compressed, &pk->a_query))) return fail(rc);
  if ((rc = decode_to_bases(ctx, 0, b1q, nb1, compressed, &pk->b_g1_query))) return fail(rc);
  if ((rc = decode_to_bases(ctx, 1, b2q, nb2, compressed, &pk->b_g2_query))) return fail(rc);
  if ((rc = decode_to_bases(ctx, 0, hq, nh, compressed, &pk->h_query_rev, pk->log_n, nh))) return fail(rc);
  if ((rc = decode_to_bases(ctx, 0, lq, nl, compressed, &pk->l_query))) return fail(rc);
  // query[0] terms added outside the MSMs (calculate_coeff)
  std::vector<uint64_t> tmp1(na * 8), tmp2(na * 16);
  if ((rc = bases_export(pk->a_query, tmp1.data()))) return fail(rc);
  memcpy(pk->a0, tmp1.data(), 64);
  if ((rc = bases_export(pk->b_g1_query, tmp1.data()))) return fail(rc);
  memcpy(pk->b1_0, tmp1.data(), 64);
  if ((rc = bases_export(pk->b_g2_query, tmp2.data()))) return fail(rc);
  memcpy(pk->b2_0, tmp2.data(), 128);
  // compressed VK bytes (Groth16Prover::compute_vk_hash hashes these)
  if (compressed) {
    pk->vk_compressed.assign(bytes, bytes + vk_end);
  } else {
    std::vector<uint8_t> v(32 + 3 * 64 + 8 + nabc * 32);
    g1_compress(pk->alpha_g1, v.data());
    g2_compress(pk->beta_g2, v.data() + 32);
    g2_compress(pk->gamma_g2, v.data() + 96);
    g2_compress(pk->delta_g2, v.data() + 160);
    for (int i = 0; i < 8; i++) v[224 + i] = (uint8_t)(nabc >> (8 * i));
    for (uint64_t i = 0; i < nabc; i++) g1_compress(&pk->gamma_abc[i * 8], v.data() + 232 + i * 32);
    pk->vk_compressed = v;
  }
  ZK_TRY(timer_flush(ctx));
  pk_asm_tables(pk);
  *out = pk;
  return 0;
}

// ------------------------------------------------------------ B-query compaction
__global__ void __launch_bounds__(256) k_gather_scalars(const uint32_t* __restrict__ z, const uint32_t* __restrict__ idx,
                                                        size_t n, uint32_t* __restrict__ out) {
  size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const uint4* s = reinterpret_cast<const uint4*>(z + (size_t)idx[k] * 8);
  uint4* d = reinterpret_cast<uint4*>(out + k * 8);
  d[0] = s[0];
  d[1] = s[1];
}
template <int PW>  // words per point
__global__ void __launch_bounds__(256) k_gather_points(const uint32_t* __restrict__ pts,
                                                       const uint32_t* __restrict__ idx, size_t n,
                                                       uint32_t* __restrict__ out) {
  size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const uint4* s = reinterpret_cast<const uint4*>(pts + (size_t)idx[k] * PW);
  uint4* d = reinterpret_cast<uint4*>(out + k * PW);
#pragma unroll
  for (int i = 0; i < PW / 4; i++) d[i] = s[i];
}
// live[i] = 1 unless both B bases of variable i are at infinity (bit 31 of a
// point's last word)
__global__ void __launch_bounds__(256) k_b_live(const uint32_t* __restrict__ b1, const uint32_t* __restrict__ b2,
                                                size_t n, uint8_t* __restrict__ live) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  live[i] = !((b1[i * 16 + 15] >> 31) & (b2[i * 32 + 31] >> 31));
}

static int gather_bases(zkmi_ctx* ctx, const zkmi_bases* src, const uint32_t* d_idx, size_t n, zkmi_bases** out) {
  const int pw = src->g2 ? 32 : 16;
  uint32_t* d_pts = nullptr;
  if (hipMalloc(&d_pts, std::max<size_t>(1, n) * pw * 4) != hipSuccess) {
    (void)hipGetLastError();
    set_error("hipMalloc(%zu) failed for compacted bases", n * pw * 4);
    return ZKMI_ENOMEM;
  }
  unsigned grid = (unsigned)((n + 255) / 256);
  if (src->g2) k_gather_points<32><<<grid, 256, 0, ctx->stream>>>(src->d_pts, d_idx, n, d_pts);
  else k_gather_points<16><<<grid, 256, 0, ctx->stream>>>(src->d_pts, d_idx, n, d_pts);
  if (hipGetLastError() != hipSuccess) {
    hipFree(d_pts);
    set_error("gather_bases: launch failed");
    return ZKMI_EHIP;
  }
  zkmi_bases* b = new zkmi_bases;
  b->ctx = ctx;
  b->g2 = src->g2;
  b->n = n;
  b->d_pts = d_pts;
  *out = b;
  return 0;
}

// Drop the B variables whose bases are both at infinity when that removes at
// least 1/8 of them (a no-op for dense keys).  One-time, at precompute.
int pk_compact_b(zkmi_pk* pk) {
  zkmi_ctx* ctx = pk->ctx;
  const size_t nv = pk->num_instance + pk->num_witness;
  if (nv < 2 || pk->b_g1_query->n < nv || pk->b_g2_query->n < nv) return 0;
  const size_t m = nv - 1;  // variables 1..V-1 (the One term is added outside the MSM)
  uint8_t* d_live;
  ZK_TRY(ctx->ws.get("g16_blive", m, (void**)&d_live));
  k_b_live<<<(unsigned)((m + 255) / 256), 256, 0, ctx->stream>>>(pk->b_g1_query->d_pts + 16, pk->b_g2_query->d_pts + 32,
                                                                 m, d_live);
  ZK_HIP(hipGetLastError());
  std::vector<uint8_t> live(m);
  ZK_HIP(hipMemcpyAsync(live.data(), d_live, m, hipMemcpyDeviceToHost, ctx->stream));
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  std::vector<uint32_t> idx;
  idx.reserve(m);
  for (size_t i = 0; i < m; i++)
    if (live[i]) idx.push_back((uint32_t)(i + 1));
  if (idx.empty() || idx.size() > m - m / 8) return 0;
  uint32_t* d_idx = nullptr;
  if (hipMalloc(&d_idx, idx.size() * 4) != hipSuccess) {
    (void)hipGetLastError();
    set_error("hipMalloc failed for the B index list");
    return ZKMI_ENOMEM;
  }
  int rc = hipMemcpy(d_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice) == hipSuccess ? 0 : ZKMI_EHIP;
  zkmi_bases *b1 = nullptr, *b2 = nullptr;
  if (!rc) rc = gather_bases(ctx, pk->b_g1_query, d_idx, idx.size(), &b1);
  if (!rc) rc = gather_bases(ctx, pk->b_g2_query, d_idx, idx.size(), &b2);
  if (!rc) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : ZKMI_EHIP;
  if (rc) {
    zkmi_bases_destroy(b1);
    zkmi_bases_destroy(b2);
    hipFree(d_idx);
    return rc;
  }
  pk->b_g1_c = b1;
  pk->b_g2_c = b2;
  pk->d_bidx = d_idx;
  pk->nb_c = idx.size();
  return 0;
}

}  // namespace zk

// A proof in flight: its five MSM jobs are queued; wait finishes their host
// epilogues and assembles A, B, C (ark-groth16 create_proof_with_assignment).
struct zkmi_proof_job {
  const zkmi_pk* pk;
  zkmi_msm_job* jobs[5];  // h, l, a, b_g1, b_g2
  uint64_t r[4], s[4];
  zk::G16Asm asm_st;  // the staged assembly (msm_host.cpp)
};

namespace zk {

// ------------------------------------------------------------ prove
// Small proofs (configs[0]: a 2^13 domain) are latency-bound: every kernel
// of an MSM is a short dependent chain, and enqueueing the ~130 launches of
// a proof costs the host about a millisecond.  So the order favours the
// critical paths: the witness map (feeding the h MSM) is queued first on the
// context stream, then l on lane 1, the B MSMs (the G2 one is the longest
// chain) on lane 0 of their own, then a and h on lane 1; all z-weighted MSMs
// fork from one event recorded before the witness map, so they run beside it.
// (A hipGraph capture of the whole small proof -- one replay launch instead
// of ~140 -- measured 3.36 ms against 3.12 ms enqueued as streams: the
// replayed DAG loses more lane overlap than the launches cost; dropped.
// Round 5: b_g2 accumulated on the other lane from a copy of the shared sort
// -- lane 0 b_g1, l, a; lane 1 b_g2, h -- measured 1.88-1.98 ms against
// 1.74-1.83 for this order; with three lanes the third lane's stream shared a
// hardware queue (GPU_MAX_HW_QUEUES = 4 with the context stream), 2.05 ms.)
constexpr size_t SMALL_PROOF_MAX = (size_t)1 << 16;  // domains up to which the small schedule applies
static int prove_submit_small(zkmi_ctx* ctx, const zkmi_pk* pk, const DevR1CS& dr, const uint32_t* dz,
                              uint32_t logn, uint32_t* dh, zkmi_msm_job** jobs) {
  const size_t l = dr.l, w = dr.w, nv = l + w, n = pk->n;
  const int nl = std::max(1, ctx->msm_lanes);
  if (!ctx->prove_fork) ZK_HIP(hipEventCreateWithFlags(&ctx->prove_fork, hipEventDisableTiming));
  uint32_t* zb = nullptr;
  if (pk->d_bidx) {
    ZK_TRY(ctx->ws.get("g16_zb", pk->nb_c * 32, (void**)&zb));
    k_gather_scalars<<<(unsigned)((pk->nb_c + 255) / 256), 256, 0, ctx->stream>>>(dz, pk->d_bidx, pk->nb_c, zb);
    ZK_HIP(hipGetLastError());
  }
  ZK_HIP(hipEventRecord(ctx->prove_fork, ctx->stream));
  ZK_TRY(witness_map_dev(ctx, dr, dz, logn, dh));
  ctx->msm_fork = ctx->prove_fork;
  int rc = 0;
  // l first (lane 1 starts while the host still queues the long B chain)
  ctx->lane_next = 1 % nl;
  rc = msm_submit(ctx, pk->l_query, 0, dz + l * 8, w, &jobs[1]);
  ctx->lane_next = 0;
  if (pk->d_bidx) {
    const zkmi_bases* bq[2] = {pk->b_g1_c, pk->b_g2_c};
    if (!rc) rc = msm_submit_shared(ctx, bq, 2, 0, zb, pk->nb_c, &jobs[3]);
    ctx->lane_next = (nl >= 3 ? 2 : 1) % nl;
    if (!rc) rc = msm_submit(ctx, pk->a_query, 1, dz + 8, nv - 1, &jobs[2]);
  } else {
    const zkmi_bases* abq[3] = {pk->a_query, pk->b_g1_query, pk->b_g2_query};
    if (!rc) rc = msm_submit_shared(ctx, abq, 3, 1, dz + 8, nv - 1, &jobs[2]);
  }
  ctx->msm_fork = nullptr;  // h forks after the witness map
  ctx->lane_next = 1 % nl;
  if (!rc) rc = msm_submit(ctx, pk->h_query_rev, 0, dh, n - 1, &jobs[0]);
  return rc;
}

// core: R1CS and full assignment z already resident in HBM.  submit queues
// everything (the witness map on the context stream, the MSMs on the lanes)
// and returns; several proofs may be in flight, finished in order by wait.
int groth16_prove_submit(zkmi_ctx* ctx, const zkmi_pk* pk, const DevR1CS& dr, const uint32_t* dz,
                         const uint64_t r[4], const uint64_t s[4], zkmi_proof_job** out) {
  *out = nullptr;
  size_t l = dr.l, w = dr.w, nv = l + w;
  uint32_t logn = domain_log(dr.m + l);
  if (l != pk->num_instance || w != pk->num_witness || ((size_t)1 << logn) != pk->n) {
    set_error("prove: circuit shape (m %zu, l %zu, w %zu) does not match the proving key (n %llu, l %llu, w %llu)",
              dr.m, l, w, (unsigned long long)pk->n, (unsigned long long)pk->num_instance,
              (unsigned long long)pk->num_witness);
    return ZKMI_EINVAL;
  }
  size_t n = pk->n;
  uint32_t* dh;
  ZK_TRY(ctx->ws.get("g16_h", n * 32, (void**)&dh));
  // The MSMs over z (l, and a / b_g1 / b_g2, which share the scalars z[1..V]
  // and so one digits + sort pass) do not need h: they are queued on the MSM
  // lanes first, the witness map then runs on the context stream beside them
  // (filling their latency-bound sort / bucket-reduction phases), and the h
  // MSM follows it.  Each host epilogue overlaps later kernels.
  zkmi_proof_job* pj = new zkmi_proof_job;
  pj->pk = pk;
  memcpy(pj->r, r, 32);
  memcpy(pj->s, s, 32);
  zkmi_msm_job** jobs = pj->jobs;
  for (int i = 0; i < 5; i++) jobs[i] = nullptr;
  int rc = 0;
// 1: large-proof schedule below (measured, 2^22 L2 proofs 34.7-34.8 ->
// 36.1-36.2/s, two in flight 35.5-35.9 -> 37.2-37.3/s; zelana_batch 81.3-81.6
// -> 84.8-85.0/s).  0: the round-5 order (all MSMs, then the witness map).
#ifndef ZK_G2_AFTER_WM
#define ZK_G2_AFTER_WM 1
#endif
  if (n <= SMALL_PROOF_MAX) {
    rc = prove_submit_small(ctx, pk, dr, dz, logn, dh, jobs);
  } else if (ZK_G2_AFTER_WM && pk->d_bidx) {
    // The witness map's NTTs are the path to the h MSM.  Beside the G2
    // accumulation (248 VGPRs, 2 waves per SIMD) no NTT wave fits on a SIMD;
    // beside the G1 ones (3 waves, LDS-capped) one does.  So the witness map is
    // queued first, the z-weighted MSMs fork from before it, and the G2
    // accumulation (b_g2, sharing b_g1's sort) waits for its end; the h MSM
    // then runs beside the G2 accumulation.
    if (!ctx->prove_fork) ZK_HIP(hipEventCreateWithFlags(&ctx->prove_fork, hipEventDisableTiming));
    if (!ctx->wm_done) ZK_HIP(hipEventCreateWithFlags(&ctx->wm_done, hipEventDisableTiming));
    uint32_t* zb;
    rc = ctx->ws.get("g16_zb", pk->nb_c * 32, (void**)&zb);
    if (!rc) {
      k_gather_scalars<<<(unsigned)((pk->nb_c + 255) / 256), 256, 0, ctx->stream>>>(dz, pk->d_bidx, pk->nb_c, zb);
      rc = hipGetLastError() == hipSuccess ? 0 : ZKMI_EHIP;
    }
    if (!rc) rc = hipEventRecord(ctx->prove_fork, ctx->stream) == hipSuccess ? 0 : ZKMI_EHIP;
    if (!rc) rc = witness_map_dev(ctx, dr, dz, logn, dh);
    if (!rc) rc = hipEventRecord(ctx->wm_done, ctx->stream) == hipSuccess ? 0 : ZKMI_EHIP;
    ctx->msm_fork = ctx->prove_fork;
    if (!rc) rc = msm_submit(ctx, pk->l_query, 0, dz + l * 8, w, &jobs[1]);
    if (!rc) rc = msm_submit(ctx, pk->a_query, 1, dz + 8, nv - 1, &jobs[2]);
    ctx->acc_gate = ctx->wm_done;
    ctx->acc_gate_set = pk->b_g2_c;
    const zkmi_bases* bq[2] = {pk->b_g1_c, pk->b_g2_c};
    if (!rc) rc = msm_submit_shared(ctx, bq, 2, 0, zb, pk->nb_c, &jobs[3]);
    ctx->acc_gate = nullptr;
    ctx->acc_gate_set = nullptr;
    ctx->msm_fork = nullptr;  // h forks after the witness map
    if (!rc) rc = msm_submit(ctx, pk->h_query_rev, 0, dh, n - 1, &jobs[0]);
  } else {
  rc = msm_submit(ctx, pk->l_query, 0, dz + l * 8, w, &jobs[1]);
  if (!rc && pk->d_bidx) {  // a over z[1..V]; b1 / b2 over the compacted B variables
    uint32_t* zb;
    rc = ctx->ws.get("g16_zb", pk->nb_c * 32, (void**)&zb);
    if (!rc) {
      k_gather_scalars<<<(unsigned)((pk->nb_c + 255) / 256), 256, 0, ctx->stream>>>(dz, pk->d_bidx, pk->nb_c, zb);
      rc = hipGetLastError() == hipSuccess ? 0 : ZKMI_EHIP;
    }
    if (!rc) rc = msm_submit(ctx, pk->a_query, 1, dz + 8, nv - 1, &jobs[2]);
    const zkmi_bases* bq[2] = {pk->b_g1_c, pk->b_g2_c};
    if (!rc) rc = msm_submit_shared(ctx, bq, 2, 0, zb, pk->nb_c, &jobs[3]);
  } else if (!rc) {
    const zkmi_bases* abq[3] = {pk->a_query, pk->b_g1_query, pk->b_g2_query};
    rc = msm_submit_shared(ctx, abq, 3, 1, dz + 8, nv - 1, &jobs[2]);
  }
  if (!rc) rc = witness_map_dev(ctx, dr, dz, logn, dh);
  if (!rc) rc = msm_submit(ctx, pk->h_query_rev, 0, dh, n - 1, &jobs[0]);
  }
  if (rc) {
    for (auto* j : pj->jobs)
      if (j) msm_job_free(j);
    delete pj;
    return rc;
  }
  // the key-only part of the assembly (r delta_1, s delta_2) while the GPU works
  groth16_asm_fixed_tab(pk->asm_d1.data(), pk->asm_d2.data(), pj->r, pj->s, &pj->asm_st);
  *out = pj;
  return 0;
}

int groth16_prove_wait(zkmi_proof_job* pj, uint64_t a_out[8], uint64_t b_out[16], uint64_t c_out[8]) {
  const zkmi_pk* pk = pj->pk;
  zkmi_msm_job** jobs = pj->jobs;
  uint64_t h_acc[8], l_acc[8], a_acc[8], b1_acc[8], b2_acc[16];
  uint64_t b_tmp[16];
  int rc = 0;
  // each assembly stage runs as soon as its MSMs are in, beside the GPU's
  // remaining work (the h MSM, after the witness map, ends last)
  if (!rc) rc = msm_wait(jobs[1], l_acc), jobs[1] = nullptr;
  if (!rc) rc = msm_wait(jobs[2], a_acc), jobs[2] = nullptr;
  if (!rc) rc = msm_wait(jobs[3], b1_acc), jobs[3] = nullptr;
  if (!rc) groth16_asm_ab(pk->alpha_g1, pk->beta_g1, pk->a0, pk->b1_0, a_acc, b1_acc, pj->r, pj->s, &pj->asm_st);
  if (!rc) rc = msm_wait(jobs[4], b2_acc), jobs[4] = nullptr;
  if (!rc) groth16_asm_b(pk->beta_g2, pk->b2_0, b2_acc, &pj->asm_st, b_tmp);
  if (!rc) rc = msm_wait(jobs[0], h_acc), jobs[0] = nullptr;
  for (int i = 0; i < 5; i++)
    if (jobs[i]) msm_job_free(jobs[i]);
  if (!rc) {
    groth16_asm_c(l_acc, h_acc, &pj->asm_st, a_out, c_out);
    memcpy(b_out, b_tmp, sizeof(b_tmp));
  }
  delete pj;
  return rc;
}

int groth16_prove_resident(zkmi_ctx* ctx, const zkmi_pk* pk, const DevR1CS& dr, const uint32_t* dz,
                           const uint64_t r[4], const uint64_t s[4], uint64_t a_out[8], uint64_t b_out[16],
                           uint64_t c_out[8]) {
  zkmi_proof_job* pj = nullptr;
  ZK_TRY(groth16_prove_submit(ctx, pk, dr, dz, r, s, &pj));
  return groth16_prove_wait(pj, a_out, b_out, c_out);
}

int groth16_prove(zkmi_ctx* ctx, const zkmi_pk* pk, const zkmi_r1cs* cs, const uint64_t* z, const uint64_t r[4],
                  const uint64_t s[4], uint64_t a_out[8], uint64_t b_out[16], uint64_t c_out[8]) {
  ZK_TRY(check_cs(cs));
  size_t nv = cs->num_instance + cs->num_witness;
  uint32_t* dz;
  ZK_TRY(ctx->ws.get("g16_z", nv * 32, (void**)&dz));
  ZK_HIP(hipMemcpyAsync(dz, z, nv * 32, hipMemcpyHostToDevice, ctx->stream));
  DevR1CS dr;
  ZK_TRY(upload_r1cs(ctx, cs, &dr));
  return groth16_prove_resident(ctx, pk, dr, dz, r, s, a_out, b_out, c_out);
}

// ------------------------------------------------------------ synthetic pk
// Random proving key of a given shape, generated in HBM (benchmarks only:
// the proof it yields does not verify, the work is identical).
int pk_synthetic(zkmi_ctx* ctx, uint64_t seed, uint32_t log_n, size_t l, size_t w, zkmi_pk** out) {
  *out = nullptr;
  size_t n = (size_t)1 << log_n, nv = l + w;
  if (l < 1 || log_n > 28) {
    set_error("pk_synthetic: bad shape");
    return ZKMI_EINVAL;
  }
  zkmi_pk* pk = new zkmi_pk;
  pk->ctx = ctx;
  pk->n = n;
  pk->log_n = log_n;
  pk->num_instance = l;
  pk->num_witness = w;
  int rc = 0;
  auto fail = [&](int code) {
    zkmi_pk_destroy(pk);
    return code;
  };
  if ((rc = bases_generate(ctx, 0, seed + 1, nv, &pk->a_query))) return fail(rc);
  if ((rc = bases_generate(ctx, 0, seed + 2, nv, &pk->b_g1_query))) return fail(rc);
  if ((rc = bases_generate(ctx, 1, seed + 3, nv, &pk->b_g2_query))) return fail(rc);
  if ((rc = bases_generate(ctx, 0, seed + 4, n - 1, &pk->h_query_rev))) return fail(rc);
  if ((rc = bases_generate(ctx, 0, seed + 5, w, &pk->l_query))) return fail(rc);
  zkmi_bases* small1;
  zkmi_bases* small2;
  if ((rc = bases_generate(ctx, 0, seed + 6, 3 + l, &small1))) return fail(rc);
  if ((rc = bases_generate(ctx, 1, seed + 7, 3, &small2))) return fail(rc);
  std::vector<uint64_t> s1((3 + l) * 8), s2(3 * 16), t1(nv * 8), t2(nv * 16);
  rc = bases_export(small1, s1.data());
  if (!rc) rc = bases_export(small2, s2.data());
  zkmi_bases_destroy(small1);
  zkmi_bases_destroy(small2);
  if (rc) return fail(rc);
  memcpy(pk->alpha_g1, &s1[0], 64);
  memcpy(pk->beta_g1, &s1[8], 64);
  memcpy(pk->delta_g1, &s1[16], 64);
  pk->gamma_abc.assign(s1.begin() + 24, s1.end());
  memcpy(pk->beta_g2, &s2[0], 128);
  memcpy(pk->gamma_g2, &s2[16], 128);
  memcpy(pk->delta_g2, &s2[32], 128);
  if ((rc = bases_export(pk->a_query, t1.data()))) return fail(rc);
  memcpy(pk->a0, t1.data(), 64);
  if ((rc = bases_export(pk->b_g1_query, t1.data()))) return fail(rc);
  memcpy(pk->b1_0, t1.data(), 64);
  if ((rc = bases_export(pk->b_g2_query, t2.data()))) return fail(rc);
  memcpy(pk->b2_0, t2.data(), 128);
  pk_asm_tables(pk);
  *out = pk;
  return 0;
}

// ------------------------------------------------------------ setup
// Groth16::circuit_specific_setup (keygen.rs:87-91) = ark-groth16 0.5
// generate_parameters_with_qap with LibsnarkReduction::instance_map_with_
// evaluation: Lagrange values u_i = L_i(t) over the radix-2 domain, column
// sums a_j(t) = sum_i A[i][j] u_i (+ u_{m+j} for the instance rows of A),
// then every query point is a scalar multiple of the G1 / G2 generator
// (fixed_base_mul).  Field results are exact, group results are exact, so the
// key equals arkworks' for the same toxic waste and generators.
__constant__ uint32_t SETUP_W28[8] = {0x725b19f0u, 0x9bd61b6eu, 0x41112ed4u, 0x402d111eu,
                                      0x8ef62abcu, 0x00e0a7ebu, 0xa58a7e85u, 0x2a3c09f0u};
__constant__ uint64_t SETUP_RM2[4] = {0x43e1f593efffffffull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                                      0x30644e72e131a029ull};  // r - 2
enum { SC_ALPHA, SC_BETA, SC_GINV, SC_DINV, SC_T, SC_OMEGA, SC_ZTN, SC_ZTD, SC_COUNT };
// tw: alpha, beta, gamma, delta, t (canonical); out: Montgomery constants
__global__ void k_setup_consts(const uint32_t* __restrict__ tw, uint32_t logn, uint32_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const uint64_t rm2[4] = {SETUP_RM2[0], SETUP_RM2[1], SETUP_RM2[2], SETUP_RM2[3]};
  Fe a = to_mont<FrP>(ld_fe(tw)), b = to_mont<FrP>(ld_fe(tw + 8)), g = to_mont<FrP>(ld_fe(tw + 16)),
     d = to_mont<FrP>(ld_fe(tw + 24)), t = to_mont<FrP>(ld_fe(tw + 32));
  Fe w = to_mont<FrP>(ldc_fe(SETUP_W28));
  for (uint32_t k = logn; k < 28; k++) w = sqr<FrP>(w);
  Fe tn = t;
  for (uint32_t k = 0; k < logn; k++) tn = sqr<FrP>(tn);
  Fe zt = sub<FrP>(tn, one<FrP>());  // vanishing polynomial at t
  Fe nn = one<FrP>();
  for (uint32_t k = 0; k < logn; k++) nn = add<FrP>(nn, nn);
  Fe di = pow<FrP>(d, rm2);
  const Fe vals[SC_COUNT] = {a, b, pow<FrP>(g, rm2), di, t, w, mul<FrP>(zt, pow<FrP>(nn, rm2)), mul<FrP>(zt, di)};
  for (int k = 0; k < SC_COUNT; k++) st_fe(out + 8 * k, reduce<FrP>(vals[k]));
}
// u_i = L_i(t) = Z(t) omega^i / (n (t - omega^i)), Montgomery (evaluate_all_lagrange_coefficients)
__global__ void __launch_bounds__(256) k_setup_lagrange(const uint32_t* __restrict__ sc, size_t n,
                                                        uint32_t* __restrict__ u) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t rm2[4] = {SETUP_RM2[0], SETUP_RM2[1], SETUP_RM2[2], SETUP_RM2[3]};
  const uint64_t e[4] = {(uint64_t)i, 0, 0, 0};
  const Fe w = pow<FrP>(ld_fe(sc + 8 * SC_OMEGA), e);
  const Fe inv = pow<FrP>(sub<FrP>(ld_fe(sc + 8 * SC_T), w), rm2);
  st_fe(u + i * 8, reduce<FrP>(mul<FrP>(mul<FrP>(ld_fe(sc + 8 * SC_ZTN), w), inv)));
}
// column sums over a CSC matrix: out_j = sum_k val_k u_{row_k} (+ u_{m+j} for
// j < l in A), canonical value form.  Columns are cut into segments of at most
// SETUP_SEG entries (one thread each) so that a dense column (the One
// variable: every row of a constant-heavy circuit) does not serialise the
// launch; a second pass adds each column's segment partials.
#define SETUP_SEG 256
__global__ void __launch_bounds__(256) k_setup_segs(const uint64_t* __restrict__ segk, size_t nseg,
                                                    const uint32_t* __restrict__ row, const uint32_t* __restrict__ val,
                                                    const uint32_t* __restrict__ u, uint32_t* __restrict__ part) {
  const size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  Fe acc = fe_zero();
  for (uint64_t k = segk[s]; k < segk[s + 1]; k++) acc = add<FrP>(acc, mul<FrP>(ld_fe(val + k * 8), ld_fe(u + (size_t)row[k] * 8)));
  st_fe(part + s * 8, acc);  // [0, 2p): fits 256 bits
}
__global__ void __launch_bounds__(256) k_setup_cols(const uint64_t* __restrict__ colseg,
                                                    const uint32_t* __restrict__ part, const uint32_t* __restrict__ u,
                                                    size_t m, size_t l, size_t nv, int is_a, uint32_t* __restrict__ out) {
  const size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (j >= nv) return;
  Fe acc = fe_zero();
  for (uint64_t s = colseg[j]; s < colseg[j + 1]; s++) acc = add<FrP>(acc, ld_fe(part + s * 8));
  if (is_a && j < l) acc = add<FrP>(acc, mul<FrP>(ld_fe(u + (m + j) * 8), Fe{{1, 0, 0, 0, 0, 0, 0, 0, 0}}));
  st_fe(out + j * 8, reduce<FrP>(acc));
}
// gamma_abc (j < l): (beta a_j + alpha b_j + c_j) / gamma; l_query (j >= l): the same / delta
__global__ void __launch_bounds__(256) k_setup_lscalars(const uint32_t* __restrict__ va, const uint32_t* __restrict__ vb,
                                                        const uint32_t* __restrict__ vc, const uint32_t* __restrict__ sc,
                                                        size_t l, size_t nv, uint32_t* __restrict__ abc,
                                                        uint32_t* __restrict__ lq) {
  const size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (j >= nv) return;
  Fe k = add<FrP>(add<FrP>(mul<FrP>(ld_fe(va + j * 8), ld_fe(sc + 8 * SC_BETA)),
                           mul<FrP>(ld_fe(vb + j * 8), ld_fe(sc + 8 * SC_ALPHA))),
                  ld_fe(vc + j * 8));
  Fe v = reduce<FrP>(mul<FrP>(k, ld_fe(sc + 8 * (j < l ? SC_GINV : SC_DINV))));
  if (j < l) st_fe(abc + j * 8, v);
  else st_fe(lq + (j - l) * 8, v);
}
// h_query scalars Z(t) t^i / delta (h_query_scalars), stored at position p with
// i = rev(p): the resident key keeps h bit-reversed (see decode_to_bases)
__global__ void __launch_bounds__(256) k_setup_h(const uint32_t* __restrict__ sc, uint32_t logn, size_t cnt,
                                                 uint32_t* __restrict__ out) {
  const size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (p >= cnt) return;
  const uint64_t e[4] = {logn ? (uint64_t)(__brev((uint32_t)p) >> (32 - logn)) : 0, 0, 0, 0};
  st_fe(out + p * 8, from_mont<FrP>(mul<FrP>(pow<FrP>(ld_fe(sc + 8 * SC_T), e), ld_fe(sc + 8 * SC_ZTD))));
}

// host CSR -> CSC (column pointers u64, row indices u32, 32-B coefficients)
static void csr_to_csc(const uint64_t* rp, const uint64_t* col, const uint64_t* val, size_t m, size_t nv,
                       std::vector<uint64_t>& cp, std::vector<uint32_t>& rows, std::vector<uint64_t>& vals) {
  const uint64_t nnz = rp[m];
  cp.assign(nv + 1, 0);
  for (uint64_t k = 0; k < nnz; k++) cp[col[k] + 1]++;
  for (size_t j = 0; j < nv; j++) cp[j + 1] += cp[j];
  std::vector<uint64_t> cur(cp.begin(), cp.end() - 1);
  rows.resize(std::max<uint64_t>(1, nnz));
  vals.resize(std::max<uint64_t>(1, nnz) * 4);
  for (size_t i = 0; i < m; i++)
    for (uint64_t k = rp[i]; k < rp[i + 1]; k++) {
      const uint64_t d = cur[col[k]]++;
      rows[d] = (uint32_t)i;
      memcpy(&vals[d * 4], &val[k * 4], 32);
    }
}

int groth16_setup(zkmi_ctx* ctx, const zkmi_r1cs* cs, const uint64_t tw[20], const uint64_t g1[8],
                  const uint64_t g2[16], zkmi_pk** out) {
  *out = nullptr;
  ZK_TRY(check_cs(cs));
  const size_t m = cs->num_constraints, l = cs->num_instance, w = cs->num_witness, nv = l + w;
  const uint32_t logn = domain_log(m + l);
  if (logn > 28 || m >= (1ull << 32)) {
    set_error("setup: domain 2^%u exceeds Fr two-adicity", logn);
    return ZKMI_EINVAL;
  }
  const size_t n = (size_t)1 << logn;
  hipStream_t st = ctx->stream;
  DevR1CS chk;
  ZK_TRY(upload_r1cs(ctx, cs, &chk));  // validation only (shapes, column range)
  uint32_t *d_tw, *d_sc, *u, *va, *vb, *vc, *abc, *lsc, *hs, *small, *pts;
  ZK_TRY(ctx->ws.get("setup_tw", 5 * 32, (void**)&d_tw));
  ZK_TRY(ctx->ws.get("setup_consts", SC_COUNT * 32, (void**)&d_sc));
  ZK_TRY(ctx->ws.get("setup_u", n * 32, (void**)&u));
  ZK_TRY(ctx->ws.get("setup_va", nv * 32, (void**)&va));
  ZK_TRY(ctx->ws.get("setup_vb", nv * 32, (void**)&vb));
  ZK_TRY(ctx->ws.get("setup_vc", nv * 32, (void**)&vc));
  ZK_TRY(ctx->ws.get("setup_abc", l * 32 + 3 * 32, (void**)&abc));
  ZK_TRY(ctx->ws.get("setup_l", std::max<size_t>(1, w) * 32, (void**)&lsc));
  ZK_TRY(ctx->ws.get("setup_h", n * 32, (void**)&hs));
  ZK_TRY(ctx->ws.get("setup_small", (l + 6) * 32, (void**)&small));
  ZK_TRY(ctx->ws.get("setup_pts", std::max(nv, n) * 128, (void**)&pts));
  ZK_HIP(hipMemcpyAsync(d_tw, tw, 5 * 32, hipMemcpyHostToDevice, st));
  k_setup_consts<<<1, 64, 0, st>>>(d_tw, logn, d_sc);
  k_setup_lagrange<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d_sc, n, u);
  const uint64_t* rps[3] = {cs->a_rowptr, cs->b_rowptr, cs->c_rowptr};
  const uint64_t* cols[3] = {cs->a_col, cs->b_col, cs->c_col};
  const uint64_t* vals[3] = {cs->a_val, cs->b_val, cs->c_val};
  uint32_t* outs[3] = {va, vb, vc};
  for (int t = 0; t < 3; t++) {
    std::vector<uint64_t> cp, cv;
    std::vector<uint32_t> rows;
    csr_to_csc(rps[t], cols[t], vals[t], m, nv, cp, rows, cv);
    // segments: column j owns [colseg[j], colseg[j + 1]), segment s covers
    // entries [segk[s], segk[s + 1])
    std::vector<uint64_t> colseg(nv + 1), segk;
    segk.reserve(cp[nv] / SETUP_SEG + nv + 1);
    for (size_t j = 0; j < nv; j++) {
      colseg[j] = segk.size();
      for (uint64_t k = cp[j]; k < cp[j + 1]; k += SETUP_SEG) segk.push_back(k);
    }
    colseg[nv] = segk.size();
    const size_t nseg = segk.size();
    segk.push_back(cp[nv]);
    uint64_t *d_colseg, *d_segk;
    uint32_t *d_rows, *d_val, *d_part;
    ZK_TRY(ctx->ws.get("setup_colseg", colseg.size() * 8, (void**)&d_colseg));
    ZK_TRY(ctx->ws.get("setup_segk", segk.size() * 8, (void**)&d_segk));
    ZK_TRY(ctx->ws.get("setup_part", std::max<size_t>(1, nseg) * 32, (void**)&d_part));
    ZK_TRY(ctx->ws.get("setup_rows", rows.size() * 4, (void**)&d_rows));
    ZK_TRY(ctx->ws.get("setup_cval", cv.size() * 8, (void**)&d_val));
    ZK_HIP(hipMemcpyAsync(d_colseg, colseg.data(), colseg.size() * 8, hipMemcpyHostToDevice, st));
    ZK_HIP(hipMemcpyAsync(d_segk, segk.data(), segk.size() * 8, hipMemcpyHostToDevice, st));
    ZK_HIP(hipMemcpyAsync(d_rows, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, st));
    ZK_HIP(hipMemcpyAsync(d_val, cv.data(), cv.size() * 8, hipMemcpyHostToDevice, st));
    if (nseg) k_setup_segs<<<(unsigned)((nseg + 255) / 256), 256, 0, st>>>(d_segk, nseg, d_rows, d_val, u, d_part);
    k_setup_cols<<<(unsigned)((nv + 255) / 256), 256, 0, st>>>(d_colseg, d_part, u, m, l, nv, t == 0, outs[t]);
    ZK_HIP(hipStreamSynchronize(st));  // host vectors die with this iteration
  }
  k_setup_lscalars<<<(unsigned)((nv + 255) / 256), 256, 0, st>>>(va, vb, vc, d_sc, l, nv, abc + 3 * 8, lsc);
  k_setup_h<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d_sc, logn, n - 1, hs);
  ZK_HIP(hipGetLastError());
  // small G1 batch [alpha, beta, delta, gamma_abc...], G2 batch [beta, gamma, delta]
  ZK_HIP(hipMemcpyAsync(abc, tw, 64, hipMemcpyHostToDevice, st));
  ZK_HIP(hipMemcpyAsync(abc + 16, tw + 12, 32, hipMemcpyHostToDevice, st));
  ZK_HIP(hipMemcpyAsync(small, tw + 4, 96, hipMemcpyHostToDevice, st));
  zkmi_pk* pk = new zkmi_pk;
  pk->ctx = ctx;
  pk->n = n;
  pk->log_n = logn;
  pk->num_instance = l;
  pk->num_witness = w;
  int rc = 0;
  auto fail = [&](int code) {
    zkmi_pk_destroy(pk);
    return code;
  };
  std::vector<uint64_t> s1((3 + l) * 8), s2(3 * 16);
  if ((rc = fixed_base_mul(ctx, 0, g1, abc, 3 + l, pts))) return fail(rc);
  if (hipMemcpy(s1.data(), pts, s1.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return fail(ZKMI_EHIP);
  if ((rc = fixed_base_mul(ctx, 1, g2, small, 3, pts))) return fail(rc);
  if (hipMemcpy(s2.data(), pts, s2.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return fail(ZKMI_EHIP);
  memcpy(pk->alpha_g1, &s1[0], 64);
  memcpy(pk->beta_g1, &s1[8], 64);
  memcpy(pk->delta_g1, &s1[16], 64);
  pk->gamma_abc.assign(s1.begin() + 24, s1.end());
  memcpy(pk->beta_g2, &s2[0], 128);
  memcpy(pk->gamma_g2, &s2[16], 128);
  memcpy(pk->delta_g2, &s2[32], 128);
  struct Q {
    int g2;
    const uint32_t* sc;
    size_t cnt;
    zkmi_bases** dst;
    uint64_t* first;
  } qs[5] = {{0, va, nv, &pk->a_query, pk->a0},
             {0, vb, nv, &pk->b_g1_query, pk->b1_0},
             {1, vb, nv, &pk->b_g2_query, pk->b2_0},
             {0, hs, n - 1, &pk->h_query_rev, nullptr},
             {0, lsc, w, &pk->l_query, nullptr}};
  for (const Q& q : qs) {
    if ((rc = fixed_base_mul(ctx, q.g2, q.g2 ? g2 : g1, q.sc, q.cnt, pts))) return fail(rc);
    if (q.first && hipMemcpy(q.first, pts, q.g2 ? 128 : 64, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(ZKMI_EHIP);
    if ((rc = bases_from_device_canon(ctx, q.g2, pts, q.cnt, q.dst))) return fail(rc);
  }
  std::vector<uint8_t> v(32 + 3 * 64 + 8 + l * 32);
  g1_compress(pk->alpha_g1, v.data());
  g2_compress(pk->beta_g2, v.data() + 32);
  g2_compress(pk->gamma_g2, v.data() + 96);
  g2_compress(pk->delta_g2, v.data() + 160);
  for (int i = 0; i < 8; i++) v[224 + i] = (uint8_t)((uint64_t)l >> (8 * i));
  for (size_t i = 0; i < l; i++) g1_compress(&pk->gamma_abc[i * 8], v.data() + 232 + i * 32);
  pk->vk_compressed = v;
  if ((rc = timer_flush(ctx))) return fail(rc);
  pk_asm_tables(pk);
  *out = pk;
  return 0;
}

// VerifyingKey::deserialize_compressed (validated: on curve, G2 in the
// subgroup; prover.rs:266-267) re-serialized: compute_vk_hash (:289-294)
// hashes exactly these bytes.
int vk_canonical(zkmi_ctx* ctx, const uint8_t* bytes, size_t len, uint8_t* out, size_t cap, size_t* out_len) {
  Rd r{bytes, len};
  const uint8_t* alpha = r.take(32);
  const uint8_t* g2s = r.take(3 * 64);
  const uint64_t nabc = r.u64();
  if (!r.ok || nabc == 0 || nabc > (1u << 24)) {
    set_error("Failed to deserialize verifying key: truncated");
    return ZKMI_EINVAL;
  }
  const uint8_t* abc = r.take(nabc * 32);
  if (!r.ok || r.off != len) {
    set_error("Failed to deserialize verifying key: %zu trailing / missing bytes", len - r.off);
    return ZKMI_EINVAL;
  }
  std::vector<uint64_t> a1(8), g2(3 * 16), ic(nabc * 8);
  ZK_TRY(decode_to_host(ctx, 0, alpha, 1, 1, a1.data()));
  ZK_TRY(decode_to_host(ctx, 1, g2s, 3, 1, g2.data()));
  ZK_TRY(decode_to_host(ctx, 0, abc, nabc, 1, ic.data()));
  *out_len = len;
  if (!out) return 0;
  if (cap < len) {
    set_error("vk_canonical: buffer too small");
    return ZKMI_EINVAL;
  }
  g1_compress(a1.data(), out);
  for (int i = 0; i < 3; i++) g2_compress(&g2[16 * i], out + 32 + 64 * i);
  for (int i = 0; i < 8; i++) out[224 + i] = (uint8_t)(nabc >> (8 * i));
  for (uint64_t i = 0; i < nabc; i++) g1_compress(&ic[8 * i], out + 232 + 32 * i);
  return 0;
}

// ProvingKey::serialize_compressed (keygen.rs:103): vk | beta_g1 | delta_g1 |
// a | b_g1 | b_g2 | h | l, each query a u64 length then points
int pk_serialize(const zkmi_pk* pk, uint8_t* buf, size_t cap, size_t* len) {
  const size_t nv = pk->num_instance + pk->num_witness, nh = pk->n - 1, nl = pk->num_witness;
  const size_t total = pk->vk_compressed.size() + 64 + (8 + 32 * nv) * 2 + (8 + 64 * nv) + (8 + 32 * nh) + (8 + 32 * nl);
  *len = total;
  if (!buf) return 0;
  if (cap < total) {
    set_error("pk_serialize: buffer of %zu bytes, need %zu", cap, total);
    return ZKMI_EINVAL;
  }
  uint8_t* o = buf;
  memcpy(o, pk->vk_compressed.data(), pk->vk_compressed.size());
  o += pk->vk_compressed.size();
  g1_compress(pk->beta_g1, o);
  g1_compress(pk->delta_g1, o + 32);
  o += 64;
  auto put_len = [&](uint64_t k) {
    for (int i = 0; i < 8; i++) o[i] = (uint8_t)(k >> (8 * i));
    o += 8;
  };
  auto put_query = [&](const zkmi_bases* b, size_t cnt, bool rev) -> int {
    const int pw = b->g2 ? 16 : 8;
    std::vector<uint64_t> pts(std::max<size_t>(1, b->n) * pw);
    ZK_TRY(bases_export(b, pts.data()));
    put_len(cnt);
    for (size_t i = 0; i < cnt; i++) {
      size_t src = i;
      if (rev) src = pk->log_n ? (__builtin_bitreverse32((uint32_t)i) >> (32 - pk->log_n)) : 0;
      if (b->g2) g2_compress(&pts[src * pw], o), o += 64;
      else g1_compress(&pts[src * pw], o), o += 32;
    }
    return 0;
  };
  ZK_TRY(put_query(pk->a_query, nv, false));
  ZK_TRY(put_query(pk->b_g1_query, nv, false));
  ZK_TRY(put_query(pk->b_g2_query, nv, false));
  ZK_TRY(put_query(pk->h_query_rev, nh, true));
  ZK_TRY(put_query(pk->l_query, nl, false));
  return 0;
}

}  // namespace zk

using namespace zk;

extern "C" {
int zkmi_witness_map(zkmi_ctx* ctx, const zkmi_r1cs* cs, const uint64_t* z, uint64_t* h_out) {
  ZK_DEVICE_GUARD(ctx);
  return witness_map_host(ctx, cs, z, h_out);
}
int zkmi_pk_load(zkmi_ctx* ctx, const uint8_t* bytes, size_t len, int compressed, zkmi_pk** out) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !bytes || !out) {
    set_error("zkmi_pk_load: null argument");
    return ZKMI_EINVAL;
  }
  return pk_load(ctx, bytes, len, compressed, out);
}
void zkmi_pk_destroy(zkmi_pk* pk) {
  ZK_DEVICE_GUARD((pk ? pk->ctx : nullptr));
  if (!pk) return;
  zkmi_bases_destroy(pk->a_query);
  zkmi_bases_destroy(pk->b_g1_query);
  zkmi_bases_destroy(pk->b_g2_query);
  zkmi_bases_destroy(pk->b_g1_c);
  zkmi_bases_destroy(pk->b_g2_c);
  if (pk->d_bidx) hipFree(pk->d_bidx);
  zkmi_bases_destroy(pk->h_query_rev);
  zkmi_bases_destroy(pk->l_query);
  delete pk;
}
int zkmi_pk_info(const zkmi_pk* pk, uint64_t out[3]) {
  out[0] = pk->n;
  out[1] = pk->num_instance;
  out[2] = pk->num_witness;
  return 0;
}
int zkmi_pk_precompute(zkmi_pk* pk, int factor) {
  ZK_DEVICE_GUARD((pk ? pk->ctx : nullptr));
  if (!pk) {
    zk::set_error("zkmi_pk_precompute: null key");
    return ZKMI_EINVAL;
  }
  if (!pk->d_bidx && !pk->b_g1_query->tc) {
    int rc = zk::pk_compact_b(pk);
    if (rc) return rc;
  }
  const bool compact = pk->d_bidx != nullptr;
  zkmi_bases* qs[5] = {pk->h_query_rev, pk->l_query, pk->a_query, compact ? pk->b_g1_c : pk->b_g1_query,
                       compact ? pk->b_g2_c : pk->b_g2_query};
  for (zkmi_bases* b : qs) {
    if (!b || b->tc) continue;
    int rc = zk::bases_precompute(b, zk::table_window(b->n, b->g2), factor);
    if (rc) return rc;
  }
  return 0;
}
int zkmi_pk_b_terms(const zkmi_pk* pk, uint64_t* out) {
  if (!pk || !out) {
    zk::set_error("zkmi_pk_b_terms: null argument");
    return ZKMI_EINVAL;
  }
  *out = pk->d_bidx ? pk->nb_c : pk->num_instance + pk->num_witness - 1;
  return 0;
}
int zkmi_pk_vk_bytes(const zkmi_pk* pk, uint8_t* buf, size_t cap, size_t* len) {
  *len = pk->vk_compressed.size();
  if (buf && cap >= *len) memcpy(buf, pk->vk_compressed.data(), *len);
  return 0;
}
int zkmi_r1cs_create(zkmi_ctx* ctx, const zkmi_r1cs* cs, zkmi_r1cs_dev** out) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !cs || !out) {
    set_error("zkmi_r1cs_create: null argument");
    return ZKMI_EINVAL;
  }
  ZK_TRY(check_cs(cs));
  zkmi_r1cs_dev* d = new zkmi_r1cs_dev;
  int rc = upload_r1cs(ctx, cs, d, true);
  if (rc == 0) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : ZKMI_EHIP;
  if (rc) {
    delete d;
    return rc;
  }
  *out = d;
  return 0;
}
void zkmi_r1cs_destroy(zkmi_r1cs_dev* d) {
  delete d;
}
int zkmi_groth16_prove_resident(zkmi_ctx* ctx, const zkmi_pk* pk, const zkmi_r1cs_dev* cs, const void* d_z,
                                const uint64_t r[4], const uint64_t s[4], uint64_t a_out[8], uint64_t b_out[16],
                                uint64_t c_out[8]) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !pk || !cs || !d_z || !r || !s) {
    set_error("zkmi_groth16_prove_resident: null argument");
    return ZKMI_EINVAL;
  }
  int rc = groth16_prove_resident(ctx, pk, *cs, (const uint32_t*)d_z, r, s, a_out, b_out, c_out);
  if (rc == 0) rc = timer_flush(ctx);
  return rc;
}
int zkmi_groth16_prove_submit(zkmi_ctx* ctx, const zkmi_pk* pk, const zkmi_r1cs_dev* cs, const void* d_z,
                              const uint64_t r[4], const uint64_t s[4], zkmi_proof_job** job) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !pk || !cs || !d_z || !r || !s || !job) {
    set_error("zkmi_groth16_prove_submit: null argument");
    return ZKMI_EINVAL;
  }
  return groth16_prove_submit(ctx, pk, *cs, (const uint32_t*)d_z, r, s, job);
}
int zkmi_groth16_prove_wait(zkmi_proof_job* job, uint64_t a_out[8], uint64_t b_out[16], uint64_t c_out[8]) {
  if (!job || !a_out || !b_out || !c_out) {
    set_error("zkmi_groth16_prove_wait: null argument");
    return ZKMI_EINVAL;
  }
  zkmi_ctx* ctx = job->pk->ctx;
  ZK_DEVICE_GUARD(ctx);
  int rc = groth16_prove_wait(job, a_out, b_out, c_out);
  if (rc == 0) rc = timer_flush(ctx, false);
  return rc;
}
int zkmi_pk_synthetic(zkmi_ctx* ctx, uint64_t seed, uint32_t log_n, size_t num_instance, size_t num_witness,
                      zkmi_pk** out) {
  ZK_DEVICE_GUARD(ctx);
  return pk_synthetic(ctx, seed, log_n, num_instance, num_witness, out);
}
int zkmi_groth16_prove(zkmi_ctx* ctx, const zkmi_pk* pk, const zkmi_r1cs* cs, const uint64_t* z, const uint64_t r[4],
                       const uint64_t s[4], uint64_t a_out[8], uint64_t b_out[16], uint64_t c_out[8]) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !pk || !cs || !z || !r || !s) {
    set_error("zkmi_groth16_prove: null argument");
    return ZKMI_EINVAL;
  }
  int rc = groth16_prove(ctx, pk, cs, z, r, s, a_out, b_out, c_out);
  if (rc == 0) rc = timer_flush(ctx);
  return rc;
}
int zkmi_groth16_setup(zkmi_ctx* ctx, const zkmi_r1cs* cs, const uint64_t toxic[20], const uint64_t g1[8],
                       const uint64_t g2[16], zkmi_pk** out) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !cs || !toxic || !g1 || !g2 || !out) {
    set_error("zkmi_groth16_setup: null argument");
    return ZKMI_EINVAL;
  }
  return groth16_setup(ctx, cs, toxic, g1, g2, out);
}
int zkmi_vk_canonical(zkmi_ctx* ctx, const uint8_t* bytes, size_t len, uint8_t* out, size_t cap, size_t* out_len) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !bytes || !out_len) {
    set_error("zkmi_vk_canonical: null argument");
    return ZKMI_EINVAL;
  }
  return vk_canonical(ctx, bytes, len, out, cap, out_len);
}
int zkmi_pk_serialize(const zkmi_pk* pk, uint8_t* buf, size_t cap, size_t* len) {
  ZK_DEVICE_GUARD((pk ? pk->ctx : nullptr));
  if (!pk || !len) {
    set_error("zkmi_pk_serialize: null argument");
    return ZKMI_EINVAL;
  }
  return pk_serialize(pk, buf, cap, len);
}
}  // extern "C"
