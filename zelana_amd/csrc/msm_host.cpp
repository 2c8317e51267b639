// msm_host.cpp — host epilogue of the GPU MSM and host-side point encodings.
//
// The GPU hands over ~c*W + W canonical XYZZ bit sums; the remaining work is a
// single strictly sequential Horner chain (~255 doublings) that a CPU core
// finishes in ~30-60 us while one GPU lane would need ~1 ms (one XYZZ doubling
// is ~2k dependent VALU ops).  Also: affine conversion, the arkworks SWFlags
// point encodings and the 256-B Solana proof layout of
// core/src/sequencer/settlement/prover.rs:304-334.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "host_field.h"
#include "zkmi_internal_host.h"

using namespace zkh;

namespace {

template <class F>
using HX = zk::Xyzz<F>;

F4 ld_canon32(const uint32_t* w) {
  uint64_t c[4];
  for (int i = 0; i < 4; i++) c[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return from_canon(c);
}
template <class F>
typename F::T ld_coord(const uint32_t* w);
template <>
F4 ld_coord<HFq>(const uint32_t* w) {
  return ld_canon32(w);
}
template <>
F42 ld_coord<HFq2>(const uint32_t* w) {
  return {ld_canon32(w), ld_canon32(w + 8)};
}
template <class F, int CW>
HX<F> ld_term(const uint32_t* p) {
  HX<F> r;
  r.x = ld_coord<F>(p);
  r.y = ld_coord<F>(p + CW);
  r.zz = ld_coord<F>(p + 2 * CW);
  r.zzz = ld_coord<F>(p + 3 * CW);
  return r;
}

F4 inv1(const F4& a) { return finv(a); }
F42 inv1(const F42& a) { return HFq2::inv(a); }
void put(uint64_t* o, const F4& a) { to_canon(o, a); }
void put(uint64_t* o, const F42& a) {
  to_canon(o, a.c0);
  to_canon(o + 4, a.c1);
}

template <class F, int CW>
void to_affine(const HX<F>& p, uint64_t* out) {
  const int K = CW / 8 * 4;  // u64 per coordinate
  if (zk::xyzz_is_inf(p)) {
    memset(out, 0, 2 * K * 8);
    return;
  }
  // x = X / ZZ, y = Y / ZZZ
  typename F::T izz = inv1(p.zz), izzz = inv1(p.zzz);
  put(out, F::mul(p.x, izz));
  put(out + K, F::mul(p.y, izzz));
}

// term k = sum of its `seg` segments (the GPU cuts long bit sums)
template <class F, int CW>
HX<F> ld_term_seg(const uint32_t* terms, size_t k, int seg) {
  constexpr int XW = 4 * CW;
  HX<F> t = ld_term<F, CW>(terms + k * seg * XW);
  for (int s = 1; s < seg; s++) t = zk::xyzz_add(t, ld_term<F, CW>(terms + (k * seg + s) * XW));
  return t;
}
template <class F, int CW>
void combine(const uint32_t* terms, int nbits, int W, int c, int seg, uint64_t* out) {
  HX<F> acc = zk::xyzz_inf<F>();
  for (int k = nbits - 1; k >= 0; k--) {
    acc = zk::xyzz_dbl(acc);
    acc = zk::xyzz_add(acc, ld_term_seg<F, CW>(terms, (size_t)k, seg));
    if (k % c == 0) acc = zk::xyzz_add(acc, ld_term_seg<F, CW>(terms, (size_t)(nbits + k / c), seg));
  }
  (void)W;
  to_affine<F, CW>(acc, out);
}

template <class F, int K>
HX<F> from_aff_canon(const uint64_t* a) {
  bool z = true;
  for (int i = 0; i < 2 * K; i++) z &= a[i] == 0;
  if (z) return zk::xyzz_inf<F>();
  zk::Aff<F> p;
  uint32_t w[16];
  (void)w;
  if constexpr (K == 4) {
    p.x = from_canon(a);
    p.y = from_canon(a + 4);
  } else {
    p.x = {from_canon(a), from_canon(a + 4)};
    p.y = {from_canon(a + 8), from_canon(a + 12)};
  }
  return zk::xyzz_from_aff(p);
}

}  // namespace

namespace zk {
void msm_host_combine_g1(const uint32_t* terms, int nbits, int W, int c, int seg, uint64_t out[8]) {
  combine<HFq, 8>(terms, nbits, W, c, seg, out);
}
void msm_host_combine_g2(const uint32_t* terms, int nbits, int W, int c, int seg, uint64_t out[16]) {
  combine<HFq2, 16>(terms, nbits, W, c, seg, out);
}
// Every rank's bit sums -> the combine's term layout -> the Horner epilogue
// (msm.hip msm_wait; host-only so tests/host/assemble_check.cpp runs it on the
// CPU).  payload r (at src + live[q] * stride) = a status block of `skip`
// words (word 3: first window << 16 | windows) then its terms, rank-major:
// window w's bb bit sums then its total, sb segments each.  Point shards:
// every term is the sum over the ranks (sb * nl segments).  Window shards:
// rank q's windows land at their global index, the rest stay all-zero
// (infinity).
void msm_host_assemble_combine(const uint32_t* src, size_t stride, size_t skip, const int* live, int nl,
                               bool wmode, int g2, int c, int W, int bb, int sb, uint64_t* out) {
  const int XW = g2 ? 64 : 32, nbits = c * W;
  const int nseg = wmode ? 1 : nl;    // ranks whose segments a term sums
  const size_t TW = (size_t)XW * sb;  // words per term and rank
  const size_t TA = TW * nseg;        // words per term over the ranks summed
  std::vector<uint32_t> all((size_t)(nbits + W) * TA, 0);
  for (int q = 0; q < nl; q++) {
    const uint32_t* stw = src + (size_t)live[q] * stride;
    const uint32_t* h = stw + skip;
    const int wr0 = wmode ? (int)(stw[3] >> 16) : 0, wrn = wmode ? (int)(stw[3] & 0xFFFF) : W;
    const size_t qo = wmode ? 0 : q * TW;
    for (int w = 0; w < wrn && wr0 + w < W; w++) {
      const int wg = wr0 + w;  // global window
      for (int j = 0; j < bb; j++)
        memcpy(&all[((size_t)c * wg + j) * TA + qo], &h[((size_t)w * (bb + 1) + j) * TW], TW * 4);
      memcpy(&all[((size_t)nbits + wg) * TA + qo], &h[((size_t)w * (bb + 1) + bb) * TW], TW * 4);
    }
  }
  if (!g2) combine<HFq, 8>(all.data(), nbits, W, c, sb * nseg, out);
  else combine<HFq2, 16>(all.data(), nbits, W, c, sb * nseg, out);
}

void host_g1_add_affine(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]) {
  auto r = xyzz_add(from_aff_canon<HFq, 4>(a), from_aff_canon<HFq, 4>(b));
  to_affine<HFq, 8>(r, out);
}
void host_g2_add_affine(const uint64_t a[16], const uint64_t b[16], uint64_t out[16]) {
  auto r = xyzz_add(from_aff_canon<HFq2, 8>(a), from_aff_canon<HFq2, 8>(b));
  to_affine<HFq2, 16>(r, out);
}

// ------------------------------------------------- Groth16 assembly (a4)
template <class F, int K>
static HX<F> smul(const uint64_t* aff, const uint64_t k[4]) {
  HX<F> base = from_aff_canon<F, K>(aff), acc = xyzz_inf<F>();
  for (int b = 255; b >= 0; b--) {
    acc = xyzz_dbl(acc);
    if ((k[b / 64] >> (b % 64)) & 1) acc = xyzz_add(acc, base);
  }
  return acc;
}
template <class F, int K>
static HX<F> pt(const uint64_t* aff) {
  return from_aff_canon<F, K>(aff);
}
static bool is_zero4(const uint64_t k[4]) { return (k[0] | k[1] | k[2] | k[3]) == 0; }

// Joint k1 P1 + k2 P2 (Straus, 4-bit windows): one doubling chain for both.
template <class F>
static HX<F> smul2(const HX<F>& p1, const uint64_t k1[4], const HX<F>& p2, const uint64_t k2[4]) {
  HX<F> t1[16], t2[16];
  t1[0] = t2[0] = xyzz_inf<F>();
  t1[1] = p1;
  t2[1] = p2;
  for (int i = 2; i < 16; i++) {
    t1[i] = xyzz_add(t1[i - 1], p1);
    t2[i] = xyzz_add(t2[i - 1], p2);
  }
  HX<F> acc = xyzz_inf<F>();
  for (int w = 63; w >= 0; w--) {
    for (int d = 0; d < 4; d++) acc = xyzz_dbl(acc);
    const int d1 = (int)((k1[w / 16] >> (4 * (w % 16))) & 15), d2 = (int)((k2[w / 16] >> (4 * (w % 16))) & 15);
    if (d1) acc = xyzz_add(acc, t1[d1]);
    if (d2) acc = xyzz_add(acc, t2[d2]);
  }
  return acc;
}
template <class F, int K>
static void st_hx(uint64_t* o, const HX<F>& p) {
  memcpy(o, &p, sizeof(HX<F>));
  static_assert(sizeof(HX<F>) == 4 * K * 8, "host XYZZ layout");
}
template <class F, int K>
static HX<F> ld_hx(const uint64_t* o) {
  HX<F> p;
  memcpy(&p, o, sizeof(HX<F>));
  return p;
}

// Groth16 assembly in three stages (ark-groth16 0.5 prover.rs
// create_proof_with_reduction_and_matrices), regrouped so
// that most of it runs while the GPU still works on the proof:
//   A  = r delta_1 + a0 + sum z a + alpha
//   B  = s delta_2 + b2_0 + sum z b_2 + beta_2
//   B1 = s delta_1 + B1',  B1' = b1_0 + sum z b_1 + beta_1   (ark: only if r != 0)
//   C  = s A + r B1 - r s delta_1 + l + h  =  s A + r B1' + l + h
// (r B1 - r s delta_1 = r B1'; with r = 0 both sides drop the term).  The
// group law is exact, so the affine A, B, C are the same field elements.
// Stage 1 (fixed): r delta_1, s delta_2 -- right after the submit, while the
// GPU runs the proof.  Stage 2 (after the a and b_g1 MSMs): A and s A + r B1'
// in one joint chain.  Then B (after b_g2) and C (after l and h): a few
// additions and an affine conversion each.  (configs[0]: the one-piece
// assembly cost ~2.1 ms of host time after the last MSM on this image's
// container CPU; staged, ~0.2 ms of it follows the last MSM.)
void groth16_asm_fixed(const uint64_t delta_g1[8], const uint64_t delta_g2[16], const uint64_t r[4],
                       const uint64_t s[4], G16Asm* st) {
  st_hx<HFq, 4>(st->rd1, smul<HFq, 4>(delta_g1, r));
  st_hx<HFq2, 8>(st->sd2, smul<HFq2, 8>(delta_g2, s));
}
// Fixed-base tables of a key's delta_1 / delta_2 (built once per key):
// entry [w][d] = d 2^(8w) delta, so r delta is 32 additions instead of a
// 256-step double-and-add (G2: ~0.1 ms instead of ~1 ms of host time here).
size_t groth16_asm_table_words(int g2) { return (size_t)32 * 256 * (g2 ? 32 : 16); }
template <class F, int K>
static void fb_table(const uint64_t* aff, uint64_t* tab) {
  HX<F> p = from_aff_canon<F, K>(aff);
  for (int w = 0; w < 32; w++) {
    HX<F> e = xyzz_inf<F>();
    for (int d = 0; d < 256; d++) {
      st_hx<F, K>(tab + ((size_t)w * 256 + d) * 4 * K, e);
      e = xyzz_add(e, p);
    }
    for (int i = 0; i < 8; i++) p = xyzz_dbl(p);
  }
}
template <class F, int K>
static HX<F> fb_mul(const uint64_t* tab, const uint64_t k[4]) {
  HX<F> acc = xyzz_inf<F>();
  for (int w = 0; w < 32; w++) {
    const int d = (int)((k[w / 8] >> (8 * (w % 8))) & 255);
    if (d) acc = xyzz_add(acc, ld_hx<F, K>(tab + ((size_t)w * 256 + d) * 4 * K));
  }
  return acc;
}
void groth16_asm_tables(const uint64_t delta_g1[8], const uint64_t delta_g2[16], uint64_t* tab1, uint64_t* tab2) {
  fb_table<HFq, 4>(delta_g1, tab1);
  fb_table<HFq2, 8>(delta_g2, tab2);
}
void groth16_asm_fixed_tab(const uint64_t* tab1, const uint64_t* tab2, const uint64_t r[4], const uint64_t s[4],
                           G16Asm* st) {
  st_hx<HFq, 4>(st->rd1, fb_mul<HFq, 4>(tab1, r));
  st_hx<HFq2, 8>(st->sd2, fb_mul<HFq2, 8>(tab2, s));
}
void groth16_asm_ab(const uint64_t alpha_g1[8], const uint64_t beta_g1[8], const uint64_t a0[8],
                    const uint64_t b1_0[8], const uint64_t a_acc[8], const uint64_t b1_acc[8], const uint64_t r[4],
                    const uint64_t s[4], G16Asm* st) {
  HX<HFq> A = ld_hx<HFq, 4>(st->rd1);
  A = xyzz_add(A, pt<HFq, 4>(a0));
  A = xyzz_add(A, pt<HFq, 4>(a_acc));
  A = xyzz_add(A, pt<HFq, 4>(alpha_g1));
  HX<HFq> B1p = xyzz_inf<HFq>();
  if (!is_zero4(r)) {
    B1p = xyzz_add(pt<HFq, 4>(b1_0), pt<HFq, 4>(b1_acc));
    B1p = xyzz_add(B1p, pt<HFq, 4>(beta_g1));
  }
  to_affine<HFq, 8>(A, st->a_aff);
  st_hx<HFq, 4>(st->c_part, smul2<HFq>(A, s, B1p, r));
}
void groth16_asm_b(const uint64_t beta_g2[16], const uint64_t b2_0[16], const uint64_t b2_acc[16], const G16Asm* st,
                   uint64_t b_out[16]) {
  HX<HFq2> B = ld_hx<HFq2, 8>(st->sd2);
  B = xyzz_add(B, pt<HFq2, 8>(b2_0));
  B = xyzz_add(B, pt<HFq2, 8>(b2_acc));
  B = xyzz_add(B, pt<HFq2, 8>(beta_g2));
  to_affine<HFq2, 16>(B, b_out);
}
void groth16_asm_c(const uint64_t l_acc[8], const uint64_t h_acc[8], const G16Asm* st, uint64_t a_out[8],
                   uint64_t c_out[8]) {
  HX<HFq> C = ld_hx<HFq, 4>(st->c_part);
  C = xyzz_add(C, pt<HFq, 4>(l_acc));
  C = xyzz_add(C, pt<HFq, 4>(h_acc));
  memcpy(a_out, st->a_aff, 64);
  to_affine<HFq, 8>(C, c_out);
}

void groth16_assemble(const uint64_t alpha_g1[8], const uint64_t beta_g1[8], const uint64_t delta_g1[8],
                      const uint64_t beta_g2[16], const uint64_t delta_g2[16], const uint64_t a0[8],
                      const uint64_t b1_0[8], const uint64_t b2_0[16], const uint64_t h_acc[8],
                      const uint64_t l_acc[8], const uint64_t a_acc[8], const uint64_t b1_acc[8],
                      const uint64_t b2_acc[16], const uint64_t r[4], const uint64_t s[4], uint64_t a_out[8],
                      uint64_t b_out[16], uint64_t c_out[8]) {
  G16Asm st;
  groth16_asm_fixed(delta_g1, delta_g2, r, s, &st);
  groth16_asm_ab(alpha_g1, beta_g1, a0, b1_0, a_acc, b1_acc, r, s, &st);
  groth16_asm_b(beta_g2, b2_0, b2_acc, &st, b_out);
  groth16_asm_c(l_acc, h_acc, &st, a_out, c_out);
}

// ---------------------------------------------------------- encodings
static void put_le(uint8_t* o, const uint64_t c[4]) {
  for (int i = 0; i < 32; i++) o[i] = (uint8_t)(c[i / 8] >> (8 * (i % 8)));
}
static int cmp_canon(const uint64_t a[4], const uint64_t b[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i] ? 1 : -1;
  }
  return 0;
}
static void neg_canon(uint64_t o[4], const uint64_t a[4]) {
  if ((a[0] | a[1] | a[2] | a[3]) == 0) {
    memset(o, 0, 32);
    return;
  }
  sub4(o, QP, a);
}
// arkworks SWFlags: bit 7 of the last byte = y > -y, bit 6 = infinity
void g1_compress(const uint64_t p[8], uint8_t out[32]) {
  bool inf = true;
  for (int i = 0; i < 8; i++) inf &= p[i] == 0;
  memset(out, 0, 32);
  if (inf) {
    out[31] |= 0x40;
    return;
  }
  put_le(out, p);
  uint64_t ny[4];
  neg_canon(ny, p + 4);
  if (cmp_canon(p + 4, ny) > 0) out[31] |= 0x80;
}
void g2_compress(const uint64_t p[16], uint8_t out[64]) {
  bool inf = true;
  for (int i = 0; i < 16; i++) inf &= p[i] == 0;
  memset(out, 0, 64);
  if (inf) {
    out[63] |= 0x40;
    return;
  }
  put_le(out, p);
  put_le(out + 32, p + 4);
  // Fq2 order: c1 first, then c0
  uint64_t n0[4], n1[4];
  neg_canon(n0, p + 8);
  neg_canon(n1, p + 12);
  int c = cmp_canon(p + 12, n1);
  if (c == 0) c = cmp_canon(p + 8, n0);
  if (c > 0) out[63] |= 0x80;
}
void proof_solana(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8], uint8_t out[256]) {
  uint64_t ny[4];
  neg_canon(ny, a + 4);
  put_le(out, a);       // -A: x unchanged
  put_le(out + 32, ny); //      y negated
  put_le(out + 64, b);
  put_le(out + 96, b + 4);
  put_le(out + 128, b + 8);
  put_le(out + 160, b + 12);
  put_le(out + 192, c);
  put_le(out + 224, c + 4);
}
}  // namespace zk
