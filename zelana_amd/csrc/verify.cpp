// verify.cpp — Groth16 verification and the on-chain (alt_bn128) encodings,
// host code of libzkmi.so.
//
// Restates, as product code, what consumes the prover's output:
//   * ark-groth16 verify_proof / the on-chain verifier's check
//     (onchain-programs/verifier/programs/onchain_verifier/src/lib.rs:497-547):
//       vk_x = IC[0] + sum_i x_i IC[i+1];  e(A, B) == e(alpha, beta) e(vk_x, gamma) e(C, delta)
//   * the alt_bn128 pairing syscall it calls (EIP-197 big-endian encoding:
//     G1 = x || y, G2 = x.c1 || x.c0 || y.c1 || y.c0; points validated on the
//     curve, G2 in the order-r subgroup; output 1 iff the product is 1),
//   * batch_inputs_to_field_elements (:479-494): the six roots as given and
//     batch_id as a 32-byte BIG-endian field element,
//   * a big-endian twin of proof_to_solana_bytes (core/src/sequencer/
//     settlement/prover.rs:304-334 writes little-endian coordinates, which the
//     BE syscalls would read differently: SURVEY.md App. B.3).
//
// Pairing: reduced Tate pairing over Fq12 = Fq[w] / (w^12 - 18 w^6 + 82)
// (w^6 = xi = 9 + u), the same construction tests/pairing.py pins against the
// reference's proof_for_onchain.json; here with Jacobian G1 steps whose lines
// are scaled by Fq factors (killed by the final exponentiation), one shared
// squaring per step for all pairs, and the final exponentiation decided
// without an Fq12 inversion: with h = (f^(q^2) f)^((q^4 - q^2 + 1) / r),
// f^((q^12 - 1) / r) = h^(q^6 - 1) = 1  <=>  h lies in Fq6 = span{w^even}.
#include <stdarg.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/zkmi.h"
#include "host_field.h"

namespace zk {
void set_error(const char* fmt, ...);
}

namespace {

using namespace zkh;

// ------------------------------------------------------------- constants
const uint64_t RP[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                        0x30644e72e131a029ULL};  // scalar field r
// (q^4 - q^2 + 1) / r, little-endian (the hard part of the final exponentiation)
const uint64_t HARD[12] = {0xe81bb482ccdf42b1ULL, 0x5abf5cc4f49c36d4ULL, 0xf1154e7e1da014fdULL,
                           0xdcc7b44c87cdbacfULL, 0xaaa441e3954bcf8aULL, 0x6b887d56d5095f23ULL,
                           0x79581e16f3fd90c6ULL, 0x3b1b1355d189227dULL, 0x4e529a5861876f6bULL,
                           0x6c0eb522d5b12278ULL, 0x331ec15183177fafULL, 0x01baaa710b0759adULL};
// q^2, little-endian
const uint64_t Q2[8] = {0x3b5458a2275d69b1ULL, 0xa602072d09eac101ULL, 0x4a50189c6d96cadcULL,
                        0x04689e957a1242c8ULL, 0x26edfa5c34c6b38dULL, 0xb00b855116375606ULL,
                        0x599a6f7c0348d21cULL, 0x0925c4b8763cbf9cULL};

F4 fsmall(uint64_t v) {
  uint64_t c[4] = {v, 0, 0, 0};
  return from_canon(c);
}
F4 fneg(const F4& a) { return fsub(F4{{0, 0, 0, 0}}, a); }
bool feq(const F4& a, const F4& b) { return memcmp(a.l, b.l, 32) == 0; }
bool lt_q(const uint64_t c[4]) { return !geq(c, QP); }
void shr(uint64_t o[4], const uint64_t a[4], int k) {
  for (int i = 0; i < 4; i++) o[i] = (a[i] >> k) | (i < 3 ? a[i + 1] << (64 - k) : 0);
}
// canonical integer compare (for the arkworks "y > -y" flag)
int cmp_canon(const F4& a, const F4& b) {
  uint64_t x[4], y[4];
  to_canon(x, a);
  to_canon(y, b);
  for (int i = 3; i >= 0; i--)
    if (x[i] != y[i]) return x[i] > y[i] ? 1 : -1;
  return 0;
}

// ------------------------------------------------------------- Fq2
using F2 = F42;
F2 f2_mul(const F2& a, const F2& b) { return HFq2::mul(a, b); }
F2 f2_add(const F2& a, const F2& b) { return HFq2::add(a, b); }
F2 f2_sub(const F2& a, const F2& b) { return HFq2::sub(a, b); }
bool f2_eq(const F2& a, const F2& b) { return feq(a.c0, b.c0) && feq(a.c1, b.c1); }
bool f2_zero(const F2& a) { return fzero(a.c0) && fzero(a.c1); }
F2 f2_pow(const F2& a, const uint64_t* e, int words) {
  F2 r = HFq2::one();
  for (int i = 64 * words - 1; i >= 0; i--) {
    r = f2_mul(r, r);
    if ((e[i / 64] >> (i % 64)) & 1) r = f2_mul(r, a);
  }
  return r;
}
// 3 / (9 + u): the twist's b
F2 twist_b() {
  F2 xi = {fsmall(9), fsmall(1)};
  F2 three = {fsmall(3), F4{{0, 0, 0, 0}}};
  return f2_mul(three, HFq2::inv(xi));
}

// sqrt in Fq (q = 3 mod 4); false if a is a non-residue
bool fq_sqrt(const F4& a, F4* out) {
  uint64_t e[4], one[4] = {1, 0, 0, 0}, t[4];
  add4(t, QP, one);
  shr(e, t, 2);  // (q + 1) / 4
  F4 s = fpow(a, e);
  if (!feq(fmul(s, s), a)) return false;
  *out = s;
  return true;
}
// sqrt in Fq2 (q = 3 mod 4): Adj & Rodriguez-Henriquez, Algorithm 9
bool fq2_sqrt(const F2& a, F2* out) {
  if (f2_zero(a)) {
    *out = a;
    return true;
  }
  uint64_t three[4] = {3, 0, 0, 0}, one[4] = {1, 0, 0, 0}, t[4], e34[4], e12[4];
  sub4(t, QP, three);
  shr(e34, t, 2);  // (q - 3) / 4
  sub4(t, QP, one);
  shr(e12, t, 1);  // (q - 1) / 2
  F2 a1 = f2_pow(a, e34, 4);
  F2 alpha = f2_mul(f2_mul(a1, a1), a);
  F2 x0 = f2_mul(a1, a);
  F2 mone = {fneg(fconst(QONE)), F4{{0, 0, 0, 0}}};
  F2 x;
  if (f2_eq(alpha, mone)) {
    x = {fneg(x0.c1), x0.c0};  // u * x0
  } else {
    F2 b = f2_pow(f2_add(HFq2::one(), alpha), e12, 4);
    x = f2_mul(b, x0);
  }
  if (!f2_eq(f2_mul(x, x), a)) return false;
  *out = x;
  return true;
}

// ------------------------------------------------------------- points
struct G1 {
  F4 x, y;
  bool inf;
};
struct G2 {
  F2 x, y;
  bool inf;
};
bool g1_on_curve(const G1& p) {
  if (p.inf) return true;
  return feq(fmul(p.y, p.y), fadd(fmul(fmul(p.x, p.x), p.x), fsmall(3)));
}
bool g2_on_curve(const G2& p) {
  if (p.inf) return true;
  return f2_eq(f2_mul(p.y, p.y), f2_add(f2_mul(f2_mul(p.x, p.x), p.x), twist_b()));
}
G1 g1_from_canon(const uint64_t p[8]) {
  G1 r;
  bool z = true;
  for (int i = 0; i < 8; i++) z &= p[i] == 0;
  r.inf = z;
  r.x = from_canon(p);
  r.y = from_canon(p + 4);
  return r;
}
G2 g2_from_canon(const uint64_t p[16]) {
  G2 r;
  bool z = true;
  for (int i = 0; i < 16; i++) z &= p[i] == 0;
  r.inf = z;
  r.x = {from_canon(p), from_canon(p + 4)};
  r.y = {from_canon(p + 8), from_canon(p + 12)};
  return r;
}
void g1_to_canon(uint64_t o[8], const G1& p) {
  if (p.inf) {
    memset(o, 0, 64);
    return;
  }
  to_canon(o, p.x);
  to_canon(o + 4, p.y);
}

// group law on G1 / G2 in XYZZ (ec.h templates over the host field)
template <class F, class P>
zk::Xyzz<F> to_xyzz(const P& p) {
  if (p.inf) return zk::xyzz_inf<F>();
  zk::Aff<F> a;
  a.x = p.x;
  a.y = p.y;
  return zk::xyzz_from_aff(a);
}
template <class F>
bool xyzz_to_aff(const zk::Xyzz<F>& p, typename F::T* x, typename F::T* y);
template <>
bool xyzz_to_aff<HFq>(const zk::Xyzz<HFq>& p, F4* x, F4* y) {
  if (zk::xyzz_is_inf(p)) return false;
  *x = fmul(p.x, finv(p.zz));
  *y = fmul(p.y, finv(p.zzz));
  return true;
}
template <>
bool xyzz_to_aff<HFq2>(const zk::Xyzz<HFq2>& p, F2* x, F2* y) {
  if (zk::xyzz_is_inf(p)) return false;
  *x = f2_mul(p.x, HFq2::inv(p.zz));
  *y = f2_mul(p.y, HFq2::inv(p.zzz));
  return true;
}
template <class F>
zk::Xyzz<F> xyzz_smul(const zk::Xyzz<F>& base, const uint64_t* k, int words) {
  zk::Xyzz<F> acc = zk::xyzz_inf<F>();
  for (int b = 64 * words - 1; b >= 0; b--) {
    acc = zk::xyzz_dbl(acc);
    if ((k[b / 64] >> (b % 64)) & 1) acc = zk::xyzz_add(acc, base);
  }
  return acc;
}
G1 g1_add(const G1& a, const G1& b) {
  zk::Xyzz<HFq> s = zk::xyzz_add(to_xyzz<HFq>(a), to_xyzz<HFq>(b));
  G1 r;
  r.inf = !xyzz_to_aff<HFq>(s, &r.x, &r.y);
  return r;
}
G1 g1_mul(const G1& p, const uint64_t k[4]) {
  zk::Xyzz<HFq> s = xyzz_smul(to_xyzz<HFq>(p), k, 4);
  G1 r;
  r.inf = !xyzz_to_aff<HFq>(s, &r.x, &r.y);
  return r;
}
bool g2_in_subgroup(const G2& p) {
  if (p.inf) return true;
  return zk::xyzz_is_inf(xyzz_smul(to_xyzz<HFq2>(p), RP, 4));
}

// arkworks SWFlags decoding (ark-serialize 0.5, as Groth16Prover::from_bytes
// reads keys): compressed G1 = x LE with bit 7 of byte 31 = "y > -y", bit 6 =
// infinity; G2 = x.c0 || x.c1 with the flags in byte 63, Fq2 ordered (c1, c0)
void le_words(uint64_t o[4], const uint8_t* b) {
  for (int i = 0; i < 4; i++) {
    o[i] = 0;
    for (int j = 0; j < 8; j++) o[i] |= (uint64_t)b[8 * i + j] << (8 * j);
  }
}
bool g1_decompress(const uint8_t in[32], G1* out) {
  const bool pos = in[31] & 0x80, infl = in[31] & 0x40;
  uint64_t x[4];
  le_words(x, in);
  x[3] &= 0x3FFFFFFFFFFFFFFFULL;
  if (infl) {
    *out = G1{F4{{0, 0, 0, 0}}, F4{{0, 0, 0, 0}}, true};
    return (x[0] | x[1] | x[2] | x[3]) == 0 && !pos;
  }
  if (!lt_q(x)) return false;
  G1 p;
  p.inf = false;
  p.x = from_canon(x);
  if (!fq_sqrt(fadd(fmul(fmul(p.x, p.x), p.x), fsmall(3)), &p.y)) return false;
  if ((cmp_canon(p.y, fneg(p.y)) > 0) != pos) p.y = fneg(p.y);
  *out = p;
  return true;
}
int f2_cmp(const F2& a, const F2& b) {
  int c = cmp_canon(a.c1, b.c1);
  return c ? c : cmp_canon(a.c0, b.c0);
}
bool g2_decompress(const uint8_t in[64], G2* out) {
  const bool pos = in[63] & 0x80, infl = in[63] & 0x40;
  uint64_t x0[4], x1[4];
  le_words(x0, in);
  le_words(x1, in + 32);
  x1[3] &= 0x3FFFFFFFFFFFFFFFULL;
  if (infl) {
    *out = G2{HFq2::zero(), HFq2::zero(), true};
    return (x0[0] | x0[1] | x0[2] | x0[3] | x1[0] | x1[1] | x1[2] | x1[3]) == 0 && !pos;
  }
  if (!lt_q(x0) || !lt_q(x1)) return false;
  G2 p;
  p.inf = false;
  p.x = {from_canon(x0), from_canon(x1)};
  if (!fq2_sqrt(f2_add(f2_mul(f2_mul(p.x, p.x), p.x), twist_b()), &p.y)) return false;
  F2 ny = HFq2::neg(p.y);
  if ((f2_cmp(p.y, ny) > 0) != pos) p.y = ny;
  if (!g2_in_subgroup(p)) return false;
  *out = p;
  return true;
}

// ------------------------------------------------------------- Fq12
struct F12 {
  F4 c[12];
};
F12 f12_one() {
  F12 r;
  memset(&r, 0, sizeof(r));
  r.c[0] = fconst(QONE);
  return r;
}
const F4& k18() {
  static const F4 v = fsmall(18);
  return v;
}
const F4& k82() {
  static const F4 v = fsmall(82);
  return v;
}
// reduce a 23-coefficient product: w^12 = 18 w^6 - 82
F12 f12_reduce(F4 acc[23]) {
  for (int k = 22; k >= 12; k--) {
    if (fzero(acc[k])) continue;
    acc[k - 6] = fadd(acc[k - 6], fmul(acc[k], k18()));
    acc[k - 12] = fsub(acc[k - 12], fmul(acc[k], k82()));
  }
  F12 r;
  for (int i = 0; i < 12; i++) r.c[i] = acc[i];
  return r;
}
F12 f12_mul(const F12& a, const F12& b) {
  F4 acc[23];
  memset(acc, 0, sizeof(acc));
  for (int i = 0; i < 12; i++) {
    if (fzero(a.c[i])) continue;
    for (int j = 0; j < 12; j++) acc[i + j] = fadd(acc[i + j], fmul(a.c[i], b.c[j]));
  }
  return f12_reduce(acc);
}
F12 f12_sqr(const F12& a) {
  F4 acc[23];
  memset(acc, 0, sizeof(acc));
  for (int i = 0; i < 12; i++) {
    acc[2 * i] = fadd(acc[2 * i], fmul(a.c[i], a.c[i]));
    for (int j = i + 1; j < 12; j++) {
      F4 t = fmul(a.c[i], a.c[j]);
      acc[i + j] = fadd(acc[i + j], fadd(t, t));
    }
  }
  return f12_reduce(acc);
}
// f * (sparse element with terms at the listed powers)
F12 f12_mul_sparse(const F12& a, const int* pw, const F4* cf, int nt) {
  F4 acc[23];
  memset(acc, 0, sizeof(acc));
  for (int t = 0; t < nt; t++)
    for (int i = 0; i < 12; i++) acc[i + pw[t]] = fadd(acc[i + pw[t]], fmul(a.c[i], cf[t]));
  return f12_reduce(acc);
}
F12 f12_pow(const F12& a, const uint64_t* e, int words) {
  // fixed 4-bit windows
  F12 tab[16];
  tab[0] = f12_one();
  for (int i = 1; i < 16; i++) tab[i] = f12_mul(tab[i - 1], a);
  F12 r = f12_one();
  bool started = false;
  for (int i = words * 16 - 1; i >= 0; i--) {
    const int d = (int)((e[i / 16] >> (4 * (i % 16))) & 15);
    if (started)
      for (int k = 0; k < 4; k++) r = f12_sqr(r);
    if (d) {
      r = started ? f12_mul(r, tab[d]) : tab[d];
      started = true;
    }
  }
  return r;
}
// Frobenius^2: f = sum f_i w^i (f_i in Fq) -> sum f_i (w^(q^2))^i
const F12* frob2_table() {
  static std::vector<F12> tab = [] {
    F12 w;
    memset(&w, 0, sizeof(w));
    w.c[1] = fconst(QONE);
    F12 wq2 = f12_pow(w, Q2, 8);
    std::vector<F12> t(12);
    t[0] = f12_one();
    for (int i = 1; i < 12; i++) t[i] = f12_mul(t[i - 1], wq2);
    return t;
  }();
  return tab.data();
}
F12 f12_frob2(const F12& a) {
  const F12* t = frob2_table();
  F12 r;
  memset(&r, 0, sizeof(r));
  for (int i = 0; i < 12; i++) {
    if (fzero(a.c[i])) continue;
    for (int j = 0; j < 12; j++) r.c[j] = fadd(r.c[j], fmul(a.c[i], t[i].c[j]));
  }
  return r;
}

// ------------------------------------------------------------- Miller loop
// G2 point untwisted into E(Fq12): x w^2, y w^3 with c0 + c1 u = (c0 - 9 c1) + c1 w^6
struct QUn {
  F4 x2, x8, y3, y9;
};
QUn untwist(const G2& q) {
  F4 nine = fsmall(9);
  return {fsub(q.x.c0, fmul(nine, q.x.c1)), q.x.c1, fsub(q.y.c0, fmul(nine, q.y.c1)), q.y.c1};
}
// f *= a*yQ - b*xQ + c   (a, b, c in Fq)
F12 mul_line(const F12& f, const QUn& q, const F4& a, const F4& b, const F4& c) {
  const int pw[5] = {0, 2, 8, 3, 9};
  F4 nb = fneg(b);
  const F4 cf[5] = {c, fmul(nb, q.x2), fmul(nb, q.x8), fmul(a, q.y3), fmul(a, q.y9)};
  return f12_mul_sparse(f, pw, cf, 5);
}
struct Jac {
  F4 X, Y, Z;
  bool inf;
};

// prod_k e(P_k, Q_k) == 1  (reduced Tate pairing)
bool pairing_product_is_one(const std::vector<G1>& ps, const std::vector<G2>& qs) {
  std::vector<size_t> idx;
  for (size_t k = 0; k < ps.size(); k++)
    if (!ps[k].inf && !qs[k].inf) idx.push_back(k);
  if (idx.empty()) return true;
  std::vector<Jac> T(ps.size());
  std::vector<QUn> Q(ps.size());
  for (size_t k : idx) {
    T[k] = {ps[k].x, ps[k].y, fconst(QONE), false};
    Q[k] = untwist(qs[k]);
  }
  int top = 255;
  while (!((RP[top / 64] >> (top % 64)) & 1)) top--;
  F12 f = f12_one();
  const F4 two = fsmall(2), three = fsmall(3);
  for (int bit = top - 1; bit >= 0; bit--) {
    f = f12_sqr(f);
    for (size_t k : idx) {
      Jac& t = T[k];
      if (t.inf) continue;
      // tangent line, scaled by 2 Y Z^3: a = 2 Y Z^3, b = 3 X^2 Z^2, c = 3 X^3 - 2 Y^2
      F4 Z2 = fmul(t.Z, t.Z), X2 = fmul(t.X, t.X), Y2 = fmul(t.Y, t.Y);
      F4 a = fmul(fmul(two, t.Y), fmul(Z2, t.Z));
      F4 b = fmul(fmul(three, X2), Z2);
      F4 c = fsub(fmul(three, fmul(X2, t.X)), fmul(two, Y2));
      f = mul_line(f, Q[k], a, b, c);
      // T = 2T (dbl-2009-l, a = 0)
      F4 C = fmul(Y2, Y2);
      F4 D = fsub(fsub(fmul(fadd(t.X, Y2), fadd(t.X, Y2)), X2), C);
      D = fadd(D, D);
      F4 E = fmul(three, X2);
      F4 X3 = fsub(fmul(E, E), fadd(D, D));
      F4 C8 = fmul(fsmall(8), C);
      F4 Y3 = fsub(fmul(E, fsub(D, X3)), C8);
      F4 Z3 = fmul(fmul(two, t.Y), t.Z);
      t = {X3, Y3, Z3, false};
    }
    if ((RP[bit / 64] >> (bit % 64)) & 1) {
      for (size_t k : idx) {
        Jac& t = T[k];
        if (t.inf) continue;
        const G1& p = ps[k];
        F4 Z2 = fmul(t.Z, t.Z);
        F4 H = fsub(fmul(p.x, Z2), t.X);
        F4 Rr = fsub(fmul(p.y, fmul(Z2, t.Z)), t.Y);
        if (fzero(H)) {
          // T = -P: the vertical line lies in Fq6 and dies in the final
          // exponentiation (the last step of the loop: r P = O)
          t.inf = true;
          continue;
        }
        F4 HZ = fmul(H, t.Z);
        f = mul_line(f, Q[k], HZ, Rr, fsub(fmul(Rr, p.x), fmul(HZ, p.y)));
        F4 HH = fmul(H, H), HHH = fmul(H, HH), V = fmul(t.X, HH);
        F4 X3 = fsub(fsub(fmul(Rr, Rr), HHH), fadd(V, V));
        F4 Y3 = fsub(fmul(Rr, fsub(V, X3)), fmul(t.Y, HHH));
        t = {X3, Y3, HZ, false};
      }
    }
  }
  // final exponentiation: h = (f^(q^2) f)^((q^4 - q^2 + 1)/r) must lie in Fq6
  F12 h = f12_pow(f12_mul(f12_frob2(f), f), HARD, 12);
  bool nonzero = false;
  for (int i = 0; i < 12; i++) nonzero |= !fzero(h.c[i]);
  if (!nonzero) return false;
  for (int i = 1; i < 12; i += 2)
    if (!fzero(h.c[i])) return false;
  return true;
}

// ------------------------------------------------------------- encodings
void put_be(uint8_t* o, const F4& a) {
  uint64_t c[4];
  to_canon(c, a);
  for (int i = 0; i < 32; i++) o[i] = (uint8_t)(c[3 - i / 8] >> (8 * (7 - i % 8)));
}
void get_be(uint64_t c[4], const uint8_t* b) {
  for (int i = 0; i < 4; i++) {
    c[3 - i] = 0;
    for (int j = 0; j < 8; j++) c[3 - i] = (c[3 - i] << 8) | b[8 * i + j];
  }
}
// EIP-196/197: (0, 0) is the point at infinity; coordinates must be < q
bool g1_from_be(const uint8_t b[64], G1* p) {
  uint64_t x[4], y[4];
  get_be(x, b);
  get_be(y, b + 32);
  if (!lt_q(x) || !lt_q(y)) return false;
  p->inf = (x[0] | x[1] | x[2] | x[3] | y[0] | y[1] | y[2] | y[3]) == 0;
  p->x = from_canon(x);
  p->y = from_canon(y);
  return g1_on_curve(*p);
}
bool g2_from_be(const uint8_t b[128], G2* p) {
  uint64_t w[4][4];
  for (int i = 0; i < 4; i++) {
    get_be(w[i], b + 32 * i);
    if (!lt_q(w[i])) return false;
  }
  bool z = true;
  for (int i = 0; i < 4; i++) z &= (w[i][0] | w[i][1] | w[i][2] | w[i][3]) == 0;
  p->inf = z;
  p->x = {from_canon(w[1]), from_canon(w[0])};  // imaginary part first
  p->y = {from_canon(w[3]), from_canon(w[2])};
  return g2_on_curve(*p) && g2_in_subgroup(*p);
}
void g1_to_be(uint8_t o[64], const G1& p) {
  if (p.inf) {
    memset(o, 0, 64);
    return;
  }
  put_be(o, p.x);
  put_be(o + 32, p.y);
}
void g2_to_be(uint8_t o[128], const G2& p) {
  if (p.inf) {
    memset(o, 0, 128);
    return;
  }
  put_be(o, p.x.c1);
  put_be(o + 32, p.x.c0);
  put_be(o + 64, p.y.c1);
  put_be(o + 96, p.y.c0);
}

// arkworks-compressed VerifyingKey<Bn254>: alpha(32) beta(64) gamma(64)
// delta(64) u64-LE count + IC x 32 (prover/l2_vk.json layout)
struct Vk {
  G1 alpha;
  G2 beta, gamma, delta;
  std::vector<G1> ic;
};
bool vk_decode(const uint8_t* b, size_t len, Vk* vk, const char** why) {
  if (len < 232) {
    *why = "verifying key shorter than 232 bytes";
    return false;
  }
  if (!g1_decompress(b, &vk->alpha) || !g2_decompress(b + 32, &vk->beta) || !g2_decompress(b + 96, &vk->gamma) ||
      !g2_decompress(b + 160, &vk->delta)) {
    *why = "invalid alpha / beta / gamma / delta point";
    return false;
  }
  uint64_t n = 0;
  for (int i = 0; i < 8; i++) n |= (uint64_t)b[224 + i] << (8 * i);
  if (n == 0 || n > (len - 232) / 32 || 232 + 32 * n != len) {
    *why = "IC length does not match the key size";
    return false;
  }
  vk->ic.resize(n);
  for (uint64_t i = 0; i < n; i++)
    if (!g1_decompress(b + 232 + 32 * i, &vk->ic[i])) {
      *why = "invalid IC point";
      return false;
    }
  return true;
}

}  // namespace

using zk::set_error;

extern "C" {

int zkmi_groth16_verify(const uint8_t* vk_bytes, size_t vk_len, const uint64_t* inputs, size_t n_inputs,
                        const uint64_t a[8], const uint64_t b[16], const uint64_t c[8], int* valid) {
  if (!vk_bytes || !a || !b || !c || !valid || (n_inputs && !inputs)) {
    set_error("zkmi_groth16_verify: null argument");
    return ZKMI_EINVAL;
  }
  *valid = 0;
  Vk vk;
  const char* why = "";
  if (!vk_decode(vk_bytes, vk_len, &vk, &why)) {
    set_error("zkmi_groth16_verify: %s", why);
    return ZKMI_EPOINT;
  }
  if (vk.ic.size() != n_inputs + 1) {
    set_error("zkmi_groth16_verify: %zu public inputs for a key with %zu IC points", n_inputs, vk.ic.size());
    return ZKMI_EINVAL;
  }
  // every proof coordinate must be canonical (< q): from_canon would reduce a
  // non-canonical encoding silently and accept it (the alt_bn128 entry points
  // refuse such inputs too)
  for (int i = 0; i < 2; i++)
    if (!lt_q(a + 4 * i) || !lt_q(c + 4 * i)) return 0;  // invalid proof
  for (int i = 0; i < 4; i++)
    if (!lt_q(b + 4 * i)) return 0;
  G1 A = g1_from_canon(a), C = g1_from_canon(c);
  G2 B = g2_from_canon(b);
  if (!g1_on_curve(A) || !g1_on_curve(C) || !g2_on_curve(B) || !g2_in_subgroup(B)) return 0;  // invalid proof
  G1 acc = vk.ic[0];
  for (size_t i = 0; i < n_inputs; i++) {
    if (geq(inputs + 4 * i, RP)) {
      set_error("zkmi_groth16_verify: public input %zu not reduced mod r", i);
      return ZKMI_EINVAL;
    }
    acc = g1_add(acc, g1_mul(vk.ic[i + 1], inputs + 4 * i));
  }
  auto neg = [](G1 p) {
    if (!p.inf) p.y = fneg(p.y);
    return p;
  };
  // e(A, B) e(-alpha, beta) e(-vk_x, gamma) e(-C, delta) == 1
  *valid = pairing_product_is_one({A, neg(vk.alpha), neg(acc), neg(C)}, {B, vk.beta, vk.gamma, vk.delta}) ? 1 : 0;
  return 0;
}

int zkmi_alt_bn128_pairing(const uint8_t* input, size_t len, uint8_t out[32]) {
  if ((!input && len) || !out || len % 192) {
    set_error("zkmi_alt_bn128_pairing: input must be k x 192 bytes");
    return ZKMI_EINVAL;
  }
  std::vector<G1> ps(len / 192);
  std::vector<G2> qs(len / 192);
  for (size_t k = 0; k < len / 192; k++) {
    if (!g1_from_be(input + 192 * k, &ps[k]) || !g2_from_be(input + 192 * k + 64, &qs[k])) {
      set_error("zkmi_alt_bn128_pairing: pair %zu is not a valid (G1, G2) point pair", k);
      return ZKMI_EPOINT;
    }
  }
  memset(out, 0, 32);
  out[31] = pairing_product_is_one(ps, qs) ? 1 : 0;
  return 0;
}

int zkmi_alt_bn128_g1_add(const uint8_t in[128], uint8_t out[64]) {
  G1 p, q;
  if (!in || !out || !g1_from_be(in, &p) || !g1_from_be(in + 64, &q)) {
    set_error("zkmi_alt_bn128_g1_add: invalid point");
    return ZKMI_EPOINT;
  }
  g1_to_be(out, g1_add(p, q));
  return 0;
}

int zkmi_alt_bn128_g1_mul(const uint8_t in[96], uint8_t out[64]) {
  G1 p;
  if (!in || !out || !g1_from_be(in, &p)) {
    set_error("zkmi_alt_bn128_g1_mul: invalid point");
    return ZKMI_EPOINT;
  }
  uint64_t k[4];
  get_be(k, in + 64);
  g1_to_be(out, g1_mul(p, k));
  return 0;
}

int zkmi_proof_to_alt_bn128_bytes(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8], uint8_t out[256]) {
  if (!a || !b || !c || !out) {
    set_error("zkmi_proof_to_alt_bn128_bytes: null argument");
    return ZKMI_EINVAL;
  }
  G1 A = g1_from_canon(a), C = g1_from_canon(c);
  if (!A.inf) A.y = fneg(A.y);  // -A, as proof_to_solana_bytes
  g1_to_be(out, A);
  g2_to_be(out + 64, g2_from_canon(b));
  g1_to_be(out + 192, C);
  return 0;
}

int zkmi_batch_inputs_alt_bn128(const uint8_t roots[6 * 32], uint64_t batch_id, uint8_t out[7 * 32]) {
  if (!roots || !out) {
    set_error("zkmi_batch_inputs_alt_bn128: null argument");
    return ZKMI_EINVAL;
  }
  memcpy(out, roots, 6 * 32);
  memset(out + 6 * 32, 0, 32);
  for (int i = 0; i < 8; i++) out[6 * 32 + 24 + i] = (uint8_t)(batch_id >> (8 * (7 - i)));
  return 0;
}

int zkmi_g1_mul(const uint64_t p[8], const uint64_t k[4], uint64_t out[8]) {
  if (!p || !k || !out) {
    set_error("zkmi_g1_mul: null argument");
    return ZKMI_EINVAL;
  }
  G1 P = g1_from_canon(p);
  if (!g1_on_curve(P)) {
    set_error("zkmi_g1_mul: point not on the curve");
    return ZKMI_EPOINT;
  }
  g1_to_canon(out, g1_mul(P, k));
  return 0;
}

}  // extern "C"
