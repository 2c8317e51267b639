// l2_circuit.cpp — see l2_circuit.h.  A line-for-line restatement of
// zelana_amd/l2block.py (itself following prover/src/l2_circuit.rs and the
// arkworks 0.5 gadgets) so the C++ host mirror needs no Python.
#include "l2_circuit.h"

#include <algorithm>
#include <set>
#include <stdexcept>

namespace zp {

// ------------------------------------------------------------------ Poseidon
namespace {

constexpr int kModulusBits = 254;

// PoseidonGrainLFSR (ark-crypto-primitives 0.5.0 sponge/poseidon/grain_lfsr.rs)
class GrainLFSR {
 public:
  GrainLFSR(uint64_t prime_bits, uint64_t state_len, uint64_t full, uint64_t partial) : bits_(prime_bits) {
    bool s[80] = {false};
    s[1] = true;  // prime field; S-box x^alpha (b5 = 0)
    auto put = [&](int lo, int hi, uint64_t v) {
      for (int i = hi; i >= lo; i--, v >>= 1) s[i] = v & 1;
    };
    put(6, 17, prime_bits);
    put(18, 29, state_len);
    put(30, 39, full);
    put(40, 49, partial);
    for (int i = 50; i < 80; i++) s[i] = true;
    for (int i = 0; i < 80; i++) s_[i] = s[i];
    for (int i = 0; i < 160; i++) update();
  }
  // MSB-first integer of prime_bits filtered bits
  void next_int(uint64_t out[4]) {
    out[0] = out[1] = out[2] = out[3] = 0;
    for (uint64_t k = 0; k < bits_; k++) {
      bool b = update();
      while (!b) {
        update();
        b = update();
      }
      bool v = update();
      // shift left by one, add v
      for (int i = 3; i > 0; i--) out[i] = (out[i] << 1) | (out[i - 1] >> 63);
      out[0] = (out[0] << 1) | (uint64_t)v;
    }
  }
  Fr rejection() {
    for (;;) {
      uint64_t v[4];
      next_int(v);
      if (!Fr::geq_p(v)) return Fr::from_canon(v);
    }
  }
  Fr mod_p() {
    uint64_t v[4];
    next_int(v);  // < 2^254 < 4r: reduce by conditional subtractions
    while (Fr::geq_p(v)) Fr::sub_p(v);
    return Fr::from_canon(v);
  }

 private:
  bool update() {
    const int h = head_;
    bool b = s_[(h + 62) % 80] ^ s_[(h + 51) % 80] ^ s_[(h + 38) % 80] ^ s_[(h + 23) % 80] ^ s_[(h + 13) % 80] ^ s_[h];
    s_[h] = b;
    head_ = (h + 1) % 80;
    return b;
  }
  bool s_[80];
  int head_ = 0;
  uint64_t bits_;
};

struct PoseidonParams {
  int rate = 2, capacity = 1, full = 8, partial = 56;
  uint64_t alpha = 5;
  std::vector<std::array<Fr, 3>> ark;
  Fr mds[3][3];
};

const PoseidonParams& poseidon_params() {  // find_poseidon_ark_and_mds(254, 2, 8, 56, 0)
  static const PoseidonParams P = [] {
    PoseidonParams p;
    GrainLFSR lfsr(kModulusBits, 3, 8, 56);
    for (int r = 0; r < 64; r++) {
      std::array<Fr, 3> row;
      for (int i = 0; i < 3; i++) row[i] = lfsr.rejection();
      p.ark.push_back(row);
    }
    Fr xs[3], ys[3];
    for (int i = 0; i < 3; i++) xs[i] = lfsr.mod_p();
    for (int i = 0; i < 3; i++) ys[i] = lfsr.mod_p();
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) p.mds[i][j] = (xs[i] + ys[j]).inverse();
    return p;
  }();
  return P;
}

// ------------------------------------------------------------------ CS
constexpr uint64_t kWit = 1ULL << 62;  // witness symbols; instance k -> k, One = 0
// A linear combination: terms sorted by symbol (what a std::map held before;
// one merge per addition instead of a node allocation per term -- the
// Poseidon partial rounds' growing combinations made that the synthesis's
// cost).  Coefficients that cancel stay as zero terms, which the matrix
// conversion skips, as it did with the map.
using LC = std::vector<std::pair<uint64_t, Fr>>;

LC lc_add(const LC& a, const LC& b, bool sub = false) {
  LC o;
  o.reserve(a.size() + b.size());
  size_t i = 0, j = 0;
  while (i < a.size() || j < b.size()) {
    if (j == b.size() || (i < a.size() && a[i].first < b[j].first)) {
      o.push_back(a[i++]);
    } else if (i == a.size() || b[j].first < a[i].first) {
      o.emplace_back(b[j].first, sub ? Fr() - b[j].second : b[j].second);
      j++;
    } else {
      o.emplace_back(a[i].first, sub ? a[i].second - b[j].second : a[i].second + b[j].second);
      i++, j++;
    }
  }
  return o;
}
LC lc_scale(const LC& a, const Fr& c) {
  LC o;
  o.reserve(a.size());
  for (const auto& kv : a) o.emplace_back(kv.first, kv.second * c);
  return o;
}

// witness-program op kinds (zkmi.h)
constexpr uint32_t WP_MUL = 1, WP_INV = 2, WP_BITS = 5, WP_NZ = 6, WP_POSEIDON = 7, WP_INV1 = 8;

struct CS {
  std::vector<Fr> inst{Fr::one()}, wit;
  std::vector<std::array<LC, 3>> rows;
  // Witness-program recording: the free inputs (symbols, allocation order)
  // and one op per computed witness group.  `mute` > 0 inside a gadget that
  // records itself as one op (a permutation, a bit decomposition).
  struct Rec {
    uint32_t kind;
    uint64_t out;  // first output symbol
    std::vector<LC> lcs;
    uint32_t aux;  // BITS: bit count; POSEIDON: round-0 variable mask
  };
  bool record = false;
  int mute = 0;
  std::vector<Rec> ops;
  std::vector<uint64_t> in_syms{0};  // One
  void op(uint32_t kind, uint64_t out, std::vector<LC> lcs, uint32_t aux = 0) {
    if (record && !mute) ops.push_back({kind, out, std::move(lcs), aux});
  }
  uint64_t next_witness() const { return kWit + wit.size(); }
  LC new_input(const Fr& v) {
    inst.push_back(v);
    in_syms.push_back(inst.size() - 1);
    return LC{{inst.size() - 1, Fr::one()}};
  }
  LC new_witness(const Fr& v) {
    wit.push_back(v);
    return LC{{kWit + wit.size() - 1, Fr::one()}};
  }
  // a witness taken from the batch's data (a free input of the program)
  LC new_data(const Fr& v) {
    in_syms.push_back(next_witness());
    return new_witness(v);
  }
  void enforce(const LC& a, const LC& b, const LC& c) { rows.push_back({a, b, c}); }
};

LC one_lc(const Fr& c) { return LC{{0, c}}; }

// FpVar<Fr>: Constant(v) (is_const) or Var(lc, v)
struct FpVar {
  CS* cs = nullptr;
  bool is_const = true;
  LC lc;
  Fr v;
  static FpVar constant(CS* cs, const Fr& v) { return FpVar{cs, true, {}, v}; }
  static FpVar input(CS* cs, const Fr& v) { return FpVar{cs, false, cs->new_input(v), v}; }
  static FpVar witness(CS* cs, const Fr& v) { return FpVar{cs, false, cs->new_witness(v), v}; }
  static FpVar data(CS* cs, const Fr& v) { return FpVar{cs, false, cs->new_data(v), v}; }
  LC term() const { return is_const ? one_lc(v) : lc; }
  FpVar operator+(const FpVar& o) const {
    if (is_const && o.is_const) return constant(cs, v + o.v);
    return FpVar{cs, false, lc_add(term(), o.term()), v + o.v};
  }
  FpVar operator+(const Fr& c) const { return *this + constant(cs, c); }
  FpVar operator-(const FpVar& o) const {
    if (is_const && o.is_const) return constant(cs, v - o.v);
    return FpVar{cs, false, lc_add(term(), o.term(), true), v - o.v};
  }
  FpVar scale(const Fr& c) const {
    if (is_const) return constant(cs, v * c);
    return FpVar{cs, false, lc_scale(lc, c), v * c};
  }
  FpVar mul(const FpVar& o) const {
    if (is_const) return o.scale(v);
    if (o.is_const) return scale(o.v);
    FpVar p = witness(cs, v * o.v);
    cs->op(WP_MUL, p.lc[0].first, {lc, o.lc});
    cs->enforce(lc, o.lc, p.lc);
    return p;
  }
  FpVar square() const {
    if (is_const) return constant(cs, v * v);
    FpVar p = witness(cs, v * v);
    cs->op(WP_MUL, p.lc[0].first, {lc, lc});
    cs->enforce(lc, lc, p.lc);
    return p;
  }
  FpVar pow_by_constant(uint64_t e) const {  // FieldVar::pow_by_constant
    FpVar res = constant(cs, Fr::one());
    int top = 63;
    while (top > 0 && !((e >> top) & 1)) top--;
    for (int b = top; b >= 0; b--) {
      res = res.square();
      if ((e >> b) & 1) res = res.mul(*this);
    }
    return res;
  }
  void enforce_equal(const FpVar& o) const {  // (x - y) * 1 = 0, constant side first
    if (is_const && o.is_const) {
      if (v != o.v) throw std::runtime_error("enforce_equal on unequal constants");
      return;
    }
    const FpVar& x = (o.is_const && !is_const) ? o : *this;
    const FpVar& y = (o.is_const && !is_const) ? *this : o;
    cs->enforce(lc_add(x.term(), y.term(), true), one_lc(Fr::one()), LC{});
  }
};

struct Boolean {
  CS* cs = nullptr;
  bool is_const = true;
  LC lc;
  bool v = false;
  LC term() const { return is_const ? (v ? one_lc(Fr::one()) : LC{}) : lc; }
  static Boolean constant(CS* cs, bool v) { return Boolean{cs, true, {}, v}; }
  static Boolean witness(CS* cs, bool v) {
    LC b = cs->new_witness(Fr::from_u64(v));
    cs->enforce(lc_add(one_lc(Fr::one()), b, true), b, LC{});  // (1 - b) * b = 0
    return Boolean{cs, false, b, v};
  }
  Boolean negate() const {
    if (is_const) return constant(cs, !v);
    return Boolean{cs, false, lc_add(one_lc(Fr::one()), lc, true), !v};
  }
  Boolean and_(const Boolean& o) const {
    if (is_const) return v ? o : *this;
    if (o.is_const) return o.v ? *this : o;
    Boolean r{cs, false, cs->new_witness(Fr::from_u64(v && o.v)), v && o.v};
    cs->op(WP_MUL, r.lc[0].first, {lc, o.lc});
    cs->enforce(lc, o.lc, r.lc);
    return r;
  }
  void enforce_equal_const(bool value) const {
    if (is_const) {
      if (v != value) throw std::runtime_error("unsatisfiable constant boolean equality");
      return;
    }
    cs->enforce(value ? lc_add(one_lc(Fr::one()), lc, true) : lc, one_lc(Fr::one()), LC{});
  }
};

// AllocatedFp(c).is_neq(v): (c - v) * m = ne, (c - v) * (1 - ne) = 0
Boolean is_neq_const(const FpVar& x, const Fr& c) {
  CS* cs = x.cs;
  const Fr d = c - x.v;
  const bool ne = !d.is_zero();
  Boolean nb{cs, false, cs->new_witness(Fr::from_u64(ne)), ne};
  FpVar mult = FpVar::witness(cs, ne ? d.inverse() : Fr::one());
  const LC diff = lc_add(one_lc(c), x.term(), true);
  cs->op(WP_NZ, nb.lc[0].first, {diff});
  cs->op(WP_INV1, mult.lc[0].first, {diff});
  cs->enforce(diff, mult.lc, nb.lc);
  cs->enforce(diff, nb.negate().term(), LC{});
  return nb;
}

Boolean kary_and(const std::vector<Boolean>& bits) {
  if (bits.size() <= 3) {
    Boolean cur = bits[0];
    for (size_t i = 1; i < bits.size(); i++) cur = cur.and_(bits[i]);
    return cur;
  }
  CS* cs = bits[0].cs;
  FpVar total = FpVar::constant(cs, Fr::zero());
  for (const Boolean& b : bits)
    total = total + (b.is_const ? FpVar::constant(cs, Fr::from_u64(b.v)) : FpVar{cs, false, b.lc, Fr::from_u64(b.v)});
  if (total.is_const) return Boolean::constant(cs, total.v == Fr::from_u64(bits.size()));
  return is_neq_const(total, Fr::from_u64(bits.size())).negate();
}

void enforce_kary_nand(const std::vector<Boolean>& bits) {
  Boolean r = kary_and(bits).negate();
  if (r.is_const) {
    if (!r.v) throw std::runtime_error("kary_nand of all-true constants");
    return;
  }
  r.enforce_equal_const(true);
}

// Boolean::enforce_smaller_or_equal_than_le(bits, element) with element < 2^256 (4 limbs)
void enforce_le(const std::vector<Boolean>& bits, const uint64_t el[4]) {
  int nbits = 256;
  while (nbits > 0 && !((el[(nbits - 1) / 64] >> ((nbits - 1) % 64)) & 1)) nbits--;
  size_t pos = 0;  // index into the big-endian bit order
  const size_t nb = bits.size();
  auto be = [&](size_t k) -> const Boolean& { return bits[nb - 1 - k]; };
  if ((int)nb > nbits) {
    if ((int)nb - nbits != 1) throw std::runtime_error("multi-bit OR chain not needed by this circuit");
    bits[nbits].enforce_equal_const(false);  // FALSE | b = b
    pos++;
  }
  Boolean last_run = Boolean::constant(bits[0].cs, true);
  std::vector<Boolean> run;
  for (int i = nbits - 1; i >= 0; i--) {
    const Boolean& a = be(pos++);
    if ((el[i / 64] >> (i % 64)) & 1) {
      run.push_back(a);
    } else {
      if (!run.empty()) {
        run.push_back(last_run);
        last_run = kary_and(run);
        run.clear();
      }
      enforce_kary_nand({last_run, a});
    }
  }
}

std::vector<Boolean> to_non_unique_bits_le(const FpVar& x) {
  CS* cs = x.cs;
  std::vector<Boolean> bits;
  cs->op(WP_BITS, cs->next_witness(), {x.term()}, kModulusBits);
  cs->mute++;
  for (int i = 0; i < kModulusBits; i++) bits.push_back(Boolean::witness(cs, x.v.bit(i)));
  cs->mute--;
  LC packed;
  Fr coeff = Fr::one();
  for (const Boolean& b : bits) {
    packed = lc_add(packed, lc_scale(b.lc, coeff));
    coeff = coeff + coeff;
  }
  cs->enforce(LC{}, LC{}, lc_add(packed, x.term(), true));
  return bits;
}

const uint64_t kHalf[4] = {0xa1f0fac9f8000000ULL, 0x9419f4243cdcb848ULL, 0xdc2822db40c0ac2eULL,
                           0x183227397098d014ULL};  // (r - 1) / 2
const uint64_t kRm1[4] = {0x43e1f593f0000000ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                          0x30644e72e131a029ULL};  // r - 1

void enforce_cmp_greater_eq(const FpVar& self, const FpVar& other) {
  // enforce_cmp(other, Greater, true): other < self + 1, both <= (r-1)/2
  const FpVar left = other, right = self + Fr::one();
  enforce_le(to_non_unique_bits_le(left), kHalf);
  enforce_le(to_non_unique_bits_le(right), kHalf);
  std::vector<Boolean> bits = to_non_unique_bits_le((left - right).scale(Fr::from_u64(2)));
  enforce_le(bits, kRm1);  // to_bits_le = non-unique bits + enforce_in_field_le
  self.cs->enforce(bits[0].term(), one_lc(Fr::one()), one_lc(Fr::one()));
}

// PoseidonSpongeVar (duplex; values double as the native sponge)
struct Sponge {
  CS* cs;
  const PoseidonParams& p;
  std::vector<FpVar> st;
  bool absorbing = true;
  int idx = 0;
  explicit Sponge(CS* c) : cs(c), p(poseidon_params()) {
    for (int i = 0; i < 3; i++) st.push_back(FpVar::constant(cs, Fr::zero()));
  }
  void permute() {
    const int half = p.full / 2;
    // one POSEIDON op: the three state combinations in, the S-box trace
    // (x^2, x^4, x^5 per S-box, round order) out; round 0 skips constant
    // elements (their powers are constants, no witnesses)
    uint32_t mask = 0;
    for (int i = 0; i < 3; i++)
      if (!st[i].is_const) mask |= 1u << i;
    const uint64_t first = cs->next_witness();
    if (mask) cs->op(WP_POSEIDON, first, {st[0].term(), st[1].term(), st[2].term()}, mask);
    cs->mute++;
    for (int rnd = 0; rnd < p.full + p.partial; rnd++) {
      for (int i = 0; i < 3; i++) st[i] = st[i] + p.ark[rnd][i];
      if (rnd < half || rnd >= half + p.partial) {
        for (int i = 0; i < 3; i++) st[i] = st[i].pow_by_constant(p.alpha);
      } else {
        st[0] = st[0].pow_by_constant(p.alpha);
      }
      std::vector<FpVar> nw;
      for (int i = 0; i < 3; i++) {
        FpVar cur = FpVar::constant(cs, Fr::zero());
        for (int j = 0; j < 3; j++) cur = cur + st[j].scale(p.mds[i][j]);
        nw.push_back(cur);
      }
      st = nw;
    }
    cs->mute--;
    const uint64_t trace = cs->next_witness() - first;
    if (trace != (mask ? 3 * (uint64_t)__builtin_popcount(mask) + 231 : 0))
      throw std::logic_error("Poseidon trace length differs from the POSEIDON op's");
  }
  void absorb_internal(int start, std::vector<FpVar> el) {
    for (;;) {
      if (start + (int)el.size() <= p.rate) {
        for (size_t i = 0; i < el.size(); i++) st[p.capacity + i + start] = st[p.capacity + i + start] + el[i];
        absorbing = true;
        idx = start + (int)el.size();
        return;
      }
      const int k = p.rate - start;
      for (int i = 0; i < k; i++) st[p.capacity + i + start] = st[p.capacity + i + start] + el[i];
      permute();
      el.erase(el.begin(), el.begin() + k);
      start = 0;
    }
  }
  void absorb(const std::vector<FpVar>& el) {
    if (el.empty()) return;
    if (absorbing) {
      int start = idx;
      if (start == p.rate) {
        permute();
        start = 0;
      }
      absorb_internal(start, el);
    } else {
      permute();
      absorb_internal(0, el);
    }
  }
  FpVar squeeze1() {
    int start = 0;
    if (absorbing) {
      permute();
    } else {
      start = idx;
      if (start == p.rate) {
        permute();
        start = 0;
      }
    }
    FpVar out = st[p.capacity + start];
    absorbing = false;
    idx = start + 1;
    return out;
  }
};

Fr fr_le(const Bytes32& b) { return Fr::from_le_bytes_mod_order(b.data(), 32); }
Fr fr_str(const char* s) { return Fr::from_le_bytes_mod_order((const uint8_t*)s, strlen(s)); }

}  // namespace

Fr poseidon_hash(const std::vector<Fr>& xs) {
  CS cs;
  Sponge sp(&cs);
  std::vector<FpVar> el;
  for (const Fr& x : xs) el.push_back(FpVar::constant(&cs, x));
  sp.absorb(el);
  return sp.squeeze1().v;
}

L2BlockCircuit L2BlockCircuit::dummy() {
  L2BlockCircuit c;
  Bytes32 a, b;
  a.fill(1);
  b.fill(2);
  c.transactions.push_back({a, b, 100});
  c.initial_accounts[a] = 1000;
  c.initial_accounts[b] = 0;
  return c;
}

namespace {
void build_program(const CS& cs, L2WitnessProgram& P);
}  // namespace

R1CSMatrices L2BlockCircuit::synthesize(std::map<std::string, Fr>* computed, L2WitnessProgram* prog) const {
  CS cs;
  CS* C = &cs;
  cs.record = prog != nullptr;
  auto sponge = [&](const std::vector<FpVar>& el) {
    Sponge sp(C);
    sp.absorb(el);
    return sp.squeeze1();
  };
  FpVar pre_state = FpVar::input(C, fr_le(pre_state_root));
  FpVar post_state = FpVar::input(C, fr_le(post_state_root));
  FpVar pre_shielded = FpVar::input(C, fr_le(pre_shielded_root));
  FpVar post_shielded = FpVar::input(C, fr_le(post_shielded_root));
  FpVar wd_root = FpVar::input(C, fr_le(withdrawal_root));
  FpVar bh = FpVar::input(C, fr_le(batch_hash));
  FpVar bid = FpVar::input(C, Fr::from_u64(batch_id));
  std::map<std::string, Fr> out;

  std::map<Bytes32, FpVar> accounts;
  for (const auto& kv : initial_accounts) accounts[kv.first] = FpVar::data(C, Fr::from_u64(kv.second));
  std::map<Bytes32, FpVar> current = accounts;
  for (const auto& tx : transactions) {
    FpVar amount = FpVar::data(C, Fr::from_u64(tx.amount));
    auto it = current.find(tx.sender_pk);
    if (it == current.end()) throw std::runtime_error("SynthesisError::AssignmentMissing: sender not in initial_accounts");
    FpVar sender = it->second;
    auto rit = current.find(tx.recipient_pk);
    FpVar recipient = rit == current.end() ? FpVar::constant(C, Fr::zero()) : rit->second;
    enforce_cmp_greater_eq(sender, amount);
    current[tx.sender_pk] = sender - amount;
    current[tx.recipient_pk] = recipient + amount;
  }
  const FpVar ds = FpVar::constant(C, fr_str("zelana:accounts-fold:v1"));
  auto fold_accounts = [&](const std::map<Bytes32, FpVar>& accts) {
    FpVar st = sponge({ds, bid});
    for (const auto& kv : accts) {
      FpVar pk = FpVar::data(C, fr_le(kv.first));
      FpVar leaf = sponge({pk, kv.second});
      st = sponge({st, leaf});
    }
    FpVar count = FpVar::data(C, Fr::from_u64(accts.size()));
    return sponge({st, count});
  };
  FpVar computed_post = fold_accounts(current);
  out["post_state_root"] = computed_post.v;
  computed_post.enforce_equal(post_state);

  FpVar sh = sponge({pre_shielded});
  for (const auto& cm : shielded_commitments) {
    FpVar cmv = FpVar::data(C, fr_le(cm));
    sh = sponge({sh, cmv});
  }
  if (shielded_commitments.empty()) {
    out["post_shielded_root"] = pre_shielded.v;
    pre_shielded.enforce_equal(post_shielded);
  } else {
    out["post_shielded_root"] = sh.v;
    sh.enforce_equal(post_shielded);
  }

  FpVar wd = sponge({FpVar::constant(C, fr_str("zelana:withdrawals:v1"))});
  for (const auto& w : withdrawals) {
    FpVar rcp = FpVar::data(C, fr_le(w.recipient));
    FpVar amt = FpVar::data(C, Fr::from_u64(w.amount));
    FpVar leaf = sponge({rcp, amt});
    wd = sponge({wd, leaf});
  }
  FpVar wd_count = FpVar::data(C, Fr::from_u64(withdrawals.size()));
  FpVar computed_wd = sponge({wd, wd_count});
  out["withdrawal_root"] = computed_wd.v;
  computed_wd.enforce_equal(wd_root);

  FpVar bst = sponge({FpVar::constant(C, fr_str("zelana:batch-hash:v1")), bid});
  for (const auto& tx : transactions) {
    FpVar s = FpVar::data(C, fr_le(tx.sender_pk));
    FpVar r = FpVar::data(C, fr_le(tx.recipient_pk));
    FpVar a = FpVar::data(C, Fr::from_u64(tx.amount));
    FpVar txh = sponge({s, r, a});
    bst = sponge({bst, txh});
  }
  FpVar tx_count = FpVar::data(C, Fr::from_u64(transactions.size()));
  FpVar computed_bh = sponge({bst, tx_count});
  out["batch_hash"] = computed_bh.v;
  computed_bh.enforce_equal(bh);

  FpVar computed_pre = fold_accounts(accounts);
  out["pre_state_root"] = computed_pre.v;
  computed_pre.enforce_equal(pre_state);
  if (computed) *computed = out;

  // to CSR: instance k -> k, witness k -> num_instance + k
  R1CSMatrices M;
  M.num_constraints = cs.rows.size();
  M.num_instance = cs.inst.size();
  M.num_witness = cs.wit.size();
  const uint64_t ni = M.num_instance;
  for (int t = 0; t < 3; t++) {
    M.rowptr[t].push_back(0);
    for (const auto& row : cs.rows) {
      for (const auto& kv : row[t]) {
        if (kv.second.is_zero()) continue;
        M.col[t].push_back(kv.first >= kWit ? ni + (kv.first - kWit) : kv.first);
        uint64_t c[4];
        kv.second.to_canon(c);
        M.val[t].insert(M.val[t].end(), c, c + 4);
      }
      M.rowptr[t].push_back(M.col[t].size());
    }
  }
  for (const Fr& v : cs.inst) {
    uint64_t c[4];
    v.to_canon(c);
    M.z.insert(M.z.end(), c, c + 4);
  }
  for (const Fr& v : cs.wit) {
    uint64_t c[4];
    v.to_canon(c);
    M.z.insert(M.z.end(), c, c + 4);
  }
  if (prog) build_program(cs, *prog);
  return M;
}

// ------------------------------------------------------- witness programs
namespace {

uint64_t op_span(uint32_t kind, uint32_t aux) {
  switch (kind) {
    case WP_MUL: return 1;
    case WP_BITS: return aux;
    case WP_POSEIDON: return 3 * (uint64_t)__builtin_popcount(aux) + 231;
    default: return 1;
  }
}

// The recorded ops scheduled into launch levels, as zelana_amd/wprog.py's
// Plan does for zelana_batch: a permutation costs ~1000x a MUL, so the key is
// (permutation stage, cheap sub-level) and every permutation runs at its
// chain's permutation depth.
void build_program(const CS& cs, L2WitnessProgram& P) {
  const uint64_t ni = cs.inst.size(), nv = ni + cs.wit.size();
  if (nv >= (1ULL << 31)) throw std::runtime_error("witness program: too many variables");
  auto zidx = [&](uint64_t sym) { return (uint32_t)(sym >= kWit ? ni + (sym - kWit) : sym); };
  P = L2WitnessProgram();
  P.num_vars = nv;
  P.num_instance = ni;
  std::map<std::array<uint64_t, 4>, uint32_t> cid;
  auto push_coeff = [&](const Fr& c, bool dedupe) {
    std::array<uint64_t, 4> k;
    c.to_canon(k.data());
    if (dedupe) {
      auto it = cid.find(k);
      if (it != cid.end()) return it->second;
    }
    const uint32_t id = (uint32_t)(P.coeff.size() / 4);
    cid.emplace(k, id);
    P.coeff.insert(P.coeff.end(), k.begin(), k.end());
    return id;
  };
  const PoseidonParams& pp = poseidon_params();  // ids 3r + i, then 192 + 3i + j (zkmi.h)
  for (int r = 0; r < 64; r++)
    for (int i = 0; i < 3; i++) push_coeff(pp.ark[r][i], false);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) push_coeff(pp.mds[i][j], false);

  std::vector<uint8_t> produced(nv, 0);
  for (uint64_t sym : cs.in_syms) {
    const uint32_t v = zidx(sym);
    if (produced[v]) throw std::logic_error("witness program: input allocated twice");
    produced[v] = 1;
    P.input_var.push_back(v);
    const Fr& val = sym >= kWit ? cs.wit[sym - kWit] : cs.inst[sym];
    uint64_t c[4];
    val.to_canon(c);
    P.template_inputs.insert(P.template_inputs.end(), c, c + 4);
  }
  constexpr uint64_t BIG = 0xFFFFFFFFULL;
  std::vector<uint32_t> pstage(nv, 0), sub(nv, 0);
  struct Sched {
    uint64_t key;
    bool pos;
    size_t i;
  };
  std::vector<Sched> order;
  for (size_t i = 0; i < cs.ops.size(); i++) {
    const CS::Rec& o = cs.ops[i];
    uint32_t s_in = 0;
    for (const LC& lc : o.lcs)
      for (const auto& t : lc)
        if (!t.second.is_zero() && t.first) s_in = std::max(s_in, pstage[zidx(t.first)]);
    const uint64_t span = op_span(o.kind, o.aux), out = zidx(o.out);
    if (out + span > nv) throw std::logic_error("witness program: op output outside z");
    uint32_t st, sl;
    uint64_t key;
    if (o.kind == WP_POSEIDON) {
      st = s_in + 1, sl = 0;
      key = ((uint64_t)s_in << 32) | BIG;
    } else {
      sl = 0;
      for (const LC& lc : o.lcs)
        for (const auto& t : lc)
          if (!t.second.is_zero() && t.first && pstage[zidx(t.first)] == s_in) sl = std::max(sl, sub[zidx(t.first)]);
      st = s_in, sl += 1;
      key = ((uint64_t)s_in << 32) | sl;
    }
    for (uint64_t v = out; v < out + span; v++) {
      if (produced[v]) throw std::logic_error("witness program: variable written twice");
      produced[v] = 1;
      pstage[v] = st;
      sub[v] = sl;
    }
    order.push_back({key, o.kind == WP_POSEIDON, i});
  }
  for (uint64_t v = 0; v < nv; v++)
    if (!produced[v]) throw std::logic_error("witness program: variable neither input nor op output");
  // Inversions nothing reads (is_neq's multipliers, constraint-only) run in
  // the last launch, beside the permutations, instead of lengthening the
  // comparison chains they hang off (each is a ~250-squaring exponentiation).
  std::vector<uint8_t> read(nv, 0);
  uint64_t last = 0;
  for (size_t i = 0; i < cs.ops.size(); i++) {
    for (const LC& lc : cs.ops[i].lcs)
      for (const auto& t : lc)
        if (!t.second.is_zero()) read[zidx(t.first)] = 1;
    last = std::max(last, order[i].key);
  }
  for (size_t i = 0; i < cs.ops.size(); i++)
    if ((cs.ops[i].kind == WP_INV1 || cs.ops[i].kind == WP_INV) && !read[zidx(cs.ops[i].out)]) {
      order[i].key = last;
      order[i].pos = false;
    }
  // within a level: permutations first (the quads of one wave share a kind)
  std::stable_sort(order.begin(), order.end(), [](const Sched& a, const Sched& b) {
    return a.key != b.key ? a.key < b.key : (a.pos && !b.pos);
  });
  auto emit = [&](const LC& lc) {
    uint32_t n = 0;
    for (const auto& t : lc) {
      if (t.second.is_zero()) continue;
      P.term.push_back(zidx(t.first));
      P.term.push_back(push_coeff(t.second, true));
      n++;
    }
    if (n >= 4096) throw std::runtime_error("witness program: linear combination over 4095 terms");
    return n;
  };
  for (size_t k = 0; k < order.size(); k++) {
    if (k == 0 || order[k].key != order[k - 1].key) P.level_start.push_back((uint32_t)k);
    const CS::Rec& o = cs.ops[order[k].i];
    const uint32_t aoff = (uint32_t)(P.term.size() / 2);
    uint32_t w[4] = {o.kind, zidx(o.out), aoff, 0};
    if (o.kind == WP_MUL) {
      const uint32_t la = emit(o.lcs[0]);
      w[3] = (uint32_t)(P.term.size() / 2);
      const uint32_t lb = emit(o.lcs[1]);
      w[0] |= la << 8 | lb << 20;
    } else if (o.kind == WP_POSEIDON) {
      const uint32_t l0 = emit(o.lcs[0]), l1 = emit(o.lcs[1]), l2 = emit(o.lcs[2]);
      w[0] |= l0 << 8 | l1 << 20;
      w[3] = l2 | o.aux << 16;
    } else {
      w[0] |= emit(o.lcs[0]) << 8;
      w[3] = o.kind == WP_BITS ? o.aux : 0;
    }
    P.op.insert(P.op.end(), w, w + 4);
  }
  P.level_start.push_back((uint32_t)order.size());
}

}  // namespace

std::vector<uint64_t> L2WitnessProgram::interpret(const std::vector<uint64_t>& inputs) const {
  if (inputs.size() != input_var.size() * 4) throw std::invalid_argument("witness program: input count");
  std::vector<Fr> z(num_vars), co(coeff.size() / 4);
  for (size_t k = 0; k < input_var.size(); k++) z[input_var[k]] = Fr::from_canon(&inputs[4 * k]);
  for (size_t k = 0; k < co.size(); k++) co[k] = Fr::from_canon(&coeff[4 * k]);
  auto ev = [&](uint32_t off, uint32_t n) {
    Fr s;
    for (uint32_t k = off; k < off + n; k++) s = s + co[term[2 * k + 1]] * z[term[2 * k]];
    return s;
  };
  for (size_t i = 0; i < op.size() / 4; i++) {
    const uint32_t* o = &op[4 * i];
    const uint32_t kind = o[0] & 0xFF, la = (o[0] >> 8) & 0xFFF, lb = o[0] >> 20, out = o[1];
    if (kind == WP_MUL) {
      z[out] = ev(o[2], la) * ev(o[3], lb);
    } else if (kind == WP_BITS) {
      const Fr a = ev(o[2], la);
      for (uint32_t b = 0; b < o[3]; b++) z[out + b] = Fr::from_u64(a.bit((int)b));
    } else if (kind == WP_NZ) {
      z[out] = Fr::from_u64(!ev(o[2], la).is_zero());
    } else if (kind == WP_INV1 || kind == WP_INV) {
      const Fr a = ev(o[2], la);
      z[out] = a.is_zero() ? (kind == WP_INV1 ? Fr::one() : Fr()) : a.inverse();
    } else if (kind == WP_POSEIDON) {
      const uint32_t l2 = o[3] & 0xFFFF, mask = o[3] >> 16;
      Fr st[3] = {ev(o[2], la), ev(o[2] + la, lb), ev(o[2] + la + lb, l2)};
      uint32_t t = out;
      for (int r = 0; r < 64; r++) {
        for (int j = 0; j < 3; j++) st[j] = st[j] + co[3 * r + j];
        const bool full = r < 4 || r >= 60;
        for (int j = 0; j < (full ? 3 : 1); j++) {
          const Fr x2 = st[j] * st[j], x4 = x2 * x2, x5 = x4 * st[j];
          if (r > 0 || ((mask >> j) & 1)) {
            z[t++] = x2;
            z[t++] = x4;
            z[t++] = x5;
          }
          st[j] = x5;
        }
        Fr nw[3];
        for (int j = 0; j < 3; j++) nw[j] = co[192 + 3 * j] * st[0] + co[192 + 3 * j + 1] * st[1] + co[192 + 3 * j + 2] * st[2];
        for (int j = 0; j < 3; j++) st[j] = nw[j];
      }
    } else {
      throw std::invalid_argument("witness program: unknown op kind");
    }
  }
  std::vector<uint64_t> zc(4 * num_vars);
  for (uint64_t v = 0; v < num_vars; v++) z[v].to_canon(&zc[4 * v]);
  return zc;
}

std::string L2BlockCircuit::shape_key() const {
  std::map<Bytes32, uint32_t> rank;
  for (const auto& kv : initial_accounts) rank[kv.first] = 0;
  for (const auto& tx : transactions) rank[tx.sender_pk] = rank[tx.recipient_pk] = 0;
  uint32_t k = 0;
  for (auto& kv : rank) kv.second = k++;
  std::string s = "t" + std::to_string(transactions.size()) + "a" + std::to_string(initial_accounts.size()) + "k" +
                  std::to_string(rank.size()) + "s" + std::to_string(shielded_commitments.size()) + "w" +
                  std::to_string(withdrawals.size()) + ":";
  std::set<Bytes32> cur;
  for (const auto& kv : initial_accounts) {
    cur.insert(kv.first);
    s += std::to_string(rank[kv.first]) + ",";
  }
  s += ":";
  for (const auto& tx : transactions) {
    if (!cur.count(tx.sender_pk))
      throw std::runtime_error("SynthesisError::AssignmentMissing: sender not in initial_accounts");
    s += std::to_string(rank[tx.sender_pk]) + ">" + std::to_string(rank[tx.recipient_pk]) +
         (cur.count(tx.recipient_pk) ? "," : "+,");
    cur.insert(tx.recipient_pk);
  }
  return s;
}

std::vector<uint64_t> L2BlockCircuit::witness_inputs() const {
  // synthesize()'s allocation order of FpVar::input / FpVar::data
  std::vector<uint64_t> out;
  auto put = [&](const Fr& v) {
    uint64_t c[4];
    v.to_canon(c);
    out.insert(out.end(), c, c + 4);
  };
  put(Fr::one());
  for (const Bytes32* r : {&pre_state_root, &post_state_root, &pre_shielded_root, &post_shielded_root,
                           &withdrawal_root, &batch_hash})
    put(fr_le(*r));
  put(Fr::from_u64(batch_id));
  std::set<Bytes32> current;
  for (const auto& kv : initial_accounts) {
    put(Fr::from_u64(kv.second));
    current.insert(kv.first);
  }
  for (const auto& tx : transactions) {
    put(Fr::from_u64(tx.amount));
    if (!current.count(tx.sender_pk))
      throw std::runtime_error("SynthesisError::AssignmentMissing: sender not in initial_accounts");
    current.insert(tx.recipient_pk);
  }
  auto fold = [&](const std::set<Bytes32>& keys) {
    for (const Bytes32& pk : keys) put(fr_le(pk));
    put(Fr::from_u64(keys.size()));
  };
  fold(current);
  for (const auto& cm : shielded_commitments) put(fr_le(cm));
  for (const auto& w : withdrawals) {
    put(fr_le(w.recipient));
    put(Fr::from_u64(w.amount));
  }
  put(Fr::from_u64(withdrawals.size()));
  for (const auto& tx : transactions) {
    put(fr_le(tx.sender_pk));
    put(fr_le(tx.recipient_pk));
    put(Fr::from_u64(tx.amount));
  }
  put(Fr::from_u64(transactions.size()));
  std::set<Bytes32> initial;
  for (const auto& kv : initial_accounts) initial.insert(kv.first);
  fold(initial);
  return out;
}

bool R1CSMatrices::is_satisfied() const {
  const size_t nv = num_instance + num_witness;
  std::vector<Fr> zz(nv);
  for (size_t i = 0; i < nv; i++) zz[i] = Fr::from_canon(&z[4 * i]);
  for (size_t r = 0; r < num_constraints; r++) {
    Fr e[3];
    for (int t = 0; t < 3; t++)
      for (uint64_t k = rowptr[t][r]; k < rowptr[t][r + 1]; k++) e[t] = e[t] + Fr::from_canon(&val[t][4 * k]) * zz[col[t][k]];
    if (e[0] * e[1] != e[2]) return false;
  }
  return true;
}

}  // namespace zp
