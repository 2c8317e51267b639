// l2_circuit.cpp — see l2_circuit.h.  A line-for-line restatement of
// zelana_amd/l2block.py (itself following prover/src/l2_circuit.rs and the
// arkworks 0.5 gadgets) so the C++ host mirror needs no Python.
#include "l2_circuit.h"

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

struct CS {
  std::vector<Fr> inst{Fr::one()}, wit;
  std::vector<std::array<LC, 3>> rows;
  LC new_input(const Fr& v) {
    inst.push_back(v);
    return LC{{inst.size() - 1, Fr::one()}};
  }
  LC new_witness(const Fr& v) {
    wit.push_back(v);
    return LC{{kWit + wit.size() - 1, Fr::one()}};
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
    cs->enforce(lc, o.lc, p.lc);
    return p;
  }
  FpVar square() const {
    if (is_const) return constant(cs, v * v);
    FpVar p = witness(cs, v * v);
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
  for (int i = 0; i < kModulusBits; i++) bits.push_back(Boolean::witness(cs, x.v.bit(i)));
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

R1CSMatrices L2BlockCircuit::synthesize(std::map<std::string, Fr>* computed) const {
  CS cs;
  CS* C = &cs;
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
  for (const auto& kv : initial_accounts) accounts[kv.first] = FpVar::witness(C, Fr::from_u64(kv.second));
  std::map<Bytes32, FpVar> current = accounts;
  for (const auto& tx : transactions) {
    FpVar amount = FpVar::witness(C, Fr::from_u64(tx.amount));
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
      FpVar pk = FpVar::witness(C, fr_le(kv.first));
      FpVar leaf = sponge({pk, kv.second});
      st = sponge({st, leaf});
    }
    FpVar count = FpVar::witness(C, Fr::from_u64(accts.size()));
    return sponge({st, count});
  };
  FpVar computed_post = fold_accounts(current);
  out["post_state_root"] = computed_post.v;
  computed_post.enforce_equal(post_state);

  FpVar sh = sponge({pre_shielded});
  for (const auto& cm : shielded_commitments) {
    FpVar cmv = FpVar::witness(C, fr_le(cm));
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
    FpVar rcp = FpVar::witness(C, fr_le(w.recipient));
    FpVar amt = FpVar::witness(C, Fr::from_u64(w.amount));
    FpVar leaf = sponge({rcp, amt});
    wd = sponge({wd, leaf});
  }
  FpVar wd_count = FpVar::witness(C, Fr::from_u64(withdrawals.size()));
  FpVar computed_wd = sponge({wd, wd_count});
  out["withdrawal_root"] = computed_wd.v;
  computed_wd.enforce_equal(wd_root);

  FpVar bst = sponge({FpVar::constant(C, fr_str("zelana:batch-hash:v1")), bid});
  for (const auto& tx : transactions) {
    FpVar s = FpVar::witness(C, fr_le(tx.sender_pk));
    FpVar r = FpVar::witness(C, fr_le(tx.recipient_pk));
    FpVar a = FpVar::witness(C, Fr::from_u64(tx.amount));
    FpVar txh = sponge({s, r, a});
    bst = sponge({bst, txh});
  }
  FpVar tx_count = FpVar::witness(C, Fr::from_u64(transactions.size()));
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
  return M;
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
