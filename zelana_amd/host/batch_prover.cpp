// batch_prover.cpp — see batch_prover.h.
#include "batch_prover.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <iterator>
#include <thread>

#include "../../include/zkmi.h"
#include "blake3.h"
#include "std_rng.h"

namespace zp {

namespace {
[[noreturn]] void fail(const std::string& what) {
  throw std::runtime_error(what + ": " + zkmi_last_error());
}
void check(int rc, const char* what) {
  if (rc != 0) fail(what);
}
template <class T>
void le_bytes(Blake3& h, T v) {
  uint8_t b[sizeof(T)];
  for (size_t i = 0; i < sizeof(T); i++) b[i] = (uint8_t)(v >> (8 * i));
  h.update(b, sizeof(T));
}
}  // namespace

// ---------------------------------------------------------------- MockProver
MockProver::MockProver(uint64_t prove_time_ms) : prove_time_ms_(prove_time_ms) {
  static const char tag[] = "zelana-mock-vk-v1";
  vk_hash_ = Blake3::hash(tag, sizeof(tag) - 1);
}

BatchProof MockProver::prove(const BatchPublicInputs& in, const BatchWitness&) const {
  std::this_thread::sleep_for(std::chrono::milliseconds(prove_time_ms_));
  Blake3 h;  // mock proof = hash of the public inputs, padded to 256 B (prover.rs:210-233)
  for (const Bytes32* r : {&in.pre_state_root, &in.post_state_root, &in.pre_shielded_root, &in.post_shielded_root,
                           &in.withdrawal_root, &in.batch_hash})
    h.update(r->data(), 32);
  le_bytes(h, in.batch_id);
  BatchProof p;
  p.public_inputs = in;
  auto d = h.finalize();
  p.proof_bytes.assign(d.begin(), d.end());
  p.proof_bytes.resize(256, 0);
  p.proving_time_ms = prove_time_ms_;
  return p;
}

// ------------------------------------------------------------- Groth16Prover
std::unique_ptr<Groth16Prover> Groth16Prover::from_bytes(const std::vector<uint8_t>& pk_bytes,
                                                         const std::vector<uint8_t>& vk_bytes, int device) {
  std::unique_ptr<Groth16Prover> p(new Groth16Prover());
  check(zkmi_ctx_create(device, &p->ctx_), "Failed to open the GPU");
  if (zkmi_pk_load(p->ctx_, pk_bytes.data(), pk_bytes.size(), 1, &p->pk_) != 0)
    fail("Failed to deserialize proving key");
  size_t len = 0;
  if (zkmi_vk_canonical(p->ctx_, vk_bytes.data(), vk_bytes.size(), nullptr, 0, &len) != 0)
    fail("Failed to deserialize verifying key");
  p->vk_.resize(len);
  check(zkmi_vk_canonical(p->ctx_, vk_bytes.data(), vk_bytes.size(), p->vk_.data(), len, &len),
        "Failed to serialize VK");
  p->vk_hash_ = Blake3::hash(p->vk_.data(), p->vk_.size());  // compute_vk_hash (:289-294)
  // fixed-base tables: one MSM window per query for every later prove
  check(zkmi_pk_precompute(p->pk_, 0), "Failed to precompute proving key tables");
  return p;
}

std::unique_ptr<Groth16Prover> Groth16Prover::from_files(const std::string& pk_path, const std::string& vk_path,
                                                         int device) {
  auto read = [](const std::string& path, const char* what) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error(std::string("Failed to read ") + what + " from " + path);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
  };
  return from_bytes(read(pk_path, "proving key"), read(vk_path, "verifying key"), device);
}

Groth16Prover::~Groth16Prover() {
  shapes_.clear();  // before the context
  if (pk_) zkmi_pk_destroy(pk_);
  if (ctx_) zkmi_ctx_destroy(ctx_);
}

L2BlockCircuit Groth16Prover::circuit_of(const BatchPublicInputs& in, const BatchWitness& w) {
  L2BlockCircuit c;
  c.pre_state_root = in.pre_state_root;
  c.post_state_root = in.post_state_root;
  c.pre_shielded_root = in.pre_shielded_root;
  c.post_shielded_root = in.post_shielded_root;
  c.withdrawal_root = in.withdrawal_root;
  c.batch_hash = in.batch_hash;
  c.batch_id = in.batch_id;
  for (const auto& tx : w.transactions) {
    if (auto* t = std::get_if<TransferTx>(&tx)) c.transactions.push_back({t->signer_pubkey, t->to, t->amount});
    if (auto* x = std::get_if<WithdrawTx>(&tx)) c.withdrawals.push_back({x->to_l1_address, x->amount});
  }
  for (const auto& s : w.pre_account_states) c.initial_accounts[s.account_id] = s.balance;
  // shielded_commitments: Some(vec![]) (prover.rs:402, a TODO in the reference)
  return c;
}

// One circuit shape's resident state (see batch_prover.h).
struct Groth16Prover::Shape {
  std::string key;
  zkmi_ctx* ctx = nullptr;
  zkmi_r1cs_dev* cs = nullptr;
  zkmi_wprog* prog = nullptr;
  void* d_z = nullptr;
  ~Shape() {
    if (prog) zkmi_wprog_destroy(prog);
    if (cs) zkmi_r1cs_destroy(cs);
    if (d_z) zkmi_dev_free(ctx, d_z);
  }
};

namespace {
zkmi_r1cs r1cs_view(const R1CSMatrices& m) {
  zkmi_r1cs cs;
  cs.num_constraints = m.num_constraints;
  cs.num_instance = m.num_instance;
  cs.num_witness = m.num_witness;
  const uint64_t** rps[3] = {&cs.a_rowptr, &cs.b_rowptr, &cs.c_rowptr};
  const uint64_t** cols[3] = {&cs.a_col, &cs.b_col, &cs.c_col};
  const uint64_t** vals[3] = {&cs.a_val, &cs.b_val, &cs.c_val};
  for (int t = 0; t < 3; t++) {
    *rps[t] = m.rowptr[t].data();
    *cols[t] = m.col[t].data();
    *vals[t] = m.val[t].data();
  }
  return cs;
}
bool host_synthesis_forced() {
  const char* e = getenv("ZP_HOST_SYNTH");  // A/B switch: the round-2 per-call host synthesis
  return e && e[0] == '1';
}
}  // namespace

BatchProof Groth16Prover::prove(const BatchPublicInputs& inputs, const BatchWitness& witness) const {
  const auto start = std::chrono::steady_clock::now();
  const L2BlockCircuit circuit = circuit_of(inputs, witness);
  if (host_synthesis_forced()) return prove_host(inputs, circuit);
  StdRng rng = StdRng::seed_from_u64(inputs.batch_id);  // prover.rs:354
  // Groth16::prove: r = Fr::rand, then s = Fr::rand
  uint64_t r[4], s[4];
  rng.fr_rand().to_canon(r);
  rng.fr_rand().to_canon(s);
  const std::string key = circuit.shape_key();  // throws synthesize's errors
  uint64_t a[8], b[16], c[8];
  {
    std::lock_guard<std::mutex> lock(gpu_mu_);
    size_t hit = shapes_.size();
    for (size_t i = 0; i < shapes_.size(); i++)
      if (shapes_[i]->key == key) hit = i;
    std::vector<uint64_t> in;
    if (hit == shapes_.size()) {
      // first batch of this shape: synthesize once, recording its program
      L2WitnessProgram prog;
      const R1CSMatrices m = circuit.synthesize(nullptr, &prog);
      std::unique_ptr<Shape> sh(new Shape());
      sh->key = key;
      sh->ctx = ctx_;
      const zkmi_r1cs view = r1cs_view(m);
      check(zkmi_r1cs_create(ctx_, &view, &sh->cs), "Failed to upload the circuit");
      zkmi_wprog_desc d;
      d.num_vars = prog.num_vars;
      d.num_inputs = prog.input_var.size();
      d.input_var = prog.input_var.data();
      d.num_ops = prog.op.size() / 4;
      d.op = prog.op.data();
      d.num_terms = prog.term.size() / 2;
      d.term = prog.term.data();
      d.num_coeffs = prog.coeff.size() / 4;
      d.coeff = prog.coeff.data();
      d.num_levels = prog.num_levels();
      d.level_start = prog.level_start.data();
      check(zkmi_wprog_create(ctx_, &d, &sh->prog), "Failed to load the witness program");
      check(zkmi_dev_alloc(ctx_, prog.num_vars * 32, &sh->d_z), "Failed to allocate the assignment");
      in = std::move(prog.template_inputs);
      if (shapes_.size() == kMaxShapes) shapes_.pop_back();
      shapes_.insert(shapes_.begin(), std::move(sh));
    } else {
      in = circuit.witness_inputs();
      std::rotate(shapes_.begin(), shapes_.begin() + hit, shapes_.begin() + hit + 1);
    }
    const Shape& sh = *shapes_.front();
    check(zkmi_wprog_run(ctx_, sh.prog, in.data(), sh.d_z, 0), "Witness generation failed");
    if (zkmi_groth16_prove_resident(ctx_, pk_, sh.cs, sh.d_z, r, s, a, b, c) != 0) fail("Proving failed");
  }
  BatchProof p;
  p.public_inputs = inputs;
  p.proof_bytes = proof_to_solana_bytes(a, b, c);
  p.proving_time_ms =
      (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - start).count();
  return p;
}

// Round-2 path (ZP_HOST_SYNTH=1): full host synthesis per call, R1CS and z uploaded
BatchProof Groth16Prover::prove_host(const BatchPublicInputs& inputs, const L2BlockCircuit& circuit) const {
  const auto start = std::chrono::steady_clock::now();
  StdRng rng = StdRng::seed_from_u64(inputs.batch_id);
  const R1CSMatrices m = circuit.synthesize();
  uint64_t r[4], s[4];
  rng.fr_rand().to_canon(r);
  rng.fr_rand().to_canon(s);
  const zkmi_r1cs cs = r1cs_view(m);
  uint64_t a[8], b[16], c[8];
  {
    std::lock_guard<std::mutex> lock(gpu_mu_);  // synthesis above runs unlocked, in parallel
    if (zkmi_groth16_prove(ctx_, pk_, &cs, m.z.data(), r, s, a, b, c) != 0) fail("Proving failed");
  }
  BatchProof p;
  p.public_inputs = inputs;
  p.proof_bytes = proof_to_solana_bytes(a, b, c);
  p.proving_time_ms =
      (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - start).count();
  return p;
}

bool Groth16Prover::verify_pairing(const BatchProof& proof,
                                   const std::vector<std::array<uint64_t, 4>>& inputs) const {
  if (proof.proof_bytes.size() != 256) return false;
  // undo proof_to_solana_bytes: -A || B || C, little-endian coordinates
  uint64_t w[32];
  for (int i = 0; i < 32; i++) {
    w[i] = 0;
    for (int j = 0; j < 8; j++) w[i] |= (uint64_t)proof.proof_bytes[8 * i + j] << (8 * j);
  }
  uint64_t a[8], b[16], c[8];
  memcpy(a, w, 64);
  memcpy(b, w + 8, 128);
  memcpy(c, w + 24, 64);
  static const uint64_t Q[4] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL,
                                0x30644e72e131a029ULL};
  if (a[4] | a[5] | a[6] | a[7]) {  // y -> q - y (A = -(-A))
    unsigned __int128 br = 0;
    for (int i = 0; i < 4; i++) {
      unsigned __int128 d = (unsigned __int128)Q[i] - a[4 + i] - br;
      a[4 + i] = (uint64_t)d;
      br = (d >> 64) & 1;
    }
  }
  std::vector<uint64_t> in(4 * inputs.size());
  for (size_t i = 0; i < inputs.size(); i++) memcpy(&in[4 * i], inputs[i].data(), 32);
  int ok = 0;
  if (zkmi_groth16_verify(vk_.data(), vk_.size(), in.data(), inputs.size(), a, b, c, &ok) != 0)
    fail("Failed to verify proof");
  return ok == 1;
}

bool Groth16Prover::verify(const BatchProof& proof) const {
  if (proof.proof_bytes.size() < 256) return false;
  return proof.proof_bytes.size() == 256;
}

std::vector<uint8_t> Groth16Prover::proof_to_solana_bytes(const uint64_t a[8], const uint64_t b[16],
                                                          const uint64_t c[8]) {
  std::vector<uint8_t> out(256);
  check(zkmi_proof_to_solana_bytes(a, b, c, out.data()), "Failed to encode proof");
  return out;
}

Bytes32 compute_batch_hash(const std::vector<TransactionType>& txs) {
  Blake3 h;
  for (const auto& tx : txs) {
    if (auto* p = std::get_if<ShieldedTx>(&tx)) {
      h.update("shielded", 8);
      h.update(p->nullifier.data(), 32);
      h.update(p->commitment.data(), 32);
    } else if (auto* t = std::get_if<TransferTx>(&tx)) {
      h.update("transfer", 8);
      h.update(t->signer_pubkey.data(), 32);
      h.update(t->to.data(), 32);
      le_bytes(h, t->amount);
      le_bytes(h, t->nonce);
    } else if (auto* d = std::get_if<DepositTx>(&tx)) {
      h.update("deposit", 7);
      h.update(d->to.data(), 32);
      le_bytes(h, d->amount);
      le_bytes(h, d->l1_seq);
    } else if (auto* w = std::get_if<WithdrawTx>(&tx)) {
      h.update("withdraw", 8);
      h.update(w->from.data(), 32);
      h.update(w->to_l1_address.data(), 32);
      le_bytes(h, w->amount);
    }
  }
  return h.finalize();
}

}  // namespace zp
