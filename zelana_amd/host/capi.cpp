// capi.cpp — extern "C" surface of the C++ host mirror (libzelana_prover.so),
// used by the Python tests to drive it exactly as a Rust / C++ caller would.
// Errors: non-zero return, message in zp_last_error() (the anyhow::Error text).
#include <string.h>

#include <string>

#include "batch_prover.h"
#include "blake3.h"
#include "std_rng.h"

using namespace zp;

namespace {
thread_local std::string g_err;
int guard(const std::exception& e) {
  g_err = e.what();
  return 1;
}
// inputs: 6 x 32-B roots then u64 LE batch_id (200 B, the settlement layout)
BatchPublicInputs parse_inputs(const uint8_t* p) {
  BatchPublicInputs in;
  Bytes32* r[6] = {&in.pre_state_root, &in.post_state_root, &in.pre_shielded_root, &in.post_shielded_root,
                   &in.withdrawal_root, &in.batch_hash};
  for (int i = 0; i < 6; i++) memcpy(r[i]->data(), p + 32 * i, 32);
  in.batch_id = 0;
  for (int i = 0; i < 8; i++) in.batch_id |= (uint64_t)p[192 + i] << (8 * i);
  return in;
}
uint64_t u64le(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}
// witness: transfers n_t x (32 signer | 32 to | u64 amount), withdrawals n_w x
// (32 from | 32 l1 | u64 amount), accounts n_a x (32 id | u64 balance)
BatchWitness parse_witness(const uint8_t* tr, size_t nt, const uint8_t* wd, size_t nw, const uint8_t* ac, size_t na) {
  BatchWitness w;
  for (size_t i = 0; i < nt; i++) {
    TransferTx t;
    memcpy(t.signer_pubkey.data(), tr + 72 * i, 32);
    memcpy(t.to.data(), tr + 72 * i + 32, 32);
    t.amount = u64le(tr + 72 * i + 64);
    w.transactions.push_back(t);
  }
  for (size_t i = 0; i < nw; i++) {
    WithdrawTx x;
    memcpy(x.from.data(), wd + 72 * i, 32);
    memcpy(x.to_l1_address.data(), wd + 72 * i + 32, 32);
    x.amount = u64le(wd + 72 * i + 64);
    w.transactions.push_back(x);
  }
  for (size_t i = 0; i < na; i++) {
    AccountStateSnapshot s;
    memcpy(s.account_id.data(), ac + 40 * i, 32);
    s.balance = u64le(ac + 40 * i + 32);
    w.pre_account_states.push_back(s);
  }
  return w;
}
}  // namespace

extern "C" {
const char* zp_last_error(void) { return g_err.c_str(); }

void zp_blake3(const uint8_t* data, size_t n, uint8_t out[32]) {
  auto h = Blake3::hash(data, n);
  memcpy(out, h.data(), 32);
}
// first k Fr::rand draws of StdRng::seed_from_u64(seed), canonical
void zp_stdrng_fr(uint64_t seed, size_t k, uint64_t* out) {
  StdRng r = StdRng::seed_from_u64(seed);
  for (size_t i = 0; i < k; i++) r.fr_rand().to_canon(out + 4 * i);
}
void zp_poseidon_hash(const uint64_t* xs, size_t n, uint64_t out[4]) {
  std::vector<Fr> v;
  for (size_t i = 0; i < n; i++) v.push_back(Fr::from_canon(xs + 4 * i));
  poseidon_hash(v).to_canon(out);
}

// L2BlockCircuit of Groth16Prover::prove for (inputs, witness): handle to the R1CS
int zp_l2_synthesize(const uint8_t* inputs, const uint8_t* tr, size_t nt, const uint8_t* wd, size_t nw,
                     const uint8_t* ac, size_t na, void** out) {
  try {
    L2BlockCircuit c = Groth16Prover::circuit_of(parse_inputs(inputs), parse_witness(tr, nt, wd, nw, ac, na));
    *out = new R1CSMatrices(c.synthesize());
    return 0;
  } catch (const std::exception& e) {
    return guard(e);
  }
}
// The same synthesis, also recording the witness program of the circuit's
// shape: *r1cs_out as zp_l2_synthesize, *prog_out a zp_wprog_* handle
int zp_l2_record(const uint8_t* inputs, const uint8_t* tr, size_t nt, const uint8_t* wd, size_t nw, const uint8_t* ac,
                 size_t na, void** r1cs_out, void** prog_out) {
  try {
    L2BlockCircuit c = Groth16Prover::circuit_of(parse_inputs(inputs), parse_witness(tr, nt, wd, nw, ac, na));
    std::unique_ptr<L2WitnessProgram> p(new L2WitnessProgram());
    *r1cs_out = new R1CSMatrices(c.synthesize(nullptr, p.get()));
    *prog_out = p.release();
    return 0;
  } catch (const std::exception& e) {
    return guard(e);
  }
}
// a batch's free inputs (num_inputs x 4 u64; call with out = NULL for the count)
int zp_l2_witness_inputs(const uint8_t* inputs, const uint8_t* tr, size_t nt, const uint8_t* wd, size_t nw,
                         const uint8_t* ac, size_t na, uint64_t* out, size_t* n_inputs) {
  try {
    L2BlockCircuit c = Groth16Prover::circuit_of(parse_inputs(inputs), parse_witness(tr, nt, wd, nw, ac, na));
    std::vector<uint64_t> v = c.witness_inputs();
    *n_inputs = v.size() / 4;
    if (out) memcpy(out, v.data(), v.size() * 8);
    return 0;
  } catch (const std::exception& e) {
    return guard(e);
  }
}
int zp_l2_shape_key(const uint8_t* inputs, const uint8_t* tr, size_t nt, const uint8_t* wd, size_t nw,
                    const uint8_t* ac, size_t na, char* out, size_t cap) {
  try {
    L2BlockCircuit c = Groth16Prover::circuit_of(parse_inputs(inputs), parse_witness(tr, nt, wd, nw, ac, na));
    const std::string k = c.shape_key();
    if (k.size() + 1 > cap) throw std::runtime_error("shape key buffer too small");
    memcpy(out, k.c_str(), k.size() + 1);
    return 0;
  } catch (const std::exception& e) {
    return guard(e);
  }
}
// sizes: num_vars, num_inputs, num_ops, num_terms, num_coeffs, num_levels
void zp_wprog_sizes(const void* h, uint64_t out[6]) {
  const L2WitnessProgram* p = (const L2WitnessProgram*)h;
  out[0] = p->num_vars, out[1] = p->input_var.size(), out[2] = p->op.size() / 4, out[3] = p->term.size() / 2;
  out[4] = p->coeff.size() / 4, out[5] = p->num_levels();
}
void zp_wprog_copy(const void* h, uint32_t* input_var, uint32_t* op, uint32_t* term, uint64_t* coeff,
                   uint32_t* level_start, uint64_t* template_inputs) {
  const L2WitnessProgram* p = (const L2WitnessProgram*)h;
  memcpy(input_var, p->input_var.data(), p->input_var.size() * 4);
  memcpy(op, p->op.data(), p->op.size() * 4);
  memcpy(term, p->term.data(), p->term.size() * 4);
  memcpy(coeff, p->coeff.data(), p->coeff.size() * 8);
  memcpy(level_start, p->level_start.data(), p->level_start.size() * 4);
  memcpy(template_inputs, p->template_inputs.data(), p->template_inputs.size() * 8);
}
int zp_wprog_interpret(const void* h, const uint64_t* inputs, uint64_t* z_out) {
  try {
    const L2WitnessProgram* p = (const L2WitnessProgram*)h;
    std::vector<uint64_t> in(inputs, inputs + 4 * p->input_var.size());
    std::vector<uint64_t> z = p->interpret(in);
    memcpy(z_out, z.data(), z.size() * 8);
    return 0;
  } catch (const std::exception& e) {
    return guard(e);
  }
}
void zp_wprog_free(void* h) { delete (L2WitnessProgram*)h; }

// sizes: m, num_instance, num_witness, nnz(a), nnz(b), nnz(c), satisfied
void zp_r1cs_sizes(const void* h, uint64_t out[7]) {
  const R1CSMatrices* m = (const R1CSMatrices*)h;
  out[0] = m->num_constraints, out[1] = m->num_instance, out[2] = m->num_witness;
  for (int t = 0; t < 3; t++) out[3 + t] = m->col[t].size();
  out[6] = m->is_satisfied();
}
void zp_r1cs_copy(const void* h, int t, uint64_t* rowptr, uint64_t* col, uint64_t* val) {
  const R1CSMatrices* m = (const R1CSMatrices*)h;
  memcpy(rowptr, m->rowptr[t].data(), m->rowptr[t].size() * 8);
  memcpy(col, m->col[t].data(), m->col[t].size() * 8);
  memcpy(val, m->val[t].data(), m->val[t].size() * 8);
}
void zp_r1cs_z(const void* h, uint64_t* z) {
  const R1CSMatrices* m = (const R1CSMatrices*)h;
  memcpy(z, m->z.data(), m->z.size() * 8);
}
void zp_r1cs_free(void* h) { delete (R1CSMatrices*)h; }

// Groth16Prover over libzkmi
int zp_groth16_from_bytes(const uint8_t* pk, size_t pk_len, const uint8_t* vk, size_t vk_len, int device, void** out) {
  try {
    *out = Groth16Prover::from_bytes(std::vector<uint8_t>(pk, pk + pk_len), std::vector<uint8_t>(vk, vk + vk_len),
                                     device)
               .release();
    return 0;
  } catch (const std::exception& e) {
    return guard(e);
  }
}
int zp_groth16_prove(const void* h, const uint8_t* inputs, const uint8_t* tr, size_t nt, const uint8_t* wd, size_t nw,
                     const uint8_t* ac, size_t na, uint8_t proof_out[256], uint64_t* time_ms) {
  try {
    BatchProof p = ((const Groth16Prover*)h)->prove(parse_inputs(inputs), parse_witness(tr, nt, wd, nw, ac, na));
    if (p.proof_bytes.size() != 256) throw std::runtime_error("proof is not 256 bytes");
    memcpy(proof_out, p.proof_bytes.data(), 256);
    if (time_ms) *time_ms = p.proving_time_ms;
    return 0;
  } catch (const std::exception& e) {
    return guard(e);
  }
}
void zp_groth16_vk_hash(const void* h, uint8_t out[32]) {
  auto v = ((const Groth16Prover*)h)->verification_key_hash();
  memcpy(out, v.data(), 32);
}
void zp_groth16_free(void* h) { delete (Groth16Prover*)h; }
}  // extern "C"
