// l2_circuit.h — L2BlockCircuit (prover/src/l2_circuit.rs:180-505) synthesized
// into an R1CS + full assignment on the host, in the C++ host mirror of the
// reference prover.  Same restatement as zelana_amd/l2block.py (the two are
// compared row for row by tests/test_host_mirror.py); see that module for the
// arkworks 0.5 gadget semantics followed and why the matrices are parity-
// unpinned.
#pragma once
#include <stdint.h>

#include <array>
#include <map>
#include <string>
#include <vector>

#include "fr.h"

namespace zp {

using Bytes32 = std::array<uint8_t, 32>;

struct TransactionWitness {  // l2_circuit.rs:45-50
  Bytes32 sender_pk, recipient_pk;
  uint64_t amount;
};
struct WithdrawalWitness {  // l2_circuit.rs:58-62
  Bytes32 recipient;
  uint64_t amount;
};

// CSR matrices (canonical 4 x u64 coefficients) and the assignment
// z = [1, instances..., witnesses...], as zkmi_r1cs expects
struct R1CSMatrices {
  size_t num_constraints = 0, num_instance = 0, num_witness = 0;
  std::vector<uint64_t> rowptr[3], col[3], val[3];
  std::vector<uint64_t> z;  // (num_instance + num_witness) x 4
  bool is_satisfied() const;
};

// The witness program of one L2BlockCircuit shape (zkmi.h "witness
// programs"): the arrays zkmi_wprog_desc points at.  Recorded once per shape
// by synthesize(); per batch only witness_inputs() changes.  Ops used: MUL,
// BITS (254-bit non-unique decomposition), NZ and INV1 (is_neq_const's two
// witnesses) and POSEIDON (one permutation's S-box trace); coefficients 0..200
// are the Poseidon constants the POSEIDON op reads.
struct L2WitnessProgram {
  uint64_t num_vars = 0, num_instance = 0;
  std::vector<uint32_t> input_var;       // z index of every free input, allocation order (input 0 = One)
  std::vector<uint32_t> op;              // 4 x u32 per op, level order
  std::vector<uint32_t> term;            // 2 x u32 per term
  std::vector<uint64_t> coeff;           // 4 x u64 canonical per coefficient
  std::vector<uint32_t> level_start;     // num_levels + 1
  std::vector<uint64_t> template_inputs; // the recorded batch's inputs (4 x u64 each)
  size_t num_levels() const { return level_start.empty() ? 0 : level_start.size() - 1; }
  // host evaluation of the program (test reference): canonical z, 4 x u64 per variable
  std::vector<uint64_t> interpret(const std::vector<uint64_t>& inputs) const;
};

struct L2BlockCircuit {  // l2_circuit.rs:94-124
  Bytes32 pre_state_root{}, post_state_root{}, pre_shielded_root{}, post_shielded_root{}, withdrawal_root{},
      batch_hash{};
  uint64_t batch_id = 0;
  std::vector<TransactionWitness> transactions;
  std::map<Bytes32, uint64_t> initial_accounts;  // BTreeMap: ordered by key bytes
  std::vector<Bytes32> shielded_commitments;
  std::vector<WithdrawalWitness> withdrawals;

  static L2BlockCircuit dummy();  // l2_circuit.rs:141-166
  // ConstraintSynthesizer::generate_constraints; `computed` receives the
  // values the circuit derives for the roots it enforces (post_state_root,
  // post_shielded_root, withdrawal_root, batch_hash, pre_state_root)
  // `prog` (optional) receives the witness program of this circuit's shape.
  R1CSMatrices synthesize(std::map<std::string, Fr>* computed = nullptr, L2WitnessProgram* prog = nullptr) const;
  // The R1CS structure depends only on this key: counts, and which account
  // slots (ranks in the sorted key set, initial or created) each transfer
  // reads and writes.  Throws synthesize's AssignmentMissing error for a
  // sender outside the accounts.
  std::string shape_key() const;
  // The free inputs of this batch in the program's input order (canonical 4 x
  // u64 each): what zkmi_wprog_run takes for a program recorded on any
  // circuit with the same shape_key().
  std::vector<uint64_t> witness_inputs() const;
};

// native PoseidonSponge (get_poseidon_config, l2_circuit.rs:68-83): absorb xs, squeeze one
Fr poseidon_hash(const std::vector<Fr>& xs);

}  // namespace zp
