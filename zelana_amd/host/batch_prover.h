// batch_prover.h — C++ host mirror of the reference's prover plugin
// interface (core/src/sequencer/settlement/prover.rs), sitting above the C ABI
// of libzkmi.so (include/zkmi.h) exactly where the reference's Rust sits above
// arkworks.  Same names, argument meaning and error behaviour: anyhow::Error
// becomes a thrown std::runtime_error carrying zkmi_last_error().
//
//   trait BatchProver { prove, verify, verification_key_hash }     :160-169
//   struct MockProver                                              :179-245
//   struct Groth16Prover { from_bytes, from_files, prove, verify,
//                          verification_key_hash,
//                          proof_to_solana_bytes }                 :252-447
//
// Every field / curve / polynomial operation of Groth16Prover::prove runs on
// the MI355X, the witness included: the first batch of a circuit shape is
// synthesized on the host (l2_circuit.h), which records the shape's witness
// program and uploads its R1CS; every later batch of that shape only extracts
// its free inputs on the host and runs the program on the GPU (zkmi_wprog_run)
// straight into the resident prove.  The host keeps the StdRng draws.
#pragma once
#include <stdint.h>

#include <array>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <variant>
#include <vector>

#include "l2_circuit.h"

struct zkmi_ctx;
struct zkmi_pk;

namespace zp {

struct BatchPublicInputs {  // prover.rs:48-63
  Bytes32 pre_state_root{}, post_state_root{}, pre_shielded_root{}, post_shielded_root{}, withdrawal_root{},
      batch_hash{};
  uint64_t batch_id = 0;
};

struct BatchProof {  // prover.rs:66-74
  BatchPublicInputs public_inputs;
  std::vector<uint8_t> proof_bytes;
  uint64_t proving_time_ms = 0;
};

// TransactionType, with the fields the prover (prover.rs:357-390) and
// compute_batch_hash (:525-558) read
struct TransferTx {
  Bytes32 signer_pubkey;
  Bytes32 to;
  uint64_t amount;
  uint64_t nonce = 0;
};
struct WithdrawTx {
  Bytes32 from;
  Bytes32 to_l1_address;
  uint64_t amount;
};
struct ShieldedTx {
  Bytes32 nullifier, commitment;
};
struct DepositTx {
  Bytes32 to;
  uint64_t amount, l1_seq;
};
using TransactionType = std::variant<TransferTx, WithdrawTx, ShieldedTx, DepositTx>;

struct AccountStateSnapshot {  // prover.rs:93-106
  Bytes32 account_id{};
  uint64_t balance = 0;
  uint64_t nonce = 0;
  std::vector<Bytes32> merkle_proof;
  std::vector<uint8_t> path_indices;
  uint64_t position = 0;
};

struct BatchWitness {  // prover.rs:78-90 (results / per-transfer paths unused by the circuit)
  std::vector<TransactionType> transactions;
  std::vector<AccountStateSnapshot> pre_account_states;
};

class BatchProver {  // prover.rs:160-169
 public:
  virtual ~BatchProver() = default;
  virtual BatchProof prove(const BatchPublicInputs& inputs, const BatchWitness& witness) const = 0;
  virtual bool verify(const BatchProof& proof) const = 0;
  virtual Bytes32 verification_key_hash() const = 0;
};

class MockProver : public BatchProver {  // prover.rs:179-245
 public:
  explicit MockProver(uint64_t prove_time_ms = 100);
  BatchProof prove(const BatchPublicInputs& inputs, const BatchWitness& witness) const override;
  bool verify(const BatchProof& proof) const override { return proof.proof_bytes.size() >= 32; }
  Bytes32 verification_key_hash() const override { return vk_hash_; }

 private:
  uint64_t prove_time_ms_;
  Bytes32 vk_hash_;
};

class Groth16Prover : public BatchProver {
 public:
  // ProvingKey / VerifyingKey::deserialize_compressed (validated) on GPU `device`
  static std::unique_ptr<Groth16Prover> from_bytes(const std::vector<uint8_t>& pk_bytes,
                                                   const std::vector<uint8_t>& vk_bytes, int device = 0);
  static std::unique_ptr<Groth16Prover> from_files(const std::string& pk_path, const std::string& vk_path,
                                                   int device = 0);
  ~Groth16Prover() override;

  BatchProof prove(const BatchPublicInputs& inputs, const BatchWitness& witness) const override;
  bool verify(const BatchProof& proof) const override;  // length check, as the reference (:427-442)
  // The on-chain verifier's pairing check (verifier lib.rs:497-547) on the
  // host, under this prover's VK: `inputs` = the circuit's 7 instance values
  // (canonical 4 x u64 each); proof.proof_bytes = the 256-B layout of prove().
  bool verify_pairing(const BatchProof& proof, const std::vector<std::array<uint64_t, 4>>& inputs) const;
  Bytes32 verification_key_hash() const override { return vk_hash_; }
  const std::vector<uint8_t>& verifying_key() const { return vk_; }
  // -A || B || C, little-endian coordinates (prover.rs:304-334)
  static std::vector<uint8_t> proof_to_solana_bytes(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8]);
  // the circuit prove() builds (prover.rs:357-405)
  static L2BlockCircuit circuit_of(const BatchPublicInputs& inputs, const BatchWitness& witness);

 private:
  Groth16Prover() = default;
  zkmi_ctx* ctx_ = nullptr;
  zkmi_pk* pk_ = nullptr;
  std::vector<uint8_t> vk_;
  Bytes32 vk_hash_{};
  // BatchProver is shared (Arc<dyn BatchProver>: Send + Sync) but a zkmi
  // context serves one call at a time (zkmi.h): prove() serialises on it
  mutable std::mutex gpu_mu_;
  // per circuit shape: witness program + resident R1CS + z buffer (most
  // recently used first, at most kMaxShapes; guarded by gpu_mu_)
  struct Shape;
  static constexpr size_t kMaxShapes = 8;
  mutable std::vector<std::unique_ptr<Shape>> shapes_;
  BatchProof prove_host(const BatchPublicInputs& inputs, const L2BlockCircuit& c) const;
};

// BLAKE3 compute_batch_hash over the transactions (prover.rs:525-558)
Bytes32 compute_batch_hash(const std::vector<TransactionType>& txs);

}  // namespace zp
