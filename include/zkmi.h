/*
 * zkmi.h — C ABI of the MI355X-native BN254 Groth16 proving backend
 * (libzkmi.so, zelana_amd/csrc/).  Drop-in replacement for the arithmetic that
 * Zelana's `Groth16Prover` delegates to arkworks 0.5.0:
 *
 *   reference call site                                   replaced by
 *   ---------------------------------------------------   --------------------------
 *   core/src/sequencer/settlement/prover.rs:263-277        zkmi_pk_load
 *     ProvingKey::<Bn254>::deserialize_compressed
 *   core/src/sequencer/settlement/prover.rs:408            zkmi_groth16_prove
 *     Groth16::<Bn254>::prove (create_proof_with_reduction)
 *   ark-groth16 LibsnarkReduction::witness_map_from_       zkmi_witness_map
 *     matrices (3P)
 *   ark-poly Radix2EvaluationDomain::{fft,ifft}[_coset]    zkmi_ntt / zkmi_ntt_device
 *     (3P, a6)
 *   ark-ec VariableBaseMSM::msm_bigint on G1 / G2          zkmi_msm_g1 / zkmi_msm_g2
 *     (3P, a7 / a8; called 4x G1 + 1x G2 per proof)        (+ _device variants)
 *   core/src/sequencer/settlement/prover.rs:304-334        zkmi_proof_to_solana_bytes
 *     Groth16Prover::proof_to_solana_bytes
 *   prover/src/snarkjs.rs:44-52 export_proof_json           zkmi_proof_serialize_compressed
 *
 * Conventions:
 *   - every function returns 0 on success, a negative ZKMI_E* code otherwise;
 *     zkmi_last_error() returns a thread-local message.  Nothing unwinds across
 *     the ABI.
 *   - field elements cross as 4 x uint64 little-endian CANONICAL integers
 *     (never Montgomery); scalars must be < r (arkworks into_bigint()).
 *   - G1 affine = x || y (8 u64), G2 affine = x.c0 || x.c1 || y.c0 || y.c1
 *     (16 u64); the point at infinity is all-zero.
 *   - buffers are caller-owned; calls are synchronous; one context per device
 *     (one process per GPU); a context must not be used by two threads at once.
 *   - the library never falls back to the CPU: without a usable gfx950 device
 *     zkmi_ctx_create fails with ZKMI_ENODEV.
 */
#ifndef ZKMI_H
#define ZKMI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZKMI_OK 0
#define ZKMI_EINVAL (-1)   /* bad argument / malformed input */
#define ZKMI_ENODEV (-2)   /* no usable GPU */
#define ZKMI_EHIP (-3)     /* HIP runtime error */
#define ZKMI_ENOMEM (-4)   /* device allocation failed */
#define ZKMI_EPOINT (-5)   /* point not on curve / not in subgroup */

typedef struct zkmi_ctx zkmi_ctx;
typedef struct zkmi_bases zkmi_bases;
typedef struct zkmi_pk zkmi_pk;
typedef struct zkmi_msm_job zkmi_msm_job;
typedef struct zkmi_r1cs_dev zkmi_r1cs_dev;

const char* zkmi_last_error(void);
int zkmi_version(void);

/* ------------------------------------------------------------- context */
int zkmi_ctx_create(int device, zkmi_ctx** out);
/* Destroy the objects made on a context (base sets, keys, device R1CS,
 * communicators, MSM jobs) before the context.  Witness programs may outlive
 * it: zkmi_ctx_destroy detaches them, and zkmi_wprog_destroy then only frees
 * their buffers. */
void zkmi_ctx_destroy(zkmi_ctx* ctx);
/* per-kernel timing with HIP events on the context's stream (bench/profiling) */
int zkmi_profile_enable(zkmi_ctx* ctx, int on);
/* total milliseconds and launch count recorded for kernel `name` */
int zkmi_profile_get(zkmi_ctx* ctx, const char* name, double* total_ms, uint64_t* count);
int zkmi_profile_reset(zkmi_ctx* ctx);
/* device memory staging (so callers can keep inputs resident in HBM) */
int zkmi_dev_alloc(zkmi_ctx* ctx, size_t bytes, void** dptr);
int zkmi_dev_free(zkmi_ctx* ctx, void* dptr);
int zkmi_h2d(zkmi_ctx* ctx, void* dst, const void* src, size_t bytes);
int zkmi_d2h(zkmi_ctx* ctx, void* dst, const void* src, size_t bytes);
int zkmi_sync(zkmi_ctx* ctx);

/* ------------------------------------------------------------- MSM */
/* Upload affine bases once (pk queries stay resident in HBM).  Points are
 * validated on-curve; converted to the device's internal Montgomery form. */
int zkmi_bases_create_g1(zkmi_ctx* ctx, const uint64_t* affine, size_t n, zkmi_bases** out);
int zkmi_bases_create_g2(zkmi_ctx* ctx, const uint64_t* affine, size_t n, zkmi_bases** out);
void zkmi_bases_destroy(zkmi_bases* b);
size_t zkmi_bases_len(const zkmi_bases* b);
/* canonical affine copy of a base set (n x 8 or n x 16 u64) */
int zkmi_bases_export(const zkmi_bases* b, uint64_t* affine_out);
/* Fixed-base table for a base set that is reused across MSMs (a proving
 * key's queries).  Stores `factor` shifted copies 2^(c*Wp*j) * P_i (Wp =
 * ceil(W(c)/factor)) in HBM; later MSMs on this set with window c (the
 * default unless zkmi_msm_set_window pins another) run Wp windows of
 * factor*n entries instead of W(c) windows of n entries: same additions,
 * 1/factor of the bucket reduction.  c = 0 picks the window for len(b);
 * factor = 0 means a full table (one window).  Results are unchanged.
 * Memory: factor x the base set.  No counterpart in the reference
 * (arkworks recomputes every window per proof). */
int zkmi_bases_precompute(zkmi_bases* b, int c, int factor);
/* [len, table window c (0 = none), copies, windows per copy] */
int zkmi_bases_info(const zkmi_bases* b, uint64_t out[4]);
/* Deterministic synthetic inputs generated directly in HBM (benchmarks):
 * bases P_i = k_i * G (k_i from a splitmix64 stream of seed), scalars uniform
 * in [0, r) by rejection.  d_scalars must hold n x 32 bytes. */
int zkmi_bases_generate_g1(zkmi_ctx* ctx, uint64_t seed, size_t n, zkmi_bases** out);
int zkmi_bases_generate_g2(zkmi_ctx* ctx, uint64_t seed, size_t n, zkmi_bases** out);
int zkmi_scalars_generate(zkmi_ctx* ctx, uint64_t seed, size_t n, void* d_scalars);
/* The same streams from global element `first` on: element i of the range is
 * element first + i of the unsharded set, so a point-sharded MSM over ranks
 * [r*n, (r+1)*n) sums to the single-GPU result (multi-GPU bench, config 5). */
int zkmi_bases_generate_range_g1(zkmi_ctx* ctx, uint64_t seed, size_t first, size_t n, zkmi_bases** out);
int zkmi_scalars_generate_range(zkmi_ctx* ctx, uint64_t seed, size_t first, size_t n, void* d_scalars);
/* SURVEY.md §8d's point stream: P_i = P0 + (first + i) * D for i < n
 * (canonical affine P0, D; the bench draws them as G1::rand from
 * StdRng::seed_from_u64(1020)), generated in HBM. */
int zkmi_bases_generate_arith_g1(zkmi_ctx* ctx, const uint64_t p0[8], const uint64_t d[8], size_t first, size_t n,
                                 zkmi_bases** out);

/* sum_{i<n} scalars[i] * bases[offset + i]; n <= len - offset.
 * Host scalars (n x 4 u64). Result: canonical affine. */
int zkmi_msm_g1(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const uint64_t* scalars, size_t n,
                uint64_t out_affine[8]);
int zkmi_msm_g2(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const uint64_t* scalars, size_t n,
                uint64_t out_affine[16]);
/* same with scalars already resident in device memory (n x 32 B) */
int zkmi_msm_g1_device(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
                       uint64_t out_affine[8]);
int zkmi_msm_g2_device(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
                       uint64_t out_affine[16]);
/* Asynchronous form: submit queues the GPU work (and the copy of the ~c*W
 * window bit-sums) on the context stream and returns at once; wait finishes
 * the O(windows) host epilogue and frees the job.  Submitting MSM k+1 before
 * waiting on MSM k overlaps k's epilogue with k+1's kernels.  Scalars must
 * stay valid until wait returns. */
int zkmi_msm_submit(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
                    zkmi_msm_job** job);
int zkmi_msm_wait(zkmi_msm_job* job, uint64_t* out_affine);
/* window size override for experiments (0 = automatic) */
/* k MSMs with the same device scalars and range over k base sets (e.g. a,
 * b_g1 and b_g2 queries of a proving key, all weighted by z): one digits +
 * sort pass is shared by every set with the same window plan.  jobs[i] is the
 * job of bs[i] (finish each with zkmi_msm_wait). */
int zkmi_msm_submit_shared(zkmi_ctx* ctx, const zkmi_bases* const* bs, int k, size_t offset, const void* d_scalars,
                           size_t n, zkmi_msm_job** jobs);
int zkmi_msm_set_window(zkmi_ctx* ctx, int c);
/* Number of MSM lanes (streams with their own scratch) used round-robin by
 * consecutive submissions so their latency-bound tails overlap; 1..8, at most
 * 2 while a communicator exists on the context (stream budget, below). */
int zkmi_msm_set_lanes(zkmi_ctx* ctx, int lanes);
/* lanes in effect (after the communicator cap) */
int zkmi_msm_get_lanes(const zkmi_ctx* ctx);
/* streams the library holds for this context (context stream, MSM lanes,
 * communicator and witness-program streams) */
int zkmi_ctx_stream_count(const zkmi_ctx* ctx);

/* canonical affine point arithmetic helpers (host) */
int zkmi_g1_add(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]);
int zkmi_g2_add(const uint64_t a[16], const uint64_t b[16], uint64_t out[16]);

/* ------------------------------------------------------------- multi-GPU
 * MSM point sharding (BASELINE.json configs[4]): one rank per
 * GPU (one process per GPU, or one host thread per GPU in one process), each
 * holding its own zkmi_ctx and the shard [first, first + count) of the bases
 * resident in its HBM (zkmi_shard_range + zkmi_bases_create_*).  A sharded MSM
 * runs the full Pippenger pipeline on every shard, then exchanges the
 * per-window bit sums (the partially reduced buckets, ~c x W XYZZ points per
 * rank) with ONE all-gather and sums them across ranks in the group-law
 * epilogue: the "all-reduce of partial bucket sums" (RCCL has no elliptic-
 * curve reduction operator).  Every rank returns the global sum.
 *
 * Transports:
 *   zkmi_comm_init       RCCL (ncclAllGather over xGMI), enqueued on the MSM
 *                        lane's stream: no host round trip in the exchange.
 *                        The ranks' unique id comes from zkmi_comm_unique_id
 *                        on one rank, broadcast by the host (like NCCL).
 *   zkmi_comm_init_host  the host supplies the all-gather (MPI, a TCP store,
 *                        pipes ...): for hosts without RCCL, or ranks that share
 *                        one GPU (RCCL refuses two ranks on one device).
 * Collectives must be issued in the same order on every rank.  Every sharded
 * MSM is exactly one all-gather of one fixed size per rank (a status block and
 * the bit sums), whatever each rank's shard, plan or local failure, so no rank
 * can block in a collective its peers skip.  Ranks' window plans must agree
 * (equal shard sizes and the same zkmi_bases_precompute / zkmi_msm_set_window
 * choice); a mismatch, or a failure on any rank, is reported as ZKMI_EINVAL
 * on every rank by zkmi_msm_wait.
 * Streams: a process with a communicator uses the context stream, at most two
 * MSM lanes (zkmi_msm_set_lanes is capped at 2 while a communicator exists)
 * and the communicator's stream: 4 = GPU_MAX_HW_QUEUES, so the RCCL kernel,
 * which waits for its peers, never shares a hardware queue with a lane's
 * kernels.  Witness programs run on the context stream then. */
typedef struct zkmi_comm zkmi_comm;
#define ZKMI_COMM_ID_BYTES 128
/* all-gather of `bytes` from every rank: recv = rank 0's bytes || rank 1's ... */
typedef int (*zkmi_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);
int zkmi_comm_unique_id(uint8_t id[ZKMI_COMM_ID_BYTES]);
int zkmi_comm_init(zkmi_ctx* ctx, const uint8_t id[ZKMI_COMM_ID_BYTES], int nranks, int rank, zkmi_comm** out);
int zkmi_comm_init_host(zkmi_ctx* ctx, int nranks, int rank, zkmi_allgather_fn allgather, void* user,
                        zkmi_comm** out);
void zkmi_comm_destroy(zkmi_comm* comm);
/* [nranks, rank, transport (0 = RCCL, 1 = host)] */
int zkmi_comm_info(const zkmi_comm* comm, int out[3]);
/* contiguous point shard of rank `rank`: the first total % nranks ranks get
 * one extra point */
int zkmi_shard_range(size_t total, int nranks, int rank, size_t* first, size_t* count);
/* sum over ALL ranks of sum_{i<n} scalars[i] * shard[offset + i]; collective.
 * Scalars are this rank's slice (device memory, n x 32 B canonical).  A
 * rank-local failure fails the MSM on every rank.  Over RCCL it is returned by
 * the submit; over a host transport the submit returns a job and
 * zkmi_msm_wait returns the error, because that transport's exchanges run in
 * wait order (the failure joins the exchange of its own job, never an earlier
 * job's still in flight). */
int zkmi_msm_sharded_submit(zkmi_comm* comm, const zkmi_bases* shard, size_t offset, const void* d_scalars,
                            size_t n, zkmi_msm_job** job);
int zkmi_msm_sharded(zkmi_comm* comm, const zkmi_bases* shard, size_t offset, const void* d_scalars, size_t n,
                     uint64_t* out_affine);
/* Window sharding (north_star's "Pippenger windows sharded across GPUs"):
 * every rank passes the WHOLE base set and scalars (n points, resident on its
 * GPU) and runs windows [r W / N, (r + 1) W / N) of the plain Pippenger plan
 * (window c = zkmi_msm_set_window, 12..17 bits, or 0 for the automatic
 * choice, clamped to 12..17; a fixed-base table is not used -- it folds
 * every window into one).  The same
 * fixed-size exchange as the point-sharded MSM hands each rank's window bit
 * sums to every rank, and zkmi_msm_wait assembles all W windows (each from
 * the one rank that ran it) before the Horner epilogue: every rank returns
 * the whole MSM.  Collective, like zkmi_msm_sharded_submit.  Replaces the
 * same call site (prover.rs:408 via ark-ec msm_bigint). */
int zkmi_msm_window_sharded_submit(zkmi_comm* comm, const zkmi_bases* bases, size_t offset, const void* d_scalars,
                                   size_t n, zkmi_msm_job** job);

/* ------------------------------------------------------------- NTT */
/* In-place radix-2 transform over Fr of length 2^log_n, natural order in and
 * out, ark-poly semantics: inverse=0 -> evaluations at omega^k (times g^i
 * coefficient scaling when coset=1, g = 5); inverse=1 -> interpolation incl.
 * n^-1 (and g^-i when coset=1).  log_n <= 28. */
int zkmi_ntt(zkmi_ctx* ctx, uint64_t* data, uint32_t log_n, int inverse, int coset);
int zkmi_ntt_device(zkmi_ctx* ctx, void* d_data, uint32_t log_n, int inverse, int coset);

/* ------------------------------------------------------------- Groth16 */
/* R1CS in CSR form; variable 0 = One, instance i -> i, witness j ->
 * num_instance + j (ark-relations to_matrices).  Coefficients canonical Fr. */
typedef struct {
  size_t num_constraints, num_instance, num_witness;
  const uint64_t* a_rowptr; const uint64_t* a_col; const uint64_t* a_val;
  const uint64_t* b_rowptr; const uint64_t* b_col; const uint64_t* b_val;
  const uint64_t* c_rowptr; const uint64_t* c_col; const uint64_t* c_val;
} zkmi_r1cs;

/* witness map: h (2^ceil(log2(m + l)) canonical Fr), natural order */
int zkmi_witness_map(zkmi_ctx* ctx, const zkmi_r1cs* cs, const uint64_t* z, uint64_t* h_out);

/* Load an arkworks-serialized ProvingKey<Bn254> (compressed=1 as read by
 * Groth16Prover::from_bytes, or uncompressed=0).  Points are decompressed /
 * validated on the GPU and stay resident. */
int zkmi_pk_load(zkmi_ctx* ctx, const uint8_t* bytes, size_t len, int compressed, zkmi_pk** out);
void zkmi_pk_destroy(zkmi_pk* pk);
/* [n_domain, num_instance, num_witness] */
int zkmi_pk_info(const zkmi_pk* pk, uint64_t out[3]);
/* arkworks-compressed VerifyingKey bytes embedded in the pk (for vk hash) */
/* Fixed-base tables for all five queries (zkmi_bases_precompute, window
 * picked per query length; factor 0 = full).  Proofs are unchanged; a full
 * table costs ~15x the key's HBM footprint (2^22 domain: ~24 GB).  When at
 * least 1/8 of the variables have both B bases at infinity (B_i(t) = 0: no B
 * row reads them), the B-query MSMs are first compacted to the others. */
int zkmi_pk_precompute(zkmi_pk* pk, int factor);
/* number of variables the B-query MSMs run over (V - 1 when not compacted) */
int zkmi_pk_b_terms(const zkmi_pk* pk, uint64_t* out);
int zkmi_pk_vk_bytes(const zkmi_pk* pk, uint8_t* buf, size_t cap, size_t* len);

/* Full proof.  z: full assignment (One, instance..., witness...), canonical.
 * r, s: the blinding scalars (the caller draws them from StdRng::seed_from_u64
 * (batch_id) in arkworks order r then s, as Groth16::prove does).
 * Outputs: canonical affine A (G1), B (G2), C (G1). */
int zkmi_groth16_prove(zkmi_ctx* ctx, const zkmi_pk* pk, const zkmi_r1cs* cs, const uint64_t* z,
                       const uint64_t r[4], const uint64_t s[4], uint64_t a_out[8], uint64_t b_out[16],
                       uint64_t c_out[8]);

/* Circuit matrices resident in HBM: a proving key fits exactly one circuit
 * shape (keygen.rs proves dummy()'s shape), so the
 * matrices are uploaded once and only the witness changes per proof. */
int zkmi_r1cs_create(zkmi_ctx* ctx, const zkmi_r1cs* cs, zkmi_r1cs_dev** out);
void zkmi_r1cs_destroy(zkmi_r1cs_dev* cs);
/* prove with R1CS and assignment z (n_vars x 32 B canonical) already in HBM */
int zkmi_groth16_prove_resident(zkmi_ctx* ctx, const zkmi_pk* pk, const zkmi_r1cs_dev* cs, const void* d_z,
                                const uint64_t r[4], const uint64_t s[4], uint64_t a_out[8], uint64_t b_out[16],
                                uint64_t c_out[8]);
/* Asynchronous form of the resident prove: submit queues the witness map and
 * the five MSMs and returns; wait finishes the MSM epilogues and the
 * assembly.  Several proofs may be in flight on one context (finish them in
 * submission order); d_z must stay unchanged until its proof's wait returns,
 * unless a zkmi_wprog_run writing it is ordered after (see there). */
typedef struct zkmi_proof_job zkmi_proof_job;
int zkmi_groth16_prove_submit(zkmi_ctx* ctx, const zkmi_pk* pk, const zkmi_r1cs_dev* cs, const void* d_z,
                              const uint64_t r[4], const uint64_t s[4], zkmi_proof_job** job);
int zkmi_groth16_prove_wait(zkmi_proof_job* job, uint64_t a_out[8], uint64_t b_out[16], uint64_t c_out[8]);
/* Benchmark helper: a random proving key of domain 2^log_n with the given
 * instance/witness counts, generated in HBM.  Proofs made with it do not
 * verify; the proving work is identical to a real key of that shape. */
int zkmi_pk_synthetic(zkmi_ctx* ctx, uint64_t seed, uint32_t log_n, size_t num_instance, size_t num_witness,
                      zkmi_pk** out);

/* Groth16 circuit-specific setup on the GPU.  Replaces
 * Groth16::<Bn254>::circuit_specific_setup (prover/src/bin/keygen.rs:87-91,
 * ark-groth16 0.5 generate_parameters_with_qap): QAP evaluation at t over the
 * radix-2 domain, then every query point as a fixed-base multiple of the
 * generators.  The caller draws the randomness in arkworks' order from its
 * StdRng (alpha, beta, gamma, delta = Fr::rand; G1::rand; G2::rand; then
 * t = Fr::rand until t^n != 1):
 *   toxic = alpha | beta | gamma | delta | t   (5 x 4 u64, canonical Fr)
 *   g1 (8 u64), g2 (16 u64)                     canonical affine generators
 * The key is resident (as after zkmi_pk_load) and equals arkworks' key for
 * the same inputs. */
int zkmi_groth16_setup(zkmi_ctx* ctx, const zkmi_r1cs* cs, const uint64_t toxic[20], const uint64_t g1[8],
                       const uint64_t g2[16], zkmi_pk** out);
/* VerifyingKey::deserialize_compressed (points decoded and validated on the
 * GPU) then serialize_compressed: the bytes Groth16Prover::compute_vk_hash
 * hashes (core/src/sequencer/settlement/prover.rs:266-267, 289-294).
 * out = NULL queries the length. */
int zkmi_vk_canonical(zkmi_ctx* ctx, const uint8_t* bytes, size_t len, uint8_t* out, size_t cap, size_t* out_len);
/* ProvingKey::serialize_compressed of a resident key (keygen.rs:101-104);
 * buf = NULL queries the length. */
int zkmi_pk_serialize(const zkmi_pk* pk, uint8_t* buf, size_t cap, size_t* len);

/* ------------------------------------------------------------- encodings */
/* 256 B Solana layout: -A (x,y LE) || B (x.c0,x.c1,y.c0,y.c1 LE) || C (x,y LE)
 * (prover.rs:304-334) */
int zkmi_proof_to_solana_bytes(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8],
                               uint8_t out[256]);
/* 128 B arkworks Proof::serialize_compressed (a 32 || b 64 || c 32) */
int zkmi_proof_serialize_compressed(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8],
                                    uint8_t out[128]);

/* ------------------------------------------------------ witness programs
 * Per-batch witness generation on the GPU: a proving
 * key fits one circuit shape, so a batch's full assignment z is a fixed
 * straight-line program over Fr of its ~thousands of free inputs (for
 * zelana_batch: Prover.toml's values; 99% of z is MiMC round values,
 * prover-worker/src/mimc.rs:52-142).  The program is recorded once on the
 * host (zelana_amd/wprog.py); per batch only the inputs travel, and z is
 * written straight into HBM for zkmi_groth16_prove_resident.
 *   op i: 4 x u32 {kind | a_len << 8 | b_len << 20, out, a_off, b_off};
 *         kinds 1 MUL z[out] = <a,z><b,z>; 2 INV z[out] = <a,z>^-1 (0 -> 0);
 *         3 BITS64 z[out+i] = bit i of <a,z>; 4 PERM MiMC permutation of
 *         <a,z>: z[out + 4r + (0..3)] = t_r^2, t_r^4, t_r^6, t_r^7 (91 rounds,
 *         t_0 = <a,z> + c_0, t_r = t_{r-1}^7 + c_r, c_i = (i+1)^3 + (i+1))
 *         5 BITS z[out+i] = bit i of <a,z>, i < b_off (1..256; b_len = 0);
 *         6 NZ z[out] = (<a,z> != 0); 8 INV1 z[out] = <a,z>^-1, or 1 when it
 *         is 0 (r1cs-std is_neq's two witnesses);
 *         7 POSEIDON one permutation of L2BlockCircuit's width-3 Poseidon
 *         sponge (prover/src/l2_circuit.rs:68-83: x^5, 8 full + 56 partial
 *         rounds).  State in: three combinations stored back to back at
 *         a_off, of lengths a_len, b_len and b_off & 0xFFFF; mask = b_off >> 16
 *         (1..7) marks the elements that are variables in round 0.  Out: x^2,
 *         x^4, x^5 of every S-box in round order (round 0 only for masked
 *         elements): 3 popcount(mask) + 231 values.  Reads the round
 *         constants ark[r][i] at coefficient 3r + i and the MDS matrix
 *         m[i][j] at 192 + 3i + j (so num_coeffs >= 201)
 *   term: 2 x u32 {z index, coefficient index}; <a,z> = sum over
 *         term[a_off .. a_off + a_len) of coeff * z
 *   levels: ops [level_start[l], level_start[l+1]) depend only on inputs and
 *         earlier levels. */
typedef struct zkmi_wprog zkmi_wprog;
typedef struct {
  size_t num_vars;                             /* |z| */
  size_t num_inputs; const uint32_t* input_var; /* z index of input k */
  size_t num_ops; const uint32_t* op;           /* num_ops x 4 */
  size_t num_terms; const uint32_t* term;       /* num_terms x 2 */
  size_t num_coeffs; const uint64_t* coeff;     /* num_coeffs x 4, canonical Fr */
  size_t num_levels; const uint32_t* level_start; /* num_levels + 1 */
} zkmi_wprog_desc;
int zkmi_wprog_create(zkmi_ctx* ctx, const zkmi_wprog_desc* desc, zkmi_wprog** out);
void zkmi_wprog_destroy(zkmi_wprog* prog);
/* z (device, num_vars x 32 B) <- the program over `inputs` (num_inputs x 4
 * u64 canonical; input 0 is One = 1).  Later work on the context (a proof
 * over z) waits for it.  async = 1: returns after queueing on the program's
 * own stream, which runs beside the context's earlier work (the previous
 * proof); it then waits only for context work queued before the PREVIOUS
 * run, so callers alternate two z buffers. */
int zkmi_wprog_run(zkmi_ctx* ctx, zkmi_wprog* prog, const uint64_t* inputs, void* d_z, int async);
/* nb batches in one run (one launch sequence; the kernels are latency-bound,
 * so nb batches take about the time of one): inputs = nb x num_inputs x 4
 * u64, batch i's z at d_z + i * z_stride bytes (z_stride >= num_vars * 32, a
 * multiple of 32).  Same ordering rules as zkmi_wprog_run, with buffer sets in
 * place of buffers. */
int zkmi_wprog_run_many(zkmi_ctx* ctx, zkmi_wprog* prog, size_t nb, const uint64_t* inputs, void* d_z,
                        size_t z_stride, int async);

/* ------------------------------------------------- verification / on-chain
 * Host code (no GPU needed).  The reference's Groth16Prover::verify is a
 * length check (prover.rs:427-442); the real check is the on-chain verifier's
 * (onchain-programs/verifier/programs/onchain_verifier/src/lib.rs:497-547),
 * restated here so a host can check its proofs before settling them. */
/* ark-groth16 verify_proof: vk = arkworks-compressed VerifyingKey bytes (as
 * Groth16Prover::from_bytes reads them; decoded and validated, G2 subgroup
 * included); inputs = n canonical Fr (4 x u64), n = IC count - 1.
 * *valid = 1 iff e(A,B) = e(alpha,beta) e(IC[0] + sum x_i IC[i+1], gamma) e(C,delta). */
int zkmi_groth16_verify(const uint8_t* vk, size_t vk_len, const uint64_t* inputs, size_t n_inputs,
                        const uint64_t a[8], const uint64_t b[16], const uint64_t c[8], int* valid);
/* The alt_bn128 syscalls the on-chain verifier calls (EIP-196/197 big-endian:
 * G1 = x || y, G2 = x.c1 || x.c0 || y.c1 || y.c0, (0,0) = infinity; points
 * validated, G2 in the order-r subgroup).  pairing: k x 192 bytes -> 32-byte
 * big-endian 1 iff prod e(P_i, Q_i) = 1. */
int zkmi_alt_bn128_pairing(const uint8_t* input, size_t len, uint8_t out[32]);
int zkmi_alt_bn128_g1_add(const uint8_t in[128], uint8_t out[64]);
int zkmi_alt_bn128_g1_mul(const uint8_t in[96], uint8_t out[64]);
/* The 256-B proof in the syscalls' big-endian encoding: -A || B || C
 * (the big-endian flag of proof_to_solana_bytes, whose reference output is
 * little-endian: SURVEY.md App. B.3). */
int zkmi_proof_to_alt_bn128_bytes(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8], uint8_t out[256]);
/* batch_inputs_to_field_elements (verifier lib.rs:479-494): the six 32-byte
 * roots as given, then batch_id as a 32-byte big-endian field element */
int zkmi_batch_inputs_alt_bn128(const uint8_t roots[6 * 32], uint64_t batch_id, uint8_t out[7 * 32]);
/* k * P on G1 (canonical affine): ProverNode::generate_fragment's single scalar
 * multiplication (forge/prover/src/lib.rs:351-358); with zkmi_g1_add it covers
 * the forge's <= 7-point Lagrange sums (:252-290) */
int zkmi_g1_mul(const uint64_t p[8], const uint64_t k[4], uint64_t out[8]);

#ifdef __cplusplus
}
#endif
#endif
