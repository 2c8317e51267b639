// zkmi_internal.h — context, error plumbing, workspace and kernel timing shared
// by the HIP translation units of libzkmi.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/zkmi.h"
#include "zkmi_internal_host.h"

namespace zk {

void set_error(const char* fmt, ...);

#define ZK_HIP(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      ::zk::set_error("HIP error %s at %s:%d (%s)", hipGetErrorString(e_), __FILE__, __LINE__, #expr); \
      return ZKMI_EHIP;                                                                    \
    }                                                                                      \
  } while (0)

#define ZK_TRY(expr)          \
  do {                        \
    int rc_ = (expr);         \
    if (rc_ != 0) return rc_; \
  } while (0)

// grow-only device scratch buffers keyed by name

struct Workspace {
  std::map<std::string, std::pair<void*, size_t>> bufs;
  int get(const char* name, size_t bytes, void** out);
  void release_all();
};

// An MSM lane: its own stream and scratch, so consecutive MSMs overlap (the
// latency-bound tail of one -- segmented and bucket reduction -- runs beside
// the sort / accumulation of the next).
struct MsmLane {
  hipStream_t st = nullptr;
  Workspace ws;
  hipEvent_t fork = nullptr, consumed = nullptr;
  hipEvent_t acc_done = nullptr;  // end of this lane's last table accumulation (msm.hip acc chain)
  int debug_sorted = 0;  // ZKMI_DEBUG_SKIP ablations only (msm.hip)
  // bin-sort counter blocks (msm.hip BsGeom): two, alternating per sort; the
  // one the last sort used (its accumulations read the item counters)
  void* bs_ctr = nullptr;
  size_t bs_ctr_words = 0;
  int bs_parity = 0;
  bool bs_dirty = false;  // a sort's kernels were not all queued: clear both blocks next time
  void* ss_clean = nullptr;   // counting-sort counts known zero in [0, ss_clean_words) (k_ss_scan clears them)
  size_t ss_clean_words = 0;
  uint32_t* bs_cur = nullptr;
};

struct KernelTimer {
  bool enabled = false;
  struct Rec {
    hipEvent_t a, b;
    std::string name;
  };
  std::vector<Rec> pending;
  std::map<std::string, std::pair<double, uint64_t>> totals;
};

}  // namespace zk

struct zkmi_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  zk::Workspace ws;
  std::vector<std::pair<void*, size_t>> pinned_free;  // pool of pinned host buffers (ptr, size)
  std::map<void*, size_t> pinned_size;                 // size of every pinned buffer handed out
  zk::KernelTimer timer;
  int msm_window = 0;  // 0 = auto
  int num_cus = 256;
  int msm_lanes = 2;  // concurrent MSM streams
  int lane_next = 0;
  std::vector<zk::MsmLane*> lanes;
  // set: MSM lanes wait on this event (recorded earlier on `stream`) instead
  // of forking from the stream's current tail (groth16 small-proof schedule)
  hipEvent_t msm_fork = nullptr;
  // the lane whose table accumulation was queued last: the next one (on another
  // lane) starts after it (msm.hip msm_acc_phase)
  zk::MsmLane* acc_last = nullptr;
  hipEvent_t prove_fork = nullptr;  // owned: the event groth16_prove_submit uses for it
  // set: the accumulation of base set acc_gate_set waits on this event
  // (groth16 large proofs: the G2 accumulation after the witness map)
  hipEvent_t acc_gate = nullptr;
  const zkmi_bases* acc_gate_set = nullptr;
  hipEvent_t wm_done = nullptr;  // owned: end of a large proof's witness map
  // Stream budget: communicators alive on this context, and the
  // streams the library holds for it (context, lanes, communicators', witness
  // programs').  While a communicator exists the lanes are capped at
  // MAX_LANES_WITH_COMM and witness programs run on the context stream, so the
  // process holds <= GPU_MAX_HW_QUEUES (4) streams and the RCCL stream never
  // shares a hardware queue with MSM work.
  int ncomm = 0;
  int nstreams = 0;
  std::vector<zkmi_wprog*> wprogs;  // live witness programs (their streams go when a communicator comes)
};
constexpr int MAX_LANES_WITH_COMM = 2;

struct zkmi_bases {
  zkmi_ctx* ctx;
  int g2;           // 0 = G1 (16 words / point), 1 = G2 (32 words / point)
  size_t n;
  uint32_t* d_pts;  // packed affine, internal Montgomery, inf flag = bit 31 of last word
  // Fixed-base table (zkmi_bases_precompute): d_pts holds tp copies of the n
  // points, copy j = 2^(tc * tw * j) * P_i (tbal: see below), so an MSM with window tc runs tw
  // windows of tp*n entries instead of tp*tw windows of n entries.
  int tc = 0;  // table window (0 = no table: plain bases, any window)
  int tp = 1;  // copies
  int tw = 0;  // windows per copy
  // 1: full table (tw = 1) with balanced window widths -- copy j is
  // 2^(offset of window j) * P_i, WinLayout<tc, true> in msm.hip
  int tbal = 0;
};

// Multi-rank communicator (zkmi.h multi-GPU section; comm.hip).
constexpr int ZKMI_COMM_RCCL = 0;
constexpr int ZKMI_COMM_HOST = 1;
struct zkmi_comm {
  zkmi_ctx* ctx = nullptr;
  uint64_t serial = 0;                  // process-unique
  int nranks = 1, rank = 0, kind = ZKMI_COMM_RCCL;
  void* nccl = nullptr;                 // ncclComm_t (RCCL transport): the sharded-MSM exchanges
  hipStream_t st = nullptr;             // every exchange, in issue order (the process's only RCCL stream)
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  zkmi_allgather_fn fn = nullptr;       // host transport
  void* user = nullptr;
  // RCCL: device buffer (fail_words = nranks x one payload) for the failure
  // exchange of a rank whose sharded MSM fails before its exchange is queued
  uint32_t* d_fail = nullptr;
  size_t fail_words = 0;
};

namespace zk {
// All-gather of `bytes` per rank from device memory, ordered after the work
// already queued on `lane_st` and before anything queued there afterwards
// (RCCL transport only).
int comm_allgather_device(zkmi_comm* c, hipStream_t lane_st, const void* d_send, void* d_recv, size_t bytes);
// Synchronous all-gather of host buffers (host transport only).
int comm_allgather_host(zkmi_comm* c, const void* send, void* recv, size_t bytes);
// windows = false: point shards (b is this rank's shard, the results are
// summed); true: window shards (b and the scalars are the whole MSM on every
// rank, each rank runs its share of the plain plan's windows)
int msm_submit_sharded(zkmi_comm* comm, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
                       zkmi_msm_job** out, bool windows = false);
// A rank whose sharded MSM fails before its exchange is queued still takes
// part in the job's exchange (`words` u32 per rank, a status block first),
// with its failure flag set, so the other ranks fail in their msm_wait instead
// of blocking in the collective.  Synchronous; issue order as the exchange.
int comm_fail_exchange(zkmi_comm* c, size_t words);
// release every witness program's own stream (after its work; wprog.hip)
void wprog_release_streams(zkmi_ctx* ctx);
// the context is being destroyed: its programs drop their streams and forget it
void wprog_detach_all(zkmi_ctx* ctx);
// words of the status block that starts every rank's sharded exchange payload
constexpr size_t SHARD_STATUS_WORDS = 4;

// HIP's current device is per host thread (default 0).  Every entry point that
// works on a context, key or base set selects that context's device for the
// duration of the call and restores the caller's device on return, so a
// context made for device k can be driven from any thread (e.g. a tokio
// blocking-pool thread) without touching GPU 0.
// a pending HIP error cleared on entry (DeviceGuard): reported on stderr (the
// first few per process), so a fault left by an earlier unchecked call is
// never lost silently
void note_cleared_error(hipError_t e, const char* fn);
struct DeviceGuard {
  int prev = -1;
  bool restore = false;
  explicit DeviceGuard(int dev, const char* fn = __builtin_FUNCTION()) {
    // an error another library (or a destructor) left in this thread's HIP
    // state must not be reported by this call's first hipGetLastError
    // (seen: "invalid device ordinal" left in the test process between two
    // contexts' lifetimes, then reported by zkmi_pk_load's launch check)
    const hipError_t pending = hipGetLastError();
    if (pending != hipSuccess) note_cleared_error(pending, fn);
    if (dev < 0) return;
    if (hipGetDevice(&prev) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    if (prev != dev && hipSetDevice(dev) == hipSuccess) restore = true;
  }
  ~DeviceGuard() {
    if (restore) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
inline int dev_of(const zkmi_ctx* c) { return c ? c->device : -1; }
inline int dev_of(const zkmi_bases* b) { return b && b->ctx ? b->ctx->device : -1; }
#define ZK_DEVICE_GUARD(obj) ::zk::DeviceGuard zk_device_guard_(::zk::dev_of(obj))

// kernel timing helpers (events on ctx->stream)
void timer_begin(zkmi_ctx* ctx, const char* name, hipEvent_t* ev, hipStream_t st);
void timer_end(zkmi_ctx* ctx, const char* name, hipEvent_t ev, hipStream_t st);
// wait = false: collect only the records whose work has finished
int timer_flush(zkmi_ctx* ctx, bool wait = true);

struct ScopedKernelTimer {
  zkmi_ctx* ctx;
  const char* name;
  hipStream_t st;
  hipEvent_t ev = nullptr;
  ScopedKernelTimer(zkmi_ctx* c, const char* n, hipStream_t s = nullptr) : ctx(c), name(n), st(s ? s : c->stream) {
    timer_begin(ctx, name, &ev, st);
  }
  ~ScopedKernelTimer() { timer_end(ctx, name, ev, st); }
};
// synchronise the context stream and every MSM lane
int ctx_sync_all(zkmi_ctx* ctx);

// pinned host staging buffers (pooled per context)
int ctx_pinned_get(zkmi_ctx* ctx, size_t bytes, void** out);
void ctx_pinned_put(zkmi_ctx* ctx, void* p);

// MSM entry (msm.hip): device scalars, result canonical affine
int msm_device(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
               uint64_t* out_affine);
int msm_submit(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
               zkmi_msm_job** job);
int msm_wait(zkmi_msm_job* job, uint64_t* out_affine);
// k MSMs sharing scalars and range over k base sets (one sort when the window
// plans agree); jobs[i] receives the job of bs[i]
int msm_submit_shared(zkmi_ctx* ctx, const zkmi_bases* const* bs, int k, size_t offset, const void* d_scalars,
                      size_t n, zkmi_msm_job** jobs);
void msm_job_free(zkmi_msm_job* job);
int bases_upload(zkmi_ctx* ctx, int g2, const uint64_t* host_affine, size_t n, zkmi_bases** out);
// convert canonical affine already in device memory (n points) into a bases set
int bases_from_device_canon(zkmi_ctx* ctx, int g2, const uint32_t* d_canon, size_t n, zkmi_bases** out);

// synthetic inputs generated in HBM (bench) and canonical export (checks)
int bases_generate(zkmi_ctx* ctx, int g2, uint64_t seed, size_t first, size_t n, zkmi_bases** out);
int bases_generate_arith_g1(zkmi_ctx* ctx, const uint64_t p0[8], const uint64_t d[8], size_t first, size_t n,
                            zkmi_bases** out);
inline int bases_generate(zkmi_ctx* ctx, int g2, uint64_t seed, size_t n, zkmi_bases** out) {
  return bases_generate(ctx, g2, seed, 0, n, out);
}
int bases_export(const zkmi_bases* b, uint64_t* host_out);
// d_out[i] = d_scalars[i] * gen: canonical scalars (8 x u32) -> canonical affine
int fixed_base_mul(zkmi_ctx* ctx, int g2, const uint64_t* gen, const uint32_t* d_scalars, size_t n, uint32_t* d_out);
int bases_precompute(zkmi_bases* b, int c, int factor);
int table_window(size_t N, int g2 = 0);
int scalars_generate(zkmi_ctx* ctx, uint64_t seed, size_t first, size_t n, void* d_out);

// NTT entry (ntt.hip): in-place on device, natural order
int ntt_device(zkmi_ctx* ctx, uint32_t* d_data, uint32_t log_n, int inverse, int coset);
// per-log_n NTT domain tables (Montgomery): g^x = lo[x mod 2^KB] * hi[x >> KB]
constexpr uint32_t COSET_KB = 14;
struct DomainCache {
  uint32_t* consts;  // [n^-1 canon | (g^n - 1)^-1 mont | n^-1 mont]
  uint32_t* ninv_m;  // = consts + 16
  uint32_t *lo_g, *hi_g, *lo_gi, *hi_gi;  // hi_g / hi_gi carry the factor n^-1
  uint32_t* hi_gf;                        // g^(h 2^KB) without n^-1
};
int domain_cache(zkmi_ctx* ctx, uint32_t logn, DomainCache* dc);

}  // namespace zk
