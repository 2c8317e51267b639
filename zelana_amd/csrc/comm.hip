// comm.hip — multi-rank communicator of libzkmi.so (include/zkmi.h, multi-GPU
// section): the one exchange step of a point-sharded MSM.
//
// The reference has no collective at all (its only scale-out is independent
// proof chunks per worker, forge/crates/prover-coordinator/src/dispatcher.rs:
// 134,290); north_star asks for an RCCL exchange of partial bucket sums over
// xGMI.  RCCL has no elliptic-curve reduction, so the exchange is an
// ncclAllGather of every rank's bit sums (tens of KB) followed by the
// group-law sum in the MSM epilogue (msm.hip msm_wait).
//
// Ordering: every collective of a communicator is issued on its own stream
// `st`, in host issue order, so MSMs running on different lanes can never
// reach RCCL in different orders on different ranks.  The lane that produced
// the bit sums hands them over with an event pair (lane -> comm stream ->
// lane), so the all-gather sits between the bucket reduction and the D2H of
// the same lane with no host round trip.
#include <string.h>

#include <atomic>
#include <vector>

#include <rccl/rccl.h>

#include "zkmi_internal.h"

namespace zk {

#define ZK_NCCL(expr)                                                                              \
  do {                                                                                             \
    ncclResult_t r_ = (expr);                                                                      \
    if (r_ != ncclSuccess) {                                                                       \
      ::zk::set_error("RCCL error %s at %s:%d (%s)", ncclGetErrorString(r_), __FILE__, __LINE__, #expr); \
      return ZKMI_EHIP;                                                                            \
    }                                                                                              \
  } while (0)

int comm_allgather_device(zkmi_comm* c, hipStream_t lane_st, const void* d_send, void* d_recv, size_t bytes) {
  if (c->kind != ZKMI_COMM_RCCL) {
    set_error("comm_allgather_device: host-transport communicator");
    return ZKMI_EINVAL;
  }
  ZK_HIP(hipEventRecord(c->ev_in, lane_st));
  ZK_HIP(hipStreamWaitEvent(c->st, c->ev_in, 0));
  {
    ScopedKernelTimer tm(c->ctx, "msm_exchange", c->st);  // per-rank exchange time (zkmi_profile)
    ZK_NCCL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, (ncclComm_t)c->nccl, c->st));
  }
  ZK_HIP(hipEventRecord(c->ev_out, c->st));
  ZK_HIP(hipStreamWaitEvent(lane_st, c->ev_out, 0));
  return 0;
}

int comm_allgather_host(zkmi_comm* c, const void* send, void* recv, size_t bytes) {
  if (c->kind != ZKMI_COMM_HOST) {
    set_error("comm_allgather_host: RCCL communicator (its exchanges run on the device)");
    return ZKMI_EINVAL;
  }
  int rc = c->fn(c->user, send, recv, bytes);
  if (rc) {
    set_error("host all-gather callback failed (%d)", rc);
    return ZKMI_EINVAL;
  }
  return 0;
}

// A failed rank's payload: zeros with the failure flag (word 0 of the status
// block) set, in the same one exchange its peers run.
int comm_fail_exchange(zkmi_comm* c, size_t words) {
  if (c->kind == ZKMI_COMM_HOST) {
    std::vector<uint32_t> me(words, 0), all(words * (size_t)c->nranks);
    me[0] = 1;
    return c->fn(c->user, me.data(), all.data(), words * 4) ? ZKMI_EINVAL : 0;
  }
  const size_t need = words * (size_t)c->nranks;
  if (need > c->fail_words) {  // beyond the buffer sized at init: best effort
    uint32_t* d = nullptr;
    if (hipMalloc((void**)&d, need * 4) != hipSuccess) {
      (void)hipGetLastError();
      return ZKMI_ENOMEM;
    }
    if (c->d_fail) (void)hipFree(c->d_fail);
    c->d_fail = d;
    c->fail_words = need;
  }
  uint32_t* mine = c->d_fail + words * (size_t)c->rank;
  const uint32_t one = 1;
  ZK_HIP(hipMemsetAsync(mine, 0, words * 4, c->st));
  ZK_HIP(hipMemcpyAsync(mine, &one, 4, hipMemcpyHostToDevice, c->st));
  ZK_NCCL(ncclAllGather(mine, c->d_fail, words * 4, ncclUint8, (ncclComm_t)c->nccl, c->st));
  ZK_HIP(hipStreamSynchronize(c->st));
  return 0;
}

static int comm_new(zkmi_ctx* ctx, int nranks, int rank, int kind, zkmi_comm** out) {
  if (!ctx || !out || nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("zkmi_comm_init: bad arguments (nranks %d, rank %d)", nranks, rank);
    return ZKMI_EINVAL;
  }
  static std::atomic<uint64_t> next_serial{1};
  zkmi_comm* c = new zkmi_comm;
  c->ctx = ctx;
  c->serial = next_serial++;
  c->nranks = nranks;
  c->rank = rank;
  c->kind = kind;
  // counted from here on; zkmi_comm_destroy uncounts a communicator with a stream
  if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) == hipSuccess) {
    ctx->nstreams++;
    ctx->ncomm++;
  } else {
    c->st = nullptr;
  }
  if (!c->st || hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    zkmi_comm_destroy(c);
    set_error("zkmi_comm_init: cannot create the communicator's stream / events");
    return ZKMI_EHIP;
  }
  // Stream budget: beside a communicator the context keeps at most
  // MAX_LANES_WITH_COMM lanes; lanes created before it beyond that go (after
  // their work), so context + lanes + this stream <= GPU_MAX_HW_QUEUES.
  if (ctx->msm_lanes > MAX_LANES_WITH_COMM) ctx->msm_lanes = MAX_LANES_WITH_COMM;
  if ((int)ctx->lanes.size() > MAX_LANES_WITH_COMM) {
    (void)ctx_sync_all(ctx);
    while ((int)ctx->lanes.size() > MAX_LANES_WITH_COMM) {
      MsmLane* l = ctx->lanes.back();
      ctx->lanes.pop_back();
      if (ctx->acc_last == l) ctx->acc_last = nullptr;
      l->ws.release_all();
      (void)hipEventDestroy(l->fork);
      (void)hipEventDestroy(l->consumed);
      (void)hipEventDestroy(l->acc_done);
      (void)hipStreamDestroy(l->st);
      delete l;
      ctx->nstreams--;
    }
    ctx->lane_next = 0;
  }
  wprog_release_streams(ctx);  // witness programs run on the context stream from here on
  *out = c;
  return 0;
}

}  // namespace zk

using namespace zk;

extern "C" {

int zkmi_comm_unique_id(uint8_t id[ZKMI_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == ZKMI_COMM_ID_BYTES, "ncclUniqueId size");
  if (!id) {
    set_error("zkmi_comm_unique_id: null id");
    return ZKMI_EINVAL;
  }
  ncclUniqueId u;
  ZK_NCCL(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return 0;
}

int zkmi_comm_init(zkmi_ctx* ctx, const uint8_t id[ZKMI_COMM_ID_BYTES], int nranks, int rank, zkmi_comm** out) {
  ZK_DEVICE_GUARD(ctx);
  if (!id) {
    set_error("zkmi_comm_init: null id");
    return ZKMI_EINVAL;
  }
  zkmi_comm* c = nullptr;
  ZK_TRY(comm_new(ctx, nranks, rank, ZKMI_COMM_RCCL, &c));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t nc = nullptr;
  ncclResult_t r = ncclCommInitRank(&nc, nranks, u, rank);
  if (r != ncclSuccess) {
    set_error("ncclCommInitRank(nranks %d, rank %d) on device %d: %s", nranks, rank, ctx->device,
              ncclGetErrorString(r));
    zkmi_comm_destroy(c);
    return ZKMI_EHIP;
  }
  c->nccl = nc;
  // failure-exchange buffer: one sharded payload per rank (msm.hip
  // SHARD_PAYLOAD_WORDS = 36,864 words)
  c->fail_words = (size_t)36864 * nranks;
  if (hipMalloc((void**)&c->d_fail, c->fail_words * 4) != hipSuccess) {
    (void)hipGetLastError();
    set_error("zkmi_comm_init: cannot allocate the failure-exchange buffer");
    zkmi_comm_destroy(c);
    return ZKMI_ENOMEM;
  }
  *out = c;
  return 0;
}

int zkmi_comm_init_host(zkmi_ctx* ctx, int nranks, int rank, zkmi_allgather_fn allgather, void* user,
                        zkmi_comm** out) {
  ZK_DEVICE_GUARD(ctx);
  if (!allgather) {
    set_error("zkmi_comm_init_host: null all-gather callback");
    return ZKMI_EINVAL;
  }
  zkmi_comm* c = nullptr;
  ZK_TRY(comm_new(ctx, nranks, rank, ZKMI_COMM_HOST, &c));
  c->fn = allgather;
  c->user = user;
  *out = c;
  return 0;
}

void zkmi_comm_destroy(zkmi_comm* c) {
  if (!c) return;
  ZK_DEVICE_GUARD(c->ctx);
  if (c->st) {
    (void)hipStreamSynchronize(c->st);
    c->ctx->nstreams--;
    c->ctx->ncomm--;
  }
  if (c->nccl) ncclCommDestroy((ncclComm_t)c->nccl);
  if (c->d_fail) (void)hipFree(c->d_fail);
  if (c->ev_in) (void)hipEventDestroy(c->ev_in);
  if (c->ev_out) (void)hipEventDestroy(c->ev_out);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
}

int zkmi_comm_info(const zkmi_comm* c, int out[3]) {
  if (!c || !out) {
    set_error("zkmi_comm_info: null argument");
    return ZKMI_EINVAL;
  }
  out[0] = c->nranks;
  out[1] = c->rank;
  out[2] = c->kind;
  return 0;
}

int zkmi_shard_range(size_t total, int nranks, int rank, size_t* first, size_t* count) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !first || !count) {
    set_error("zkmi_shard_range: bad arguments");
    return ZKMI_EINVAL;
  }
  const size_t q = total / (size_t)nranks, rem = total % (size_t)nranks, r = (size_t)rank;
  *first = r * q + (r < rem ? r : rem);
  *count = q + (r < rem ? 1 : 0);
  return 0;
}

int zkmi_msm_sharded_submit(zkmi_comm* comm, const zkmi_bases* shard, size_t offset, const void* d_scalars,
                            size_t n, zkmi_msm_job** job) {
  if (!comm || !shard || !job || (n && !d_scalars)) {
    set_error("zkmi_msm_sharded_submit: bad arguments");
    return ZKMI_EINVAL;
  }
  ZK_DEVICE_GUARD(comm->ctx);
  return msm_submit_sharded(comm, shard, offset, d_scalars, n, job);
}

int zkmi_msm_window_sharded_submit(zkmi_comm* comm, const zkmi_bases* bases, size_t offset, const void* d_scalars,
                                   size_t n, zkmi_msm_job** job) {
  if (!comm || !bases || !job || (n && !d_scalars)) {
    set_error("zkmi_msm_window_sharded_submit: bad arguments");
    return ZKMI_EINVAL;
  }
  ZK_DEVICE_GUARD(comm->ctx);
  return msm_submit_sharded(comm, bases, offset, d_scalars, n, job, true);
}

int zkmi_msm_sharded(zkmi_comm* comm, const zkmi_bases* shard, size_t offset, const void* d_scalars, size_t n,
                     uint64_t* out_affine) {
  zkmi_msm_job* job = nullptr;
  ZK_TRY(zkmi_msm_sharded_submit(comm, shard, offset, d_scalars, n, &job));
  return zkmi_msm_wait(job, out_affine);
}

}  // extern "C"
