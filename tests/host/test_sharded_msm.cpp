// test_sharded_msm.cpp — two ranks drive a point-sharded BN254 G1 MSM through
// include/zkmi.h alone (no torch, no Python): the C++ host a maintainer would
// write over the boundary.  Built by zelana_amd/
// build_native.py into zelana_amd/test_sharded_msm; run by
// tests/test_gpu_multi.py on the GPU box.
//
//   test_sharded_msm [dev0 dev1]
//
// The process forks into rank 0 and rank 1 BEFORE any HIP call.  Each rank
// owns the shard zkmi_shard_range(total, 2, rank) of one global synthetic set
// (zkmi_bases_generate_range_g1 / zkmi_scalars_generate_range), and the
// sharded MSM must equal the 1-rank MSM over the whole set, which every rank
// also computes.  Transports:
//   * host: the all-gather callback runs over a pipe pair (ranks may share one
//     GPU, as on a 1-GPU box: RCCL refuses two ranks on one device);
//   * RCCL: when dev0 != dev1 (the unique id travels over the pipe).
// Cases: plain and fixed-base-table shards, a ragged total, an empty shard,
// window plans that differ between the ranks (a table on one rank only, or a
// window pinned on one rank only, with MSMs of an agreed plan before it: must
// fail on both ranks, never hang), several MSMs in flight over one shard
// (host transport: exactly one all-gather per MSM), local-check failures and
// an injected failure.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <vector>

#include "zkmi.h"

namespace {

struct Link {
  int rank, wr, rd;
  int calls = 0;  // host all-gathers issued (plan headers + bit-sum exchanges)
};

bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = write(fd, c, n);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
bool read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = read(fd, c, n);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

// zkmi_allgather_fn over the pipe pair: rank 0 writes first, rank 1 reads
// first, so neither blocks on a full pipe.
int pipe_allgather(void* user, const void* send, void* recv, size_t bytes) {
  Link* l = (Link*)user;
  l->calls++;
  char* out = (char*)recv;
  memcpy(out + (size_t)l->rank * bytes, send, bytes);
  char* peer = out + (size_t)(1 - l->rank) * bytes;
  if (l->rank == 0) {
    if (!write_all(l->wr, send, bytes) || !read_all(l->rd, peer, bytes)) return 1;
  } else {
    if (!read_all(l->rd, peer, bytes) || !write_all(l->wr, send, bytes)) return 1;
  }
  return 0;
}

int g_fail = 0;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      fprintf(stderr, "[rank %d] FAIL %s:%d: ", rank, __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, " (%s)\n", zkmi_last_error());      \
      g_fail++;                                           \
    }                                                     \
  } while (0)

// the whole set on this rank's GPU: the reference result
bool full_msm(zkmi_ctx* ctx, uint64_t pseed, uint64_t sseed, size_t total, uint64_t out[8]) {
  zkmi_bases* b = nullptr;
  void* d = nullptr;
  bool ok = zkmi_bases_generate_range_g1(ctx, pseed, 0, total, &b) == 0 &&
            zkmi_dev_alloc(ctx, total * 32 + 32, &d) == 0 &&
            zkmi_scalars_generate_range(ctx, sseed, 0, total, d) == 0 &&
            zkmi_msm_g1_device(ctx, b, 0, d, total, out) == 0;
  if (d) zkmi_dev_free(ctx, d);
  zkmi_bases_destroy(b);
  return ok;
}

// one sharded MSM; table: precompute the shard's fixed-base table first
int sharded_msm(zkmi_comm* comm, zkmi_ctx* ctx, int rank, uint64_t pseed, uint64_t sseed, size_t total, bool table,
                uint64_t out[8]) {
  size_t first = 0, count = 0;
  if (zkmi_shard_range(total, 2, rank, &first, &count)) return -100;
  zkmi_bases* b = nullptr;
  void* d = nullptr;
  int rc = zkmi_bases_generate_range_g1(ctx, pseed, first, count, &b);
  if (!rc) rc = zkmi_dev_alloc(ctx, count * 32 + 32, &d);
  if (!rc && count) rc = zkmi_scalars_generate_range(ctx, sseed, first, count, d);
  if (!rc && table && count) rc = zkmi_bases_precompute(b, 0, 0);
  if (!rc) rc = zkmi_msm_sharded(comm, b, 0, d, count, out);
  if (d) zkmi_dev_free(ctx, d);
  zkmi_bases_destroy(b);
  return rc;
}

int run_rank(int rank, int dev, Link link, bool use_rccl) {
  const int& link_calls = link.calls;
  zkmi_ctx* ctx = nullptr;
  if (zkmi_ctx_create(dev, &ctx)) {
    fprintf(stderr, "[rank %d] zkmi_ctx_create(%d): %s\n", rank, dev, zkmi_last_error());
    return 2;
  }
  zkmi_comm* comm = nullptr;
  if (use_rccl) {
    uint8_t id[ZKMI_COMM_ID_BYTES];
    if (rank == 0) {
      CHECK(zkmi_comm_unique_id(id) == 0, "unique id");
      CHECK(write_all(link.wr, id, sizeof(id)), "send id");
    } else {
      CHECK(read_all(link.rd, id, sizeof(id)), "recv id");
    }
    CHECK(zkmi_comm_init(ctx, id, 2, rank, &comm) == 0, "zkmi_comm_init");
  } else {
    CHECK(zkmi_comm_init_host(ctx, 2, rank, pipe_allgather, &link, &comm) == 0, "zkmi_comm_init_host");
  }
  if (!comm) return 3;
  int info[3];
  CHECK(zkmi_comm_info(comm, info) == 0 && info[0] == 2 && info[1] == rank && info[2] == (use_rccl ? 0 : 1),
        "comm info");
  struct Case {
    size_t total;
    bool table;
    uint64_t pseed, sseed;
  } cases[] = {
      {1u << 16, false, 1026, 26},            // equal shards, plain Pippenger
      {(1u << 16) + 3, false, 7, 8},          // ragged: shards differ by one point
      {1u << 18, true, 1026, 26},             // fixed-base tables on both shards
      {1, false, 11, 12},                     // rank 1's shard is empty
  };
  for (const Case& k : cases) {
    uint64_t got[8] = {0}, want[8] = {0};
    int rc = sharded_msm(comm, ctx, rank, k.pseed, k.sseed, k.total, k.table, got);
    CHECK(rc == 0, "sharded MSM total %zu table %d rc %d", k.total, (int)k.table, rc);
    CHECK(full_msm(ctx, k.pseed, k.sseed, k.total, want), "full MSM total %zu", k.total);
    CHECK(memcmp(got, want, sizeof(got)) == 0, "sharded != global MSM (total %zu, table %d)", k.total, (int)k.table);
    if (rank == 0) printf("case total=%zu table=%d: %s\n", k.total, (int)k.table, memcmp(got, want, 64) ? "MISMATCH" : "ok");
  }
  // one shard, several MSMs in flight: every sharded MSM is exactly one
  // exchange (no plan-agreement collective); pinning another window on both
  // ranks changes the plan everywhere
  {
    const size_t total = (1u << 17) + 5;
    size_t first = 0, count = 0;
    zkmi_shard_range(total, 2, rank, &first, &count);
    zkmi_bases* b = nullptr;
    void* d = nullptr;
    CHECK(zkmi_bases_generate_range_g1(ctx, 21, first, count, &b) == 0 &&
              zkmi_dev_alloc(ctx, count * 32 + 32, &d) == 0 &&
              zkmi_scalars_generate_range(ctx, 22, first, count, d) == 0,
          "inputs");
    uint64_t want[8] = {0};
    CHECK(full_msm(ctx, 21, 22, total, want), "full MSM");
    for (int win : {0, 15}) {
      CHECK(zkmi_msm_set_window(ctx, win) == 0, "set window %d", win);
      const int calls0 = link_calls;
      zkmi_msm_job* jobs[3] = {nullptr, nullptr, nullptr};
      for (auto& j : jobs) CHECK(zkmi_msm_sharded_submit(comm, b, 0, d, count, &j) == 0, "submit");
      for (auto& j : jobs) {
        uint64_t got[8] = {0};
        CHECK(j && zkmi_msm_wait(j, got) == 0 && memcmp(got, want, sizeof(got)) == 0,
              "pipelined sharded MSM (window %d) != global", win);
      }
      if (!use_rccl)  // three exchanges, nothing else
        CHECK(link_calls - calls0 == 3, "window %d: %d host all-gathers for 3 MSMs", win, link_calls - calls0);
    }
    // a rank-local failure between two good MSMs in flight: the
    // failure joins its own job's exchange -- over the host transport in
    // zkmi_msm_wait, in wait order -- so the jobs around it stay correct on
    // both ranks and the failed one fails on both
    {
      zkmi_msm_job *j0 = nullptr, *j1 = nullptr, *j2 = nullptr;
      CHECK(zkmi_msm_sharded_submit(comm, b, 0, d, count, &j0) == 0, "submit before the failure");
      setenv("ZKMI_DEBUG_SHARD_FAIL", "0", 1);
      int rc1 = zkmi_msm_sharded_submit(comm, b, 0, d, count, &j1);
      unsetenv("ZKMI_DEBUG_SHARD_FAIL");
      CHECK(zkmi_msm_sharded_submit(comm, b, 0, d, count, &j2) == 0, "submit after the failure");
      uint64_t got[8] = {0};
      CHECK(j0 && zkmi_msm_wait(j0, got) == 0 && memcmp(got, want, sizeof(got)) == 0,
            "rank %d: the MSM before the in-flight failure != global", rank);
      if (rc1 == 0) rc1 = zkmi_msm_wait(j1, got);
      CHECK(rc1 != 0, "in-flight failure injected on rank 0: rank %d returned %d", rank, rc1);
      memset(got, 0, sizeof(got));
      CHECK(j2 && zkmi_msm_wait(j2, got) == 0 && memcmp(got, want, sizeof(got)) == 0,
            "rank %d: the MSM after the in-flight failure != global", rank);
    }
    // the window changes on rank 1 only, after MSMs of one plan ran: both
    // ranks fail (no rank waits in a collective the other skipped), and the
    // communicator stays in step
    CHECK(zkmi_msm_set_window(ctx, rank == 1 ? 11 : 0) == 0, "set window");  // auto = 13 at this shard size
    {
      zkmi_msm_job* j = nullptr;
      uint64_t got[8] = {0};
      int rc = zkmi_msm_sharded_submit(comm, b, 0, d, count, &j);
      if (rc == 0) rc = zkmi_msm_wait(j, got);
      CHECK(rc == ZKMI_EINVAL, "window changed on rank 1 only: rank %d returned %d", rank, rc);
    }
    CHECK(zkmi_msm_set_window(ctx, 0) == 0, "set window 0");
    {
      uint64_t got[8] = {0};
      CHECK(zkmi_msm_sharded(comm, b, 0, d, count, got) == 0 && memcmp(got, want, sizeof(got)) == 0,
            "sharded MSM after the one-rank window change != global");
    }
    zkmi_dev_free(ctx, d);
    zkmi_bases_destroy(b);
    if (rank == 0) printf("pipelined + one-rank window change: ok\n");
  }
  // different window plans on the two ranks must fail on BOTH ranks
  {
    uint64_t got[8];
    int rc = sharded_msm(comm, ctx, rank, 3, 4, 1u << 17, rank == 0, got);
    CHECK(rc == ZKMI_EINVAL, "mismatched plans returned %d", rc);
  }
  // a rank that fails its local checks (range outside its base set) fails the
  // MSM on BOTH ranks, and neither blocks in a collective
  {
    size_t first = 0, count = 0;
    zkmi_shard_range(1u << 16, 2, rank, &first, &count);
    zkmi_bases* b = nullptr;
    void* d = nullptr;
    CHECK(zkmi_bases_generate_range_g1(ctx, 5, first, count, &b) == 0 && zkmi_dev_alloc(ctx, count * 32 + 32, &d) == 0 &&
              zkmi_scalars_generate_range(ctx, 6, first, count, d) == 0,
          "inputs");
    uint64_t got[8];
    int rc = zkmi_msm_sharded(comm, b, rank == 1 ? 1 : 0, d, count, got);  // rank 1: [1, count + 1) out of range
    CHECK(rc == ZKMI_EINVAL, "bad range on rank 1: rank %d returned %d", rank, rc);
    // a failure after the plan agreement (injected on rank 0): both fail
    setenv("ZKMI_DEBUG_SHARD_FAIL", "0", 1);
    rc = zkmi_msm_sharded(comm, b, 0, d, count, got);
    unsetenv("ZKMI_DEBUG_SHARD_FAIL");
    CHECK(rc != 0, "injected failure on rank 0: rank %d returned %d", rank, rc);
    zkmi_dev_free(ctx, d);
    zkmi_bases_destroy(b);
    // the communicator is still in step: a good MSM follows
    uint64_t want[8] = {0};
    rc = sharded_msm(comm, ctx, rank, 1026, 26, 1u << 16, false, got);
    CHECK(rc == 0 && full_msm(ctx, 1026, 26, 1u << 16, want) && memcmp(got, want, sizeof(got)) == 0,
          "sharded MSM after the failures (rc %d)", rc);
    if (rank == 0) printf("failure cases: ok\n");
  }
  zkmi_comm_destroy(comm);
  zkmi_ctx_destroy(ctx);
  return g_fail ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  int dev0 = argc > 2 ? atoi(argv[1]) : 0, dev1 = argc > 2 ? atoi(argv[2]) : 0;
  const bool rccl = dev0 != dev1;
  int p01[2], p10[2];
  if (pipe(p01) || pipe(p10)) {
    perror("pipe");
    return 2;
  }
  fflush(stdout);
  pid_t pid = fork();  // before any HIP call: a forked child cannot use a parent's GPU context
  if (pid < 0) {
    perror("fork");
    return 2;
  }
  if (pid == 0) {
    close(p01[1]);
    close(p10[0]);
    int rc = run_rank(1, dev1, Link{1, p10[1], p01[0]}, rccl);
    fflush(stdout);
    _exit(rc);
  }
  close(p01[0]);
  close(p10[1]);
  int rc0 = run_rank(0, dev0, Link{0, p01[1], p10[0]}, rccl);
  close(p01[1]);
  close(p10[0]);
  int st = 0;
  waitpid(pid, &st, 0);
  int rc1 = WIFEXITED(st) ? WEXITSTATUS(st) : 100;
  printf("%s transport: rank0 %s, rank1 %s\n", rccl ? "RCCL" : "host", rc0 ? "FAIL" : "PASS", rc1 ? "FAIL" : "PASS");
  return rc0 || rc1 ? 1 : 0;
}
