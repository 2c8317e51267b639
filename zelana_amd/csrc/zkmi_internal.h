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
  std::vector<std::pair<void*, size_t>> pinned_free;  // pool of pinned host buffers
  zk::KernelTimer timer;
  int msm_window = 0;  // 0 = auto
  int num_cus = 256;
};

struct zkmi_bases {
  zkmi_ctx* ctx;
  int g2;           // 0 = G1 (16 words / point), 1 = G2 (32 words / point)
  size_t n;
  uint32_t* d_pts;  // packed affine, internal Montgomery, inf flag = bit 31 of last word
};

namespace zk {
// kernel timing helpers (events on ctx->stream)
void timer_begin(zkmi_ctx* ctx, const char* name, hipEvent_t* ev);
void timer_end(zkmi_ctx* ctx, const char* name, hipEvent_t ev);
int timer_flush(zkmi_ctx* ctx);

struct ScopedKernelTimer {
  zkmi_ctx* ctx;
  const char* name;
  hipEvent_t ev = nullptr;
  ScopedKernelTimer(zkmi_ctx* c, const char* n) : ctx(c), name(n) { timer_begin(ctx, name, &ev); }
  ~ScopedKernelTimer() { timer_end(ctx, name, ev); }
};

// pinned host staging buffers (pooled per context)
int ctx_pinned_get(zkmi_ctx* ctx, size_t bytes, void** out);
void ctx_pinned_put(zkmi_ctx* ctx, void* p);

// MSM entry (msm.hip): device scalars, result canonical affine
int msm_device(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
               uint64_t* out_affine);
int msm_submit(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
               zkmi_msm_job** job);
int msm_wait(zkmi_msm_job* job, uint64_t* out_affine);
void msm_job_free(zkmi_msm_job* job);
int bases_upload(zkmi_ctx* ctx, int g2, const uint64_t* host_affine, size_t n, zkmi_bases** out);
// convert canonical affine already in device memory (n points) into a bases set
int bases_from_device_canon(zkmi_ctx* ctx, int g2, const uint32_t* d_canon, size_t n, zkmi_bases** out);

// synthetic inputs generated in HBM (bench) and canonical export (checks)
int bases_generate(zkmi_ctx* ctx, int g2, uint64_t seed, size_t n, zkmi_bases** out);
int bases_export(const zkmi_bases* b, uint64_t* host_out);
int scalars_generate(zkmi_ctx* ctx, uint64_t seed, size_t n, void* d_out);

// NTT entry (ntt.hip): in-place on device, natural order
int ntt_device(zkmi_ctx* ctx, uint32_t* d_data, uint32_t log_n, int inverse, int coset);

}  // namespace zk
