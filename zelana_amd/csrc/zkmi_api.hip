// zkmi_api.hip — the extern "C" boundary of libzkmi.so (include/zkmi.h):
// context / device memory, kernel timing, MSM and NTT entry points, encodings.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include <atomic>

#include "zkmi_internal.h"

namespace zk {

static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void note_cleared_error(hipError_t e, const char* fn) {
  static std::atomic<int> seen{0};
  if (seen.fetch_add(1) < 8)
    fprintf(stderr, "libzkmi: %s entered with a pending HIP error (%s); cleared\n", fn ? fn : "?",
            hipGetErrorString(e));
}


int Workspace::get(const char* name, size_t bytes, void** out) {
  auto it = bufs.find(name);
  if (it != bufs.end() && it->second.second >= bytes) {
    *out = it->second.first;
    return 0;
  }
  if (it != bufs.end()) {
    hipFree(it->second.first);
    bufs.erase(it);
  }
  void* p = nullptr;
  size_t sz = bytes < 256 ? 256 : bytes;
  if (hipMalloc(&p, sz) != hipSuccess) {
    (void)hipGetLastError();
    set_error("workspace '%s': hipMalloc(%zu) failed", name, sz);
    return ZKMI_ENOMEM;
  }
  bufs[name] = {p, sz};
  *out = p;
  return 0;
}
void Workspace::release_all() {
  for (auto& kv : bufs) hipFree(kv.second.first);
  bufs.clear();
}

void timer_begin(zkmi_ctx* ctx, const char* name, hipEvent_t* ev, hipStream_t st) {
  *ev = nullptr;
  if (!ctx->timer.enabled) return;
  if (hipEventCreate(ev) != hipSuccess) {
    *ev = nullptr;
    return;
  }
  hipEventRecord(*ev, st);
}
void timer_end(zkmi_ctx* ctx, const char* name, hipEvent_t ev, hipStream_t st) {
  if (!ctx->timer.enabled || !ev) return;
  hipEvent_t e2;
  if (hipEventCreate(&e2) != hipSuccess) return;
  hipEventRecord(e2, st);
  ctx->timer.pending.push_back({ev, e2, name});
}
int timer_flush(zkmi_ctx* ctx, bool wait) {
  if (ctx->timer.pending.empty()) return 0;
  std::vector<KernelTimer::Rec> keep;
  for (auto& r : ctx->timer.pending) {
    if (!wait && hipEventQuery(r.b) != hipSuccess) {
      keep.push_back(r);
      continue;
    }
    ZK_HIP(hipEventSynchronize(r.b));
    float ms = 0;
    hipEventElapsedTime(&ms, r.a, r.b);
    auto& t = ctx->timer.totals[r.name];
    t.first += ms;
    t.second += 1;
    hipEventDestroy(r.a);
    hipEventDestroy(r.b);
  }
  ctx->timer.pending.swap(keep);
  return 0;
}
int ctx_sync_all(zkmi_ctx* ctx) {
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  for (auto* l : ctx->lanes) ZK_HIP(hipStreamSynchronize(l->st));
  return 0;
}

// Pinned staging buffers, pooled per context (a context is single-threaded,
// so its pool needs no lock; two contexts never share one).
int ctx_pinned_get(zkmi_ctx* ctx, size_t bytes, void** out) {
  for (size_t i = 0; i < ctx->pinned_free.size(); i++) {
    if (ctx->pinned_free[i].second >= bytes) {
      *out = ctx->pinned_free[i].first;
      ctx->pinned_free.erase(ctx->pinned_free.begin() + i);
      return 0;
    }
  }
  size_t sz = bytes < 4096 ? 4096 : bytes;
  if (hipHostMalloc(out, sz, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    set_error("hipHostMalloc(%zu) failed", sz);
    return ZKMI_ENOMEM;
  }
  ctx->pinned_size[*out] = sz;
  return 0;
}
void ctx_pinned_put(zkmi_ctx* ctx, void* p) {
  auto it = ctx->pinned_size.find(p);
  ctx->pinned_free.push_back({p, it == ctx->pinned_size.end() ? 0 : it->second});
}

}  // namespace zk

using namespace zk;

extern "C" {

const char* zkmi_last_error(void) { return g_err; }
int zkmi_version(void) { return 1; }

int zkmi_ctx_create(int device, zkmi_ctx** out) {
  if (!out) {
    set_error("zkmi_ctx_create: null out");
    return ZKMI_EINVAL;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    set_error("no HIP device available (libzkmi has no CPU fallback)");
    return ZKMI_ENODEV;
  }
  if (device < 0 || device >= ndev) {
    set_error("device %d out of range (%d devices)", device, ndev);
    return ZKMI_ENODEV;
  }
  hipDeviceProp_t prop;
  ZK_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error("device %d is %s; libzkmi is built for gfx950 (MI355X) only", device, prop.gcnArchName);
    return ZKMI_ENODEV;
  }
  DeviceGuard guard(device);  // the stream belongs to `device`; the caller's device is restored
  zkmi_ctx* c = new zkmi_ctx;
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  // The context stream carries a proof's witness map (mat-vecs, 7 NTTs, the
  // QAP step), the critical path to the h MSM, while the lanes run the
  // z-weighted MSMs beside it.  The G2 accumulation holds 248 VGPRs, two
  // waves per SIMD, so an NTT wave gets a SIMD only when an accumulation wave
  // retires; at the highest queue priority the dispatcher hands it that slot
  // first (round 6 trace: NTT passes of 2.4-4.1 ms beside the G2 accumulation
  // against ~0.2 ms alone).  Measured (tools/r06_ab2.sh, 2 repeats): 2^22
  // proofs 33.3-33.4 -> 34.0/s, two in flight 33.7 -> 34.6-35.0/s; batch 70
  // resident 81.5-81.6 -> 82.2-82.3/s, end to end (4 per witness run)
  // 78.8-78.9 -> 80.3-81.0/s.
#ifndef ZK_CTX_PRIO
#define ZK_CTX_PRIO 1
#endif
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, ZK_CTX_PRIO ? prio_hi : prio_lo) != hipSuccess) {
    delete c;
    set_error("hipStreamCreate failed");
    return ZKMI_EHIP;
  }
  c->nstreams = 1;
  *out = c;
  return 0;
}
void zkmi_ctx_destroy(zkmi_ctx* ctx) {
  if (!ctx) return;
  ZK_DEVICE_GUARD(ctx);
  ctx_sync_all(ctx);
  timer_flush(ctx);
  wprog_detach_all(ctx);
  ctx->ws.release_all();
  for (auto* l : ctx->lanes) {
    l->ws.release_all();
    hipEventDestroy(l->fork);
    hipEventDestroy(l->consumed);
    hipEventDestroy(l->acc_done);
    hipStreamDestroy(l->st);
    delete l;
  }
  ctx->lanes.clear();
  ctx->nstreams = 1;
  if (ctx->prove_fork) hipEventDestroy(ctx->prove_fork);
  if (ctx->wm_done) hipEventDestroy(ctx->wm_done);
  for (auto& pb : ctx->pinned_free) hipHostFree(pb.first);
  ctx->pinned_free.clear();
  ctx->pinned_size.clear();
  hipStreamDestroy(ctx->stream);
  delete ctx;
}
int zkmi_profile_enable(zkmi_ctx* ctx, int on) {
  ctx->timer.enabled = on != 0;
  return 0;
}
int zkmi_profile_get(zkmi_ctx* ctx, const char* name, double* total_ms, uint64_t* count) {
  ZK_DEVICE_GUARD(ctx);
  ZK_TRY(timer_flush(ctx));
  auto it = ctx->timer.totals.find(name);
  *total_ms = it == ctx->timer.totals.end() ? 0.0 : it->second.first;
  *count = it == ctx->timer.totals.end() ? 0 : it->second.second;
  return 0;
}
int zkmi_profile_reset(zkmi_ctx* ctx) {
  ZK_DEVICE_GUARD(ctx);
  ZK_TRY(timer_flush(ctx));
  ctx->timer.totals.clear();
  return 0;
}
int zkmi_dev_alloc(zkmi_ctx* ctx, size_t bytes, void** dptr) {
  ZK_DEVICE_GUARD(ctx);
  if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess) {
    (void)hipGetLastError();
    set_error("hipMalloc(%zu) failed", bytes);
    return ZKMI_ENOMEM;
  }
  return 0;
}
int zkmi_dev_free(zkmi_ctx* ctx, void* dptr) {
  ZK_DEVICE_GUARD(ctx);
  ZK_HIP(hipFree(dptr));
  return 0;
}
int zkmi_h2d(zkmi_ctx* ctx, void* dst, const void* src, size_t bytes) {
  ZK_DEVICE_GUARD(ctx);
  ZK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  return 0;
}
int zkmi_d2h(zkmi_ctx* ctx, void* dst, const void* src, size_t bytes) {
  ZK_DEVICE_GUARD(ctx);
  ZK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  return 0;
}
int zkmi_sync(zkmi_ctx* ctx) {
  ZK_DEVICE_GUARD(ctx);
  return ctx_sync_all(ctx);
}

// ------------------------------------------------------------------ MSM
int zkmi_bases_create_g1(zkmi_ctx* ctx, const uint64_t* affine, size_t n, zkmi_bases** out) {
  ZK_DEVICE_GUARD(ctx);
  return bases_upload(ctx, 0, affine, n, out);
}
int zkmi_bases_create_g2(zkmi_ctx* ctx, const uint64_t* affine, size_t n, zkmi_bases** out) {
  ZK_DEVICE_GUARD(ctx);
  return bases_upload(ctx, 1, affine, n, out);
}
void zkmi_bases_destroy(zkmi_bases* b) {
  ZK_DEVICE_GUARD(b);
  if (!b) return;
  hipFree(b->d_pts);
  delete b;
}
size_t zkmi_bases_len(const zkmi_bases* b) { return b ? b->n : 0; }
int zkmi_bases_export(const zkmi_bases* b, uint64_t* affine_out) {
  ZK_DEVICE_GUARD(b);
  if (!b) {
    set_error("zkmi_bases_export: null bases");
    return ZKMI_EINVAL;
  }
  return bases_export(b, affine_out);
}
int zkmi_bases_precompute(zkmi_bases* b, int c, int factor) {
  ZK_DEVICE_GUARD(b);
  if (!b) {
    set_error("zkmi_bases_precompute: null bases");
    return ZKMI_EINVAL;
  }
  if (b->tc) {
    set_error("zkmi_bases_precompute: base set already has a table (window %d)", b->tc);
    return ZKMI_EINVAL;
  }
  return bases_precompute(b, c > 0 ? c : table_window(b->n, b->g2), factor);
}
int zkmi_bases_info(const zkmi_bases* b, uint64_t out[4]) {
  if (!b) {
    set_error("zkmi_bases_info: null bases");
    return ZKMI_EINVAL;
  }
  out[0] = b->n;
  out[1] = (uint64_t)b->tc;
  out[2] = (uint64_t)b->tp;
  out[3] = (uint64_t)b->tw;
  return 0;
}
int zkmi_bases_generate_g1(zkmi_ctx* ctx, uint64_t seed, size_t n, zkmi_bases** out) {
  ZK_DEVICE_GUARD(ctx);
  return bases_generate(ctx, 0, seed, n, out);
}
int zkmi_bases_generate_g2(zkmi_ctx* ctx, uint64_t seed, size_t n, zkmi_bases** out) {
  ZK_DEVICE_GUARD(ctx);
  return bases_generate(ctx, 1, seed, n, out);
}
int zkmi_scalars_generate(zkmi_ctx* ctx, uint64_t seed, size_t n, void* d_scalars) {
  ZK_DEVICE_GUARD(ctx);
  return scalars_generate(ctx, seed, 0, n, d_scalars);
}
int zkmi_bases_generate_range_g1(zkmi_ctx* ctx, uint64_t seed, size_t first, size_t n, zkmi_bases** out) {
  ZK_DEVICE_GUARD(ctx);
  return bases_generate(ctx, 0, seed, first, n, out);
}
int zkmi_bases_generate_arith_g1(zkmi_ctx* ctx, const uint64_t p0[8], const uint64_t d[8], size_t first, size_t n,
                                 zkmi_bases** out) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !p0 || !d || !out) {
    set_error("zkmi_bases_generate_arith_g1: null argument");
    return ZKMI_EINVAL;
  }
  return bases_generate_arith_g1(ctx, p0, d, first, n, out);
}
int zkmi_scalars_generate_range(zkmi_ctx* ctx, uint64_t seed, size_t first, size_t n, void* d_scalars) {
  ZK_DEVICE_GUARD(ctx);
  return scalars_generate(ctx, seed, first, n, d_scalars);
}

static int msm_host_scalars(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const uint64_t* scalars, size_t n,
                            uint64_t* out) {
  void* d;
  ZK_TRY(ctx->ws.get("msm_scalars_stage", n * 32 + 32, &d));
  if (n) ZK_HIP(hipMemcpyAsync(d, scalars, n * 32, hipMemcpyHostToDevice, ctx->stream));
  return msm_device(ctx, b, offset, d, n, out);
}
int zkmi_msm_g1(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const uint64_t* scalars, size_t n,
                uint64_t out_affine[8]) {
  ZK_DEVICE_GUARD(ctx);
  if (!b || b->g2) {
    set_error("zkmi_msm_g1: G1 base set required");
    return ZKMI_EINVAL;
  }
  return msm_host_scalars(ctx, b, offset, scalars, n, out_affine);
}
int zkmi_msm_g2(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const uint64_t* scalars, size_t n,
                uint64_t out_affine[16]) {
  ZK_DEVICE_GUARD(ctx);
  if (!b || !b->g2) {
    set_error("zkmi_msm_g2: G2 base set required");
    return ZKMI_EINVAL;
  }
  return msm_host_scalars(ctx, b, offset, scalars, n, out_affine);
}
int zkmi_msm_g1_device(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
                       uint64_t out_affine[8]) {
  ZK_DEVICE_GUARD(ctx);
  if (!b || b->g2) {
    set_error("zkmi_msm_g1_device: G1 base set required");
    return ZKMI_EINVAL;
  }
  return msm_device(ctx, b, offset, d_scalars, n, out_affine);
}
int zkmi_msm_g2_device(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
                       uint64_t out_affine[16]) {
  ZK_DEVICE_GUARD(ctx);
  if (!b || !b->g2) {
    set_error("zkmi_msm_g2_device: G2 base set required");
    return ZKMI_EINVAL;
  }
  return msm_device(ctx, b, offset, d_scalars, n, out_affine);
}
int zkmi_msm_submit(zkmi_ctx* ctx, const zkmi_bases* b, size_t offset, const void* d_scalars, size_t n,
                    zkmi_msm_job** job) {
  ZK_DEVICE_GUARD(ctx);
  return msm_submit(ctx, b, offset, d_scalars, n, job);
}
int zkmi_msm_wait(zkmi_msm_job* job, uint64_t* out_affine) { return msm_wait(job, out_affine); }
int zkmi_msm_submit_shared(zkmi_ctx* ctx, const zkmi_bases* const* bs, int k, size_t offset, const void* d_scalars,
                           size_t n, zkmi_msm_job** jobs) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !bs || !jobs || k < 1 || (n && !d_scalars)) {
    set_error("zkmi_msm_submit_shared: bad arguments");
    return ZKMI_EINVAL;
  }
  return msm_submit_shared(ctx, bs, k, offset, d_scalars, n, jobs);
}
int zkmi_msm_set_lanes(zkmi_ctx* ctx, int lanes) {
  if (!ctx || lanes < 1 || lanes > 8) {
    set_error("zkmi_msm_set_lanes: lanes must be in [1, 8]");
    return ZKMI_EINVAL;
  }
  // stream budget: at most MAX_LANES_WITH_COMM lanes beside a communicator
  ctx->msm_lanes = ctx->ncomm ? std::min(lanes, MAX_LANES_WITH_COMM) : lanes;
  return 0;
}
int zkmi_msm_get_lanes(const zkmi_ctx* ctx) { return ctx ? ctx->msm_lanes : -1; }
int zkmi_ctx_stream_count(const zkmi_ctx* ctx) { return ctx ? ctx->nstreams : -1; }
int zkmi_msm_set_window(zkmi_ctx* ctx, int c) {
  if (c != 0 && (c < 4 || c > 17)) {
    set_error("window %d outside [4, 17]", c);
    return ZKMI_EINVAL;
  }
  ctx->msm_window = c;
  return 0;
}
int zkmi_g1_add(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]) {
  host_g1_add_affine(a, b, out);
  return 0;
}
int zkmi_g2_add(const uint64_t a[16], const uint64_t b[16], uint64_t out[16]) {
  host_g2_add_affine(a, b, out);
  return 0;
}

// ------------------------------------------------------------------ NTT
int zkmi_ntt_device(zkmi_ctx* ctx, void* d_data, uint32_t log_n, int inverse, int coset) {
  ZK_DEVICE_GUARD(ctx);
  ZK_TRY(ntt_device(ctx, (uint32_t*)d_data, log_n, inverse, coset));
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  return timer_flush(ctx);
}
int zkmi_ntt(zkmi_ctx* ctx, uint64_t* data, uint32_t log_n, int inverse, int coset) {
  ZK_DEVICE_GUARD(ctx);
  if (log_n > 28) {
    set_error("ntt: log_n %u > 28", log_n);
    return ZKMI_EINVAL;
  }
  size_t bytes = ((size_t)1 << log_n) * 32;
  void* d;
  ZK_TRY(ctx->ws.get("ntt_stage", bytes, &d));
  ZK_HIP(hipMemcpyAsync(d, data, bytes, hipMemcpyHostToDevice, ctx->stream));
  ZK_TRY(ntt_device(ctx, (uint32_t*)d, log_n, inverse, coset));
  ZK_HIP(hipMemcpyAsync(data, d, bytes, hipMemcpyDeviceToHost, ctx->stream));
  ZK_HIP(hipStreamSynchronize(ctx->stream));
  return timer_flush(ctx);
}

// ------------------------------------------------------------- encodings
int zkmi_proof_to_solana_bytes(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8], uint8_t out[256]) {
  proof_solana(a, b, c, out);
  return 0;
}
int zkmi_proof_serialize_compressed(const uint64_t a[8], const uint64_t b[16], const uint64_t c[8],
                                    uint8_t out[128]) {
  g1_compress(a, out);
  g2_compress(b, out + 32);
  g1_compress(c, out + 96);
  return 0;
}

}  // extern "C"
